# Round-3 baseline on the GPU: smoke, parity suite, bench line, every rank of
# N = 2, 4, 8 (rank_sim --ranks all), per-trip path-engine timelines
# (PT_WPROF build in build_wprof), then a PC-sampling attempt of the path engine.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3 gpurun_out/wprof || exit 1
O=gpurun_out/r3
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $O/host.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 600 python3 tools/rank_sim.py --worlds 1 2 4 8 --ranks all --steps 2 > $O/ranksim_all.jsonl 2> $O/ranksim_all.err || { echo SIM_FAIL; tail -20 $O/ranksim_all.err; exit 1; }
grep -E 'min_mray|"world": 1,' $O/ranksim_all.jsonl
for w in 1 8; do
  rm -f /tmp/wg.bin
  PT_LIB=raytracing-course_amd/build_wprof/libpt.so PT_TUNE=wgprof=/tmp/wg.bin timeout -k 10 300 python3 tools/rank_sim.py --worlds $w --steps 1 > gpurun_out/wprof/w$w.jsonl 2> gpurun_out/wprof/w$w.err || { echo WPROF_FAIL; exit 1; }
  echo "== wprof w$w $(tail -1 gpurun_out/wprof/w$w.jsonl)"
  python3 tools/wg_path.py /tmp/wg.bin 1024 > gpurun_out/wprof/path_w$w.txt && cat gpurun_out/wprof/path_w$w.txt
done
if [ "${PCS:-1}" = "1" ]; then
  timeout -s KILL 60 rocprofv3 -L > $O/rocprof_L.txt 2>&1; echo "LIST_RC=$?"
  grep -i -A3 -E 'pc.?sampl|host_trap|stochastic' $O/rocprof_L.txt | head -30
  timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 50 --kernel-include-regex k_wpath -d $O/pcs -o pcs --output-format csv -- python3 tools/rank_sim.py --worlds 1 --steps 1 > $O/pcs.log 2>&1; echo "PCS_RC=$?"
  tail -5 $O/pcs.log
  find $O/pcs -type f | head
fi
