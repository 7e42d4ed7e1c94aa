# Path-engine per-trip timelines (PT_WPROF build in build_wprof) at WORLDS, after
# the parity suite and bench line of the default build (TESTS=0 / BENCH=0 skip them).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3 gpurun_out/wprof || exit 1
O=gpurun_out/r3
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'])"
fi
for w in ${WORLDS:-1 8}; do
  rm -f /tmp/wg.bin
  PT_LIB=raytracing-course_amd/${WLIB:-build_wprof}/libpt.so PT_TUNE=wgprof=/tmp/wg.bin timeout -k 10 300 python3 tools/rank_sim.py --worlds $w --steps 1 > gpurun_out/wprof/w$w.jsonl 2> gpurun_out/wprof/w$w.err || { echo WPROF_FAIL; tail gpurun_out/wprof/w$w.err; exit 1; }
  echo "== wprof w$w $(tail -1 gpurun_out/wprof/w$w.jsonl)"
  python3 tools/wg_path.py /tmp/wg.bin 1024 > gpurun_out/wprof/path_w$w.txt && cat gpurun_out/wprof/path_w$w.txt
done
