# GPU round check: smoke, GPU parity tests, default bench line, rank-of-N simulation.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; } > gpurun_out/host.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread --durations=30 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo PYTEST_RC=$rc
tail -5 gpurun_out/pytest_gpu.log
[ $rc = 0 ] || exit 1
if [ "${PT_BENCH:-1}" = "1" ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err; echo BENCH_RC=$?
  cat gpurun_out/bench.json
fi
if [ -n "${WORLDS:-}" ]; then
  timeout -k 10 600 python3 tools/rank_sim.py --worlds $WORLDS --steps ${STEPS:-2} > gpurun_out/ranksim.jsonl 2> gpurun_out/ranksim.err; echo SIM_RC=$?
  cat gpurun_out/ranksim.jsonl
fi
