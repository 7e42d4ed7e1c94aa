# GPU round check: smoke, GPU parity tests, default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python -m pytest tests/test_gpu.py -x -q --durations=30 > gpurun_out/pytest_gpu.log 2>&1; echo PYTEST_RC=$?
tail -5 gpurun_out/pytest_gpu.log
if [ "${PT_BENCH:-1}" = "1" ]; then
  timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; echo BENCH_RC=$?
  cat gpurun_out/bench.json
fi
