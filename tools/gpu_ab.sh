# GPU parity suite, then an interleaved A/B of library builds on rank-of-1 and
# rank-of-8 throughput (tools/rank_sim.py):  VARS="name:libdir[:ENV=v,..] ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${PT_TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit 1
fi
WORLDS="${WORLDS:-1 8}" bash tools/gpu_variants2.sh
