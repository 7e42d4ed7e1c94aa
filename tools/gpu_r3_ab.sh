# A/B within one call: the parity suite on the default build (TESTS=0 skips), then
# tools/gpu_variants2.sh over VARS (rank_sim at WORLDS) -- interleave repeats in VARS.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3 || exit 1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r3/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r3/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/r3/pytest_gpu.log
fi
bash tools/gpu_variants2.sh
