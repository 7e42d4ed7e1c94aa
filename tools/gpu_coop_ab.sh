# cooperative engine A/B: the GPU parity tests that exercise it, the phase profile, then rank_sim over builds
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/coop || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-each_engine or suspended or coop or golden_images_bit_exact}" > gpurun_out/coop/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/coop/pytest.log; [ $rc = 0 ] || exit 1
if [ -n "${CPROF:-}" ]; then COOPS="$CPROF" bash tools/gpu_cprof.sh || exit 1; fi
VARS="${VARS:-}" bash tools/gpu_variants2.sh
