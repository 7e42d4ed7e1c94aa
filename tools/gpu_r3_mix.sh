# Round-3 step-mix A/B: parity suite + bench on the default build, then rank_sim
# (WORLDS, rank 0) over VARS interleaved (tools/gpu_variants2.sh).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3 || exit 1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r3/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r3/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/r3/pytest_gpu.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/r3/bench.json 2> gpurun_out/r3/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r3/bench.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r3/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'])"
fi
bash tools/gpu_variants2.sh
