# Round-4 check: smoke, the GPU parity suite, the N-GPU wall-clock projection
# (tools/wallclock_ngpu.py, same_device=2), the default bench line.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r4c || exit 1
O=gpurun_out/r4c
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
if [ "${WALL:-1}" = "1" ]; then
  timeout -k 10 600 python3 tools/wallclock_ngpu.py --repeat ${REPEAT:-2} > $O/wall_ngpu.jsonl 2> $O/wall_ngpu.err || { echo WALL_FAIL; tail -20 $O/wall_ngpu.err; exit 1; }
  python3 -c "
import json
for l in open('$O/wall_ngpu.jsonl'):
    d=json.loads(l); print('N=%d wall %.3f proj %.3f setup_max %.1f render_max %.1f gather %.1f md5ok %s' % (d['ngpu'], d['wall_s'], d['projected_wall_s'], d['setup_ms_max'], d['render_ms_max'], d['gather_ms'] or 0, d['md5_same_as_n1']))"
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('render_256spp_mray_s'))"
fi
