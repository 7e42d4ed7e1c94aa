# Round 6 check: smoke, the GPU parity suite (PYTEST_K subset or all), the default bench
# line at the driver's --steps 20 --warmup 5 (BENCH_ARGS extra), and (DIST=1) the 2-rank
# strong-scaling line on one GPU (--same-device --dist-backend gloo).  Output: gpurun_out/r6k
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6k || exit 1
O=gpurun_out/r6k
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1500 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 900 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench.json')); w=d.get('wall_to_ppm') or {}; r=d['roofline']; c=d.get('cpu_baseline') or {}
print('BENCH', round(d['value']), round(d['ms_per_step'],2), round(r['frac'],3), {k: (round(v,3) if isinstance(v,float) else v) for k,v in (r.get('coop') or {}).items()}, 'r256', d.get('render_256spp_mray_s'), d.get('render_256spp_wall_mray_s'), 'ppm_s', w.get('seconds'), 'teardown', w.get('teardown_s'), 'fb=cli', d.get('framebuffer_equals_cli_ppm'), 'cpu', c.get('value'), (c.get('configs') or {}).get('c3', {}).get('render_s'))"
fi
if [ "${DIST:-0}" = "1" ]; then
  for sc in strong weak; do
    timeout -k 10 600 python bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 --scaling $sc --no-cpu-baseline --no-wallclock > $O/dist2_$sc.json 2> $O/dist2_$sc.err || { echo DIST_FAIL; tail -20 $O/dist2_$sc.err; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/dist2_$sc.json') if l.startswith('{')][-1]); print('DIST2', d['scaling'], round(d['value']), round(d['ms_per_step'],2), d['pass_spp'], d['framebuffer_md5'], [round(r['mray_s']) for r in d['per_rank']])"
  done
fi
