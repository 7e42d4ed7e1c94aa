# Round-4 baseline on the GPU: smoke, the default bench line, then every rank of
# N = 1, 2, 4, 8 at the driver's pass length (rank_sim --steps $STEPS, default 20).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r4 || exit 1
O=gpurun_out/r4
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('wall_to_ppm'))"
fi
timeout -k 10 600 python3 tools/rank_sim.py --worlds ${WORLDS:-1 2 4 8} --ranks ${RANKS:-all} --steps ${STEPS:-20} > $O/ranksim.jsonl 2> $O/ranksim.err || { echo SIM_FAIL; tail -20 $O/ranksim.err; exit 1; }
grep -E 'min_mray|"world": 1,' $O/ranksim.jsonl
