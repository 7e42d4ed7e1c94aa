# rank_sim under different env settings: SWEEP="name:VAR=val,VAR=val ..." WORLDS="1 8"
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/sweep || exit 1
for spec in $SWEEP; do
  name=${spec%%:*}; vars=${spec#*:}
  envs=$(echo "$vars" | tr ',' ' ')
  env $envs timeout -k 10 300 python3 tools/rank_sim.py --worlds ${WORLDS:-1 8} --steps ${STEPS:-2} > gpurun_out/sweep/$name.jsonl 2> gpurun_out/sweep/$name.err || { echo "FAILED $name"; tail -5 gpurun_out/sweep/$name.err; exit 1; }
  echo "$name: $(python3 -c "
import json
for l in open('gpurun_out/sweep/$name.jsonl'):
    d=json.loads(l); print('w%d %.1f Mray/s %.3f ms/round %d rounds;' % (d['world'], d['mray_s'], d['isect_ms_per_round'], d['rounds_per_step']), end=' ')
")"
done
