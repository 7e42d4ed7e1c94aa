# rank_sim over PT_TUNE settings with the default library: VARS="name:key=v+key=v ..."
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/envsweep || exit 1
for spec in $VARS; do
  IFS=: read name tune <<< "$spec"
  PT_TUNE=$(echo "$tune" | tr '+' ',') timeout -k 10 300 python3 tools/rank_sim.py --worlds ${WORLDS:-1 8} --steps ${STEPS:-2} > gpurun_out/envsweep/$name.jsonl 2> gpurun_out/envsweep/$name.err || { echo "FAILED $name"; tail -3 gpurun_out/envsweep/$name.err; exit 1; }
  echo "$name: $(python3 -c "
import json
for l in open('gpurun_out/envsweep/$name.jsonl'):
    d=json.loads(l); print('w%d %.1f (%d rounds);' % (d['world'], d['mray_s'], d['rounds_per_step']), end=' ')
")"
done
