# rank_sim over library builds: VARS="name:libdir[:key=v+key=v] ..." (optional PT_TUNE settings);
# WORLDS, RANKS (rank_sim --ranks), STEPS
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/var2 || exit 1
for spec in $VARS; do
  IFS=: read name lib tune <<< "$spec"
  PT_LIB=raytracing-course_amd/$lib/libpt.so PT_TUNE=$(echo "$tune" | tr '+' ',') timeout -k 10 300 python3 tools/rank_sim.py --worlds ${WORLDS:-1 8} --ranks ${RANKS:-first} --steps ${STEPS:-2} > gpurun_out/var2/$name.jsonl 2> gpurun_out/var2/$name.err || { echo "FAILED $name"; tail -3 gpurun_out/var2/$name.err; exit 1; }
  echo "$name: $(python3 -c "
import json
for l in open('gpurun_out/var2/$name.jsonl'):
    d=json.loads(l)
    if 'rank' in d: print('w%d/%d %.1f;' % (d['world'], d['rank'], d['mray_s']), end=' ')
")"
done
