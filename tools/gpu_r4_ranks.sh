# Every rank of N = 1, 2, 4, 8 at the driver's pass length (rank_sim --steps 20),
# for one library build (LIB, default build) and PT_TUNE settings (TUNE), REPEAT times.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ranks || exit 1
O=gpurun_out/ranks
for r in $(seq 1 ${REPEAT:-1}); do
  PT_LIB=raytracing-course_amd/${LIB:-build}/libpt.so PT_TUNE=${TUNE:-} timeout -k 10 600 python3 tools/rank_sim.py --worlds ${WORLDS:-1 2 4 8} --ranks ${RANKS:-all} --steps ${STEPS:-20} > $O/${TAG:-ranks}.$r.jsonl 2> $O/${TAG:-ranks}.$r.err || { echo SIM_FAIL; tail -5 $O/${TAG:-ranks}.$r.err; exit 1; }
  echo "#$r $(python3 -c "
import json
for l in open('$O/${TAG:-ranks}.$r.jsonl'):
    d=json.loads(l)
    if 'min_mray_s' in d: print('w%d min %.0f max %.0f;' % (d['world'], d['min_mray_s'], d['max_mray_s']), end=' ')
    elif d.get('world') == 1: print('w1 %.0f;' % d['mray_s'], end=' ')
")"
done
