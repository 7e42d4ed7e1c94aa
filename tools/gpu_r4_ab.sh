# A/B of library builds: (optional) the GPU parity suite on the candidate build
# (PT_LIB=$CAND), then rank_sim over VARS (tools/gpu_variants2.sh), REPEAT times
# interleaved.  CAND=build_dev VARS="base:build_r4a dev:build_dev" WORLDS="1 8" STEPS=20
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ab || exit 1
O=gpurun_out/ab
if [ -n "${CAND:-}" ]; then
  PT_LIB=raytracing-course_amd/$CAND/libpt.so timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_$CAND.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_$CAND.log; exit 1; }
  tail -2 $O/pytest_$CAND.log
fi
for r in $(seq 1 ${REPEAT:-1}); do
  for spec in $VARS; do
    IFS=: read name lib tune <<< "$spec"
    PT_LIB=raytracing-course_amd/$lib/libpt.so PT_TUNE=$(echo "$tune" | tr '+' ',') timeout -k 10 300 python3 tools/rank_sim.py --worlds ${WORLDS:-1 8} --ranks ${RANKS:-first} --steps ${STEPS:-20} > $O/$name.$r.jsonl 2> $O/$name.$r.err || { echo "FAILED $name"; tail -3 $O/$name.$r.err; exit 1; }
    echo "$name#$r: $(python3 -c "
import json
for l in open('$O/$name.$r.jsonl'):
    d=json.loads(l)
    if 'rank' in d: print('w%d/%d %.0f (coop %.1f ms);' % (d['world'], d['rank'], d['mray_s'], d['coop_ms_per_step']), end=' ')
")"
  done
done
if [ "${PREP:-0}" = "1" ]; then
  for i in 1 2; do PT_TUNE=prepstats=1 PT_STATS=2 PT_QUIET=1 timeout -k 10 120 ./run.sh scenes/gen/c3.txt /tmp/c3.ppm > /dev/null 2> $O/prep$i.err; done
  grep -h "prepare\|phases" $O/prep*.err
fi
