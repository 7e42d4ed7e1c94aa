# Round 5: smoke, then the N-GPU wall-clock projection (tools/wallclock_ngpu.py, one GPU,
# same_device=2) for each PT_TUNE variant in TUNES (space-separated; "-" = defaults),
# REPEAT repeats each.  Output: gpurun_out/r5w/wall_<i>.jsonl
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r5w || exit 1
O=gpurun_out/r5w
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
i=0
for T in ${TUNES:--}; do
  tune="same_device=2"; [ "$T" != "-" ] && tune="same_device=2,$T"
  timeout -k 10 500 python3 tools/wallclock_ngpu.py --repeat ${REPEAT:-2} --ngpu ${NGPU:-1 2 4 8} --tune "$tune" > $O/wall_$i.jsonl 2> $O/wall_$i.err || { echo WALL_FAIL $T; tail -20 $O/wall_$i.err; exit 1; }
  python3 -c "
import json
for l in open('$O/wall_$i.jsonl'):
    d=json.loads(l); print('$T', 'N=%d wall %.3f proj %.3f render %s md5ok %s' % (d['ngpu'], d['wall_s'], d['projected_wall_s'], [round(x) for x in d['render_ms']], d['md5_same_as_n1']))"
  i=$((i+1))
done
