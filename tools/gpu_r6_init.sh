# Round 6: the CLI's start-up phases (PT_STATS=3: hipInit / device enumeration / properties /
# context / code objects / first copy; pt_scene_prepare's stages) over REPEAT runs of config
# CFG, then the N-GPU wall-clock projection (tools/wallclock_ngpu.py, same_device=2).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6i || exit 1
O=gpurun_out/r6i
python3 -c "import sys; sys.path.insert(0,'.'); import bench; bench.scene_file('${CFG:-c3}')"
for i in $(seq 1 ${REPEAT:-3}); do
  PT_STATS=3 PT_QUIET=1 timeout -k 10 60 ./run.sh scenes/gen/${CFG:-c3}.txt /tmp/o.ppm 2> $O/run_$i.err || { echo FAIL; tail -5 $O/run_$i.err; exit 1; }
  grep -E "pt_device_init|phases_ms|prepare |gather ms" $O/run_$i.err | tr '\n' ' '; echo
done
if [ "${WALL:-1}" = "1" ]; then
  timeout -k 10 500 python3 tools/wallclock_ngpu.py --repeat ${WREPEAT:-2} --ngpu ${NGPU:-1 4 8} --tune "same_device=2" > $O/wall.jsonl 2> $O/wall.err || { echo WALL_FAIL; tail -20 $O/wall.err; exit 1; }
  python3 -c "
import json
for l in open('$O/wall.jsonl'):
    d=json.loads(l); print('N=%d wall %.3f proj %.3f render %s md5ok %s' % (d['ngpu'], d['wall_s'], d['projected_wall_s'], [round(x) for x in d['render_ms']], d['md5_same_as_n1']))"
fi
