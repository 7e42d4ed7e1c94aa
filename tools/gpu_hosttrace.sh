# Host timeline of the drop-in CLI on small configs: rocprofv3 HIP API + kernel
# trace (no PMC in the same run), then the wall-clock table of run.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/host
rm -rf $OUT; mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0,'tools'); import wallclock as w; [w.scene(c) for c in ('c1','c2','c4_metal')]"
for c in ${CONFIGS:-c1 c2}; do
  PT_FULL_EXIT=1 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $OUT/$c -o run -- \
    raytracing-course_amd/build/pt_render scenes/gen/$c.txt /tmp/$c.ppm > $OUT/$c.out 2> $OUT/$c.err || exit 1
  echo "TRACE_$c OK"
done
PT_QUIET=1 timeout -k 10 600 python3 tools/wallclock.py ${WALL:-c1 c2 c1 c2 c4_metal} > $OUT/wall.jsonl 2> $OUT/wall.err || exit 1
cat $OUT/wall.jsonl
