# Round 5: the CLI's start-up phases (PT_STATS=3: pt_device_init's parts) over REPEAT runs of a config
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/init || exit 1
python3 -c "import sys; sys.path.insert(0,'.'); import bench; bench.scene_file('${CFG:-c3}')"
for i in $(seq 1 ${REPEAT:-5}); do
  PT_STATS=3 PT_QUIET=1 timeout -k 10 60 ./run.sh scenes/gen/${CFG:-c3}.txt /tmp/o.ppm 2> gpurun_out/init/run_$i.err || { echo FAIL; tail -5 gpurun_out/init/run_$i.err; exit 1; }
  grep -E "pt_device_init|phases_ms|hip runtime|gather ms" gpurun_out/init/run_$i.err | tr '\n' ' '; echo
done
