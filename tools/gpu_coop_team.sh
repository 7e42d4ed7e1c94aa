cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/coop
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-each_engine or suspended or coop}" > gpurun_out/coop/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/coop/pytest.log; [ $rc = 0 ] || exit 1
for t in ${TEAMS:-64 32 16}; do
  PT_LIB=raytracing-course_amd/build_cprof/libpt.so PT_TUNE=cprof=1,coop=100000000,coop_team=$t timeout -k 10 300 python3 tools/rank_sim.py --worlds 8 --steps 1 > gpurun_out/coop/cp$t.jsonl 2> gpurun_out/coop/cp$t.err || exit 1
  echo "team $t"; grep "coop chains" gpurun_out/coop/cp$t.err | tail -1
done
VARS="${VARS:-t16:build:coop=65536+coop_team=16}" bash tools/gpu_variants2.sh
