# Round 6: the pooled cooperative query -- the full GPU suite on the new build, then an
# interleaved A/B against the round's base build (build_base) on one rank's 256-spp pass
# (tools/gpu_r5_ab.sh), then the per-phase cycles of the new build (build_cprof).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp || exit 1
if [ "${TESTS:-1}" = "1" ]; then
  BENCH=0 bash tools/gpu_r6_check.sh || exit 1
fi
TAG=${TAG:-pool} VARS=${VARS:-"base:-:build_base pool:-:build"} PTS=${PTS:-"8:0 8:3 4:0 1:0"} REPEAT=${REPEAT:-2} bash tools/gpu_r5_ab.sh || exit 1
if [ "${CPROF:-1}" = "1" ]; then
  mkdir -p gpurun_out/r6c
  PT_LIB=raytracing-course_amd/build_cprof/libpt.so timeout -k 10 120 python3 tools/pass_log.py --world 8 --rank 0 --level 0 --tune cprof=1 > gpurun_out/r6c/cprof_pool_w8.txt 2> gpurun_out/r6c/cprof_pool_w8.err || { echo CPROF_FAIL; tail -5 gpurun_out/r6c/cprof_pool_w8.err; exit 1; }
  cut -c1-300 gpurun_out/r6c/cprof_pool_w8.txt
fi
