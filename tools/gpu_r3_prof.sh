cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TESTS=0 BENCH=0 WORLDS="" WPROF_WORLDS="1" WLIB=build_wprof bash tools/gpu_r3_check.sh && cp gpurun_out/wprof/path_w1.txt gpurun_out/wprof/path_w1_wprof.txt && \
TESTS=0 BENCH=0 WORLDS="" WPROF_WORLDS="1" WLIB=build_qprof bash tools/gpu_r3_check.sh
