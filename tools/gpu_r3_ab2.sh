# A/B (tools/gpu_r3_ab.sh) followed by one PT_WPROF timeline per build in WLIBS (world 1)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/wprof || exit 1
TESTS=${TESTS:-0} bash tools/gpu_r3_ab.sh || exit 1
for wl in ${WLIBS:-build_wprof}; do
  rm -f /tmp/wg.bin
  PT_LIB=raytracing-course_amd/$wl/libpt.so PT_TUNE=wgprof=/tmp/wg.bin timeout -k 10 300 python3 tools/rank_sim.py --worlds 1 --steps 1 > gpurun_out/wprof/$wl.jsonl 2> gpurun_out/wprof/$wl.err || { echo WPROF_FAIL $wl; exit 1; }
  echo "== wprof $wl"
  python3 tools/wg_path.py /tmp/wg.bin 1024 > gpurun_out/wprof/path_$wl.txt && cat gpurun_out/wprof/path_$wl.txt
done
