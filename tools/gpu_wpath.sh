cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/wprof || exit 1
for w in ${WORLDS:-8 1}; do
  rm -f /tmp/wg.bin
  PT_LIB=raytracing-course_amd/build_wprof/libpt.so PT_WGPROF=/tmp/wg.bin timeout -k 10 300 python3 tools/rank_sim.py --worlds $w --steps 1 > gpurun_out/wprof/path_w$w.jsonl 2>&1 || exit 1
  echo "== w$w $(tail -1 gpurun_out/wprof/path_w$w.jsonl)"
  python3 tools/wg_path.py /tmp/wg.bin 768 || exit 1
done
