# Per-round timeline of the path engine for a rank-of-W simulation (PT_WPROF build)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/wprof || exit 1
for w in ${WS:-8}; do
  rm -f /tmp/wg.bin
  PT_LIB=raytracing-course_amd/build_wprof/libpt.so PT_WGPROF=/tmp/wg.bin timeout -k 10 300 python3 tools/rank_sim.py --worlds $w --steps 1 > gpurun_out/wprof/rl_$w.jsonl 2> gpurun_out/wprof/roundlog_$w.txt || { echo FAIL; tail gpurun_out/wprof/roundlog_$w.txt; exit 1; }
  echo "== world $w"; tail -1 gpurun_out/wprof/rl_$w.jsonl
  python3 tools/wg_rounds.py /tmp/wg.bin 768 gpurun_out/wprof/roundlog_$w.txt > gpurun_out/wprof/rounds_$w.txt
  python3 tools/wg_tail.py /tmp/wg.bin 768 > gpurun_out/wprof/tail_$w.txt
done
