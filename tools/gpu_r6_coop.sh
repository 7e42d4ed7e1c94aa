# Round 6: the cooperative engine's evidence at the point where it matters (one rank's
# 256-spp pass of config 3 as rank 0 of 8 and of 1, tools/pass_log.py):
#   1. smoke(), then the pass (coop_ms, coop_rays) at each PTS point, REPEAT times
#   2. (CPROF=1) per-phase cycles of k_wcoop on the -DPT_CPROF build (build_cprof)
#   3. (PMC=1) rocprofv3 PMC passes of the same rank-of-8 pass, one counter group each:
#      SQ issue/wait, L2 hit/miss, FETCH_SIZE, WRITE_SIZE; pmc_quick.py prints them per kernel
# Output: gpurun_out/r6c
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6c || exit 1
O=gpurun_out/r6c
LIBD=${LIB:-build}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
for rep in $(seq 1 ${REPEAT:-2}); do
  for pt in ${PTS:-8:0 1:0}; do
    IFS=: read w r <<< "$pt"
    PT_LIB=raytracing-course_amd/$LIBD/libpt.so timeout -k 10 120 python3 tools/pass_log.py --world $w --rank $r --level 0 ${PTUNE:+--tune "$PTUNE"} > $O/pass_w${w}_r${r}_$rep.txt 2> $O/pass_w${w}_r${r}_$rep.err || { echo FAIL w$w r$r; tail -20 $O/pass_w${w}_r${r}_$rep.err; exit 1; }
    tail -1 $O/pass_w${w}_r${r}_$rep.txt
  done
done
if [ "${CPROF:-1}" = "1" ]; then
  PT_LIB=raytracing-course_amd/build_cprof/libpt.so timeout -k 10 120 python3 tools/pass_log.py --world 8 --rank 0 --level 0 --tune cprof=1${PTUNE:+,$PTUNE} > $O/cprof_w8.txt 2> $O/cprof_w8.err || { echo CPROF_FAIL; tail -20 $O/cprof_w8.err; exit 1; }
  tail -1 $O/cprof_w8.txt; grep -iE "coop|cprof" $O/cprof_w8.err | tail -30
fi
if [ "${PMC:-1}" = "1" ]; then
  P="python3 tools/pass_log.py --world 8 --rank 0 --level 0"
  export PT_LIB=raytracing-course_amd/$LIBD/libpt.so
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o run -- $P > $O/pmc$i.txt 2> $O/pmc$i.err || { echo "PMC pass $i FAILED"; tail -5 $O/pmc$i.err; exit 1; }
    echo "pmc pass $i ok"
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $P > $O/kt.txt 2> $O/kt.err && echo KT_OK || { echo KT_FAIL; exit 1; }
  for i in 1 2 3 4 5; do python3 tools/pmc_quick.py $O/pmc$i; done > $O/pmc_summary.txt 2>&1
  cat $O/pmc_summary.txt | head -80
fi
