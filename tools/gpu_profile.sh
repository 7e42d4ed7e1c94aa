# rocprofv3 evidence for the bench workload: kernel trace + stats, then PMC
# passes (one counter group per pass, never combined with other trace domains;
# each pass stays within the per-block slot limits: SQ 8, TCC 4, GRBM 2), then
# the default bench line (with the CPU baseline and the wall-clock run).
#   bash tools/gpu_profile.sh  ->  gpurun_out/prof ; summarise with
#   python tools/pmc_summary.py gpurun_out/prof profiles/<tag> --key c3_n1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof
rm -rf $OUT
mkdir -p $OUT
STEPS=${STEPS:-20}
B="python3 bench.py --no-cpu-baseline --no-wallclock --steps $STEPS --warmup 5"
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  $B > $OUT/bench_kt.json 2> $OUT/bench_kt.err && echo KT_OK &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  $B > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err && echo FETCH_OK &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  $B > $OUT/bench_write.json 2> $OUT/bench_write.err && echo WRITE_OK &&
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_l2 -o run -- \
  $B > $OUT/bench_l2.json 2> $OUT/bench_l2.err && echo L2_OK &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq -o run -- \
  $B > $OUT/bench_sq.json 2> $OUT/bench_sq.err && echo SQ_OK &&
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench_default.json 2> $OUT/bench_default.err && echo BENCH_OK &&
cat $OUT/bench_default.json || exit 1
# instruction-mix pass: only the counters this rocprofv3 lists
SQ2=""
for c in SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS \
         SQ_ACTIVE_INST_MISC; do
  grep -q "\b$c\b" $OUT/avail.txt && SQ2="$SQ2 $c"
done
if [ -n "$SQ2" ]; then
  timeout -s KILL 300 rocprofv3 --pmc $SQ2 --output-format csv -d $OUT/pmc_sq2 -o run -- \
    $B > $OUT/bench_sq2.json 2> $OUT/bench_sq2.err && echo SQ2_OK
fi
