# rocprofv3 evidence for the bench workload: kernel trace + stats, then PMC
# passes (one counter group per pass, never combined with other trace domains),
# then the default bench line (with the CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof
rm -rf $OUT
mkdir -p $OUT
STEPS=${STEPS:-4}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --no-cpu-baseline --no-wallclock --steps $STEPS --warmup 1 > $OUT/bench_kt.json 2> $OUT/bench_kt.err && echo KT_OK &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 bench.py --no-cpu-baseline --no-wallclock --steps $STEPS --warmup 1 > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err && echo FETCH_OK &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 bench.py --no-cpu-baseline --no-wallclock --steps $STEPS --warmup 1 > $OUT/bench_write.json 2> $OUT/bench_write.err && echo WRITE_OK &&
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_l2 -o run -- \
  python3 bench.py --no-cpu-baseline --no-wallclock --steps $STEPS --warmup 1 > $OUT/bench_l2.json 2> $OUT/bench_l2.err && echo L2_OK &&
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- \
  python3 bench.py --no-cpu-baseline --no-wallclock --steps $STEPS --warmup 1 > $OUT/bench_sq.json 2> $OUT/bench_sq.err && echo SQ_OK &&
timeout -k 10 900 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && echo BENCH_OK
cat $OUT/bench_default.json
