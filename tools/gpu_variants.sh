# A/B of the k_trace variants on the bench workload, with per-workgroup timelines.
#   PT_VARIANT bit 0 = filtered node tests + flat replay, bit 1 = XCD-banded tile order
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/var
mkdir -p $OUT
for v in ${VARIANTS:-0 1 2 3}; do
  rm -f $OUT/wg_$v.bin
  PT_VARIANT=$v PT_WGPROF=$OUT/wg_$v.bin timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 \
     > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit $?
  echo "variant $v: $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print(round(d['value'],2),'Mray/s',round(d['roofline']['launch_ms'],2),'ms/launch')")"
done
