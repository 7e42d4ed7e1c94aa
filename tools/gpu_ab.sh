# A/B runs of bench.py under different env settings; each setting is "NAME:VAR=val,VAR=val".
#   AB="wave:PT_ENGINE=wave mega:PT_ENGINE=mega,PT_VARIANT=0" bash tools/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab
mkdir -p $OUT
for spec in $AB; do
  name=${spec%%:*}; vars=${spec#*:}
  envs=$(echo "$vars" | tr ',' ' ')
  env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps ${STEPS:-4} --warmup 1 $BENCH_ARGS \
     > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "FAILED $name"; tail -5 $OUT/bench_$name.err; exit 1; }
  echo "$name: $(python3 -c "import json;d=json.load(open('$OUT/bench_$name.json'));print(round(d['value'],2),'Mray/s', round(d['ms_per_step'],2),'ms/step', 'fb', d['fallback_rate'], 'err', d['exactness_errors'], 'nodes/ray', round(d['node_visits_per_ray'],1), 'aux/ray', round(d['aux_visits_per_ray'],1))")"
done
