# rank simulation of the N-GPU bench (tools/rank_sim.py) + optional extra bench configs ($CONFIGS)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/sim &&
timeout -k 10 300 python3 tools/rank_sim.py --ranks ${RANKS:-first} > gpurun_out/sim/rank_sim.jsonl 2> gpurun_out/sim/rank_sim.err &&
for c in ${CONFIGS:-}; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --config $c > gpurun_out/sim/$c.json 2> gpurun_out/sim/$c.err || exit 1
done
