# SQ counters of the path engine vs the round engine on the rank-of-1 simulation
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmce || exit 1
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
for eng in path round; do
  PT_ENGINE=$eng timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d gpurun_out/pmce/$eng -o run -- python3 tools/rank_sim.py --worlds ${W:-1} --steps 1 > gpurun_out/pmce/$eng.log 2>&1 || { echo "FAILED $eng"; tail -5 gpurun_out/pmce/$eng.log; exit 1; }
  echo "== $eng"; python3 tools/pmc_quick.py gpurun_out/pmce/$eng
done
