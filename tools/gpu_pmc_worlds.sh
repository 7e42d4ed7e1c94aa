# SQ counters of the path engine on rank-of-W simulations (default library)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmcw || exit 1
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
for w in ${WORLDS:-1 8}; do
  timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d gpurun_out/pmcw/w$w -o run -- python3 tools/rank_sim.py --worlds $w --steps 1 > gpurun_out/pmcw/w$w.log 2>&1 || { echo "FAILED $w"; tail -5 gpurun_out/pmcw/w$w.log; exit 1; }
  echo "== w$w $(grep world gpurun_out/pmcw/w$w.log)"; python3 tools/pmc_quick.py gpurun_out/pmcw/w$w | grep -A10 k_wpath
done
