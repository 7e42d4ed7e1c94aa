# cooperative engine bring-up: GPU parity suite, then rank_sim over coop thresholds (PT_TUNE coop=N)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/coop || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/coop/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/coop/pytest.log; [ $rc = 0 ] || exit 1
for c in ${COOPS:-0 4096}; do
  PT_TUNE=coop=$c${TUNE_EXTRA:+,$TUNE_EXTRA} timeout -k 10 300 python3 tools/rank_sim.py --worlds ${WORLDS:-1 8} --steps 2 > gpurun_out/coop/sim_$c.jsonl 2> gpurun_out/coop/sim_$c.err || { echo SIM_FAIL $c; tail -5 gpurun_out/coop/sim_$c.err; exit 1; }
  echo "coop=$c"; cat gpurun_out/coop/sim_$c.jsonl
done
