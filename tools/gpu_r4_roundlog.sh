# The GPU parity suite on the product build, then one rank's per-round log
# (PT_TUNE roundlog=1) at ranks of 1 and 8: where a pass's time goes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/rl || exit 1
O=gpurun_out/rl
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for w in ${WORLDS:-1 8}; do
  PT_TUNE=roundlog=${ROUNDLOG:-1}${TUNE:+,$TUNE} timeout -k 10 300 python3 tools/rank_sim.py --worlds $w --ranks ${RANKS:-first} --steps ${STEPS:-4} > $O/w$w.jsonl 2> $O/w$w.err || { echo "FAILED w$w"; tail -5 $O/w$w.err; exit 1; }
  cat $O/w$w.jsonl
done
