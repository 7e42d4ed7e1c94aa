# Round-3 verification of the committed tree: smoke, parity suite, rocprofv3
# kernel trace + PMC passes + the default bench line (tools/gpu_profile.sh),
# every rank of N = 2, 4, 8 (rank_sim --ranks all), round logs of rank 0 of 8.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3 || exit 1
O=gpurun_out/r3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/gpu_profile.sh || { echo PROFILE_FAIL; exit 1; }
timeout -k 10 600 python3 tools/rank_sim.py --worlds 2 4 8 --ranks all --steps ${STEPS:-4} > $O/ranksim_all.jsonl 2> $O/ranksim_all.err || { echo SIM_FAIL; tail -20 $O/ranksim_all.err; exit 1; }
grep -E 'min_mray' $O/ranksim_all.jsonl
for k in 1 2; do
  PT_TUNE=roundlog=$k timeout -k 10 120 python3 tools/rank_sim.py --worlds 8 --steps 4 > $O/roundlog${k}_w8.jsonl 2> $O/roundlog${k}_w8.txt || { echo RL_FAIL; exit 1; }
done
