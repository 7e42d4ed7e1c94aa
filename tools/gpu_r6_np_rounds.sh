# Round 6: the concurrent-session parity check (tools/gpu_r5_npcheck.sh, TUNES) and then
# one-GPU round logs of rank 0 of 1 and of 8 (tools/pass_log.py --level 2).
# Output: gpurun_out/np, gpurun_out/rl
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/rl gpurun_out/np || exit 1
[ "${NP:-1}" = "1" ] && { bash tools/gpu_r5_npcheck.sh | tee gpurun_out/np/summary.txt
grep -q "rc=0" gpurun_out/np/summary.txt || exit 1; }
for pt in 1:0 8:0; do
  IFS=: read w r <<< "$pt"
  timeout -k 10 120 python3 tools/pass_log.py --world $w --rank $r --level 2 > gpurun_out/rl/w${w}r${r}.txt 2>&1 || { echo RL_FAIL $pt; tail -5 gpurun_out/rl/w${w}r${r}.txt; exit 1; }
done
echo RL_OK
