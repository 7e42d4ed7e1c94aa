cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/micro &&
timeout -k 10 60 tools/micro/atomics > gpurun_out/micro/atomics.txt 2>&1 && cat gpurun_out/micro/atomics.txt &&
PT_WGPROF=/tmp/wg8.bin timeout -k 10 300 python3 tools/rank_sim.py --worlds 8 --steps 1 > gpurun_out/micro/w8.jsonl 2>&1 &&
python3 tools/wg_iters.py /tmp/wg8.bin 768 && rm -f /tmp/wg8.bin &&
PT_WGPROF=/tmp/wg1.bin timeout -k 10 300 python3 tools/rank_sim.py --worlds 1 --steps 1 > gpurun_out/micro/w1.jsonl 2>&1 &&
python3 tools/wg_iters.py /tmp/wg1.bin 768
