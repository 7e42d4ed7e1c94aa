# The multi-process bench path on a one-GPU box: N ranks on cuda:0 with gloo
# collectives; the gathered framebuffer must equal the one-rank render of the
# same samples (spp per rank per step = 16*N, so N=1 uses 16*N too).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/dist || exit 1
for n in ${NS:-2 7}; do
  spp=$((16 * n))
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --spp-per-step $spp --no-cpu-baseline --no-wallclock > gpurun_out/dist/w1_$n.json 2> gpurun_out/dist/w1_$n.err || { echo "FAIL w1 $n"; tail -5 gpurun_out/dist/w1_$n.err; exit 1; }
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 --no-cpu-baseline --no-wallclock --dist-backend gloo --same-device > gpurun_out/dist/wn_$n.json 2> gpurun_out/dist/wn_$n.err || { echo "FAIL wn $n"; tail -20 gpurun_out/dist/wn_$n.err; exit 1; }
  python3 -c "
import json
a=json.loads(open('gpurun_out/dist/w1_$n.json').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/dist/wn_$n.json').read().strip().splitlines()[-1])
print('N=$n', 'w1 md5', a['framebuffer_md5'], 'rays', int(a['rays']), '| wN md5', b['framebuffer_md5'], 'rays', int(b['rays']), 'n_gpus', b['n_gpus'], 'value', round(b['value'],1), 'SAME' if a['framebuffer_md5']==b['framebuffer_md5'] and a['rays']==b['rays'] else 'DIFFERENT')"
done
