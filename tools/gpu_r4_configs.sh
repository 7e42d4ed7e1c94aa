# Current-tree rates of every BASELINE config: the drop-in CLI's wall-clock to PPM
# on c1, c2 (md5 vs the reference), c3 and c4 metal/glass (1024 spp), one GPU; then
# config 5's per-GPU share (every rank of 8, 4K frame, 512-spp passes: rank_sim).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/cfg || exit 1
O=gpurun_out/cfg
timeout -k 10 600 python3 tools/wallclock.py c1 c2 c3 c4_metal c4_glass > $O/wallclock.jsonl 2> $O/wallclock.err || { echo WALL_FAIL; tail -5 $O/wallclock.err; exit 1; }
python3 -c "
import json
for l in open('$O/wallclock.jsonl'):
    d=json.loads(l); print(d['config'], 'wall %.3f s'%d['wall_to_ppm_s'], 'kernel %.1f ms'%d['kernel_ms'], 'rays', d['rays'], 'Mray/s(kernel) %.0f'%(d['rays']/max(d['kernel_ms'],1e-9)/1e3), d.get('md5_matches_reference',''))"
if [ "${C5:-1}" = "1" ]; then
  timeout -k 10 600 python3 tools/rank_sim.py --config c5 --worlds 8 --ranks all --spp-per-step 16 --steps 4 > $O/c5_rank8.jsonl 2> $O/c5_rank8.err || { echo C5_FAIL; tail -5 $O/c5_rank8.err; exit 1; }
  grep -E 'min_mray' $O/c5_rank8.jsonl
fi
