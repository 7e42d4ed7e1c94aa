# iteration loop: GPU parity tests, then the rank simulation of the N-GPU bench ($ENGINES)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/iter &&
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/iter/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/iter/pytest.log; [ $rc -eq 0 ] || exit $rc
for eng in ${ENGINES:-path}; do
PT_ENGINE=$eng timeout -k 10 300 python3 tools/rank_sim.py --worlds ${WORLDS:-1 2 4 8} --steps ${STEPS:-2} > gpurun_out/iter/rank_sim_$eng.jsonl 2> gpurun_out/iter/rank_sim_$eng.err || exit $?
python3 -c "
import json
for l in open('gpurun_out/iter/rank_sim_$eng.jsonl'):
    d=json.loads(l); print('$eng w%d %.1f Mray/s %.3f ms/round %d rounds/step %.0f rays/round' % (d['world'], d['mray_s'], d['isect_ms_per_round'], d['rounds_per_step'], d['rays_per_round']))
"
done
