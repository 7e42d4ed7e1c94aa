# per-round chain counts and pixel lag (PT_TUNE roundlog=2) of REPS rank_sim runs: WORLDS, REPS, LIB, TUNE
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/roundlog || exit 1
for i in $(seq 1 ${REPS:-4}); do
  for w in ${WORLDS:-8}; do
    PT_LIB=raytracing-course_amd/${LIB:-build}/libpt.so PT_TUNE=roundlog=2${TUNE:+,$TUNE} timeout -k 10 300 python3 tools/rank_sim.py --worlds $w --steps ${STEPS:-2} > gpurun_out/roundlog/w${w}_$i.jsonl 2> gpurun_out/roundlog/w${w}_$i.err || exit 1
    echo "== w$w rep $i: $(python3 -c "import json; d=json.loads(open('gpurun_out/roundlog/w${w}_$i.jsonl').readlines()[-1]); print('%.1f Mray/s coop %.1f ms share %.3f' % (d['mray_s'], d['coop_ms_per_step'], d['coop_ray_share']))")"
    grep -E "^round" gpurun_out/roundlog/w${w}_$i.err | tail -${TAILN:-6}
  done
done
