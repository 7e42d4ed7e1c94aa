# cooperative engine phase profile (-DPT_CPROF build in build_cprof) + round log: COOPS thresholds x WORLDS
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/cprof || exit 1
for c in ${COOPS:-131072}; do
  PT_LIB=raytracing-course_amd/${CLIB:-build_cprof}/libpt.so PT_TUNE=cprof=1,roundlog=1,coop=$c${TUNE_EXTRA:+,$TUNE_EXTRA} timeout -k 10 300 python3 tools/rank_sim.py --worlds ${WORLDS:-8} --steps ${STEPS:-1} > gpurun_out/cprof/c$c.jsonl 2> gpurun_out/cprof/c$c.err || { echo FAIL; tail -3 gpurun_out/cprof/c$c.err; exit 1; }
  echo "== coop=$c"; cat gpurun_out/cprof/c$c.jsonl; grep -E "coop chains|rounds_ms" gpurun_out/cprof/c$c.err
done
