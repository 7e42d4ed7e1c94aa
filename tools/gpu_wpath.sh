# path-engine diagnostics (PT_WPROF builds): LIBS="name:libdir[:key=v+key=v] ..." x WORLDS
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/wprof || exit 1
for spec in ${LIBS:-wprof:build_wprof}; do
  IFS=: read name lib tune <<< "$spec"
  for w in ${WORLDS:-8 1}; do
    rm -f /tmp/wg.bin
    PT_LIB=raytracing-course_amd/$lib/libpt.so PT_TUNE=wgprof=/tmp/wg.bin$(echo "${tune:+,$tune}" | tr '+' ',') timeout -k 10 300 python3 tools/rank_sim.py --worlds $w --steps ${STEPS:-1} > gpurun_out/wprof/${name}_w$w.jsonl 2> gpurun_out/wprof/${name}_w$w.err || exit 1
    echo "== $name w$w $(tail -1 gpurun_out/wprof/${name}_w$w.jsonl)"
    python3 tools/wg_path.py /tmp/wg.bin ${NWG:-1024} || exit 1
    python3 tools/wg_tail.py /tmp/wg.bin ${NWG:-1024} > gpurun_out/wprof/${name}_tail_w$w.txt
    python3 tools/wg_rounds.py /tmp/wg.bin ${NWG:-1024} gpurun_out/wprof/${name}_w$w.err > gpurun_out/wprof/${name}_rounds_w$w.txt
  done
done
