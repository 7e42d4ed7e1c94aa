# per-round isect workgroup timelines with the PT_WPROF build (build_wprof/libpt.so)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/wprof || exit 1
for spec in ${SPECS:-w8s64:8:64 w8s8:8:8 w1s64:1:64}; do
  IFS=: read name w s <<< "$spec"
  rm -f /tmp/wg.bin
  PT_LIB=raytracing-course_amd/build_wprof/libpt.so PT_STRAGGLER=$s PT_WGPROF=/tmp/wg.bin timeout -k 10 300 python3 tools/rank_sim.py --worlds $w --steps 1 > gpurun_out/wprof/$name.jsonl 2>&1 || exit 1
  echo "== $name $(cat gpurun_out/wprof/$name.jsonl | tail -1)"
  python3 tools/wg_iters.py /tmp/wg.bin 768 || exit 1
done
