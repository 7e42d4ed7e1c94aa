# bench.py (no CPU baseline) over library variants: VARS="name:libdir ..."
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/benchab || exit 1
for spec in $VARS; do
  IFS=: read name lib <<< "$spec"
  PT_LIB=raytracing-course_amd/$lib/libpt.so timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/benchab/$name.json 2> gpurun_out/benchab/$name.err || { echo "FAILED $name"; tail -3 gpurun_out/benchab/$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/benchab/$name.json'))
print('$name: %.1f Mray/s, %.1f ms/step, fallbacks %d, launch %.3f ms' % (d['value'], d['ms_per_step'], d['fallbacks'], d['roofline']['launch_ms']))"
done
