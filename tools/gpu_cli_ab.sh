# drop-in CLI (progress bar on, the run.sh default) on config 3 over two builds,
# alternating: wall time, kernel time, image md5 and the number of bar lines
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/cli || exit 1
for exe in ${EXES:-build_old build build_old build}; do
  s=$(date +%s%N)
  PT_STATS=1 timeout -k 10 120 raytracing-course_amd/$exe/pt_render scenes/gen/c3.txt /tmp/c3_$exe.ppm > gpurun_out/cli/$exe.out 2> gpurun_out/cli/$exe.err || { echo FAIL $exe; exit 1; }
  e=$(date +%s%N)
  echo "$exe wall_ms $(( (e - s) / 1000000 )) $(tail -1 gpurun_out/cli/$exe.err) md5 $(md5sum < /tmp/c3_$exe.ppm | cut -c1-12) bar_lines $(grep -c Loading gpurun_out/cli/$exe.out)"
done
