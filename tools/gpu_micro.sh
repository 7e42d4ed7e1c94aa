# atomics micro-benchmark (tools/micro/atomics.hip; build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/atomics tools/micro/atomics.hip)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/micro &&
timeout -k 10 60 tools/micro/atomics > gpurun_out/micro/atomics.txt 2>&1 && cat gpurun_out/micro/atomics.txt
