#!/bin/sh
# Drop-in for hw5/run.sh:1-2:  ./run.sh <scene.txt> <out.ppm>
# Extras via env: PT_NGPU, PT_DEVICE, PT_SPP_LAUNCH, PT_QUIET, PT_STATS (see cli/main.cpp).
exec "$(dirname "$0")/raytracing-course_amd/build/pt_render" "$1" "$2"
