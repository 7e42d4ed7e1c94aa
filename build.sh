#!/bin/sh
# Drop-in for hw5/build.sh:1-5 (the reference builds build/raytracing_hw5 with cmake):
# builds libpt.so (HIP kernels for gfx950 + C ABI) and the pt_render CLI.
set -e
cd "$(dirname "$0")"
make -s -j"${MAX_JOBS:-8}" -C raytracing-course_amd
