#!/bin/sh
# Build the UNMODIFIED reference hw5 renderer (FeggieBoss/raytracing-course) from
# its sources where they lie under /root/reference, straight with g++ (no cmake).
# Flags mirror hw5/CMakeLists.txt:5 (-std=c++17 -O3) + Release (-DNDEBUG) + the
# OpenMP link of hw5/CMakeLists.txt:23-24.  Output goes ONLY to oracle/_ref/
# (git-ignored; it travels to the GPU box with the gpurun snapshot).
#
#   oracle/_ref/raytracing_hw5      the reference CLI (main.cpp), used as the
#                                   bench.py cpu_baseline ("kind": "reference")
#   oracle/_ref/ref_harness         reference sources + oracle/ref_harness.cpp,
#                                   used only to generate tests/golden fixtures
set -e
REF=${REF:-/root/reference/hw5}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
mkdir -p "$OUT"
if [ ! -d "$REF/src" ]; then
  echo "reference not present at $REF; skipping reference build" >&2
  exit 0
fi
CXX=${CXX:-g++}
FLAGS="-std=c++17 -O3 -DNDEBUG -fopenmp -w -I$REF/include -I$REF"
$CXX $FLAGS "$REF"/src/*.cpp -o "$OUT/raytracing_hw5"
# harness: every reference TU except main.cpp, plus our fixture dumper.
SRCS=""
for f in "$REF"/src/*.cpp; do
  case "$f" in */main.cpp) ;; *) SRCS="$SRCS $f" ;; esac
done
$CXX $FLAGS $SRCS "$HERE/ref_harness.cpp" -o "$OUT/ref_harness"
echo "built $OUT/raytracing_hw5 $OUT/ref_harness"
