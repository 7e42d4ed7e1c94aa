# PMC counter passes over the bench (one counter group per pass), plus the counter list.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
i=0
for grp in "${@}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
    python3 bench.py --no-cpu-baseline --steps ${STEPS:-1} --warmup 0 > $OUT/b$i.json 2> $OUT/b$i.err || echo "pass $i FAILED"
  echo "pass $i ($grp) ok"
done
