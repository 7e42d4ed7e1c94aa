# Round 5 A/B of PT_TUNE variants on one rank's 256-spp pass (tools/pass_log.py, no log):
# VARS="name:key=v+key=v[:builddir] ..." ("-" = defaults), at "world:rank" points PTS, REPEAT
# interleaved repeats.  Output: gpurun_out/r5ab/<tag>.jsonl, one summary line per variant.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ab || exit 1
O=gpurun_out/r5ab/${TAG:-ab}.jsonl
: > $O
for rep in $(seq 1 ${REPEAT:-2}); do
  for spec in $VARS; do
    IFS=: read name tune vlib <<< "$spec"
    [ "$tune" = "-" ] && tune=""
    for pt in ${PTS:-8:0 8:3 4:0 1:0}; do
      IFS=: read w r <<< "$pt"
      line=$(PT_LIB=raytracing-course_amd/${vlib:-${LIB:-build}}/libpt.so timeout -k 10 120 python3 tools/pass_log.py --world $w --rank $r --level 0 --tune "$(echo $tune | tr '+' ',')" 2> gpurun_out/r5ab/last.err | tail -1) || { echo FAIL $name $pt; tail -5 gpurun_out/r5ab/last.err; exit 1; }
      echo "{\"var\": \"$name\", \"rep\": $rep, \"pt\": \"$pt\", \"r\": $line}" >> $O
    done
  done
done
python3 - "$O" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    x = json.loads(l); d[(x["var"], x["pt"])].append(x["r"]["pass_ms"])
vs = sorted({k[0] for k in d}, key=lambda v: [k[0] for k in d].index(v))
pts = sorted({k[1] for k in d}, key=lambda p: [k[1] for k in d].index(p))
print("var " + " ".join("%12s" % p for p in pts))
for v in vs:
    print(v + " " + " ".join("%12s" % "/".join("%.1f" % t for t in d[(v, p)]) for p in pts))
PY
