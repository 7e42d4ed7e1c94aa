# bench.py's own N-rank launch on a one-GPU box: `--gpus 2 --same-device` (every
# rank on cuda:0, gloo collectives) must start 2 ranks unaided and gather the
# same framebuffer as one rank advancing every pixel by the same samples.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dist
timeout -k 10 300 python3 bench.py --gpus 2 --same-device --dist-backend gloo --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/dist/n2.json 2> gpurun_out/dist/n2.err && echo N2_OK &&
timeout -k 10 300 python3 bench.py --gpus 1 --spp-per-step 32 --steps 2 --warmup 1 --no-cpu-baseline --no-wallclock \
  > gpurun_out/dist/n1.json 2> gpurun_out/dist/n1.err && echo N1_OK &&
python3 - <<'PY'
import json
L = lambda p: json.loads([l for l in open(p) if l.startswith("{")][-1])
a, b = L("gpurun_out/dist/n2.json"), L("gpurun_out/dist/n1.json")
print("n2: n_gpus=%d md5=%s rays=%d launched_by=%s | n1: md5=%s rays=%d" % (
    a["n_gpus"], a["framebuffer_md5"], a["rays"], a["distributed"]["launched_by"], b["framebuffer_md5"], b["rays"]))
assert a["n_gpus"] == 2 and a["framebuffer_md5"] == b["framebuffer_md5"] and a["rays"] == b["rays"]
print("DIST_MATCH")
PY
