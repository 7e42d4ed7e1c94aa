#!/usr/bin/env python3
"""Wall-clock to PPM of the drop-in CLI at N GPUs, measured on ONE GPU.

`PT_NGPU=N run.sh <scene> <out.ppm>` drives N sessions (rank g of N, tiles
(tx + ty) % N == g) from one process: one host thread per GPU sets up its
session (the device's scene upload, the session buffers) and renders it, then
the packed 8-bit tiles are gathered.  With PT_TUNE=same_device=2 every session
lives on device 0 and, once all are set up, the ranks render ONE AFTER ANOTHER,
so each rank's render time (PT_STATS=2) is its time alone on a GPU.  The
projection for N real GPUs replaces the serialized renders by the slowest one:

    projected = measured wall - sum(rank render) + max(rank render)

(set-up still runs N threads against one device here, so its figure is an
upper bound for N devices; the host gather stands in for ncclGather, which moves
the same 6.2 MB (c3) over xGMI).  The PPM's md5 is checked against N = 1.
  python tools/wallclock_ngpu.py [--config c3] [--ngpu 1 2 4 8] [--repeat 2]
"""
import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def run(src, n, tune):
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), "pt_wall_n%d_%d.ppm" % (n, os.getpid()))
    env = dict(os.environ, PT_STATS="2", PT_QUIET="1", PT_NGPU=str(n))
    if n > 1:
        env["PT_TUNE"] = tune
        env["PT_GATHER"] = "host"
    t0 = time.perf_counter()
    u0 = time.time()
    r = subprocess.run([os.path.join(REPO, "run.sh"), src, out], env=env, capture_output=True, text=True, timeout=300)
    wall = time.perf_counter() - t0
    u1 = time.time()
    um = re.search(r"unix_main=([\d.]+) unix_written=([\d.]+)", r.stderr)
    # before main(): exec + dynamic loading; after the PPM is closed: process exit (the runtime's teardown)
    before_main = float(um.group(1)) - u0 if um else None
    after_write = u1 - float(um.group(2)) if um else None
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-400:])
    md5 = hashlib.md5(open(out, "rb").read()).hexdigest()
    os.unlink(out)
    ranks = [{k: float(v) for k, v in re.findall(r"(\w+)=([\d.]+)", ln)}
             for ln in r.stderr.splitlines() if ln.startswith("pt_render rank")]
    cli = {}
    for ln in r.stderr.splitlines():
        if ln.startswith("phases_ms:"):
            cli = {k: float(v) for k, v in re.findall(r"(\w+)=([\d.]+)", ln)}
    g = re.search(r"pt_render gather_ms=([\d.]+)", r.stderr)
    st = dict(re.findall(r"(\w+(?:/\w+)?)=([\d.]+)", [ln for ln in r.stderr.splitlines() if ln.startswith("rays=")][-1]))
    renders = [x["render_ms"] for x in ranks]
    proj = wall - sum(renders) / 1e3 + max(renders) / 1e3
    return {"ngpu": n, "wall_s": wall, "projected_wall_s": proj, "rays": int(st["rays"]), "ppm_md5": md5,
            "before_main_s": before_main, "after_ppm_s": after_write,
            "cli_phases_ms": cli, "gather_ms": float(g.group(1)) if g else None,
            "setup_ms_max": max(x["setup_ms"] for x in ranks), "setup_ms": [x["setup_ms"] for x in ranks],
            "scene_upload_ms": [x["scene_upload_ms"] for x in ranks], "render_ms": renders,
            "render_ms_max": max(renders), "resolve_ms": [x["resolve_ms"] for x in ranks],
            "coop_ms": [x.get("coop_ms") for x in ranks], "isect_ms": [x.get("isect_ms") for x in ranks],
            "rounds": [x.get("rounds") for x in ranks], "rank_rays": [x.get("rays") for x in ranks]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--ngpu", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--tune", default="same_device=2")
    a = ap.parse_args()
    src = bench.scene_file(a.config)
    base = None
    for _ in range(a.repeat):
        for n in a.ngpu:
            rec = run(src, n, a.tune)
            rec["config"] = a.config
            if n == 1:
                base = rec["ppm_md5"]
            rec["md5_same_as_n1"] = base is None or rec["ppm_md5"] == base
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
