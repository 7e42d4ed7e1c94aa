#!/usr/bin/env python3
"""Wall-clock to PPM of the drop-in CLI (run.sh <scene.txt> <out.ppm>) on the
BASELINE configs: process start -> PPM closed (parse + reference BVH build +
aux BVH + upload + full render + tonemap + P6 write), one GPU; the process's exit
after the PPM (the runtime's teardown) is in wall_to_exit_s.  Configs 1 and 2
are also checked against the reference's full-resolution md5s.
  python tools/wallclock.py [c1 c2 c3 c4_metal c4_glass]
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scenes"))
import make_scene  # noqa: E402

GOLDEN_MD5 = {"c1": "99f1bc9386a22892970f058bfa8114c7", "c2": "a16f6cf46a6443244ecbd0c9d856c295"}


def scene(config):
    p = os.path.join(REPO, "scenes", "gen", config + ".txt")
    if not os.path.exists(p):
        os.makedirs(os.path.dirname(p), exist_ok=True)
        make_scene.make(config, p + ".tmp")
        os.replace(p + ".tmp", p)
    return p


def main():
    configs = sys.argv[1:] or ["c1", "c2", "c3", "c4_metal", "c4_glass"]
    out_dir = os.environ.get("TMPDIR", "/tmp")
    for c in configs:
        src = scene(c)
        out = os.path.join(out_dir, "pt_%s.ppm" % c)
        env = dict(os.environ, PT_STATS="2", PT_QUIET="1")
        u0 = time.time()
        t0 = time.perf_counter()
        r = subprocess.run([os.path.join(REPO, "run.sh"), src, out], env=env, capture_output=True, text=True)
        wall_exit = time.perf_counter() - t0
        # the metric stops when the PPM is closed (the CLI's PT_STATS=2 stamp); the exit after it apart
        um = re.search(r"unix_main=([\d.]+) unix_written=([\d.]+)", r.stderr)
        wall = float(um.group(2)) - u0 if um else wall_exit
        if r.returncode != 0:
            print(json.dumps({"config": c, "error": r.stderr.strip()[-400:]}), flush=True)
            sys.exit(1)
        m = dict(re.findall(r"(\w+(?:/\w+)?)=([\d.]+)", r.stderr))
        md5 = hashlib.md5(open(out, "rb").read()).hexdigest()
        os.unlink(out)
        rays = int(m.get("rays", 0))
        rec = {"config": c, "wall_to_ppm_s": wall, "wall_to_exit_s": wall_exit, "rays": rays, "render_ms": float(m.get("wall_ms", 0)),
               "kernel_ms": float(m.get("kernel_ms", 0)), "mray_s_wall": rays / wall / 1e6,
               "mray_s_render": rays / (float(m.get("wall_ms", 1)) * 1e3), "ppm_md5": md5,
               "fallbacks": int(m.get("fallbacks", 0)), "rounds": int(m.get("rounds", 0))}
        ph = re.search(r"phases_ms: (.*)", r.stderr)
        if ph:
            rec["phases_ms"] = {k: float(v) for k, v in re.findall(r"(\w+)=([\d.]+)", ph.group(1))}
        if c in GOLDEN_MD5:
            rec["md5_matches_reference"] = md5 == GOLDEN_MD5[c]
        ref = os.path.join(REPO, "oracle", "_ref", "raytracing_hw5")
        if c in ("c1",) and os.path.exists(ref):
            # the reference CLI on the same scene and host (hw5/run.sh), for the same wall-clock
            t0 = time.perf_counter()
            rr = subprocess.run([ref, src, out], capture_output=True)
            rec["reference_wall_s"] = time.perf_counter() - t0
            if rr.returncode == 0:
                rec["reference_md5_same"] = hashlib.md5(open(out, "rb").read()).hexdigest() == md5
                os.unlink(out)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
