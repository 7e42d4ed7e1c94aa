#!/usr/bin/env python3
"""One rank's 256-spp pass of a config, with the library's per-round log.

Runs rank r of world N (a session alone on the local GPU, as one GPU of an N-GPU
render sees it) for ONE coalesced pass of --spp samples (the metric's job: every
pixel 256 spp), after one warm-up pass, under PT_TUNE roundlog=<level> (plus --tune):
each round's chains in and out, its kind (full / low, +side for an early
cooperative launch), wall ms and rays, and at level 3 the unfinished pixels'
remaining samples.  Prints the log lines of the timed pass and one JSON summary
(--first: also the process's first pass, whose code and buffers are cold).
  python tools/pass_log.py [--config c3] [--world 8] [--rank 0] [--spp 256] [--level 2]
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, REPO)
    import bench
    pt = bench.load_ptrace()
    with pt.Scene.load(bench.scene_file(a.config)) as s:
        s.prepare()
        for it in range(2):
            ss = pt.Session(s, device=0, rank=a.rank, world=a.world)
            ss.sync()
            print("PASS_START %d" % it, file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            ss.trace(a.spp)
            ss.sync()
            dt = time.perf_counter() - t0
            st = ss.stats()
            print("PASS_END %d" % it, file=sys.stderr, flush=True)
            if it == 1 or a.first:
                print(json.dumps({"pass": it, "world": a.world, "rank": a.rank, "spp": a.spp, "pass_ms": dt * 1e3,
                                  "rays": st["rays"], "mray_s": st["rays"] / dt / 1e6, "rounds": st["rounds"],
                                  "coop_ms": st["coop_ms"], "coop_launches": st["coop_launches"],
                                  "coop_rays": st["coop_rays"], "isect_ms": st["isect_ms"],
                                  "kernel_ms": st["kernel_ms"], "tune": os.environ.get("PT_TUNE", "")}))
            ss.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--level", type=int, default=2)
    ap.add_argument("--tune", default="")
    ap.add_argument("--first", action="store_true", help="also the first (cold) pass of the process")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    tune = "roundlog=%d" % a.level + ("," + a.tune if a.tune else "")
    env = dict(os.environ, PT_TUNE=tune)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"] + sys.argv[1:], env=env,
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-2000:])
        sys.exit(r.returncode)
    lines = r.stderr.splitlines()
    if a.first:
        for ln in lines[lines.index("PASS_START 0") + 1:lines.index("PASS_END 0")]:
            print("pass0 " + ln)
    i0 = lines.index("PASS_START 1")
    i1 = lines.index("PASS_END 1")
    for ln in lines[i0 + 1:i1]:
        print(ln)
    print(r.stdout.strip())


if __name__ == "__main__":
    main()
