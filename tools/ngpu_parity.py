#!/usr/bin/env python3
"""pt_render(ngpu = N) on one device under several PT_TUNE settings, each REPEAT
times: the gathered image's md5 and the ray count against the reference's
(tests/golden manifest).  A diagnostics companion of
test_render_ngpu_sessions_on_one_device for settings the test does not take.
  python tools/ngpu_parity.py --cfg c2 --ngpu 2 --repeat 3 --tunes same_device=1 same_device=1,early=0
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import _util as U  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="c2")
    ap.add_argument("--ngpu", type=int, default=2)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--tunes", nargs="+", default=["same_device=1"])
    a = ap.parse_args()
    pt = bench.load_ptrace()
    full = U.manifest()["full"][a.cfg]
    bad = 0
    with pt.Scene.load(U.scene_path(a.cfg)) as s:
        s.prepare()
        w, h = s.info["width"], s.info["height"]
        for r in range(a.repeat):
            for t in a.tunes:
                os.environ["PT_TUNE"] = t
                try:
                    rgb, _, st = s.render(ngpu=a.ngpu)
                except pt.PTError as e:   # (e.g. the resolve's lost-chain error)
                    bad += 1
                    print(json.dumps({"repeat": r, "tune": t, "ok": False, "error": str(e)}), flush=True)
                    continue
                ppm = b"P6\n%d %d\n255\n" % (w, h) + rgb.tobytes()
                ok = U.md5(ppm) == full["md5"] and st["rays"] == full["rays"] and st["errors"] == 0
                bad += 0 if ok else 1
                print(json.dumps({"repeat": r, "tune": t, "ok": ok, "rays": st["rays"], "ref_rays": full["rays"],
                                  "errors": st["errors"]}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
