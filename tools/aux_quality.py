#!/usr/bin/env python3
"""Per-query work of the replay traversal on the CPU (host self-test render).

Renders a grid of windows of a bench config through the host build of the
wavefront query (pt_query.h, the same code the GPU runs) with PT_TUNE
qstats=<file>, and prints the mean aux-node visits, reference-node tests and
primitive tests per query plus their tail.  Used to compare auxiliary-BVH
builds without a GPU:
  python tools/aux_quality.py [--config c3] [--grid 6x4] [--win 32] [--spp 2]
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--grid", default="6x4")
    ap.add_argument("--win", type=int, default=32)
    ap.add_argument("--spp", type=int, default=2)
    a = ap.parse_args()
    gx, gy = (int(v) for v in a.grid.split("x"))
    qfile = os.path.join(tempfile.mkdtemp(), "q.bin")
    tune = os.environ.get("PT_TUNE", "")
    os.environ["PT_TUNE"] = (tune + "," if tune else "") + "qstats=" + qfile
    pt = bench.load_ptrace()
    rows = []
    with pt.Scene.load(bench.scene_file(a.config)) as s:
        s.prepare()
        W, H = s.info["width"], s.info["height"]
        for j in range(gy):
            for i in range(gx):
                x0 = (W - a.win) * i // max(gx - 1, 1)
                y0 = (H - a.win) * j // max(gy - 1, 1)
                s.selftest_render_host(x0, y0, a.win, a.win, spp=a.spp)
                rows.append(np.fromfile(qfile, dtype=np.uint32).reshape(-1, 4))
    q = np.concatenate(rows)
    aux, nodes, pt_ = q[:, 0].astype(np.float64), q[:, 1].astype(np.float64), (q[:, 2] & 0x7fffffff).astype(np.float64)
    out = {
        "queries": int(len(q)),
        "aux_per_query": aux.mean(),
        "aux_p99": float(np.percentile(aux, 99)),
        "aux_max": float(aux.max()),
        "nodes_per_query": nodes.mean(),
        "ptests_per_query": pt_.mean(),
        "bytes_per_query": 128 * aux.mean() + 32 * nodes.mean() + 48 * pt_.mean(),
        "exact": int((q[:, 2] >> 31).sum()),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
