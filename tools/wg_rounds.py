#!/usr/bin/env python3
"""Per-round spans of a path-engine PT_TUNE wgprof dump, next to the round log (n in)."""
import re
import sys
import numpy as np

a = np.fromfile(sys.argv[1], np.uint64).reshape(-1, int(sys.argv[2]), 64).astype(np.int64)
L = [l for l in open(sys.argv[3]) if l.startswith("round")]
tot = 0.0
for i, r in enumerate(a):
    rr = r[r[:, 0] > 0]
    span = (rr[:, 1].max() - rr[:, 0].min()) / 100.0 if len(rr) else 0.0
    tot += span
    m = re.search(r"in fresh (\d+) carry (\d+)", L[i]) if i < len(L) else None
    n = int(m.group(1)) + int(m.group(2)) if m else -1
    if i < 400:
        g = max(len(rr), 1)
        print("round %3d n_in %7d span %8.0f us  WG dur p50 %6.0f max %6.0f  trips/QW %6.0f lane util %.2f sleep %.2f "
              "pulled %7d rays(lane0) %9d budget exits %.2f" % (
            i, n, span, np.median((rr[:, 1] - rr[:, 0]) / 100.0) if len(rr) else 0,
            ((rr[:, 1] - rr[:, 0]) / 100.0).max() if len(rr) else 0, rr[:, 2].sum() / (2.0 * g),
            rr[:, 3].sum() / max(64.0 * rr[:, 2].sum(), 1), rr[:, 4].sum() / max(rr[:, 2].sum(), 1),
            rr[:, 11].sum(), rr[:, 6].sum(), rr[:, 12].sum() / (2.0 * g)))
print("total span ms %.1f" % (tot / 1e3))
