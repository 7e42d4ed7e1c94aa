#!/usr/bin/env python3
"""Per-round breakdown of a path-engine PT_TUNE wgprof dump (64 u64 per WG per round)."""
import sys
import numpy as np

G = int(sys.argv[2])
a = np.fromfile(sys.argv[1], np.uint64).reshape(-1, G, 64).astype(np.float64)
sel = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else range(len(a))
for i in sel:
    r = a[i]
    r = r[r[:, 0] > 0]
    if not len(r):
        continue
    span = (r[:, 1].max() - r[:, 0].min()) / 100.0
    t = r.sum(0)
    print("round %d: span %.0f us, WGs %d; QW trips/wave %.0f, util %.3f, sleep %.3f, cyc/trip %.0f; queries %d (%.0f per WG), "
          "lat %.0f cyc, trips/query %.1f; SW batches/WG %.0f, items/batch %.1f, spins/batch %.1f, cyc/batch %.0f"
          % (i, span, len(r), t[2] / (3 * len(r)), t[3] / max(64 * t[2], 1), t[4] / max(t[2], 1), t[16] / max(t[2], 1),
             t[18], t[18] / len(r), t[17] / max(t[18], 1), t[19] / max(t[18], 1), t[7] / len(r), t[8] / max(t[7], 1),
             t[9] / max(t[7], 1), t[10] / max(t[7], 1)))
