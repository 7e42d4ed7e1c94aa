#!/usr/bin/env python3
"""Summarise a PT_WGPROF dump (9 x u64 per isect workgroup per round: start, end
(100 MHz realtime), HW_ID, XCC_ID, loop trips, and with a -DPT_WPROF build the
wave-0 cycles in refill / step, active lane-trips, aux lane-trips) -> per-round
span, trips, time per trip, lane utilisation."""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], np.uint64).reshape(-1, int(sys.argv[2]), 9).astype(np.int64)
rows = []
for r in a:
    r = r[r[:, 0] > 0]
    if len(r) == 0:
        continue
    span = (r[:, 1].max() - r[:, 0].min()) / 100.0
    dur = (r[:, 1] - r[:, 0]) / 100.0
    trips = r[:, 4]
    util = r[:, 7].sum() / max(64 * trips.sum(), 1)
    refill = r[:, 5].sum() / max(r[:, 5].sum() + r[:, 6].sum(), 1)
    rows.append((span, trips.max(), trips.mean(), dur.mean(), util, refill, r[:, 8].sum() / max(r[:, 7].sum(), 1)))
R = np.array(rows)
print("rounds %d" % len(R))
for name, k in [("span us", 0), ("max trips", 1), ("mean trips", 2), ("mean WG dur us", 3), ("lane util", 4),
                ("refill cycle frac", 5), ("aux frac of active", 6)]:
    v = R[:, k]
    print("  %-20s mean %9.3f p10 %9.3f p50 %9.3f p90 %9.3f" % (name, v.mean(), *np.percentile(v, [10, 50, 90])))
print("  us per trip (span/max trips) p50 %.2f; total span ms %.1f" % (np.median(R[:, 0] / np.maximum(R[:, 1], 1)), R[:, 0].sum() / 1e3))
