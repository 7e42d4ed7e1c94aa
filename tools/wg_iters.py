#!/usr/bin/env python3
"""Summarise a PT_WGPROF dump (9 x u64 per isect workgroup per round: start, end
(100 MHz realtime), HW_ID, XCC_ID, loop trips, [PT_WPROF cycles]) -> per-round
span, trips and time per trip."""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], np.uint64).reshape(-1, int(sys.argv[2]), 9).astype(np.int64)
spans, trips, wgdur = [], [], []
for r in a:
    r = r[r[:, 0] > 0]
    if len(r) == 0:
        continue
    spans.append((r[:, 1].max() - r[:, 0].min()) / 100.0)
    trips.append(r[:, 4].max())
    wgdur.append(((r[:, 1] - r[:, 0]) / 100.0).mean())
spans, trips, wgdur = map(np.array, (spans, trips, wgdur))
print("rounds %d: span us mean %.1f p50 %.1f p90 %.1f; max trips/WG mean %.1f p50 %.0f; mean WG dur %.1f us; us/trip %.2f"
      % (len(spans), spans.mean(), np.median(spans), np.percentile(spans, 90), trips.mean(), np.median(trips),
         wgdur.mean(), (spans / np.maximum(trips, 1)).mean()))
