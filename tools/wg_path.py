#!/usr/bin/env python3
"""Summarise a PT_TUNE wgprof dump of the path engine (-DPT_WPROF build): 64 u64 per
workgroup per round: start, end (100 MHz), QW trips, QW active lane-trips, QW
sleep trips, ring takes, rays, SW batches, SW items, SW spins, SW busy cycles."""
import sys
import numpy as np

G = int(sys.argv[2])
NQ = int(sys.argv[3]) if len(sys.argv) > 3 else 2   # query waves per workgroup (PT_NQ)
a = np.fromfile(sys.argv[1], np.uint64).reshape(-1, G, 64).astype(np.int64)
tot = a.sum(axis=(0, 1))
span = []
for r in a:
    r = r[r[:, 0] > 0]
    if len(r):
        span.append((r[:, 1].max() - r[:, 0].min()) / 100.0)
span = np.array(span)
print("rounds %d, span us mean %.0f p50 %.0f max %.0f, total ms %.1f" % (len(span), span.mean(), np.median(span), span.max(), span.sum() / 1e3))
qw_wave_trips = tot[2]
print("QW: trips/wave-round %.0f, lane util %.3f, sleep frac %.3f, ring takes %d, rays(lane0) %d, rays per wave-trip %.3f"
      % (qw_wave_trips / max(len(span) * G * NQ, 1), tot[3] / max(64 * tot[2], 1), tot[4] / max(tot[2], 1), tot[5], tot[6], tot[6] / max(tot[2], 1)))
print("SW: batches %d, items/batch %.1f, spins/batch %.2f, busy cycles/batch %.0f, SW busy frac of span %.3f (shader clocks / 24 per 100-MHz tick)"
      % (tot[7], tot[8] / max(tot[7], 1), tot[9] / max(tot[7], 1), tot[10] / max(tot[7], 1),
         tot[10] / 24.0 / 100.0 / max(span.sum() * G, 1)))
print("QW trip samples: mean resident %.1f, done-ring %.1f, ray-ring %.1f; chains pulled per WG-round %.1f; waves ending on the budget %.3f"
      % (tot[13] / max(tot[2], 1), tot[14] / max(tot[2], 1), tot[15] / max(tot[2], 1), tot[11] / max(len(span) * G, 1),
         tot[12] / max(len(span) * G * NQ, 1)))
print("QW cycles per trip %.0f (refill part %.0f); query latency %.0f cycles over %.1f trips (%d queries)"
      % (tot[16] / max(tot[2], 1), tot[21] / max(tot[2], 1), tot[17] / max(tot[18], 1), tot[19] / max(tot[18], 1), tot[18]))
print("QW cycles per trip: refill %.0f, step %.0f, done %.0f; trips with aux lanes %.3f, with a replay kind %.3f; lanes stepped per trip %.1f"
      % (tot[21] / max(tot[2], 1), tot[22] / max(tot[2], 1), tot[26] / max(tot[2], 1), tot[23] / max(tot[2], 1),
         tot[24] / max(tot[2], 1), tot[25] / max(tot[2], 1)))
print("SW cycles per batch: shade_item %.0f, next-ray push + publish %.0f, the rest (ring reads, fences) %.0f"
      % (tot[27] / max(tot[7], 1), tot[28] / max(tot[7], 1), (tot[10] - tot[27] - tot[28]) / max(tot[7], 1)))
print("QW step: load wait %.0f + exec %.0f cycles per stepping trip; refill data wait %.0f cycles per refilling trip (%.3f of trips)"
      % (tot[32] / max(tot[2] - tot[4], 1), tot[33] / max(tot[2] - tot[4], 1), tot[34] / max(tot[35], 1), tot[35] / max(tot[2], 1)))
print("SW per batch: ring read wait %.0f; shade_item phases: pixel+prim %.0f, vertex %.0f, fold+sum %.0f, next ray+store %.0f"
      % (tot[36] / max(tot[7], 1), tot[40] / max(tot[7], 1), tot[41] / max(tot[7], 1), tot[42] / max(tot[7], 1),
         tot[43] / max(tot[7], 1)))
if tot[54:59].sum():
    names = ["aux node", "probe", "leaf check", "walk entries", "walk nodes"]
    print("QW exec by step kind (cycles per trip with that kind, share of trips): " + "; ".join(
        "%s %.0f (%.2f)" % (n, tot[48 + i] / max(tot[54 + i], 1), tot[54 + i] / max(tot[2] - tot[4], 1)) for i, n in enumerate(names))
        + "; before the first kind %.0f per stepping trip" % (tot[53] / max(tot[2] - tot[4], 1)))
if tot[[37, 38, 39, 44, 45]].sum():
    names = ["aux node", "probe", "leaf check", "walk entries", "walk nodes"]
    iss = tot[[37, 38, 39, 44, 45]]
    print("QW step kinds (-DPT_WPROF): issues per stepping trip / mean lanes per issue: " + "; ".join(
        "%s %.3f / %.1f" % (n, iss[i] / max(tot[2] - tot[4], 1), tot[59 + i] / max(iss[i], 1)) for i, n in enumerate(names))
        + "; all kinds: %.2f issues per trip, %.1f lanes per issue" % (iss.sum() / max(tot[2] - tot[4], 1),
                                                                     tot[59:64].sum() / max(iss.sum(), 1)))
