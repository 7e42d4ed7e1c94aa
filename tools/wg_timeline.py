#!/usr/bin/env python3
"""Analyse PT_WGPROF per-workgroup timelines: {start, end (100 MHz), HW_ID, XCC_ID} x tiles x launches."""
import sys
import numpy as np

def main(path, n_tiles):
    a = np.fromfile(path, np.uint64).reshape(-1, n_tiles, 4)
    L = a[-1].astype(np.int64)
    L = L[L[:, 0] > 0]
    t0 = L[:, 0].min()
    s = (L[:, 0] - t0) / 100.0  # us
    e = (L[:, 1] - t0) / 100.0
    d = e - s
    span = e.max()
    hw = L[:, 2]
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    xcc = L[:, 3] & 0xF
    print("launches %d, wgs %d, span %.1f ms" % (a.shape[0], len(L), span / 1e3))
    print("wg duration us: mean %.0f p50 %.0f p90 %.0f p99 %.0f max %.0f" % (d.mean(), *np.percentile(d, [50, 90, 99, 100])))
    # concurrency over time
    ts = np.linspace(0, span, 21)
    conc = [((s <= t) & (e > t)).sum() for t in ts]
    print("concurrent wgs over time:", conc)
    print("mean concurrency %.1f (sum dur / span)" % (d.sum() / span))
    print("per-XCC wgs", np.bincount(xcc, minlength=8), "busy ms", [round(d[xcc == k].sum() / 1e3, 1) for k in range(8)])
    last = np.sort(e)[-20:]
    print("last 20 ends (ms)", np.round(last / 1e3, 2))
    # per-tile duration map quantiles by tile row
    return d

if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
