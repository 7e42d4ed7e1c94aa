#!/usr/bin/env python3
"""Per-rank throughput of the N-GPU bench workload, simulated on one GPU.

bench.py at N GPUs gives each rank 1/N of the 1080p tiles and N x spp-per-step
samples per step.  This runs that one rank's session alone (rank r of world N)
on the local GPU and reports its Mray/s, so the weak-scaling behaviour of the
engine (sparser rounds as N grows) can be measured without N GPUs.
  python tools/rank_sim.py [--config c3] [--worlds 1 2 4 8] [--steps 2]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--ranks", default="first",
                    help="first | last | both | all | a comma list of ranks (in that order, repeats allowed)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--spp-per-step", type=int, default=16)
    a = ap.parse_args()
    pt = bench.load_ptrace()
    path = bench.scene_file(a.config)
    out = []
    with pt.Scene.load(path) as s:
        s.prepare()
        for w in a.worlds:
            named = {"first": [0], "last": [w - 1], "both": sorted({0, w - 1}), "all": list(range(w))}
            ranks = named[a.ranks] if a.ranks in named else [int(x) % w for x in a.ranks.split(",")]
            for r in ranks:
                ss = pt.Session(s, device=0, rank=r, world=w)
                spp = a.spp_per_step * w
                ss.trace(spp)   # warmup step
                ss.sync()
                st0 = ss.stats()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    ss.trace(spp)
                ss.sync()
                dt = time.perf_counter() - t0
                st1 = ss.stats()
                rays = st1["rays"] - st0["rays"]
                rounds = st1["rounds"] - st0["rounds"]
                rec = {"world": w, "rank": r, "session": len(out), "tiles": ss.n_tiles, "spp_per_step": spp, "mray_s": rays / dt / 1e6,
                       "ms_per_step": dt * 1e3 / a.steps, "rounds_per_step": rounds / a.steps,
                       "rays_per_round": rays / max(rounds, 1),
                       "isect_ms_per_round": (st1["isect_ms"] - st0["isect_ms"]) / max(rounds, 1),
                       "coop_ms_per_step": (st1["coop_ms"] - st0["coop_ms"]) / a.steps,
                       "coop_ray_share": (st1["coop_rays"] - st0["coop_rays"]) / max(rays, 1),
                       "fallbacks": st1["fallbacks"] - st0["fallbacks"],
                       "kernel_ms_per_step": (st1["kernel_ms"] - st0["kernel_ms"]) / a.steps}
                out.append(rec)
                print(json.dumps(rec), flush=True)
                ss.close()
            per = [r["mray_s"] for r in out if r["world"] == w]
            if len(per) > 1:
                # an N-GPU job ends with its slowest rank
                print(json.dumps({"world": w, "ranks": len(per), "min_mray_s": min(per), "max_mray_s": max(per),
                                  "spread": (max(per) - min(per)) / max(per)}), flush=True)
    return out


if __name__ == "__main__":
    main()
