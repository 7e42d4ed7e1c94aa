#!/usr/bin/env python3
"""Benchmark of the hw5 render path on MI355X (BASELINE.json metric).

Workload (N=1): config 3 of BASELINE.json -- the md5-pinned ~90k-triangle
dragon stand-in (scenes/make_scene.py c3; the reference's dragon_100k file is
missing) at 1920x1080, RAY_DEPTH 6.  One "step" = `--spp-per-step` (default 16)
samples for every pixel of the frame: the reference's spp loop advanced by
that many (each pixel's minstd_rand stream and f32 sum stay resident in HBM,
so K steps are exactly the first K*spp of the 256 spp).  `value` = Mray/s =
closest-hit queries (Scene::RayIntersection calls, counted on the GPU) over
the timed region.

Multi-GPU (torchrun, one process per GPU): the frame's 16x16 tiles are dealt
round-robin to ranks (no data-path collective) and every rank advances its
pixels by spp-per-step x N samples per step, so the per-GPU work is fixed as N
grows ("weak" scaling); the timed region ends with the framebuffer resolve
(tonemap on device) and an RCCL gather of the packed 8-bit tiles to rank 0.

Also reported: roofline of the dominant kernel (k_wpath, the persistent path
engine: closest-hit queries + shading) from in-kernel counters and HIP-event
launch times, and the reference CPU renderer timed on this host on a bounded
sample of the same scene.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "scenes"))
import make_scene  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_ptrace():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ptrace", os.path.join(REPO, "raytracing-course_amd", "ptrace.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def scene_file(config):
    gen = os.path.join(REPO, "scenes", "gen")
    os.makedirs(gen, exist_ok=True)
    p = os.path.join(gen, config + ".txt")
    if not os.path.exists(p):
        tmp = p + ".%d.tmp" % os.getpid()
        make_scene.make(config, tmp)
        os.replace(tmp, p)
    return p


def gather_tiles(dist, packed, rank, world, width, height, device):
    """RCCL/gloo gather of every rank's packed 8-bit tiles to rank 0 and the
    host un-interleave into the W*H*3 framebuffer (rank 0 returns it)."""
    import torch
    n_tiles = (width + 15) // 16 * ((height + 15) // 16)
    per_rank = [((n_tiles - r + world - 1) // world) * 768 for r in range(world)]
    cap = max(per_rank)
    buf = torch.zeros(cap, dtype=torch.uint8, device=device)
    buf[: packed.numel()] = packed
    if world == 1:
        parts = [buf]
    else:
        parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
        dist.gather(buf, parts, dst=0)
    if rank != 0:
        return None
    tiles_x, tiles_y = (width + 15) // 16, (height + 15) // 16
    pad = np.zeros((tiles_y, tiles_x, 16, 16, 3), np.uint8)   # [ty, tx, row, col, rgb]
    for r in range(world):
        p = parts[r][: per_rank[r]].cpu().numpy().reshape(-1, 16, 16, 3)
        gt = np.arange(p.shape[0]) * world + r                  # local tile lt is global tile lt*world + r
        pad[gt // tiles_x, gt % tiles_x] = p
    img = pad.transpose(0, 2, 1, 3, 4).reshape(tiles_y * 16, tiles_x * 16, 3)[:height, :width]
    return img


def cpu_baseline(pt, args):
    """The reference hw5 renderer (oracle/_ref, built from /root/reference by
    oracle/build_ref.sh) on a bounded sample of the same scene; rays of the
    sample counted by the GPU renderer (identical path decisions)."""
    W, H = args.cpu_sample
    src = os.path.join(REPO, "scenes", "gen", "cpu_sample_%dx%d.txt" % (W, H))
    make_scene.make_custom(os.path.join(REPO, "scenes", "practice5_dragon_10k.txt"), W, H, 1, True, "diffuse", src)
    ref = os.path.join(REPO, "oracle", "_ref", "raytracing_hw5")
    port = os.path.join(REPO, "oracle", "_build", "pt_oracle")
    out = os.path.join("/tmp", "pt_cpu_sample_%d.ppm" % os.getpid())
    cores = os.cpu_count()
    if os.path.exists(ref):
        kind, cmd = "reference", [ref, src, out]
    elif os.path.exists(port):
        kind, cmd = "port", [port, src, out, str(cores)]
    else:
        return None
    t0 = time.perf_counter()
    subprocess.check_call(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    dt = time.perf_counter() - t0
    with pt.Scene.load(src) as s:
        gimg, _, st = s.render(device=0)
    with open(out, "rb") as f:
        same = f.read() == b"P6\n%d %d\n255\n" % (W, H) + gimg.tobytes()
    os.unlink(out)
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = cores
    return {"value": st["rays"] / dt / 1e6, "unit": "Mray/s", "cores": cores, "kind": kind,
            "sample": "stand-in dragon %dx%d x 1 spp (%d rays, %.1f s wall, load+BVH included; "
                      "threads = hardware_concurrency = %d, affinity %d CPUs; GPU image of the sample %s)"
                      % (W, H, st["rays"], dt, cores, aff, "byte-identical" if same else "DIFFERS")}


def wall_to_ppm(config):
    """The drop-in CLI (run.sh <scene.txt> <out.ppm>) on the whole config: process
    start -> PPM closed (parse, reference BVH, aux BVH, upload, full render,
    tonemap, P6 write), as the reference's `run.sh` is timed."""
    import re
    src = scene_file(config)
    out = os.path.join("/tmp", "pt_bench_%s_%d.ppm" % (config, os.getpid()))
    env = dict(os.environ, PT_STATS="1", PT_QUIET="1")
    t0 = time.perf_counter()
    r = subprocess.run([os.path.join(REPO, "run.sh"), src, out], env=env, capture_output=True, text=True)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(r.stderr.strip()[-300:])
    os.unlink(out)
    rays = int(re.search(r"rays=(\d+)", r.stderr).group(1))
    return {"config": config, "seconds": dt, "rays": rays, "mray_s": rays / dt / 1e6,
            "what": "run.sh <scene> <out.ppm> on one GPU, process start to PPM closed (all spp of the config)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--spp-per-step", type=int, default=16, help="samples per pixel per step, per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wallclock", action="store_true", help="skip the full-config CLI run (wall_to_ppm)")
    ap.add_argument("--cpu-sample", type=int, nargs=2, default=[480, 270])
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--traversal", default="replay", choices=["replay", "exact"])
    # testing the multi-process path on a one-GPU box: every rank on cuda:0, gloo collectives
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"], help=argparse.SUPPRESS)
    ap.add_argument("--same-device", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus if args.gpus == 1 else 1)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    coll_device = device if args.dist_backend == "nccl" else torch.device("cpu")   # where collectives run

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    pt = load_ptrace()
    if rank == 0:
        path = scene_file(args.config)
    barrier()
    path = scene_file(args.config)
    t_load = time.perf_counter()
    scene = pt.Scene.load(path)
    t_prep = time.perf_counter()
    scene.prepare()
    t_sess = time.perf_counter()
    info = scene.info
    W, H = info["width"], info["height"]
    trav = pt.TRAVERSAL_REPLAY if args.traversal == "replay" else pt.TRAVERSAL_EXACT
    ss = pt.Session(scene, device=local, rank=rank, world=world, traversal=trav)
    ss.sync()
    t_ready = time.perf_counter()
    spp = args.spp_per_step * world   # weak scaling: a rank owns 1/world of the pixels
    for _ in range(args.warmup):
        ss.trace(spp)
    ss.sync()
    st0 = ss.stats()

    packed = torch.empty(max(ss.packed_bytes, 1), dtype=torch.uint8, device=device)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ss.trace(spp)
    ss.resolve(dev_out=packed.data_ptr() if ss.packed_bytes else None)
    ss.sync()
    img = gather_tiles(dist, packed[: ss.packed_bytes].to(coll_device), rank, world, W, H, coll_device)
    barrier()
    t1 = time.perf_counter()
    st1 = ss.stats()

    elapsed = t1 - t0
    rays = st1["rays"] - st0["rays"]
    nodes = st1["node_visits"] - st0["node_visits"]
    ptests = st1["prim_tests"] - st0["prim_tests"]
    auxv = st1["aux_visits"] - st0["aux_visits"]
    fb = st1["fallbacks"] - st0["fallbacks"]
    kms = st1["kernel_ms"] - st0["kernel_ms"]
    errs = st1["errors"]
    t = torch.tensor([elapsed, float(rays), float(nodes), float(ptests), kms, float(errs), float(auxv), float(fb)],
                     dtype=torch.float64, device=coll_device)
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    else:
        tmax = tsum = t
    if rank == 0:
        T = float(tmax[0])
        total_rays = float(tsum[1])
        # roofline of the dominant kernel (k_wpath: the path engine's persistent
        # query + shade kernel, >99% of GPU time, both instantiations -- main and
        # end-of-pass): algorithmic bytes per launch / mean launch time, both from
        # rank 0; launch times are HIP events recorded around each k_wpath launch on
        # the session's stream
        launches = max(st1["isect_launches"] - st0["isect_launches"], 1)
        isect_ms = st1["isect_ms"] - st0["isect_ms"]
        alg_bytes = (nodes * st1["node_bytes"] + ptests * st1["prim_bytes"] + auxv * st1["aux_bytes"]) / launches
        launch_s = (isect_ms / 1e3) / launches
        achieved = alg_bytes / launch_s / 1e9 if launch_s > 0 else 0.0
        traffic = None
        traffic_src = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                key = "%s_spp%d_n%d" % (args.config, spp, world)
                if key in tj:
                    # profiled per-launch fabric bytes x (this run's launches / the profile's):
                    # kept per launch like `achieved`
                    traffic = tj[key]["hbm_bytes_per_launch"]
                    traffic_src = tj[key].get("source")
            except Exception:
                pass
        res = {
            "metric": "Mray/s (closest-hit queries/s), dragon stand-in 1080p, RAY_DEPTH 6",
            "value": total_rays / T / 1e6,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": T * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: md5-pinned 89,928-triangle dragon stand-in (SURVEY §8d), per-pixel reference seeds",
            "config": {"workload": "config 3: %s %dx%d, %d spp per step (of 256), RAY_DEPTH %d; %s traversal of the "
                                   "reference tree (bit-exact)" % (args.config, W, H, spp,
                                                                   info["ray_depth"], args.traversal),
                       "pixels": W * H, "samples_per_step": W * H * spp,
                       "parallelism": "pixel tiles x%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_wpath", "alg_bytes_per_launch": alg_bytes, "launch_ms": launch_s * 1e3,
                         "launches": launches, "traffic_source": traffic_src,
                         "note": "algorithmic = 4-wide aux BVH nodes (128 B) + reference node records (32 B) + "
                                 "compact primitive records (48 B) per visit; the ~25 MB working set is "
                                 "L2/Infinity-Cache resident, and the kernel is bound by VALU issue (divergent "
                                 "per-lane state machines), not bandwidth (DESIGN.md §4)"},
            "wavefront_rounds": int(st1["rounds"] - st0["rounds"]),
            "kernel_ms_per_step": kms / args.steps,
            "rays": total_rays,
            "msamples_per_s": W * H * spp * args.steps / T / 1e6,
            "node_visits_per_ray": float(tsum[2]) / max(total_rays, 1),
            "aux_visits_per_ray": float(tsum[6]) / max(total_rays, 1),
            "fallback_rate": float(tsum[7]) / max(total_rays, 1),
            "fallbacks": int(tsum[7]),
            "exactness_errors": int(tsum[5]),
            "wall": {"load_s": t_prep - t_load, "prepare_bvh_s": t_sess - t_prep, "session_upload_s": t_ready - t_sess},
            "framebuffer_gathered": img is not None and img.shape == (H, W, 3),
            "framebuffer_md5": hashlib.md5(img.tobytes()).hexdigest() if img is not None else None,
        }
        res["projected_c3_render_s"] = (256.0 / (spp * args.steps)) * T
        if world == 1 and not args.no_cpu_baseline:
            try:
                res["cpu_baseline"] = cpu_baseline(pt, args)
            except Exception as e:  # never lose the GPU line over the baseline
                log("cpu baseline failed:", e)
                res["cpu_baseline"] = None
        else:
            res["cpu_baseline"] = None
        if world == 1 and not args.no_wallclock:
            try:
                res["wall_to_ppm"] = wall_to_ppm(args.config)
            except Exception as e:
                log("wall-clock run failed:", e)
                res["wall_to_ppm"] = None
        print(json.dumps(res))
    ss.close()
    scene.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
