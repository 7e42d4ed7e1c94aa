#!/usr/bin/env python3
"""Benchmark of the hw5 render path on MI355X (BASELINE.json metric).

Workload (N=1): config 3 of BASELINE.json -- the md5-pinned ~90k-triangle
dragon stand-in (scenes/make_scene.py c3; the reference's dragon_100k file is
missing) at 1920x1080, RAY_DEPTH 6.  One "step" = the metric's job: the whole
frame at `--spp-per-step` (default 256, the config's SAMPLES) samples per pixel,
as ONE pass from sample 0 (pt_session_reset re-seeds every pixel's minstd_rand
stream and zeroes its f32 sum), then the device tonemap and the gather of the
8-bit framebuffer -- so every step pays the pass's end tail exactly as the
metric's render does, and the last step's framebuffer is the 256-spp image
(checked against the CLI's PPM).  `value` = Mray/s = closest-hit queries
(Scene::RayIntersection calls, counted on the GPU) over the timed region.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` (no WORLD_SIZE in
the environment) starts the N ranks itself under torch.distributed.run before
anything touches a GPU; under torchrun it runs as the rank it is given and
exits non-zero if WORLD_SIZE != --gpus.  The frame's 16x16 tiles are dealt to
ranks in diagonal stripes (no data-path collective).  `--scaling strong` (the
default, the metric's own job: "1080p/256spp, 1/2/4/8 GPU"): a step is
spp-per-step samples of EVERY pixel of the frame at any N, each rank rendering
its 1/N of the pixels, so the job is fixed and N GPUs should finish it N times
faster.  `--scaling weak`: every rank renders its pixels at spp-per-step x N
samples per step (per-GPU work fixed as N grows; a longer pass per rank, which
hides more of the end-of-pass tail).  Every step ends with the framebuffer
resolve (tonemap on device) and an RCCL gather of the packed 8-bit tiles to
rank 0.

Also reported: the roofline of the dominant kernel (k_wpath, the persistent
path engine: closest-hit queries + shading) from in-kernel counters and
HIP-event launch times, per rank; the reference CPU renderer timed on this
host (per-config bounded samples, render only); and the wall-clock to PPM of
the drop-in CLI on the whole config, on N GPUs in one process (PT_NGPU=N).
"""
import argparse
import hashlib
import json
import os
import re
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "scenes"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import make_scene  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
REF_MD5 = {"c1": "99f1bc9386a22892970f058bfa8114c7", "c2": "a16f6cf46a6443244ecbd0c9d856c295"}


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


# ------------------------------------------------------------------ launch --
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(args, argv):
    """--gpus N > 1 without a torchrun environment: start N ranks (one process
    per GPU) under torch.distributed.run as CHILD processes and return their
    exit code.  Nothing in this process has touched a GPU (device_count does not
    initialise the runtime on this image)."""
    if not args.same_device and not args.probe_ranks:
        import torch
        have = torch.cuda.device_count()
        if have < args.gpus:
            log("bench: --gpus %d but only %d GPU(s) visible" % (args.gpus, have))
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0", PT_BENCH_SPAWNED="1")
    return subprocess.call(cmd, env=env)


def rank_spp(spp_per_step, world, scaling):
    """samples per pixel a rank's pixels advance per step: strong scaling, the frame's
    spp-per-step at any N (each rank owns 1/N of the pixels: the job is fixed); weak, N
    times that (the rank's work per step is the one-GPU step's)"""
    return spp_per_step * (world if scaling == "weak" else 1)


def probe_ranks(args, rank, world):
    """CPU check of the launch path (tests/test_dist.py): every rank joins a gloo
    group and rank 0 prints the ranks it sees.  No GPU is touched."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "pid": os.getpid(), "local_rank": int(os.environ.get("LOCAL_RANK", 0))})
    if rank == 0:
        # (no scene here: the default spp is config 3's SAMPLES, 256; every step is one pass)
        spp = rank_spp(args.spp_per_step or 256, world, args.scaling)
        print(json.dumps({"probe": True, "n_gpus": world, "gpus_arg": args.gpus, "ranks": got,
                          "scaling": args.scaling, "rank_spp_per_step": spp, "pass_spp": spp}))
    dist.destroy_process_group()
    del torch


# ------------------------------------------------------------------ tiles --
def gather_tiles(dist, packed, rank, world, width, height, device):
    """RCCL/gloo gather of every rank's packed 8-bit tiles to rank 0, the
    un-interleave into the H x W x 3 framebuffer on rank 0's device, and one
    copy of it to the host (rank 0 returns it as a numpy array).

    Rank r holds the tiles (tx, ty) with (tx + ty) % world == r, in ascending
    order (include/pt.h sessions), 16 x 16 x 3 bytes each; the gathered
    [world, cap_tiles] blocks are put in global tile order by one index gather."""
    import torch
    tiles_x, tiles_y = (width + 15) // 16, (height + 15) // 16
    n_tiles = tiles_x * tiles_y
    t_all = np.arange(n_tiles)
    owner = (t_all % tiles_x + t_all // tiles_x) % world
    cap_tiles = int(np.bincount(owner, minlength=world).max())
    cap = cap_tiles * 768
    if packed.numel() == cap:
        buf = packed.contiguous()
    else:
        buf = torch.zeros(cap, dtype=torch.uint8, device=device)
        buf[: packed.numel()] = packed
    if world == 1:
        parts = buf.view(1, cap)
    else:
        parts = torch.empty((world, cap), dtype=torch.uint8, device=device) if rank == 0 else None
        dist.gather(buf, list(parts.unbind(0)) if rank == 0 else None, dst=0)
    if rank != 0:
        return None
    # source block of every global tile: owner * cap_tiles + its rank in the owner's list
    local = np.zeros(n_tiles, np.int64)
    for r in range(world):
        m = owner == r
        local[m] = np.arange(int(m.sum()))
    src = torch.from_numpy(owner.astype(np.int64) * cap_tiles + local).to(parts.device)
    t = parts.view(world * cap_tiles, 16, 16, 3).index_select(0, src)
    img = t.view(tiles_y, tiles_x, 16, 16, 3).permute(0, 2, 1, 3, 4).reshape(tiles_y * 16, tiles_x * 16, 3)
    return img[:height, :width].cpu().numpy()


# ------------------------------------------------------------ CPU baseline --
def host_cpus():
    """(usable CPUs, description): the affinity mask capped by the cgroup CPU quota."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except Exception:
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    omp = os.environ.get("OMP_NUM_THREADS")
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return usable, {"cpu_model": model, "affinity_cpus": aff, "cgroup_quota_cpus": quota, "OMP_NUM_THREADS": omp,
                    "os_cpu_count": os.cpu_count()}


# bounded samples of every BASELINE config (render only, load + BVH timed apart):
#   name -> (scene config, spp override, x0, y0, w, rows, row stride)
# Rows are spread over the frame (stride) so the sample's per-ray cost is the
# frame's, not one band's.  c1 is the full image at full spp; c3, the workload of
# `value`, the full frame at 1 spp (the smallest spp of >= 60 s).
CPU_SAMPLES = {
    "c1": ("c1", 0, 0, 0, 256, 256, 1),
    "c2": ("c2", 0, 0, 4, 512, 8, 64),
    "c3": ("c3", 1, 0, 0, 1920, 1080, 1),   # the full frame at SAMPLES 1 (~2 min on 16 threads)
    "c4_metal": ("c4_metal", 1, 0, 9, 1920, 6, 180),
    "c4_glass": ("c4_glass", 1, 0, 9, 1920, 6, 180),
    "c5": ("c5", 1, 0, 18, 3840, 4, 540),
}
FULL_SPP = {"c1": 16, "c2": 64, "c3": 256, "c4_metal": 1024, "c4_glass": 1024, "c5": 4096}


def cpu_baseline(pt, args):
    """The reference hw5 renderer on this host's CPUs: oracle/_ref/ref_harness =
    the UNMODIFIED reference sources (Scene::Load/InitScene/Sample) around a
    restatement of Scene::Render's pixel loop that can render a row sample and
    times load+InitScene and the render separately.  Rays of each sample are
    counted by the GPU renderer on the same pixels (identical path decisions;
    the GPU image of the sample is checked byte-identical)."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    usable, cpu = host_cpus()
    rows = {}
    for name in args.cpu_configs:
        cfg, spp, x0, y0, w, nrow, stride = CPU_SAMPLES[name]
        src = scene_file(cfg)
        if spp:
            # the same scene text with only the SAMPLES line changed (per-sample work is i.i.d.)
            text = open(src).read()
            text = re.sub(r"(?m)^SAMPLES\s+\d+", "SAMPLES %d" % spp, text, count=1)
            src = os.path.join(REPO, "scenes", "gen", "%s_spp%d.txt" % (cfg, spp))
            if not os.path.exists(src) or open(src).read() != text:
                open(src, "w").write(text)
        out_ppm = "/tmp/pt_cpu_%s_%d.ppm" % (name, os.getpid())
        out_rad = out_ppm + ".f32"
        env = dict(os.environ, REF_THREADS=str(usable))
        r = subprocess.run([harness, "render", src, out_ppm, out_rad, str(x0), str(y0), str(w), str(nrow), str(stride)],
                           env=env, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("ref_harness %s: %s" % (name, r.stderr[-300:]))
        m = dict(re.findall(r"(\w+)=([\d.]+)", r.stderr.splitlines()[-1]))
        ref_img = open(out_ppm, "rb").read()
        os.unlink(out_ppm)
        os.unlink(out_rad)
        # the GPU renders the same rows (one window per row: global-index seeds)
        rays = 0
        gpu_rows = []
        with pt.Scene.load(src) as s:
            if nrow * stride == s.info["height"] and stride == 1 and w == s.info["width"]:
                img, _, st = s.render(device=0)
                gpu_rows.append(img)
                rays = st["rays"]
            else:
                for k in range(nrow):
                    img, _, st = s.render(device=0, window=(x0, y0 + k * stride, w, 1))
                    gpu_rows.append(img)
                    rays += st["rays"]
        gimg = np.concatenate(gpu_rows, axis=0)
        same = ref_img == b"P6\n%d %d\n255\n" % (w, nrow) + gimg.tobytes()
        render_s = float(m["render_s"])
        spp_eff = spp or FULL_SPP[name]
        row = {"render_s": render_s, "load_init_s": float(m["load_init_s"]), "rays": rays,
               "mray_s": rays / render_s / 1e6, "msample_s": w * nrow * spp_eff / render_s / 1e6,
               "pixels": w * nrow, "spp": spp_eff, "threads": int(m["threads"]),
               "sample": "%d rows x %d px from row %d, stride %d, %d spp" % (nrow, w, y0, stride, spp_eff),
               "gpu_image_identical": same}
        if spp:
            # config time scaled to the full spp and frame (per-sample work is i.i.d. per pixel)
            W, H = {"c5": (3840, 2160), "c2": (512, 512)}.get(cfg, (1920, 1080))
            row["projected_full_render_s"] = render_s * (W * H) / (w * nrow) * FULL_SPP[name] / spp
        elif (w * nrow, stride) != (256 * 256, 1):
            W, H = (512, 512) if cfg == "c2" else (1920, 1080)
            row["projected_full_render_s"] = render_s * (W * H) / (w * nrow)
        if name in REF_MD5 and nrow * stride == 256 and w == 256:
            row["md5_matches_reference"] = hashlib.md5(ref_img).hexdigest() == REF_MD5[name]
        rows[name] = row
        log("cpu baseline %s: %.2f Mray/s (%d rays, %.2f s render, %d threads), GPU image %s"
            % (name, row["mray_s"], rays, render_s, row["threads"], "identical" if same else "DIFFERS"))
    main_row = rows.get(args.config) or next(iter(rows.values()))
    return {"value": main_row["mray_s"], "unit": "Mray/s", "cores": main_row["threads"], "kind": "reference",
            "sample": "config %s: %s, render only (load + InitScene %.2f s timed apart); unmodified reference "
                      "sources (oracle/_ref/ref_harness), OpenMP threads = usable CPUs of this host"
                      % (args.config, main_row["sample"], main_row["load_init_s"]),
            "host": cpu, "configs": rows}


# ------------------------------------------------------------- wall clock --
def wall_to_ppm(config, ngpu):
    """The drop-in CLI (run.sh <scene.txt> <out.ppm>) on the whole config: process
    start -> PPM closed (parse, reference BVH, aux BVH, upload, full render,
    tonemap, gather, P6 write), as the reference's `run.sh` is timed (SURVEY §8d:
    the metric stops at "PPM closed"; the process's exit after it -- the HIP
    runtime's teardown -- is reported apart as `teardown_s`).  ngpu > 1: one
    process drives ngpu GPUs (PT_NGPU) and gathers with RCCL."""
    src = scene_file(config)
    out = os.path.join("/tmp", "pt_bench_%s_%d.ppm" % (config, os.getpid()))
    env = dict(os.environ, PT_STATS="2", PT_QUIET="1", PT_NGPU=str(ngpu))
    if ngpu > 1:
        env["PT_GATHER"] = "rccl"
    u0 = time.time()
    t0 = time.perf_counter()
    # bounded (120 s; c3 takes ~1 s): a hung CLI (e.g. RCCL initialisation) must not hold back the bench line
    r = subprocess.run([os.path.join(REPO, "run.sh"), src, out], env=env, capture_output=True, text=True,
                       timeout=120)
    dt_exit = time.perf_counter() - t0
    u1 = time.time()
    if r.returncode != 0:
        raise RuntimeError(r.stderr.strip()[-300:])
    # the CLI prints the wall-clock time at which the PPM was closed (PT_STATS=2)
    um = re.search(r"unix_main=([\d.]+) unix_written=([\d.]+)", r.stderr)
    written = float(um.group(2)) if um else None
    dt = (written - u0) if written else dt_exit
    teardown = (u1 - written) if written else None
    md5 = hashlib.md5(open(out, "rb").read()).hexdigest()
    os.unlink(out)
    stats = [ln for ln in r.stderr.splitlines() if ln.startswith("rays=")]
    m = dict(re.findall(r"(\w+(?:/\w+)?)=([\d.]+)", stats[-1] if stats else r.stderr))
    rays = int(m["rays"])
    # PT_STATS=2: the CLI's phases and pt_render's per-rank set-up / render / resolve and the gather
    phases = {}
    for ln in r.stderr.splitlines():
        if ln.startswith("phases_ms:"):
            phases["cli_ms"] = {k: float(v) for k, v in re.findall(r"(\w+)=([\d.]+)", ln)}
        elif ln.startswith("pt_render rank"):
            phases.setdefault("ranks", []).append({k: float(v) for k, v in re.findall(r"(\w+)=([\d.]+)", ln)})
        elif ln.startswith("pt_render gather_ms"):
            phases["gather_ms"] = float(re.search(r"gather_ms=([\d.]+)", ln).group(1))
    render_ms = float(m["wall_ms"])
    kernel_ms = float(m["kernel_ms"])
    return {"config": config, "ngpu": ngpu, "seconds": dt, "seconds_to_exit": dt_exit, "teardown_s": teardown,
            "rays": rays, "mray_s": rays / dt / 1e6,
            "render_ms": render_ms, "kernel_ms": kernel_ms,
            # the same pass over two clocks: the pass's kernels (HIP events) and pt_render's own wall
            # (session set-up + the pass + tonemap + gather)
            "render_mray_s": rays / kernel_ms / 1e3 if kernel_ms > 0 else None,
            "render_wall_mray_s": rays / render_ms / 1e3 if render_ms > 0 else None,
            "gather_rccl": int(m.get("gather_rccl", 0)), "ppm_md5": md5, "phases": phases,
            "what": "PT_NGPU=%d run.sh <scene> <out.ppm>: one process; seconds = process start to PPM closed "
                    "(all spp of the config), teardown_s = the process exit after it; render_ms = pt_render's "
                    "wall (session set-up, the pass, tonemap, gather), kernel_ms = the pass's kernels (HIP "
                    "events, slowest GPU)" % ngpu}


# -------------------------------------------------------------- roofline --
def roofline(st0, st1, traffic_json, key):
    """k_wpath roofline record of this rank: algorithmic bytes per launch (in-kernel
    visit counters x record sizes) / mean launch time (HIP events on the session's
    stream).  `traffic` = this run's algorithmic bytes x the profiled ratio of
    memory-side bytes to algorithmic bytes (rocprofv3 FETCH/WRITE passes of the
    same workload, profiles/traffic.json), so it scales with this run's launches."""
    # the path engine's share: the cooperative end-of-pass launches (k_wcoop) are counted
    # apart (pt_stats coop_*) and reported in `coop`
    d = {k: st1[k] - st0[k] for k in ("isect_launches", "isect_ms", "node_visits", "prim_tests", "aux_visits", "rays",
                                      "coop_launches", "coop_ms", "coop_node_visits", "coop_prim_tests",
                                      "coop_aux_visits", "coop_rays")}
    launches = max(d["isect_launches"] - d["coop_launches"], 1)
    isect_ms = d["isect_ms"] - d["coop_ms"]
    nodes = d["node_visits"] - d["coop_node_visits"]
    ptests = d["prim_tests"] - d["coop_prim_tests"]
    auxv = d["aux_visits"] - d["coop_aux_visits"]
    alg_bytes = (nodes * st1["node_bytes"] + ptests * st1["prim_bytes"] + auxv * st1["aux_bytes"]) / launches
    launch_s = (isect_ms / 1e3) / launches
    achieved = alg_bytes / launch_s / 1e9 if launch_s > 0 else 0.0
    rec = {"bound": "hbm", "priced_against": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "k_wpath",
           "alg_bytes_per_launch": alg_bytes, "launch_ms": launch_s * 1e3, "launches": launches,
           "rays_share": (d["rays"] - d["coop_rays"]) / max(d["rays"], 1),
           "alg_bytes_per_ray": alg_bytes * launches / max(d["rays"] - d["coop_rays"], 1)}
    if d["coop_launches"]:
        # its algorithmic bytes (the same record sizes x its own visit counters) over its summed
        # launch time (HIP events; the early launch runs beside path rounds, so this is the rate
        # the cooperative teams drew while they ran, not an exclusive one)
        cbytes = (d["coop_node_visits"] * st1["node_bytes"] + d["coop_prim_tests"] * st1["prim_bytes"] +
                  d["coop_aux_visits"] * st1["aux_bytes"])
        cach = cbytes / (d["coop_ms"] / 1e3) / 1e9 if d["coop_ms"] > 0 else 0.0
        rec["coop"] = {"kernel": "k_wcoop (end of pass)", "launches": d["coop_launches"], "ms": d["coop_ms"],
                       "rays": d["coop_rays"], "mray_s": d["coop_rays"] / max(d["coop_ms"], 1e-9) / 1e3,
                       "alg_bytes": cbytes, "alg_bytes_per_ray": cbytes / max(d["coop_rays"], 1),
                       "achieved": cach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": cach / HBM_PEAK_GBS}
    prof = None
    try:
        prof = json.load(open(traffic_json)).get(key)
    except Exception:
        pass
    if prof and "traffic_per_alg_byte" in prof:
        rec["traffic"] = prof["traffic_per_alg_byte"] * alg_bytes
        rec["traffic_per_alg_byte"] = prof["traffic_per_alg_byte"]
        rec["traffic_source"] = ("profiles/%s: rocprofv3 --pmc FETCH_SIZE (KiB, x2 gfx950) + WRITE_SIZE (KiB) over the "
                                 "same workload's timed launches, as a ratio to that run's algorithmic bytes, times "
                                 "this run's algorithmic bytes per launch" % prof.get("profile", "?"))
        for k in ("l2_hit_rate", "write_bytes_per_ray", "fetch_bytes_per_ray", "limiter", "valu_issue_frac",
                  "wait_frac", "vgpr", "waves_per_simd"):
            if k in prof:
                rec[k] = prof[k]
        if "wait_any_frac" in prof and "valu_issue_frac" in prof:
            # what the SQ counters of that profile say bounds the kernel: the
            # roofline is priced against HBM, but neither HBM nor VALU issue is saturated
            hbm = rec["traffic"] / launch_s / 1e9 / HBM_PEAK_GBS if launch_s > 0 else 0.0
            rec["limiter"] = {
                "verdict": "latency" if max(hbm, prof["valu_issue_frac"]) < 0.6 else
                           ("hbm" if hbm >= prof["valu_issue_frac"] else "valu_issue"),
                "memory_side_frac_of_hbm_peak": hbm, "valu_issue_frac": prof["valu_issue_frac"],
                "wave_wait_any_frac": prof["wait_any_frac"],
                "source": "profiles/%s SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU / SQ_WAIT_ANY per wave-cycle"
                          % prof.get("profile", "?")}
            # `bound` names what the counters say limits the kernel; `peak`/`frac` stay priced
            # against HBM (the kernel has no MFMA work)
            rec["bound"] = rec["limiter"]["verdict"]
    rec["note"] = ("algorithmic = 4-wide aux BVH nodes (128 B) + reference node records (32 B) + primitive geometry "
                   "(48 B; the 64-B compact record adds a precomputed normal, a probe's 96-B leaf bundle carries its "
                   "first primitive and the leaf box) per visit; the ~30 MB working set "
                   "is L2/Infinity-Cache resident; the query's work per ray fell from ~1.5 KB (round 1) to ~0.7 KB, so "
                   "frac falls as Mray/s rises; what limits the kernel is in `limiter` (rocprofv3 SQ counters, "
                   "DESIGN.md §4)")
    return rec


def kernel_resources():
    """the compiler's resource report of the path engine's two instantiations and the
    cooperative engine's two small-team ones (teams of 4, the default, and 8; tools/kernel_resources.py)"""
    try:
        import kernel_resources as KR
        ks = KR.kernel("k_wpath")
        out = {("end_of_pass" if "ILb1" in k else "main"): v for k, v in ks.items()}
        for k, v in KR.kernel("k_wcoop").items():
            if "ILj8ELb0" in k:
                out["coop_team8"] = v
            if "ILj4ELb0" in k:
                out["coop_team4"] = v
        return out
    except Exception:
        return None


# ------------------------------------------------------------------ main --
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--spp-per-step", type=int, default=0,
                    help="samples per pixel per step: one pass from sample 0 (default: the config's SAMPLES, 256 "
                         "for c3; strong: of every pixel of the frame; weak: x N per rank)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong (default): the frame's job split over N GPUs; weak: per-GPU work fixed")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wallclock", action="store_true", help="skip the full-config CLI run (wall_to_ppm)")
    ap.add_argument("--cpu-configs", nargs="+", default=list(CPU_SAMPLES), choices=list(CPU_SAMPLES))
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--traversal", default="replay", choices=["replay", "exact"])
    # testing the multi-process path on a one-GPU box: every rank on cuda:0, gloo collectives
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"], help=argparse.SUPPRESS)
    ap.add_argument("--same-device", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--probe-ranks", action="store_true", help=argparse.SUPPRESS)
    argv = sys.argv[1:]
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(spawn_ranks(args, argv))
        world, rank, local = 1, 0, 0
    else:
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if world != args.gpus:
            log("bench: WORLD_SIZE=%d but --gpus %d: refusing to report a different GPU count" % (world, args.gpus))
            sys.exit(2)
    if args.probe_ranks:
        probe_ranks(args, rank, world)
        return

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
    # strong: every pixel of the frame advances spp-per-step per step at any N (a rank owns 1/N of
    # them); weak: a rank's pixels advance N times as far, so its work per step is the one-GPU work
    spp = rank_spp(args.spp_per_step or info["samples"], world, args.scaling)
    packed = torch.empty(max(ss.packed_bytes, 1), dtype=torch.uint8, device=device)

    def step():
        # the job: every owned pixel from sample 0 through `spp` samples as one pass, the
        # device tonemap, and the 8-bit framebuffer's gather to rank 0
        ss.reset()
        ss.trace(spp)
        ss.resolve(dev_out=packed.data_ptr() if ss.packed_bytes else None)
        ss.sync()
        return gather_tiles(dist, packed[: ss.packed_bytes].to(coll_device), rank, world, W, H, coll_device)

    # (the warmup's first resolve and gather load code objects and set up the collective)
    for _ in range(max(args.warmup, 0)):
        step()
    ss.sync()
    st0 = ss.stats()

    barrier()
    t0 = time.perf_counter()
    img = None
    for _ in range(args.steps):
        img = step()
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
    roof = roofline(st0, st1, args.traffic_json, "%s_n1" % args.config)
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"rank": rank, "mray_s": rays / elapsed / 1e6, "frac": roof["frac"],
                                          "achieved": roof["achieved"], "launch_ms": roof["launch_ms"],
                                          "launches": roof["launches"], "tiles": ss.n_tiles})
    else:
        tmax = tsum = t
        per_rank = None
    res = None
    if rank == 0:
        T = float(tmax[0])
        total_rays = float(tsum[1])
        res = {
            "metric": "Mray/s (closest-hit queries/s), dragon stand-in 1080p/%d spp, RAY_DEPTH 6" % spp,
            "value": total_rays / T / 1e6,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": T * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: md5-pinned 89,928-triangle dragon stand-in (SURVEY §8d), per-pixel reference seeds",
            "config": {"workload": "config 3: %s %dx%d, one step = the job: every pixel from sample 0 through "
                                   "%d spp as one pass + device tonemap + gather (%s scaling), RAY_DEPTH %d; %s "
                                   "traversal of the reference tree (bit-exact)"
                                   % (args.config, W, H, spp, args.scaling, info["ray_depth"], args.traversal),
                       "pixels": W * H, "samples_per_step": W * H * spp,
                       "spp_per_step_per_pixel": spp, "scaling": args.scaling,
                       "parallelism": "pixel tiles x%d" % world},
            "roofline": roof,
            "wavefront_rounds": int(st1["rounds"] - st0["rounds"]),
            "kernel_ms_per_step": kms / args.steps,
            "rays": total_rays,
            "msamples_per_s": W * H * spp * args.steps / T / 1e6,
            "pass_spp": spp,
            "node_visits_per_ray": float(tsum[2]) / max(total_rays, 1),
            "aux_visits_per_ray": float(tsum[6]) / max(total_rays, 1),
            "fallback_rate": float(tsum[7]) / max(total_rays, 1),
            "fallbacks": int(tsum[7]),
            "exactness_errors": int(tsum[5]),
            "wall": {"load_s": t_prep - t_load, "prepare_bvh_s": t_sess - t_prep, "session_upload_s": t_ready - t_sess},
            "framebuffer_gathered": img is not None and img.shape == (H, W, 3),
            "framebuffer_md5": hashlib.md5(img.tobytes()).hexdigest() if img is not None else None,
            "distributed": {"world_size": world, "backend": args.dist_backend if world > 1 else None,
                            "collective_ranks": dist.get_world_size() if world > 1 else 1,
                            "launched_by": "bench.py --gpus" if os.environ.get("PT_BENCH_SPAWNED") else
                                           ("torch.distributed.run" if world > 1 else "single process")},
            "kernel_resources": kernel_resources(),
        }
        if per_rank:
            res["per_rank"] = per_rank
        res["job_s"] = T / max(args.steps, 1)   # one job (step): the frame's pass, tonemap and gather
    ss.close()
    scene.close()
    # the host-side legs run after the timed region, on rank 0 only; the other
    # ranks wait at the final barrier (their GPUs are free for the N-GPU CLI run)
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            try:
                res["cpu_baseline"] = cpu_baseline(pt, args)
            except Exception as e:  # never lose the GPU line over the baseline
                log("cpu baseline failed:", e)
                res["cpu_baseline"] = None
        else:
            res["cpu_baseline"] = None
        if not args.no_wallclock:
            ngpu = world if not args.same_device else 1
            try:
                res["wall_to_ppm"] = wall_to_ppm(args.config, ngpu)
                # the metric's own pass: the whole config (256 spp for c3) as ONE pass, rays over its
                # kernel time (HIP events) and over pt_render's wall -- beside `value`, whose 16-spp
                # steps coalesce into a pass of steps x 16
                res["render_256spp_mray_s"] = res["wall_to_ppm"]["render_mray_s"]
                if res["framebuffer_md5"] and spp == info["samples"]:
                    # the last step's framebuffer is the config's image: the CLI's PPM payload
                    ppm = b"P6\n%d %d\n255\n" % (W, H) + img.tobytes()
                    res["framebuffer_equals_cli_ppm"] = hashlib.md5(ppm).hexdigest() == res["wall_to_ppm"]["ppm_md5"]
                res["render_256spp_wall_mray_s"] = res["wall_to_ppm"]["render_wall_mray_s"]
                res["render_256spp_clocks"] = ("render_256spp_mray_s: rays / the pass's kernel time (HIP "
                                               "events); render_256spp_wall_mray_s: rays / pt_render's wall "
                                               "(session set-up + pass + tonemap + gather)")
            except Exception as e:
                log("wall-clock run failed:", e)
                res["wall_to_ppm"] = None
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
