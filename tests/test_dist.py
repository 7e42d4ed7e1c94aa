"""Multi-rank path on CPU: world-size-2 gloo runs of bench.py's tile deal and
framebuffer gather (the N>1 data path; on the GPU box the same code runs
over RCCL).  Tiles are 16x16, tile (tx, ty) belongs to rank (tx + ty) % world
(include/pt.h sessions, bench.py gather_tiles)."""
import importlib.util
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import _util as U

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _expected(W, H):
    y, x = np.mgrid[0:H, 0:W]
    img = np.stack([(x * 7 + y) % 251, (y * 3 + x // 16) % 253, (x ^ y) % 255], axis=-1)
    return img.astype(np.uint8)


def _packed_for_rank(img, rank, world):
    """what a rank's session resolves into: its tiles in local order, 256 px each, row-major"""
    H, W, _ = img.shape
    tx, ty = (W + 15) // 16, (H + 15) // 16
    out = []
    for gt in range(tx * ty):
        if (gt % tx + gt // tx) % world != rank:
            continue
        t = np.zeros((16, 16, 3), np.uint8)
        x0, y0 = (gt % tx) * 16, (gt // tx) * 16
        blk = img[y0:y0 + 16, x0:x0 + 16]
        t[:blk.shape[0], :blk.shape[1]] = blk
        out.append(t.reshape(-1))
    return np.concatenate(out) if out else np.zeros(0, np.uint8)


def _worker(rank, world, port, W, H, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    img = _expected(W, H)
    packed = torch.from_numpy(_packed_for_rank(img, rank, world))
    got = bench.gather_tiles(dist, packed, rank, world, W, H, torch.device("cpu"))
    # the max-over-ranks timing reduction bench.py uses
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((got.tobytes(), float(t[0])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("W,H", [(64, 48), (50, 37), (16, 16), (7, 3)])
def test_gloo_gather_two_ranks(W, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, W, H, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.frombuffer(got, np.uint8).reshape(H, W, 3).tolist() == _expected(W, H).tolist()
    assert tmax == 2.0


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_unpack_tiles_abi_matches_deal(world):
    """pt_unpack_tiles (C ABI) inverts the round-robin tile deal for every rank"""
    pt = U.ptrace()
    W, H = 83, 45
    img = _expected(W, H)
    out = np.zeros_like(img)
    for r in range(world):
        pt.unpack_tiles(_packed_for_rank(img, r, world), W, H, r, world, out=out)
    assert np.array_equal(out, img)


def _bench(args, env_extra=None):
    import json
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=300)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_starts_n_ranks(n):
    """`bench.py --gpus N` (as the driver calls it, no torchrun environment)
    starts N ranks itself: rank 0 sees exactly N distinct rank processes."""
    rc, out, err = _bench(["--gpus", str(n), "--probe-ranks"])
    assert rc == 0, err[-2000:]
    assert out["probe"] and out["n_gpus"] == n and out["gpus_arg"] == n
    assert sorted(r["rank"] for r in out["ranks"]) == list(range(n))
    assert len({r["pid"] for r in out["ranks"]}) == n
    assert sorted(r["local_rank"] for r in out["ranks"]) == list(range(n))


@pytest.mark.parametrize("scaling,spp", [("strong", 256), ("weak", 512), (None, 256)])
def test_bench_scaling_modes(scaling, spp):
    """`--scaling strong` (default): a step is the metric's fixed job -- every pixel of
    the frame at 256 spp (config 3's SAMPLES), one pass from sample 0, at any N;
    `--scaling weak`: a rank's pixels take N x 256 spp per step (per-GPU work fixed)."""
    args = ["--gpus", "2", "--probe-ranks", "--steps", "3"] + (["--scaling", scaling] if scaling else [])
    rc, out, err = _bench(args)
    assert rc == 0, err[-2000:]
    assert out["scaling"] == (scaling or "strong")
    assert out["rank_spp_per_step"] == spp and out["pass_spp"] == spp
    assert sorted(r["rank"] for r in out["ranks"]) == [0, 1]


def test_bench_refuses_mismatched_world():
    """under torchrun, a WORLD_SIZE that differs from --gpus is an error, not a
    silently relabelled run"""
    rc, out, err = _bench(["--gpus", "2", "--probe-ranks"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert rc == 2 and out is None
    assert "refusing" in err


def test_bench_roofline_counts_the_path_engine_alone(tmp_path):
    """bench.py's k_wpath roofline subtracts the cooperative engine's share
    (pt_stats coop_* fields) from the visit counts, time and launches, and
    scales the profiled traffic ratio by the path engine's own bytes."""
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    keys = ("isect_launches", "isect_ms", "node_visits", "prim_tests", "aux_visits", "rays", "coop_launches",
            "coop_ms", "coop_node_visits", "coop_prim_tests", "coop_aux_visits", "coop_rays")
    st0 = dict.fromkeys(keys, 0)
    st0.update(node_bytes=32, prim_bytes=48, aux_bytes=128)
    st1 = dict(st0, isect_launches=6, isect_ms=110.0, node_visits=1000, prim_tests=400, aux_visits=2000, rays=500,
               coop_launches=1, coop_ms=10.0, coop_node_visits=100, coop_prim_tests=40, coop_aux_visits=200,
               coop_rays=50)
    tj = tmp_path / "traffic.json"
    tj.write_text(json.dumps({"k": {"traffic_per_alg_byte": 1.5, "profile": "p"}}))
    r = bench.roofline(st0, st1, str(tj), "k")
    alg = (900 * 32 + 360 * 48 + 1800 * 128) / 5.0
    assert r["launches"] == 5 and abs(r["launch_ms"] - 20.0) < 1e-9
    assert abs(r["alg_bytes_per_launch"] - alg) < 1e-6
    assert abs(r["achieved"] - alg / 0.020 / 1e9) < 1e-9
    assert abs(r["traffic"] - 1.5 * alg) < 1e-6 and abs(r["rays_share"] - 0.9) < 1e-12
    assert r["coop"]["launches"] == 1 and r["coop"]["rays"] == 50
