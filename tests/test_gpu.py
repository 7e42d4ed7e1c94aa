"""GPU parity tests (MI355X): the HIP render path through the C ABI vs the
reference's golden outputs and vs the CPU oracle.  Bar: bit-exact -- the
renderer reproduces the reference's RNG streams, tree and float op order, so
images (8-bit) and pre-tonemap fp32 radiance must match exactly.
"""
import numpy as np
import pytest

import _util as U

pytestmark = pytest.mark.gpu
M = U.manifest()


@pytest.fixture(scope="module")
def pt():
    mod = U.ptrace()
    if not U.gpu_available():
        pytest.fail("GPU tests need a visible gfx950 device")
    return mod


TRAVERSALS = {"replay": 0, "exact": 1, "replay_div": 2}


@pytest.mark.parametrize("trav", sorted(TRAVERSALS))
@pytest.mark.parametrize("name", sorted(M["images"]))
def test_golden_images_bit_exact(pt, name, trav):
    # default engine choice: windows of at most 4,096 pixels run the cooperative
    # engine (one wave per chain) from the start, larger ones the path engine first
    m, img, rad = U.golden_image(name)
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        s.prepare()
        win = tuple(m["window"]) if m["window"] else None
        rgb, r, st = s.render(radiance=True, window=win, traversal=TRAVERSALS[trav])
    assert st["errors"] == 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)


def test_config1_full_md5_and_ray_count(pt):
    full = M["full"]["c1"]
    with pt.Scene.load(U.scene_path("c1")) as s:
        rgb, _, st = s.render()
    ppm = b"P6\n256 256\n255\n" + rgb.tobytes()
    assert U.md5(ppm) == full["md5"]
    assert st["rays"] == full["rays"]


def test_config2_full_md5_and_ray_count(pt, tmp_path):
    # dragon_10k 512x512x64 = the reference's 320 s render
    full = M["full"]["c2"]
    with pt.Scene.load(U.scene_path("c2")) as s:
        rgb, _, st = s.render()
    out = tmp_path / "c2.ppm"
    pt.write_ppm(str(out), rgb)
    assert U.md5(out.read_bytes()) == full["md5"]
    assert st["rays"] == full["rays"]
    assert np.allclose(rgb.reshape(-1, 3).mean(0), full["mean8"], atol=5e-5)


def test_standin_windows_vs_oracle_with_counters(pt):
    # 1080p stand-in (config 3 geometry) at 2 spp: random windows vs the oracle,
    # including the traversal work counters (same tree, same visits)
    p = U.scene_path("c3")
    o = U.OracleScene(p)
    rng = np.random.default_rng(7)
    with pt.Scene.load(p) as s:
        for _ in range(3):
            x0, y0 = int(rng.integers(0, 1920 - 24)), int(rng.integers(0, 1080 - 16))
            orgb, orad, octr = o.render(x0, y0, 24, 16, spp=2)
            rgb, rad, st = s.render(samples=2, radiance=True, window=(x0, y0, 24, 16), traversal=1)
            assert rad.view(np.uint32).tolist() == orad.view(np.uint32).tolist()
            assert np.array_equal(rgb, orgb)
            assert st["rays"] == octr["rays"]
            assert st["node_visits"] == octr["nodes"]
            assert st["prim_tests"] == octr["prim_tests"]
            assert st["plane_tests"] == octr["planes"]
            # candidate replay: same image, same rays, far fewer node records
            rgb2, rad2, st2 = s.render(samples=2, radiance=True, window=(x0, y0, 24, 16), traversal=0)
            assert np.array_equal(rad2.view(np.uint32), orad.view(np.uint32))
            assert st2["rays"] == octr["rays"] and st2["errors"] == 0
            assert st2["node_visits"] * 10 < st["node_visits"]


@pytest.mark.parametrize("variant", ["metal", "glass"])
def test_deep_bounce_variants_vs_oracle(pt, variant):
    p = U.scene_path("practice5_dragon_10k.txt", (96, 96, 4, False, variant))
    o = U.OracleScene(p)
    orgb, orad, octr = o.render()
    with pt.Scene.load(p) as s:
        rgb, rad, st = s.render(radiance=True)
    assert rad.view(np.uint32).tolist() == orad.view(np.uint32).tolist()
    assert np.array_equal(rgb, orgb)
    assert st["rays"] == octr["rays"]


def test_tile_sharding_and_progressive_chunks_identical(pt):
    # ranks 0..world-1 on one device, stitched == single-rank render; spp split
    # into launches of 1, 3 and 7 samples == one launch (streams continue exactly)
    p = U.scene_path("practice5_dragon_10k.txt", (80, 56, 7, False, "diffuse"))
    with pt.Scene.load(p) as s:
        s.prepare()
        ref, _, _ = s.render(spp_per_launch=7)
        for chunk in (1, 3):
            img, _, _ = s.render(spp_per_launch=chunk)
            assert np.array_equal(img, ref)
        for world in (2, 3, 5):
            out = np.zeros_like(ref)
            for r in range(world):
                ss = pt.Session(s, rank=r, world=world)
                ss.trace(4)
                ss.trace(3)
                ss.resolve()
                ss.sync()
                pt.unpack_tiles(ss.read_packed(), 80, 56, r, world, out=out)
                ss.close()
            assert np.array_equal(out, ref)


def test_determinism_repeat(pt):
    p = U.scene_path("hw3_sample4.txt", (64, 64, 8, False, "diffuse"))
    with pt.Scene.load(p) as s:
        a, ra, _ = s.render(radiance=True)
        b, rb, _ = s.render(radiance=True)
    assert np.array_equal(a, b) and np.array_equal(ra.view(np.uint32), rb.view(np.uint32))


def test_cli_drop_in_config1(pt, tmp_path):
    # build.sh/run.sh surface: `pt_render scene.txt out.ppm` (hw5/run.sh:1-2)
    import subprocess
    out = tmp_path / "c1.ppm"
    exe = U.os.path.join(U.PKG, "build", "pt_render")
    r = subprocess.run([exe, U.scene_path("c1"), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    # the bar is reported from inside one pass (finished-sample counter): all ten steps, in order
    bars = [l for l in r.stdout.splitlines() if l.startswith("Loading: [")]
    assert [b.split()[-2] for b in bars] == ["%d%%" % (10 * k) for k in range(1, 11)], bars
    assert U.md5(out.read_bytes()) == M["full"]["c1"]["md5"]
    # quiet: same bytes, no bar
    out2 = tmp_path / "c1q.ppm"
    r = subprocess.run([exe, U.scene_path("c1"), str(out2)], capture_output=True, text=True, timeout=300,
                       env=dict(U.os.environ, PT_QUIET="1"))
    assert r.returncode == 0 and "Loading" not in r.stdout, r.stderr
    assert out2.read_bytes() == out.read_bytes()


def test_device_init(pt):
    # optional runtime start-up (the CLI runs it beside the scene parse): idempotent,
    # and a bad index fails loudly
    assert pt._lib.pt_device_init(0) == pt.PT_OK
    assert pt._lib.pt_device_init(0) == pt.PT_OK
    assert pt._lib.pt_device_init(4096) == pt.PT_E_NO_GPU


@pytest.mark.parametrize("engine", ["coop64", "coop32", "coop16", "coop8", "coop4", "coop8grow", "path"])
@pytest.mark.parametrize("name", sorted(M["images"]))
def test_golden_images_each_engine(pt, name, engine, monkeypatch):
    """The replay traversal with one engine for the whole pass: the cooperative
    engine (a team of 64, 32, 16, 8 or 4 lanes per chain: breadth-first aux expansion,
    all candidate leaves at once, root paths a block of nodes per round;
    pt_coop.h) or the path engine alone (coop=0).  All must reproduce the
    reference's bytes and ray count.  coop8grow: teams of 8 that hand their last 64
    chains to whole-wave teams (a second launch, coop_grow)."""
    coop = engine.startswith("coop")
    grow = engine.endswith("grow")
    team = engine[4:].replace("grow", "") if coop else "64"
    monkeypatch.setenv("PT_TUNE", "coop=%s,coop_team=%s,coop_grow=%d" % ("100000000" if coop else "0", team,
                                                                       64 if grow else 0))
    m, img, rad = U.golden_image(name)
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        s.prepare()
        win = tuple(m["window"]) if m["window"] else None
        rgb, r, st = s.render(radiance=True, window=win, traversal=0)
    assert st["errors"] == 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)
    if coop:
        # (the hand-over happens only if a chain is still running at a chain cycle after
        # all but 64 have ended: at a few spp the last ones can all end in that cycle)
        assert st["rounds"] in ((1, 2) if grow else (1,))


@pytest.mark.parametrize("team", ["64", "16", "8", "4", "8grow"])
@pytest.mark.parametrize("cfg", ["c1", "c2"])
def test_coop_engine_full_config_md5(pt, cfg, team, monkeypatch):
    """Configs 1 and 2 entirely on the cooperative engine: reference md5 and ray count
    (8grow: teams of 8, the last 1,024 chains to whole-wave teams -- the default
    hand-over of the pass's final launch)."""
    grow = team.endswith("grow")
    monkeypatch.setenv("PT_TUNE", "coop=100000000,coop_team=%s,coop_grow=%d" % (team.replace("grow", ""),
                                                                             1024 if grow else 0))
    full = M["full"][cfg]
    with pt.Scene.load(U.scene_path(cfg)) as s:
        rgb, _, st = s.render()
        w, h = s.info["width"], s.info["height"]
    ppm = b"P6\n%d %d\n255\n" % (w, h) + rgb.tobytes()
    assert U.md5(ppm) == full["md5"]
    assert st["rays"] == full["rays"] and st["rounds"] == (2 if grow else 1)


@pytest.mark.parametrize("engine", ["path", "path_dense", "path_coop"])
@pytest.mark.parametrize("budget", ["1", "3"])
@pytest.mark.parametrize("name", ["c3s4_win_944_520_16x16", "c4glass_s4_win_900_560_16x16", "dragon_64x64x16",
                                  "hw3s4_48x48x8", "c2_win_240_200_24x24"])
def test_suspended_queries_resume_bit_exact(pt, name, budget, engine, monkeypatch):
    """Force the path engine to suspend almost every query 1-3 loop trips after
    its wave ran out of round work (PT_TUNE budget, read at session creation):
    queries then resume from the carry queue over many rounds, interleaving
    pixels' samples arbitrarily -- results must not change.  "path" lets the
    engine switch to its end-of-pass (sparse) kernel once few chains are left,
    as it does by default; "path_dense" keeps the main kernel for every round;
    "path_coop" hands the suspended queries and queued rays to the cooperative
    engine once fewer than a quarter of the pixels have chains left."""
    m, img, rad = U.golden_image(name)
    npx = int(np.prod(img.shape[:2]))
    coop = npx // 4 if engine == "path_coop" else 0
    monkeypatch.setenv("PT_TUNE", "budget=%s,sparse=%s,coop=%d" % (
        budget, "0" if engine == "path_dense" else "100000000", coop))
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        s.prepare()
        win = tuple(m["window"]) if m["window"] else None
        rgb, r, st = s.render(radiance=True, window=win, traversal=0)
    assert st["errors"] == 0
    assert st["rounds"] > (1 if engine == "path_coop" else 0)
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)


@pytest.mark.parametrize("name", ["dragon_64x64x16", "c3s4_win_944_520_16x16", "rabbid_48x48x4"])
def test_aux_stack_overflow_takes_exact_dfs(pt, name, monkeypatch):
    """A path-engine query whose pending aux items outgrow its LDS stack (PT_TUNE
    lstack=1 here; PT_LSTACK words by default) hands its ray to k_wexact (the replay
    again with a stack as deep as the aux tree needs, then the exact DFS if the
    replay cannot take it): same bytes and ray count, and the hand-over is counted."""
    monkeypatch.setenv("PT_TUNE", "lstack=1,coop=0")
    m, img, rad = U.golden_image(name)
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        s.prepare()
        win = tuple(m["window"]) if m["window"] else None
        rgb, r, st = s.render(radiance=True, window=win)
    assert st["errors"] == 0 and st["fallbacks"] > 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)


def test_exact_handover_beyond_the_query_lanes(pt, monkeypatch):
    """More hand-overs to k_wexact in one round than the path engine has query lanes
    (PT_TUNE lstack=1 on config 2's 262,144 pixels at one sample: nearly every query
    outgrows a one-word stack; 256 CUs x 4 workgroups x 128 query lanes = 131,072):
    the hand-over queues hold one entry per pixel, so the image and radiance equal the
    default stack's bit for bit (which the config-2 md5 test pins to the reference)."""
    with pt.Scene.load(U.scene_path("c2")) as s:
        s.prepare()
        ref, rref, st0 = s.render(samples=1, radiance=True)
        monkeypatch.setenv("PT_TUNE", "lstack=1,coop=0")
        rgb, r, st = s.render(samples=1, radiance=True)
    assert st["errors"] == 0 and st["fallbacks"] > 140000
    assert st["rays"] == st0["rays"]
    assert r.view(np.uint32).tolist() == rref.view(np.uint32).tolist()
    assert np.array_equal(rgb, ref)


def test_megakernel_engine_bit_exact(pt, monkeypatch):
    """PT_TUNE engine=mega: the megakernel (one lane per pixel, whole paths) on the
    replay traversal gives the same bytes as the path engine"""
    monkeypatch.setenv("PT_TUNE", "engine=mega")
    m, img, rad = U.golden_image("dragon_64x64x16")
    with pt.Scene.load(U.golden_scene_path("dragon_64x64x16")) as s:
        rgb, r, st = s.render(radiance=True, traversal=0)
    assert st["rounds"] == 0 and st["errors"] == 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)


C5_WINDOWS = ["c5s4_win_1920_1072_16x16", "c5s4_win_1952_1072_32x16", "c5s4_win_1760_1200_16x16",
              "c5s4_win_3824_2144_16x16"]


def test_config5_rank_of_8_sessions_vs_reference_windows(pt):
    """Config 5 (3840x2160, the BASELINE's 8-GPU config) as the 8-rank run renders it:
    a session per rank owning every 8th 16x16 tile of the 4K frame (seeds y*3840+x),
    4 spp.  The pixels of the reference's golden windows must come out of the
    ranks that own them bit-exactly (8-bit and fp32 radiance)."""
    import torch
    world, W, H = 8, 3840, 2160
    wins = {n: U.golden_image(n) for n in C5_WINDOWS}
    m0 = wins[C5_WINDOWS[0]][0]
    tiles_x = W // 16
    owners = {}
    for n, (m, _, _) in wins.items():
        x0, y0, w, h = m["window"]
        for ty in range(y0 // 16, (y0 + h + 15) // 16):
            for tx in range(x0 // 16, (x0 + w + 15) // 16):
                owners.setdefault((tx + ty) % world, set()).add(n)
    assert len(owners) >= 4   # the windows span several ranks (1, 3, 5, 6)
    rgb = np.zeros((H, W, 3), np.uint8)
    rad = np.zeros((H, W, 3), np.float32)
    covered = np.zeros((H, W), bool)
    with pt.Scene.load(U.golden_scene_path(C5_WINDOWS[0])) as s:
        s.prepare()
        assert (s.info["width"], s.info["height"], s.info["samples"]) == (W, H, 4)
        for r in sorted(owners):
            ss = pt.Session(s, rank=r, world=world)
            ss.trace(4)
            drad = torch.empty(ss.n_tiles * 256 * 3, dtype=torch.float32, device="cuda")
            ss.resolve(dev_rad=drad.data_ptr())
            ss.sync()
            assert ss.stats()["errors"] == 0
            pt.unpack_tiles(ss.read_packed(), W, H, r, world, out=rgb)
            pt.unpack_tiles_f32(drad.cpu().numpy(), W, H, r, world, out=rad)
            mine = np.zeros(((H + 15) // 16, tiles_x), bool)
            mine.reshape(-1)[pt.rank_tiles(W, H, r, world)] = True
            covered |= np.repeat(np.repeat(mine, 16, 0), 16, 1)[:H, :W]
            ss.close()
    assert m0["gen"][:3] == [W, H, 4]
    for n, (m, img, wrad) in wins.items():
        x0, y0, w, h = m["window"]
        assert covered[y0:y0 + h, x0:x0 + w].all(), n
        assert rad[y0:y0 + h, x0:x0 + w].view(np.uint32).tolist() == wrad.view(np.uint32).tolist(), n
        assert np.array_equal(rgb[y0:y0 + h, x0:x0 + w], img), n


@pytest.mark.parametrize("ngpu_gather", ["rccl", "host", "auto"])
def test_render_gather_paths(pt, ngpu_gather):
    """pt_render's framebuffer gather: PT_GATHER_RCCL runs the ncclGather path
    (ncclCommInitAll + grouped ncclGather, a one-rank communicator on one GPU) and
    must give the same bytes as the host gather; gather_rccl records which ran."""
    mode = {"rccl": pt.GATHER_RCCL, "host": pt.GATHER_HOST, "auto": pt.GATHER_AUTO}[ngpu_gather]
    m, img, rad = U.golden_image("dragon_64x64x16")
    with pt.Scene.load(U.golden_scene_path("dragon_64x64x16")) as s:
        rgb, r, st = s.render(radiance=True, gather=mode)
        rgb2, _, st2 = s.render(gather=mode)   # the cached communicator is reused
        rgb3, _, st3 = s.render(gather=mode)   # ... and its buffers: nothing allocated
    assert st["gather_rccl"] == (1 if ngpu_gather == "rccl" else 0)
    assert st2["gather_rccl"] == st3["gather_rccl"] == st["gather_rccl"]
    assert st2["gather_allocs"] == st3["gather_allocs"] == 0
    if ngpu_gather != "rccl":
        assert st["gather_allocs"] == 0
    assert np.array_equal(rgb, img) and np.array_equal(rgb2, img) and np.array_equal(rgb3, img)
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()


def test_session_reset_renders_the_job_again(pt):
    """pt_session_reset restarts every owned pixel at sample 0: after any pass, reset +
    trace(S) gives the bytes, radiance and rays of a new session's trace(S) (bench.py
    repeats the metric's frame this way)."""
    m, img, rad = U.golden_image("dragon_64x64x16")
    with pt.Scene.load(U.golden_scene_path("dragon_64x64x16")) as s:
        s.prepare()
        spp = s.info["samples"]
        outs = []
        ss = pt.Session(s, device=0)
        for pre in (0, 5, spp):
            if pre:
                ss.trace(pre)
                ss.sync()
                ss.reset()
            st0 = ss.stats()
            ss.trace(spp)
            ss.resolve()
            ss.sync()
            st1 = ss.stats()
            outs.append((ss.read_packed(), st1["rays"] - st0["rays"]))
        ss.close()
        ref, _, st = s.render()
    for packed, rays in outs:
        got = np.zeros_like(ref)
        pt.unpack_tiles(packed, ref.shape[1], ref.shape[0], 0, 1, got)
        assert np.array_equal(got, img) and rays == st["rays"]


def test_rccl_gather_buffers_grow_once(pt):
    """The RCCL gather's send / receive buffers are kept per communicator: a render of a
    larger frame than any before grows them once (gather_allocs > 0), and the next
    renders of either size allocate nothing and keep the bytes."""
    with pt.Scene.load(U.scene_path("c1")) as s:
        big, _, st = s.render(gather=pt.GATHER_RCCL)
        small, _, st2 = s.render(gather=pt.GATHER_RCCL, window=(16, 32, 64, 48))
        big2, _, st3 = s.render(gather=pt.GATHER_RCCL)
    assert st["gather_rccl"] == st2["gather_rccl"] == st3["gather_rccl"] == 1
    assert st2["gather_allocs"] == 0 and st3["gather_allocs"] == 0
    assert np.array_equal(big, big2) and np.array_equal(small, big[32:80, 16:80])
    ppm = b"P6\n%d %d\n255\n" % (big.shape[1], big.shape[0]) + big.tobytes()
    assert U.md5(ppm) == M["full"]["c1"]["md5"]


def test_rccl_gather_fails_over_to_the_host(pt, monkeypatch):
    """PT_GATHER_AUTO: when the RCCL gather fails (PT_TUNE inject_rccl=1 fails it before
    any RCCL call), pt_render gathers through the host: the same bytes, gather_rccl = 0,
    and the reason in pt_last_error.  PT_GATHER_RCCL makes the same failure an error."""
    monkeypatch.setenv("PT_TUNE", "inject_rccl=1")
    m, img, rad = U.golden_image("dragon_64x64x16")
    with pt.Scene.load(U.golden_scene_path("dragon_64x64x16")) as s:
        rgb, r, st = s.render(radiance=True, gather=pt.GATHER_AUTO)
        assert "injected RCCL gather failure" in pt.last_error()
        with pytest.raises(pt.PTError, match="injected RCCL gather failure"):
            s.render(gather=pt.GATHER_RCCL)
    assert st["gather_rccl"] == 0 and st["gather_allocs"] == 0
    assert np.array_equal(rgb, img)
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()


@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("ngpu", [2, 3, 8])
@pytest.mark.parametrize("cfg", ["c1", "c2"])
def test_render_ngpu_sessions_on_one_device(pt, cfg, ngpu, mode, monkeypatch):
    """pt_render(ngpu = n): n host threads, each setting up its own tile session
    (rank g of n) and driving it -- the drop-in's own multi-GPU path -- run here with
    every session on device 0 (PT_TUNE same_device=1, framebuffer through the host;
    same_device=2: the ranks render one after another once all are set up).  The
    gathered image and the summed ray count must equal the reference's (= ngpu 1)."""
    monkeypatch.setenv("PT_TUNE", "same_device=" + mode)
    full = M["full"][cfg]
    with pt.Scene.load(U.scene_path(cfg)) as s:
        rgb, _, st = s.render(ngpu=ngpu)
        w, h = s.info["width"], s.info["height"]
    ppm = b"P6\n%d %d\n255\n" % (w, h) + rgb.tobytes()
    assert U.md5(ppm) == full["md5"]
    assert st["rays"] == full["rays"] and st["errors"] == 0 and st["gather_rccl"] == 0


def test_render_ngpu_concurrent_sessions_repeated(pt, monkeypatch):
    """Four sessions rendering config 2 at once on device 0 (same_device=1), ten times:
    their workgroups start late and interleave differently on each render, which is how
    the final launch's hand-on bug showed (2 failed renders in 40 before its fix;
    DESIGN §5).  Every render must give the reference's bytes and ray count."""
    monkeypatch.setenv("PT_TUNE", "same_device=1")
    full = M["full"]["c2"]
    with pt.Scene.load(U.scene_path("c2")) as s:
        w, h = s.info["width"], s.info["height"]
        for _ in range(10):
            rgb, _, st = s.render(ngpu=4)
            ppm = b"P6\n%d %d\n255\n" % (w, h) + rgb.tobytes()
            assert U.md5(ppm) == full["md5"]
            assert st["rays"] == full["rays"] and st["errors"] == 0 and st["short_pixels"] == 0


@pytest.mark.parametrize("mode", ["1", "2"])
def test_cli_ngpu_sessions_on_one_device(pt, tmp_path, mode):
    """The CLI with PT_NGPU=4 (4 sessions on device 0, PT_TUNE same_device=1 or 2): the
    reference's config-1 bytes; the communicator set-up is done on the start-up
    thread (phases_ms comm_init), not after the render; PT_STATS=2 prints every
    rank's set-up / render / resolve times and the gather's."""
    import re
    import subprocess
    out = tmp_path / "c1.ppm"
    exe = U.os.path.join(U.PKG, "build", "pt_render")
    r = subprocess.run([exe, U.scene_path("c1"), str(out)], capture_output=True, text=True, timeout=300,
                       env=dict(U.os.environ, PT_QUIET="1", PT_STATS="2", PT_NGPU="4", PT_TUNE="same_device=" + mode))
    assert r.returncode == 0, r.stderr
    assert "ngpu=4" in r.stderr and "comm_init=" in r.stderr, r.stderr
    ranks = re.findall(r"pt_render rank (\d)/4: setup_ms=[\d.]+ scene_upload_ms=([\d.]+) wait_ms=[\d.]+ "
                       r"render_ms=[\d.]+ resolve_ms=[\d.]+", r.stderr)
    assert sorted(int(g) for g, _ in ranks) == [0, 1, 2, 3], r.stderr
    # one device: exactly one session uploads the scene
    assert sum(float(u) > 0 for _, u in ranks) == 1, r.stderr
    assert "pt_render gather_ms=" in r.stderr
    assert U.md5(out.read_bytes()) == M["full"]["c1"]["md5"]


# Every scheduling knob of PT_TUNE must leave the bytes alone: a
# knob changes which chains run where and when, never a pixel's stream or its float
# order.  Each runs the path engine (coop=0, budget=2: many rounds, suspensions) on a
# dragon window against the reference's fixture.  (engine, budget, runend, sparse,
# coop, coop_team, lstack, same_device: the tests above.)
TUNE_KEYS = ["wg_per_cu=2", "wg_per_cu=1", "runend=1000000", "sparse_steps=2", "sparse_steps=16", "round_batch=4",
             "probe_every=1", "probe_min=1", "aux_extra=0", "aux_extra=3", "lowq=0", "lowq=100000000",
             "lowq=100000000,lowq_wg=1", "lowq=100000000,lowq_budget_us=20", "lowq=100000000,lowq_probe_every=1,lowq_probe_min=2,lowq_aux_extra=2",
             "cap=64", "batch=1", "batch=64", "budget_us=20", "budget_us=0", "roundlog=1", "roundlog=2", "roundlog=3", "prepstats=1",
             # the cooperative engine after the path rounds, intake in queue order / by samples left
             "coop=300,coop_order=0", "coop=300,coop_order=1",
             # its last chains handed to whole-wave teams (a second launch), or never
             "coop=300,coop_grow=100", "coop=300,coop_grow=1", "coop=300,coop_grow=0",
             "coop=300,coop_grow=50,coop_grow_mid=200", "coop=300,coop_grow=0,coop_grow_mid=200",
             # the early cooperative launch on a second stream (the heaviest chains, from the first
             # count on), beside the path rounds
             "coop=300,early=1,early_at=100000000", "coop=300,early=64,early_at=100000000,early_wg=2",
             "coop=300,early=0", "coop=300,early=1,early_at=100000000,coop_order=1",
             # more early workgroups than fit beside the round (the late ones find it over and
             # hand their untaken items on)
             "coop=300,early=1,early_at=100000000,early_wg=8",
             # every early workgroup a late one (side_late), the side stream at each priority
             "coop=300,early=1,early_at=100000000,side_late=1",
             "coop=300,early=1,early_at=100000000,side_prio=0", "coop=300,early=1,early_at=100000000,side_prio=2",
             "coop=300,early=1,early_at=100000000,side_team=16", "coop=300,early=1,early_at=100000000,side_team=8",
             "coop=300,coop_team=8",
             # diagnostics hooks (their counters are compiled in only with -DPT_CPROF / -DPT_WPROF;
             # the host side runs in every build)
             "coop=300,cprof=1", "wgprof=/tmp/pt_wgprof_test.bin"]


@pytest.mark.parametrize("tune", TUNE_KEYS)
@pytest.mark.parametrize("name", ["dragon_64x64x16", "c2_win_240_200_24x24"])
def test_tuning_keys_bit_exact(pt, name, tune, monkeypatch):
    monkeypatch.setenv("PT_TUNE", ("" if tune.startswith("coop=") else "coop=0,") + "budget=2," + tune)
    m, img, rad = U.golden_image(name)
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        s.prepare()
        win = tuple(m["window"]) if m["window"] else None
        rgb, r, st = s.render(radiance=True, window=win, traversal=0)
    assert st["errors"] == 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)


SIDE = "coop=300,budget=2,early=1,early_at=100000000,early_wg=8,side_late=1"


@pytest.mark.parametrize("name", ["dragon_64x64x16", "c2_win_240_200_24x24"])
def test_side_launch_hand_on_runs_and_is_counted(pt, name, monkeypatch):
    """The early cooperative launch's workgroups that find their round over take nothing
    and hand the round's untaken work items on (k_wcoop, after its main loop).  PT_TUNE
    side_late=1 makes every workgroup such a late one, so the hand-on path certainly runs:
    pt_stats.handed_on counts its items, and the bytes stay the reference's."""
    monkeypatch.setenv("PT_TUNE", SIDE)
    m, img, rad = U.golden_image(name)
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        win = tuple(m["window"]) if m["window"] else None
        rgb, r, st = s.render(radiance=True, window=win)
    assert st["handed_on"] > 0 and st["short_pixels"] == 0 and st["errors"] == 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)


@pytest.mark.parametrize("name", ["dragon_64x64x16", "c2_win_240_200_24x24"])
def test_final_launch_hand_on_follows_the_intake_order(pt, name, monkeypatch):
    """The pass's final cooperative launch takes its work items through the intake order
    (coop_order) and, with a grow stop (coop_grow), hands the ones no team took on to the
    next launch.  A workgroup that starts late (a device shared with other sessions) finds
    such items; they must be handed on through the same order, or one item runs twice and
    another never (pixels +1 / -1 samples).  PT_TUNE grow_late=1 makes the odd workgroups
    late ones."""
    monkeypatch.setenv("PT_TUNE", "coop=100000000,coop_order=1,coop_grow=1,grow_late=1")
    m, img, rad = U.golden_image(name)
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        win = tuple(m["window"]) if m["window"] else None
        rgb, r, st = s.render(radiance=True, window=win)
    assert st["handed_on"] > 0 and st["short_pixels"] == 0 and st["errors"] == 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)


def test_lost_chains_fail_the_resolve(pt, monkeypatch):
    """A chain the engines lose leaves its pixel short of the pass target.  The resolve
    counts the owned pixels whose sample count differs from the samples traced and fails
    (src/scene.cpp:192-199: every pixel takes exactly SAMPLES samples): with the hand-on
    loop disabled (PT_TUNE handon=0) the untaken items are dropped, and pt_render must
    return that error, not an image."""
    monkeypatch.setenv("PT_TUNE", SIDE + ",handon=0")
    with pt.Scene.load(U.golden_scene_path("dragon_64x64x16")) as s:
        with pytest.raises(pt.PTError, match="did not take exactly"):
            s.render()


# Every place where work changes hands between the engines' launches, waves and queues
# (DESIGN.md §4 "Hand-off sites"), with the PT_TUNE setting that makes it certainly run.
# pt_stats.handoff counts each site's items where they change hands.
HANDOFF_FORCE = {
    "suspend": "coop=0,runend=0,budget=2",                      # path round end: running queries -> carry queue
    "flush": "coop=0,runend=0,budget=2,shade_hold=1",          # shade wave after the query waves left -> fresh queue
    "ringout": "coop=0,runend=0,budget=2",                     # ray-ring leftovers at the shade wave's exit
    "exact": "coop=0,lstack=1",                         # path query -> k_wexact / k_wshade
    "side_take": "coop=300,budget=2,early=1,early_at=100000000",                    # early launch's intake
    "side_yield": "coop=300,budget=2,early=1,early_at=100000000,side_stop_now=1",   # its stop: yields
    "side_handon": "coop=300,budget=2,early=1,early_at=100000000,early_wg=8,side_late=1",   # late workgroups
    "grow_yield": "coop=100000000,coop_grow=100",        # final launch's grow stop: yields
    "grow_handon": "coop=100000000,coop_order=1,coop_grow=1,grow_late=1",   # its late workgroups
}


# every site with the defaults, the early launch's sites also with teams of 8 (the default is 4)
# and the final launch's also with teams of 8 (the default is 4)
HANDOFF_CASES = [(k, "") for k in sorted(HANDOFF_FORCE)] + \
    [(k, ",side_team=8") for k in sorted(HANDOFF_FORCE) if k.startswith("side_")] + \
    [(k, ",coop_team=8") for k in sorted(HANDOFF_FORCE) if k.startswith("grow_")]


@pytest.mark.parametrize("site,team", HANDOFF_CASES)
def test_handoff_site_runs_and_keeps_every_sample(pt, site, team, monkeypatch):
    """Each hand-off site, forced: its items are counted (pt_stats.handoff > 0), no pixel
    is short of its samples, and the bytes and radiance bits are the reference's."""
    monkeypatch.setenv("PT_TUNE", HANDOFF_FORCE[site] + team)
    m, img, rad = U.golden_image("dragon_64x64x16")
    with pt.Scene.load(U.golden_scene_path("dragon_64x64x16")) as s:
        rgb, r, st = s.render(radiance=True)
    assert st["handoff"][site] > 0, st["handoff"]
    assert st["short_pixels"] == 0 and st["errors"] == 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)


@pytest.mark.parametrize("site,team", HANDOFF_CASES)
def test_handoff_site_dropped_fails_the_resolve(pt, site, team, monkeypatch):
    """The same site forced with its hand-on disabled (PT_TUNE drop=<site>: its items are
    dropped, not handed on): the chains are lost, and pt_render must return the resolve's
    lost-chain error (src/scene.cpp:192-199: every pixel takes exactly SAMPLES samples)."""
    monkeypatch.setenv("PT_TUNE", HANDOFF_FORCE[site] + team + ",drop=" + site)
    with pt.Scene.load(U.golden_scene_path("dragon_64x64x16")) as s:
        with pytest.raises(pt.PTError, match="did not take exactly"):
            s.render()


def test_handoff_drop_names_are_checked(pt, monkeypatch):
    monkeypatch.setenv("PT_TUNE", "drop=nowhere")
    with pt.Scene.load(U.golden_scene_path("dragon_64x64x16")) as s:
        with pytest.raises(pt.PTError, match="no such hand-off site"):
            s.render()


@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("bad", [0, 1, 2])
def test_render_ngpu_failed_rank_returns(pt, mode, bad, monkeypatch):
    """pt_render(ngpu = 3) with one rank failing after its set-up (PT_TUNE inject_fail):
    the call returns that rank's error -- with same_device=2 (ranks rendering in turn) a
    failed rank must not leave a later one waiting for its turn."""
    monkeypatch.setenv("PT_TUNE", "same_device=%s,inject_fail=%d" % (mode, bad))
    with pt.Scene.load(U.scene_path("c1")) as s:
        with pytest.raises(pt.PTError, match="injected failure"):
            s.render(ngpu=3)


def test_gather_init_one_rank(pt):
    """pt_gather_init creates (and caches) the RCCL communicator pt_render's gather uses."""
    assert pt._lib.pt_gather_init(0, 1) == pt.PT_OK
    assert pt._lib.pt_gather_init(0, 1) == pt.PT_OK


def test_cli_rccl_gather_config1(pt, tmp_path):
    """The drop-in CLI's multi-GPU gather (PT_GATHER=rccl; PT_NGPU=n uses the
    same code with n ranks) on config 1: same bytes as the reference."""
    import subprocess
    out = tmp_path / "c1.ppm"
    exe = U.os.path.join(U.PKG, "build", "pt_render")
    r = subprocess.run([exe, U.scene_path("c1"), str(out)], capture_output=True, text=True, timeout=300,
                       env=dict(U.os.environ, PT_QUIET="1", PT_STATS="1", PT_GATHER="rccl"))
    assert r.returncode == 0, r.stderr
    assert "gather_rccl=1" in r.stderr, r.stderr
    assert U.md5(out.read_bytes()) == M["full"]["c1"]["md5"]


@pytest.mark.parametrize("engine", ["path", "coop8", "coop64"])
def test_many_hitting_leaves_vs_oracle(pt, tmp_path, engine, monkeypatch):
    """A stack of tilted triangles whose hit regions (their copies on the plane
    through the origin) overlap: camera and bounce rays have dozens of hitting
    leaves, so the path engine's query runs overflow passes and hands rays to the
    exact DFS; every engine must give the oracle's bytes and ray count."""
    import test_host as H
    text = H._stack_scene().replace("DIMENSIONS 8 8", "DIMENSIONS 40 32").replace("SAMPLES 1", "SAMPLES 4")
    text = text.replace("RAY_DEPTH 1", "RAY_DEPTH 3")
    text += "NEW_PRIMITIVE\nPLANE 0 0 1\nPOSITION 0 0 -1\nCOLOR 0.7 0.7 0.7\n"
    text += "NEW_PRIMITIVE\nBOX 0.5 0.5 0.5\nPOSITION 0 0 8\nEMISSION 4 4 4\n"
    p = tmp_path / "stack.txt"
    p.write_text(text)
    o = U.OracleScene(str(p))
    orgb, orad, octr = o.render()
    coop = engine.startswith("coop")
    monkeypatch.setenv("PT_TUNE", "coop=%s,coop_team=%s" % ("100000000" if coop else "0", engine[4:] if coop else "64"))
    with pt.Scene.load(str(p)) as s:
        rgb, rad, st = s.render(radiance=True, traversal=0)
    assert st["errors"] == 0
    assert rad.view(np.uint32).tolist() == orad.view(np.uint32).tolist()
    assert np.array_equal(rgb, orgb)
    assert st["rays"] == octr["rays"]
    if not coop:
        assert st["fallbacks"] > 0


# ---- deep stream positions (round 3): windows at each config's own spp, RAY_DEPTH 10,
# and a scene beyond the cooperative engine's LDS tables (manifest "deep"; the ray
# counts are the CPU restatement's, whose images equal the reference's)
DEEP = M.get("deep", {})


@pytest.mark.parametrize("name", sorted(DEEP))
def test_deep_windows_bit_exact(pt, name):
    """The window alone (its pixels' full sample streams: 256 / 1024 / 4096 spp for
    configs 3 / 4 / 5), bit-exact with the reference, and the restatement's ray count."""
    m = DEEP[name]
    img = U.read_ppm(U.os.path.join(U.GOLDEN, "img_%s.ppm" % name))
    rad = np.fromfile(U.os.path.join(U.GOLDEN, "rad_%s.f32" % name), np.float32).reshape(img.shape)
    with pt.Scene.load(U.scene_path(m["scene"], tuple(m["gen"]) if m["gen"] else None)) as s:
        s.prepare()
        win = tuple(m["window"]) if m["window"] else None
        rgb, r, st = s.render(radiance=True, window=win)
    assert st["errors"] == 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)
    assert st["rays"] == m["rays"]


@pytest.mark.parametrize("cfg", ["c3", "c4_metal", "c4_glass"])
def test_deep_full_frame_contains_reference_windows(pt, cfg):
    """The whole 1920x1080 frame at the config's own spp (256 / 1024) -- the bench's
    path: path-engine rounds, suspension, the cooperative hand-over at the pass end --
    must hold the reference's deep windows bit-exactly."""
    names = [n for n, m in DEEP.items() if m["scene"] == cfg and m["gen"] is None]
    assert names
    with pt.Scene.load(U.scene_path(cfg)) as s:
        rgb, rad, st = s.render(radiance=True)
    assert st["errors"] == 0
    for n in names:
        x0, y0, w, h = DEEP[n]["window"]
        img = U.read_ppm(U.os.path.join(U.GOLDEN, "img_%s.ppm" % n))
        wrad = np.fromfile(U.os.path.join(U.GOLDEN, "rad_%s.f32" % n), np.float32).reshape(img.shape)
        assert rad[y0:y0 + h, x0:x0 + w].view(np.uint32).tolist() == wrad.view(np.uint32).tolist(), n
        assert np.array_equal(rgb[y0:y0 + h, x0:x0 + w], img), n


def test_deep_config5_rank_of_8_at_4096_spp(pt):
    """Config 5 as the 8-GPU run renders it, to its full 4096 spp: the sessions of the
    ranks owning the reference's deep 4K windows (rank = (tx + ty) % 8), each the whole
    rank's share of the frame in one coalesced pass."""
    import torch
    world, W, H = 8, 3840, 2160
    names = [n for n, m in DEEP.items() if m["scene"] == "c5"]
    assert names
    tiles_x = W // 16
    owner = {}
    for n in names:
        x0, y0, w, h = DEEP[n]["window"]
        assert x0 // 16 == (x0 + w - 1) // 16 and y0 // 16 == (y0 + h - 1) // 16   # one tile each
        owner[n] = pt.tile_owner((y0 // 16) * tiles_x + x0 // 16, tiles_x, world)
    with pt.Scene.load(U.scene_path("c5")) as s:
        s.prepare()
        assert (s.info["width"], s.info["height"], s.info["samples"]) == (W, H, 4096)
        for r in sorted(set(owner.values())):
            ss = pt.Session(s, rank=r, world=world)
            for _ in range(4):
                ss.trace(1024)   # coalesced into one 4096-spp pass
            drad = torch.empty(ss.n_tiles * 256 * 3, dtype=torch.float32, device="cuda")
            ss.resolve(dev_rad=drad.data_ptr())
            ss.sync()
            assert ss.stats()["errors"] == 0
            rgb = pt.unpack_tiles(ss.read_packed(), W, H, r, world)
            rad = pt.unpack_tiles_f32(drad.cpu().numpy(), W, H, r, world)
            ss.close()
            for n in [k for k, v in owner.items() if v == r]:
                x0, y0, w, h = DEEP[n]["window"]
                img = U.read_ppm(U.os.path.join(U.GOLDEN, "img_%s.ppm" % n))
                wrad = np.fromfile(U.os.path.join(U.GOLDEN, "rad_%s.f32" % n), np.float32).reshape(img.shape)
                assert rad[y0:y0 + h, x0:x0 + w].view(np.uint32).tolist() == wrad.view(np.uint32).tolist(), n
                assert np.array_equal(rgb[y0:y0 + h, x0:x0 + w], img), n


@pytest.mark.parametrize("engine", ["path", "coop8", "coop64"])
@pytest.mark.parametrize("name", ["dragon_d10_metal_48x48x16", "dragon_d10_glass_48x48x16", "many_lights_48x48x8"])
def test_deep_engines_beyond_coop_tables(pt, name, engine, monkeypatch):
    """RAY_DEPTH 10 / 8, 10 planes and 10 emitters: each engine alone for the whole pass
    (the path engine with coop=0; the cooperative engine forced) gives the reference's bytes."""
    if name not in DEEP:
        pytest.fail("deep fixture %s missing" % name)
    coop = engine.startswith("coop")
    monkeypatch.setenv("PT_TUNE", "coop=%s,coop_team=%s" % ("100000000" if coop else "0", engine[4:] if coop else "8"))
    m = DEEP[name]
    img = U.read_ppm(U.os.path.join(U.GOLDEN, "img_%s.ppm" % name))
    rad = np.fromfile(U.os.path.join(U.GOLDEN, "rad_%s.f32" % name), np.float32).reshape(img.shape)
    with pt.Scene.load(U.scene_path(m["scene"], tuple(m["gen"]))) as s:
        rgb, r, st = s.render(radiance=True)
    assert st["errors"] == 0
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)
    assert st["rays"] == m["rays"]
    if coop:
        assert st["coop_launches"] >= 1


# A closed mirror box: every path runs until RAY_DEPTH cuts it, so a pixel's vertex
# count passes 255 (the packed vertex-count field is 24 bits wide).
MIRROR_BOX = """DIMENSIONS 8 8
RAY_DEPTH %d
SAMPLES 2

BG_COLOR 0.1 0.2 0.3

CAMERA_POSITION 0 0 0
CAMERA_RIGHT 1 0 0
CAMERA_UP 0 1 0
CAMERA_FORWARD 0 0 -1
CAMERA_FOV_X 1.2
""" + "".join("""
NEW_PRIMITIVE
PLANE %s
POSITION %s
COLOR 0.99 0.98 0.97
METALLIC
""" % (n, p) for n, p in [("0 1 0", "0 -3 0"), ("0 -1 0", "0 3 0"), ("1 0 0", "-3 0 0"), ("-1 0 0", "3 0 0"),
                          ("0 0 1", "0 0 -3"), ("0 0 -1", "0 0 3")]) + """
NEW_PRIMITIVE
ELLIPSOID 0.15 0.15 0.15
POSITION 1 1 -2
COLOR 0 0 0
EMISSION 40 40 40

NEW_PRIMITIVE
ELLIPSOID 0.6 0.4 0.5
POSITION -1 -1 -2
COLOR 0.9 0.9 0.9
DIELECTRIC
IOR 1.5

NEW_PRIMITIVE
TRIANGLE 0 0 0 1 0 0 0 1 0
POSITION -0.5 0.5 -2.5
ROTATION 0 0.3826834 0 0.9238795
COLOR 0.8 0.6 0.4
METALLIC

NEW_PRIMITIVE
BOX 0.3 0.2 0.4
POSITION 0.8 -1.2 -1.5
COLOR 0.5 0.5 1.0
METALLIC
"""


@pytest.mark.parametrize("engine", ["default", "path", "coop8"])
def test_depth_beyond_255_mirror_box(pt, tmp_path, engine, monkeypatch):
    """RAY_DEPTH 300 in a closed mirror box (paths of up to 300 vertices): the image, the
    radiance bits and the ray count equal the oracle's, in each engine."""
    if engine != "default":
        monkeypatch.setenv("PT_TUNE", "coop=%s,coop_team=8" % ("100000000" if engine == "coop8" else "0"))
    path = str(tmp_path / "mirror_box_d300.txt")
    with open(path, "w") as f:
        f.write(MIRROR_BOX % 300)
    orgb, orad, octr = U.OracleScene(path).render()
    assert octr["rays"] > 64 * 2 * 256   # most paths are longer than 255 vertices
    with pt.Scene.load(path) as s:
        rgb, rad, st = s.render(radiance=True)
    assert st["errors"] == 0
    assert rad.view(np.uint32).tolist() == orad.view(np.uint32).tolist()
    assert np.array_equal(rgb, orgb)
    assert st["rays"] == octr["rays"]
