"""CPU tests of the product library (libpt.so) -- no GPU needed.

* the C ABI loads and exports every function include/pt.h declares;
* host logic: the quirk-faithful loader and the bit-faithful reference BVH
  (fingerprints vs the reference's own md5s), the gamma/8-bit threshold table;
* the device traversal/integrator code of pt_trace.h executed on the host
  (pt_selftest_* hooks) against the reference's traversal KAT and fp32 radiance;
* without a GPU, rendering fails loudly (PT_E_NO_GPU) -- there is no CPU fallback.
"""
import ctypes
import os
import re

import numpy as np
import pytest

import _util as U

M = U.manifest()
pt = U.ptrace()


def declared_functions():
    with open(os.path.join(U.REPO, "include", "pt.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_abi_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 25
    lib = ctypes.CDLL(pt.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(pt.EXPORTED)
    assert pt.abi_version() == pt.ABI_VERSION == 6


@pytest.mark.parametrize("name", sorted(M["bvh"]))
def test_product_bvh_fingerprints(name):
    b = M["bvh"][name]
    with pt.Scene.load(U.scene_path(b["scene"])) as s:
        s.prepare()
        nodes, prims = s.dump_bvh()
        assert s.info["n_nodes"] == b["n_nodes"]
        assert U.md5(nodes) == b["nodes_md5"]
        assert U.md5(prims) == b["prims_md5"]


def test_scene_info_standin():
    with pt.Scene.load(U.scene_path("c3")) as s:
        s.prepare()
        i = s.info
        assert (i["width"], i["height"], i["samples"], i["ray_depth"]) == (1920, 1080, 256, 6)
        assert i["n_bvh_prims"] == 89929 and i["n_planes"] == 5 and i["n_emitters"] == 1
        assert i["n_nodes"] == 179797
        assert 0 < i["max_stack"] < i["tree_depth"] <= 64


QUIRK_SCENES = {
    # BG_COLOR right after a primitive block is re-dispatched with the stale
    # NEW_PRIMITIVE line stream: its arguments are never read (background stays 0)
    "stale_bg": "DIMENSIONS 16 16\nRAY_DEPTH 3\nSAMPLES 2\nCAMERA_POSITION 0 0 3\nCAMERA_RIGHT 1 0 0\n"
                "CAMERA_UP 0 1 0\nCAMERA_FORWARD 0 0 -1\nCAMERA_FOV_X 1.2\nNEW_PRIMITIVE\nBOX 0.5 0.5 0.5\n"
                "COLOR 1 0 0\nBG_COLOR 1 1 1\n",
    # a type line resets the primitive (POSITION before it is lost); unknown commands skipped
    "reset_and_unknown": "DIMENSIONS 16 12\nRAY_DEPTH 4\nSAMPLES 2\nBG_COLOR 0.2 0.3 0.4\nFOO 1 2\n"
                         "CAMERA_POSITION 0 0 4\nCAMERA_RIGHT 1 0 0\nCAMERA_UP 0 1 0\nCAMERA_FORWARD 0 0 -1\n"
                         "CAMERA_FOV_X 1.0\n\nNEW_PRIMITIVE\nPOSITION 3 3 3\nELLIPSOID 1 0.5 0.7\nCOLOR 0.9 0.9 0.2\n"
                         "ROTATION 0.1 0.2 0.3 0.9\n\nNEW_PRIMITIVE\nPLANE 0 1 0\nPOSITION 0 -1 0\nCOLOR 1 1 1\n"
                         "NEW_PRIMITIVE\nBOX 0.3 0.3 0.3\nPOSITION 0 1.5 0\nEMISSION 4 4 4\n",
    # numeric extraction failure stores 0 and poisons the rest of the line
    "bad_number": "DIMENSIONS 8 8\nRAY_DEPTH 2\nSAMPLES 1\nBG_COLOR 1 x 1\nCAMERA_POSITION 0 0 3\n"
                  "CAMERA_RIGHT 1 0 0\nCAMERA_UP 0 1 0\nCAMERA_FORWARD 0 0 -1\nCAMERA_FOV_X 1.2\n"
                  "NEW_PRIMITIVE\nTRIANGLE 0 0 0 1 0 0 0 1 0\nCOLOR 0.5 0.5 0.5\n",
}


@pytest.mark.parametrize("name", sorted(QUIRK_SCENES))
def test_loader_quirks_match_oracle(tmp_path, name):
    p = tmp_path / (name + ".txt")
    p.write_text(QUIRK_SCENES[name])
    o = U.OracleScene(str(p))
    _, orad, _ = o.render()
    with pt.Scene.load(str(p)) as s:
        s.prepare()
        assert s.info["width"] == o.W and s.info["height"] == o.H
        nodes, prims = s.dump_bvh()
        onodes, oprims = o.dump_bvh()
        assert nodes == onodes and prims == oprims
        rad = s.selftest_render_host(0, 0, o.W, o.H)
    assert np.array_equal(rad.view(np.uint32), orad.view(np.uint32))


def _big_quirky_scene(n_blocks=24000, seed=3):
    """> 1 MB of scene text (the loader parses it in stretches on several threads) with
    the grammar's quirks spread through it: top-level commands right after a block (the
    stale-stream re-dispatch), partial top-level lines, unknown commands, blocks without
    a blank line between them, leading whitespace, a POSITION before the type line, and
    numbers in every form the fast decimal path takes or leaves to strtof."""
    rng = np.random.default_rng(seed)
    forms = ["%.6g", "%.9g", "%.3e", "%.1f", "%.12f", "%g"]
    L = ["DIMENSIONS 16 12", "RAY_DEPTH 3", "SAMPLES 2", "CAMERA_POSITION 0 0 6", "CAMERA_RIGHT 1 0 0",
         "CAMERA_UP 0 1 0", "CAMERA_FORWARD 0 0 -1", "CAMERA_FOV_X 1.1", ""]
    unknown = 0
    for i in range(n_blocks):
        v = rng.normal(0, 1.5, 9)
        f = forms[i % len(forms)]
        lead = "   " if i % 97 == 5 else ""
        L.append(lead + "NEW_PRIMITIVE")
        if i % 211 == 7:
            L.append("POSITION 3 3 3")             # lost: the type line resets the primitive
        L.append("TRIANGLE " + " ".join(f % x for x in v))
        L.append("COLOR %s %s 1" % (f % abs(v[0] / 3), "-0" if i % 13 == 0 else "1e-3"))
        if i % 5 == 0:
            L.append("EMISSION 0 0 0")
        if i % 1009 == 11:
            L.append("BG_COLOR 0.25 0.5 0.75")     # ends the block: re-dispatched on the stale stream
        elif i % 1013 == 17:
            L += ["", "SAMPLES 3", "DIMENSIONS 20"]  # a partial top-level line: H keeps its value
        elif i % 1021 == 19:
            L += ["FOO 1 2"]                       # unknown (warning), after the block
            unknown += 1
        elif i % 3 == 0:
            continue                               # no blank line before the next NEW_PRIMITIVE
        L.append("")
    return "\n".join(L) + "\n", unknown


def test_parallel_parse_matches_oracle(tmp_path):
    """The loader's multi-threaded stretch parse gives the reference parse: same header
    values, same primitives in the same order (BVH fingerprints against the oracle's own
    loader), the same warnings; and the same image at 2 spp."""
    text, unknown = _big_quirky_scene()
    assert len(text) > (1 << 20)
    p = tmp_path / "big.txt"
    p.write_text(text)
    o = U.OracleScene(str(p))
    with pt.Scene.load(str(p)) as s:
        s.prepare()
        inf = s.info
        assert (inf["width"], inf["height"], inf["samples"], inf["ray_depth"]) == (o.W, o.H, o.samples, o.depth)
        assert inf["n_prims"] == o.n_prims and inf["n_warnings"] == unknown
        nodes, prims = s.dump_bvh()
        onodes, oprims = o.dump_bvh()
        assert prims == oprims and nodes == onodes
        rad = s.selftest_render_host(0, 0, 8, 6, spp=2)
    _, orad, _ = o.render(0, 0, 8, 6, spp=2)
    assert np.array_equal(rad.view(np.uint32), orad.view(np.uint32))


def test_scene_errors():
    with pytest.raises(pt.PTError) as e:
        pt.Scene.load("/nonexistent/scene.txt")
    assert e.value.code == pt.PT_E_IO
    # only planes: the reference aborts in BVH_t; we report PT_E_SCENE
    with pt.Scene.loads("DIMENSIONS 4 4\nSAMPLES 1\nRAY_DEPTH 1\nNEW_PRIMITIVE\nPLANE 0 1 0\n") as s:
        with pytest.raises(pt.PTError) as e:
            s.prepare()
        assert e.value.code == pt.PT_E_SCENE
    # a primitive block without a type line
    with pt.Scene.loads("DIMENSIONS 4 4\nNEW_PRIMITIVE\nCOLOR 1 1 1\n") as s:
        with pytest.raises(pt.PTError) as e:
            s.prepare()
        assert e.value.code == pt.PT_E_SCENE



def test_degenerate_sah_split_is_an_error_not_a_crash():
    # 200 boxes at x = 1.3^i: every SAH cut cost overflows (the reference's
    # bvh.cpp recursion then runs on an empty range and crashes); the library
    # reports PT_E_SCENE instead of taking the calling process down
    lines = ["DIMENSIONS 4 4", "SAMPLES 1", "RAY_DEPTH 1"]
    for i in range(200):
        lines += ["NEW_PRIMITIVE", "BOX 1 1 1", "POSITION %.6g 0 0" % (1.3 ** i)]
    with pt.Scene.loads("\n".join(lines) + "\n") as s:
        with pytest.raises(pt.PTError) as e:
            s.prepare()
        assert e.value.code == pt.PT_E_SCENE
        assert "degenerate SAH split" in str(e.value)


TRAVERSALS = {"replay": 0, "exact": 1, "replay_div": 2}


@pytest.mark.parametrize("trav", sorted(TRAVERSALS))
@pytest.mark.parametrize("name", sorted(M["trav"]))
def test_traversal_matches_reference_kat(name, trav):
    t = M["trav"][name]
    rays, ((ids, f, inter), _) = U.read_trav(name)
    with pt.Scene.load(U.scene_path(t["scene"])) as s:
        s.prepare()
        gids, ghits, ctr = s.selftest_ray_intersection(rays, traversal=TRAVERSALS[trav])
    assert np.array_equal(gids, ids)
    hit = ids != -1
    assert np.array_equal(ghits[hit, :4].view(np.uint32), f[hit].view(np.uint32))
    assert np.array_equal(ghits[hit, 4].astype(np.uint32), inter[hit])


HOST_RENDER = ["p51_64x48x16", "p52_64x48x16", "dragon_metal_64x64x8", "dragon_glass_64x64x8",
               "hw3s2_48x48x8", "hw3s3_48x48x8", "hw3s4_48x48x8", "hw3s5_48x48x8", "rabbid_48x48x4",
               "c2_win_240_200_24x24"]


@pytest.mark.parametrize("trav", sorted(TRAVERSALS))
@pytest.mark.parametrize("name", HOST_RENDER)
def test_device_integrator_on_host_bit_exact(name, trav):
    m, img, rad = U.golden_image(name)
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        s.prepare()
        if m["window"]:
            x0, y0, w, h = m["window"]
        else:
            x0, y0, h, w = 0, 0, img.shape[0], img.shape[1]
        got = s.selftest_render_host(x0, y0, w, h, traversal=TRAVERSALS[trav])
    assert got.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(U.oracle_tonemap(got).reshape(img.shape), img)


@pytest.mark.parametrize("name", sorted(M["trav"]))
def test_coop_query_matches_reference_kat(name, monkeypatch):
    """The cooperative engine's query algorithm (pt_coop.h qc_run: every candidate
    leaf's bound-free result first, then only the hitting leaves' root paths with
    the carried bounds), run on the host: the reference's closest hits.  The path
    engine's query probes the same candidates but decides a hitting leaf from its
    record or the part of its root path below the LCA with the last hit, so it
    reads no more node records than the whole root paths."""
    t = M["trav"][name]
    rays, ((ids, f, inter), _) = U.read_trav(name)
    with pt.Scene.load(U.scene_path(t["scene"])) as s:
        s.prepare()
        _, _, rctr = s.selftest_ray_intersection(rays, traversal=0)
        monkeypatch.setenv("PT_TUNE", "qengine=coop")
        gids, ghits, ctr = s.selftest_ray_intersection(rays, traversal=0)
    assert np.array_equal(gids, ids)
    hit = ids != -1
    assert np.array_equal(ghits[hit, :4].view(np.uint32), f[hit].view(np.uint32))
    assert np.array_equal(ghits[hit, 4].astype(np.uint32), inter[hit])
    assert rctr["nodes"] <= ctr["nodes"]


@pytest.mark.parametrize("name", HOST_RENDER[:6])
def test_coop_integrator_on_host_bit_exact(name, monkeypatch):
    monkeypatch.setenv("PT_TUNE", "qengine=coop")
    m, img, rad = U.golden_image(name)
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        s.prepare()
        if m["window"]:
            x0, y0, w, h = m["window"]
        else:
            x0, y0, h, w = 0, 0, img.shape[0], img.shape[1]
        got = s.selftest_render_host(x0, y0, w, h, traversal=0)
    assert got.view(np.uint32).tolist() == rad.view(np.uint32).tolist()


def test_query_log_on_host(tmp_path, monkeypatch):
    """PT_TUNE qstats=FILE: the host render logs one 16-B record per query
    (aux visits, node records, primitive tests | exact-DFS bit), and the image
    stays the same."""
    name = HOST_RENDER[0]
    m, img, rad = U.golden_image(name)
    log = tmp_path / "q.bin"
    monkeypatch.setenv("PT_TUNE", "qstats=%s" % log)
    with pt.Scene.load(U.golden_scene_path(name)) as s:
        s.prepare()
        if m["window"]:
            x0, y0, w, h = m["window"]
        else:
            x0, y0, h, w = 0, 0, img.shape[0], img.shape[1]
        got = s.selftest_render_host(x0, y0, w, h, traversal=0)
    assert got.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    q = np.fromfile(log, dtype=np.uint32).reshape(-1, 4)
    assert len(q) >= w * h   # at least one query per sample
    assert q[:, 0].sum() > 0


def test_aux_tree_quality_on_standin(tmp_path, monkeypatch):
    """The wide aux tree's quality, the wavefront query's dominant cost: aux-node visits per
    query of the host build of the query (the code the GPU runs) on six 32x32 windows of
    the config-3 stand-in at 1 spp (tools/aux_quality.py's measure).  4.24 per query when
    this test was written, with the region-weighted collapse of aux_bvh.cpp (which took
    tools/aux_quality.py's default sample from 4.754 to 4.710); a builder change that costs
    more than 3 % fails here, on the CPU."""
    log = tmp_path / "q.bin"
    monkeypatch.setenv("PT_TUNE", "qstats=%s" % log)
    rows = []
    with pt.Scene.load(U.scene_path("c3")) as s:
        s.prepare()
        W, H = s.info["width"], s.info["height"]
        for j in range(2):
            for i in range(3):
                x0, y0 = (W - 32) * i // 2, (H - 32) * j
                got = s.selftest_render_host(x0, y0, 32, 32, spp=1, traversal=0)
                assert np.isfinite(got).all()
                rows.append(np.fromfile(log, dtype=np.uint32).reshape(-1, 4))
    q = np.concatenate(rows)
    assert len(q) > 20000 and int((q[:, 2] >> 31).sum()) == 0
    assert q[:, 0].mean() <= 4.24 * 1.03


def _gamma_table():
    with pt.Scene.load(U.scene_path("practice5_1.txt")) as s:
        s.prepare()
        return s.gamma_table()


def test_gamma_table_matches_host_quantiser():
    thr = _gamma_table()
    assert np.all(np.diff(thr[:255]) > 0) and np.isinf(thr[255])
    v = thr[:255]
    cand = np.concatenate([v, np.nextafter(v, np.float32(0)), np.nextafter(v, np.float32(2)),
                           np.linspace(0, 1, 200001, dtype=np.float32)])
    cand = np.clip(cand, 0, 1).astype(np.float32)
    q = np.searchsorted(v, cand, side="right")   # = number of thresholds <= x (device rule)
    ref = np.zeros(len(cand), np.uint8)
    U.oracle().oracle_gamma_u8(len(cand), U._p(cand), U._p(ref))
    assert np.array_equal(q, ref.astype(np.int64))


@pytest.mark.slow
def test_gamma_table_exhaustive():
    # every float in [0, 1] quantises through the table exactly as glibc powf + round
    thr = _gamma_table()
    assert U.oracle().oracle_check_gamma_table(U._p(thr)) == 0


def test_render_without_gpu_fails_loudly():
    if U.gpu_available():
        pytest.skip("GPU present")
    with pt.Scene.load(U.scene_path("practice5_1.txt")) as s:
        s.override(16, 16, 1, 0)
        with pytest.raises(pt.PTError) as e:
            s.render()
        assert e.value.code in (pt.PT_E_NO_GPU, pt.PT_E_HIP)


def test_device_init_without_gpu_fails_loudly():
    if U.gpu_available():
        pytest.skip("GPU present")
    assert pt._lib.pt_device_init(0) in (pt.PT_E_NO_GPU, pt.PT_E_HIP)
    assert pt._lib.pt_gather_init(0, 0) == pt.PT_E_INVALID


def _stack_scene(n=60, seed=7):
    """n small triangles stacked along z above the plane z = 0, with small tilts:
    IntersectTriangle hits the plane through the origin (src/primitives.cpp:156-157),
    so their hit regions all overlap near (0, 0, 0) while their own boxes are
    spread along z -- a ray crossing the stack has dozens of hitting leaves (the
    query's overflow passes and its exact-DFS hand-over)."""
    rng = np.random.default_rng(seed)
    lines = ["DIMENSIONS 8 8", "SAMPLES 1", "RAY_DEPTH 1",
             "CAMERA_POSITION 0 0 5", "CAMERA_RIGHT 1 0 0", "CAMERA_UP 0 1 0", "CAMERA_FORWARD 0 0 -1",
             "CAMERA_FOV_X 1.0"]
    for k in range(n):
        z = 0.5 + 0.05 * k
        v = np.array([[-0.3, -0.3, z], [0.3, -0.3, z], [0.0, 0.3, z]]) + rng.normal(0, 0.02, (3, 3))
        lines += ["NEW_PRIMITIVE", "TRIANGLE " + " ".join("%.5f" % x for x in v.ravel()), "COLOR 0.5 0.5 0.5"]
    return "\n".join(lines) + "\n"


def _stack_rays(n=1500, seed=11):
    rng = np.random.default_rng(seed)
    o = np.concatenate([rng.uniform(-0.4, 0.4, (n, 2)), rng.choice([-2.0, 6.0], (n, 1))], axis=1)
    tgt = np.concatenate([rng.uniform(-0.3, 0.3, (n, 2)), rng.uniform(-0.5, 3.5, (n, 1))], axis=1)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], axis=1).astype(np.float32)


@pytest.mark.parametrize("engine", ["replay", "coop"])
def test_many_hitting_leaves_match_oracle(tmp_path, engine, monkeypatch):
    """Rays with up to ~60 hitting leaves: the path engine's query keeps 6 per
    pass and hands rays with 6 entered hits and another hit to the exact DFS;
    the cooperative query holds them all.  Both give the oracle's closest hit."""
    p = tmp_path / "stack.txt"
    p.write_text(_stack_scene())
    rays = _stack_rays()
    o = U.OracleScene(str(p))
    oids, ohits = o.ray_intersection(rays)
    if engine == "coop":
        monkeypatch.setenv("PT_TUNE", "qengine=coop")
    with pt.Scene.load(str(p)) as s:
        s.prepare()
        ids, hits, ctr = s.selftest_ray_intersection(rays, traversal=0)
    assert (oids >= 0).sum() > len(rays) // 2
    assert np.array_equal(ids, oids)
    hit = oids != -1
    assert np.array_equal(hits[hit].view(np.uint32), ohits[hit].view(np.uint32))
    if engine == "replay":
        assert ctr["fallbacks"] > 0          # some rays exceed the list: the exact DFS took them


def _moved_scene(src, dst, k, d):
    """`src` with every length (positions, vertices, box sizes, camera position)
    multiplied by k, then every position moved by d along x: far from the origin the
    binary16 step (2^(e-10)) dwarfs small leaf boxes, and past 65504 they are infinite."""
    out = []
    for line in open(src):
        w = line.split()
        if w and w[0] in ("POSITION", "TRIANGLE", "BOX", "ELLIPSOID", "CAMERA_POSITION"):
            v = [float(x) * k for x in w[1:]]
            if w[0] in ("POSITION", "CAMERA_POSITION"):
                v[0] += d
            line = " ".join([w[0]] + [repr(x) for x in v]) + "\n"
        out.append(line)
    with open(dst, "w") as f:
        f.writelines(out)


@pytest.mark.parametrize("k,d", [(1.0, 3.0e4), (1.0e5, 0.0)])
def test_coarse_binary16_aux_boxes_warn_and_stay_exact(tmp_path, capfd, k, d):
    """far-out coordinates make the binary16 aux boxes coarse (a step of 16
    at 3e4, infinite past 65504).  pt_scene_prepare says so on stderr, and the replay
    still returns the exact traversal's result bit for bit (only the culling degrades)."""
    path = str(tmp_path / "dragon_moved.txt")
    _moved_scene(U.scene_path("practice5_dragon_10k.txt"), path, k, d)
    with pt.Scene.load(U.scene_path("practice5_dragon_10k.txt")) as s:
        s.prepare()
    assert "binary16" not in capfd.readouterr().err
    with pt.Scene.load(path) as s:
        s.prepare()
        assert "binary16" in capfd.readouterr().err
        got = {t: s.selftest_render_host(232, 200, 16, 16, spp=2, traversal=v) for t, v in TRAVERSALS.items()}
    assert got["replay"].view(np.uint32).tolist() == got["exact"].view(np.uint32).tolist()
    assert got["replay_div"].view(np.uint32).tolist() == got["exact"].view(np.uint32).tolist()


def test_handoff_sites_mirror_the_abi():
    """pt_stats.handoff's sites (include/pt.h PT_HO_*) in ptrace's order (HANDOFF_SITES, the
    PT_TUNE drop=<name> names), and pt_stats.handoff wide enough for them."""
    import re
    hdr = open(os.path.join(U.REPO, "include", "pt.h")).read()
    ids = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"PT_HO_([A-Z_]+) = (\d+)", hdr)}
    n = ids.pop("n")
    assert sorted(ids.values()) == list(range(n))
    assert tuple(sorted(ids, key=ids.get)) == pt.HANDOFF_SITES
    assert re.search(r"uint64_t handoff\[(\d+)\]", hdr).group(1) == str(dict(pt.Stats._fields_)["handoff"]._length_)
