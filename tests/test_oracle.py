"""Pin the CPU oracle (oracle/pt_oracle.cpp) against the reference's own outputs.

Every fixture under tests/golden/ was produced by the UNMODIFIED reference
(tests/golden/make_golden.py); the oracle must reproduce all of them bit for bit.
"""
import numpy as np
import pytest

import _util as U

M = U.manifest()


@pytest.mark.parametrize("seed", sorted(M["rng"], key=int))
def test_rng_known_answers(seed):
    n = M["rng"][seed]["n"]
    ref = np.fromfile(U.os.path.join(U.GOLDEN, "rng_%s.f32" % seed), np.float32)
    got = U.oracle_rng(int(seed), n)
    assert got.view(np.uint32).tolist() == ref.view(np.uint32).tolist()


@pytest.mark.parametrize("name", sorted(M["bvh"]))
def test_bvh_fingerprints(name):
    b = M["bvh"][name]
    o = U.OracleScene(U.scene_path(b["scene"]))
    nodes, prims = o.dump_bvh()
    assert o.n_nodes == b["n_nodes"]
    assert U.md5(nodes) == b["nodes_md5"]
    assert U.md5(prims) == b["prims_md5"]


@pytest.mark.parametrize("name", sorted(M["images"]))
def test_images_bit_exact(name):
    m, img, rad = U.golden_image(name)
    o = U.OracleScene(U.golden_scene_path(name))
    if m["window"]:
        x0, y0, w, h = m["window"]
        rgb, r, _ = o.render(x0, y0, w, h)
    else:
        rgb, r, _ = o.render()
    assert r.view(np.uint32).tolist() == rad.view(np.uint32).tolist()
    assert np.array_equal(rgb, img)


@pytest.mark.parametrize("name", sorted(M["trav"]))
def test_traversal_kat(name):
    t = M["trav"][name]
    rays, ((ids, f, inter), _) = U.read_trav(name)
    o = U.OracleScene(U.scene_path(t["scene"]))
    gids, ghits = o.ray_intersection(rays)
    assert np.array_equal(gids, ids)
    hit = ids != -1
    assert np.array_equal(ghits[hit, :4].view(np.uint32), f[hit].view(np.uint32))
    assert np.array_equal(ghits[hit, 4].astype(np.uint32), inter[hit])


def test_config1_full_md5_and_rays():
    full = M["full"]["c1"]
    o = U.OracleScene(U.scene_path("c1"))
    rgb, _, ctr = o.render()
    ppm = b"P6\n%d %d\n255\n" % (o.W, o.H) + rgb.tobytes()
    assert U.md5(ppm) == full["md5"]
    assert ctr["rays"] == full["rays"]
    assert np.allclose(rgb.reshape(-1, 3).mean(0), full["mean8"], atol=5e-5)


def test_scene_generator_md5():
    # every pinned configuration scene regenerates byte-exactly
    for name in ("c1", "c2", "c3"):
        p = U.scene_path(name)
        with open(p, "rb") as f:
            assert U.md5(f.read()) == U.make_scene.CONFIGS[name][6]
