#!/usr/bin/env python3
"""Regenerate tests/golden/* from the UNMODIFIED reference renderer.

Runs only where /root/reference exists (the build container): it builds
oracle/_ref/{raytracing_hw5,ref_harness} (oracle/build_ref.sh) and records
their outputs as data fixtures.  The fixtures are inputs + expected outputs
only (images, fp32 radiance, fingerprints, RNG and traversal known answers);
no reference source is copied.

Outputs (all little-endian):
  manifest.json                  index of every fixture below + md5s
  img_<name>.ppm                 reference P6 output (window crop when windowed)
  rad_<name>.f32                 reference pre-tonemap mean radiance, w*h*3 f32
  rng_<seed>.f32                 3*N floats: N uniform, N normal, N mixed draws
  trav_<scene>.bin               per ray: o,d (6 f32) + 2 x (id i32, t, n.xyz f32,
                                 interior u32) for RayIntersection / BVH_t::Intersect
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "scenes"))
import make_scene  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref")
SCENES = os.path.join(REPO, "scenes")

# name -> (scene source, generator args or None, window or None)
#   generator args: (W, H, S, subdivide, variant)
IMAGES = {
    "p51_64x48x16": ("practice5_1.txt", (64, 48, 16, False, "diffuse"), None),
    "p52_64x48x16": ("practice5_2.txt", (64, 48, 16, False, "diffuse"), None),
    "dragon_64x64x16": ("practice5_dragon_10k.txt", (64, 64, 16, False, "diffuse"), None),
    "dragon_metal_64x64x8": ("practice5_dragon_10k.txt", (64, 64, 8, False, "metal"), None),
    "dragon_glass_64x64x8": ("practice5_dragon_10k.txt", (64, 64, 8, False, "glass"), None),
    "standin_48x32x4": ("practice5_dragon_10k.txt", (48, 32, 4, True, "diffuse"), None),
    "hw3s1_48x48x8": ("hw3_sample1.txt", (48, 48, 8, False, "diffuse"), None),
    "hw3s2_48x48x8": ("hw3_sample2.txt", (48, 48, 8, False, "diffuse"), None),
    "hw3s3_48x48x8": ("hw3_sample3.txt", (48, 48, 8, False, "diffuse"), None),
    "hw3s4_48x48x8": ("hw3_sample4.txt", (48, 48, 8, False, "diffuse"), None),
    "hw3s5_48x48x8": ("hw3_sample5.txt", (48, 48, 8, False, "diffuse"), None),
    "hw3s6_48x48x8": ("hw3_sample6.txt", (48, 48, 8, False, "diffuse"), None),
    "rabbid_48x48x4": ("rabbid_sample.txt", (48, 48, 4, False, "diffuse"), None),
    # windows of the benchmark configurations (global-index seeds kept)
    "c2_win_240_200_24x24": ("c2", None, (240, 200, 24, 24)),
    "c3s4_win_944_520_16x16": ("c3", (1920, 1080, 4, True, "diffuse"), (944, 520, 16, 16)),
    "c4glass_s4_win_900_560_16x16": ("c4_glass", (1920, 1080, 4, True, "glass"), (900, 560, 16, 16)),
    "c4metal_s4_win_900_560_16x16": ("c4_metal", (1920, 1080, 4, True, "metal"), (900, 560, 16, 16)),
    # more windows of configs 3/4: the frame's corners (edge tiles), a window off the
    # 16x16 tile grid, and further regions of the metal and glass variants
    "c3s4_win_0_0_16x16": ("c3", (1920, 1080, 4, True, "diffuse"), (0, 0, 16, 16)),
    "c3s4_win_1896_1064_24x16": ("c3", (1920, 1080, 4, True, "diffuse"), (1896, 1064, 24, 16)),
    "c3s4_win_1001_537_24x12": ("c3", (1920, 1080, 4, True, "diffuse"), (1001, 537, 24, 12)),
    "c4metal_s4_win_1010_470_16x16": ("c4_metal", (1920, 1080, 4, True, "metal"), (1010, 470, 16, 16)),
    "c4glass_s4_win_830_610_16x16": ("c4_glass", (1920, 1080, 4, True, "glass"), (830, 610, 16, 16)),
    # config 5 (3840x2160, pixel-tiled over 8 GPUs): windows whose 16x16 tiles belong to
    # ranks 3, 5+6, 1 and 5 of 8 (tile (tx, ty) -> rank (tx + ty) % 8; until round 3 the
    # deal was t % 8 -> ranks 0, 2+3, 6, 7); seeds y*3840+x
    "c5s4_win_1920_1072_16x16": ("c5", (3840, 2160, 4, True, "diffuse"), (1920, 1072, 16, 16)),
    "c5s4_win_1952_1072_32x16": ("c5", (3840, 2160, 4, True, "diffuse"), (1952, 1072, 32, 16)),
    "c5s4_win_1760_1200_16x16": ("c5", (3840, 2160, 4, True, "diffuse"), (1760, 1200, 16, 16)),
    "c5s4_win_3824_2144_16x16": ("c5", (3840, 2160, 4, True, "diffuse"), (3824, 2144, 16, 16)),
}

# Deep stream positions: windows of the benchmark configurations at their OWN spp
# (c3 256, c4 1024, c5 4096), RAY_DEPTH 10 paths, and a scene beyond the
# cooperative engine's LDS limits (10 planes, 10 box/ellipsoid emitters, depth 8).
# Each gets the reference's image + radiance (ref_harness) and a ray count from the
# CPU restatement (oracle/pt_oracle.cpp), whose image must equal the reference's
# byte-for-byte here; the ray count is then the restatement's count of
# Scene::RayIntersection calls for those same pixels.
DEEP = {
    "c3_win_944_520_16x16": ("c3", None, (944, 520, 16, 16)),
    "c4metal_win_900_560_16x16": ("c4_metal", None, (900, 560, 16, 16)),
    "c4glass_win_900_560_16x16": ("c4_glass", None, (900, 560, 16, 16)),
    # config 5 tiles of ranks 3 and 5 of 8 (tile (tx, ty) -> rank (tx + ty) % 8)
    "c5_win_1920_1072_8x8": ("c5", None, (1920, 1072, 8, 8)),
    "c5_win_3832_2152_8x8": ("c5", None, (3832, 2152, 8, 8)),
    "dragon_d10_metal_48x48x16": ("practice5_dragon_10k.txt", (48, 48, 16, False, "metal", 10), None),
    "dragon_d10_glass_48x48x16": ("practice5_dragon_10k.txt", (48, 48, 16, False, "glass", 10), None),
    "c4glass_d10_s16_win_900_560_16x16": ("c3", (1920, 1080, 16, True, "glass", 10), (900, 560, 16, 16)),
    "many_lights_48x48x8": ("many_lights.txt", (48, 48, 8, False, "diffuse"), None),
}

RNG_SEEDS = [0, 1, 2, 12345, 262143, 2073599, 2147483646, 4294967295]
RNG_N = 2048

TRAV = {"dragon10k": ("practice5_dragon_10k.txt", None), "standin": ("c3", None)}
TRAV_RAYS = 4096

# full-resolution reference md5s measured in the survey container;
# config 1 is re-measured here, config 2 (320 s) is carried over.
FULL_MD5 = {"c1": "99f1bc9386a22892970f058bfa8114c7", "c2": "a16f6cf46a6443244ecbd0c9d856c295"}
FULL_MEAN8 = {"c1": [196.4152, 193.6256, 214.1081], "c2": [116.1553, 116.5566, 87.3717]}
FULL_RAYS = {"c1": 1650687, "c2": 67011212}


def md5f(path):
    with open(path, "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


def scene_file(tmp, src, gen):
    """Return a path to the scene text for fixture generation."""
    if src in make_scene.CONFIGS and gen is None:
        out = os.path.join(tmp, src + ".txt")
        if not os.path.exists(out):
            make_scene.make(src, out)
        return out
    if src in make_scene.CONFIGS:
        base = make_scene.CONFIGS[src][0]
    else:
        base = src
    W, H, S, sub, var = gen[:5]
    depth = gen[5] if len(gen) > 5 else None   # optional RAY_DEPTH override
    out = os.path.join(tmp, "%s_%d_%d_%d_%d_%s%s.txt" % (os.path.splitext(base)[0], W, H, S, sub, var,
                                                      "_d%d" % depth if depth is not None else ""))
    if not os.path.exists(out):
        make_scene.make_custom(os.path.join(SCENES, base), W, H, S, sub, var, out, depth)
    return out


def render_image(harness, tmp, name, table=None):
    src, gen, win = (table or IMAGES)[name]
    sc = scene_file(tmp, src, gen)
    ppm = os.path.join(HERE, "img_%s.ppm" % name)
    rad = os.path.join(HERE, "rad_%s.f32" % name)
    cmd = [harness, "render", sc, ppm, rad]
    if win:
        cmd += [str(v) for v in win]
    subprocess.check_call(cmd)
    entry = {"scene": src, "gen": list(gen) if gen else None, "window": list(win) if win else None,
             "ppm_md5": md5f(ppm), "rad_md5": md5f(rad)}
    if not win:
        # the windowless harness render must equal the real CLI byte-for-byte
        cli_ppm = os.path.join(tmp, name + "_cli.ppm")
        subprocess.check_call([os.path.join(REF, "raytracing_hw5"), sc, cli_ppm], stdout=subprocess.DEVNULL)
        assert md5f(cli_ppm) == entry["ppm_md5"], name
    print("image", name, entry["ppm_md5"])
    return entry


def render_deep(harness, tmp, name):
    """A DEEP fixture: the reference's window + the restatement's ray count."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _util as U
    entry = render_image(harness, tmp, name, DEEP)
    src, gen, win = DEEP[name]
    sc = scene_file(tmp, src, gen)
    o = U.OracleScene(sc)
    x0, y0, w, h = win if win else (0, 0, None, None)
    rgb, rad, ctr = o.render(x0, y0, w, h)
    ref_rad = np.fromfile(os.path.join(HERE, "rad_%s.f32" % name), np.float32).reshape(rad.shape)
    ref_img = U.read_ppm(os.path.join(HERE, "img_%s.ppm" % name))
    assert np.array_equal(rad.view(np.uint32), ref_rad.view(np.uint32)), name + ": restatement radiance differs"
    assert np.array_equal(rgb, ref_img), name + ": restatement image differs"
    entry["rays"] = int(ctr["rays"])
    print("deep", name, entry["rays"], "rays")
    return entry


def main():
    if not os.path.isdir("/root/reference/hw5"):
        print("reference not present; cannot regenerate fixtures", file=sys.stderr)
        return 1
    subprocess.check_call(["sh", os.path.join(REPO, "oracle", "build_ref.sh")])
    harness = os.path.join(REF, "ref_harness")
    if len(sys.argv) > 1 and sys.argv[1] == "--deep":
        # (re)generate the deep fixtures (all, or the named ones) in the existing manifest
        with open(os.path.join(HERE, "manifest.json")) as f:
            manifest = json.load(f)
        deep = manifest.setdefault("deep", {})
        with tempfile.TemporaryDirectory() as tmp:
            for name in (sys.argv[2:] or list(DEEP)):
                deep[name] = render_deep(harness, tmp, name)
                with open(os.path.join(HERE, "manifest.json"), "w") as f:
                    json.dump(manifest, f, indent=1, sort_keys=True)
        return 0
    if len(sys.argv) > 2 and sys.argv[1] == "--images":
        # add / refresh only the named image fixtures in the existing manifest
        with open(os.path.join(HERE, "manifest.json")) as f:
            manifest = json.load(f)
        with tempfile.TemporaryDirectory() as tmp:
            for name in sys.argv[2:]:
                manifest["images"][name] = render_image(harness, tmp, name)
        with open(os.path.join(HERE, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return 0
    manifest = {"images": {}, "rng": {}, "trav": {}, "bvh": {}, "full": {},
                "generator": "tests/golden/make_golden.py", "reference": "FeggieBoss/raytracing-course hw5"}
    with tempfile.TemporaryDirectory() as tmp:
        for name in IMAGES:
            manifest["images"][name] = render_image(harness, tmp, name)
        for seed in RNG_SEEDS:
            p = os.path.join(HERE, "rng_%d.f32" % seed)
            subprocess.check_call([harness, "rng", str(seed), str(RNG_N), p])
            manifest["rng"][str(seed)] = {"n": RNG_N, "md5": md5f(p)}
        for name, (src, gen) in TRAV.items():
            sc = scene_file(tmp, src, gen) if src in make_scene.CONFIGS else os.path.join(SCENES, src)
            p = os.path.join(HERE, "trav_%s.bin" % name)
            subprocess.check_call([harness, "trav", sc, str(TRAV_RAYS), "20241015", p])
            manifest["trav"][name] = {"scene": src, "rays": TRAV_RAYS, "md5": md5f(p)}
        for name, src in [("practice5_1", "practice5_1.txt"), ("practice5_2", "practice5_2.txt"),
                          ("dragon10k", "practice5_dragon_10k.txt"), ("standin", "c3")]:
            sc = scene_file(tmp, src, None) if src in make_scene.CONFIGS else os.path.join(SCENES, src)
            n = os.path.join(tmp, "n.bin")
            pr = os.path.join(tmp, "p.bin")
            subprocess.check_call([harness, "bvh", sc, n, pr])
            manifest["bvh"][name] = {"scene": src, "nodes_md5": md5f(n), "prims_md5": md5f(pr),
                                     "n_nodes": os.path.getsize(n) // 40, "n_prims": os.path.getsize(pr) // 52}
            print("bvh", name, manifest["bvh"][name])
        # config 1 full image re-measured with the real CLI
        c1 = scene_file(tmp, "c1", None)
        c1_ppm = os.path.join(tmp, "c1.ppm")
        subprocess.check_call([os.path.join(REF, "raytracing_hw5"), c1, c1_ppm], stdout=subprocess.DEVNULL)
        assert md5f(c1_ppm) == FULL_MD5["c1"]
        for k in FULL_MD5:
            manifest["full"][k] = {"md5": FULL_MD5[k], "mean8": FULL_MEAN8[k], "rays": FULL_RAYS[k],
                                   "scene_md5": make_scene.CONFIGS[k][6]}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
