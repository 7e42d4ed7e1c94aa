#!/usr/bin/env python3
"""Deterministic scene-file generator for the benchmark configurations.

The reference's `practice5_dragon_100k*.txt` inputs are missing from the
reference tree (`/root/reference/.MISSING_LARGE_BLOBS:1-4`).  SURVEY.md §8(d)
pins a byte-exact ~90k-triangle stand-in derived from
`hw5/practice5_dragon_10k.txt` (copied here as `scenes/practice5_dragon_10k.txt`):
every TRIANGLE is subdivided 3x3 (9 sub-triangles, 89,928 total), with the
material lines METALLIC / DIELECTRIC+IOR 1.5 appended for the metal/glass
variants.  The md5 of every generated file is checked against SURVEY.md.

Usage:
  python scenes/make_scene.py CONFIG OUT.txt          # CONFIG in CONFIGS below
  python scenes/make_scene.py --custom SRC W H S [--variant diffuse|metal|glass] [--subdiv] OUT.txt
"""
import argparse
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

# name -> (source scene, W, H, spp, subdivide, variant, md5 of the output or None)
CONFIGS = {
    "c1": ("practice5_1.txt", 256, 256, 16, False, "diffuse",
           "6041756826f3abb219e6e8c064e056df"),
    "c2": ("practice5_dragon_10k.txt", 512, 512, 64, False, "diffuse",
           "65b72cb5a1255a5038be2d68a8dbc7e4"),
    "c3": ("practice5_dragon_10k.txt", 1920, 1080, 256, True, "diffuse",
           "4ba4a022600ec8f2eff6eed017465ebe"),
    "c4_metal": ("practice5_dragon_10k.txt", 1920, 1080, 1024, True, "metal",
                 "7d239ef5a6a641d253b07173b6acd7fd"),
    "c4_glass": ("practice5_dragon_10k.txt", 1920, 1080, 1024, True, "glass",
                 "f248a59d418a6a99c53ac223bedc38db"),
    "c5": ("practice5_dragon_10k.txt", 3840, 2160, 4096, True, "diffuse",
           "fd7446716980978cb48db9670be5d941"),
}


def _first_token(line):
    parts = line.split()
    return parts[0] if parts else ""


def _fmt(x):
    return "%.6g" % x


def generate(src_text, W, H, S, subdivide, variant, depth=None):
    """Return the generated scene text (SURVEY.md §8(d) recipe); `depth`
    replaces the RAY_DEPTH line (test fixtures only, not a pinned config)."""
    lines = src_text.split("\n")
    out = []
    extra = {"diffuse": [], "metal": ["METALLIC"], "glass": ["DIELECTRIC", "IOR 1.5"]}[variant]
    i = 0
    n = len(lines)
    while i < n:
        line = lines[i]
        tok = _first_token(line)
        if tok == "DIMENSIONS":
            out.append("DIMENSIONS %d %d" % (W, H))
            i += 1
            continue
        if tok == "SAMPLES":
            out.append("SAMPLES %d" % S)
            i += 1
            continue
        if tok == "RAY_DEPTH" and depth is not None:
            out.append("RAY_DEPTH %d" % depth)
            i += 1
            continue
        if tok == "TRIANGLE" and (subdivide or extra):
            v = [float(t) for t in line.split()[1:10]]
            a, b, c = v[0:3], v[3:6], v[6:9]
            body = []
            j = i + 1
            while j < n and lines[j] != "" and _first_token(lines[j]) != "NEW_PRIMITIVE":
                body.append(lines[j])
                j += 1
            body = body + extra
            if subdivide:
                def P(ii, jj):
                    return [a[k] + (b[k] - a[k]) * ii / 3 + (c[k] - a[k]) * jj / 3 for k in range(3)]
                tris = []
                for ii in range(3):
                    for jj in range(3 - ii):
                        tris.append((P(ii, jj), P(ii + 1, jj), P(ii, jj + 1)))
                        if ii + jj < 2:
                            tris.append((P(ii + 1, jj), P(ii + 1, jj + 1), P(ii, jj + 1)))
            else:
                tris = [(a, b, c)]
            for t_idx, (pa, pb, pc) in enumerate(tris):
                if t_idx > 0:
                    out.append("NEW_PRIMITIVE")
                if subdivide:
                    out.append("TRIANGLE " + " ".join(_fmt(x) for x in pa + pb + pc))
                else:
                    out.append(line)
                out.extend(body)
            i = j
            continue
        out.append(line)
        i += 1
    return "\n".join(out)


def make(config, out_path, check=True):
    src, W, H, S, sub, variant, md5 = CONFIGS[config]
    with open(os.path.join(HERE, src), "r", newline="") as f:
        text = f.read()
    res = generate(text, W, H, S, sub, variant).encode()
    got = hashlib.md5(res).hexdigest()
    if check and md5 is not None and got != md5:
        raise RuntimeError("scene %s: md5 %s != pinned %s" % (config, got, md5))
    with open(out_path, "wb") as f:
        f.write(res)
    return got


def make_custom(src, W, H, S, subdivide, variant, out_path, depth=None):
    with open(src, "r", newline="") as f:
        text = f.read()
    res = generate(text, W, H, S, subdivide, variant, depth).encode()
    with open(out_path, "wb") as f:
        f.write(res)
    return hashlib.md5(res).hexdigest()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--custom", nargs=4, metavar=("SRC", "W", "H", "S"))
    ap.add_argument("--variant", default="diffuse", choices=["diffuse", "metal", "glass"])
    ap.add_argument("--subdiv", action="store_true")
    a = ap.parse_args(argv)
    if a.custom:
        out = a.config if a.out is None else a.out
        src, W, H, S = a.custom
        print(make_custom(src, int(W), int(H), int(S), a.subdiv, a.variant, out))
        return 0
    if a.config not in CONFIGS or a.out is None:
        ap.error("config must be one of %s" % ", ".join(CONFIGS))
    print(make(a.config, a.out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
