#!/usr/bin/env python3
"""Instruction counts per step kind of q_exec (tools/micro/qexec_sizes.hip):
    python tools/micro/qexec_sizes.py   (compiles with hipcc -S for gfx950)"""
import collections, os, re, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "raytracing-course_amd")
out = "/tmp/qexec_sizes.s"
subprocess.check_call(["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-ffp-contract=off", "-fno-fast-math", "--offload-arch=gfx950",
                       "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(PKG, "csrc"), "-I" + os.path.join(PKG, "csrc", "device"),
                       "-S", "--cuda-device-only", os.path.join(REPO, "tools", "micro", "qexec_sizes.hip"), "-o", out] + sys.argv[1:])
names = ["aux node", "probe", "leaf check", "walk entries", "walk nodes"]
text = open(out).read()
for k, n in enumerate(names):
    m = re.search(r"^_Z6k_kindILi%dEEvN2pt9SceneViewEPNS0_5QueryEPKNS0_2F4EPNS0_7QCountsEPj:(.*?)^\.Lfunc_end" % k, text, re.S | re.M)
    body = m.group(1)
    c = collections.Counter()
    for l in body.split("\n"):
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c["valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "lds" if op.startswith("ds_") else "other"] += 1
    print("%-13s %s" % (n, dict(c)))
