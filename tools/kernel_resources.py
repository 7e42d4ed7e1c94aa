#!/usr/bin/env python3
"""Per-kernel register/occupancy figures from the compiler's resource report
(raytracing-course_amd/build/*.resources.txt, written by the Makefile with
-Rpass-analysis=kernel-resource-usage).  These are the allocation-relevant
numbers (arch VGPRs, AGPRs, spills, waves/SIMD); rocprofv3's kernel-trace
VGPR_Count column is in allocation granules and must not be read as registers.

    python tools/kernel_resources.py [build_dir] [--kernel k_wpath]
"""
import argparse
import glob
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "TotalSGPRs": "sgpr", "ScratchSize [bytes/lane]": "scratch_bytes",
          "Occupancy [waves/SIMD]": "waves_per_simd", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
          "LDS Size [bytes/block]": "lds_static_bytes"}


def read(build_dir=None):
    build_dir = build_dir or os.path.join(REPO, "raytracing-course_amd", "build")
    out, cur = {}, None
    for path in sorted(glob.glob(os.path.join(build_dir, "*.resources.txt"))):
        for line in open(path):
            m = re.search(r"remark:\s+Function Name: (\S+)", line)
            if m:
                cur = out.setdefault(m.group(1), {})
                continue
            m = re.search(r"remark:\s+([A-Za-z][^:]*?): (\d+)", line)
            if m and cur is not None and m.group(1).strip() in FIELDS:
                cur[FIELDS[m.group(1).strip()]] = int(m.group(2))
    return out


def kernel(name_part, build_dir=None):
    """{mangled name: figures} of the kernels whose mangled name contains name_part"""
    key = name_part.replace("pt::", "")
    return {k: v for k, v in read(build_dir).items() if key in k}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("build_dir", nargs="?")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    print(json.dumps(kernel(a.kernel, a.build_dir), indent=1))
