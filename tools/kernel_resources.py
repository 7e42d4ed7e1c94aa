#!/usr/bin/env python3
"""Per-kernel register/occupancy figures from the compiler's resource report
(raytracing-course_amd/build/*.resources.txt, written by the Makefile with
-Rpass-analysis=kernel-resource-usage).  These are the allocation-relevant
numbers (arch VGPRs, AGPRs, spills, waves/SIMD); rocprofv3's kernel-trace
VGPR_Count column is in allocation granules and must not be read as registers.

`scratch_insts` counts each kernel's scratch (private-memory) instructions in the
shipped code object (the objects' fat binary, unbundled and disassembled with the
ROCm LLVM tools): a ScratchSize the compiler reserves but no instruction touches
(a frame left behind by lowering, 20 B in k_wcoop) costs nothing at run time.

    python tools/kernel_resources.py [build_dir] [--kernel k_wpath]
"""
import argparse
import glob
import json
import os
import re
import subprocess
import tempfile

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


LLVM = "/opt/rocm/lib/llvm/bin"


def scratch_insts(obj):
    """{mangled kernel name: scratch_* / buffer_* instructions} of a hipcc device object"""
    counts, cur = {}, None
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "dev.co")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb], check=True,
                       capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fb,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True,
                       capture_output=True)
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True, capture_output=True,
                             text=True).stdout
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            counts[cur] = 0
        elif cur and re.search(r"\s(scratch|buffer)_(load|store)", line):
            counts[cur] += 1
    return counts


def read_isa(build_dir=None):
    """read() plus scratch_insts per kernel (null where the code object cannot be read)"""
    build_dir = build_dir or os.path.join(REPO, "raytracing-course_amd", "build")
    out = read(build_dir)
    for obj in sorted(glob.glob(os.path.join(build_dir, "pt_*.o"))):
        try:
            c = scratch_insts(obj)
        except (OSError, subprocess.CalledProcessError):
            continue
        for k, v in c.items():
            if k in out:
                out[k]["scratch_insts"] = v
    return out


def kernel(name_part, build_dir=None):
    """{mangled name: figures} of the kernels whose mangled name contains name_part"""
    key = name_part.replace("pt::", "")
    return {k: v for k, v in read_isa(build_dir).items() if key in k}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("build_dir", nargs="?")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    print(json.dumps(kernel(a.kernel, a.build_dir), indent=1))
