#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh run (rocprofv3 kernel trace + PMC passes)
into a committed profile summary and the per-launch HBM traffic table that
bench.py reads (profiles/traffic.json).

    python tools/pmc_summary.py gpurun_out/prof profiles/r01_<tag> [--key c3_spp1_n1]

Counter conventions (MI355X_MICROARCH.md, HBM/rocprofv3 section):
  * FETCH_SIZE / WRITE_SIZE are in KiB and count the L2's memory-side requests
    (Infinity-Cache hits included).
  * gfx950: FETCH_SIZE reports half the bytes of 128-B requests -> doubled here.
    Cross-checked against TCC_MISS_sum x 128 B from a separate pass.
"""
import argparse
import collections
import sys
import csv
import json
import os
import shutil


sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, kernel=None, last=0):
    """{kernel: ({counter: sum}, dispatches)}; with `kernel` (substring) and `last`
    > 0, only the last `last` dispatches of the matching kernels, pooled under `kernel`."""
    rows = list(csv.DictReader(open(path)))
    keep = None
    if kernel and last:
        ids = sorted({int(r["Dispatch_Id"]) for r in rows if kernel in r["Kernel_Name"]})
        keep = set(ids[-last:])
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"]
        if keep is not None:
            if int(r["Dispatch_Id"]) not in keep:
                continue
            k = kernel
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: ({c: v for c, v in d.items()}, len(disp[k])) for k, d in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="pt::k_wpath",
                    help="substring of the kernel name; every instantiation that matches is pooled (calls-weighted)")
    ap.add_argument("--key", default="c3_spp1_n1")
    ap.add_argument("--traffic-json", default=os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                            "traffic.json"))
    ap.add_argument("--timed", type=int, default=-1,
                    help="average over the last N launches only (default: the bench's timed launches, "
                         "roofline.launches of bench_kt.json; 0 = all launches)")
    a = ap.parse_args()
    if a.timed < 0:
        a.timed = 0
        try:
            a.timed = int(json.load(open(os.path.join(a.prof, "bench_kt.json")))["roofline"]["launches"])
        except Exception:
            pass
    os.makedirs(a.out, exist_ok=True)
    kt = os.path.join(a.prof, "kt")
    for f in ("run_kernel_stats.csv",):
        shutil.copy(os.path.join(kt, f), os.path.join(a.out, "kernel_stats.csv"))
    lines = ["# rocprofv3 summary (%s)" % os.path.basename(os.path.normpath(a.out)), ""]
    lines.append("## kernel trace (--kernel-trace --stats)")
    lines.append("")
    lines.append("| kernel | calls | avg ms | total ms | % |")
    lines.append("|---|---|---|---|---|")
    avg_ns = None
    calls = tot_ns = 0.0
    for r in csv.DictReader(open(os.path.join(kt, "run_kernel_stats.csv"))):
        lines.append("| `%s` | %s | %.3f | %.3f | %s |" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6,
                                                          float(r["TotalDurationNs"]) / 1e6, r["Percentage"]))
        if a.kernel in r["Name"]:
            calls += float(r["Calls"])
            tot_ns += float(r["TotalDurationNs"])
    if calls:
        avg_ns = tot_ns / calls
        lines += ["", "`%s` (all instantiations): %d launches, mean %.3f ms" % (a.kernel, calls, avg_ns / 1e6)]
    if a.timed:
        # the bench's timed region = the last `timed` launches (the warm-up pass comes first)
        d = sorted((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                   for r in csv.DictReader(open(os.path.join(kt, "run_kernel_trace.csv"))) if a.kernel in r["Kernel_Name"])
        d = [x[1] for x in d[-a.timed:]]
        avg_ns = sum(d) / len(d)
        lines += ["`%s` over the bench's timed region (last %d launches, kernel trace): mean %.3f ms"
                  % (a.kernel, len(d), avg_ns / 1e6)]
    # resources of the kernel: registers from the compiler's report (the trace's
    # VGPR_Count column is in allocation granules, not registers); grid from the trace
    import kernel_resources
    res_k = kernel_resources.kernel(a.kernel)
    for name, v in sorted(res_k.items()):
        lines += ["", "`%s` (compiler): %d VGPRs + %d AGPRs, %d SGPRs, %d VGPR / %d SGPR spills, scratch %d B/lane, "
                  "%d waves/SIMD" % (name, v.get("vgpr", 0), v.get("agpr", 0), v.get("sgpr", 0), v.get("vgpr_spill", 0),
                                     v.get("sgpr_spill", 0), v.get("scratch_bytes", 0), v.get("waves_per_simd", 0))]
    for r in csv.DictReader(open(os.path.join(kt, "run_kernel_trace.csv"))):
        if a.kernel in r["Kernel_Name"]:
            lines += ["`%s` (trace): LDS %s B, grid %s x wg %s" % (
                a.kernel, r["LDS_Block_Size"], r["Grid_Size_X"], r["Workgroup_Size_X"])]
            break
    pmc = {}
    per_alg, per_ray = {}, {}   # counter totals over the timed launches / that pass's algorithmic bytes, rays
    for sub in sorted(os.listdir(a.prof)):
        p = os.path.join(a.prof, sub, "run_counter_collection.csv")
        if sub.startswith("pmc") and os.path.exists(p):
            bj = None
            bjp = os.path.join(a.prof, "bench_%s.json" % sub[4:])
            if os.path.exists(bjp):
                try:
                    bj = json.load(open(bjp))
                except Exception:
                    bj = None
            timed = int(bj["roofline"]["launches"]) if bj else a.timed
            tot, nd = collections.defaultdict(float), 0
            for k, (d, n) in per_kernel(p, a.kernel, timed).items():
                if a.kernel in k:
                    nd += n
                    for c, v in d.items():
                        tot[c] += v
            for c, v in tot.items():
                pmc[c] = v / nd
                if bj:
                    per_alg[c] = v / (bj["roofline"]["alg_bytes_per_launch"] * nd)
                    per_ray[c] = v / bj["rays"]
    lines += ["", "## PMC, per %s launch (separate --pmc passes%s)"
              % (a.kernel, ", last %d launches" % a.timed if a.timed else ""), ""]
    for c, v in sorted(pmc.items()):
        lines.append("* %s = %.6g" % (c, v))
    res = {}
    if "FETCH_SIZE" in pmc:
        fetch = pmc["FETCH_SIZE"] * 1024.0 * 2.0
        write = pmc.get("WRITE_SIZE", 0.0) * 1024.0
        res = {"hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
               "source": "rocprofv3 --pmc FETCH_SIZE (KiB, x2 gfx950 correction) + WRITE_SIZE (KiB), per launch; "
                         "L2 memory-side bytes (Infinity-Cache hits included)"}
        if "TCC_MISS_sum" in pmc:
            res["tcc_miss_x128_bytes"] = pmc["TCC_MISS_sum"] * 128.0
            res["l2_hit_rate"] = pmc["TCC_HIT_sum"] / (pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"])
        if avg_ns:
            res["avg_launch_ms"] = avg_ns / 1e6
            res["traffic_GBps"] = res["hbm_bytes_per_launch"] / avg_ns
        lines += ["", "## derived", ""]
        for k, v in res.items():
            lines.append("* %s = %s" % (k, v if isinstance(v, str) else "%.6g" % v))
    if "FETCH_SIZE" in per_alg:
        res["traffic_per_alg_byte"] = per_alg["FETCH_SIZE"] * 2048.0 + per_alg.get("WRITE_SIZE", 0.0) * 1024.0
        res["fetch_bytes_per_ray"] = per_ray["FETCH_SIZE"] * 2048.0
        if "WRITE_SIZE" in per_ray:
            res["write_bytes_per_ray"] = per_ray["WRITE_SIZE"] * 1024.0
        lines.append("* traffic / algorithmic bytes (per pass, same launches) = %.4g" % res["traffic_per_alg_byte"])
        lines.append("* fetch bytes per ray = %.4g, write bytes per ray = %.4g"
                     % (res["fetch_bytes_per_ray"], res.get("write_bytes_per_ray", 0.0)))
    if "SQ_INSTS_VALU" in pmc and "SQ_WAVES" in pmc:
        lines.append("* VALU instructions per wave = %.6g" % (pmc["SQ_INSTS_VALU"] / pmc["SQ_WAVES"]))
    if "SQ_INSTS_VALU" in per_ray:
        lines.append("* VALU wave-instructions per ray = %.4g" % per_ray["SQ_INSTS_VALU"])
    # what limits the kernel (SQ_* cycle counters are per wave, in quad-cycles; a
    # SIMD issues one wave64 VALU instruction per 2 cycles)
    if "SQ_WAVE_CYCLES" in pmc and "SQ_ACTIVE_INST_VALU" in pmc:
        wc = pmc["SQ_WAVE_CYCLES"]
        busy = pmc.get("SQ_BUSY_CYCLES")
        lim = {"active_valu_frac": pmc["SQ_ACTIVE_INST_VALU"] / wc}
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC"):
            if c in pmc:
                lim[c.lower().replace("sq_", "") + "_frac"] = pmc[c] / wc
        if "SQ_INSTS_VALU" in pmc and res.get("avg_launch_ms"):
            # VALU issue share of the chip: 2 cycles per wave64 instruction, 1024 SIMDs, the clock from GRBM
            clk = pmc["GRBM_GUI_ACTIVE"] / 8.0 / (res["avg_launch_ms"] * 1e-3) if "GRBM_GUI_ACTIVE" in pmc else 2.4e9
            lim["valu_issue_frac"] = pmc["SQ_INSTS_VALU"] * 2.0 / (1024 * clk * res["avg_launch_ms"] * 1e-3)
            lim["clock_ghz"] = clk / 1e9
        res.update(lim)
        lines += ["", "## what limits k_wpath (fractions of wave cycles)", ""]
        for k, v in sorted(lim.items()):
            lines.append("* %s = %.4g" % (k, v))
    open(os.path.join(a.out, "SUMMARY.md"), "w").write("\n".join(lines) + "\n")
    for f in os.listdir(a.prof):
        if f.endswith(".json"):
            shutil.copy(os.path.join(a.prof, f), os.path.join(a.out, f))
    if res:
        tj = {}
        if os.path.exists(a.traffic_json):
            tj = json.load(open(a.traffic_json))
        res["profile"] = os.path.relpath(a.out, os.path.dirname(os.path.abspath(a.traffic_json)))
        tj[a.key] = res
        json.dump(tj, open(a.traffic_json, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
