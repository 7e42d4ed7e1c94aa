#!/usr/bin/env python3
"""Per-kernel totals of a rocprofv3 --pmc CSV directory (counter_collection.csv files)."""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, d in vals.items():
    if "k_w" not in k:
        continue
    print("%s (%d dispatches)" % (k, len(disp[k])))
    for c, v in sorted(d.items()):
        print("   %-24s %.4g" % (c, v))
    if "SQ_WAVE_CYCLES" in d:
        wc = d["SQ_WAVE_CYCLES"]
        print("   fractions of wave cycles: " + ", ".join("%s %.3f" % (c, v / wc) for c, v in sorted(d.items())
                                                          if c.startswith(("SQ_WAIT", "SQ_ACTIVE"))))
