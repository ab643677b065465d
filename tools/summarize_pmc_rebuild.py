#!/usr/bin/env python3
"""Summarise tools/pmc_rebuild.sh output: per shape and rebuild path, the
encode MAC, the rebuild MAC (or fused kernel) and the decode kernel --
average duration (kernel trace) and per-dispatch medians of every counter.
  usage: summarize_pmc_rebuild.py [gpurun_out/pmc_rebuild] > profiles/<tag>.md"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_rebuild"


def short(name):
    if "gf_rebuild_kernel" in name:
        return "gf_rebuild_kernel (fused)"
    if "gf_mac_images_kernel" in name:
        return "gf_mac_images_kernel rebuild MAC"
    if "gf_mac_kernel" in name:
        return "gf_mac_kernel rebuild MAC" if name.rstrip(")").split("(")[0].endswith("true>") \
            else "gf_mac_kernel encode"
    if "decode_coef" in name:
        return "decode_coef_kernel"
    return None


rows = []
for d in sorted(glob.glob(os.path.join(base, "*_f*"))):
    tag = os.path.basename(d)
    k, m, B, n, path = tag.split("_")
    dur = {}
    st = os.path.join(d, "trace", "trace_kernel_stats.csv")
    if os.path.exists(st):
        for r in csv.DictReader(open(st)):
            s = short(r["Name"])
            if s:
                dur[s] = float(r["AverageNs"]) / 1e3
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            s = short(r["Kernel_Name"])
            if s:
                cnt[s][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("## RS(%s,%s), %s x %s-byte blocks, e = m, path %s" % (k, m, n, B,
          "fused" if path == "f1" else "rows (two-kernel)"))
    names = sorted(set(dur) | set(cnt))
    keys = sorted({c for s in cnt.values() for c in s})
    print("")
    print("| counter | " + " | ".join(names) + " |")
    print("|---|" + "---|" * len(names))
    print("| avg us (trace) | " + " | ".join("%.1f" % dur.get(x, float("nan")) for x in names) + " |")
    for c in keys:
        vals = []
        for x in names:
            v = cnt[x].get(c)
            vals.append("%.4g" % statistics.median(v) if v else "")
        print("| %s | %s |" % (c, " | ".join(vals)))
    print("")
