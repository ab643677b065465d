#!/usr/bin/env python3
"""Summarise tools/pmc_4k.sh output: for each shape, the encode MAC, the
rebuild MAC and the decode-rows kernel -- average duration (kernel trace),
per-dispatch medians of every counter, and the derived figures:
  clock      = GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md,
               DVFS give-back);
  valu_busy  = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction holds a
               SIMD-32 for 2 cycles) / (1024 SIMDs x clock x duration);
  per wave   = SQ_ACTIVE_INST_ANY / SQ_WAIT_INST_ANY / SQ_WAIT_ANY (quad
               cycles) / SQ_WAVES: issuing, issue-stalled, parked;
  salu_per_wave, valu_per_wave, lds_per_wave.
  usage: summarize_pmc_4k.py [gpurun_out/.../pmc_4k] > profiles/<tag>.md"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_4k"
SIMDS = 256 * 4


def short(name):
    if "gf_rebuild_kernel" in name:
        return "gf_rebuild_kernel (fused)"
    if "gf_mac_images_kernel" in name:
        return "rebuild MAC"
    if "gf_mac_kernel" in name:
        return "rebuild MAC" if name.rstrip(")").split("(")[0].endswith("true>") else "encode MAC"
    if "decode_" in name:
        return "decode rows"
    return None


for d in sorted(glob.glob(os.path.join(base, "*_f*"))):
    k, m, B, n, _ = os.path.basename(d).split("_")
    dur = {}
    st = os.path.join(d, "trace", "trace_kernel_stats.csv")
    if os.path.exists(st):
        for r in csv.DictReader(open(st)):
            s = short(r["Name"])
            if s:
                dur[s] = float(r["AverageNs"]) * 1e-9
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            s = short(r["Kernel_Name"])
            if s:
                cnt[s][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = [x for x in ("encode MAC", "rebuild MAC", "decode rows") if x in dur or x in cnt]
    med = {x: {c: statistics.median(v) for c, v in cnt[x].items()} for x in names}
    print("## RS(%s,%s), %s x %s-byte blocks, e = m, rows path\n" % (k, m, n, B))
    print("| | " + " | ".join(names) + " |")
    print("|---|" + "---|" * len(names))

    def row(label, f):
        vals = []
        for x in names:
            try:
                vals.append(f(x))
            except (KeyError, ZeroDivisionError, TypeError):
                vals.append("")
        print("| %s | %s |" % (label, " | ".join(vals)))

    row("avg us (trace)", lambda x: "%.1f" % (dur[x] * 1e6))
    row("clock GHz (GRBM_GUI_ACTIVE/8/dur)", lambda x: "%.2f" % (med[x]["GRBM_GUI_ACTIVE"] / 8 / dur[x] / 1e9))

    def busy(x):
        clk = med[x]["GRBM_GUI_ACTIVE"] / 8 / dur[x]
        return "%.1f%%" % (100 * med[x]["SQ_INSTS_VALU"] * 2 / (SIMDS * clk * dur[x]))
    row("valu_busy (INSTS_VALU x 2 / SIMD cycles)", busy)
    for lab, c in (("VALU instr / wave", "SQ_INSTS_VALU"), ("SALU instr / wave", "SQ_INSTS_SALU"),
                   ("LDS instr / wave", "SQ_INSTS_LDS"), ("VMEM rd / wave", "SQ_INSTS_VMEM_RD")):
        row(lab, lambda x, c=c: "%.0f" % (med[x][c] / med[x]["SQ_WAVES"]))
    for lab, c in (("issuing, cycles / wave", "SQ_ACTIVE_INST_ANY"),
                   ("issue-stalled, cycles / wave", "SQ_WAIT_INST_ANY"),
                   ("parked (waitcnt/barrier), cycles / wave", "SQ_WAIT_ANY"),
                   ("LDS issue stall, cycles / wave", "SQ_WAIT_INST_LDS")):
        row(lab, lambda x, c=c: "%.0f" % (4 * med[x][c] / med[x]["SQ_WAVES"]))
    row("LDS bank conflict / LDS active cycles",
        lambda x: "%.3f" % (med[x]["SQ_LDS_BANK_CONFLICT"] / max(1.0, med[x]["SQ_LDS_IDX_ACTIVE"])))
    keys = sorted({c for x in names for c in med[x]})
    print("\nraw per-dispatch medians:\n")
    print("| counter | " + " | ".join(names) + " |")
    print("|---|" + "---|" * len(names))
    for c in keys:
        print("| %s | %s |" % (c, " | ".join("%.4g" % med[x][c] if c in med[x] else "" for x in names)))
    print("")
