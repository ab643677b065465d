"""Summarise tools/profile.sh output (gpurun_out/prof) into profiles/.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.csv            per-dispatch FETCH_SIZE / WRITE_SIZE of the
                                    encode MAC and the rebuild MAC
  profiles/<tag>_summary.md         kernel times, algorithmic vs PMC bytes
(bench.py measures roofline.traffic itself, with its own counter passes.)

The encode (gf_mac_kernel<KC, R, NT, false>) and the rebuild MAC
(gf_mac_images_kernel<KC, R, NT> over per-block table images, or
gf_mac_kernel<..., true> with tables built in LDS; after the decode-rows
kernel) are told apart by their names.  HBM bytes per launch = (2 * FETCH_SIZE +
WRITE_SIZE) * 1024: on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read and WRITE_SIZE is exact for 16-byte-per-lane stores
(MI355X_MICROARCH.md, HBM).
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def kind(name):
    if "gf_mac_images_kernel" in name:
        return "rebuild_mac"
    if name.startswith("void memo_ec::gf_mac_kernel") or name.startswith("memo_ec::gf_mac_kernel"):
        return "rebuild_mac" if name.split("(")[0].rstrip(">").rstrip().endswith("true") else "encode"
    if "gf_rebuild_kernel" in name:
        return "rebuild_fused"
    if "decode_" in name:
        return "decode"
    return None


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    prof = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof")
    k, m, B, n, e = 10, 4, 1 << 20, 4096, 4
    S = ((B + k - 1) // k + 63) // 64 * 64
    alg = {"encode": (k + m) * S * n, "rebuild_mac": (k + e) * S * n}
    out_dir = os.path.join(ROOT, "profiles")
    stats = os.path.join(prof, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out_dir, "%s_kernel_stats.csv" % tag))
    trace = rows(os.path.join(prof, "trace", "trace_kernel_trace.csv"))
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = {}
    for r in trace:
        kd = kind(r["Kernel_Name"])
        if kd:
            durs.setdefault(kd, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    live = None
    for line in open(os.path.join(prof, "trace.log")):
        if line.startswith("{"):
            live = json.loads(line)
    steps = live["steps"] if live else 25
    pmc = {}
    for what in ("fetch", "write"):
        for r in rows(os.path.join(prof, what, "%s_counter_collection.csv" % what)):
            kd = kind(r["Kernel_Name"])
            if kd in alg:
                pmc.setdefault((kd, what), []).append(float(r["Counter_Value"]))
    with open(os.path.join(out_dir, "%s_pmc.csv" % tag), "w") as f:
        f.write("kernel,launch,FETCH_SIZE_KB,WRITE_SIZE_KB\n")
        for kd in alg:
            for i, (a, b) in enumerate(zip(pmc.get((kd, "fetch"), []), pmc.get((kd, "write"), []))):
                f.write("%s,%d,%.1f,%.1f\n" % (kd, i, a, b))
    md = ["# %s profile: RS(10,4) encode (C2) + 4-erasure rebuild (C3), 4096 x 1 MiB blocks, 1 MI355X" % tag,
          "", "Command: `tools/profile.sh` -- rocprofv3 --kernel-trace --stats on `python3 bench.py "
          "--no-cpu --no-e2e --no-small --no-pmc --no-verify --no-c5 --no-plugin --no-sha` (the "
          "contract's step: one encode + one rebuild, and the achievable-rate probe); then "
          "--pmc FETCH_SIZE and --pmc WRITE_SIZE passes, each its own run.", "",
          "| kernel | calls | avg us | min us | max us |", "|---|---|---|---|---|"]
    for r in rows(stats):
        md.append("| %s | %s | %.1f | %.1f | %.1f |" % (r["Name"].replace("|", "/"), r["Calls"],
                                                      float(r["AverageNs"]) / 1e3,
                                                      float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
    md.append("")
    for kd, label, key in (("encode", "encode MAC (gf_mac_kernel<10, 4, true, false>)",
                            "encode_%d_%d_%d_%d" % (k, m, B, n)),
                           ("rebuild_mac", "rebuild MAC (gf_mac_images_kernel<10, 4, true>, or "
                            "gf_mac_kernel<10, 4, true, true> with tables built in LDS)",
                            "rebuild_%d_%d_%d_%d_e%d" % (k, m, B, n, e))):
        d = durs.get(kd, [])
        if not d:
            continue
        timed = d[-steps:]
        t_avg = statistics.mean(timed)
        line = ("%s: the %d timed launches average %.1f us -> %.0f GB/s algorithmic (%.1f%% of "
                "8000 GB/s); all %d launches %.1f us." % (label, len(timed), t_avg * 1e3,
                                                        alg[kd] / (t_avg * 1e-3) / 1e9,
                                                        alg[kd] / (t_avg * 1e-3) / 1e9 / 80,
                                                        len(d), statistics.mean(d) * 1e3))
        if live:
            ev = live["roofline"]["kernel_ms_avg"] if kd == "encode" else None
            if ev:
                line += " The bench line of the same process (HIP events): %.4f ms (%.1f%% apart)." % (
                    ev, abs(t_avg - ev) / ev * 100)
        md.append(line)
        fe, wr = pmc.get((kd, "fetch")), pmc.get((kd, "write"))
        if fe and wr:
            f_med, w_med = statistics.median(fe), statistics.median(wr)
            hbm = (2 * f_med + w_med) * 1024
            md.append("PMC HBM bytes per %s launch: (2*%.0f + %.0f) KB * 1024 = %d (%.3f x the %d "
                      "algorithmic bytes)." % (kd, f_med, w_med, hbm, hbm / alg[kd], alg[kd]))
        md.append("")
    if "decode" in durs:
        dd = durs["decode"][-steps:]
        md.append("Decode rows (4096 blocks, column-per-lane kernel): %.1f us per rebuild step." %
                  (statistics.mean(dd) * 1e3))
    open(os.path.join(out_dir, "%s_summary.md" % tag), "w").write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
