"""Summarise tools/profile.sh output (gpurun_out/prof) into profiles/.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.csv            per-dispatch FETCH_SIZE / WRITE_SIZE of gf_mac_kernel
  profiles/<tag>_summary.md         kernel time, algorithmic vs PMC bytes, GB/s
  profiles/pmc_traffic.json         per-launch HBM traffic read by bench.py

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read and
WRITE_SIZE is exact for 16-byte-per-lane stores (MI355X_MICROARCH.md, HBM).
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


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    prof = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof")
    k, m, B, n = 10, 4, 1 << 20, 4096
    S = ((B + k - 1) // k + 63) // 64 * 64
    alg = (k + m) * S * n
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    stats = os.path.join(prof, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out_dir, "%s_kernel_stats.csv" % tag))
    st = {r["Name"]: r for r in rows(stats)}
    mac = st["gf_mac_kernel"]
    trace = [r for r in rows(os.path.join(prof, "trace", "trace_kernel_trace.csv"))
             if r["Kernel_Name"].startswith("gf_mac_kernel")]
    # bench order: the encode section (warmup + timed launches) comes first;
    # the rebuild sections follow
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace]
    fetch = [float(r["Counter_Value"]) for r in rows(os.path.join(prof, "fetch", "fetch_counter_collection.csv"))
             if r["Kernel_Name"].startswith("gf_mac_kernel")]
    write = [float(r["Counter_Value"]) for r in rows(os.path.join(prof, "write", "write_counter_collection.csv"))
             if r["Kernel_Name"].startswith("gf_mac_kernel")]
    f_med, w_med = statistics.median(fetch), statistics.median(write)
    hbm = (2 * f_med + w_med) * 1024
    with open(os.path.join(out_dir, "%s_pmc.csv" % tag), "w") as f:
        f.write("launch,FETCH_SIZE_KB,WRITE_SIZE_KB\n")
        for i, (a, b) in enumerate(zip(fetch, write)):
            f.write("%d,%.1f,%.1f\n" % (i, a, b))
    live = None
    for line in open(os.path.join(prof, "trace.log")):
        if line.startswith("{"):
            live = json.loads(line)
    enc = durs[:live["warmup"] + live["steps"]] if live else durs
    e_avg = statistics.mean(enc)
    tj = os.path.join(out_dir, "pmc_traffic.json")
    t = json.load(open(tj)) if os.path.exists(tj) else {}
    t["encode_%d_%d_%d_%d" % (k, m, B, n)] = {
        "hbm_bytes_per_launch": int(hbm), "algorithmic_bytes": alg,
        "ratio": round(hbm / alg, 4),
        "fetch_kb_median": f_med, "write_kb_median": w_med,
        "source": "profiles/%s_pmc.csv (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                  "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024)" % tag}
    json.dump(t, open(tj, "w"), indent=1)
    md = ["# %s profile: RS(10,4) encode + rebuild, 4096 x 1 MiB blocks, 1 MI355X" % tag, "",
          "Command: `tools/profile.sh` (rocprofv3 --kernel-trace --stats; then --pmc FETCH_SIZE; "
          "then --pmc WRITE_SIZE, each on `python3 bench.py --no-cpu --no-e2e` with the default 60 warmup + 50 timed launches).", "",
          "| kernel | calls | avg us | min us | max us |", "|---|---|---|---|---|"]
    for name, r in st.items():
        md.append("| %s | %s | %.1f | %.1f | %.1f |" % (name, r["Calls"], float(r["AverageNs"]) / 1e3,
                                                      float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
    timed = enc[-live["steps"]:] if live else enc
    t_avg = statistics.mean(timed)
    md += ["", "gf_mac_kernel, the %d timed encode launches: mean %.1f us -> %.0f GB/s algorithmic "
           "(%.1f%% of 8000 GB/s). All %d encode launches including warmup: mean %.1f us."
           % (len(timed), t_avg * 1e3, alg / (t_avg * 1e-3) / 1e9, alg / (t_avg * 1e-3) / 1e9 / 80,
              len(enc), e_avg * 1e3),
           ] + ([] if live is None else [
           "", "The bench line of the same profiled process measured the same kernel with HIP events "
           "on its stream: kernel_ms_avg %.4f ms over the %d timed steps (%.1f%% of 8000 GB/s); "
           "rocprofv3 mean over the same timed launches: %.4f ms (%.1f%% apart)."
           % (live["roofline"]["kernel_ms_avg"], live["steps"], live["roofline"]["frac"] * 100,
              statistics.mean(enc[-live["steps"]:]),
              abs(statistics.mean(enc[-live["steps"]:]) - live["roofline"]["kernel_ms_avg"])
              / live["roofline"]["kernel_ms_avg"] * 100)]) + [
           "", "Algorithmic bytes per encode launch: (k+m)*S*n = %d." % alg,
           "PMC HBM bytes per encode launch: (2*%.0f + %.0f) KB * 1024 = %d (%.3f x algorithmic)."
           % (f_med, w_med, hbm, hbm / alg)]
    open(os.path.join(out_dir, "%s_summary.md" % tag), "w").write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
