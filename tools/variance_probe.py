"""Where does the run-to-run spread of the C2 encode kernel come from?

Allocates several independent (data, parity) buffer sets of the C2 shape and
times the encode kernel on each, interleaved, for `--seconds`.  A spread
between sets (stable within a set) points at physical placement; a drift
with elapsed time at clocks/thermals.  One JSON line per round; run on the
GPU box from the repo root: python tools/variance_probe.py
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=4)
    ap.add_argument("--seconds", type=float, default=40.0)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--ramp", action="store_true",
                    help="per-launch times of back-to-back encodes after an idle gap")
    ap.add_argument("--phases", action="store_true",
                    help="diagonal timings between phases of other traffic (read, copy, cross pairs)")
    ap.add_argument("--cross", action="store_true",
                    help="time every (data set, parity set) pair and a plain copy per set")
    a = ap.parse_args()
    import torch
    from memo_amd import ec
    k, m, B, n = 10, 4, 1 << 20, 4096
    S = ec.shard_size(B, k)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    c = ec.Codec(0)
    c.set_stream(st)
    sets = []
    for i in range(a.sets):
        d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
        c.fill_blocks(0x6D656D6F, 0, n, B, k, S, d)
        sets.append((d, p))
    torch.cuda.synchronize()
    alg = (k + m) * S * n

    def timed(fn):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.launches)]
        fn()
        for x, y in ev:
            x.record(st)
            fn()
            y.record(st)
        torch.cuda.synchronize()
        return float(np.median([x.elapsed_time(y) for x, y in ev]))

    t00 = time.perf_counter()

    def diag(tag):
        for r in range(3):
            row = {"phase": tag, "t": round(time.perf_counter() - t00, 2)}
            for i, (d, p) in enumerate(sets):
                row["set%d" % i] = round(alg / (timed(lambda: c.encode(k, m, d, p)) * 1e-3) / 8e12, 4)
            print(json.dumps(row), flush=True)

    if a.ramp:
        d, p = sets[0]
        for idle in (2.0, 0.5, 0.1, 0.02):
            time.sleep(idle)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(120)]
            for x, y in ev:
                x.record(st)
                c.encode(k, m, d, p)
                y.record(st)
            torch.cuda.synchronize()
            fr = [round(alg / (x.elapsed_time(y) * 1e-3) / 8e12, 3) for x, y in ev]
            print(json.dumps({"idle_s": idle, "first_20": fr[:20],
                              "mean_by_10": [round(float(np.mean(fr[i:i + 10])), 4)
                                             for i in range(0, 120, 10)]}), flush=True)
        return

    if a.phases:
        diag("A-initial")
        for d, _ in sets:
            for _ in range(6):
                d.view(torch.int64).sum()
        torch.cuda.synchronize()
        diag("B-after-reads")
        dst = sets[0][1].view(-1)
        for d, _ in sets:
            for _ in range(6):
                dst.copy_(d.view(-1)[:dst.numel()])
        torch.cuda.synchronize()
        diag("C-after-copies")
        for d, _ in sets:
            for _, p in sets:
                for _ in range(6):
                    c.encode(k, m, d, p)
        torch.cuda.synchronize()
        diag("D-after-cross-pairs")
        time.sleep(5)
        diag("E-after-5s-idle")
        return

    if a.cross:
        for rep in range(2):
            for i, (d, _) in enumerate(sets):
                row = {"rep": rep, "data_set": i}
                for j, (_, p) in enumerate(sets):
                    row["parity_set%d" % j] = round(alg / (timed(lambda: c.encode(k, m, d, p)) * 1e-3) / 8e12, 4)
                # read+write copy of this data set into parity set 0's memory
                # (first m*S*n bytes) and a read-only reduction over it
                dst = sets[0][1].view(-1)
                src = d.view(-1)[:dst.numel()]
                row["copy_TBs"] = round(2 * dst.numel() / (timed(lambda: dst.copy_(src)) * 1e-3) / 1e12, 3)
                row["read_TBs"] = round(d.numel() / (timed(lambda: d.view(torch.int64).sum()) * 1e-3) / 1e12, 3)
                print(json.dumps(row), flush=True)
        return
    t0, rnd = time.perf_counter(), 0
    while time.perf_counter() - t0 < a.seconds:
        row = {"round": rnd, "t": round(time.perf_counter() - t0, 2)}
        for i, (d, p) in enumerate(sets):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.launches)]
            c.encode(k, m, d, p)
            for x, y in ev:
                x.record(st)
                c.encode(k, m, d, p)
                y.record(st)
            torch.cuda.synchronize()
            ms = float(np.median([x.elapsed_time(y) for x, y in ev]))
            row["set%d" % i] = round(alg / (ms * 1e-3) / 8e12, 4)
        print(json.dumps(row), flush=True)
        rnd += 1
        time.sleep(0.5)
    print(json.dumps({"data_ptrs_mod_2MiB": [int(d.data_ptr() % (2 << 20)) for d, _ in sets],
                      "parity_ptrs_mod_2MiB": [int(p.data_ptr() % (2 << 20)) for _, p in sets]}))


if __name__ == "__main__":
    main()
