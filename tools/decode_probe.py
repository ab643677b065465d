#!/usr/bin/env python3
"""Decode-rows kernel time by batch size: the column-per-lane kernel
(decode_coef_wide_kernel) against the one-lane-per-block kernels
(decode_rows_k_kernel / decode_coef_kernel), alternating in groups of 5
launches, median HIP-event time of each; both outputs compared.  Sets the
MEMO_EC_OPT_DECODE_WIDE_MAX default.  Prints one JSON line per (k, m, n).
  usage: decode_probe.py [k,m ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from memo_amd import ec
    codes = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [(10, 4), (16, 4), (4, 2), (12, 4)]
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    c = ec.Codec(0)
    c.set_stream(st)
    if not os.environ.get("MEMO_EC_LIB"):  # MEMO_EC_LIB: another build (an A/B's other side)
        ec.check_build()

    def timed(fn, cnt):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(cnt)]
        for a, b in ev:
            a.record(st)
            fn()
            b.record(st)
        torch.cuda.synchronize()
        return [a.elapsed_time(b) * 1e3 for a, b in ev]  # us

    for k, m in codes:
        for n in (256, 1024, 4096, 8192, 16384, 32768, 65536):
            e = m
            s, l = ec.erasures(0x6D656D6F, 0, n, k, m, e)
            sd, ld = torch.from_numpy(s).cuda(), torch.from_numpy(l).cuda()
            rows = {w: torch.zeros((n, e * k), dtype=torch.uint8, device="cuda") for w in ("wide", "lane")}
            times = {"wide": [], "lane": []}
            for cyc in range(12):
                for w in (("wide", "lane") if cyc % 2 == 0 else ("lane", "wide")):
                    with c.options(decode_wide_max=(1 << 40) if w == "wide" else 0):
                        times[w] += timed(lambda: c.decode_rows(k, m, sd, ld, rows[w]), 5)
            c.synchronize()
            row = {"k": k, "m": m, "n": n, "e": e,
                   "wide_us": round(float(np.median(times["wide"])), 2),
                   "lane_us": round(float(np.median(times["lane"])), 2),
                   "equal": bool(torch.equal(rows["wide"], rows["lane"]))}
            print(json.dumps(row), flush=True)
    c.close()


if __name__ == "__main__":
    main()
