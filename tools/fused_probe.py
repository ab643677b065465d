"""Fused mixed-geometry encode (memo_ec_encode_segments) against the same
segments launched one by one, for one library build.  Run on the GPU box:
  python tools/fused_probe.py [--lib <another libmemo_ec.so build>]
One JSON line.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--scan", action="store_true",
                    help="also time RS(10,4) 1 MiB encode over grid sizes (XCD-order threshold)")
    a = ap.parse_args()
    import torch
    from memo_amd import ec
    if a.lib:
        ec.LIB_PATH = os.path.abspath(a.lib)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    c = ec.Codec(0)
    c.set_stream(st)
    segs, alg = [], 0
    for (k, m) in [(4, 2), (10, 4), (16, 4)]:
        for B in [4 << 10, 64 << 10, 1 << 20, 4 << 20]:
            S = ec.shard_size(B, k)
            n = max(1, int(a.gib * 2**30 / 12) // B)
            d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
            c.fill_blocks(0x6D656D6F, 0, n, B, k, S, d)
            segs.append((k, m, S, n, d, p))
            alg += (k + m) * S * n
    torch.cuda.synchronize()

    def timed(fn, warm=60, iters=12):
        for _ in range(warm):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(iters)]
        for x, y in ev:
            x.record(st)
            fn()
            y.record(st)
        torch.cuda.synchronize()
        return [x.elapsed_time(y) for x, y in ev]

    fused = timed(lambda: c.encode_segments(segs))
    # the same bytes as 12 separate launches per step
    sep = timed(lambda: [c.encode(k, m, d, p) for (k, m, S, n, d, p) in segs])
    # fused with only the (10,4) segments (one KC specialisation)
    only10 = [s for s in segs if s[0] == 10]
    alg10 = sum((k + m) * S * n for (k, m, S, n, d, p) in only10)
    f10 = timed(lambda: c.encode_segments(only10))
    out = {"lib": os.path.basename(ec.LIB_PATH),
           "fused_ms": round(float(np.median(fused)), 4),
           "fused_frac": round(alg / (np.median(fused) * 1e-3) / 8e12, 4),
           "fused_first_last": [round(fused[0], 4), round(fused[-1], 4)],
           "separate_ms": round(float(np.median(sep)), 4),
           "separate_frac": round(alg / (np.median(sep) * 1e-3) / 8e12, 4),
           "fused_10_4_only_frac": round(alg10 / (np.median(f10) * 1e-3) / 8e12, 4)}
    if a.scan:
        k, m, B = 10, 4, 1 << 20
        S = ec.shard_size(B, k)
        for n in (256, 512, 1024, 2048, 4096, 8192):
            d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
            c.fill_blocks(0x6D656D6F, 0, n, B, k, S, d)
            ms = float(np.median(timed(lambda: c.encode(k, m, d, p), warm=max(60, 60 * 4096 // n),
                                       iters=20)))
            out["scan_n%d_tiles%d" % (n, n * S // 16 // 256)] = round((k + m) * S * n / (ms * 1e-3) / 8e12, 4)
            del d, p
    out["xcd_min_tiles"] = os.environ.get("MEMO_EC_XCD_MIN_TILES", "default")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
