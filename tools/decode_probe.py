"""Cost split of the batched GF(2^8) inversion (decode rows) for C3's
shape: RS(10,4), 4 random erasures per block, 4096 blocks.  Times
memo_ec_decode_rows (rows only) and a rebuild with 64-byte shards (decode +
table images + a negligible MAC).  Run on the GPU box:
  python tools/decode_probe.py [--lib path/to/variant.so]
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
    ap.add_argument("--n", type=int, default=4096)
    a = ap.parse_args()
    import torch
    from memo_amd import ec
    if a.lib:
        ec.LIB_PATH = os.path.abspath(a.lib)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    c = ec.Codec(0)
    c.set_stream(st)
    out = {"lib": os.path.basename(ec.LIB_PATH)}
    for (k, m, e) in [(10, 4, 4), (10, 4, 1), (16, 4, 4), (4, 2, 2)]:
        n, S = a.n, 64
        s, l = ec.erasures(0x6D656D6F, 0, n, k, m, e)
        sd, ld = torch.from_numpy(s).cuda(), torch.from_numpy(l).cuda()
        rows = torch.empty((n, e * k), dtype=torch.uint8, device="cuda")
        surv = torch.zeros((n, k * S), dtype=torch.uint8, device="cuda")
        o = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")

        def timed(fn, warm=50, iters=50):
            for _ in range(warm):
                fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(iters)]
            for x, y in ev:
                x.record(st)
                fn()
                y.record(st)
            torch.cuda.synchronize()
            return round(float(np.median([x.elapsed_time(y) for x, y in ev])) * 1e3, 1)

        out["rs%d_%d_e%d" % (k, m, e)] = {
            "decode_rows_us": timed(lambda: c.decode_rows(k, m, sd, ld, rows)),
            "rebuild_S64_us": timed(lambda: c.rebuild(k, m, sd, surv, ld, o))}
    c.synchronize()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
