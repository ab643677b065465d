"""Write-side rate of the encode's parity traffic by buffer placement: the
stream probe's write-only and copy modes (memo_ec_stream_probe) on the C2
shape, the parity buffer at several byte offsets inside one allocation and
in several separate allocations, rounds interleaved.  One JSON line per
(placement, round).
  python tools/write_probe.py [--rounds 3]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from memo_amd import ec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    k, m, B, n = 10, 4, 1 << 20, 4096
    S = ec.shard_size(B, k)
    c = ec.Codec(0)
    st = torch.cuda.Stream()
    c.set_stream(st)
    data = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    c.fill_blocks(0x6D656D6F, 0, n, B, k, S, data)
    big = torch.empty(n * m * S + (8 << 20), dtype=torch.uint8, device="cuda")
    places = {}
    for off in (0, 4096, 65536, 1 << 20, 2 << 20, 4 << 20):
        places["offset_%d" % off] = big[off:off + n * m * S].view(n, m * S)
    for j in range(4):
        places["alloc_%d" % j] = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    for p in places.values():
        p.zero_()
    torch.cuda.synchronize()

    def timed(fn, reps=10):
        with torch.cuda.stream(st):
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.1:
                fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for e0, e1 in ev:
                e0.record(st)
                fn()
                e1.record(st)
            st.synchronize()
        return float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))

    for r in range(a.rounds):
        for name, p in places.items():
            w = timed(lambda: c.stream_probe(k, m, data, p, mode="write"))
            cp = timed(lambda: c.stream_probe(k, m, data, p, mode="copy"))
            en = timed(lambda: c.encode(k, m, data, p))
            print(json.dumps({"round": r, "placement": name, "addr_mod_2MiB": p.data_ptr() % (2 << 20),
                              "write_ms": round(w, 4), "copy_ms": round(cp, 4), "encode_ms": round(en, 4),
                              "encode_frac": round(n * (k + m) * S / en / 8e9, 4)}), flush=True)
    c.close()


if __name__ == "__main__":
    main()
