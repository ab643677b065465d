"""Encode and write-only probe rates over a long stretch of back-to-back
launches (C2 shape): every ~0.25 s a sample of 10 encodes and 10 write-only
probes (HIP events), for --seconds.  Shows whether the memory side speeds up
or slows down under sustained load beyond the core clock's ~40 ms ramp.
One JSON line per sample.
  python tools/long_ramp.py [--seconds 20]"""
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
    ap.add_argument("--seconds", type=float, default=20.0)
    a = ap.parse_args()
    k, m, B, n = 10, 4, 1 << 20, 4096
    S = ec.shard_size(B, k)
    c = ec.Codec(0)
    st = torch.cuda.Stream()
    c.set_stream(st)
    data = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    c.fill_blocks(0x6D656D6F, 0, n, B, k, S, data)
    par = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    bytes_enc = n * (k + m) * S
    t_start = time.perf_counter()
    with torch.cuda.stream(st):
        while time.perf_counter() - t_start < a.seconds:
            ev = []
            for fn in (lambda: c.encode(k, m, data, par), lambda: c.stream_probe(k, m, data, par, mode="write")):
                e = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
                for e0, e1 in e:
                    e0.record(st)
                    fn()
                    e1.record(st)
                ev.append(e)
            # filler launches between samples keep the load continuous
            for _ in range(100):
                c.encode(k, m, data, par)
            st.synchronize()
            enc = float(np.median([x.elapsed_time(y) for x, y in ev[0]]))
            wr = float(np.median([x.elapsed_time(y) for x, y in ev[1]]))
            print(json.dumps({"t_s": round(time.perf_counter() - t_start, 2), "encode_ms": round(enc, 4),
                              "encode_frac": round(bytes_enc / enc / 8e9, 4), "write_ms": round(wr, 4)}),
                  flush=True)
    c.close()


if __name__ == "__main__":
    main()
