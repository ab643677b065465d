"""Latency floor of a one-block host call on this box: a 1-element torch
kernel + stream synchronize (launch + completion round trip), against
libmemo_ec's one-block RS(10,4) encode / 1-erasure rebuild from pageable and
from pinned host memory (median of 400 calls each).  One JSON line.
  python tools/latency_floor.py"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from memo_amd import ec  # noqa: E402


def med_us(fn, reps=400):
    for _ in range(20):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return round(float(np.median(t)) * 1e6, 1)


def main():
    x = torch.zeros(1, device="cuda")
    res = {"torch_1elem_kernel_sync_us": med_us(lambda: (x.add_(1), torch.cuda.synchronize()))}
    c = ec.Codec(0)
    k, m = 10, 4
    for B in (4096, 1 << 20):
        S = ec.shard_size(B, k)
        d = np.random.default_rng(1).integers(0, 256, size=(1, k * S), dtype=np.uint8)
        p = np.empty((1, m * S), dtype=np.uint8)
        res["encode_%d_pageable_us" % B] = med_us(lambda: c.encode(k, m, d, p))
        dp = torch.from_numpy(d).pin_memory()
        pp = torch.empty((1, m * S), dtype=torch.uint8).pin_memory()
        res["encode_%d_pinned_us" % B] = med_us(lambda: c.encode(k, m, dp, pp))
    print(json.dumps(res), flush=True)
    c.close()


if __name__ == "__main__":
    main()
