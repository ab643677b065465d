"""Interleaved A/B of host-memory encode throughput (pageable and pinned
numpy buffers, RS(10,4), 1024 x 1 MiB) between libmemo_ec builds, in one
process.  Usage: python tools/e2e_ab.py lib_a.so lib_b.so [--rounds 4]"""
import argparse
import ctypes
import json
import os
import statistics
import time

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    import torch  # pinned host buffers
    k, m, B, n = 10, 4, 1 << 20, 1024
    S = ((B + k - 1) // k + 63) // 64 * 64
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, size=n * k * S, dtype=np.uint8)
    par = np.zeros(n * m * S, dtype=np.uint8)
    pdata = torch.from_numpy(data).pin_memory()
    ppar = torch.zeros(n * m * S, dtype=torch.uint8).pin_memory()
    libs = []
    for p in a.libs:
        L = ctypes.CDLL(os.path.abspath(p))
        vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.memo_ec_ctx_create.argtypes = [ci, ctypes.POINTER(vp)]
        L.memo_ec_encode_batch.argtypes = [vp, ci, ci, sz, sz, vp, vp, ci]
        ctx = vp()
        assert L.memo_ec_ctx_create(0, ctypes.byref(ctx)) == 0
        libs.append((os.path.basename(p), L, ctx))
    res = {}
    for _ in range(a.rounds):
        for name, L, ctx in libs:
            for kind, d, p, where in (("pageable", data.ctypes.data, par.ctypes.data, 0),
                                      ("pinned", pdata.data_ptr(), ppar.data_ptr(), 1)):
                L.memo_ec_encode_batch(ctx, k, m, S, n, d, p, where)
                for _ in range(3):
                    t = time.perf_counter()
                    assert L.memo_ec_encode_batch(ctx, k, m, S, n, d, p, where) == 0
                    res.setdefault((name, kind), []).append(n * B / (time.perf_counter() - t) / 2**30)
    for (name, kind), v in res.items():
        print(json.dumps({"lib": name, "path": kind, "GiBs_median": round(statistics.median(v), 2),
                          "GiBs_max": round(max(v), 2)}))


if __name__ == "__main__":
    main()
