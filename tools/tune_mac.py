"""Interleaved A/B timing of MAC-kernel variants (tools/build_variants.sh)
on the C2 encode / C3 rebuild workloads, in ONE process (rule: perf deltas
from interleaved rounds).  Usage:
  python tools/tune_mac.py lib_a.so lib_b.so ... [--wg 4,8,16] [--rounds 5]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEED = 0x6D656D6F


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.memo_ec_ctx_create.argtypes = [ci, ctypes.POINTER(vp)]
    L.memo_ec_set_stream.argtypes = [vp, vp]
    L.memo_ec_encode_batch.argtypes = [vp, ci, ci, sz, sz, vp, vp, ci]
    L.memo_ec_rebuild_batch.argtypes = [vp, ci, ci, sz, sz, vp, vp, vp, ci, vp, ci]
    L.memo_ec_synchronize.argtypes = [vp]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--wg", default="0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--warm", type=int, default=50,
                    help="untimed back-to-back launches before each timed series (clock ramp)")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--B", type=int, default=1 << 20)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--e", type=int, default=4)
    a = ap.parse_args()
    import torch
    from memo_amd import ec
    k, m, B, n, e = a.k, a.m, a.B, a.n, a.e
    S = ec.shard_size(B, k)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    ref = ec.Codec(0)
    ref.set_stream(st)
    data = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    ref.fill_blocks(SEED, 0, n, B, k, S, data)
    want = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    ref.encode(k, m, data, want)
    s, l = ec.erasures(SEED, 0, n, k, m, e)
    sd, ld = torch.from_numpy(s).cuda(), torch.from_numpy(l).cuda()
    surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    ref.gather_shards(k, m, S, n, data, want, sd, surv)
    rwant = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
    ref.gather_shards(k, m, S, n, data, want, ld, rwant)
    par = torch.empty_like(want)
    out = torch.empty_like(rwant)
    torch.cuda.synchronize()

    variants = []
    for path in a.libs:
        L = load(path)
        for w in [int(x) for x in a.wg.split(",")]:
            os.environ["MEMO_EC_WG_PER_CU"] = str(w)
            ctx = ctypes.c_void_p()
            assert L.memo_ec_ctx_create(0, ctypes.byref(ctx)) == 0
            L.memo_ec_set_stream(ctx, st.cuda_stream)
            variants.append((os.path.basename(path) + ":wg%d" % w, L, ctx))
    alg_e = (k + m) * S * n
    alg_r = (k + e) * S * n
    res = {v[0]: {"enc": [], "reb": []} for v in variants}
    for r in range(a.rounds):
        for name, L, ctx in variants:
            for kind in ("enc", "reb"):
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(a.iters)]
                for _ in range(a.warm):
                    if kind == "enc":
                        L.memo_ec_encode_batch(ctx, k, m, S, n, data.data_ptr(), par.data_ptr(), 2)
                    else:
                        L.memo_ec_rebuild_batch(ctx, k, m, S, n, sd.data_ptr(), surv.data_ptr(),
                                                ld.data_ptr(), e, out.data_ptr(), 2)
                for x, y in evs:
                    x.record(st)
                    if kind == "enc":
                        rc = L.memo_ec_encode_batch(ctx, k, m, S, n, data.data_ptr(), par.data_ptr(), 2)
                    else:
                        rc = L.memo_ec_rebuild_batch(ctx, k, m, S, n, sd.data_ptr(), surv.data_ptr(),
                                                     ld.data_ptr(), e, out.data_ptr(), 2)
                    assert rc == 0, rc
                    y.record(st)
                torch.cuda.synchronize()
                res[name][kind].extend(x.elapsed_time(y) for x, y in evs[1:])
            if "diag" not in name:
                assert torch.equal(par, want), name
                assert torch.equal(out, rwant), name
            par.zero_(); out.zero_()
    rows = []
    for name, d in res.items():
        me, mr = statistics.median(d["enc"]), statistics.median(d["reb"])
        rows.append({"variant": name, "enc_ms_med": round(me, 4), "enc_ms_min": round(min(d["enc"]), 4),
                     "enc_TBs": round(alg_e / me / 1e9, 3), "enc_frac": round(alg_e / me / 1e9 / 8.0, 4),
                     "reb_ms_med": round(mr, 4), "reb_TBs": round(alg_r / mr / 1e9, 3),
                     "reb_frac": round(alg_r / mr / 1e9 / 8.0, 4)})
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
