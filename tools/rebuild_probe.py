#!/usr/bin/env python3
"""Encode and rebuild of one shape, back to back, for rocprofv3 passes
(tools/pmc_rebuild.sh): `launches` encode launches, then `launches`
rebuild launches with `e` random erasures per block, after a clock-settling
burst.  The rebuild path follows MEMO_EC_REBUILD_FUSED (1: gf_rebuild_kernel,
0: decode_coef_kernel + gf_mac_kernel), so the kernels are told apart by name.
Prints one JSON line with HIP-event times.
  usage: rebuild_probe.py k m block_bytes blocks [e] [launches]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from memo_amd import ec
    if os.environ.get("MEMO_EC_PROBE_LIB"):  # another build of the library (an A/B's other side)
        ec.LIB_PATH = os.environ["MEMO_EC_PROBE_LIB"]
    k, m, B, n = (int(x) for x in sys.argv[1:5])
    e = int(sys.argv[5]) if len(sys.argv) > 5 else m
    launches = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    seed = 0x6D656D6F
    S = ec.shard_size(B, k)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    c = ec.Codec(0)
    c.set_stream(st)
    d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    c.fill_blocks(seed, 0, n, B, k, S, d)
    c.encode(k, m, d, p)
    s, l = ec.erasures(seed, 0, n, k, m, e)
    sd, ld = torch.from_numpy(s).cuda(), torch.from_numpy(l).cuda()
    surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    c.gather_shards(k, m, S, n, d, p, sd, surv)
    want = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
    c.gather_shards(k, m, S, n, d, p, ld, want)
    out = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:  # settle the clocks
        c.encode(k, m, d, p)
        c.rebuild(k, m, sd, surv, ld, out)
        torch.cuda.synchronize()
    res = {"k": k, "m": m, "B": B, "n": n, "e": e, "S": S, "path": c.rebuild_path(n, k, S)}
    for name, fn, alg in (("encode", lambda: c.encode(k, m, d, p), (k + m) * S * n),
                          ("rebuild", lambda: c.rebuild(k, m, sd, surv, ld, out), (k + e) * S * n)):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(launches)]
        for a, b in ev:
            a.record(st)
            fn()
            b.record(st)
        torch.cuda.synchronize()
        ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        res[name] = {"ms": round(ms, 4), "frac": round(alg / (ms * 1e-3) / 8e12, 4)}
    c.synchronize()
    res["bit_exact"] = bool(torch.equal(out, want))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
