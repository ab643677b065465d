#!/usr/bin/env python3
# EXPERIMENT ONLY: needs a library built with the MEMO_EC_PERM_TEST hook (not
# kept in memo_amd/csrc; DESIGN.md section 9 has the result).
"""EXPERIMENT (pattern-grouped rebuild feasibility): the uniform-pattern
rebuild of 1M x 4 KiB RS(16,4) blocks with the MAC's blocks taken through a
permutation (MEMO_EC_PERM_TEST=r: random order of runs of r blocks; 0: none),
alternating in one process; outputs must be identical."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from memo_amd import ec
    k, m, B, n, e = 16, 4, 4096, 1 << 20, 4
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
    si = np.array([i for i in range(k + m) if i not in (1, 5, 9, 17)][:k], np.uint8)
    li = np.array([1, 5, 9, 17], np.uint8)
    sd = torch.from_numpy(np.tile(si, (n, 1))).cuda()
    surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    c.gather_shards(k, m, S, n, d, p, sd, surv)
    outs = {}
    alg = (k + e) * S * n
    res = {}
    variants = [int(x) for x in (sys.argv[1:] or ["0", "1", "16"])]
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        c.rebuild_uniform(k, m, si, surv, li, torch.empty((n, e * S), dtype=torch.uint8, device="cuda"))
        torch.cuda.synchronize()
    for rnd in range(3):
        for v in variants:
            os.environ["MEMO_EC_PERM_TEST"] = str(v)
            out = outs.setdefault(v, torch.empty((n, e * S), dtype=torch.uint8, device="cuda"))
            c.rebuild_uniform(k, m, si, surv, li, out)  # perm built outside the timing
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for a, b in ev:
                a.record(st)
                c.rebuild_uniform(k, m, si, surv, li, out)
                b.record(st)
            torch.cuda.synchronize()
            ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
            res.setdefault(str(v), []).append(round(alg / (ms * 1e-3) / 8e12, 4))
    same = all(torch.equal(outs[v], outs[variants[0]]) for v in variants)
    print(json.dumps({"frac": res, "identical": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
