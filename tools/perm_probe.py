#!/usr/bin/env python3
"""The per-code pattern-table probe of VERDICT r05 item 4, on the
MEMO_EC_PERM_PROBE build of the library (memo_amd/_lib/probe/, `make -C
memo_amd/csrc probe`): 1,048,576 blocks, e = m random lost shards per block
(survivors and lost shards in ascending order), three variants alternating
in groups of two launches, HIP events on one stream:
  rows    the product rebuild: decode rows (decode_rows_k_kernel) + the rows
          MAC, which builds each tile's product tables in LDS from the rows;
  perm    the MAC alone, each block's product images copied from a table of
          every erasure pattern's images (C(k+m, m) patterns x R x k slots x
          20 B, L2/MALL-resident) at the block's pattern rank -- no decode
          launch, no per-tile build (the ranks are precomputed on the host:
          the probe's time leaves out a rank kernel);
  encode  the encode of the same blocks (the ceiling).
The perm output is compared with the product rebuild's and with the original
shards.  Prints one JSON line per code.
  usage: perm_probe.py [rounds] [launches] [code ...]   code = k,m[,B] (4096)"""
import json
import os
import sys
import time
from itertools import combinations
from math import comb

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def images(coefs):
    """Product-table images (q: 4 dwords, lo: 1 dword) of coefficient bytes,
    the layout ec_kernels.hip's coef_image writes: lo = c*{0,1,2,3},
    q = [c*{0..3}<<2, c*{4..7}<<2, c*{0..3}<<5, c*{4..7}<<5]."""
    c = coefs.astype(np.uint32)
    d = [c]
    for _ in range(7):
        x = d[-1]
        d.append(((x << 1) ^ ((x >> 7) * 0x11D)) & 0xFF)

    def pack(a, b, cc, dd):
        return (a | (b << 8) | (cc << 16) | (dd << 24)).astype(np.uint32)

    z = np.zeros_like(c)
    d0, d1, d2, d3, d4, d5, d6, d7 = d
    q = np.stack([pack(z, d2, d3, d2 ^ d3), pack(d4, d4 ^ d2, d4 ^ d3, d4 ^ d3 ^ d2),
                  pack(z, d5, d6, d5 ^ d6), pack(d7, d7 ^ d5, d7 ^ d6, d7 ^ d6 ^ d5)], axis=-1)
    lo = pack(z, d0, d1, d0 ^ d1)
    return q, lo


def rank_of(lost):
    """Combinatorial rank of each row's ascending lost set (colex order)."""
    r = np.zeros(lost.shape[0], dtype=np.int64)
    for i in range(lost.shape[1]):
        li = lost[:, i].astype(np.int64)
        r += np.array([comb(int(v), i + 1) for v in range(lost.max() + 1)], dtype=np.int64)[li]
    return r


def main():
    import ctypes

    import torch
    from memo_amd import ec
    ec.LIB_PATH = os.path.join(ROOT, "memo_amd", "_lib", "probe", "libmemo_ec.so")
    lib = ec._lib()
    lib.memo_ec_probe_perm_mac.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                           ctypes.c_size_t] + [ctypes.c_void_p] * 5
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    codes = sys.argv[3:] or ["16,4", "10,4"]
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    c = ec.Codec(0)
    c.set_stream(st)
    rng = np.random.default_rng(0x6D656D6F)
    for code in codes:
        f = [int(x) for x in code.split(",")]
        k, m = f[:2]
        B = f[2] if len(f) > 2 else 4096
        e, n = m, 1 << 20
        S = ec.shard_size(B, k)
        d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
        c.fill_blocks(0x6D656D6F, 0, n, B, k, S, d)
        c.encode(k, m, d, p)
        # ascending lost sets, survivors their ascending complement
        keys = rng.random((n, k + m))
        lost = np.sort(np.argsort(keys, axis=1)[:, :e], axis=1).astype(np.uint8)
        mask = np.ones((n, k + m), dtype=bool)
        mask[np.arange(n)[:, None], lost] = False
        surv = np.nonzero(mask)[1].reshape(n, k).astype(np.uint8)
        sd, ld = torch.from_numpy(surv).cuda(), torch.from_numpy(lost).cuda()
        sv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        c.gather_shards(k, m, S, n, d, p, sd, sv)
        want = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        c.gather_shards(k, m, S, n, d, p, ld, want)
        # every pattern, in rank order (colex), its decode rows and images
        pats = np.array(sorted(combinations(range(k + m), e), key=lambda s: sum(comb(v, i + 1) for i, v in enumerate(s))),
                        dtype=np.uint8)
        assert (rank_of(pats) == np.arange(len(pats))).all()
        pm = np.ones((len(pats), k + m), dtype=bool)
        pm[np.arange(len(pats))[:, None], pats] = False
        psurv = np.nonzero(pm)[1].reshape(len(pats), k).astype(np.uint8)
        rows = torch.empty((len(pats), e * k), dtype=torch.uint8, device="cuda")
        c.decode_rows(k, m, torch.from_numpy(psurv).cuda(), torch.from_numpy(pats).cuda(), rows)
        c.synchronize()
        q, lo = images(rows.cpu().numpy())                     # slot = row * k + column
        qtab = torch.from_numpy(np.ascontiguousarray(q).reshape(-1)).cuda()
        lotab = torch.from_numpy(np.ascontiguousarray(lo).reshape(-1)).cuda()
        prank = torch.from_numpy(rank_of(lost).astype(np.uint16)).cuda()
        out_rows = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        out_perm = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")

        def perm():
            rc = lib.memo_ec_probe_perm_mac(c._ctx, k, m, S, n, sv.data_ptr(), out_perm.data_ptr(),
                                            prank.data_ptr(), qtab.data_ptr(), lotab.data_ptr())
            if rc:
                raise RuntimeError("probe_perm_mac: %d" % rc)

        variants = {"rows": lambda: c.rebuild(k, m, sd, sv, ld, out_rows), "perm": perm,
                    "encode": lambda: c.encode(k, m, d, p)}
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:  # settle the clocks
            for fn in variants.values():
                fn()
            torch.cuda.synchronize()
        times = {v: [] for v in variants}
        names = list(variants)
        for r in range(rounds * launches // 2):
            order = names[r % 3:] + names[:r % 3]
            for v in order:
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(2)]
                for a, b in ev:
                    a.record(st)
                    variants[v]()
                    b.record(st)
                torch.cuda.synchronize()
                times[v] += [a.elapsed_time(b) for a, b in ev]
        c.synchronize()
        alg = (k + e) * S * n
        res = {"code": "RS(%d,%d)" % (k, m), "B": B, "blocks": n, "patterns": len(pats),
               "table_bytes": int(qtab.numel() * 4 + lotab.numel() * 4)}
        for v, ts in times.items():
            ms = float(np.median(ts))
            a = (k + m) * S * n if v == "encode" else alg
            res[v] = {"ms": round(ms, 4), "frac": round(a / (ms * 1e-3) / 8e12, 4), "n": len(ts)}
        res["perm_bit_exact_vs_rows"] = bool(torch.equal(out_perm, out_rows))
        res["perm_bit_exact_vs_shards"] = bool(torch.equal(out_perm, want))
        res["rows_bit_exact_vs_shards"] = bool(torch.equal(out_rows, want))
        res["path"] = c.rebuild_path(n, k, S)
        print(json.dumps(res), flush=True)
        del d, p, sv, want, out_rows, out_perm, qtab, lotab, prank, rows
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
