#!/usr/bin/env python3
"""Interleaved A/B of the rows-path rebuild MAC: tables built in LDS per tile
(image_min_tiles 0) against per-block table images through HBM + the encode
body (image_min_tiles 1), beside the encode of the same blocks, per shape.
The variants alternate in groups of two launches (rotating order), and every
fifth group's output is compared with the original shards it rebuilds.
Prints one JSON line per shape: median launch times.
  usage: image_ab.py [rounds] [launches] [shape ...]   shape = k,m,B[,MiB] (payload,
  default 4 GiB); rounds x launches launches per variant; AB_FUSED=1 adds the
  fused gf_rebuild_kernel as a fourth variant"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = ["16,4,4096", "16,4,16384", "16,4,65536", "16,4,262144", "16,4,1048576", "16,4,4194304",
          "10,4,4096", "10,4,65536", "10,4,262144", "10,4,1048576", "10,4,4194304",
          "4,2,65536", "4,2,1048576"]


def main():
    import torch
    from memo_amd import ec
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    shapes = sys.argv[3:] or SHAPES
    seed = 0x6D656D6F
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    c = ec.Codec(0)
    c.set_stream(st)
    ec.check_build()

    def timed(fn, cnt):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(cnt)]
        for a, b in ev:
            a.record(st)
            fn()
            b.record(st)
        torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b in ev]

    for shape in shapes:
        f = [int(x) for x in shape.split(",")]
        k, m, B = f[:3]
        mib = f[3] if len(f) > 3 else 4096  # payload per shape
        e = m
        S = ec.shard_size(B, k)
        n = max(1, (mib << 20) // B)
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
        del d
        out = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.15:  # settle the clocks
            c.encode(k, m, surv, p)
            torch.cuda.synchronize()
        alg_enc = (k + m) * S * n
        alg_reb = (k + e) * S * n
        # variants alternate in groups of 2 launches, the order rotating per
        # cycle, so clock and power drift fall on every variant alike
        variants = [("encode", None), ("lds", 0), ("images", 1)]
        if os.environ.get("AB_FUSED"):
            variants.append(("fused", -1))
        times = {v: [] for v, _ in variants}
        ok = {"lds": True, "images": True, "fused": True}
        for cyc in range(rounds * launches // 2):
            rot = cyc % len(variants)
            for name, img in variants[rot:] + variants[:rot]:
                if img is None:
                    times[name] += timed(lambda: c.encode(k, m, surv, p), 2)
                    continue
                opts = dict(rebuild_path=1) if img < 0 else dict(rebuild_path=0, image_min_tiles=img,
                                                                  image_min_coefs=0)
                with c.options(**opts):
                    times[name] += timed(lambda: c.rebuild(k, m, sd, surv, ld, out), 2)
                    if cyc % 5 == 0:
                        c.synchronize()
                        ok[name] &= bool(torch.equal(out, want))
                        out.fill_(0)
        row = {"k": k, "m": m, "B": B, "n": n, "S": S, "tiles_per_block": -(-S // 4096),
               "launches": len(times["encode"])}
        for name, _ in variants:
            med = float(np.median(times[name]))
            alg = alg_enc if name == "encode" else alg_reb
            row[name + "_ms"] = round(med, 4)
            row[name + "_pct"] = round(100 * alg / (med * 1e-3) / 8e12, 2)
            if name in ok:
                row[name + "_ok"] = ok[name]
        print(json.dumps(row), flush=True)
        del surv, want, out, p, sd, ld
        torch.cuda.empty_cache()
    c.close()


if __name__ == "__main__":
    main()
