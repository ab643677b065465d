"""Encode and rebuild rates over common codes x block sizes (device-resident,
~4 GiB of payload per point, steady clocks).  Run on the GPU box:
  python tools/code_matrix.py > gpurun_out/code_matrix.jsonl
One JSON line per point; every rebuild is checked against the gathered
shards of the same encode."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SEED = 0x6D656D6F


def main():
    import torch
    from memo_amd import ec
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    c = ec.Codec(0)
    c.set_stream(st)

    def timed(fn, warm=40, iters=10):
        for _ in range(warm):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(iters)]
        for a, b in ev:
            a.record(st)
            fn()
            b.record(st)
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    for (k, m) in [(3, 2), (4, 2), (6, 3), (8, 3), (10, 4), (12, 4), (16, 4)]:
        for B in [4096, 65536, 1 << 20]:
            S = ec.shard_size(B, k)
            n = (4 << 30) // B
            e = m
            d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
            c.fill_blocks(SEED, 0, n, B, k, S, d)
            ems = timed(lambda: c.encode(k, m, d, p))
            s, l = ec.erasures(SEED, 0, n, k, m, e)
            sd, ld = torch.from_numpy(s).cuda(), torch.from_numpy(l).cuda()
            surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            c.gather_shards(k, m, S, n, d, p, sd, surv)
            want = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
            c.gather_shards(k, m, S, n, d, p, ld, want)
            del d, p
            out = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
            rms = timed(lambda: c.rebuild(k, m, sd, surv, ld, out))
            c.synchronize()
            ok = bool(torch.equal(out, want))
            print(json.dumps({
                "k": k, "m": m, "block_bytes": B, "blocks": n, "shard_bytes": S,
                "encode_ms": round(ems, 4),
                "encode_frac": round((k + m) * S * n / (ems * 1e-3) / 8e12, 4),
                "rebuild_e": e, "rebuild_ms": round(rms, 4),
                "rebuild_frac": round((k + e) * S * n / (rms * 1e-3) / 8e12, 4),
                "rebuild_bit_exact": ok}), flush=True)
            del surv, want, out, sd, ld
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
