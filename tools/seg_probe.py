"""C5 mixed-call probe: bench.py's 12 groups ((4,2)/(10,4)/(16,4) x 4 KiB /
64 KiB / 1 MiB / 4 MiB, ~gib GiB of payload) as one encode_segments and one
rebuild_segments call, timed with HIP events (run under rocprofv3
--kernel-trace for the launches inside each call).  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from memo_amd import ec  # noqa: E402

if len(sys.argv) > 3:  # another build of the library (an A/B's other side)
    ec.LIB_PATH = sys.argv[3]

SEED = 0x6D656D6F
# untimed calls before each timed series; ~150 settle the clocks (the ramp
# after a load step: profiles/HISTORY.md "Clock ramp")
WARMUP = int(os.environ.get("SEG_PROBE_WARMUP", "5"))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    gib = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
    with ec.Codec(0) as c:
        st = torch.cuda.Stream()
        c.set_stream(st.cuda_stream)
        segs, rsegs, checks, alg, ralg = [], [], [], 0, 0
        for gi, (k, m) in enumerate([(4, 2), (10, 4), (16, 4)]):
            for B in [4 << 10, 64 << 10, 1 << 20, 4 << 20]:
                S = ec.shard_size(B, k)
                n = max(1, int(gib * 2**30 / 12) // B)
                d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
                p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
                c.fill_blocks(SEED, 0, n, B, k, S, d)
                c.encode(k, m, d, p)
                s, l = ec.erasures(SEED, gi, n, k, m, m)
                sd, ld = torch.from_numpy(s).cuda(), torch.from_numpy(l).cuda()
                surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
                c.gather_shards(k, m, S, n, d, p, sd, surv)
                want = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
                c.gather_shards(k, m, S, n, d, p, ld, want)
                out = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
                segs.append((k, m, S, n, d, p))
                rsegs.append(dict(k=k, m=m, surv_idx=sd, surv=surv, lost_idx=ld, out=out))
                checks.append((out, want))
                alg += (k + m) * S * n
                ralg += (k + m) * S * n
        for rep in range(2):
            res = {"rep": rep}
            for name, fn, nbytes in [("encode", lambda: c.encode_segments(segs), alg),
                                     ("rebuild", lambda: c.rebuild_segments(rsegs), ralg)]:
                for _ in range(WARMUP):
                    fn()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
                ev[0].record(st)
                for i in range(steps):
                    fn()
                    ev[i + 1].record(st)
                c.synchronize()
                ms = float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]))
                res[name] = {"ms": round(ms, 4), "frac": round(nbytes / (ms * 1e-3) / 8e12, 4)}
            res["rebuild"]["bit_exact"] = all(bool(torch.equal(o, w)) for o, w in checks)
            for o, _ in checks:
                o.zero_()
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
