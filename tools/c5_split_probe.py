"""Where the C5 mixed call loses against its parts: bench.py's 12 C5 groups
((4,2)/(10,4)/(16,4) x 4 KiB / 64 KiB / 1 MiB / 4 MiB, ~gib GiB of payload)
timed as one call, as one call per code class, and one call per group, for
encode_segments and rebuild_segments (HIP events, mean of `steps` calls after
5 warm-up calls).  Prints one JSON line per (op, split, part) with its
fraction of 8 TB/s over the algorithmic bytes ((k + m) x S per block)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from memo_amd import ec  # noqa: E402

SEED = 0x6D656D6F


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    gib = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
    with ec.Codec(0) as c:
        st = torch.cuda.Stream()
        c.set_stream(st.cuda_stream)
        groups = []
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
                out = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
                groups.append(dict(k=k, m=m, B=B, nbytes=(k + m) * S * n, enc=(k, m, S, n, d, p),
                                   reb=dict(k=k, m=m, surv_idx=sd, surv=surv, lost_idx=ld, out=out)))

        def timed(fn):
            for _ in range(5):
                fn()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
            ev[0].record(st)
            for i in range(steps):
                fn()
                ev[i + 1].record(st)
            c.synchronize()
            return float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]))

        if "--alt" in sys.argv:
            alt_probe(c, st, groups, timed)
            return
        splits = {"one_call": [groups],
                  "per_class": [groups[i:i + 4] for i in range(0, 12, 4)],
                  "per_group": [[g] for g in groups]}
        for op in ("encode", "rebuild"):
            for name, parts in splits.items():
                total = 0.0
                for part in parts:
                    if op == "encode":
                        ms = timed(lambda: c.encode_segments([g["enc"] for g in part]))
                    else:
                        ms = timed(lambda: c.rebuild_segments([g["reb"] for g in part]))
                    nb = sum(g["nbytes"] for g in part)
                    total += ms
                    tag = "all" if len(part) == 12 else ",".join(f"{g['k']}.{g['m']}.{g['B'] >> 10}K" for g in part)
                    print(json.dumps({"op": op, "split": name, "part": tag, "ms": round(ms, 4),
                                      "frac": round(nb / (ms * 1e-3) / 8e12, 4)}), flush=True)
                nb = sum(g["nbytes"] for g in groups)
                print(json.dumps({"op": op, "split": name, "part": "sum", "ms": round(total, 4),
                                  "frac": round(nb / (total * 1e-3) / 8e12, 4)}), flush=True)


def alt_probe(c, st, groups, timed):
    """Is a launch class slower after another class's launch than after its
    own?  seq_calls: the three classes as three calls per step; same: the
    (10,4) class twice on the same buffers; alt: on two buffer sets in
    turn (same shapes, separate allocations)."""
    import torch
    cls = [groups[i:i + 4] for i in range(0, 12, 4)]
    twin = []
    for g in cls[1]:
        k, m, S, n, d, p = g["enc"]
        twin.append(dict(g, enc=(k, m, S, n, d.clone(), torch.empty_like(p))))
    nb10 = sum(g["nbytes"] for g in cls[1])
    runs = {
        "seq_calls": (lambda: [c.encode_segments([g["enc"] for g in part]) for part in cls],
                      sum(g["nbytes"] for g in groups), 3),
        "same_10_4": (lambda: [c.encode_segments([g["enc"] for g in cls[1]]) for _ in range(2)], nb10 * 2, 2),
        "alt_10_4": (lambda: [c.encode_segments([g["enc"] for g in x]) for x in (cls[1], twin)], nb10 * 2, 2),
        "one_call": (lambda: c.encode_segments([g["enc"] for g in groups]), sum(g["nbytes"] for g in groups), 1),
        "reverse": (lambda: c.encode_segments([g["enc"] for g in groups[::-1]]), sum(g["nbytes"] for g in groups), 1),
    }
    for name, (fn, nb, calls) in runs.items():
        ms = timed(fn)
        print(json.dumps({"op": "encode", "run": name, "calls": calls, "ms": round(ms, 4),
                          "frac": round(nb / (ms * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
