"""One-block host-call latency, A/B of environment knobs read per call, in
one process (interleaved rounds).  Usage on the GPU box:
  python tools/latency_ab.py MEMO_EC_SPIN=0 MEMO_EC_SPIN=1
One JSON line per (setting, call)."""
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from memo_amd import ec
    settings = [a.split("=", 1) for a in sys.argv[1:]]
    k, m = 10, 4
    c = ec.Codec(0)
    res = {}
    for rnd in range(4):
        for name, val in settings:
            os.environ[name] = val
            for B in (4096, 1 << 20):
                S = ec.shard_size(B, k)
                d = np.frombuffer(np.random.default_rng(1).bytes(k * S), np.uint8).reshape(1, -1).copy()
                p = np.zeros((1, m * S), np.uint8)
                s = np.arange(1, k + 1, dtype=np.uint8).reshape(1, k)
                l = np.zeros((1, 1), np.uint8)
                o = np.zeros((1, S), np.uint8)
                for call, fn in (("encode", lambda: c.encode(k, m, d, p)),
                                 ("rebuild_e1", lambda: c.rebuild(k, m, s, d, l, o))):
                    for _ in range(10):
                        fn()
                    for _ in range(100):
                        t = time.perf_counter()
                        fn()
                        res.setdefault((name + "=" + val, call, B), []).append(time.perf_counter() - t)
    for (setting, call, B), ts in res.items():
        print(json.dumps({"setting": setting, "call": call, "block_bytes": B,
                          "median_us": round(statistics.median(ts) * 1e6, 1)}))


if __name__ == "__main__":
    main()
