"""Host-memory call latency: zero-copy (kernels on pinned host memory) vs the
DMA pipeline, by call size.  Run on the GPU box:  python tools/zc_probe.py
One JSON line per (kind, blocks)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from memo_amd import ec
    k, m, B = 10, 4, 1 << 20
    S = ec.shard_size(B, k)
    c = ec.Codec(0)
    rng = np.random.default_rng(3)
    for n in (1, 2, 4, 8, 16, 32, 60):
        d = np.frombuffer(rng.bytes(n * k * S), np.uint8).reshape(n, -1).copy()
        p = np.zeros((n, m * S), np.uint8)
        s = np.tile(np.arange(1, k + 1, dtype=np.uint8), (n, 1))
        l = np.zeros((n, 1), np.uint8)
        o = np.zeros((n, S), np.uint8)
        row = {"blocks": n, "MiB_in": round(n * k * S / 2**20, 2)}
        for zc in ("1000000", "0"):
            os.environ["MEMO_EC_ZC_KB"] = zc
            for name, fn in (("encode", lambda: c.encode(k, m, d, p)),
                             ("rebuild_e1", lambda: c.rebuild(k, m, s, d, l, o))):
                for _ in range(5):
                    fn()
                ts = []
                for _ in range(30):
                    t = time.perf_counter()
                    fn()
                    ts.append(time.perf_counter() - t)
                row["%s_%s_us" % (name, "zc" if zc != "0" else "dma")] = round(float(np.median(ts)) * 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
