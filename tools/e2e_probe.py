"""PCIe end-to-end probe: pinned HtoD / DtoH copy rates and the codec's host
pipeline (MEMO_EC_HOST_PINNED / MEMO_EC_HOST) for several batch sizes."""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from memo_amd import ec
    nbytes = 1 << 30
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for name, f in [("HtoD", lambda: d.copy_(h, non_blocking=True)),
                    ("DtoH", lambda: h.copy_(d, non_blocking=True))]:
        f(); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        print(json.dumps({"copy": name, "GBs": round(5 * nbytes / (time.perf_counter() - t) / 1e9, 2)}))
    del h, d
    k, m, B, n = 10, 4, 1 << 20, 1024
    S = ec.shard_size(B, k)
    hd = torch.empty((n, k * S), dtype=torch.uint8).pin_memory()
    hp = torch.empty((n, m * S), dtype=torch.uint8).pin_memory()
    for mb in [16, 32, 64, 128, 256]:
        os.environ["MEMO_EC_PIPE_MB"] = str(mb)
        with ec.Codec(0) as c:
            c.encode(k, m, hd, hp)
            t = time.perf_counter()
            for _ in range(3):
                c.encode(k, m, hd, hp)
            el = time.perf_counter() - t
            pin = 3 * n * B / el / 2**30
            nd = np.ones((n, k * S), dtype=np.uint8)  # pageable, pre-faulted
            npar = np.ones((n, m * S), dtype=np.uint8)
            c.encode(k, m, nd, npar)
            t = time.perf_counter()
            for _ in range(3):
                c.encode(k, m, nd, npar)
            page = 3 * n * B / (time.perf_counter() - t) / 2**30
        print(json.dumps({"pipe_mb": mb, "pinned_GiBs": round(pin, 2), "pageable_GiBs": round(page, 2)}))


if __name__ == "__main__":
    main()
