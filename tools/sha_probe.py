"""sha256_kernel on n x B device-resident blocks with a 64-byte prefix (the
CHB address hash), settled clocks, HIP-event timing; one JSON line.  Used
under rocprofv3 for the kernel's counters (tools/pmc_sha.sh).
  python tools/sha_probe.py [--n 1048576] [--B 4096] [--reps 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from memo_amd import ec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    c = ec.Codec(0)
    st = torch.cuda.Stream()
    c.set_stream(st)
    msg = torch.empty((a.n, a.B), dtype=torch.uint8, device="cuda")
    c.fill_blocks(0x6D656D6F, 0, a.n, a.B, 1, a.B, msg)
    pre = torch.zeros((a.n, 64), dtype=torch.uint8, device="cuda")
    dig = torch.empty((a.n, 32), dtype=torch.uint8, device="cuda")
    with torch.cuda.stream(st):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.15:
            c.sha256(msg, dig, prefix=pre)
            st.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e0, e1 in ev:
            e0.record(st)
            c.sha256(msg, dig, prefix=pre)
            e1.record(st)
        st.synchronize()
    ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
    import hashlib
    ok = dig[0].cpu().numpy().tobytes() == hashlib.sha256(bytes(64) + msg[0].cpu().numpy().tobytes()).digest()
    print(json.dumps({"n": a.n, "B": a.B, "kernel_ms": round(ms, 4),
                      "GBs": round(a.n * (a.B + 64) / ms / 1e6, 1), "bit_exact_first": ok}), flush=True)
    c.close()


if __name__ == "__main__":
    main()
