"""Can HtoD and DtoH run concurrently on this box (separate streams)?"""
import json
import time

import torch

n = 1 << 30
h1 = torch.empty(n, dtype=torch.uint8).pin_memory()
h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
for rep in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    with torch.cuda.stream(s1):
        for _ in range(4):
            d1.copy_(h1, non_blocking=True)
    with torch.cuda.stream(s2):
        for _ in range(4):
            h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(json.dumps({"duplex_total_GBs": round(8 * n / el / 1e9, 2), "per_dir_GBs": round(4 * n / el / 1e9, 2)}))
# chunked: many 64 MiB copies alternating streams
c = 64 << 20
torch.cuda.synchronize()
t = time.perf_counter()
for i in range(0, n, c):
    with torch.cuda.stream(s1):
        d1[i:i + c].copy_(h1[i:i + c], non_blocking=True)
    with torch.cuda.stream(s2):
        h2[i:i + c].copy_(d2[i:i + c], non_blocking=True)
torch.cuda.synchronize()
el = time.perf_counter() - t
print(json.dumps({"chunked_duplex_total_GBs": round(2 * n / el / 1e9, 2)}))
