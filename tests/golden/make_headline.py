"""Generate tests/golden/rs_headline.json: SHA-256 digests of the independent
numpy restatement's (oracle/rs_numpy.py) parity and rebuilt shards for
sample blocks of BASELINE.json's headline batches, at their full shapes:

  C2/C3  RS(10,4), 4096 x 1 MiB, rebuild with 4 random erasures per block
  C1     RS(3,2), 1000 x 64 KiB, rebuild with 1 and with 2 erasures
  4 KiB  RS(16,4) and RS(10,4), 1,048,576 blocks (bench.py rebuild_small)
  4 MiB  RS(4,2), 1024 blocks (the largest C5 block size)

Each sample is one block of the batch (first, an interior one, last), its
synthetic bytes (digest of the data, to pin the fill), its erasure pattern
(memo_ec_erasures / rs_numpy.erasures of that block index), and the digests
of its m parity shards and its e rebuilt shards.  tests/test_gpu_parity.py
runs each batch whole on the GPU and checks the samples' digests, so the HIP
output is compared with the restatement that shares no code with the C
oracle, at the sizes the bench measures.  Deterministic; re-run with
`python tests/golden/make_headline.py` (about a minute).
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import rs_numpy as N  # noqa: E402

SEED = 0x6D656D6F
# name, k, m, B, blocks in the batch, erasure counts, sample block indices
BATCHES = [
    ("C2_C3", 10, 4, 1 << 20, 4096, [4], [0, 2049, 4095]),
    ("C1", 3, 2, 65536, 1000, [1, 2], [0, 500, 999]),
    ("small_16_4", 16, 4, 4096, 1 << 20, [4], [0, 777777, (1 << 20) - 1]),
    ("small_10_4", 10, 4, 4096, 1 << 20, [4], [0, 123457, (1 << 20) - 1]),
    ("C5_4MiB_4_2", 4, 2, 4 << 20, 1024, [2], [0, 1023]),
]


def sha(x):
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def main():
    out = {"seed": SEED, "source": "oracle/rs_numpy.py (independent restatement)", "batches": []}
    for name, k, m, B, n, es, picks in BATCHES:
        S = N.shard_size(B, k)
        C = N.cauchy(k, m)
        samples = []
        for b in picks:
            data = N.fill_block(SEED, b, B, k, S)
            par = N.encode(k, m, S, data[None])[0]
            shards = np.concatenate([data, par]).reshape(k + m, S)
            smp = {"block": b, "data_sha256": sha(data), "parity_sha256": sha(par), "rebuild": []}
            for e in es:
                surv, lost = N.erasures(SEED, b, k, m, e)
                rows = N.decode_matrix(k, m, surv, lost)
                rebuilt = N.mac(rows, shards[surv])
                assert np.array_equal(rebuilt, shards[lost]), (name, b, e)  # round trip
                smp["rebuild"].append({"e": e, "surv": [int(x) for x in surv],
                                       "lost": [int(x) for x in lost],
                                       "out_sha256": sha(rebuilt)})
            samples.append(smp)
        out["batches"].append({"name": name, "k": k, "m": m, "block_bytes": B, "blocks": n,
                               "shard_bytes": S, "erasures": es, "samples": samples})
        print(name, "done", flush=True)
    with open(os.path.join(HERE, "rs_headline.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
