"""Generate tests/golden/rs_golden.npz from the independent numpy restatement
(oracle/rs_numpy.py).  Committed together with its output; re-run with
`python tests/golden/make_golden.py` (deterministic).

The reference (infinit/memo) has no erasure code, so these vectors are pinned
by (1) the published GF(2^8)/0x11D values of ISO/IEC 18004 (checked in
tests/test_oracle.py) and (2) this restatement's independence from
oracle/rs_oracle.c (carry-less multiply, no log tables).
"""
import hashlib
import itertools
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import rs_numpy as N  # noqa: E402

SEED = 0x6D656D6F
# (k, m, B, first_block, nblocks, e)
ENCODE_CASES = [
    (3, 2, 65536, 0, 2, 2),
    (3, 2, 1000, 5, 3, 1),
    (3, 2, 0, 0, 1, 2),
    (3, 2, 1, 9, 1, 2),
    (4, 2, 4096, 0, 3, 2),
    (4, 2, 4095, 2, 2, 1),
    (10, 4, 5000, 0, 2, 4),
    (10, 4, 1 << 16, 7, 1, 3),
    (16, 4, 4096, 0, 2, 4),
    (16, 4, 16385, 3, 1, 2),
]


def main():
    out = {}
    out["gf_exp"] = np.array([N.gf_pow(2, i) for i in range(255)], dtype=np.uint8)
    for (k, m) in [(3, 2), (4, 2), (10, 4), (16, 4)]:
        out["gen_%d_%d" % (k, m)] = N.cauchy(k, m)
    cases = []
    for ci, (k, m, B, fb, nb, e) in enumerate(ENCODE_CASES):
        S = N.shard_size(B, k)
        data = np.stack([N.fill_block(SEED, fb + i, B, k, S) for i in range(nb)])
        par = N.encode(k, m, S, data)
        out["case%d_parity" % ci] = par
        out["case%d_data_sha256" % ci] = np.frombuffer(hashlib.sha256(data.tobytes()).digest(), np.uint8)
        surv, lost, rows = [], [], []
        for i in range(nb):
            s, l = N.erasures(SEED, fb + i, k, m, e)
            surv.append(s); lost.append(l)
            rows.append(N.decode_matrix(k, m, s, l))
        out["case%d_surv" % ci] = np.array(surv, dtype=np.uint8)
        out["case%d_lost" % ci] = np.array(lost, dtype=np.uint8)
        out["case%d_rows" % ci] = np.array(rows, dtype=np.uint8)
        cases.append((k, m, B, fb, nb, e, S))
    out["cases"] = np.array(cases, dtype=np.int64)
    # exhaustive decode matrices for every erasure set of size <= m, small codes
    for (k, m) in [(3, 2), (4, 2)]:
        pats, mats = [], []
        for e in range(1, m + 1):
            for lost in itertools.combinations(range(k + m), e):
                surv = [i for i in range(k + m) if i not in lost][:k]
                M = np.zeros((m, k), dtype=np.uint8)
                M[:e] = N.decode_matrix(k, m, surv, list(lost))
                p = np.full(m, 255, dtype=np.uint8); p[:e] = lost
                pats.append(p); mats.append(M)
        out["exh_%d_%d_lost" % (k, m)] = np.array(pats)
        out["exh_%d_%d_rows" % (k, m)] = np.array(mats)
    np.savez_compressed(os.path.join(HERE, "rs_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "rs_golden.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
