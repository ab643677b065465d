"""Independent numpy restatement of the erasure codec (TEST INFRASTRUCTURE).

Used only to generate and re-check the golden fixtures under tests/golden/.
It shares no code with oracle/rs_oracle.c: field multiplication here is the
carry-less "Russian peasant" product reduced by 0x11D (no log/antilog
tables), inversion is a^254 by square-and-multiply, and matrix inversion is a
Python Gauss-Jordan.  See oracle/rs_oracle.c for the convention and why it is
"parity unpinned by the reference" (infinit/memo has no erasure code; its
redundancy is replication, src/memo/model/doughnut/consensus/Paxos.cc:315-391).
"""
import numpy as np

POLY = 0x11D
GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def gf_mul_vec(a, b):
    """Carry-less multiply of uint8 arrays a*b mod x^8+x^4+x^3+x^2+1."""
    a = np.asarray(a, dtype=np.uint16).copy()
    b = np.asarray(b, dtype=np.uint16).copy()
    a, b = np.broadcast_arrays(a, b)
    a = a.copy(); b = b.copy()
    r = np.zeros(a.shape, dtype=np.uint16)
    for _ in range(8):
        r ^= np.where(b & 1, a, 0).astype(np.uint16)
        b >>= 1
        a <<= 1
        a = np.where(a & 0x100, a ^ POLY, a).astype(np.uint16)
    return r.astype(np.uint8)


def gf_mul(a, b):
    return int(gf_mul_vec(np.uint8(a), np.uint8(b)))


def gf_pow(a, e):
    r, x = 1, a
    while e:
        if e & 1:
            r = gf_mul(r, x)
        x = gf_mul(x, x)
        e >>= 1
    return r


def gf_inv(a):
    if a == 0:
        return 0
    return gf_pow(a, 254)


_TABLE = None


def mul_table():
    global _TABLE
    if _TABLE is None:
        a = np.arange(256, dtype=np.uint8)[:, None]
        b = np.arange(256, dtype=np.uint8)[None, :]
        _TABLE = gf_mul_vec(a, b)
    return _TABLE


def shard_size(B, k):
    per = max(1, -(-B // k))
    return (per + 63) // 64 * 64


def cauchy(k, m):
    a = np.zeros((k + m, k), dtype=np.uint8)
    for i in range(k):
        a[i, i] = 1
    for i in range(k, k + m):
        for j in range(k):
            a[i, j] = gf_inv(i ^ j)
    return a


def invert(A):
    n = A.shape[0]
    w = [list(map(int, row)) for row in A]
    o = [[int(i == j) for j in range(n)] for i in range(n)]
    for c in range(n):
        p = next((r for r in range(c, n) if w[r][c]), None)
        if p is None:
            raise ValueError("singular")
        w[c], w[p] = w[p], w[c]
        o[c], o[p] = o[p], o[c]
        iv = gf_inv(w[c][c])
        w[c] = [gf_mul(iv, x) for x in w[c]]
        o[c] = [gf_mul(iv, x) for x in o[c]]
        for r in range(n):
            if r != c and w[r][c]:
                f = w[r][c]
                w[r] = [x ^ gf_mul(f, y) for x, y in zip(w[r], w[c])]
                o[r] = [x ^ gf_mul(f, y) for x, y in zip(o[r], o[c])]
    return np.array(o, dtype=np.uint8)


def matmul(A, B):
    """GF matrix product of small uint8 matrices."""
    T = mul_table()
    out = np.zeros((A.shape[0], B.shape[1]), dtype=np.uint8)
    for t in range(A.shape[1]):
        out ^= T[A[:, t][:, None], B[t, :][None, :]]
    return out


def decode_matrix(k, m, surv, lost):
    C = cauchy(k, m)
    inv = invert(C[list(surv)])
    return matmul(C[list(lost)], inv)


def mac(M, shards):
    """shards: (kin, S) uint8; M: (r, kin) -> (r, S)."""
    T = mul_table()
    out = np.zeros((M.shape[0], shards.shape[1]), dtype=np.uint8)
    for r in range(M.shape[0]):
        for j in range(M.shape[1]):
            out[r] ^= T[M[r, j]][shards[j]]
    return out


def encode(k, m, S, data):
    """data: (n, k*S) uint8 -> parity (n, m*S)."""
    C = cauchy(k, m)[k:]
    n = data.shape[0]
    par = np.zeros((n, m * S), dtype=np.uint8)
    for b in range(n):
        par[b] = mac(C, data[b].reshape(k, S)).reshape(-1)
    return par


def _mix(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def block_key(seed, block):
    with np.errstate(over="ignore"):
        return _mix(_mix(np.uint64(seed)) ^ (np.uint64(block) * GAMMA))


def fill_block(seed, block, B, k, S):
    key = block_key(seed, block)
    nw = -(-B // 8)
    with np.errstate(over="ignore"):
        ctr = (np.arange(1, nw + 1, dtype=np.uint64) * GAMMA) + key
    words = _mix(ctr).astype("<u8")
    out = np.zeros(k * S, dtype=np.uint8)
    out[:B] = words.view(np.uint8)[:B]
    return out


def erasures(seed, block, k, m, e):
    total = k + m
    key = block_key(seed + 1, block)
    perm = list(range(total))
    for i in range(e):
        with np.errstate(over="ignore"):
            w = int(_mix(key + np.uint64(i + 1) * GAMMA))
        r = i + w % (total - i)
        perm[i], perm[r] = perm[r], perm[i]
    lost = sorted(perm[:e])
    surv = [i for i in range(total) if i not in lost][:k]
    return surv, lost
