"""ctypes loader for the C oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / the CPU baseline.  The product path
(memo_amd.ec -> libmemo_ec.so) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "librs_oracle.so")
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
sz = ctypes.c_size_t


def build(force=False):
    if force or not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "rs_oracle.c"))):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.memo_oracle_gf_mul.restype = ctypes.c_uint8
        L.memo_oracle_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.memo_oracle_gf_exp.restype = ctypes.c_uint8
        L.memo_oracle_gf_exp.argtypes = [ctypes.c_int]
        L.memo_oracle_gf_log.restype = ctypes.c_uint8
        L.memo_oracle_gf_log.argtypes = [ctypes.c_uint8]
        L.memo_oracle_gf_inv.restype = ctypes.c_uint8
        L.memo_oracle_gf_inv.argtypes = [ctypes.c_uint8]
        L.memo_oracle_shard_size.restype = sz
        L.memo_oracle_shard_size.argtypes = [sz, ctypes.c_int]
        L.memo_oracle_cauchy.argtypes = [ctypes.c_int, ctypes.c_int, u8p]
        L.memo_oracle_invert.argtypes = [ctypes.c_int, u8p, u8p]
        L.memo_oracle_decode_matrix.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p, ctypes.c_int, u8p]
        L.memo_oracle_encode.argtypes = [ctypes.c_int, ctypes.c_int, sz, sz, u8p, u8p]
        L.memo_oracle_encode_mt.argtypes = [ctypes.c_int, ctypes.c_int, sz, sz, u8p, u8p, ctypes.c_int]
        L.memo_oracle_encode_simd_mt.argtypes = [ctypes.c_int, ctypes.c_int, sz, sz, u8p, u8p,
                                                 ctypes.c_int, ctypes.c_int]
        L.memo_oracle_simd_isa.argtypes = []
        L.memo_oracle_rebuild_simd_mt.argtypes = [ctypes.c_int, ctypes.c_int, sz, sz, u8p, u8p, u8p,
                                                  ctypes.c_int, u8p, ctypes.c_int, ctypes.c_int]
        L.memo_oracle_rebuild.argtypes = [ctypes.c_int, ctypes.c_int, sz, sz, u8p, u8p, u8p, ctypes.c_int, u8p]
        L.memo_oracle_rebuild_mt.argtypes = [ctypes.c_int, ctypes.c_int, sz, sz, u8p, u8p, u8p,
                                             ctypes.c_int, u8p, ctypes.c_int]
        L.memo_oracle_block_key.restype = ctypes.c_uint64
        L.memo_oracle_block_key.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.memo_oracle_fill_blocks.argtypes = [ctypes.c_uint64, ctypes.c_uint64, sz, sz, ctypes.c_int, sz, u8p]
        L.memo_oracle_erasures.argtypes = [ctypes.c_uint64, ctypes.c_uint64, sz, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, u8p, u8p]
        L.memo_oracle_gather.argtypes = [ctypes.c_int, ctypes.c_int, sz, sz, u8p, u8p, u8p, ctypes.c_int, u8p]
        _lib = L
    return _lib


def _p(a):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u8p)


def gf_mul(a, b):
    return lib().memo_oracle_gf_mul(a, b)


def gf_exp(i):
    return lib().memo_oracle_gf_exp(i)


def gf_log(a):
    return lib().memo_oracle_gf_log(a)


def gf_inv(a):
    return lib().memo_oracle_gf_inv(a)


def shard_size(B, k):
    return lib().memo_oracle_shard_size(B, k)


def cauchy(k, m):
    a = np.zeros((k + m, k), dtype=np.uint8)
    if lib().memo_oracle_cauchy(k, m, _p(a)):
        raise ValueError("bad (k, m)")
    return a


def invert(A):
    A = np.ascontiguousarray(A, dtype=np.uint8)
    out = np.zeros_like(A)
    rc = lib().memo_oracle_invert(A.shape[0], _p(A), _p(out))
    if rc:
        raise ValueError("singular")
    return out


def decode_matrix(k, m, surv, lost):
    s = np.ascontiguousarray(surv, dtype=np.uint8)
    l = np.ascontiguousarray(lost, dtype=np.uint8)
    out = np.zeros((len(l), k), dtype=np.uint8)
    rc = lib().memo_oracle_decode_matrix(k, m, _p(s), _p(l), len(l), _p(out))
    if rc:
        raise ValueError("decode_matrix rc=%d" % rc)
    return out


def encode(k, m, S, data, threads=1):
    data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1, k * S)
    n = data.shape[0]
    par = np.zeros((n, m * S), dtype=np.uint8)
    if threads == 1:
        rc = lib().memo_oracle_encode(k, m, S, n, _p(data), _p(par))
    else:
        rc = lib().memo_oracle_encode_mt(k, m, S, n, _p(data), _p(par), threads)
    if rc:
        raise ValueError("encode rc=%d" % rc)
    return par


def aligned_empty(shape, align=64):
    """uint8 array whose data pointer is `align`-byte aligned (numpy only
    guarantees 16): lets encode_simd use streaming stores."""
    nb = int(np.prod(shape))
    raw = np.empty(nb + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nb].reshape(shape)


SIMD_ISA = {0: "scalar", 1: "avx2-pshufb", 2: "gfni-avx512"}


def simd_isa():
    """Best vector ISA of this host for encode_simd (0 scalar, 1 AVX2, 2 GFNI)."""
    return lib().memo_oracle_simd_isa()


def encode_simd(k, m, S, data, threads=1, isa=-1, out=None):
    """Vectorised encode (rs_simd.c), same bytes as encode(); returns
    (parity, isa_used)."""
    data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1, k * S)
    n = data.shape[0]
    par = np.zeros((n, m * S), dtype=np.uint8) if out is None else out
    used = lib().memo_oracle_encode_simd_mt(k, m, S, n, _p(data), _p(par), threads, isa)
    if used < 0:
        raise ValueError("encode_simd rejected k=%d m=%d" % (k, m))
    return par, used


def rebuild_simd(k, m, S, surv_idx, surv, lost_idx, threads=1, isa=-1, out=None):
    """Vectorised CPU rebuild (rs_simd.c): per-block decode rows by the scalar
    oracle, the MAC by GFNI/AVX-512 or AVX2.  Returns (out, isa used)."""
    surv_idx = np.ascontiguousarray(surv_idx, dtype=np.uint8)
    lost_idx = np.ascontiguousarray(lost_idx, dtype=np.uint8)
    n, e = lost_idx.shape
    surv = np.ascontiguousarray(surv, dtype=np.uint8).reshape(n, k * S)
    if out is None:
        out = np.zeros((n, e * S), dtype=np.uint8)
    used = lib().memo_oracle_rebuild_simd_mt(k, m, S, n, _p(surv_idx), _p(surv), _p(lost_idx), e,
                                             _p(out), threads, isa)
    if used < 0:
        raise ValueError("rebuild_simd rejected the input")
    return out, used


def rebuild(k, m, S, surv_idx, surv, lost_idx, threads=1):
    surv_idx = np.ascontiguousarray(surv_idx, dtype=np.uint8)
    lost_idx = np.ascontiguousarray(lost_idx, dtype=np.uint8)
    n = surv_idx.shape[0]
    e = lost_idx.shape[1] if lost_idx.ndim == 2 else 0
    surv = np.ascontiguousarray(surv, dtype=np.uint8).reshape(n, k * S)
    out = np.zeros((n, e * S), dtype=np.uint8)
    if threads == 1:
        rc = lib().memo_oracle_rebuild(k, m, S, n, _p(surv_idx), _p(surv), _p(lost_idx), e, _p(out))
    else:
        rc = lib().memo_oracle_rebuild_mt(k, m, S, n, _p(surv_idx), _p(surv), _p(lost_idx), e, _p(out),
                                          threads)
    if rc:
        raise ValueError("rebuild rc=%d" % rc)
    return out


def fill_blocks(seed, first_block, n, B, k, S):
    out = np.empty((n, k * S), dtype=np.uint8)
    lib().memo_oracle_fill_blocks(seed, first_block, n, B, k, S, _p(out))
    return out


def erasures(seed, first_block, n, k, m, e):
    s = np.zeros((n, k), dtype=np.uint8)
    l = np.zeros((n, e), dtype=np.uint8)
    lib().memo_oracle_erasures(seed, first_block, n, k, m, e, _p(s), _p(l))
    return s, l


def gather(k, m, S, data, parity, idx):
    idx = np.ascontiguousarray(idx, dtype=np.uint8)
    n, cnt = idx.shape
    data = np.ascontiguousarray(data, dtype=np.uint8)
    parity = np.ascontiguousarray(parity, dtype=np.uint8)
    out = np.empty((n, cnt * S), dtype=np.uint8)
    lib().memo_oracle_gather(k, m, S, n, _p(data), _p(parity), _p(idx), cnt, _p(out))
    return out
