"""Python binding of libmemo_ec.so (the C ABI in include/memo_ec.h).

This is plumbing for tests and bench.py: every call goes through the C ABI
into the gfx950 HIP kernels.  There is no CPU fallback -- if the library is
missing or no GPU is present, the calls raise.

Device buffers are torch uint8 CUDA tensors (PyTorch-ROCm provides the HBM
allocations and streams); host buffers are numpy uint8 arrays.

Reference call sites the codec replaces (infinit/memo, read-only):
  encode  <- Paxos::Details::send_immutable_block, consensus/Paxos.cc:315-391
  rebuild <- Paxos::Details::_fetch (immutable), Paxos.cc:486-519, and the
             _rebalance repair loop, Paxos.cc:1012-1246
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MEMO_EC_LIB points the binding at another build of the same ABI (the
# tuning variants of tools/build_variants.sh); default: the in-tree library.
LIB_PATH = os.environ.get("MEMO_EC_LIB") or os.path.join(_HERE, "_lib", "libmemo_ec.so")

HOST, HOST_PINNED, DEVICE = 0, 1, 2
MAX_K, MAX_M, MAX_SEGMENTS = 64, 16, 12

_u8p = ctypes.c_void_p
_sz = ctypes.c_size_t


class MemoECError(RuntimeError):
    """Raised for a negative memo_ec status code (memo_ec_strerror text)."""

    def __init__(self, code, what=""):
        self.code = code
        msg = _lib().memo_ec_strerror(code).decode() if _LIB is not None else str(code)
        super().__init__("%s%s (code %d)" % (what + ": " if what else "", msg, code))


class Segment(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int), ("m", ctypes.c_int), ("S", _sz), ("n", _sz),
                ("data", ctypes.c_void_p), ("parity", ctypes.c_void_p)]


class RebuildSegment(ctypes.Structure):
    """memo_ec_rebuild_segment (include/memo_ec.h)."""
    _fields_ = [("k", ctypes.c_int), ("m", ctypes.c_int), ("S", _sz), ("n", _sz),
                ("surv_idx", ctypes.c_void_p), ("surv", ctypes.c_void_p),
                ("lost_idx", ctypes.c_void_p), ("e", ctypes.c_int), ("uniform", ctypes.c_int),
                ("out", ctypes.c_void_p)]


# memo_ec_option (include/memo_ec.h)
OPTIONS = {"rebuild_path": 1, "fused_max_bytes": 2, "zero_copy_bytes": 3, "pipe_bytes": 4,
           "copy_threads": 5, "max_launch_tiles": 6, "xcd_min_tiles": 7, "decode_wide_max": 8,
           "decode_exact": 9, "decode_stage": 10, "image_min_tiles": 11,
           "image_min_coefs": 12, "decode_overlap": 13}
MAX_REBUILD_SEGMENTS = 256
PROBE_MODES = {"copy": 0, "read": 1, "write": 2}  # memo_ec_probe_mode

# The sources memo_ec_build_id() hashes, in its order (memo_amd/csrc/Makefile).
_ROOT = os.path.dirname(_HERE)
BUILD_SOURCES = [os.path.join(_ROOT, "include", "memo_ec.h"),
                 os.path.join(_HERE, "csrc", "ec_kernels.h"),
                 os.path.join(_HERE, "csrc", "ec_kernels.hip"),
                 os.path.join(_HERE, "csrc", "memo_ec.cpp")]


_LIB = None

EXPORTS = [
    "memo_ec_ctx_create", "memo_ec_ctx_destroy", "memo_ec_set_stream", "memo_ec_get_stream",
    "memo_ec_synchronize", "memo_ec_shard_size", "memo_ec_generator", "memo_ec_encode_batch",
    "memo_ec_rebuild_batch", "memo_ec_rebuild_uniform", "memo_ec_decode_rows",
    "memo_ec_host_alloc", "memo_ec_host_free", "memo_ec_encode_segments",
    "memo_ec_sha256_batch", "memo_ec_fill_blocks", "memo_ec_erasures", "memo_ec_gather_shards",
    "memo_ec_strerror",
    "memo_ec_version", "memo_ec_device_count", "memo_ec_rebuild_segments",
    "memo_ec_ctx_set_option", "memo_ec_ctx_get_option", "memo_ec_build_id",
    "memo_ec_device_identity", "memo_ec_stream_probe",
]


def _lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libmemo_ec.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        c_int, c_u64 = ctypes.c_int, ctypes.c_uint64
        L.memo_ec_ctx_create.argtypes = [c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.memo_ec_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.memo_ec_set_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.memo_ec_get_stream.argtypes = [ctypes.c_void_p]
        L.memo_ec_get_stream.restype = ctypes.c_void_p
        L.memo_ec_synchronize.argtypes = [ctypes.c_void_p]
        L.memo_ec_shard_size.argtypes = [_sz, c_int]
        L.memo_ec_shard_size.restype = _sz
        L.memo_ec_generator.argtypes = [c_int, c_int, _u8p]
        L.memo_ec_encode_batch.argtypes = [ctypes.c_void_p, c_int, c_int, _sz, _sz, _u8p, _u8p, c_int]
        L.memo_ec_rebuild_batch.argtypes = [ctypes.c_void_p, c_int, c_int, _sz, _sz, _u8p, _u8p,
                                            _u8p, c_int, _u8p, c_int]
        L.memo_ec_rebuild_uniform.argtypes = [ctypes.c_void_p, c_int, c_int, _sz, _sz, _u8p, _u8p,
                                              _u8p, c_int, _u8p, c_int]
        L.memo_ec_host_alloc.argtypes = [_sz]
        L.memo_ec_host_alloc.restype = ctypes.c_void_p
        L.memo_ec_host_free.argtypes = [ctypes.c_void_p]
        L.memo_ec_decode_rows.argtypes = [ctypes.c_void_p, c_int, c_int, _sz, _u8p, _u8p, c_int, _u8p]
        L.memo_ec_encode_segments.argtypes = [ctypes.c_void_p, c_int, ctypes.POINTER(Segment)]
        L.memo_ec_sha256_batch.argtypes = [ctypes.c_void_p, _sz, _u8p, _sz, _sz, _u8p, _sz,
                                           ctypes.c_void_p, _sz, _u8p]
        L.memo_ec_fill_blocks.argtypes = [ctypes.c_void_p, c_u64, c_u64, _sz, _sz, c_int, _sz, _u8p]
        L.memo_ec_erasures.argtypes = [c_u64, c_u64, _sz, c_int, c_int, c_int, _u8p, _u8p]
        L.memo_ec_gather_shards.argtypes = [ctypes.c_void_p, c_int, c_int, _sz, _sz, _u8p, _u8p,
                                            _u8p, c_int, _u8p]
        L.memo_ec_strerror.argtypes = [c_int]
        L.memo_ec_strerror.restype = ctypes.c_char_p
        L.memo_ec_version.restype = c_int
        L.memo_ec_device_count.restype = c_int
        L.memo_ec_rebuild_segments.argtypes = [ctypes.c_void_p, c_int, ctypes.POINTER(RebuildSegment),
                                               c_int]
        L.memo_ec_ctx_set_option.argtypes = [ctypes.c_void_p, c_int, ctypes.c_int64]
        L.memo_ec_ctx_get_option.argtypes = [ctypes.c_void_p, c_int, ctypes.POINTER(ctypes.c_int64)]
        L.memo_ec_build_id.restype = ctypes.c_char_p
        L.memo_ec_device_identity.argtypes = [c_int, ctypes.c_char_p, _sz, ctypes.c_char_p, _sz]
        L.memo_ec_stream_probe.argtypes = [ctypes.c_void_p, c_int, c_int, _sz, _sz, _u8p, _u8p, c_int]
        _LIB = L
    return _LIB


def _check(rc, what=""):
    if rc != 0:
        raise MemoECError(rc, what)


def build_id():
    """SHA-256 of the sources the loaded library was built from."""
    return _lib().memo_ec_build_id().decode()


def source_id():
    """SHA-256 of the library's sources in this tree (what build_id() must be)."""
    import hashlib
    h = hashlib.sha256()
    for p in BUILD_SOURCES:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def check_build():
    """Raise unless the loaded library was built from this tree's sources."""
    b, s = build_id(), source_id()
    if b != s:
        raise RuntimeError("libmemo_ec.so build id %s does not match the sources (%s): rebuild "
                           "with __graft_entry__.build()" % (b[:16], s[:16]))
    return b


def device_identity(device):
    """{"pci_bus_id", "uuid"} of GPU `device` (memo_ec_device_identity)."""
    pci = ctypes.create_string_buffer(64)
    uid = ctypes.create_string_buffer(64)
    _check(_lib().memo_ec_device_identity(device, pci, 64, uid, 64), "device_identity")
    return {"pci_bus_id": pci.value.decode(), "uuid": uid.value.decode()}


def shard_size(block_bytes, k):
    """S = round_up(ceil(B / k), 64) -- the shard size of a B-byte block."""
    return _lib().memo_ec_shard_size(block_bytes, k)


def generator(k, m):
    """(k+m) x k generator matrix (identity over ISA-L cauchy1 rows)."""
    out = np.zeros((k + m, k), dtype=np.uint8)
    _check(_lib().memo_ec_generator(k, m, out.ctypes.data), "generator")
    return out


def erasures(seed, first_block, n, k, m, e):
    """Synthetic erasure patterns (host): (surv_idx n x k, lost_idx n x e)."""
    s = np.zeros((n, k), dtype=np.uint8)
    l = np.zeros((n, max(e, 1)), dtype=np.uint8)
    _check(_lib().memo_ec_erasures(seed, first_block, n, k, m, e, s.ctypes.data, l.ctypes.data),
           "erasures")
    return s, l[:, :e].copy()


REBUILD_KERNELS = {"fused": "gf_rebuild_kernel (decode rows per tile + MAC, one launch)",
                   "rows": "decode_coef*/decode_rows_k + gf_mac_kernel (rows through HBM, "
                           "tables built in LDS)",
                   "images": "decode_coef_wide_kernel forming per-block table images beside "
                             "the rows + gf_mac_kernel encode body (images through HBM)"}


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _ptr(x):
    """(pointer, where) of a uint8 buffer: CUDA tensor -> DEVICE, numpy -> HOST."""
    if _is_torch(x):
        import torch
        if x.dtype != torch.uint8:
            raise TypeError("expected a uint8 tensor")
        if not x.is_contiguous():
            raise ValueError("expected a contiguous tensor")
        if x.is_cuda:
            return x.data_ptr(), DEVICE
        return x.data_ptr(), HOST_PINNED if x.is_pinned() else HOST
    if isinstance(x, np.ndarray):
        if x.dtype != np.uint8 or not x.flags["C_CONTIGUOUS"]:
            raise TypeError("expected a C-contiguous uint8 array")
        return x.ctypes.data, HOST
    raise TypeError("unsupported buffer type %r" % type(x))


class Codec:
    """One memo_ec context on one GPU (one per thread, like the reference's
    background pool threads; elle/src/elle/reactor/scheduler.cc:562-602)."""

    def __init__(self, device=0):
        self._ctx = ctypes.c_void_p()
        _check(_lib().memo_ec_ctx_create(device, ctypes.byref(self._ctx)), "ctx_create")
        self.device = device

    def close(self):
        if self._ctx:
            _lib().memo_ec_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- streams
    def set_stream(self, stream):
        """Enqueue device work on a torch.cuda.Stream / raw hipStream_t (None = own)."""
        if stream is None:
            h = None
        elif isinstance(stream, int):
            h = stream
        else:
            h = stream.cuda_stream
        _check(_lib().memo_ec_set_stream(self._ctx, h), "set_stream")

    @property
    def stream(self):
        return _lib().memo_ec_get_stream(self._ctx)

    def synchronize(self):
        _check(_lib().memo_ec_synchronize(self._ctx), "synchronize")

    # -- tuning (memo_ec_ctx_set_option)
    def set_option(self, name, value):
        _check(_lib().memo_ec_ctx_set_option(self._ctx, OPTIONS[name], int(value)), "set_option")

    def get_option(self, name):
        v = ctypes.c_int64()
        _check(_lib().memo_ec_ctx_get_option(self._ctx, OPTIONS[name], ctypes.byref(v)), "get_option")
        return v.value

    def options(self, **kw):
        """Context manager: set options for a block of calls, then restore them."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = {k: self.get_option(k) for k in kw}
            try:
                for k, v in kw.items():
                    self.set_option(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_option(k, v)
        return cm()

    def rebuild_path(self, n, k, S, e=None):
        """The device rebuild this ctx runs for n blocks of k survivor shards
        of S bytes (memo_ec.cpp rebuild_fused, from the ctx's options as set
        by the environment or set_option): 'fused' (one gf_rebuild_kernel
        launch whose tiles derive their blocks' decode rows), 'rows'
        (decode rows through HBM, then gf_mac_kernel building each tile's
        tables in LDS) or 'images' (decode rows, then per-block table images
        through HBM for blocks of >= image_min_tiles 4 KiB shard tiles with
        costly tables (uses_images), then gf_mac_kernel's encode body).  e
        (lost shards per block) defaults to 4."""
        path = self.get_option("rebuild_path")
        if path < 0:
            path = 1 if n * k * S <= self.get_option("fused_max_bytes") else 0
        if path:
            return "fused"
        return "images" if self.uses_images(k, S, e) else "rows"

    def uses_images(self, k, S, e=None):
        """Whether the rows path forms per-block table images in HBM for
        this geometry (memo_ec.cpp rows_images): shards of >= image_min_tiles
        whole 4 KiB tiles whose R x kpad coefficients reach image_min_coefs,
        or any k without a straight-line MAC body.  e defaults to 4."""
        try:
            t = self.get_option("image_min_tiles")
        except MemoECError:  # a library from before the option (A/B runs of older builds)
            return False
        if not t or S // 4096 < t:
            return False
        R = mac_rbound(4 if e is None else e)
        KC = mac_kchunk(k, R)
        kpad = -(-k // KC) * KC
        return KC != k or R * kpad >= self.get_option("image_min_coefs")

    def rebuild_kernel_name(self, n, k, S, e=None):
        return REBUILD_KERNELS[self.rebuild_path(n, k, S, e)]

    # -- codec
    def encode(self, k, m, data, parity, S=None, n=None):
        """parity (n x m x S) <- data (n x k x S); device (async) or host (sync)."""
        dp, dw = _ptr(data)
        pp, pw = _ptr(parity)
        if (dw == DEVICE) != (pw == DEVICE):
            raise ValueError("data and parity must both be device or both host buffers")
        if S is None:
            n, S = _infer_nS(data, k)
        where = DEVICE if dw == DEVICE else (HOST_PINNED if dw == pw == HOST_PINNED else HOST)
        _check(_lib().memo_ec_encode_batch(self._ctx, k, m, S, n, dp, pp, where), "encode")
        return parity

    def rebuild(self, k, m, surv_idx, surv, lost_idx, out, S=None, n=None):
        """out (n x e x S) <- the k survivor shards surv (n x k x S) of each block."""
        sp, sw = _ptr(surv)
        op, ow = _ptr(out)
        ip, iw = _ptr(surv_idx)
        lp, lw = _ptr(lost_idx)
        if S is None:
            n, S = _infer_nS(surv, k)
        e = lost_idx.shape[1] if len(lost_idx.shape) == 2 else 0
        if sw == DEVICE:
            if not (ow == iw == lw == DEVICE):
                raise ValueError("device rebuild needs every buffer on the device")
            where = DEVICE
        else:
            if DEVICE in (ow, iw, lw):
                raise ValueError("host rebuild needs every buffer in host memory")
            where = HOST_PINNED if sw == ow == HOST_PINNED else HOST
        _check(_lib().memo_ec_rebuild_batch(self._ctx, k, m, S, n, ip, sp, lp, e, op, where),
               "rebuild")
        return out

    def rebuild_uniform(self, k, m, surv_idx, surv, lost_idx, out, S=None, n=None):
        """out (n x e x S) <- surv (n x k x S) with ONE erasure pattern for the
        whole batch: surv_idx (k) and lost_idx (e) are host sequences."""
        sp, sw = _ptr(surv)
        op, ow = _ptr(out)
        if (sw == DEVICE) != (ow == DEVICE):
            raise ValueError("surv and out must both be device or both host buffers")
        si = np.ascontiguousarray(np.asarray(surv_idx, dtype=np.uint8).reshape(-1))
        li = np.ascontiguousarray(np.asarray(lost_idx, dtype=np.uint8).reshape(-1))
        _check_pattern(si, li, k, m)
        if S is None:
            n, S = _infer_nS(surv, k)
        where = DEVICE if sw == DEVICE else (HOST_PINNED if sw == ow == HOST_PINNED else HOST)
        _check(_lib().memo_ec_rebuild_uniform(self._ctx, k, m, S, n, si.ctypes.data, sp,
                                              li.ctypes.data, len(li), op, where), "rebuild_uniform")
        return out

    def decode_rows(self, k, m, surv_idx, lost_idx, rows):
        n, e = lost_idx.shape
        _check(_lib().memo_ec_decode_rows(self._ctx, k, m, n, _ptr(surv_idx)[0], _ptr(lost_idx)[0],
                                          e, _ptr(rows)[0]), "decode_rows")
        return rows

    def rebuild_segments(self, segs):
        """One memo_ec_rebuild_segments call.  segs: list of dicts with k, m,
        surv_idx, surv, lost_idx, out and optionally uniform (then surv_idx /
        lost_idx are host sequences of k / e indices).  Buffers: all device
        tensors (asynchronous) or all host (numpy / pinned torch; synchronous)."""
        arr = (RebuildSegment * len(segs))()
        keep, wheres = [], set()
        for i, s in enumerate(segs):
            k, m = s["k"], s["m"]
            sp, sw = _ptr(s["surv"])
            op, ow = _ptr(s["out"])
            n, S = (s["n"], s["S"]) if "S" in s else _infer_nS(s["surv"], k)
            uni = bool(s.get("uniform", False))
            if uni:
                si = np.ascontiguousarray(np.asarray(s["surv_idx"], dtype=np.uint8).reshape(-1))
                li = np.ascontiguousarray(np.asarray(s["lost_idx"], dtype=np.uint8).reshape(-1))
                _check_pattern(si, li, k, m)
                keep += [si, li]
                ip, lp, e = si.ctypes.data, li.ctypes.data, len(li)
            else:
                ip, iw = _ptr(s["surv_idx"])
                lp, lw = _ptr(s["lost_idx"])
                e = s["lost_idx"].shape[1]
                wheres.update({iw if iw == DEVICE else HOST, lw if lw == DEVICE else HOST})
            wheres.update({sw if sw == DEVICE else HOST, ow if ow == DEVICE else HOST})
            arr[i] = RebuildSegment(k, m, S, n, ip, sp, lp, e, int(uni), op)
        if len(wheres) > 1:
            raise ValueError("rebuild_segments: mix of device and host buffers")
        if DEVICE in wheres:
            where = DEVICE
        else:
            allp = all(_ptr(s["surv"])[1] == HOST_PINNED and _ptr(s["out"])[1] == HOST_PINNED
                       for s in segs)
            where = HOST_PINNED if allp else HOST
        _check(_lib().memo_ec_rebuild_segments(self._ctx, len(segs), arr, where), "rebuild_segments")

    def encode_segments(self, segs):
        """segs: list of (k, m, S, n, data_tensor, parity_tensor) on this device."""
        arr = (Segment * len(segs))()
        for i, (k, m, S, n, d, p) in enumerate(segs):
            arr[i] = Segment(k, m, S, n, _ptr(d)[0], _ptr(p)[0])
        _check(_lib().memo_ec_encode_segments(self._ctx, len(segs), arr), "encode_segments")

    def sha256(self, msg, digest, prefix=None, msg_len=None, uniform_len=None, msg_stride=None):
        """digest[i] = SHA-256(prefix[i] || msg[i]) on the GPU (CHB address hash).
        msg: uint8 (n, stride) device tensor; msg_len: int64 device tensor or
        None (uniform_len bytes, default the row length); prefix: (n, P) or None."""
        n = msg.shape[0]
        stride = msg_stride if msg_stride is not None else msg.shape[1]
        pp, pl, ps = (0, 0, 0) if prefix is None else (_ptr(prefix)[0], prefix.shape[1], prefix.shape[1])
        lp = 0 if msg_len is None else msg_len.data_ptr()
        ul = stride if uniform_len is None else uniform_len
        _check(_lib().memo_ec_sha256_batch(self._ctx, n, pp or None, pl, ps, _ptr(msg)[0], stride,
                                           lp or None, ul, _ptr(digest)[0]), "sha256")
        return digest

    def stream_probe(self, kin, r, inp, out, mode="copy"):
        """memo_ec_stream_probe: the encode's traffic for (k, m) = (kin, r)
        without the GF arithmetic (device tensors; asynchronous); mode
        'copy' (loads and stores), 'read' or 'write' (one side alone)."""
        n, S = _infer_nS(inp, kin)
        _check(_lib().memo_ec_stream_probe(self._ctx, kin, r, S, n, _ptr(inp)[0], _ptr(out)[0],
                                           PROBE_MODES[mode]), "stream_probe")
        return out

    def fill_blocks(self, seed, first_block, n, B, k, S, out):
        _check(_lib().memo_ec_fill_blocks(self._ctx, seed, first_block, n, B, k, S, _ptr(out)[0]),
               "fill_blocks")
        return out

    def gather_shards(self, k, m, S, n, data, parity, idx, out):
        cnt = idx.shape[1]
        _check(_lib().memo_ec_gather_shards(self._ctx, k, m, S, n, _ptr(data)[0], _ptr(parity)[0],
                                            _ptr(idx)[0], cnt, _ptr(out)[0]), "gather_shards")
        return out


def mac_rbound(r):
    """Compile-time output-row bound of the MAC (ec_kernels.hip mac_rbound)."""
    return r if r <= 4 else 6 if r <= 6 else 8 if r <= 8 else 12 if r <= 12 else 16


def mac_kchunk(k, R):
    """Straight-line shard chunk of the MAC (ec_kernels.hip mac_kchunk)."""
    if k in (2, 3, 4, 10, 16):
        return k
    if k in (6, 12, 14):
        return k if R <= 4 else 4
    return 4


def _check_pattern(si, li, k, m):
    """A shared erasure pattern: the C side reads exactly k survivor and e
    lost indices from these host arrays, so their lengths are checked here."""
    if len(si) != k:
        raise ValueError("surv_idx has %d entries, k = %d" % (len(si), k))
    if not 1 <= len(li) <= m:
        raise ValueError("lost_idx has %d entries, need 1..m = %d" % (len(li), m))


def _infer_nS(buf, k):
    shape = tuple(buf.shape)
    if len(shape) == 3:
        return shape[0], shape[2]
    if len(shape) == 2:
        if shape[1] % k:
            raise ValueError("row length not a multiple of k")
        return shape[0], shape[1] // k
    raise ValueError("pass S and n for a flat buffer")
