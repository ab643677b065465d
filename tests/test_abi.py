"""C-ABI library checks that need no GPU: it loads, exports every symbol
include/memo_ec.h declares, and its host-only functions agree with the
oracle.  No compute call is made here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, SEED


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "memo_ec.h")).read()
    return sorted(set(re.findall(r"\b(memo_ec_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    from memo_amd import ec
    assert sorted(ec.EXPORTS) == header_symbols()


def test_option_ids_agree_with_header():
    """memo_amd.ec.OPTIONS names every memo_ec_option of the header, with
    the header's value (MEMO_EC_OPT_IMAGE_MIN_TILES -> "image_min_tiles")."""
    from memo_amd import ec
    txt = open(os.path.join(ROOT, "include", "memo_ec.h")).read()
    hdr = {n.lower(): int(v) for n, v in re.findall(r"\bMEMO_EC_OPT_([A-Z0-9_]+)\s*=\s*(\d+)", txt)}
    assert hdr and ec.OPTIONS == hdr


def test_library_exports_every_header_symbol():
    from memo_amd import ec
    lib = ctypes.CDLL(ec.LIB_PATH)
    for name in header_symbols():
        assert hasattr(lib, name), name


def test_library_is_gfx950_code():
    from memo_amd import ec
    blob = open(ec.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_host_functions_match_oracle(O):
    from memo_amd import ec
    for B in [0, 1, 63, 64, 1000, 65536, 1 << 20, 4 << 20]:
        for k in [3, 4, 10, 16]:
            assert ec.shard_size(B, k) == O.shard_size(B, k)
    for (k, m) in [(3, 2), (4, 2), (10, 4), (16, 4), (64, 16)]:
        assert np.array_equal(ec.generator(k, m), O.cauchy(k, m))
    for (k, m, e) in [(3, 2, 2), (10, 4, 4), (16, 4, 1), (4, 2, 0)]:
        s, l = ec.erasures(SEED, 17, 50, k, m, e)
        so, lo = O.erasures(SEED, 17, 50, k, m, e)
        assert np.array_equal(s, so) and np.array_equal(l, lo)


def test_error_codes_and_limits():
    from memo_amd import ec
    L = ec._lib()
    assert L.memo_ec_version() == 2
    assert L.memo_ec_strerror(-4) == b"survivor shards cannot rebuild the block"
    with pytest.raises(ec.MemoECError):
        ec.generator(65, 4)
    with pytest.raises(ec.MemoECError):
        ec.generator(0, 4)
    assert L.memo_ec_encode_batch(None, 10, 4, 64, 1, None, None, 2) == -1
    assert L.memo_ec_rebuild_segments(None, 0, None, 2) == -1
    assert L.memo_ec_ctx_set_option(None, 1, 0) == -1
    assert L.memo_ec_stream_probe(None, 10, 4, 64, 1, None, None, 0) == -1
    buf = ctypes.create_string_buffer(64)
    assert L.memo_ec_device_identity(0, buf, 8, buf, 64) == -1       # short bus-id buffer
    assert L.memo_ec_device_identity(0, buf, 64, buf, 16) == -1      # short UUID buffer
    if L.memo_ec_device_count() == 0:                                # no GPU here: no device 0
        assert L.memo_ec_device_identity(0, buf, 64, buf, 64) == -5


def test_build_id_matches_sources():
    """The library in the tree was built from the sources in the tree
    (memo_ec_build_id() == SHA-256 of include/memo_ec.h + the csrc files)."""
    from memo_amd import ec
    assert len(ec.build_id()) == 64
    assert ec.check_build() == ec.source_id()


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from memo_amd import ec
    with pytest.raises(ec.MemoECError):
        ec.Codec(0)


def test_shared_pattern_lengths_checked():
    """rebuild_uniform / shared-pattern segments: the C side reads exactly k
    and e host indices, so short sequences are refused before the call (no
    GPU needed: the check comes first)."""
    from memo_amd import ec
    import numpy as np
    c = ec.Codec.__new__(ec.Codec)  # no ctx: the check must raise before any call
    buf = np.zeros((2, 10 * 64), np.uint8)
    out = np.zeros((2, 64), np.uint8)
    with pytest.raises(ValueError):
        c.rebuild_uniform(10, 4, [0, 1, 2], buf, [12], out)
    with pytest.raises(ValueError):
        c.rebuild_uniform(10, 4, list(range(10)), buf, [], out)
    with pytest.raises(ValueError):
        c.rebuild_uniform(10, 4, list(range(10)), buf, [10, 11, 12, 13, 9], out)
    with pytest.raises(ValueError):
        c.rebuild_segments([dict(k=10, m=4, surv=buf, out=out, uniform=True, surv_idx=[0], lost_idx=[12])])
