"""CPU oracle checks: published GF(2^8)/0x11D values, golden fixtures from
the independent numpy restatement, and codec properties."""
import hashlib
import itertools
import os

import numpy as np
import pytest

from conftest import ROOT, SEED

# ISO/IEC 18004 (QR code) antilog table for x^8+x^4+x^3+x^2+1, first 30 values.
QR_EXP = [1, 2, 4, 8, 16, 32, 64, 128, 29, 58, 116, 232, 205, 135, 19, 38, 76, 152, 45, 90,
          180, 117, 234, 201, 143, 3, 6, 12, 24, 48]
# Published QR "HELLO WORLD" version 1-M: 16 data codewords -> 10 EC codewords.
QR_DATA = [32, 91, 11, 120, 209, 114, 220, 77, 67, 64, 236, 17, 236, 17, 236, 17]
QR_EC = [196, 35, 39, 119, 235, 215, 231, 226, 93, 23]


def test_field_published_values(O):
    assert [O.gf_exp(i) for i in range(30)] == QR_EXP
    assert O.gf_exp(255) == 1
    for a in range(1, 256):
        assert O.gf_mul(a, O.gf_inv(a)) == 1
    assert O.gf_mul(0x53, 0xCA) == 0x8F


def test_field_qr_hello_world(O):
    g = [1]
    for i in range(10):
        a = O.gf_exp(i)
        ng = [0] * (len(g) + 1)
        for j, c in enumerate(g):
            ng[j] ^= c
            ng[j + 1] ^= O.gf_mul(c, a)
        g = ng
    msg = QR_DATA + [0] * 10
    for i in range(len(QR_DATA)):
        c = msg[i]
        if c:
            for j in range(1, len(g)):
                msg[i + j] ^= O.gf_mul(g[j], c)
    assert msg[len(QR_DATA):] == QR_EC


def test_survey_self_checks(O):
    C = O.cauchy(3, 2)
    assert C[3:].tobytes().hex() == "f48e0147a77a"
    assert O.cauchy(10, 4)[10].tobytes().hex() == "dd98ad9d5d963daa8ef4"
    for (k, m, want) in [(3, 2, "7b9a"), (10, 4, "5353c9c9"), (16, 4, "1f1f1f1f")]:
        p = O.encode(k, m, 64, np.ones((1, k * 64), np.uint8))
        assert p[0, ::64].tobytes().hex() == want


def test_generators_match_golden(O, golden):
    for (k, m) in [(3, 2), (4, 2), (10, 4), (16, 4)]:
        assert np.array_equal(O.cauchy(k, m), golden["gen_%d_%d" % (k, m)])
    assert np.array_equal(np.array([O.gf_exp(i) for i in range(255)], np.uint8), golden["gf_exp"])


def test_encode_rebuild_match_golden(O, golden):
    for ci, (k, m, B, fb, nb, e, S) in enumerate(golden["cases"]):
        k, m, B, fb, nb, e, S = map(int, (k, m, B, fb, nb, e, S))
        assert O.shard_size(B, k) == S
        data = O.fill_blocks(SEED, fb, nb, B, k, S)
        assert hashlib.sha256(data.tobytes()).digest() == golden["case%d_data_sha256" % ci].tobytes()
        par = O.encode(k, m, S, data)
        assert np.array_equal(par, golden["case%d_parity" % ci]), ci
        s, l = O.erasures(SEED, fb, nb, k, m, e)
        assert np.array_equal(s, golden["case%d_surv" % ci])
        assert np.array_equal(l, golden["case%d_lost" % ci])
        for b in range(nb):
            assert np.array_equal(O.decode_matrix(k, m, s[b], l[b]), golden["case%d_rows" % ci][b])
        surv = O.gather(k, m, S, data, par, s)
        want = O.gather(k, m, S, data, par, l)
        assert np.array_equal(O.rebuild(k, m, S, s, surv, l), want)


@pytest.mark.parametrize("k,m", [(3, 2), (4, 2)])
def test_exhaustive_erasure_patterns(O, golden, k, m):
    lost_all = golden["exh_%d_%d_lost" % (k, m)]
    rows_all = golden["exh_%d_%d_rows" % (k, m)]
    S = 64
    data = O.fill_blocks(SEED, 11, 1, k * S, k, S)
    par = O.encode(k, m, S, data)
    full = np.concatenate([data.reshape(k, S), par.reshape(m, S)])
    for lp, want_rows in zip(lost_all, rows_all):
        lost = [int(x) for x in lp if x != 255]
        e = len(lost)
        surv = [i for i in range(k + m) if i not in lost][:k]
        assert np.array_equal(O.decode_matrix(k, m, surv, lost), want_rows[:e])
        out = O.rebuild(k, m, S, np.array([surv]), full[surv].reshape(1, -1), np.array([lost]))
        assert np.array_equal(out.reshape(e, S), full[lost])


def test_properties(O):
    k, m, S = 10, 4, 256
    a = O.fill_blocks(SEED, 1, 2, k * S, k, S)
    b = O.fill_blocks(SEED, 2, 2, k * S, k, S)
    # zero data -> zero parity; linearity; systematic identity
    assert not O.encode(k, m, S, np.zeros_like(a)).any()
    assert np.array_equal(O.encode(k, m, S, a ^ b), O.encode(k, m, S, a) ^ O.encode(k, m, S, b))
    C = O.cauchy(k, m)
    assert np.array_equal(C[:k], np.eye(k, dtype=np.uint8))
    # MDS: every k-subset of rows is invertible (sampled)
    rng = np.random.default_rng(0)
    for _ in range(200):
        rows = sorted(rng.choice(k + m, k, replace=False))
        inv = O.invert(C[rows])
        from oracle import rs_numpy as N
        assert np.array_equal(N.matmul(C[rows], inv), np.eye(k, dtype=np.uint8))


def test_threaded_baseline_matches_scalar(O):
    k, m, B = 10, 4, 100000
    S = O.shard_size(B, k)
    d = O.fill_blocks(SEED, 0, 9, B, k, S)
    assert np.array_equal(O.encode(k, m, S, d, threads=4), O.encode(k, m, S, d))
    s, l = O.erasures(SEED, 0, 9, k, m, 4)
    p = O.encode(k, m, S, d)
    surv = O.gather(k, m, S, d, p, s)
    assert np.array_equal(O.rebuild(k, m, S, s, surv, l, threads=3), O.gather(k, m, S, d, p, l))


def test_singular_survivors_rejected(O):
    with pytest.raises(ValueError):
        O.decode_matrix(4, 2, [0, 1, 1, 2], [3])


@pytest.mark.parametrize("k,m,S,n", [(10, 4, 104896, 3), (3, 2, 21888, 5), (16, 4, 256, 33),
                                     (4, 2, 1000, 7), (1, 1, 64, 3), (64, 16, 192, 2),
                                     (5, 3, 33, 4)])
def test_vectorised_baseline_matches_scalar(O, k, m, S, n):
    """oracle/rs_simd.c (the CPU baseline bench.py times) is bit-exact with
    the scalar oracle on every ISA this host has, aligned (streaming stores)
    and unaligned outputs, and odd shard sizes (scalar tail)."""
    rng = np.random.default_rng(k * 100 + m)
    data = O.aligned_empty((n, k * S))
    data[:] = rng.integers(0, 256, (n, k * S), dtype=np.uint8)
    ref = O.encode(k, m, S, data)
    for isa in range(O.simd_isa() + 1):
        out = O.aligned_empty((n, m * S))
        par, used = O.encode_simd(k, m, S, data, threads=3, isa=isa, out=out)
        assert used == isa and np.array_equal(par, ref), (isa, k, m, S)
        par, _ = O.encode_simd(k, m, S, data, threads=2, isa=isa)
        assert np.array_equal(par, ref), (isa, "unaligned")


def test_c1_round_trip(O):
    """BASELINE.json C1, the reference-runnable CPU case: RS(3,2) encode +
    rebuild of 1000 x 64 KiB blocks with e in {1, 2} random erasures per
    block; the rebuilt shards are bit-exact."""
    k, m, B, n = 3, 2, 65536, 1000
    S = O.shard_size(B, k)
    assert S == 21888
    data = O.fill_blocks(0x6D656D6F, 0, n, B, k, S)
    par = O.encode(k, m, S, data, threads=4)
    for e in (1, 2):
        surv, lost = O.erasures(0x6D656D6F, 0, n, k, m, e)
        shards = np.concatenate([data.reshape(n, k, S), par.reshape(n, m, S)], axis=1)
        got = O.rebuild(k, m, S, surv, O.gather(k, m, S, data, par, surv), lost, threads=4)
        want = np.take_along_axis(shards, lost.astype(np.int64)[:, :, None], axis=1)
        assert np.array_equal(got.reshape(n, e, S), want)


# Randomised agreement of the two restatements (C oracle vs the numpy one,
# which shares no code with it): any geometry, any block size, any seed.
from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(k=st.integers(1, 24), m=st.integers(1, 8), B=st.integers(0, 6000),
       seed=st.integers(0, 2**63 - 1), block=st.integers(0, 2**40), data=st.data())
def test_two_restatements_agree(O, k, m, B, seed, block, data):
    from oracle import rs_numpy as N
    S = O.shard_size(B, k)
    assert S == N.shard_size(B, k)
    d = O.fill_blocks(seed, block, 1, B, k, S)
    assert np.array_equal(d[0], N.fill_block(seed, block, B, k, S))
    par = O.encode(k, m, S, d)
    assert np.array_equal(par, N.encode(k, m, S, d))
    e = data.draw(st.integers(1, m))
    s, l = O.erasures(seed, block, 1, k, m, e)
    ns, nl = N.erasures(seed, block, k, m, e)
    assert list(s[0]) == list(ns) and list(l[0]) == list(nl)
    assert np.array_equal(O.decode_matrix(k, m, s[0], l[0]), N.decode_matrix(k, m, s[0], l[0]))
    got = O.rebuild(k, m, S, s, O.gather(k, m, S, d, par, s), l)
    assert np.array_equal(got, O.gather(k, m, S, d, par, l))


def test_c_oracle_matches_headline_digests(O):
    """The C oracle (rs_oracle.c) reproduces the numpy restatement's digests
    for the headline shapes' sample blocks (tests/golden/rs_headline.json):
    fill, parity and every rebuilt shard."""
    import hashlib
    import json
    with open(os.path.join(ROOT, "tests", "golden", "rs_headline.json")) as f:
        hl = json.load(f)
    sha = lambda x: hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()  # noqa: E731
    for bt in hl["batches"]:
        k, m, B, S = bt["k"], bt["m"], bt["block_bytes"], bt["shard_bytes"]
        for smp in bt["samples"]:
            b = smp["block"]
            data = O.fill_blocks(SEED, b, 1, B, k, S)
            assert sha(data) == smp["data_sha256"], (bt["name"], b)
            par = O.encode(k, m, S, data)
            assert sha(par) == smp["parity_sha256"], (bt["name"], b)
            for r in smp["rebuild"]:
                s, l = O.erasures(SEED, b, 1, k, m, r["e"])
                assert list(s[0]) == r["surv"] and list(l[0]) == r["lost"]
                out = O.rebuild(k, m, S, s, O.gather(k, m, S, data, par, s), l)
                assert sha(out) == r["out_sha256"], (bt["name"], b, r["e"])


@pytest.mark.parametrize("k,m,B", [(10, 4, 100000), (3, 2, 65536), (16, 4, 4096), (5, 3, 777)])
def test_simd_rebuild_matches_scalar(O, k, m, B):
    """oracle/rs_simd.c's rebuild (the CPU baseline of the rebuild configs)
    is bit-exact with the scalar oracle on every ISA this CPU has."""
    S = O.shard_size(B, k)
    n = 9
    data = O.fill_blocks(SEED, 3, n, B, k, S)
    par = O.encode(k, m, S, data)
    for e in sorted({1, m}):
        s, l = O.erasures(SEED, 3, n, k, m, e)
        surv = O.gather(k, m, S, data, par, s)
        want = O.gather(k, m, S, data, par, l)
        for isa in range(O.simd_isa() + 1):
            out, used = O.rebuild_simd(k, m, S, s, surv, l, threads=3, isa=isa)
            assert used == isa and np.array_equal(out, want), (k, m, B, e, isa)
