"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and
the golden fixtures, bit-exact.  Full-size configs (BASELINE.json C2/C3)
are checked through size-independent properties (rebuild round trips,
sampled blocks against the oracle)."""
import itertools
import os

import numpy as np
import pytest

from conftest import SEED

pytestmark = pytest.mark.gpu


def dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def empty(*shape):
    import torch
    return torch.empty(shape, dtype=torch.uint8, device="cuda")


def host(t):
    return t.cpu().numpy()


def fill(codec, fb, n, B, k, S):
    d = empty(n, k * S)
    codec.fill_blocks(SEED, fb, n, B, k, S, d)
    return d


def test_fill_matches_oracle(codec, O):
    for (B, k) in [(0, 3), (1, 3), (7, 4), (1000, 3), (4095, 4), (5000, 10), (1 << 16, 16)]:
        S = O.shard_size(B, k)
        d = fill(codec, 3, 5, B, k, S)
        codec.synchronize()
        assert np.array_equal(host(d), O.fill_blocks(SEED, 3, 5, B, k, S)), (B, k)


def test_golden_cases(codec, golden, O, rebuild_path):
    for ci, row in enumerate(golden["cases"]):
        k, m, B, fb, nb, e, S = map(int, row)
        d = fill(codec, fb, nb, B, k, S)
        p = empty(nb, m * S)
        codec.encode(k, m, d, p)
        codec.synchronize()
        assert np.array_equal(host(p), golden["case%d_parity" % ci]), ci
        s, l = dev(golden["case%d_surv" % ci]), dev(golden["case%d_lost" % ci])
        rows = empty(nb, e * k)
        codec.decode_rows(k, m, s, l, rows)
        codec.synchronize()
        assert np.array_equal(host(rows).reshape(nb, e, k), golden["case%d_rows" % ci]), ci
        surv = empty(nb, k * S)
        codec.gather_shards(k, m, S, nb, d, p, s, surv)
        out = empty(nb, e * S)
        codec.rebuild(k, m, s, surv, l, out)
        want = empty(nb, e * S)
        codec.gather_shards(k, m, S, nb, d, p, l, want)
        codec.synchronize()
        assert np.array_equal(host(out), host(want)), ci


CONFIGS = [(1, 1), (2, 1), (3, 2), (4, 2), (5, 3), (6, 3), (6, 6), (8, 5), (10, 4), (12, 4),
           (12, 7), (14, 2), (16, 4), (20, 8), (33, 12), (64, 16)]


@pytest.mark.parametrize("k,m", CONFIGS)
def test_encode_rebuild_vs_oracle(codec, O, k, m, rebuild_path):
    rng = np.random.default_rng(k * 100 + m)
    for B in [64 * k, 4096, 12345, 300000]:
        S = O.shard_size(B, k)
        n = int(rng.integers(1, 9))
        fb = int(rng.integers(0, 1000))
        d = fill(codec, fb, n, B, k, S)
        p = empty(n, m * S)
        codec.encode(k, m, d, p)
        data = O.fill_blocks(SEED, fb, n, B, k, S)
        want = O.encode(k, m, S, data)
        codec.synchronize()
        assert np.array_equal(host(p), want), (k, m, B)
        for e in sorted({1, m}):
            s, l = O.erasures(SEED, fb, n, k, m, e)
            surv = O.gather(k, m, S, data, want, s)
            out = empty(n, e * S)
            codec.rebuild(k, m, dev(s), dev(surv), dev(l), out)
            codec.synchronize()
            assert np.array_equal(host(out), O.gather(k, m, S, data, want, l)), (k, m, B, e)


@pytest.mark.parametrize("seed", range(int(os.environ.get("MEMO_EC_STRESS_SEEDS", "6"))))
def test_random_geometries_vs_oracle(codec, O, seed, rebuild_path):
    """Seeded random codes and sizes (k 1..24, m 1..10, B 1..200000 B, 1..12
    blocks, any e <= m, every block its own erasure pattern in a random
    survivor order), device and pageable-host buffers, encode, per-block
    rebuild and the one-pattern rebuild, all against the oracle.
    MEMO_EC_STRESS_SEEDS widens the seed range for a longer run."""
    rng = np.random.default_rng(0xC0DE + seed)
    for it in range(4):
        k, m = int(rng.integers(1, 25)), int(rng.integers(1, 11))
        B = int(rng.integers(1, 200001)) if it else int(rng.integers(1, 64))
        n = int(rng.integers(1, 13))
        S = O.shard_size(B, k)
        fb = int(rng.integers(0, 1 << 20))
        data = O.fill_blocks(SEED, fb, n, B, k, S)
        want = O.encode(k, m, S, data)
        case = (seed, it, k, m, B, n)
        p = empty(n, m * S)
        codec.encode(k, m, dev(data), p)
        ph = np.zeros((n, m * S), np.uint8)
        codec.encode(k, m, data, ph)
        codec.synchronize()
        assert np.array_equal(host(p), want), case
        assert np.array_equal(ph, want), case
        e = int(rng.integers(1, m + 1))
        surv_idx = np.stack([rng.permutation(k + m)[:k] for _ in range(n)]).astype(np.uint8)
        lost_idx = np.stack([np.setdiff1d(np.arange(k + m), s)[rng.permutation(m)[:e]]
                             for s in surv_idx]).astype(np.uint8)
        surv = O.gather(k, m, S, data, want, surv_idx)
        lost = O.gather(k, m, S, data, want, lost_idx)
        out = empty(n, e * S)
        codec.rebuild(k, m, dev(surv_idx), dev(surv), dev(lost_idx), out)
        oh = np.zeros((n, e * S), np.uint8)
        codec.rebuild(k, m, surv_idx, surv, lost_idx, oh)
        codec.synchronize()
        assert np.array_equal(host(out), lost), case + (e,)
        assert np.array_equal(oh, lost), case + (e,)
        # one pattern for the batch: block 0's
        su = np.repeat(surv_idx[:1], n, axis=0)
        lu = np.repeat(lost_idx[:1], n, axis=0)
        ou = empty(n, e * S)
        codec.rebuild_uniform(k, m, surv_idx[0], dev(O.gather(k, m, S, data, want, su)), lost_idx[0], ou)
        codec.synchronize()
        assert np.array_equal(host(ou), O.gather(k, m, S, data, want, lu)), case + (e, "uniform")


@pytest.fixture
def split_launches(codec):
    with codec.options(max_launch_tiles=600):  # 22 1-MiB RS(10,4) blocks per launch
        yield


def test_batches_split_across_launches(codec, O, split_launches, rebuild_path):
    """A batch larger than one launch's grid is split into several MAC
    launches (memo_ec.cpp max_blocks_per_launch); the bound is lowered so the
    split happens at a testable size.  Encode and rebuild, device and host."""
    k, m, B, n = 10, 4, 1 << 20, 64
    S = O.shard_size(B, k)
    data = O.fill_blocks(SEED, 9, n, B, k, S)
    want = O.encode(k, m, S, data, threads=4)
    p = empty(n, m * S)
    codec.encode(k, m, dev(data), p)
    codec.synchronize()
    assert np.array_equal(host(p), want)
    hp = np.zeros_like(want)
    codec.encode(k, m, data, hp)
    assert np.array_equal(hp, want)
    s, l = O.erasures(SEED, 9, n, k, m, 3)
    surv = O.gather(k, m, S, data, want, s)
    out = empty(n, 3 * S)
    codec.rebuild(k, m, dev(s), dev(surv), dev(l), out)
    codec.synchronize()
    assert np.array_equal(host(out), O.gather(k, m, S, data, want, l))
    # one pattern for every block (memo_ec_rebuild_uniform), split the same way
    su, lu = s[0], l[0]
    svu = O.gather(k, m, S, data, want, np.tile(su, (n, 1)))
    outu = empty(n, 3 * S)
    codec.rebuild_uniform(k, m, su, dev(svu), lu, outu)
    codec.synchronize()
    assert np.array_equal(host(outu), O.gather(k, m, S, data, want, np.tile(lu, (n, 1))))


def test_c1_full_size_vs_oracle(codec, O):
    """BASELINE.json C1 at its full size: RS(3,2) encode + rebuild of 1000 x
    64 KiB blocks, e in {1, 2} random erasures per block, bit-exact against
    the oracle (the whole batch, not a sample)."""
    k, m, B, n = 3, 2, 65536, 1000
    S = O.shard_size(B, k)
    data = O.fill_blocks(SEED, 0, n, B, k, S)
    want = O.encode(k, m, S, data, threads=4)
    d = fill(codec, 0, n, B, k, S)
    p = empty(n, m * S)
    codec.encode(k, m, d, p)
    codec.synchronize()
    assert np.array_equal(host(d), data)
    assert np.array_equal(host(p), want)
    for e in (1, 2):
        s, l = O.erasures(SEED, 0, n, k, m, e)
        surv = empty(n, k * S)
        codec.gather_shards(k, m, S, n, d, p, dev(s), surv)
        out = empty(n, e * S)
        codec.rebuild(k, m, dev(s), surv, dev(l), out)
        codec.synchronize()
        assert np.array_equal(host(out), O.gather(k, m, S, data, want, l)), e


@pytest.mark.parametrize("k,m", [(3, 2), (4, 2), (6, 3), (10, 4), (12, 4), (16, 4)])
def test_every_erasure_pattern_in_one_batch(codec, O, k, m, rebuild_path):
    """Each block of the batch has a different erasure pattern (per-block
    decode tables in one launch): for every e = 1..m, every set of e lost
    shards of the code (C(k+m, e) blocks; RS(16,4): 20 + 190 + 1140 + 4845),
    rebuilt from the first k survivors, against the oracle's gather of the
    encoded shards."""
    for e in range(1, m + 1):
        pats = list(itertools.combinations(range(k + m), e))
        n, B = len(pats), 3000 if k <= 4 else 1000
        S = O.shard_size(B, k)
        data = O.fill_blocks(SEED, e, n, B, k, S)
        par = O.encode(k, m, S, data)
        lost = np.array(pats, dtype=np.uint8)
        surv = np.array([[i for i in range(k + m) if i not in p][:k] for p in pats], dtype=np.uint8)
        sv = O.gather(k, m, S, data, par, surv)
        out = empty(n, e * S)
        codec.rebuild(k, m, dev(surv), dev(sv), dev(lost), out)
        codec.synchronize()
        assert np.array_equal(host(out), O.gather(k, m, S, data, par, lost)), (k, m, e)


@pytest.mark.parametrize("k,m", [(1, 1), (2, 2), (3, 2), (4, 2), (6, 3), (7, 5), (8, 8), (10, 4),
                                 (12, 4), (14, 2), (16, 4), (16, 16), (20, 8), (33, 12), (64, 16)])
@pytest.mark.parametrize("kernel", ["wide", "per_block", "per_block_staged", "per_block_generic"])
def test_decode_rows_vs_oracle(codec, O, k, m, kernel):
    """Closed-form decode rows against the oracle's Gauss-Jordan rows
    C[lost] * inv(C[surv]): random survivor orders, lost shards that are
    data, parity or themselves survivors (unit rows), e = 1..m, over 700
    blocks (several workgroups).  Both kernels: column-per-lane
    (decode_coef_wide_kernel: forced by decode_exact=0 for every k) and
    one lane per block (decode_rows_k_kernel for k in {2, 3, 4, 6, 8, 10,
    12, 14, 16}, decode_coef_kernel otherwise -- forced by decode_wide_max=0
    -- or with decode_exact=0).  The exact-k kernel stores whole-dword rows from
    registers, other rows through LDS (all of them with decode_stage=1)."""
    with codec.options(**DECODE_KERNELS[kernel]):
        _decode_rows_vs_oracle(codec, O, k, m)


DECODE_KERNELS = {"wide": {"decode_exact": 0, "decode_wide_max": 1 << 20}, "per_block": {"decode_wide_max": 0},
                  "per_block_staged": {"decode_wide_max": 0, "decode_stage": 1},
                  "per_block_generic": {"decode_wide_max": 0, "decode_exact": 0}}


def _decode_rows_vs_oracle(codec, O, k, m):
    rng = np.random.default_rng(k * 1000 + m)
    n = 700
    for e in sorted({1, (m + 1) // 2, m}):
        surv = np.stack([rng.permutation(k + m)[:k] for _ in range(n)]).astype(np.uint8)
        lost = np.stack([rng.permutation(k + m)[:e] for _ in range(n)]).astype(np.uint8)
        rows = empty(n, e * k)
        codec.decode_rows(k, m, dev(surv), dev(lost), rows)
        codec.synchronize()
        got = host(rows).reshape(n, e, k)
        for b in range(0, n, 7):
            want = O.decode_matrix(k, m, surv[b], lost[b])
            assert np.array_equal(got[b], want), (k, m, e, b)


def test_one_huge_ragged_block(codec, O):
    """One 1 GiB + 7 byte block (RS(10,4): S = 107,374,208, the last data
    shard mostly padding): encode and a 4-erasure rebuild, the whole block
    against the oracle."""
    k, m, B, n = 10, 4, (1 << 30) + 7, 1
    S = O.shard_size(B, k)
    data = O.fill_blocks(SEED, 9001, n, B, k, S)
    want = O.encode(k, m, S, data, threads=8)
    d = dev(data)
    p = empty(n, m * S)
    codec.encode(k, m, d, p)
    codec.synchronize()
    assert np.array_equal(host(p), want)
    s = np.array([[3, 4, 5, 6, 7, 8, 10, 11, 12, 13]], np.uint8)
    l = np.array([[0, 9, 1, 2]], np.uint8)
    surv = empty(n, k * S)
    codec.gather_shards(k, m, S, n, d, p, dev(s), surv)
    del d
    out = empty(n, 4 * S)
    codec.rebuild(k, m, dev(s), surv, dev(l), out)
    codec.synchronize()
    assert np.array_equal(host(out), O.gather(k, m, S, data, want, l))


def test_block_beyond_32bit_offsets(codec, O):
    """One 5 GiB + 3 byte RS(2,1) block: S = 2.5 GiB (above 2^31), the
    second data shard and the block's end past 2^32 bytes, so every shard
    and column offset needs 64 bits.  Encode, then rebuild data shard 0 from
    (data shard 1, parity) on both rebuild paths, whole shards against the
    oracle."""
    k, m, B, n = 2, 1, (5 << 30) + 3, 1
    S = O.shard_size(B, k)
    assert S > (1 << 31) and k * S > (1 << 32)
    data = O.fill_blocks(SEED, 77, n, B, k, S)
    par, _ = O.encode_simd(k, m, S, data, threads=16)
    d = empty(n, k * S)
    codec.fill_blocks(SEED, 77, n, B, k, S, d)
    p = empty(n, m * S)
    codec.encode(k, m, d, p)
    codec.synchronize()
    assert np.array_equal(host(p), par)
    s, l = np.array([[1, 2]], np.uint8), np.array([[0]], np.uint8)
    surv = empty(n, k * S)
    codec.gather_shards(k, m, S, n, d, p, dev(s), surv)
    del d, p
    for path, img in ((0, 0), (0, 1), (1, 0)):
        out = empty(n, S)
        with codec.options(rebuild_path=path, image_min_tiles=img, image_min_coefs=0):
            codec.rebuild(k, m, dev(s), surv, dev(l), out)
            codec.synchronize()
        assert np.array_equal(host(out)[0], data[0, :S]), (path, img)
        del out


def test_small_blocks_many_per_tile(codec, O, rebuild_path):
    # 4 KiB blocks with k=16: S=256, 16 columns per block, tables for ~17
    # blocks per tile in the rebuild kernel.
    k, m, B, n = 16, 4, 4096, 300
    S = O.shard_size(B, k)
    data = O.fill_blocks(SEED, 40, n, B, k, S)
    par = O.encode(k, m, S, data)
    d = dev(data)
    p = empty(n, m * S)
    codec.encode(k, m, d, p)
    s, l = O.erasures(SEED, 40, n, k, m, 4)
    out = empty(n, 4 * S)
    codec.rebuild(k, m, dev(s), dev(O.gather(k, m, S, data, par, s)), dev(l), out)
    codec.synchronize()
    assert np.array_equal(host(p), par)
    assert np.array_equal(host(out), O.gather(k, m, S, data, par, l))


def test_mixed_segments_one_launch(codec, O):
    segs, want = [], []
    for i, (k, m, B, n) in enumerate([(4, 2, 4096, 37), (10, 4, 1 << 20, 3), (16, 4, 65536, 11),
                                      (10, 4, 16384, 20), (4, 2, 4 << 20, 1)]):
        S = O.shard_size(B, k)
        data = O.fill_blocks(SEED, 100 * i, n, B, k, S)
        p = empty(n, m * S)
        segs.append((k, m, S, n, dev(data), p))
        want.append(O.encode(k, m, S, data))
    codec.encode_segments(segs)
    codec.synchronize()
    for (k, m, S, n, d, p), w in zip(segs, want):
        assert np.array_equal(host(p), w), (k, m, S)


@pytest.mark.parametrize("codes", [
    [(3, 2, 5000, 9), (7, 3, 70000, 4), (20, 4, 300000, 3), (12, 1, 4096, 40), (16, 4, 4096, 33)],
    [(4, 2, 4096, 5), (10, 6, 100000, 2), (2, 1, 64, 300)],  # R > 4: the chunk loop
    [(6, 3, 4096, 9), (6, 6, 30000, 3), (12, 4, 70000, 2), (14, 1, 4096, 20), (12, 5, 999, 7)],
])
def test_mixed_segments_any_k(codec, O, codes):
    """Mixed k in one launch, including k outside {4, 10, 16}, k > 16 and
    m > 4 (gf_mac_multi_kernel's variable-k body and its fallbacks)."""
    segs, want = [], []
    for i, (k, m, B, n) in enumerate(codes):
        S = O.shard_size(B, k)
        data = O.fill_blocks(SEED, 1000 + 100 * i, n, B, k, S)
        p = empty(n, m * S)
        segs.append((k, m, S, n, dev(data), p))
        want.append(O.encode(k, m, S, data))
    codec.encode_segments(segs)
    codec.synchronize()
    for (k, m, S, n, d, p), w in zip(segs, want):
        assert np.array_equal(host(p), w), (k, m, S)


def test_host_memory_paths(codec, O):
    import torch
    k, m, B, n = 10, 4, 1 << 20, 70  # > one 64 MiB pipeline batch
    S = O.shard_size(B, k)
    data = O.fill_blocks(SEED, 5, n, B, k, S)
    want = O.encode(k, m, S, data)
    par = np.zeros((n, m * S), np.uint8)
    codec.encode(k, m, data, par)                       # pageable
    assert np.array_equal(par, want)
    pd = torch.from_numpy(data).pin_memory()
    pp = torch.zeros((n, m * S), dtype=torch.uint8).pin_memory()
    codec.encode(k, m, pd, pp)                          # pinned
    assert np.array_equal(pp.numpy(), want)
    s, l = O.erasures(SEED, 5, n, k, m, 3)
    surv = O.gather(k, m, S, data, want, s)
    out = np.zeros((n, 3 * S), np.uint8)
    codec.rebuild(k, m, s, surv, l, out)
    assert np.array_equal(out, O.gather(k, m, S, data, want, l))


@pytest.mark.parametrize("zc_kb", [256, 0])
def test_small_host_calls(codec, O, zc_kb):
    """One-block and few-block calls from pageable and pinned host memory,
    with the zero-copy path (kernels on pinned host memory) and without it
    (DMA copies)."""
    with codec.options(zero_copy_bytes=zc_kb << 10):
        _small_host_calls(codec, O)


def _small_host_calls(codec, O):
    import torch
    k, m = 10, 4
    for B, n in ((4096, 1), (100000, 3), (4096, 7)):
        S = O.shard_size(B, k)
        data = O.fill_blocks(SEED, 500 + n, n, B, k, S)
        want = O.encode(k, m, S, data)
        par = np.zeros((n, m * S), np.uint8)
        codec.encode(k, m, data, par)
        assert np.array_equal(par, want), (B, n)
        pd = torch.from_numpy(data).pin_memory()
        pp = torch.zeros((n, m * S), dtype=torch.uint8).pin_memory()
        codec.encode(k, m, pd, pp)
        assert np.array_equal(pp.numpy(), want), (B, n)
        for e in (1, m):
            s, l = O.erasures(SEED, 500 + n, n, k, m, e)
            surv = O.gather(k, m, S, data, want, s)
            out = np.zeros((n, e * S), np.uint8)
            codec.rebuild(k, m, s, surv, l, out)
            assert np.array_equal(out, O.gather(k, m, S, data, want, l)), (B, n, e)


def test_singular_survivors_reported(codec, rebuild_path):
    from memo_amd import ec
    k, m, S, n = 4, 2, 64, 2
    surv = dev(np.array([[0, 1, 2, 3], [0, 1, 1, 2]], np.uint8))  # block 1: duplicate
    lost = dev(np.array([[4], [3]], np.uint8))
    out = empty(n, S)
    codec.rebuild(k, m, surv, empty(n, k * S).zero_(), lost, out)
    with pytest.raises(ec.MemoECError) as ei:
        codec.synchronize()
    assert ei.value.code == -4
    codec.synchronize()  # error is cleared


@pytest.mark.parametrize("kernel", ["wide", "per_block", "per_block_staged", "per_block_generic"])
def test_invalid_sets_give_zero_rows(codec, O, kernel):
    """Duplicate survivors, a survivor index >= k+m and a lost index >= k+m
    zero that block's rows (only that block's) and raise ESINGULAR once."""
    with codec.options(**DECODE_KERNELS[kernel]):
        _invalid_sets_give_zero_rows(codec, O)


def _invalid_sets_give_zero_rows(codec, O):
    from memo_amd import ec
    k, m, e = 10, 4, 2
    surv = np.array([list(range(10)), [0, 1, 2, 3, 4, 5, 6, 7, 8, 8], [0, 1, 2, 3, 4, 5, 6, 7, 8, 14],
                     [13, 1, 2, 3, 4, 5, 6, 7, 8, 9], list(range(10))], np.uint8)
    lost = np.array([[10, 11], [10, 11], [10, 11], [0, 12], [11, 14]], np.uint8)
    rows = empty(5, e * k)
    codec.decode_rows(k, m, dev(surv), dev(lost), rows)
    with pytest.raises(ec.MemoECError) as ei:
        codec.synchronize()
    assert ei.value.code == -4
    got = host(rows).reshape(5, e, k)
    for b in (1, 2, 4):
        assert not got[b].any(), b
    for b in (0, 3):
        assert np.array_equal(got[b], O.decode_matrix(k, m, surv[b], lost[b])), b
    codec.synchronize()


@pytest.mark.parametrize("B,n", [(1 << 16, 40), (4096, 5)])
def test_singular_survivors_reported_host_paths(codec, O, monkeypatch, B, n, rebuild_path):
    """Host-memory rebuilds report a bad survivor set from any pipeline batch
    (the status word is read behind the last batch) or from a small
    zero-copy call (status word in the pinned slot), the good blocks are
    still rebuilt, and the error does not leak into the next call."""
    import torch
    from memo_amd import ec
    k, m = 4, 2
    S = O.shard_size(B, k)
    monkeypatch.setenv("MEMO_EC_PIPE_MB", "1")  # several pipeline batches
    if n > 5:
        monkeypatch.setenv("MEMO_EC_ZC_KB", "0")  # the copy pipeline, not zero-copy
    c2 = ec.Codec(0)  # the pipeline size is read at ctx creation
    data = O.fill_blocks(SEED, 0, n, B, k, S)
    par = O.encode(k, m, S, data)
    s, l = O.erasures(SEED, 0, n, k, m, 1)
    surv = O.gather(k, m, S, data, par, s)
    want = O.gather(k, m, S, data, par, l)
    bad = s.copy()
    bad[3, 1] = bad[3, 0]  # a duplicate survivor in the first batch
    for pinned in (False, True):
        sv = torch.from_numpy(surv).pin_memory() if pinned else surv
        out = torch.zeros((n, S), dtype=torch.uint8).pin_memory() if pinned else np.zeros((n, S), np.uint8)
        with pytest.raises(ec.MemoECError) as ei:
            c2.rebuild(k, m, bad, sv, l, out)
        assert ei.value.code == -4
        got = np.asarray(out)
        good = np.ones(n, bool)
        good[3] = False
        assert np.array_equal(got[good], want.reshape(n, S)[good])
        c2.rebuild(k, m, s, sv, l, out)  # clean call afterwards: no stale error
        assert np.array_equal(np.asarray(out), want.reshape(n, S))
    del c2


def test_noops_and_argument_errors(codec):
    from memo_amd import ec
    d = empty(1, 10 * 64)
    codec.encode(10, 4, d, empty(0), S=64, n=0)
    with pytest.raises(ec.MemoECError):
        codec.encode(10, 4, d, empty(1, 4 * 64), S=48, n=1)   # S not a multiple of 64
    with pytest.raises(ec.MemoECError):
        codec.encode(65, 4, d, empty(1, 4 * 64), S=64, n=1)   # k beyond limit
    codec.synchronize()


def test_call_size_overflow_refused(codec):
    """Block counts whose byte products overflow, or pass 2^50 bytes, are
    refused with ERANGE before any scratch or grid is sized from them and
    before anything is launched (the ctx stays usable).  Each call's n is
    taken just past 2^50 bytes, past 2^64 (a wrapping product), and 2^62."""
    import ctypes
    from memo_amd import ec
    L = ec._lib()
    d = empty(1, 16 * 64)
    p = d.data_ptr()
    cx = codec._ctx

    def ns(per):
        return [(1 << 50) // per + 1, (1 << 64) // per + 1, 1 << 62]

    for n in ns(14 * 64):
        assert L.memo_ec_encode_batch(cx, 10, 4, 64, n, p, p, 2) == -6, n
    for n in ns(14 * 64 + 14):
        assert L.memo_ec_rebuild_batch(cx, 10, 4, 64, n, p, p, p, 4, p, 2) == -6, n
        assert L.memo_ec_rebuild_uniform(cx, 10, 4, 64, n, p, p, p, 4, p, 2) == -6, n
        seg = ec.RebuildSegment(k=10, m=4, S=64, n=n, surv_idx=p, surv=p, lost_idx=p, e=4,
                                uniform=0, out=p)
        assert L.memo_ec_rebuild_segments(cx, 1, ctypes.byref(seg), 2) == -6, n
    for n in ns(4 * 10 + 14):
        assert L.memo_ec_decode_rows(cx, 10, 4, n, p, p, 4, p) == -6, n
    for n in ns(10 * 64):
        assert L.memo_ec_fill_blocks(cx, 1, 0, n, 64, 10, 64, p) == -6, n
    for n in ns(4 * 64 + 4):
        assert L.memo_ec_gather_shards(cx, 10, 4, 64, n, p, p, p, 4, p) == -6, n
    codec.synchronize()
    assert L.memo_ec_encode_batch(cx, 10, 4, 64, 1, p, p, 2) == 0
    codec.synchronize()


def test_full_size_c2_c3_round_trip(codec, O, rebuild_path):
    """BASELINE.json C2/C3 at full size (4096 x 1 MiB, RS(10,4), e=4), the
    WHOLE batch against the CPU oracle: all 4096 blocks' data and parity
    (vectorised oracle encode, oracle/rs_simd.c, bit-exact with the scalar
    oracle) and all 4096 x 4 rebuilt shards (the oracle's own per-block
    decode rows + vectorised MAC); then data shards alone (lost = all
    parity) re-encode identically."""
    import torch
    k, m, B, n, e = 10, 4, 1 << 20, 4096, 4
    S = O.shard_size(B, k)
    d = fill(codec, 0, n, B, k, S)
    p = empty(n, m * S)
    codec.encode(k, m, d, p)
    s, l = ec_erasures(n, k, m, e)
    sd, ld = dev(s), dev(l)
    surv = empty(n, k * S)
    codec.gather_shards(k, m, S, n, d, p, sd, surv)
    out = empty(n, e * S)
    codec.rebuild(k, m, sd, surv, ld, out)
    codec.synchronize()
    data = O.fill_blocks(SEED, 0, n, B, k, S)
    assert np.array_equal(host(d), data)
    par, _ = O.encode_simd(k, m, S, data, threads=16)
    assert np.array_equal(host(p), par)
    del surv
    hs = O.gather(k, m, S, data, par, s)
    want, _ = O.rebuild_simd(k, m, S, s, hs, l, threads=16)
    del hs
    assert np.array_equal(host(out), want)
    assert np.array_equal(want, O.gather(k, m, S, data, par, l))
    del want, out
    # data shards alone (lost = all parity) re-encode identically
    lp = dev(np.tile(np.arange(k, k + m, dtype=np.uint8), (n, 1)))
    sp = dev(np.tile(np.arange(k, dtype=np.uint8), (n, 1)))
    out2 = empty(n, m * S)
    codec.rebuild(k, m, sp, d, lp, out2)
    codec.synchronize()
    assert torch.equal(out2, p)


@pytest.mark.parametrize("k,m,B,n", [(10, 4, 1 << 20, 4096), (16, 4, 4096, 1 << 20)])
def test_full_size_linearity(codec, k, m, B, n, rebuild_path):
    """Size-independent properties of the code at full headline size (C2 /
    C3's 4096 x 1 MiB RS(10,4) and the 1M x 4 KiB RS(16,4) batch), over the
    whole batch: encode and rebuild are GF(2)-linear, enc(a ^ b) = enc(a) ^
    enc(b) and rebuild(a ^ b) = rebuild(a) ^ rebuild(b) with the same
    erasure patterns; zero data encodes and rebuilds to zero."""
    import torch
    S = _shard_size(B, k)
    e = m
    a, b = fill(codec, 0, n, B, k, S), fill(codec, n, n, B, k, S)
    pa, pb, pab = empty(n, m * S), empty(n, m * S), empty(n, m * S)
    codec.encode(k, m, a, pa)
    codec.encode(k, m, b, pb)
    codec.synchronize()  # the codec's stream is not torch's: order by hand
    ab = torch.bitwise_xor(a, b)
    torch.cuda.synchronize()
    codec.encode(k, m, ab, pab)
    codec.synchronize()
    assert torch.equal(pab, torch.bitwise_xor(pa, pb))
    s, l = ec_erasures(n, k, m, e)
    sd, ld = dev(s), dev(l)
    ra, rb, rab = empty(n, e * S), empty(n, e * S), empty(n, e * S)
    surv = empty(n, k * S)
    for d, p, r in [(a, pa, ra), (b, pb, rb), (ab, pab, rab)]:
        codec.gather_shards(k, m, S, n, d, p, sd, surv)
        codec.rebuild(k, m, sd, surv, ld, r)
    codec.synchronize()
    assert torch.equal(rab, torch.bitwise_xor(ra, rb))
    del b, pb, rb, ab, pab, rab
    a.zero_()
    torch.cuda.synchronize()
    codec.encode(k, m, a, pa)
    codec.gather_shards(k, m, S, n, a, pa, sd, surv)
    codec.rebuild(k, m, sd, surv, ld, ra)
    codec.synchronize()
    assert not pa.any() and not ra.any()


def _shard_size(B, k):
    from memo_amd import ec
    return ec.shard_size(B, k)


@pytest.mark.parametrize("k,m", [(16, 4), (10, 4)])
def test_full_size_small_block_rebuild(codec, O, k, m):
    """bench.py's rebuild_small batches at full size: 1,048,576 x 4 KiB
    blocks, 4 random erasures each (every block its own decode rows), the
    WHOLE batch against the oracle (vectorised encode; per-block decode rows
    by the oracle + vectorised MAC) on the default rebuild path."""
    B, n, e = 4096, 1 << 20, 4
    S = O.shard_size(B, k)
    d = fill(codec, 0, n, B, k, S)
    p = empty(n, m * S)
    codec.encode(k, m, d, p)
    s, l = ec_erasures(n, k, m, e)
    sd, ld = dev(s), dev(l)
    surv = empty(n, k * S)
    codec.gather_shards(k, m, S, n, d, p, sd, surv)
    out = empty(n, e * S)
    codec.rebuild(k, m, sd, surv, ld, out)
    codec.synchronize()
    del surv
    data = O.fill_blocks(SEED, 0, n, B, k, S)
    assert np.array_equal(host(d), data)
    del d
    par, _ = O.encode_simd(k, m, S, data, threads=16)
    assert np.array_equal(host(p), par)
    del p
    hs = O.gather(k, m, S, data, par, s)
    want, _ = O.rebuild_simd(k, m, S, s, hs, l, threads=16)
    assert np.array_equal(host(out), want)


def ec_erasures(n, k, m, e):
    from memo_amd import ec
    return ec.erasures(SEED, 0, n, k, m, e)


def test_scratch_reuse_is_ordered(O):
    """Back-to-back rebuilds that reuse the ctx's decode-row scratch from
    different queues: an async device rebuild, then a host-memory rebuild
    (pipeline streams), then a switch to another stream and a second device
    rebuild.  Each must read its own rows."""
    import torch
    from memo_amd import ec
    k, m, B, n = 10, 4, 1 << 20, 64
    S = O.shard_size(B, k)
    data = O.fill_blocks(SEED, 77, n, B, k, S)
    par = O.encode(k, m, S, data, threads=4)
    cases = []
    for e, seed in ((4, 1), (2, 2), (3, 3)):
        s, l = O.erasures(SEED + seed, 77, n, k, m, e)
        cases.append((s, l, O.gather(k, m, S, data, par, s), O.gather(k, m, S, data, par, l)))
    with ec.Codec(0) as c:
        st_a, st_b = torch.cuda.Stream(), torch.cuda.Stream()
        c.set_stream(st_a)
        s, l, sv, want0 = cases[0]
        with torch.cuda.stream(st_a):
            sd, ld, svd = dev(s), dev(l), dev(sv)
            out0 = empty(n, 4 * S)
        torch.cuda.synchronize()
        c.rebuild(k, m, sd, svd, ld, out0)                   # async on st_a
        s1, l1, sv1, want1 = cases[1]
        out1 = np.zeros((n, 2 * S), np.uint8)
        c.rebuild(k, m, s1, sv1, l1, out1)                   # host pipeline
        s2, l2, sv2, want2 = cases[2]
        with torch.cuda.stream(st_b):
            sd2, ld2, svd2 = dev(s2), dev(l2), dev(sv2)
            out2 = empty(n, 3 * S)
        torch.cuda.synchronize()
        c.set_stream(st_a)
        c.rebuild(k, m, sd, svd, ld, out0)
        c.set_stream(st_b)
        c.rebuild(k, m, sd2, svd2, ld2, out2)                # async on st_b
        c.synchronize()
        torch.cuda.synchronize()
        assert np.array_equal(out1, want1)
        assert np.array_equal(host(out0), want0)
        assert np.array_equal(host(out2), want2)


def test_hip_graph_capture_replay(codec, O):
    """Device-resident encode + rebuild captured into one HIP graph (via
    torch.cuda.CUDAGraph on ROCm) and replayed on new inputs: launch-bound
    callers can replay instead of re-launching."""
    import torch
    k, m, B, n, e = 10, 4, 200000, 24, 3
    S = O.shard_size(B, k)
    d = empty(n, k * S)
    p = empty(n, m * S)
    s, l = O.erasures(SEED, 0, n, k, m, e)
    sd, ld = dev(s), dev(l)
    surv = empty(n, k * S)
    out = empty(n, e * S)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        codec.set_stream(st)
        codec.fill_blocks(SEED, 0, n, B, k, S, d)
        codec.encode(k, m, d, p)                      # warm-up: table cache, scratch
        codec.gather_shards(k, m, S, n, d, p, sd, surv)
        codec.rebuild(k, m, sd, surv, ld, out)
    torch.cuda.synchronize()
    # the uniform rebuild's table image is formed on its first call, before
    # capture (a capture may only enqueue work)
    su, lu = s[0], l[0]
    sdu = dev(np.tile(su, (n, 1)))
    survu = empty(n, k * S)
    outu = empty(n, e * S)
    with torch.cuda.stream(st):
        codec.gather_shards(k, m, S, n, d, p, sdu, survu)
        codec.rebuild_uniform(k, m, su, survu, lu, outu)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cs = torch.cuda.current_stream()
        codec.set_stream(cs)
        codec.encode(k, m, d, p)
        codec.gather_shards(k, m, S, n, d, p, sd, surv)
        codec.rebuild(k, m, sd, surv, ld, out)
        codec.gather_shards(k, m, S, n, d, p, sdu, survu)
        codec.rebuild_uniform(k, m, su, survu, lu, outu)
    codec.set_stream(None)
    for fb in [100, 200]:
        codec.fill_blocks(SEED, fb, n, B, k, S, d)
        codec.synchronize()
        g.replay()
        torch.cuda.synchronize()
        data = O.fill_blocks(SEED, fb, n, B, k, S)
        want = O.encode(k, m, S, data)
        assert np.array_equal(host(p), want)
        assert np.array_equal(host(out), O.gather(k, m, S, data, want, l))
        assert np.array_equal(host(outu), O.gather(k, m, S, data, want, np.tile(lu, (n, 1))))


def test_concurrent_contexts_from_threads(O):
    """One context per thread, all encoding at once (memo's background pool,
    elle/src/elle/reactor/scheduler.cc:562-602): contexts are independent."""
    import threading
    import torch
    from memo_amd import ec
    k, m, B, n = 10, 4, 65536, 64
    S = O.shard_size(B, k)
    errs, results = [], {}

    def work(t):
        try:
            with ec.Codec(0) as c:
                d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
                p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
                for it in range(5):
                    c.fill_blocks(SEED, 1000 * t + it, n, B, k, S, d)
                    c.encode(k, m, d, p)
                c.synchronize()
                results[t] = host(p)
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    ts = [threading.Thread(target=work, args=(t,)) for t in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    for t in range(6):
        data = O.fill_blocks(SEED, 1000 * t + 4, n, B, k, S)
        assert np.array_equal(results[t], O.encode(k, m, S, data))


def test_concurrent_host_calls_from_threads(O):
    """The plugin's usage: pool threads, one ctx each, issuing host-memory
    encode and degraded-read rebuilds of mixed sizes at once (zero-copy and
    copy-pipeline calls interleaved), every result checked."""
    import threading
    from memo_amd import ec
    k, m = 10, 4
    cases = []
    for i, (B, n) in enumerate([(4096, 1), (65536, 3), (1 << 20, 6), (4096, 40), (300000, 20)]):
        S = O.shard_size(B, k)
        data = O.fill_blocks(SEED, 7000 + i, n, B, k, S)
        par = O.encode(k, m, S, data)
        s, l = O.erasures(SEED, 7000 + i, n, k, m, 2)
        cases.append((S, n, data, par, s, O.gather(k, m, S, data, par, s), l,
                      O.gather(k, m, S, data, par, l)))
    errs = []

    def work(t):
        try:
            with ec.Codec(0) as c:
                for it in range(12):
                    S, n, data, par, s, surv, l, want = cases[(t + it) % len(cases)]
                    p = np.zeros((n, m * S), np.uint8)
                    c.encode(k, m, data, p)
                    if not np.array_equal(p, par):
                        errs.append(("encode", t, it))
                    out = np.zeros((n, 2 * S), np.uint8)
                    c.rebuild(k, m, s, surv, l, out)
                    if not np.array_equal(out, want):
                        errs.append(("rebuild", t, it))
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    ts = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs


@pytest.mark.parametrize("k,m,B", [(10, 4, 4096), (16, 4, 4096), (4, 2, 100), (3, 2, 5000),
                                   (2, 2, 64), (5, 3, 4096), (12, 4, 7000), (20, 8, 3000),
                                   (64, 16, 5000), (10, 4, 300000)])
def test_fused_rebuild_random_orders(codec, O, k, m, B):
    """The fused rebuild (each tile decodes its blocks' rows itself) on
    per-block random survivor orders and lost sets that mix data, parity and
    survivor shards (unit rows), over tiles holding 1 to 65 blocks (S = 64
    packs 4 columns per block) and through the generic chunk loop (k = 5,
    20, 64), against the true shards."""
    rng = np.random.default_rng(k * 7 + m + B)
    S = O.shard_size(B, k)
    n = 300
    data = O.fill_blocks(SEED, 11, n, B, k, S)
    par = O.encode(k, m, S, data)
    for e in sorted({1, m}):
        surv = np.stack([rng.permutation(k + m)[:k] for _ in range(n)]).astype(np.uint8)
        lost = np.stack([rng.permutation(k + m)[:e] for _ in range(n)]).astype(np.uint8)
        sv = O.gather(k, m, S, data, par, surv)
        out = empty(n, e * S)
        codec.rebuild(k, m, dev(surv), dev(sv), dev(lost), out)
        codec.synchronize()
        assert np.array_equal(host(out), O.gather(k, m, S, data, par, lost)), (k, m, B, e)


@pytest.mark.parametrize("B", [4096, 1 << 20])
def test_fused_invalid_sets_zero_only_that_block(codec, O, B):
    """Duplicate survivors, a survivor index >= k+m and a lost index >= k+m
    zero that block's output only (its neighbours in the same tile are
    rebuilt) and raise ESINGULAR once."""
    from memo_amd import ec
    k, m, e = 10, 4, 2
    S = O.shard_size(B, k)
    n = 6
    data = O.fill_blocks(SEED, 3, n, B, k, S)
    par = O.encode(k, m, S, data)
    surv = np.array([list(range(10)), [0, 1, 2, 3, 4, 5, 6, 7, 8, 8], [0, 1, 2, 3, 4, 5, 6, 7, 8, 14],
                     [13, 1, 2, 3, 4, 5, 6, 7, 8, 9], list(range(10)), [12, 1, 2, 3, 4, 5, 6, 7, 8, 9]],
                    np.uint8)
    lost = np.array([[10, 11], [10, 11], [10, 11], [0, 12], [11, 14], [0, 9]], np.uint8)
    sv = O.gather(k, m, S, data, par, np.minimum(surv, k + m - 1))
    out = empty(n, e * S)
    codec.rebuild(k, m, dev(surv), dev(sv), dev(lost), out)
    with pytest.raises(ec.MemoECError) as ei:
        codec.synchronize()
    assert ei.value.code == -4
    got = host(out).reshape(n, e * S)
    for b in (1, 2, 4):
        assert not got[b].any(), b
    for b in (0, 3, 5):
        assert np.array_equal(got[b], O.gather(k, m, S, data[b:b + 1], par[b:b + 1],
                                               lost[b:b + 1]).reshape(-1)), b
    codec.synchronize()


def test_device_fault_does_not_leak_into_host_pipeline(O, monkeypatch):
    """A device rebuild with a bad survivor set, then a good host-memory
    rebuild through the copy pipeline on the same ctx: the host call
    succeeds (its own status word), and the device fault is still reported
    by the next synchronize."""
    from memo_amd import ec
    k, m, B, n = 4, 2, 1 << 16, 40
    S = O.shard_size(B, k)
    monkeypatch.setenv("MEMO_EC_PIPE_MB", "1")
    monkeypatch.setenv("MEMO_EC_ZC_KB", "0")
    data = O.fill_blocks(SEED, 0, n, B, k, S)
    par = O.encode(k, m, S, data)
    s, l = O.erasures(SEED, 0, n, k, m, 1)
    surv = O.gather(k, m, S, data, par, s)
    want = O.gather(k, m, S, data, par, l)
    bad = s.copy()
    bad[5, 1] = bad[5, 0]
    with ec.Codec(0) as c:
        c.rebuild(k, m, dev(bad), dev(surv), dev(l), empty(n, S))   # device, async, faulty
        out = np.zeros((n, S), np.uint8)
        c.rebuild(k, m, s, surv, l, out)                             # host pipeline, good
        assert np.array_equal(out, want.reshape(n, S))
        with pytest.raises(ec.MemoECError) as ei:
            c.synchronize()
        assert ei.value.code == -4
        c.synchronize()


def _headline():
    import json
    import os
    from conftest import ROOT
    with open(os.path.join(ROOT, "tests", "golden", "rs_headline.json")) as f:
        return json.load(f)


def _sha(x):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["C2_C3", "C1", "small_16_4", "small_10_4", "C5_4MiB_4_2"])
def test_headline_batches_vs_numpy_digests(codec, name, rebuild_path):
    """Each headline batch (BASELINE.json C1/C2/C3, the 4 KiB rebuild_small
    batches, 4 MiB RS(4,2)) runs whole on the GPU -- encode, then a rebuild
    with the batch's random erasure patterns -- and its sample blocks' data,
    parity and rebuilt shards match the SHA-256 digests of the independent
    numpy restatement (tests/golden/rs_headline.json, make_headline.py)."""
    import torch
    from memo_amd import ec
    bt = [b for b in _headline()["batches"] if b["name"] == name][0]
    k, m, B, n, S = bt["k"], bt["m"], bt["block_bytes"], bt["blocks"], bt["shard_bytes"]
    assert ec.shard_size(B, k) == S
    d = fill(codec, 0, n, B, k, S)
    p = empty(n, m * S)
    codec.encode(k, m, d, p)
    codec.synchronize()
    for smp in bt["samples"]:
        b = smp["block"]
        assert _sha(host(d[b])) == smp["data_sha256"], (name, b)
        assert _sha(host(p[b])) == smp["parity_sha256"], (name, b)
    for e in bt["erasures"]:
        s, l = ec.erasures(SEED, 0, n, k, m, e)
        sd, ld = dev(s), dev(l)
        surv = empty(n, k * S)
        codec.gather_shards(k, m, S, n, d, p, sd, surv)
        out = empty(n, e * S)
        codec.rebuild(k, m, sd, surv, ld, out)
        codec.synchronize()
        for smp in bt["samples"]:
            b = smp["block"]
            r = [x for x in smp["rebuild"] if x["e"] == e][0]
            assert list(s[b]) == r["surv"] and list(l[b]) == r["lost"], (name, b, e)
            assert _sha(host(out[b])) == r["out_sha256"], (name, b, e)
        del surv, out
    del d, p
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k,m", [(3, 2), (4, 2), (10, 4), (16, 4), (6, 3), (12, 4), (20, 8), (64, 16)])
def test_rebuild_uniform_vs_oracle(codec, O, k, m):
    """One erasure pattern for a whole batch (the repair of one lost node):
    device-resident and host-memory calls (zero-copy and pipeline), lost
    shards that are data, parity or survivors (unit rows), against the
    true shards."""
    import torch
    rng = np.random.default_rng(k * 31 + m)
    for B, n in [(4096, 300), (100000, 5), (1 << 20, 70)]:
        S = O.shard_size(B, k)
        data = O.fill_blocks(SEED, 50, n, B, k, S)
        par = O.encode(k, m, S, data, threads=4)
        for e in sorted({1, m}):
            perm = rng.permutation(k + m)
            surv = np.sort(perm[:k]).astype(np.uint8) if e % 2 else perm[:k].astype(np.uint8)
            lost = rng.permutation(k + m)[:e].astype(np.uint8)
            s_all = np.tile(surv, (n, 1))
            want = O.gather(k, m, S, data, par, np.tile(lost, (n, 1)))
            sv = O.gather(k, m, S, data, par, s_all)
            out = empty(n, e * S)
            codec.rebuild_uniform(k, m, surv, dev(sv), lost, out)
            codec.synchronize()
            assert np.array_equal(host(out), want), (k, m, B, e, "device")
            ho = np.zeros((n, e * S), np.uint8)
            codec.rebuild_uniform(k, m, surv, sv, lost, ho)
            assert np.array_equal(ho, want), (k, m, B, e, "host")
            po = torch.zeros((n, e * S), dtype=torch.uint8).pin_memory()
            codec.rebuild_uniform(k, m, surv, torch.from_numpy(sv).pin_memory(), lost, po)
            assert np.array_equal(po.numpy(), want), (k, m, B, e, "pinned")


def test_rebuild_uniform_invalid_and_cache(codec, O):
    """An invalid pattern is refused before anything is enqueued; more
    distinct patterns than the ctx caches (64) are each rebuilt right."""
    from memo_amd import ec
    k, m, B, n = 10, 4, 5000, 7
    S = O.shard_size(B, k)
    sv = empty(n, k * S).zero_()
    out = empty(n, S)
    for surv, lost in ([[0, 1, 2, 3, 4, 5, 6, 7, 8, 8], [9]], [[0, 1, 2, 3, 4, 5, 6, 7, 8, 14], [9]],
                       [list(range(10)), [14]]):
        with pytest.raises(ec.MemoECError) as ei:
            codec.rebuild_uniform(k, m, surv, sv, lost, out)
        assert ei.value.code == -4
    codec.synchronize()
    data = O.fill_blocks(SEED, 1, n, B, k, S)
    par = O.encode(k, m, S, data)
    rng = np.random.default_rng(5)
    for i in range(80):
        perm = rng.permutation(k + m)
        surv, lost = perm[:k].astype(np.uint8), perm[k:k + 2].astype(np.uint8)
        o = empty(n, 2 * S)
        codec.rebuild_uniform(k, m, surv, dev(O.gather(k, m, S, data, par, np.tile(surv, (n, 1)))),
                              lost, o)
        codec.synchronize()
        assert np.array_equal(host(o), O.gather(k, m, S, data, par, np.tile(lost, (n, 1)))), i


def test_ctx_options_round_trip(codec):
    """memo_ec_ctx_set_option / get_option: every option reads back what was
    set, out-of-range values and unknown options are refused (EINVAL) and
    leave the option unchanged, and a fresh ctx starts from the environment
    defaults, not from another ctx's settings."""
    from memo_amd import ec
    values = {"rebuild_path": 0, "fused_max_bytes": 1 << 20, "zero_copy_bytes": 0,
              "pipe_bytes": 8 << 20, "copy_threads": 2, "max_launch_tiles": 1000,
              "xcd_min_tiles": 1, "decode_wide_max": 0, "decode_exact": 0, "decode_stage": 1,
              "image_min_tiles": 1, "image_min_coefs": 0, "decode_overlap": 0}
    old = {k: codec.get_option(k) for k in values}
    with codec.options(**values):
        assert {k: codec.get_option(k) for k in values} == values
        with ec.Codec(0) as fresh:
            assert {k: fresh.get_option(k) for k in values} == old
    assert {k: codec.get_option(k) for k in values} == old
    for name, bad in [("rebuild_path", 2), ("rebuild_path", -2), ("pipe_bytes", 1000),
                      ("decode_exact", 3), ("copy_threads", -1), ("image_min_tiles", -1),
                      ("image_min_coefs", -1), ("decode_overlap", 2), ("decode_overlap", -1)]:
        with pytest.raises(ec.MemoECError) as ei:
            codec.set_option(name, bad)
        assert ei.value.code == -1
        assert codec.get_option(name) == old[name]
    L = ec._lib()
    assert L.memo_ec_ctx_set_option(codec._ctx, 99, 0) == -1


def test_env_options_keep_their_meanings(monkeypatch, capfd):
    """The environment defaults keep what each variable meant when every
    call read it: any nonzero MEMO_EC_REBUILD_FUSED forces the fused path
    (negative: auto), MEMO_EC_COPY_THREADS=0 copies on the calling thread
    only; an unusable value is ignored with a warning on stderr."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from memo_amd import ec
    for val, want in [("2", 1), ("1", 1), ("0", 0), ("-1", -1), ("-7", -1)]:
        monkeypatch.setenv("MEMO_EC_REBUILD_FUSED", val)
        with ec.Codec(0) as c:
            assert c.get_option("rebuild_path") == want, val
            assert c.rebuild_path(1, 16, 1 << 30) == ("fused" if want == 1 else "images")
            assert c.rebuild_path(1, 4, 1 << 30, 2) == ("fused" if want == 1 else "rows")
            assert c.rebuild_path(1 << 20, 16, 256) == ("fused" if want == 1 else "rows")
    monkeypatch.delenv("MEMO_EC_REBUILD_FUSED")
    for val, want in [("0", 0), ("1", 1), ("16", 16)]:
        monkeypatch.setenv("MEMO_EC_IMAGE_MIN_TILES", val)
        monkeypatch.setenv("MEMO_EC_IMAGE_MIN_COEFS", val)
        with ec.Codec(0) as c:
            assert c.get_option("image_min_tiles") == want, val
            assert c.get_option("image_min_coefs") == want, val
    monkeypatch.delenv("MEMO_EC_IMAGE_MIN_TILES")
    monkeypatch.delenv("MEMO_EC_IMAGE_MIN_COEFS")
    with ec.Codec(0) as c:
        assert (c.get_option("image_min_tiles"), c.get_option("image_min_coefs")) == (1, 40)
        assert c.get_option("decode_overlap") == 1
    monkeypatch.setenv("MEMO_EC_DECODE_OVERLAP", "0")
    with ec.Codec(0) as c:
        assert c.get_option("decode_overlap") == 0
    monkeypatch.delenv("MEMO_EC_DECODE_OVERLAP")
    monkeypatch.setenv("MEMO_EC_COPY_THREADS", "0")
    with ec.Codec(0) as c:
        assert c.get_option("copy_threads") == 1
    monkeypatch.setenv("MEMO_EC_COPY_THREADS", "lots")
    capfd.readouterr()
    with ec.Codec(0) as c:
        assert c.get_option("copy_threads") == 0
    assert "ignoring MEMO_EC_COPY_THREADS=lots" in capfd.readouterr().err


def test_rebuild_path_label_follows_ctx_options(codec):
    """Codec.rebuild_path reads the ctx's own options (bench.py labels its
    rebuild kernel with it), not the environment."""
    with codec.options(rebuild_path=-1, fused_max_bytes=1 << 20):
        assert codec.rebuild_path(16, 10, 4096) == "fused"
        assert codec.rebuild_path(1024, 10, 2048) == "rows"
    with codec.options(rebuild_path=1):
        assert codec.rebuild_path(1 << 20, 10, 1 << 20) == "fused"
        assert "gf_rebuild_kernel" in codec.rebuild_kernel_name(1 << 20, 10, 1 << 20)
    with codec.options(rebuild_path=0, image_min_tiles=1, image_min_coefs=40):
        assert codec.rebuild_path(1, 16, 64) == "rows"
        assert codec.rebuild_path(1, 16, 4096 - 64) == "rows"     # less than one whole tile
        assert codec.rebuild_path(1, 16, 4096) == "images"        # RS(16,4): 64 coefficients
        assert codec.rebuild_path(1, 10, 1 << 20) == "images"     # RS(10,4): 40
        assert codec.rebuild_path(1, 6, 1 << 20, 3) == "rows"     # RS(6,3): 18
        assert codec.rebuild_path(1, 4, 1 << 20, 2) == "rows"     # RS(4,2): 8
        assert codec.rebuild_path(1, 8, 1 << 20) == "images"      # k = 8: chunk-loop body
        assert "table images" in codec.rebuild_kernel_name(1, 16, 1 << 20)
    with codec.options(rebuild_path=0, image_min_tiles=0):
        assert codec.rebuild_path(1, 16, 1 << 30) == "rows"


@pytest.mark.parametrize("kin,r,B,n", [(10, 4, 1 << 20, 64), (16, 4, 4096, 3000), (4, 2, 5000, 33),
                                        (7, 3, 70000, 9), (20, 6, 4096, 100)])
def test_stream_probe_bytes(codec, kin, r, B, n):
    """memo_ec_stream_probe writes out shard i of block b = XOR of its kin
    input shards, every byte XOR i (the encode's traffic without the GF
    arithmetic), for straight-line and chunked shard counts."""
    import torch
    from memo_amd import ec
    S = ec.shard_size(B, kin)
    rng = np.random.default_rng(kin * 1000 + n)
    x = rng.integers(0, 256, size=(n, kin * S), dtype=np.uint8)
    out = torch.full((n, r * S), 0xA5, dtype=torch.uint8, device="cuda")
    codec.stream_probe(kin, r, dev(x), out)
    codec.synchronize()
    acc = np.bitwise_xor.reduce(x.reshape(n, kin, S), axis=1)
    want = np.stack([acc ^ np.uint8(i) for i in range(r)], axis=1).reshape(n, r * S)
    assert np.array_equal(host(out), want)
    # the one-sided modes run (read: out untouched for these inputs; write:
    # every output byte written) and a bad mode is refused
    codec.stream_probe(kin, r, dev(x), out, "read")
    codec.synchronize()
    assert np.array_equal(host(out), want)
    codec.stream_probe(kin, r, dev(x), out, "write")
    codec.synchronize()
    assert not np.array_equal(host(out), want)
    L = ec._lib()
    assert L.memo_ec_stream_probe(codec._ctx, kin, r, S, n, out.data_ptr(), out.data_ptr(), 3) == -1


def test_device_identity(codec):
    """memo_ec_device_identity: the PCI bus id torch reports for cuda:0
    and a 32-digit UUID; a missing device is ENODEV, short buffers EINVAL."""
    import ctypes
    import re
    import torch
    from memo_amd import ec
    ident = ec.device_identity(0)
    assert re.fullmatch(r"[0-9a-fA-F]{4}:[0-9a-fA-F]{2}:[0-9a-fA-F]{2}\.[0-9a-fA-F]", ident["pci_bus_id"])
    assert re.fullmatch(r"[0-9a-f]{32}", ident["uuid"])
    props = torch.cuda.get_device_properties(0)
    if hasattr(props, "pci_bus_id"):
        assert int(ident["pci_bus_id"].split(":")[1], 16) == props.pci_bus_id
    L = ec._lib()
    buf = ctypes.create_string_buffer(64)
    assert L.memo_ec_device_identity(ec._lib().memo_ec_device_count(), buf, 64, buf, 64) == -5
    assert L.memo_ec_device_identity(0, buf, 8, buf, 64) == -1
