"""GPU batched SHA-256 (the CHB address hash, CHB.cc:264-289) against the
FIPS 180 known answers and hashlib (OpenSSL, the hash elle::cryptography
uses in the reference)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KATS = [  # FIPS 180-2 / NIST CAVP examples
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    (b"a" * 1000000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
]


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_fips_known_answers(codec):
    import torch
    for msg, want in KATS:
        buf = np.zeros((1, max(len(msg), 16) + 16), np.uint8)
        buf[0, :len(msg)] = np.frombuffer(msg, np.uint8)
        out = torch.empty((1, 32), dtype=torch.uint8, device="cuda")
        codec.sha256(_dev(buf), out, uniform_len=len(msg))
        codec.synchronize()
        assert out.cpu().numpy().tobytes().hex() == want, msg[:10]


@pytest.mark.parametrize("P", [0, 32, 64, 7])
def test_random_batches_vs_hashlib(codec, P):
    import torch
    rng = np.random.default_rng(P)
    n, stride = 300, 4096 + 64
    msg = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    lens = rng.integers(0, stride, n).astype(np.int64)
    lens[:70] = np.arange(70)          # every padding boundary around 55/56/64
    pre = rng.integers(0, 256, (n, max(P, 1)), dtype=np.uint8)[:, :P] if P else None
    out = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    codec.sha256(_dev(msg), out, prefix=_dev(pre) if P else None, msg_len=_dev(lens))
    codec.synchronize()
    got = out.cpu().numpy()
    for i in range(n):
        h = hashlib.sha256()
        if P:
            h.update(pre[i].tobytes())
        h.update(msg[i, :lens[i]].tobytes())
        assert got[i].tobytes() == h.digest(), i


def test_chb_addresses_of_encoded_batch(codec, O):
    """CHB addresses of a whole batch of 1 MiB blocks (salt||owner prefix,
    data = the padded block's first B bytes): the write path's hash."""
    import torch
    k, B, n = 10, 1 << 20, 8
    S = O.shard_size(B, k)
    d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    codec.fill_blocks(0x6D656D6F, 0, n, B, k, S, d)
    salt_owner = np.random.default_rng(1).integers(0, 256, (n, 64), dtype=np.uint8)
    out = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    codec.sha256(d, out, prefix=_dev(salt_owner), uniform_len=B)
    codec.synchronize()
    data = d.cpu().numpy()
    for i in range(n):
        assert out[i].cpu().numpy().tobytes() == hashlib.sha256(
            salt_owner[i].tobytes() + data[i, :B].tobytes()).digest()
