"""Randomised soak of the C ABI, the way the plugin drives it: a few host
threads, one context each, issuing a seeded mix of encode, per-block rebuild
and one-pattern rebuild calls on device, pageable and pinned buffers, small
(zero-copy) and large (the copy pipeline, in 2 MiB batches) -- with
device calls left in flight
while host-memory calls run on the same context, whose per-block decode
scratch the two share (ordered by the ctx's ev_order event,
memo_amd/csrc/memo_ec.cpp).  Every output is checked against the C oracle."""
import threading

import numpy as np
import pytest

from conftest import SEED

pytestmark = pytest.mark.gpu


def _case(O, rng):
    k, m = int(rng.integers(1, 17)), int(rng.integers(1, 7))
    size = int(rng.integers(0, 4))
    B = (int(rng.integers(1, 5000)), int(rng.integers(5000, 300000)), 1 << 20, 4 << 20)[size]
    n = int(rng.integers(1, 9)) if size < 2 else int(rng.integers(1, 5))
    S = O.shard_size(B, k)
    fb = int(rng.integers(0, 1 << 20))
    data = O.fill_blocks(SEED, fb, n, B, k, S)
    return k, m, S, n, data, O.encode(k, m, S, data)


def test_soak_mixed_calls_threads(O, monkeypatch):
    import torch
    from memo_amd import ec
    # 2 MiB host-pipeline batches (read at ctx creation): calls past the
    # zero-copy limit stream through several batches of the 3-slot ring
    monkeypatch.setenv("MEMO_EC_PIPE_MB", "2")

    errs = []

    def buf(x, where):
        t = torch.from_numpy(np.ascontiguousarray(x))
        if where == "device":
            return t.cuda()
        return t.pin_memory() if where == "pinned" else t

    def empty(shape, where):
        if where == "device":
            # torch.empty launches nothing: a zero fill would run on torch's
            # stream, unordered with the codec's (non-blocking) ctx stream,
            # and could land after the kernel that writes the output
            return torch.empty(shape, dtype=torch.uint8, device="cuda")
        return torch.zeros(shape, dtype=torch.uint8, pin_memory=(where == "pinned"))

    def work(t):
        rng = np.random.default_rng(0x50A0 + t)
        try:
            with ec.Codec(0) as c:
                pending = []  # device calls not yet synchronized: (inputs, out, want, what)
                for it in range(120):
                    k, m, S, n, data, par = _case(O, rng)
                    op = int(rng.integers(0, 3))
                    where = ("device", "host", "pinned")[int(rng.integers(0, 3))]
                    what = (t, it, k, m, S, n, op, where)
                    if op == 0:
                        d, p = buf(data, where), empty((n, m * S), where)
                        c.encode(k, m, d, p)
                        inputs, out, want = [d], p, par
                    else:
                        e = int(rng.integers(1, m + 1))
                        if op == 1:  # every block its own pattern, shuffled survivors
                            sidx = np.stack([rng.permutation(k + m)[:k] for _ in range(n)]).astype(np.uint8)
                            lidx = np.stack([np.setdiff1d(np.arange(k + m), s)[rng.permutation(m)[:e]]
                                             for s in sidx]).astype(np.uint8)
                        else:  # one pattern for the batch
                            s0 = rng.permutation(k + m)[:k].astype(np.uint8)
                            l0 = np.setdiff1d(np.arange(k + m), s0)[rng.permutation(m)[:e]].astype(np.uint8)
                            sidx, lidx = np.tile(s0, (n, 1)), np.tile(l0, (n, 1))
                        surv = buf(O.gather(k, m, S, data, par, sidx), where)
                        out = empty((n, e * S), where)
                        want = O.gather(k, m, S, data, par, lidx)
                        if op == 1:
                            si = buf(sidx, "device" if where == "device" else "host")
                            li = buf(lidx, "device" if where == "device" else "host")
                            c.rebuild(k, m, si, surv, li, out)
                            inputs = [si, li, surv]
                        else:
                            c.rebuild_uniform(k, m, sidx[0], surv, lidx[0], out)
                            inputs = [surv]
                    if where == "device":
                        pending.append((inputs, out, want, what))
                        if len(pending) < 4 and rng.integers(0, 3):
                            continue  # leave it in flight under the next calls
                        c.synchronize()
                        for _, o, w, wh in pending:
                            if not np.array_equal(o.cpu().numpy(), w):
                                errs.append(("device", wh))
                        pending.clear()
                    elif not np.array_equal(out.numpy(), want):
                        errs.append(("host", what))
                c.synchronize()
                for _, o, w, wh in pending:
                    if not np.array_equal(o.cpu().numpy(), w):
                        errs.append(("device", wh))
        except Exception as ex:  # pragma: no cover
            errs.append(("exception", t, repr(ex)))

    ts = [threading.Thread(target=work, args=(t,)) for t in range(6)]
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    assert not errs, errs[:5]
