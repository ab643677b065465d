"""Multi-rank path on CPU (gloo, world_size 2): block-index partition is
disjoint and complete, per-rank synthetic inputs equal the single-rank
global batch, and the job time is the max over ranks."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, SEED


def test_block_range_covers_exactly():
    from memo_amd.partition import block_range
    for n in [0, 1, 7, 4096, 32768]:
        for w in [1, 2, 3, 4, 8]:
            got = [block_range(n, w, r) for r in range(w)]
            assert sum(c for _, c in got) == n
            pos = 0
            for lo, c in got:
                assert lo == pos
                pos += c
    with pytest.raises(ValueError):
        block_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from memo_amd.partition import block_range, max_over_ranks
    from oracle import oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    k, m, B, n = 4, 2, 3000, 10
    S = O.shard_size(B, k)
    lo, cnt = block_range(n, world, rank)
    data = O.fill_blocks(SEED, lo, cnt, B, k, S)
    par = O.encode(k, m, S, data)
    # gather every rank's parity on rank 0 (test only: the product never does this)
    t = torch.from_numpy(np.ascontiguousarray(par.reshape(-1)))
    bufs = [torch.zeros_like(t) for _ in range(world)]  # equal shares: n % world == 0
    dist.all_gather(bufs, t)
    mx = max_over_ranks(0.5 + rank, dist)
    if rank == 0:
        q.put((mx, [b.numpy() for b in bufs]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_partition_gloo():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    mx, parts = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert mx == 1.5
    from oracle import oracle as O
    k, m, B, n = 4, 2, 3000, 10
    S = O.shard_size(B, k)
    whole = O.encode(k, m, S, O.fill_blocks(SEED, 0, n, B, k, S)).reshape(-1)
    assert np.array_equal(np.concatenate(parts), whole)


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    """bench.py's N>1 path end to end on the one GPU of a test box: two
    ranks under torch.distributed.run (gloo for the barrier/max, both ranks
    on cuda:0), each encoding its own block range; rank 0 prints one JSON
    line with the whole-job value.  The 8-GPU RCCL run is the driver's."""
    import json
    import subprocess
    import sys
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--same-device", "--dist-backend", "gloo", "--steps", "3", "--warmup", "2",
           "--blocks", "64", "--no-cpu", "--no-e2e"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_blocks"] == 128
    assert res["value"] > 0 and res["rebuild"]["round_trip_bit_exact"]
