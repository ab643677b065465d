"""Block-index partitioning across the GPUs of one node.

Blocks are independent, so GPU g of G encodes/rebuilds the contiguous block
range [g*N/G, (g+1)*N/G) in its own HBM; no collective touches the data.
The only cross-rank traffic is the timing barrier and a max-reduction of
elapsed times (bench.py), over gloo on the host: there is no RCCL anywhere
on this path.

The reference fans a stored block out to its owners in parallel, one
coroutine per peer (Paxos::Details::send_immutable_block,
src/memo/model/doughnut/consensus/Paxos.cc:324-360); the GPU analogue is
one process per device, all started together (`launch_local_ranks`).
"""
import os
import socket
import subprocess
import sys
import time


def block_range(n_total, world, rank):
    """(first_block, count) of `rank`'s share of n_total blocks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi - lo


def weak_range(per_rank, rank):
    """Weak scaling: every rank owns `per_rank` blocks (BASELINE.json C4)."""
    return rank * per_rank, per_rank


def max_over_ranks(value, dist=None, device=None):
    """Max of a float over all ranks (the slowest rank sets the job time)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_env(rank, world, port, same_device=False, base=None):
    """Environment of local rank `rank` of `world` (torch.distributed env://
    rendezvous on 127.0.0.1).  LOCAL_RANK selects the GPU; with same_device
    every rank reports LOCAL_RANK 0 (N ranks rehearsed on one card)."""
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(0 if same_device else rank),
               LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    return env


def launch_local_ranks(script, argv, world, same_device=False, timeout=None):
    """Start `world` processes of `script argv` on this node, one per GPU,
    before this process touches any GPU (children are started, never
    exec'd), and wait for all of them.  If one fails the others are stopped
    (by their own PIDs).  Returns the first non-zero exit code, else 0."""
    if world < 1:
        raise ValueError("world must be >= 1")
    port = free_port()
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen([sys.executable, script] + list(argv),
                                      env=rank_env(r, world, port, same_device)))
    t0 = time.monotonic()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.terminate()
        if timeout is not None and time.monotonic() - t0 > timeout and live:
            for q in live:
                q.kill()
            rc = rc or 124
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def node_report(rows, bytes_key="payload_bytes", time_key="seconds"):
    """Per-rank rates and the whole-node figure of a weak-scaling run.

    rows: one dict per rank with the bytes it processed (`bytes_key`) in its
    own timed region of `time_key` seconds.  Per-GPU GiB/s = bytes_g / t_g;
    node sum = sum_g bytes_g / max_g t_g, since the job ends
    when the slowest GPU does."""
    if not rows:
        raise ValueError("no ranks")
    per = [r[bytes_key] / r[time_key] / 2**30 for r in rows]
    tmax = max(r[time_key] for r in rows)
    total = sum(r[bytes_key] for r in rows)
    return {"per_gpu_GiBs": [round(x, 3) for x in per],
            "node_sum_GiBs": round(total / tmax / 2**30, 3),
            "sum_of_per_gpu_GiBs": round(sum(per), 3),
            "slowest_rank": max(range(len(rows)), key=lambda i: rows[i][time_key])}
