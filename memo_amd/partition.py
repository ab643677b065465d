"""Block-index partitioning across the GPUs of one node.

Blocks are independent, so GPU g of G encodes/rebuilds the contiguous block
range [g*N/G, (g+1)*N/G) in its own HBM; no collective touches the data.
The only cross-rank traffic is the timing barrier and a max-reduction of
elapsed times (bench.py).
"""


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
