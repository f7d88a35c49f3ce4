"""Multi-GPU layout of one large buffer.

The buffer is split into contiguous shards aligned to deflate's 1 MiB segment
(restart) interval, one per rank; every rank deflates its shard with halo 0
and final = (last rank), so the shards are independent segments and their
streams concatenate, in rank order, into one valid raw DEFLATE stream whose
segment markers let inflate run segment-parallel.  There is no collective on
the data path; only timing uses a max-reduction (and the ratio a sum), over
gloo on the host.
"""
SEGMENT = 1 << 20


def shard_range(n, world, rank, align=SEGMENT):
    """[lo, hi) of rank's shard: contiguous, aligned to `align`, tiling [0, n)."""
    units = (n + align - 1) // align
    per, extra = divmod(units, world)
    lo_u = rank * per + min(rank, extra)
    hi_u = lo_u + per + (1 if rank < extra else 0)
    return min(n, lo_u * align), min(n, hi_u * align)


def max_over_ranks(value, dist=None, device="cpu"):
    """Max of a float over all ranks (the bench's timing rule)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, dist=None):
    """Sum of an integer over all ranks (total compressed bytes)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return int(value)
    import torch

    t = torch.tensor([int(value)], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
