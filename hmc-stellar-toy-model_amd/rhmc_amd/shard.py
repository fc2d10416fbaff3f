"""Chain sharding across GPUs (one process per GPU).

Chains are independent: rank r of N takes a contiguous slice of the chain
index range and runs it on its own GPU with its own copy of the image.  There
is no exchange step during sampling; the only collectives are host-side:
a barrier, a max-reduction of timings and an optional final gather of the
chain states to rank 0 (torch.distributed, gloo on CPU tensors)."""
import numpy as np


def shard_range(n_total, world, rank):
    """Contiguous [lo, hi) of rank `rank`; the first n_total % world ranks get
    one extra chain."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(int(n_total), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_chains(local, n_total, dist=None):
    """Gather per-rank [n_local, ...] float64 arrays into [n_total, ...] on
    rank 0 (None elsewhere).  Host-side (gloo-compatible)."""
    import torch
    if dist is None:
        import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    local = np.ascontiguousarray(local, dtype=np.float64)
    tail = local.shape[1:]
    sizes = [shard_range(n_total, world, r) for r in range(world)]
    width = max(hi - lo for lo, hi in sizes)
    buf = torch.zeros((width,) + tail, dtype=torch.float64)
    buf[:local.shape[0]] = torch.from_numpy(local)
    outs = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=outs, dst=0)
    if rank != 0:
        return None
    return np.concatenate([outs[r][:hi - lo].numpy() for r, (lo, hi) in enumerate(sizes)])


def max_over_ranks(value, dist=None):
    """Max of a host float over all ranks (the bench's timing rule)."""
    import torch
    if dist is None:
        import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, dist=None):
    """Sum of a host number over all ranks (e.g. the chain-steps each rank did)."""
    import torch
    if dist is None:
        import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
