"""Multi-GPU sharding of independent rollouts.

One process per GPU (``torch.distributed``; backend ``nccl`` = RCCL over xGMI on ROCm, ``gloo``
for the CPU tests).  Graphs are independent units: each rank takes a contiguous block of
graph ids and rolls them out with no data-path communication; the only collective is one
all-gather of the per-graph AUDC (float64) and removal counts (int32) at the end.
"""
import numpy as np


def shard(n_items, rank, world):
    """Contiguous block of [0, n_items) owned by `rank` (sizes differ by at most one)."""
    q, r = divmod(int(n_items), int(world))
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def gather_results(dist, audc, removals, device=None):
    """All-gather per-graph AUDC and removal counts of every rank (ordered by rank).

    dist: the ``torch.distributed`` module (initialised); device: tensor device for the
    collective ("cuda" under RCCL, None / "cpu" under gloo).  Blocks of different sizes are
    padded to the largest block and trimmed after the gather.
    """
    import torch
    world = dist.get_world_size()
    n = torch.tensor([len(audc)], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes) if sizes else 0
    a = torch.zeros(m, dtype=torch.float64, device=device)
    r = torch.zeros(m, dtype=torch.int32, device=device)
    if len(audc):
        a[: len(audc)] = torch.as_tensor(np.asarray(audc, dtype=np.float64), device=device)
        r[: len(removals)] = torch.as_tensor(np.asarray(removals, dtype=np.int32), device=device)
    ga = [torch.zeros_like(a) for _ in range(world)]
    gr = [torch.zeros_like(r) for _ in range(world)]
    dist.all_gather(ga, a)
    dist.all_gather(gr, r)
    out_a, out_r = [], []
    for k, s in enumerate(sizes):
        out_a.extend(ga[k][:s].cpu().tolist())
        out_r.extend(gr[k][:s].cpu().tolist())
    return out_a, out_r


def max_over_ranks(dist, value, device=None):
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, value, device=None):
    import torch
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
