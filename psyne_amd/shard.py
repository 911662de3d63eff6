"""Message sharding across ranks: one process per GPU, independent shards.

TDT messages are independent, so a batch splits into contiguous per-rank shards with no data
exchange: the only collectives are the timing barrier and the max/min reductions of
bench.py.  Shards are balanced by BYTES (an exclusive prefix sum of message sizes cut at the
k/N quantiles), which matters for the Zipf-sized mix (BASELINE.json configs[3]) where message
counts and bytes are far apart.
"""
from __future__ import annotations

import numpy as np


def shard_bounds(sizes, world: int) -> np.ndarray:
    """Message index bounds (world + 1 entries): rank r owns messages [b[r], b[r+1]).

    Cut points are the first message whose byte prefix reaches r/world of the total, so every
    shard is contiguous and the byte imbalance is at most one message."""
    sizes = np.asarray(sizes, dtype=np.int64)
    n = sizes.size
    if world < 1:
        raise ValueError("world must be >= 1")
    pre = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(sizes, out=pre[1:])
    total = int(pre[-1])
    b = np.empty(world + 1, dtype=np.int64)
    b[0], b[world] = 0, n
    for r in range(1, world):
        if total == 0:
            b[r] = (n * r) // world
        else:
            b[r] = int(np.searchsorted(pre, (total * r + world - 1) // world, side="left"))
    return np.maximum.accumulate(b)


def shard_offsets(offsets, bounds, rank: int) -> np.ndarray:
    """Offsets of rank's shard rebased to 0 (what its device batch is built from)."""
    off = np.asarray(offsets, dtype=np.int64)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    return off[lo:hi + 1] - off[lo]


def reduce_max(value: float, device=None) -> float:
    """Max over ranks (bench.py's whole-job time); identity without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_true(flag: bool, device=None) -> bool:
    """Logical AND over ranks (every rank's round trip verified)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def reduce_sum(value: float, device=None) -> float:
    """Sum over ranks (the job's payload bytes); identity without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
