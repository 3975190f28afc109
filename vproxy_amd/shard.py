"""Packet sharding across GPUs: packets are independent, so each rank takes a
contiguous descriptor range and runs its own stream; no collective touches the data path."""
from __future__ import annotations

import numpy as np


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Packet i goes to rank floor(i * world / n): contiguous, sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return (n * rank) // world, (n * (rank + 1)) // world


def shard_by_bytes(lengths: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous ranges with (nearly) equal byte totals, for ragged batches (C3/C4):
    boundaries from a prefix sum over the lengths."""
    lengths = np.asarray(lengths, dtype=np.int64)
    n = len(lengths)
    if n == 0:
        return [(0, 0)] * world
    cs = np.cumsum(lengths)
    total = int(cs[-1])
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cs, total * r / world, side="left")) + 1)
    cuts.append(n)
    cuts = [min(max(c, 0), n) for c in cuts]
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def rank_seed_first_index(n_per_rank: int, rank: int) -> int:
    """Disjoint synthetic sub-streams per rank: rank r generates packets [r*n, (r+1)*n) of the
    counter-based stream, so every rank's bytes differ and any packet can be regenerated."""
    return n_per_rank * rank


def max_over_ranks(x: float) -> float:
    """Max of a float over all ranks (bench timing); identity without torch.distributed."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float) -> float:
    """Sum of a float over all ranks (bench: algorithmic bytes of all shards); identity without
    torch.distributed."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def all_ranks_ok(ok: bool) -> bool:
    """True only if every rank reports ok (bench verify gate)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def gather_over_ranks(obj) -> list:
    """Every rank's `obj` (a small JSON-able value) in rank order; [obj] without torch.distributed
    (bench: per-rank kernel times and devices of a multi-GPU line)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
