"""Multi-GPU partitioning of independent segments.

Segments share nothing, so N GPUs process contiguous blocks of segments with
no collective on the data path; the only cross-rank steps are a barrier and a
max-over-ranks of the timed interval (bench.py) — torch.distributed over RCCL
on GPUs, gloo on CPU (tests/test_multirank.py).
"""
from __future__ import annotations


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block partition: (first segment index, count) for `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def segment_seed(index: int) -> int:
    """Seed of synthetic segment `index` (0x5EED0000 + index)."""
    return 0x5EED0000 + index


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank float over the default process group (identity when
    torch.distributed is not initialised)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(value: int, device=None) -> int:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())
