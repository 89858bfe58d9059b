"""Multi-GPU partitioning for the encode+bitrot batch.

Objects (and their 1 MiB blocks) are independent: each rank owns a contiguous,
disjoint range of object ids and runs the kernels on its own GPU.  There is no
data-path collective; torch.distributed (gloo) carries only the timing barrier
and the max-over-ranks reduction of the bench.
"""
from __future__ import annotations

import os


def rank_env() -> tuple[int, int, int]:
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def object_range(rank: int, per_rank: int) -> tuple[int, int]:
    """Weak scaling: rank r owns object ids [r*per_rank, (r+1)*per_rank)."""
    return rank * per_rank, (rank + 1) * per_rank


def split_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Strong scaling (BASELINE config 4: a fixed stream split over N GPUs):
    contiguous near-equal ranges, the first total % world ranks one longer."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def max_over_ranks(values, world: int):
    """Max of each value over all ranks (timing: the slowest rank defines the step)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t]
