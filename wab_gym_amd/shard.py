"""Multi-GPU sharding of the env batch: independent shards, no collective.

Rank r of N owns global env ids [r*B, (r+1)*B).  Every random draw is keyed by the global
id, so the union of the shards reproduces one batch of N*B envs exactly (tested).  The
only collectives are out of the data path and run over a CPU (gloo) process group: a
barrier around the timed region, a MAX reduction of the elapsed time and a gather of the
per-rank figures (bench.py).  RCCL is never initialised.
"""
from __future__ import annotations

import os


def rank_info():
    """(rank, world, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def env_id_base(rank: int, batch_per_rank: int) -> int:
    return rank * batch_per_rank


def _initialised():
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def max_over_ranks(value: float) -> float:
    """MAX of a per-rank float over the default (CPU, gloo) process group; identity when not
    initialised."""
    import torch
    import torch.distributed as dist

    if not _initialised():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_objects(obj):
    """Every rank's `obj`, in rank order (a one-element list when not initialised)."""
    import torch.distributed as dist

    if not _initialised():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
