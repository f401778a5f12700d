"""Utterance sharding across the GPUs of one node.

The forward has no cross-utterance dependency (every GroupNorm / attention mean is per utterance,
reference model/model.py:123-124,198,201,274,310-319), so a batch is split into contiguous
per-rank shards, each rank runs its shard on its own GPU with its own weight replica, and the only
communication is an optional gather of the outputs to one rank (never on the timed data path).
One process per GPU, launched by torchrun; `torch.distributed` over RCCL ("nccl") on the GPU
box, gloo in the CPU tests.
"""
from __future__ import annotations

import torch


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, end) of utterances owned by `rank` (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def run_shard(fn, x_all: torch.Tensor, rank: int, world: int):
    """Apply `fn` (e.g. a SeparationModel on this rank's device) to this rank's shard of x_all."""
    s, e = shard_range(x_all.shape[0], rank, world)
    return fn(x_all[s:e])


def gather_shards(local: torch.Tensor, n_total: int, group=None, dst: int = 0):
    """Gather variable-size shards (split by shard_range) to rank `dst`; returns the concatenated
    tensor on `dst` and None elsewhere. Shards are padded to the largest shard for the collective."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    cap = max(e - s for s, e in sizes)
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    if rank == dst:
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.gather(pad, gather_list=bufs, dst=dst, group=group)
        return torch.cat([bufs[r][: e - s] for r, (s, e) in enumerate(sizes)], dim=0)
    dist.gather(pad, dst=dst, group=group)
    return None
