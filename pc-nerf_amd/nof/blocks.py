"""Parent-block sharding across the GPUs of one node.

PC-NeRF splits a scene into parent blocks, each with its own coarse/fine NOF pair; a block's rays never touch
another block's weights.  So the render path shards by block with no collective on the data path: rank r renders
blocks ``blocks_of_rank(r, world, n_blocks)``.  The only exchange is the final gather of per-ray outputs (depth,
flags or points) to the rank that writes them -- ``gather_rows`` -- which runs over RCCL (backend "nccl") on
MI355X and over gloo in the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def blocks_of_rank(rank: int, world: int, n_blocks: int) -> list[int]:
    """Contiguous block ranges, sizes differing by at most one (config 4: 4 blocks / 4 GPUs; config 5: 8 / 8)."""
    if not (0 <= rank < world) or n_blocks < 0:
        raise ValueError("bad rank/world/n_blocks")
    q, r = divmod(n_blocks, world)
    start = rank * q + min(rank, r)
    return list(range(start, start + q + (1 if rank < r else 0)))


def gather_rows(local: torch.Tensor, dst: int = 0, group=None) -> torch.Tensor | None:
    """Concatenate every rank's ``local`` rows (ragged first dimension) in rank order on ``dst``.

    Implemented as size exchange + padded all_gather (the collective RCCL implements best over xGMI); returns
    the concatenation on ``dst`` and None elsewhere.  Single-process: returns ``local``."""
    if not dist.is_available() or not dist.is_initialized():
        return local
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s) for s in sizes]
    m = max(sizes)
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    if rank != dst:
        return None
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], 0)


def max_over_ranks(value: float, device=None, group=None) -> float:
    """Max of a float over ranks (bench: the job's time is its slowest rank's)."""
    if not dist.is_available() or not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t)
