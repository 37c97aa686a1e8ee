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


def shard_batch(idx: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """This rank's slice of one global batch of ray indices (contiguous, sizes differing by at most one) -- the
    data-parallel training split of one parent block: whole rays per rank, so each rank's BatchNorm chunks are
    the reference's chunks of its own batch."""
    n = idx.shape[0]
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return idx[start:start + q + (1 if rank < r else 0)]


def allreduce_grads(params, group=None, average=True) -> None:
    """Average the gradients of ``params`` over ranks with ONE all_reduce of a flat bucket (coarse + fine NOF =
    3.98 MB fp32: one ring over xGMI costs tens of microseconds against a ~1 s step, so there is nothing to gain
    from per-layer buckets or overlap with the backward).  Parameters without a gradient contribute zeros, so
    every rank issues the same collective."""
    if not dist.is_available() or not dist.is_initialized():
        return
    params = [p for p in params if p.requires_grad]
    if not params:
        return
    world = dist.get_world_size(group)
    flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params])
    dist.all_reduce(flat, group=group)
    if average:
        flat /= world
    o = 0
    for p in params:
        n = p.numel()
        g = flat[o:o + n].view_as(p)
        if p.grad is None:
            p.grad = g.clone()
        else:
            p.grad.copy_(g)
        o += n
