"""Parent-block sharding across the GPUs of one node.

PC-NeRF splits a scene into parent blocks, each with its own coarse/fine NOF pair; a block's rays never touch
another block's weights.  So the render path shards by block with no collective on the data path: rank r renders
blocks ``blocks_of_rank(r, world, n_blocks)``.  The only exchange is the final gather of per-ray outputs (depth,
flags or points) to the rank that writes them -- ``gather_rows`` -- which runs over RCCL (backend "nccl") on
MI355X and over gloo in the CPU tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def blocks_of_rank(rank: int, world: int, n_blocks: int) -> list[int]:
    """Contiguous block ranges, sizes differing by at most one (config 4: 4 blocks / 4 GPUs; config 5: 8 / 8)."""
    if not (0 <= rank < world) or n_blocks < 0:
        raise ValueError("bad rank/world/n_blocks")
    q, r = divmod(n_blocks, world)
    start = rank * q + min(rank, r)
    return list(range(start, start + q + (1 if rank < r else 0)))


def split_groups(group_col, world: int, start: int = 0, end: int | None = None) -> list[tuple[int, int]]:
    """Rows [start, end) of a two-step row table cut into ``world`` contiguous ranges of WHOLE ray groups with
    near-equal row counts (by parent block, then by contiguous ray groups; a group is never split, as
    in the reference's own batching, eval_kitti_render.py:1120-1130).  ``group_col``: column 12 of the rows (k-1 on
    a group's first row, -1 on its continuation rows).  Cut r goes to the group start nearest r/world of the rows,
    so no range is more than half a group (<= 14 rows on the reference's KITTI frames) off its share."""
    col = np.asarray(group_col).reshape(-1)
    end = col.shape[0] if end is None else int(end)
    if world < 1 or not 0 <= start <= end <= col.shape[0]:
        raise ValueError("bad world / row range")
    starts = start + np.flatnonzero(col[start:end] >= -0.5)
    bounds = [start]
    for r in range(1, world):
        target = start + r * (end - start) / world
        j = int(np.searchsorted(starts, target))
        cand = [c for c in (starts[j - 1] if j > 0 else start, starts[j] if j < starts.shape[0] else end)]
        pick = int(min(cand, key=lambda c: abs(c - target)))
        bounds.append(max(pick, bounds[-1]))
    bounds.append(end)
    return [(bounds[i], bounds[i + 1]) for i in range(world)]


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
