"""Rank-independent BatchNorm running statistics under data parallelism.

In train mode every BatchNorm chunk of a NOF query updates running_mean / running_var with momentum, chunk after
chunk (models.py:183-203 under render.py:47-50's chunk loop; nn.BatchNorm1d's update: momentum x batch statistic +
(1 - momentum) x running, the variance unbiased).  Under data parallelism a rank sees only its slice of the global
batch, so left alone (Lightning's DDP default, no sync_batchnorm) every rank's running statistics follow its own
chunks and the ranks' checkpoints differ from each other and from a one-process run.

BnSync records, for each train-mode query of a step (nof._ops.query / nof_forward_embedded under the default train
math or the train fold), every chunk's batch mean (bias included) and biased variance -- read from the query's fold
state right after its forward, before the backward touches it -- together with the running statistics the step
started from.  ``sync()`` all-gathers every rank's records and replays the momentum updates from those starting
values over the chunks in GLOBAL order: for each query in call order, rank 0's chunks, then rank 1's, ... -- with
the forward's own arithmetic (pcnerf_bn_running_replay).  Every rank then holds exactly the statistics one process
gets by running the ranks' slices one after another, and num_batches_tracked counts every rank's chunks.

The batch statistics themselves (what normalises each chunk) stay per rank, as the reference computes them per
chunk of its own batch: only the running buffers -- what a checkpoint carries into eval mode -- are synchronised.

What the synchronised statistics equal, and what they do not: they are the ranks' slices run back to back, chunked
per rank.  They equal neither the reference's Lightning DDP checkpoint (rank 0's own statistics) nor a single process
running the GLOBAL batch, whose chunking differs whenever a rank's sample count is not a multiple of chunk (the
reference shell's 256 rays x 768 samples = 196,608 < 262,144 per rank: each rank one partial chunk, one process
262,144 + 131,072).  No reference run pins them: they are rank-independent by construction, parity-unpinned.

Under a layered train math (f16x2_3, f16x2_4, fp32) the queries keep no per-chunk record: sync() then warns once
and leaves each rank's running statistics as its own forward set them (per-rank, as before this module existed).
"""
from __future__ import annotations

import contextlib
import warnings

import torch
import torch.distributed as dist

from . import _ops


def _chunk_sizes(total: int, chunk: int) -> list[int]:
    return [min(chunk, total - c * chunk) for c in range(-(-total // chunk))]


class BnSync:
    """Record one step's BatchNorm chunk statistics (``with sync.record(): forward``) and make the running
    statistics rank-independent (``sync.sync()`` after the forward, on every rank)."""

    _warned = False

    def __init__(self):
        self._snap = {}    # id(model) -> (model, running_mean clones, running_var clones, num_batches_tracked clones)
        self._recs = []    # (model, stats (C, 8, 2, 256) float64, total samples, chunk)
        self._unsupported = False   # a query of this step kept no record (layered train math)

    def mark_unsupported(self) -> None:
        self._unsupported = True

    # -- hooks called by nof._ops around every train-mode query
    def before(self, model) -> None:
        if id(model) not in self._snap:
            norms = model.norms()
            self._snap[id(model)] = (model, [b.running_mean.detach().clone() for b in norms],
                                     [b.running_var.detach().clone() for b in norms],
                                     [None if b.num_batches_tracked is None else b.num_batches_tracked.clone()
                                      for b in norms])

    def after(self, model, state: torch.Tensor, total: int, chunk: int) -> None:
        chunk = max(1, min(int(chunk), int(total)))
        self._recs.append((model, _ops.bn_chunk_stats(state, total, chunk), int(total), chunk))

    def add_record(self, model, stats: torch.Tensor, total: int, chunk: int) -> None:
        """Append a record directly (tests; callers with statistics from elsewhere)."""
        self.before(model)
        self._recs.append((model, stats, int(total), max(1, min(int(chunk), int(total)))))

    @contextlib.contextmanager
    def record(self):
        if _ops._BN_REC is not None:
            raise RuntimeError("a BatchNorm recording is already active")
        _ops._BN_REC = self
        try:
            yield self
        finally:
            _ops._BN_REC = None

    def sync(self, group=None, replay=None) -> None:
        """Replay every rank's recorded chunks in global order onto the step's starting statistics (a collective:
        every rank calls it after the same sequence of queries).  ``replay(model, stats, ns)``: the update
        (default nof._ops.bn_running_replay, the HIP kernel).  Single-process: the forward's own update already is
        the sequential one; the records are dropped."""
        recs, snap, unsupported = self._recs, self._snap, self._unsupported
        self._recs, self._snap, self._unsupported = [], {}, False
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
            return
        replay = replay or _ops.bn_running_replay
        world = dist.get_world_size(group)
        cpu_comm = dist.get_backend(group) == "gloo"
        dev = recs[0][1].device if recs else (torch.device("cuda", torch.cuda.current_device())
                                              if not cpu_comm and torch.cuda.is_available() else torch.device("cpu"))
        comm_dev = torch.device("cpu") if cpu_comm else dev
        # the ranks must have made the same queries (same models in the same order): the counts are checked first,
        # with whether any rank's step had a query that kept no record
        n = torch.tensor([len(recs), int(unsupported)], dtype=torch.int64, device=comm_dev)
        ns = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(ns, n, group=group)
        if any(int(x[1]) for x in ns):
            if not BnSync._warned:
                warnings.warn("nof.bn_sync: a layered train math keeps no per-chunk BatchNorm statistics; the "
                              "running statistics stay per rank (select the default train math f16x2_3_fused for "
                              "rank-independent ones)", RuntimeWarning, stacklevel=2)
                BnSync._warned = True
            return
        if any(int(x[0]) != len(recs) for x in ns):
            raise RuntimeError(f"BnSync.sync: ranks recorded different numbers of queries {[int(x[0]) for x in ns]}")
        if not recs:
            return
        meta = torch.tensor([[t, c] for (_, _, t, c) in recs], dtype=torch.int64, device=comm_dev)
        metas = [torch.empty_like(meta) for _ in range(world)]
        dist.all_gather(metas, meta, group=group)
        metas = [m.cpu().tolist() for m in metas]
        # back to the step's starting statistics, then every record's global chunk sequence in call order
        for model, rm, rv, nbt in snap.values():
            for b, m, v, t in zip(model.norms(), rm, rv, nbt):
                b.running_mean.copy_(m)
                b.running_var.copy_(v)
                if t is not None:
                    b.num_batches_tracked.copy_(t)
        for i, (model, st, total, chunk) in enumerate(recs):
            sizes = [_chunk_sizes(metas[r][i][0], metas[r][i][1]) for r in range(world)]
            cmax = max(len(s) for s in sizes)
            pad = torch.zeros((cmax,) + tuple(st.shape[1:]), dtype=st.dtype, device=comm_dev)
            pad[:st.shape[0]] = st.to(comm_dev)
            bufs = [torch.empty_like(pad) for _ in range(world)]
            dist.all_gather(bufs, pad, group=group)
            allst = torch.cat([b[:len(s)] for b, s in zip(bufs, sizes)], 0).to(dev)
            counts = torch.tensor([x for s in sizes for x in s], dtype=torch.int64, device=dev)
            replay(model, allst, counts)
            for b in model.norms():
                if b.num_batches_tracked is not None:
                    b.num_batches_tracked.add_(int(counts.numel()))

