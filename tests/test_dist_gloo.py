"""Multi-process (world size 2, gloo on CPU) coverage of the N>1 path: block sharding, ragged row gather and the
max-over-ranks time used by bench.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nof.blocks import blocks_of_rank, gather_rows, max_over_ranks


def test_blocks_partition():
    for world in (1, 2, 3, 4, 8):
        for nb in (0, 1, 4, 7, 8, 13):
            got = [b for r in range(world) for b in blocks_of_rank(r, world, nb)]
            assert got == list(range(nb))
            sizes = [len(blocks_of_rank(r, world, nb)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r holds 3 + r rows of (depth, flag) for its blocks
        local = torch.stack([torch.arange(3 + rank, dtype=torch.float32) + 100 * rank,
                             torch.full((3 + rank,), float(rank))], 1)
        out = gather_rows(local, dst=0)
        t = max_over_ranks(1.0 + rank)
        q.put((rank, None if out is None else out.tolist(), t, blocks_of_rank(rank, world, 4)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gather_and_max_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, out, t, blocks = q.get(timeout=90)
        res[rank] = (out, t, blocks)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    out0, t0, b0 = res[0]
    assert res[1][0] is None
    assert [row[0] for row in out0] == [0, 1, 2, 100, 101, 102, 103]
    assert [row[1] for row in out0] == [0, 0, 0, 1, 1, 1, 1]
    assert t0 == res[1][1] == 2.0
    assert b0 == [0, 1] and res[1][2] == [2, 3]
