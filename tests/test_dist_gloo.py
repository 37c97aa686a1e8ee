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


def test_shard_batch_partition():
    from nof.blocks import shard_batch
    for n in (0, 1, 5, 256, 257):
        idx = torch.randperm(n)
        for world in (1, 2, 3, 8):
            parts = [shard_batch(idx, r, world) for r in range(world)]
            assert torch.equal(torch.cat(parts), idx)
            sizes = [p.numel() for p in parts]
            assert max(sizes) - min(sizes) <= 1


def _dp_worker(rank, world, port, q):
    """Data-parallel step of train_kitti.fit on CPU: each rank's shard of one global batch, mean loss per rank,
    gradients averaged by allreduce_grads -> must equal the single-process gradient of the whole batch (equal
    shards), and every rank must end with identical parameters after the optimizer step."""
    from nof.blocks import allreduce_grads, shard_batch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(7, 16), torch.nn.Linear(16, 1))
        unused = torch.nn.Parameter(torch.ones(3))          # never receives a gradient
        x, y = torch.randn(64, 7), torch.randn(64, 1)
        idx = shard_batch(torch.arange(64), rank, world)
        loss = torch.nn.functional.mse_loss(net(x[idx]), y[idx])
        loss.backward()
        params = list(net.parameters()) + [unused]
        allreduce_grads(params)
        g = torch.cat([p.grad.reshape(-1) for p in params]).clone()
        opt = torch.optim.Adam(params, lr=1e-2)
        opt.step()
        w = torch.cat([p.detach().reshape(-1) for p in params])
        q.put((rank, g.tolist(), w.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_data_parallel_gradients_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, g, w = q.get(timeout=90)
        res[rank] = (torch.tensor(g), torch.tensor(w))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 16), torch.nn.Linear(16, 1))
    x, y = torch.randn(64, 7), torch.randn(64, 1)
    torch.nn.functional.mse_loss(net(x), y).backward()
    full = torch.cat([p.grad.reshape(-1) for p in net.parameters()] + [torch.zeros(3)])
    torch.testing.assert_close(res[0][0], full, rtol=1e-5, atol=1e-7)
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


@pytest.mark.timeout(300)
def test_bench_launcher_spawns_ranks():
    """bench.py --gpus 2 with no WORLD_SIZE starts torch.distributed.run itself (child process, nothing touched the
    GPU) and relays rank 0's line; --dry-run runs the distributed skeleton (gloo barrier, timed steps, max over
    ranks) without a GPU.  Under an external launcher --gpus must equal WORLD_SIZE."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "2",
                          "--warmup", "1", "--config", "5"], capture_output=True, text=True, env=env, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["dry_run"] and lines[0]["rank0_blocks"] == [0, 1, 2, 3]
    bad = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "4", "--dry-run"],
                         capture_output=True, text=True, env={**env, "WORLD_SIZE": "2"}, timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr
