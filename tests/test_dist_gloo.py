"""Multi-process (world size 2, gloo on CPU) coverage of the N>1 path: block sharding, ragged row gather and the
max-over-ranks time used by bench.py."""
import os
import socket

import numpy as np
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
    # config 5: every rank renders a row-balanced share of each of the 8 blocks
    assert lines[0]["n_gpus"] == 2 and lines[0]["dry_run"] and lines[0]["rank0_blocks"] == list(range(8))
    # the self-proving N-rank record: backend, ranks seen, per-rank rays / ms / collective ms
    d = lines[0]["dist"]
    assert d["backend"] == "gloo" and d["ranks_seen"] == 2
    for k in ("rays_per_rank", "ms_per_step_per_rank", "collective_ms_per_step_per_rank"):
        assert len(d[k]) == 2 and all(v >= 0 for v in d[k])
    assert d["rays_per_rank"] == [2048, 2048]
    assert all(c <= m for c, m in zip(d["collective_ms_per_step_per_rank"], d["ms_per_step_per_rank"]))
    bad = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "4", "--dry-run"],
                         capture_output=True, text=True, env={**env, "WORLD_SIZE": "2"}, timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr


def _col12(sizes):
    """Column 12 of two-step rows with these ray-group sizes (k-1 on a group's first row, -1 on the others)."""
    import numpy as np
    col = np.full(int(np.sum(sizes)), -1.0, dtype=np.float32)
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    col[starts] = np.asarray(sizes, dtype=np.float32) - 1
    return col


def test_split_groups_reference_group_sizes():
    """The row-balanced split of the eval driver on the reference's own two-step rows
    (tests/golden/view_group_sizes.npz: KITTI frames 1153 / 1178, groups of 1-28 rows): whole groups only, every
    row once, and the largest share within 2 % of the mean at 2, 4 and 8 ranks."""
    import numpy as np
    from conftest import golden
    from nof.blocks import split_groups
    g = golden("view_group_sizes")
    for key in ("f1153", "f1178"):
        col = _col12(g[key].astype(np.int64))
        n = col.shape[0]
        for world in (1, 2, 4, 8):
            parts = split_groups(col, world)
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            assert all(col[s] >= -0.5 for s, e in parts if s < n)            # each share starts a group
            sizes = [e - s for s, e in parts]
            assert max(sizes) / (n / world) <= 1.02, (key, world, sizes)
        # a sub-range (the rows the reference's batching renders) splits the same way
        parts = split_groups(col, 8, 0, n - 1 if col[n - 1] >= -0.5 else n)
        assert sum(e - s for s, e in parts) in (n - 1, n)


def test_group_batches_whole_groups():
    import numpy as np
    import eval_kitti_render as E
    rng = np.random.default_rng(3)
    col = _col12(rng.integers(1, 12, size=500))
    for s0, e0 in ((0, col.shape[0]), (37 if col[37] >= -0.5 else 0, col.shape[0])):
        for bs in (1, 16, 1000):
            sl = E.group_batches(col, s0, e0, bs)
            assert sl[0][0] == s0 and sl[-1][1] == e0
            assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
            assert all(e == e0 or col[e] >= -0.5 for _, e in sl)


def _fake_view_render(mc, mf, emb, rows, other, **kw):
    """Per-row stand-in for render_rays_view_0525_2_2 (CPU): what render_frame's slicing must preserve."""
    flag = (rows[:, 0] * 7 + rows[:, 1]).floor().remainder(3) != 0
    return {"rays_effective_flag_fine": flag.reshape(-1, 1), "points_inference_fine": rows[:, :3] * 2 + rows[:, 12:13]}


def _eval_worker(rank, world, port, q, rows, other, batch_rows):
    import argparse
    import eval_kitti_render as E
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        E.render_rays_view_0525_2_2 = _fake_view_render
        h = argparse.Namespace(N_samples=8, N_importance=16, use_disp=False, perturb=0, noise_std=0, chunk=1024,
                               depth_inference_method=2)
        pts, n = E.render_frame((None, None, None), rows, other, h, batch_rows, rank, world)
        q.put((rank, None if pts is None else pts.numpy(), n))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("tail", ["group", "lone_row"])
def test_eval_render_frame_world2_matches_one_process(tail):
    """render_frame over 2 gloo ranks (whole-group shares, points gathered to rank 0 in rank order) returns exactly
    the single-process cloud and row count -- including the reference's dropped lone last row."""
    import numpy as np
    import eval_kitti_render as E
    rng = np.random.default_rng(11)
    sizes = list(rng.integers(1, 9, size=700)) + ([1] if tail == "lone_row" else [3])
    col = _col12(sizes)
    rows = torch.zeros((col.shape[0], 13))
    rows[:, :3] = torch.from_numpy(rng.normal(size=(col.shape[0], 3)).astype(np.float32)) * 10
    rows[:, 12] = torch.from_numpy(col)
    other = torch.zeros(col.shape[0], dtype=torch.int64)
    bs = 512 if tail == "group" else 16
    E.render_rays_view_0525_2_2, keep = _fake_view_render, E.render_rays_view_0525_2_2
    try:
        want, n1 = E.render_frame((None, None, None), rows, other,
                                  __import__("argparse").Namespace(N_samples=8, N_importance=16, use_disp=False,
                                                                   perturb=0, noise_std=0, chunk=1024,
                                                                   depth_inference_method=2), bs)
    finally:
        E.render_rays_view_0525_2_2 = keep
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_eval_worker, args=(r, 2, port, q, rows, other, bs)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, pts, n = q.get(timeout=90)
        res[r] = (pts, n)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert res[1][0] is None and res[0][1] == res[1][1] == n1
    np.testing.assert_array_equal(res[0][0], want.numpy())


def _bn_records(rank, seed):
    """Rank ``rank``'s synthetic chunk-statistics records: (model index, stats, total, chunk), ragged per rank."""
    g = torch.Generator().manual_seed(1000 * seed + rank)
    out = []
    for mi, total, chunk in ((0, 1000 + 300 * rank, 256), (1, 700 - 200 * rank, 128), (0, 513 + 7 * rank, 512)):
        C = -(-total // chunk)
        st = torch.empty((C, 8, 2, 256), dtype=torch.float64)
        st[:, :, 0] = torch.randn((C, 8, 256), generator=g, dtype=torch.float64)
        st[:, :, 1] = torch.rand((C, 8, 256), generator=g, dtype=torch.float64) * 2 + 0.01
        out.append((mi, st, total, chunk))
    return out


def _bn_models():
    from nof import synthetic as syn
    from nof.networks import NOF_coarse, NOF_fine
    return [syn.load_into(NOF_coarse(), syn.init_nof_params(11)), syn.load_into(NOF_fine(), syn.init_nof_params(12))]


def _bn_worker(rank, world, port, q):
    from bn_replay_ref import replay_reference
    from nof.bn_sync import BnSync
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        models = _bn_models()
        bns = BnSync()
        for mi, st, total, chunk in _bn_records(rank, 3):
            bns.add_record(models[mi], st, total, chunk)
            for b in models[mi].norms():   # the rank's own forward moved its buffers (sync must start over)
                b.running_mean.add_(rank + 1.0)
                b.num_batches_tracked.add_(-(-total // chunk))
        bns.sync(replay=replay_reference)
        q.put((rank, [{k: v.numpy().copy() for k, v in m.state_dict().items()} for m in models]))
    finally:
        dist.destroy_process_group()


def test_bn_sync_world2_rank_independent_running_stats():
    """nof.bn_sync under gloo world 2: every rank ends with the same BatchNorm running statistics, equal to one
    process applying rank 0's then rank 1's chunks (per query, in call order) from the step's starting values, and
    num_batches_tracked counting both ranks' chunks.  Ragged chunk counts per rank."""
    from bn_replay_ref import replay_reference
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bn_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    models = _bn_models()
    recs = [_bn_records(r, 3) for r in range(2)]
    for i in range(3):
        mi = recs[0][i][0]
        st = torch.cat([recs[r][i][1] for r in range(2)], 0)
        ns = [min(c, t - k * c) for r in range(2) for t, c in [recs[r][i][2:]] for k in range(-(-t // c))]
        replay_reference(models[mi], st, torch.tensor(ns))
        for b in models[mi].norms():
            b.num_batches_tracked.add_(len(ns))
    for m, s0, s1 in zip(models, got[0], got[1]):
        for k, v in m.state_dict().items():
            np.testing.assert_array_equal(s0[k], s1[k], err_msg=k)
            np.testing.assert_array_equal(s0[k], v.numpy(), err_msg=k)


def _bn_unsup_worker(rank, world, port, q):
    import warnings
    from nof import _ops
    from nof.bn_sync import BnSync
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        models = _bn_models()
        bns = BnSync()
        with bns.record():
            bns.before(models[0])
            for b in models[0].norms():   # the rank's own (layered-math) forward moved its buffers
                b.running_mean.add_(rank + 1.0)
            if rank == 1:                 # one rank's query kept no record: every rank must skip the replay
                _ops._bn_unsupported()
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            bns.sync()
        q.put((rank, [b.running_mean.numpy().copy() for b in models[0].norms()],
               any(issubclass(x.category, RuntimeWarning) for x in w)))
    finally:
        dist.destroy_process_group()


def test_bn_sync_layered_math_keeps_per_rank_stats():
    """a train-mode query under a layered train math (no per-chunk record) inside BnSync.record() no
    longer raises; sync() warns and leaves each rank's running statistics as its own forward set them, on every rank
    (the flag is all-gathered, so the ranks agree on skipping)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bn_unsup_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (m, w) for r, m, w in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    base = _bn_models()[0]
    for r in range(2):
        means, _ = got[r]
        for m, b in zip(means, base.norms()):
            np.testing.assert_array_equal(m, b.running_mean.numpy() + (r + 1.0))
    assert got[0][1] or got[1][1]   # warned (once per process)
