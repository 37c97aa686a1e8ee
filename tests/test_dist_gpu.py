"""The distributed path on the GPU box (one MI355X): RCCL initialised for real, and data-parallel HIP gradients.

* ``backend="nccl"`` (RCCL on ROCm) with a single rank: gather_rows / max_over_ranks / allreduce_grads run their
  collectives on device tensors -- the code path bench.py --gpus N and train_kitti.py take on a node.
* data parallel over 2 processes sharing the GPU (gloo carries the CUDA tensors: RCCL needs one GPU per rank):
  each rank renders its shard of one global batch through the HIP kernels (train-mode BatchNorm over its own
  chunks), backward, nof.blocks.allreduce_grads -- the averaged gradients must equal the mean of the two shards'
  gradients computed one after the other in a single process (DESIGN (e): per-rank BatchNorm chunks, one
  all_reduce of a flat bucket).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_single_rank_collectives():
    from nof.blocks import allreduce_grads, gather_rows, max_over_ranks
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        rows = torch.arange(12, dtype=torch.float32, device="cuda").reshape(6, 2)
        assert torch.equal(gather_rows(rows, dst=0), rows)
        assert max_over_ranks(3.5, device=torch.device("cuda", 0)) == 3.5
        p = torch.nn.Parameter(torch.ones(5, device="cuda"))
        p.grad = torch.full((5,), 2.0, device="cuda")
        q = torch.nn.Parameter(torch.ones(3, device="cuda"))   # no gradient: contributes zeros
        allreduce_grads([p, q])
        assert torch.equal(p.grad, torch.full((5,), 2.0, device="cuda")) and torch.equal(q.grad, torch.zeros(3,
                                                                                                         device="cuda"))
    finally:
        dist.destroy_process_group()


KW = dict(sub_nerf_test_num=32, N_samples=32, N_importance=64, perturb=0, noise_std=0, chunk=4096, issegmentated=1,
          childnerf_ratio=0.1, use_child_nerf_divide=0, use_child_nerf_loss=1)


def _shard_grads(rays, seed_c=1234, seed_f=5678):
    """Gradients of the train_kitti.py:117-155 loss on one shard, single process."""
    from nof import synthetic as syn
    from nof.criteria import nof_loss
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_train
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(seed_c)).cuda().train()
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(seed_f)).cuda().train()
    res = render_rays_train(mc, mf, Embedding(3, 10), rays, **KW)
    sl1 = nof_loss["smoothl1"]()
    gt = rays[:, 14]
    loss = (1e-1 * sl1(1e1 * res["depth"], 1e1 * gt) + 1e-1 * sl1(1e1 * res["depth_fine"], 1e1 * gt)
            + 1e6 * (res["child_free_loss"] + res["child_free_loss_fine"])
            + 1e5 * (res["child_depth_loss"] + res["child_depth_loss_fine"]))
    loss.backward()
    return list(mc.parameters()) + list(mf.parameters())


def _dp_rank(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "pc-nerf_amd"), here):
        sys.path.insert(0, p)
    from nof import synthetic as syn
    from nof.blocks import allreduce_grads, shard_batch
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        rays = torch.from_numpy(syn.make_rays(384, seed=41)).cuda()
        idx = shard_batch(torch.arange(384, device="cuda"), rank, world)
        params = _shard_grads(rays[idx].contiguous())
        allreduce_grads(params)
        q.put((rank, [p.grad.cpu().numpy() for p in params]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_data_parallel_hip_gradients_two_ranks():
    from nof import synthetic as syn
    from nof.blocks import shard_batch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_dp_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, g = q.get(timeout=200)
        got[r] = g
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    rays = torch.from_numpy(syn.make_rays(384, seed=41)).cuda()
    shards = [shard_batch(torch.arange(384, device="cuda"), r, 2) for r in range(2)]
    g0 = [p.grad.cpu().numpy() for p in _shard_grads(rays[shards[0]].contiguous())]
    g1 = [p.grad.cpu().numpy() for p in _shard_grads(rays[shards[1]].contiguous())]
    for a, b, x, y in zip(got[0], got[1], g0, g1):
        np.testing.assert_array_equal(a, b)                       # every rank ends with the same gradients
        want = (x + y) / 2
        np.testing.assert_allclose(a, want, rtol=1e-6, atol=1e-6 * max(np.abs(want).max(), 1e-30))


def _bn_step(models, rays, bns=None):
    """One train_kitti.py:117-155 step's forward + backward on ``rays`` (recorded by ``bns`` when given)."""
    from nof.criteria import nof_loss
    from nof.networks import Embedding
    from nof.render import render_rays_train
    import contextlib
    mc, mf = models
    with (bns.record() if bns is not None else contextlib.nullcontext()):
        res = render_rays_train(mc, mf, Embedding(3, 10), rays, **KW)
    sl1 = nof_loss["smoothl1"]()
    gt = rays[:, 14]
    loss = 1e-1 * sl1(1e1 * res["depth"], 1e1 * gt) + 1e-1 * sl1(1e1 * res["depth_fine"], 1e1 * gt)
    loss.backward()


def _bn_models_gpu(chunk_seed=0):
    from nof import synthetic as syn
    from nof.networks import NOF_coarse, NOF_fine
    return (syn.load_into(NOF_coarse(), syn.init_nof_params(1234)).cuda().train(),
            syn.load_into(NOF_fine(), syn.init_nof_params(5678)).cuda().train())


def _bn_rank(rank, world, port, q, math=None):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "pc-nerf_amd"), here):
        sys.path.insert(0, p)
    from nof import _ops
    from nof import synthetic as syn
    if math is not None:
        _ops.set_train_math(math)
    from nof.blocks import allreduce_grads, shard_batch
    from nof.bn_sync import BnSync
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        rays = torch.from_numpy(syn.make_rays(401, seed=43)).cuda()
        idx = shard_batch(torch.arange(401, device="cuda"), rank, world)
        models = _bn_models_gpu()
        bns = BnSync()
        _bn_step(models, rays[idx].contiguous(), bns)
        allreduce_grads([p for m in models for p in m.parameters()])
        bns.sync()
        q.put((rank, [{k: v.cpu().numpy() for k, v in m.state_dict().items()} for m in models]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_data_parallel_batchnorm_running_stats_rank_independent():
    """Data parallel over 2 gloo ranks sharing the GPU, the default train math: after nof.bn_sync every rank's
    state_dict (weights' gradients aside: running_mean / running_var / num_batches_tracked included) is identical,
    and the running statistics equal one process rendering rank 0's shard and then rank 1's (train mode, chunk
    4096: 201 / 200 rays, so the ranks' tail chunks differ) -- bit for bit (the HIP replay of every chunk's recorded
    statistics in global order, pcnerf_nof_train_bn_stats + pcnerf_bn_running_replay)."""
    from nof import synthetic as syn
    from nof.blocks import shard_batch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_bn_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=200) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    rays = torch.from_numpy(syn.make_rays(401, seed=43)).cuda()
    models = _bn_models_gpu()
    for r in range(2):
        _bn_step(models, rays[shard_batch(torch.arange(401, device="cuda"), r, 2)].contiguous())
    for m, s0, s1 in zip(models, got[0], got[1]):
        for k, v in m.state_dict().items():
            np.testing.assert_array_equal(s0[k], s1[k], err_msg=k)
            if "running" in k or "num_batches" in k:
                np.testing.assert_array_equal(s0[k], v.cpu().numpy(), err_msg=k)


@pytest.mark.timeout(240)
def test_data_parallel_layered_math_bn_per_rank():
    """data-parallel training under a layered train math (f16x2_3: no per-chunk statistics record) no
    longer raises inside BnSync.record(); each rank keeps the running statistics its own forward set (equal to one
    process rendering that rank's shard), with a warning."""
    from nof import _ops
    from nof import synthetic as syn
    from nof.blocks import shard_batch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_bn_rank, args=(r, 2, port, q, "f16x2_3")) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=200) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    prev = _ops.set_train_math("f16x2_3")
    try:
        rays = torch.from_numpy(syn.make_rays(401, seed=43)).cuda()
        for r in range(2):
            models = _bn_models_gpu()
            _bn_step(models, rays[shard_batch(torch.arange(401, device="cuda"), r, 2)].contiguous())
            for m, s in zip(models, got[r]):
                for k, v in m.state_dict().items():
                    if "running" in k or "num_batches" in k:
                        np.testing.assert_array_equal(s[k], v.cpu().numpy(), err_msg=k)
    finally:
        _ops.set_train_math(prev)


def _fit_rank(rank, world, port, tmp, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "pc-nerf_amd"), here):
        sys.path.insert(0, p)
    import train_kitti as T
    from nof.nof_utils import get_opts
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        root, pose_path = os.path.join(tmp, "pcd"), os.path.join(tmp, "poses.txt")
        out = os.path.join(tmp, f"run{rank}")
        args = f"""--datasettype kitti_dataload --root_dir {root} --pose_path {pose_path} --data_start 1150
         --data_end 1155 --re_loaddata 1 --result_path {out} --N_samples 32 --N_importance 64 --perturb 1
         --noise_std 0 --chunk 4096 --batch_size 96 --batch_size_val 64 --cloud_size_val 128 --num_epochs 1
         --optimizer adam --lr 5e-4 --weight_decay 1e-3 --decay_gamma 0.2 --use_child_nerf_divide 0
         --use_child_nerf_loss 1 --use_segmentated_sample 1 --segmentated_child_nerf_ratio 0.1 --lambda_loss 1
         --lambda_loss_fine 1 --lambda_child_free_loss 1000000 --lambda_child_depth_loss 100000 --range_delete_x 3
         --range_delete_y 2 --range_delete_z 1.25 --surface_expand 0.05 --interest_x 20 --interest_y 20
         --visualize 0 --seed 42"""
        h = get_opts(args.split())
        torch.manual_seed(0)
        system = T.NOFSystem(h)
        system.prepare_data()
        h.sub_nerf_test_num = system.train_dataset.sub_nerf_test_num
        res = T.fit(system, max_steps=3)
        q.put((rank, res["steps"], [{k: v.cpu().numpy() for k, v in m.state_dict().items()}
                                    for m in (system.nof_coarse, system.nof_fine)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(280)
def test_fit_data_parallel_checkpoints_rank_independent(tmp_path):
    """train_kitti.fit() data parallel over 2 gloo ranks sharing the GPU (3 steps on the KITTI fixture scene, each
    rank its half of every global batch, BatchNorm chunks of 4096 samples): both ranks end with the same state_dict
    -- weights (one all_reduce of the gradients, the same Adam step) AND running_mean / running_var /
    num_batches_tracked (nof.bn_sync replaying both ranks' chunk statistics in global order), so the checkpoint does
    not depend on which rank writes it."""
    from test_dataset import write_scene
    root, pose_path, _ = write_scene(str(tmp_path))
    assert os.path.samefile(root, os.path.join(str(tmp_path), "pcd"))
    assert os.path.samefile(pose_path, os.path.join(str(tmp_path), "poses.txt"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_fit_rank, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, steps, sd = q.get(timeout=250)
        got[r] = (steps, sd)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert got[0][0] == got[1][0] == 3
    for s0, s1 in zip(got[0][1], got[1][1]):
        assert s0.keys() == s1.keys()
        for k in s0:
            np.testing.assert_array_equal(s0[k], s1[k], err_msg=k)
        nbt = [k for k in s0 if k.endswith("num_batches_tracked")]
        assert nbt and all(int(s0[k]) > 3 for k in nbt)   # every rank's chunks counted


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
@pytest.mark.timeout(300)
def test_bench_two_ranks_on_one_gpu(cfg, tmp_path):
    """bench.py --gpus 2 end to end -- launcher, one process per rank, the config's sharding (2: a block per rank;
    3: a data-parallel batch with the gradient all-reduce; 4: blocks dealt and depths gathered; 5: every block's
    whole ray groups split and gathered), barrier-bracketed timing, max over ranks, rank 0's line with the rank
    report -- with both ranks on the one GPU of this box over gloo (PCNERF_BENCH_SHARE_GPU: RCCL needs a GPU per
    rank; the driver's N-GPU runs take the same code with nccl)."""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, PCNERF_BENCH_SHARE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(os.path.dirname(here), "bench.py"), "--gpus", "2", "--config", str(cfg),
           "--steps", "2", "--warmup", "1", "--samples", "32", "--importance", "64", "--no-ceiling",
           "--detail", str(tmp_path / "detail.json")] + ([] if cfg == 5 else ["--rays", "4096"])
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    d = line["dist"]
    assert line["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["backend"] == "gloo"
    assert len(d["rays_per_rank"]) == 2 and min(d["rays_per_rank"]) > 0 and line["value"] > 0
    assert line["config"]["rays_per_step"] == sum(d["rays_per_rank"])
    if cfg in (2, 3):   # weak scaling: every rank its own 4,096 rays
        assert d["rays_per_rank"] == [4096, 4096]
    if cfg == 5:        # whole ray groups of every block, shares within a few percent
        assert max(d["rays_per_rank"]) <= 1.1 * min(d["rays_per_rank"])
    assert line["cpu_baseline"] is None   # the CPU baseline belongs to the N = 1 line


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
@pytest.mark.timeout(300)
def test_bench_one_rank_rccl(cfg, tmp_path):
    """bench.py under torch.distributed.run with one process and PCNERF_BENCH_FORCE_DIST=1: the N-rank code path
    (barriers, max over ranks, the config's gather / gradient all-reduce, the rank report) over a one-rank RCCL
    group, so every collective the driver's N-GPU runs issue executes through RCCL on this box's one GPU."""
    import json
    import socket
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PCNERF_BENCH_FORCE_DIST="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "PCNERF_BENCH_SHARE_GPU"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(os.path.dirname(here), "bench.py"), "--gpus", "1", "--config", str(cfg),
           "--steps", "2", "--warmup", "1", "--samples", "32", "--importance", "64", "--no-ceiling",
           "--no-cpu-baseline", "--no-extra", "--detail", str(tmp_path / "detail.json")] + \
        ([] if cfg == 5 else ["--rays", "4096"])
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    d = line["dist"]
    assert line["n_gpus"] == 1 and d["ranks_seen"] == 1 and d["backend"] == "nccl"
    assert d["rays_per_rank"] == [line["config"]["rays_per_step"]] and line["value"] > 0
    if cfg in (3, 4, 5):   # the step's collective ran (gradient all-reduce / depth gather) and was timed
        assert d["collective_ms_per_step_per_rank"][0] > 0
