"""Benchmark: LiDAR rays/s (render + loss) at 128 samples/ray on MI355X -- BASELINE.json config 2.

Default (--mode train_fwd): one step = the reference training step's forward on one batch
(train_kitti.py:117-155 without backward):
``render_rays_train`` (train-mode BatchNorm over 262,144-sample chunks, segmented sampling ratio 0.1, child
free/depth losses, perturb 1, noise_std 0) over 65,536 synthetic rays of one parent block with 32 child AABBs at
N_samples=128 / N_importance=256 (512 MLP samples per ray), plus the SmoothL1 range losses and the weighted total
loss.  Inputs are resident in HBM before timing starts.
--mode train_step adds what Lightning does with that loss: loss.backward() through the HIP backward kernels and
the reference's optimizer step (Adam lr 5e-4, eps 1e-8, weight_decay 1e-3 over both networks, nof_utils.py:162-173)
-- the end-to-end training iteration of config 3 on config 2's batch.  --mode val: render_rays_val (eval BN).
--mode view: config 5's two-step coarse-to-fine inference (render_rays_view_0525_2_2, method 2) on 13-column rows
grouped per LiDAR ray; value counts LiDAR rays (groups), rows_per_gpu the rendered rows.

Multi-GPU (``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``): one process per GPU, each
rank renders its own parent block (own rays, own NOF weights) -- weak scaling with no collective
inside the timed region; the only collectives are the barrier around it and the max-over-ranks of the time.

Prints ONE JSON line (rank 0) with the throughput, the dominant kernel's roofline (HIP events over the timed
region, on the kernels' own stream) and a CPU baseline (the CPU oracle on a bounded sample, rank 0 only).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "pc-nerf_amd"))
sys.path.insert(0, HERE)

FP32_MFMA_PEAK_TFLOPS = 157.3  # /opt/skills/guides/MI355X_MICROARCH.md (F32 MFMA = vector peak, no xf32)
HBM_PEAK_GBS = 8000.0          # same guide (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rays", type=int, default=None,
                    help="LiDAR rays per GPU (default 65,536; 16,384 ray groups = ~52k two-step rows for --mode view)")
    ap.add_argument("--samples", type=int, default=128)
    ap.add_argument("--importance", type=int, default=256)
    ap.add_argument("--chunk", type=int, default=262144)
    ap.add_argument("--mode", choices=["train_fwd", "train_step", "val", "view"], default="train_fwd")
    ap.add_argument("--cpu-rays", type=int, default=None,
                    help="bounded CPU-baseline sample (rays; default 4096, 1024 for train_step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fold", action="store_true",
                    help="val/view only: the opt-in exact affine fold of the eval network (SURVEY fact 1), reported "
                         "as its own line, never the headline")
    ap.add_argument("--gather", action="store_true",
                    help="gather every rank's depth_fine to rank 0 inside each step (eval-driver output path)")
    return ap.parse_args()


def prof_read(L, tag):
    t, n, f, b = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
    rc = L.pcnerf_prof_read(tag, ctypes.byref(t), ctypes.byref(n), ctypes.byref(f), ctypes.byref(b))
    if rc:
        raise RuntimeError(L.pcnerf_last_error().decode())
    return t.value, n.value, f.value, b.value


def pmc_traffic(kernel_name: str):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary (profiles/), or None."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d.get(kernel_name, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from nof import _hip, _ops, synthetic as syn
    from nof.blocks import blocks_of_rank, gather_rows, max_over_ranks
    from nof.criteria import nof_loss
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_train, render_rays_val, render_rays_view_0525_2_2

    # this rank's parent block (one per GPU): its own child layout, rays and coarse/fine weights
    (block,) = blocks_of_rank(rank, world, world)
    view = a.mode == "view"
    if a.rays is None:
        a.rays = 16384 if view else 65536
    if view:   # config 5: two-step rows grouped per ray (group sizes of the reference's KITTI test frames)
        vr, vo, vg = syn.make_view_rows(a.rays, n_children=32, seed=1000 * block)
        rays = torch.from_numpy(vr).to(dev)
        other = torch.from_numpy(vo).to(dev)
        gt = torch.from_numpy(vg).to(dev)
    else:
        rays = torch.from_numpy(syn.make_rays(a.rays, n_children=32, seed=1000 * block)).to(dev)
    train = a.mode in ("train_fwd", "train_step")
    grad = a.mode == "train_step"
    if a.fold:
        if train:
            raise SystemExit("--fold applies to the eval modes (val, view) only")
        _ops.set_eval_fold(True)
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(1234 + block)).to(dev).train(train)
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(5678 + block)).to(dev).train(train)
    emb = Embedding(3, 10)
    loss_fn = nof_loss["smoothl1"]()
    if not view:
        gt = rays[:, 14].contiguous()
    opt = None
    if grad:
        params = list(mc.parameters()) + list(mf.parameters())
        opt = torch.optim.Adam(params, lr=5e-4, eps=1e-8, weight_decay=1e-3)   # nof_utils.py:167-169

    def step():
        if grad:
            opt.zero_grad(set_to_none=True)
        if train:
            res = render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=32, N_samples=a.samples,
                                    N_importance=a.importance, perturb=1, noise_std=0, chunk=a.chunk,
                                    issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0,
                                    use_child_nerf_loss=1)
            lr = 1e-1 * loss_fn(1e1 * res["depth"], 1e1 * gt)           # train_kitti.py:145-146
            lrf = 1e-1 * loss_fn(1e1 * res["depth_fine"], 1e1 * gt)
            loss = (lr + lrf + 1e6 * res["child_free_loss_fine"] + 1e6 * res["child_free_loss"]
                    + 1e5 * res["child_depth_loss_fine"] + 1e5 * res["child_depth_loss"])
        elif view:   # eval_kitti_render.py:1147-1161: two-step inference, effective rows' points kept
            res = render_rays_view_0525_2_2(mc, mf, emb, rays, other, N_samples=a.samples,
                                            N_importance=a.importance, perturb=0, noise_std=0, chunk=a.chunk,
                                            depth_inference_method=2)
            keep = res["rays_effective_flag_fine"].reshape(-1)
            pts = res["points_inference_fine"][keep]
            loss = pts.abs().mean()
        else:
            res = render_rays_val(mc, mf, emb, rays, N_samples=a.samples, N_importance=a.importance, perturb=0,
                                  noise_std=0, chunk=a.chunk)
            loss = 1e-1 * loss_fn(1e1 * res["depth_fine"], 1e1 * gt)
        if a.gather:
            gather_rows(res["depth_fine"][:, None], dst=0)
        if grad:
            loss.backward()
            opt.step()
        return loss.detach()

    L = _hip.lib()
    with (torch.enable_grad() if grad else torch.no_grad()):
        for _ in range(a.warmup):
            loss = step()
        torch.cuda.synchronize(dev)
        if dist:
            tdist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(a.steps):
            # per-kernel HIP events (kernel breakdown + roofline) around every launch of the LAST timed step
            # only: their own cost (two hipEventRecord per launch) then weighs 1/steps on the timed region
            if i == a.steps - 1:
                L.pcnerf_prof_enable(1)
            loss = step()
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        if dist:
            tdist.barrier()
        loss_val = float(loss)
    if not np.isfinite(loss_val):
        raise RuntimeError(f"non-finite loss {loss_val}")
    elapsed = max_over_ranks(elapsed, device=dev)

    # dominant kernel: the MFMA kernel with the most time per step -- the 256 -> 256 pre-BN Linear of train mode
    # (k_train_ws<0,true>: 6 of 9 GEMMs per chunk), or the fused eval query
    knames = {0: "k_nof_eval", 1: "k_train_ws<0,true>", 2: "k_train_ws<8,false>",
              3: "k_train_ws<8,true>", 10: "k_wgrad", 11: "k_dgrad_ws", 13: "k_nof_eval_fold"}
    tag = max(knames, key=lambda t: prof_read(L, t)[0])
    kname = knames[tag]
    ktime_ms, klaunch, kflops, kbytes = prof_read(L, tag)
    kernels = {}
    for t, nm in ((0, "eval_query"), (1, "train_hidden"), (2, "train_first"), (3, "train_skip"), (4, "train_out"),
                  (5, "bn_fold"), (6, "composite"), (7, "resample"), (8, "sample"), (9, "composite_bwd"),
                  (10, "wgrad"), (11, "dgrad"), (12, "bwd_other"), (13, "eval_fold")):
        tm, n, f, b = prof_read(L, t)
        if n:
            kernels[nm] = {"ms_per_step": round(tm, 3), "launches_per_step": n,
                           "avg_us": round(1e3 * tm / n, 2),
                           "TFLOP/s": round(f / (tm * 1e-3) / 1e12, 2) if f else None,
                           "GB/s": round(b / (tm * 1e-3) / 1e9, 1) if b else None}
    L.pcnerf_prof_enable(0)
    avg_s = ktime_ms * 1e-3 / max(klaunch, 1)
    achieved = (kflops / max(klaunch, 1)) / avg_s / 1e12
    traffic = pmc_traffic(kname)
    if a.fold:   # no MLP left: the query moves 8 B per sample (+ ray rows) and is bound by its sincos (VALU)
        roof = {"kernel": kname, "bound": "hbm", "achieved": round(kbytes / max(klaunch, 1) / avg_s / 1e9, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(kbytes / max(klaunch, 1) / avg_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                "avg_launch_us": round(avg_s * 1e6, 2), "algorithmic_bytes_per_launch": kbytes / max(klaunch, 1),
                "note": "VALU-bound (60 sincosf per sample); HBM fraction reported as the contract asks"}
    else:
        roof = {"kernel": kname, "bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                "avg_launch_us": round(avg_s * 1e6, 2), "algorithmic_flop_per_launch": kflops / max(klaunch, 1)}

    cpu = cdref = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:   # the CPU baseline belongs to the N=1 line only
        if a.cpu_rays is None:
            a.cpu_rays = 1024 if grad else 512 if view else 4096
        cpu, ext = cpu_baseline(a, syn)
        cdref = (cd_vs_ref_view if view else cd_vs_ref)(a, syn, ext, dev)

    if rank != 0:
        if dist:
            tdist.destroy_process_group()
        return
    rays_total = a.rays * world * a.steps
    value = rays_total / elapsed
    out = {
        "metric": "LiDAR rays/s (render+loss) at 128 samples/ray; CD vs ref depth",
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": ("synthetic (config-2 parent block, 32 child AABBs; seeded NOF weights -- checkpoints absent)"
                 + ("; ray groups with the group-size histogram of the reference's KITTI test frames" if view
                    else "")),
        "config": {"workload": {"train_fwd": "render_rays_train fwd + range/child losses",
                                "train_step": "render_rays_train fwd + losses + backward + Adam step",
                                "val": "render_rays_val fwd",
                                "view": "render_rays_view_0525_2_2 two-step inference (method 2) + effective points"
                                }[a.mode] + (" -- exact affine fold of the eval network (opt-in)" if a.fold else ""),
                   "rays_per_gpu": a.rays, "N_samples": a.samples, "N_importance": a.importance,
                   "rows_per_gpu": int(rays.shape[0]),
                   "mlp_samples_per_ray": a.samples + a.samples + a.importance, "chunk": a.chunk,
                   "batchnorm": "train (batch stats per chunk)" if train else "eval (folded)",
                   "network": "affine fold (sigmoid(a.e + c))" if a.fold else "9 Linear layers as written",
                   "segmented_ratio": 0.1 if train else None, "perturb": 1 if train else 0,
                   "parallelism": f"blocks{world}", "gather": bool(a.gather)},
        "roofline": roof,
        "cpu_baseline": cpu,
        "cd_vs_ref": cdref,
        "loss": loss_val,
        "kernels": kernels,
    }
    print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


def cpu_baseline(a, syn):
    """The CPU oracle (oracle/ref_cpu.py, the reference's arithmetic on torch CPU) on a bounded sample of the
    same workload: ``--cpu-rays`` rays of the same block, same settings, forward + losses (+ backward + Adam in
    train_step mode).  The RNG draws are generated here and returned with the oracle's depths, so the HIP path can
    be run on the identical inputs for the "CD vs ref depth" half of the metric."""
    from oracle import ref_cpu as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    if a.mode == "view":
        return cpu_baseline_view(a, syn, O, threads)
    rays = torch.from_numpy(syn.make_rays(a.cpu_rays, n_children=32, seed=0))
    Pc = O.params_from_numpy(syn.init_nof_params(1234))
    Pf = O.params_from_numpy(syn.init_nof_params(5678))
    train = a.mode in ("train_fwd", "train_step")
    grad = a.mode == "train_step"
    gen = torch.Generator().manual_seed(7)
    R = rays.shape[0]
    draws = {"perturb_rand": torch.rand(R, a.samples, generator=gen),
             "u": torch.rand(R, a.importance, generator=gen)} if train else {}
    leaves = []
    if grad:
        for P in (Pc, Pf):
            for k in P:
                if k.endswith(".weight") or k.endswith(".bias"):
                    leaves.append(P[k].requires_grad_(True))
        opt = torch.optim.Adam(leaves, lr=5e-4, eps=1e-8, weight_decay=1e-3)

    def run(r, dr, step):
        if train:
            res = O.render_rays_train(Pc, Pf, r, sub_nerf_test_num=32, N_samples=a.samples, N_importance=a.importance,
                                      perturb=1, noise_std=0, chunk=a.chunk, issegmentated=1, childnerf_ratio=0.1,
                                      use_child_nerf_loss=1, training=True, draws=dr)
            lr, lrf = O.range_losses(res["depth"], res["depth_fine"], r[:, 14])
            loss = O.total_loss(res, lr, lrf)
            if grad and step:
                opt.zero_grad()
                loss.backward()
                opt.step()
            return res
        return O.render_rays_val(Pc, Pf, r, N_samples=a.samples, N_importance=a.importance, perturb=0, noise_std=0,
                                 chunk=a.chunk)

    with (torch.enable_grad() if grad else torch.no_grad()):
        run(rays[:64], {k: v[:64] for k, v in draws.items()}, False)  # warm-up (no parameter update)
        t0 = time.perf_counter()
        res = run(rays, draws, True)
        dt = time.perf_counter() - t0
    base = {"value": round(a.cpu_rays / dt, 2), "unit": "rays/s", "cores": threads, "kind": "port",
            "sample": f"{a.cpu_rays} rays of the same workload ({a.mode}, {a.samples}/{a.importance} samples, "
                      f"chunk {a.chunk}) through oracle/ref_cpu.py on torch CPU, {dt:.1f} s"}
    return base, {"rays": rays, "draws": draws, "depth_fine": res["depth_fine"].detach()}


def cpu_baseline_view(a, syn, O, threads):
    """Two-step inference (render.py:614-699 restated in oracle/ref_cpu.py) on ``--cpu-rays`` ray groups."""
    vr, vo, _ = syn.make_view_rows(a.cpu_rays, n_children=32, seed=0)
    rows, other = torch.from_numpy(vr), torch.from_numpy(vo)
    Pc = O.params_from_numpy(syn.init_nof_params(1234))
    Pf = O.params_from_numpy(syn.init_nof_params(5678))
    with torch.no_grad():
        O.render_rays_view(Pc, Pf, rows[:16], torch.zeros(16, dtype=torch.int64), a.samples, a.importance, a.chunk,
                           method=2)   # warm-up
        t0 = time.perf_counter()
        res = O.render_rays_view(Pc, Pf, rows, other, a.samples, a.importance, a.chunk, method=2)
        dt = time.perf_counter() - t0
    base = {"value": round(a.cpu_rays / dt, 2), "unit": "rays/s", "cores": threads, "kind": "port",
            "sample": f"{a.cpu_rays} ray groups ({rows.shape[0]} two-step rows, {a.samples}/{a.importance} samples, "
                      f"method 2) through oracle/ref_cpu.py on torch CPU, {dt:.1f} s"}
    return base, {"rows": rows, "other": other, "res": res}


def cd_vs_ref_view(a, syn, ext, dev):
    """HIP two-step inference on the CPU sample's rows vs the oracle: effective-row flags must agree; CD / F-score
    of the effective rows' fine points (what eval_kitti_render.py writes to the PCD)."""
    from nof import metrics as NM
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_view_0525_2_2
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(1234)).to(dev).eval()
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(5678)).to(dev).eval()
    rows, other, ref = ext["rows"].to(dev), ext["other"].to(dev), ext["res"]
    with torch.no_grad():
        res = render_rays_view_0525_2_2(mc, mf, Embedding(3, 10), rows, other, N_samples=a.samples,
                                        N_importance=a.importance, perturb=0, noise_std=0, chunk=a.chunk,
                                        depth_inference_method=2)
    fh = res["rays_effective_flag_fine"].reshape(-1).cpu()
    fr = ref["rays_effective_flag_fine"].reshape(-1)
    p_hip = res["points_inference_fine"][fh.to(dev)]
    p_ref = ref["points_inference_fine"][fr].to(dev)
    cd, f = NM.eval_pts(p_hip, p_ref, 0.2)
    d_hip, d_ref = res["depth_fine"].cpu(), ref["depth_fine"]
    rel = float(((d_hip - d_ref).abs() / d_ref.abs().clamp_min(1e-6)).max())
    return {"cd_m": cd, "fscore": f, "max_rel_depth_err": rel, "flags_equal": bool(torch.equal(fh, fr)),
            "rays": int(rows.shape[0]), "vs": "oracle two-step points of the effective rows (same rows and weights)"}


def cd_vs_ref(a, syn, ext, dev):
    """The HIP path on the CPU sample's rays and draws (fresh weights of the same seeds) vs the oracle's depths:
    Chamfer distance / F-score (0.2 m) of the rendered points o + d * depth_fine (nof.metrics on the GPU) and the
    largest relative depth error."""
    from nof import metrics as NM
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_train, render_rays_val
    train = a.mode in ("train_fwd", "train_step")
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(1234)).to(dev).train(train)
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(5678)).to(dev).train(train)
    rays = ext["rays"].to(dev)
    with torch.no_grad():
        if train:
            res = render_rays_train(mc, mf, Embedding(3, 10), rays, sub_nerf_test_num=32, N_samples=a.samples,
                                    N_importance=a.importance, perturb=1, noise_std=0, chunk=a.chunk,
                                    issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0,
                                    use_child_nerf_loss=1, rng={k: v.to(dev) for k, v in ext["draws"].items()})
        else:
            res = render_rays_val(mc, mf, Embedding(3, 10), rays, N_samples=a.samples, N_importance=a.importance,
                                  perturb=0, noise_std=0, chunk=a.chunk)
    d_hip, d_ref = res["depth_fine"], ext["depth_fine"].to(dev)
    p_hip = rays[:, 0:3] + rays[:, 3:6] * d_hip[:, None]
    p_ref = rays[:, 0:3] + rays[:, 3:6] * d_ref[:, None]
    cd, f = NM.eval_pts(p_hip, p_ref, 0.2)
    rel = float(((d_hip - d_ref).abs() / d_ref.abs().clamp_min(1e-6)).max())
    return {"cd_m": cd, "fscore": f, "max_rel_depth_err": rel, "rays": int(rays.shape[0]),
            "vs": "oracle depth_fine on the cpu_baseline sample (same rays, draws and initial weights)"}


if __name__ == "__main__":
    main()
