"""Diagnostic (GPU box): the 1,000-sample BatchNorm-chunk gradient case of test_train_grads_vs_oracle_small_chunks
under each train math, per-tensor error statistics of the fine network's gradients against the oracle's float64
evaluation, beside the float32 oracle's own.  Prints one line per (math, tensor): RMS / max error over the tensor's
max, and for layer1.0.weight the error's column profile (encoding column groups: xyz, then sin/cos per frequency)."""
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pc-nerf_amd"))
import test_backward_gpu as T  # noqa: E402
from nof import synthetic as syn, _ops  # noqa: E402
from nof import render as R  # noqa: E402
from oracle import ref_cpu as O  # noqa: E402

R_, S, I = 96, 16, 32
rays_np = syn.make_rays(R_, seed=31)
kw = dict(sub_nerf_test_num=32, N_samples=S, N_importance=I, perturb=0, noise_std=0, chunk=1000,
          issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0, use_child_nerf_loss=1)
rays_c = torch.from_numpy(rays_np)


def oracle(f64):
    P = []
    for seed in (T.SEED_C, T.SEED_F):
        Q = O.params_from_numpy(syn.init_nof_params(seed))
        if f64:
            Q = {k: (v.double() if v.is_floating_point() else v) for k, v in Q.items()}
        for k in Q:
            if k.endswith(".weight") or k.endswith(".bias"):
                Q[k].requires_grad_(True)
        P.append(Q)
    r = rays_c.double() if f64 else rays_c
    ro = O.render_rays_train(P[0], P[1], rays_c, **kw, f64=f64) if f64 else O.render_rays_train(P[0], P[1], rays_c, **kw)
    lr, lrf = O.range_losses(ro["depth"], ro["depth_fine"], r[:, 14])
    O.total_loss(ro, lr, lrf).sum().backward()
    return [{k: v.grad.double().numpy() for k, v in Q.items() if getattr(v, "grad", None) is not None} for Q in P]


g64 = oracle(True)
g32 = oracle(False)
torch.set_num_threads(3)
g32b = oracle(False)


def report(tag, gh):
    for net, nm in ((0, "c"), (1, "f")):
        for k in ("layer1.0.weight", "layer1.3.weight", "layer2.0.weight"):
            if k not in g64[net]:
                continue
            ref = g64[net][k]
            e = gh[net][k] - ref
            m = np.abs(ref).max()
            line = f"{tag:14s} {nm}:{k:16s} rms/max {np.sqrt(np.mean(e ** 2)) / m:.3e} max/max {np.abs(e).max() / m:.3e}"
            if k == "layer1.0.weight":
                cols = np.sqrt(np.mean(e ** 2, axis=0)) / m
                line += " cols[xyz,sin/cos by freq] " + " ".join(
                    f"{cols[:3].max():.1e}" if j == 0 else f"{cols[3 + 6 * (j - 1):9 + 6 * (j - 1)].max():.1e}"
                    for j in range(11))
            print(line, flush=True)


report("oracle_f32", g32)
report("oracle_f32_t3", g32b)
for math in ("fp32", "f16x2_3", "f16x2_3_fused"):
    prev = _ops.set_train_math(math)
    emb, mc, mf = T.models()
    rays = torch.from_numpy(rays_np).to("cuda")
    res = R.render_rays_train(mc, mf, emb, rays, **kw)
    lr, lrf = T.range_losses(res["depth"], res["depth_fine"], rays[:, 14], rays, 0, 32)
    T.total(res, lr, lrf).sum().backward()
    gh = [{k: v.grad.double().cpu().numpy() for k, v in m.named_parameters()} for m in (mc, mf)]
    report("hip_" + math, gh)
    _ops.set_train_math(prev)
