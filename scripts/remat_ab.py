"""Same-process A/B of the default train math's two backwards: "remat" (no activation store, layer inputs
rematerialised from the encoding) against "store" (round 4: the forward writes every chunk's layer outputs).
Config-2 training step (65,536 rays at 128/256 by default), identical weights and draws: gradient agreement per
tensor, then ms per step of each.  Usage: python scripts/remat_ab.py [--rays N] [--steps K]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pc-nerf_amd"))
from nof import _ops, synthetic as syn  # noqa: E402
from nof.criteria import nof_loss  # noqa: E402
from nof.networks import Embedding, NOF_coarse, NOF_fine  # noqa: E402
from nof.render import render_rays_train  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rays", type=int, default=65536)
ap.add_argument("--samples", type=int, default=128)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--chunk", type=int, default=262144)
a = ap.parse_args()
dev = torch.device("cuda", 0)
rays = torch.from_numpy(syn.make_rays(a.rays, seed=0)).to(dev)
emb = Embedding(3, 10)
loss_fn = nof_loss["smoothl1"]()
_ops.set_activation_store_budget(1 << 62)


def models():
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(42)).to(dev).train(True)
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(43)).to(dev).train(True)
    return mc, mf


def step(mc, mf, seed):
    torch.manual_seed(seed)
    res = render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=32, N_samples=a.samples,
                            N_importance=2 * a.samples, perturb=1, noise_std=0, chunk=a.chunk, issegmentated=1,
                            childnerf_ratio=0.1, use_child_nerf_divide=0, use_child_nerf_loss=1)
    gt = rays[:, 14]
    loss = (1e-1 * loss_fn(1e1 * res["depth"], 1e1 * gt) + 1e-1 * loss_fn(1e1 * res["depth_fine"], 1e1 * gt)
            + 1e6 * res["child_free_loss_fine"] + 1e6 * res["child_free_loss"]
            + 1e5 * res["child_depth_loss_fine"] + 1e5 * res["child_depth_loss"])
    loss.backward()
    return loss


grads = {}
for mode in ("store", "remat"):
    _ops.set_train_backward(mode)
    mc, mf = models()
    loss = step(mc, mf, 7)
    grads[mode] = [p.grad.clone() for m in (mc, mf) for p in m.parameters()]
    print(f"{mode}: loss {float(loss):.6f}", flush=True)
worst = 0.0
names = [n for m in ("c", "f") for n, _ in NOF_coarse().named_parameters()]
for n, x, y in zip(names, grads["store"], grads["remat"]):
    sc = float(x.abs().max())
    d = float((x - y).abs().max()) / sc if sc > 0 else 0.0
    if n.endswith("weight") and x.dim() == 2:
        worst = max(worst, d)
    print(f"  {n:24s} max|store|={sc:.3e}  max|diff|/max={d:.2e}")
print(f"worst weight-matrix rel diff {worst:.2e}", flush=True)
for mode in ("store", "remat", "store", "remat"):
    _ops.set_train_backward(mode)
    mc, mf = models()
    step(mc, mf, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        for m in (mc, mf):
            m.zero_grad(set_to_none=True)
        step(mc, mf, 2 + i)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / a.steps
    print(f"{mode}: {ms:.1f} ms/step  {a.rays / ms * 1e3:.0f} rays/s (fwd+bwd, no optimizer)", flush=True)
    del mc, mf
    torch.cuda.empty_cache()
