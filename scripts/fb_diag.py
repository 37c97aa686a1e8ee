"""Diagnostic (GPU): the one-pass training backward (k_bwd_fused, activation store + fold state) against the
two-pass backward (no store) and the reference's gradient goldens, per parameter tensor."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "pc-nerf_amd"),
                os.path.join(os.path.dirname(HERE), "tests")]
from conftest import golden  # noqa: E402
from nof import _ops, synthetic as syn  # noqa: E402
from nof.criteria import nof_loss  # noqa: E402
from nof.networks import Embedding, NOF_coarse, NOF_fine  # noqa: E402
from nof import render as R  # noqa: E402

DEV = "cuda"


def grads(name, budget):
    g = golden(f"grads_{name}")
    prev = _ops.set_activation_store_budget(budget)
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(1234)).to(DEV).train(True)
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(5678)).to(DEV).train(True)
    rays = torch.from_numpy(g["rays"]).to(DEV)
    res = R.render_rays_train(mc, mf, Embedding(3, 10), rays, sub_nerf_test_num=32, N_samples=64, N_importance=128,
                              perturb=0, noise_std=0, chunk=4096, issegmentated=int(g["issegmentated"]),
                              childnerf_ratio=0.1, use_child_nerf_divide=int(g["use_child_nerf_divide"]),
                              use_child_nerf_loss=int(g["use_child_nerf_loss"]))
    loss = nof_loss["smoothl1"]()
    gt = rays[:, 14]
    tot = (1e-1 * loss(1e1 * res["depth"], 1e1 * gt) + 1e-1 * loss(1e1 * res["depth_fine"], 1e1 * gt)
           + 1e6 * (res["child_free_loss_fine"] + res["child_free_loss"])
           + 1e5 * (res["child_depth_loss_fine"] + res["child_depth_loss"]))
    tot.sum().backward()
    _ops.set_activation_store_budget(prev)
    out = {}
    for pre, m in (("c:", mc), ("f:", mf)):
        for k, p in m.named_parameters():
            out[pre + k] = p.grad.detach().cpu().numpy().copy()
    return out, g


for name in sys.argv[1:] or ["pcnerf", "original"]:
    a, g = grads(name, 1 << 40)   # store: the one-pass backward
    b, _ = grads(name, 0)         # no store: two-pass backward, chunks recomputed
    print(f"== {name}: max |one-pass - two-pass| / max |two-pass|, and each vs the reference golden")
    for k in a:
        if not k.endswith("weight"):
            continue
        ref = g[k] if k in g else None
        if ref is None and k + "@idx" in g:
            idx = g[k + "@idx"]
            ra, rb, rr = a[k].reshape(-1)[idx], b[k].reshape(-1)[idx], g[k + "@val"]
        else:
            ra, rb, rr = a[k].reshape(-1), b[k].reshape(-1), (ref.reshape(-1) if ref is not None else None)
        sc = np.abs(rb).max() + 1e-30
        line = f"{k:24s} a-b {np.abs(ra - rb).max() / sc:.2e}"
        if rr is not None:
            line += f"  a-ref {np.abs(ra - rr).max() / sc:.2e}  b-ref {np.abs(rb - rr).max() / sc:.2e}"
        print(line)
