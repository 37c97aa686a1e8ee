"""A/B of the train-mode layer arithmetic in one process (diagnostic): fp32 MFMA vs the split-fp16 products.

For each mode: accuracy of render_rays_train on BASELINE config 2 at full size (65,536 rays, perturb 0) and on
the config-1 KITTI batch against the reference fixtures and the float64 evaluation (tests/golden/*_f64.npz), then
the headline step's time (train_fwd, perturb 1) with the per-kernel HIP events of its last step.
    python scripts/math_ab.py [--modes fp32,f16x2_3,f16x2_4] [--steps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "pc-nerf_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

from conftest import golden  # noqa: E402
from nof import _hip, _ops, synthetic as syn  # noqa: E402
from nof.criteria import nof_loss  # noqa: E402
from nof.networks import Embedding, NOF_coarse, NOF_fine  # noqa: E402
from nof.render import render_rays_train  # noqa: E402

DEV = torch.device("cuda")
KW = dict(use_child_nerf_loss=1, issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0, noise_std=0,
          chunk=262144)


def models(train=True):
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(1234)).to(DEV).train(train)
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(5678)).to(DEV).train(train)
    return mc, mf


def rel(a, b):
    a = a.detach().cpu().numpy().astype(np.float64) if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), 1e-6)


def accuracy(name, rays, g, f64, sub, S, I):
    mc, mf = models()
    with torch.no_grad():
        res = render_rays_train(mc, mf, Embedding(3, 10), rays, sub_nerf_test_num=sub, N_samples=S, N_importance=I,
                                perturb=0, **KW)
    out = {"depth_vs_ref_max": rel(res["depth"], g["depth"]).max(),
           "depth_vs_f64_max": rel(res["depth"], f64["depth"]).max(),
           "depth_fine_vs_f64_max": rel(res["depth_fine"], f64["depth_fine"]).max(),
           "depth_fine_vs_f64_p99": np.quantile(rel(res["depth_fine"], f64["depth_fine"]), 0.99),
           "depth_fine_vs_ref_max": rel(res["depth_fine"], g["depth_fine"]).max(),
           "depth_fine_vs_ref_frac_gt_1e-4": (rel(res["depth_fine"], g["depth_fine"]) > 1e-4).mean(),
           "ref_vs_f64_max": rel(g["depth_fine"], f64["depth_fine"]).max()}
    for k in ("child_free_loss", "child_depth_loss", "child_free_loss_fine", "child_depth_loss_fine"):
        out[k + "_vs_ref"] = rel(res[k], g[k]).max()
    return {name + ":" + k: float(v) for k, v in out.items()}


def timing(steps):
    rays = torch.from_numpy(syn.make_rays(65536, n_children=32, seed=0)).to(DEV)
    mc, mf = models()
    emb, sl1 = Embedding(3, 10), nof_loss["smoothl1"]()
    gt = rays[:, 14]
    L = _hip.lib()

    def step():
        res = render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=32, N_samples=128, N_importance=256, perturb=1,
                                **KW)
        return (1e-1 * sl1(1e1 * res["depth"], 1e1 * gt) + 1e-1 * sl1(1e1 * res["depth_fine"], 1e1 * gt)
                + 1e6 * (res["child_free_loss"] + res["child_free_loss_fine"])
                + 1e5 * (res["child_depth_loss"] + res["child_depth_loss_fine"]))

    with torch.no_grad():
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            if i == steps - 1:
                L.pcnerf_prof_enable(1)
            loss = step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
    ks = {}
    for tag, nm in ((1, "hidden"), (2, "first"), (3, "skip"), (4, "out")):
        tm, n, f, b = (ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double())
        L.pcnerf_prof_read(tag, ctypes.byref(tm), ctypes.byref(n), ctypes.byref(f), ctypes.byref(b))
        if n.value:
            ks[nm + "_us"] = round(1e3 * tm.value / n.value, 2)
            ks[nm + "_GBs"] = round(b.value / (tm.value * 1e-3) / 1e9, 1)
    L.pcnerf_prof_enable(0)
    return {"ms_per_step": round(1e3 * dt, 2), "rays_per_s": round(65536 / dt, 1), "loss": float(loss), **ks}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="fp32,f16x2_3,f16x2_4")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    g2, f2 = golden("config2_full"), golden("config2_full_f64")
    sc, g1, f1 = golden("scene_rays"), golden("config1_kitti"), golden("config1_kitti_f64")
    rays2 = torch.from_numpy(syn.make_rays(65536, n_children=32, seed=0)).to(DEV)
    rays1 = torch.from_numpy(sc["kitti_train"]).to(DEV)
    for mode in a.modes.split(","):
        _ops.set_train_math(mode)
        out = {"mode": mode}
        out.update(accuracy("config2", rays2, g2, f2, 32, 128, 256))
        out.update(accuracy("config1", rays1, g1, f1, int(g1["sub_nerf_test_num"]), 64, 128))
        out.update(timing(a.steps))
        print(json.dumps(out), flush=True)
    _ops.set_train_math("fp32")


if __name__ == "__main__":
    main()
