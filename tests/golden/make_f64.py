"""Float64 evaluations of the configs' render (fixtures <config>_f64.npz) and how far the reference's own float32
result is from them.

render_rays_train's depths are evaluated in float64 by the oracle (oracle/ref_cpu.py, the restatement pinned
against the reference at float32) from the reference's own float32 coarse sample positions and the same weights:
coarse z and points are rounded exactly as the reference rounds them (render.py:429-458), everything after --
embedding, network, BatchNorm statistics, compositing, sample_pdf, fine points -- runs in float64.  The reference's
float32 depth_fine sits up to ~1e-4 (config 2) / ~8e-4 (config 1, KITTI ranges) from this evaluation, as far as it
sits from itself run with another thread count (gen_self_spread in make_golden.py): the fine samples land where
the 2^9 encoding frequency turns one ulp of position into ~1e-4 of occupancy.  The GPU tests therefore hold the
HIP depth_fine to 1e-4 of this float64 evaluation, and to the reference within the reference's own spread.

    python tests/golden/make_f64.py config1 [--save]   (KITTI-00 4,096-ray batch, 64/128)
    python tests/golden/make_f64.py config4 [--save]   (MaiCity blocks, 128/256)
    python tests/golden/make_f64.py config2 [--save]   (65,536 rays, 128/256; ~10 minutes on 8 cores)
    (config 3's float64 evaluation: tests/golden/make_config3_full.py f64)
    python tests/golden/make_f64.py grads [--save]     (float64 gradients of the 96-ray gradient goldens)
Optional: --hip <npz with depth, depth_fine> compares a HIP run too.
Test infrastructure (imports the oracle)."""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "pc-nerf_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from conftest import golden  # noqa: E402
from nof import synthetic as syn  # noqa: E402
from oracle import ref_cpu as O  # noqa: E402


def render64(Pc, Pf, rays32, S, I, chunk, ratio=0.1, training=True):
    """render_rays_train (training, segmented) or render_rays_val (eval BatchNorm, plain linspace) depths."""
    P64 = lambda P: {k: (v.double() if v.is_floating_point() else v) for k, v in P.items()}
    Pc, Pf = P64(Pc), P64(Pf)
    z = O.coarse_z(rays32, S, training, ratio)                   # float32 positions, as the reference
    pts = O.points(rays32, z).double()
    rays = rays32.double()

    def q(P, pts):
        R_, S_ = pts.shape[:2]
        flat = pts.reshape(-1, 3)
        out = [O.nof_forward(P, O.embed(flat[i:i + chunk]), training) for i in range(0, flat.shape[0], chunk)]
        return torch.cat(out).view(R_, S_)

    p = q(Pc, pts)
    w, depth = O.composite(p, z.double())
    zmid = .5 * (z[..., 1:] + z[..., :-1]).double()
    zs = O.sample_pdf(zmid, w[..., 1:-1], I, det=True)
    zf = torch.sort(torch.cat([z.double(), zs], -1), -1)[0]
    pf = q(Pf, rays[:, None, 0:3] + rays[:, None, 3:6] * zf[..., None])
    _, depth_f = O.composite(pf, zf)
    return depth.numpy(), depth_f.numpy()


def stats(name, a, b):
    rel = np.abs(a.astype(np.float64) - b) / np.maximum(np.abs(b), 1e-6)
    print(f"{name:28s} max {rel.max():.3e}  p99.9 {np.quantile(rel, 0.999):.3e}  p99 {np.quantile(rel, 0.99):.3e}  "
          f"median {np.median(rel):.3e}  >1e-4: {(rel > 1e-4).mean() * 100:.3f} %")


def grads64(save):
    """Float64 parameter gradients for the 96-ray gradient goldens (grads_<case>.npz, made from the reference by
    make_golden.gen_grads): the oracle's render_rays_train(f64=True) -- the reference's float32 coarse positions,
    everything after them in float64 -- with float64 leaves, the train_kitti.py:117-155 loss, backward.  Stored in
    the same golden file under ``f64:`` keys at the golden's own entry indices: how far the reference's float32
    gradients sit from the exact evaluation, per entry (the fine network's gradients go through fine samples that
    sample_pdf places where one float32 ulp of a coarse weight moves them)."""
    cases = {"pcnerf": 0, "divide": 1, "original": 0}
    for name, div in cases.items():
        path = os.path.join(HERE, f"grads_{name}.npz")
        g = dict(np.load(path, allow_pickle=False))
        P = {}
        for pre, seed in (("c:", 1234), ("f:", 5678)):
            Q = O.params_from_numpy(syn.init_nof_params(seed))
            Q = {k: (v.double() if v.is_floating_point() else v) for k, v in Q.items()}
            for k in Q:
                if k.endswith(".weight") or k.endswith(".bias"):
                    Q[k].requires_grad_(True)
            P[pre] = Q
        rays = torch.from_numpy(g["rays"])
        cl, seg = int(g["use_child_nerf_loss"]), int(g["issegmentated"])
        ro = O.render_rays_train(P["c:"], P["f:"], rays, sub_nerf_test_num=32, N_samples=64, N_importance=128,
                                 perturb=0, noise_std=0, chunk=4096, issegmentated=seg, childnerf_ratio=0.1,
                                 use_child_nerf_divide=div, use_child_nerf_loss=cl, f64=True)
        r64 = rays.double()
        lr, lrf = O.range_losses(ro["depth"], ro["depth_fine"], r64[:, 14], r64, div, 32)
        tot = O.total_loss(ro, lr, lrf)
        tot.sum().backward()
        out = {"f64:loss_total": tot.detach().numpy()}
        for pre, Q in P.items():
            for k, t in Q.items():
                if t.grad is None:
                    continue
                gr = t.grad.numpy()
                if pre + k in g:
                    out["f64:" + pre + k] = gr
                elif pre + k + "@idx" in g:
                    out["f64:" + pre + k + "@val"] = gr.reshape(-1)[g[pre + k + "@idx"]]
                    out["f64:" + pre + k + "@norm"] = np.linalg.norm(gr)
        i = list(g["f:layer1.0.weight@idx"]).index(g["f:layer1.0.weight@idx"][0])
        print(name, "loss ref", float(g["loss_total"].sum()), "f64", float(tot.sum()))
        if save:
            g = {k: v for k, v in g.items() if not k.startswith("f64:")}
            g.update(out)
            np.savez_compressed(path, **g)
            print("wrote", path)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "grads":
        torch.set_num_threads(os.cpu_count() or 1)
        grads64("--save" in sys.argv)
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["config1", "config2", "config4"])
    ap.add_argument("--hip", default=None)
    ap.add_argument("--save", action="store_true", help=f"write tests/golden/<config>_f64.npz")
    a = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 1)
    cases = []
    if a.config == "config1":
        sc, g = golden("scene_rays"), golden("config1_kitti")
        cases.append(("", torch.from_numpy(sc["kitti_train"]), 1234, 5678, 64, 128, g))
    elif a.config == "config4":
        sc, g = golden("scene_rays"), golden("config4_maicity")
        for b in range(4):
            cases.append((f"b{b}_", torch.from_numpy(sc[f"maicity_b{b}"]), 1234 + b, 5678 + b, 128, 256, g))
    else:
        g = golden("config2_full")
        cases.append(("", torch.from_numpy(syn.make_rays(65536, seed=0)), 1234, 5678, 128, 256, g))
    hip = dict(np.load(a.hip)) if a.hip else None
    saved = {}
    with torch.no_grad():
        for pre, rays, sc_, sf_, S, I, g in cases:
            d64, df64 = render64(O.params_from_numpy(syn.init_nof_params(sc_)),
                                 O.params_from_numpy(syn.init_nof_params(sf_)), rays, S, I, 262144)
            saved[pre + "depth"], saved[pre + "depth_fine"] = d64, df64
            if a.config == "config1":   # the val split through render_rays_val (eval mode)
                v64, vf64 = render64(O.params_from_numpy(syn.init_nof_params(sc_)),
                                     O.params_from_numpy(syn.init_nof_params(sf_)),
                                     torch.from_numpy(golden("scene_rays")["kitti_val"]), S, I, 262144, training=False)
                saved["val_depth"], saved["val_depth_fine"] = v64, vf64
                stats("config1 val ref depth_fine", g["val_depth_fine"], vf64)
            stats(f"{a.config} {pre}ref depth", g[pre + "depth"], d64)
            stats(f"{a.config} {pre}ref depth_fine", g[pre + "depth_fine"], df64)
            if hip is not None:
                stats(f"{a.config} {pre}hip depth", hip[pre + "depth"], d64)
                stats(f"{a.config} {pre}hip depth_fine", hip[pre + "depth_fine"], df64)
                stats(f"{a.config} {pre}hip vs ref depth_fine", hip[pre + "depth_fine"], g[pre + "depth_fine"])
    if a.save:
        name = {"config1": "config1_kitti", "config2": "config2_full", "config4": "config4_maicity"}[a.config]
        path = os.path.join(HERE, name + "_f64.npz")
        np.savez_compressed(path, **saved)
        print("wrote", path)


if __name__ == "__main__":
    main()
