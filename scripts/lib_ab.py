"""Same-process timing A/B of variant libraries (pc-nerf_amd/lib/variants/libpcnerf_<name>.so, built with
`make -C pc-nerf_amd variants`) on the config-2 training step (fwd + bwd, no optimizer): each variant is loaded in
its own subprocess in turn, ROUNDS times interleaved; prints ms/step per variant and round.  Timing-only variants
(ablations) give wrong numbers by design.   usage: python scripts/lib_ab.py name1 name2 ... [--rays N]"""
import argparse
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ap = argparse.ArgumentParser()
ap.add_argument("names", nargs="+")
ap.add_argument("--rays", type=int, default=65536)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--fwd", action="store_true", help="the render + loss forward only (the headline), no backward")
a = ap.parse_args()
CHILD = r'''
import sys, time, torch
sys.path.insert(0, "%s")
from nof import _ops, synthetic as syn
from nof.criteria import nof_loss
from nof.networks import Embedding, NOF_coarse, NOF_fine
from nof.render import render_rays_train
dev = torch.device("cuda", 0)
rays = torch.from_numpy(syn.make_rays(%d, seed=0)).to(dev)
emb = Embedding(3, 10); lf = nof_loss["smoothl1"]()
mc = syn.load_into(NOF_coarse(), syn.init_nof_params(42)).to(dev).train(True)
mf = syn.load_into(NOF_fine(), syn.init_nof_params(43)).to(dev).train(True)
def step():
  with torch.set_grad_enabled(%s):
    for m in (mc, mf): m.zero_grad(set_to_none=True)
    r = render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=32, N_samples=128, N_importance=256, perturb=1,
                          noise_std=0, chunk=262144, issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0,
                          use_child_nerf_loss=1)
    gt = rays[:, 14]
    loss = (1e-1 * lf(1e1 * r["depth"], 1e1 * gt) + 1e-1 * lf(1e1 * r["depth_fine"], 1e1 * gt)
            + 1e6 * r["child_free_loss_fine"] + 1e5 * r["child_depth_loss_fine"])
    if %s: loss.backward()
step(); torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(%d): step()
torch.cuda.synchronize()
print("%%.2f" %% (1e3 * (time.perf_counter() - t0) / %d))
''' % (os.path.join(HERE, "..", "pc-nerf_amd"), a.rays, not a.fwd, not a.fwd, a.steps, a.steps)
for rnd in range(a.rounds):
    for nm in a.names:
        lib = os.path.join(HERE, "..", "pc-nerf_amd", "lib", "variants", f"libpcnerf_{nm}.so")
        env = dict(os.environ, PCNERF_HIP_LIB=lib)
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        ms = out.stdout.strip().splitlines()[-1] if out.returncode == 0 and out.stdout.strip() else "FAIL " + out.stderr[-300:]
        print(f"round {rnd} {nm}: {ms} ms/step", flush=True)
