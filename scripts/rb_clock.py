"""Per-wave phase cycles of k_bwd_remat2 (diagnostic library built with -DPCN_RB_CLK=1:
`make -C pc-nerf_amd variants VARIANTS="clk:-DPCN_RB_CLK=1"`).  Runs one config-2 training step (forward +
backward) on that library and prints, per role (D = waves 0-3, W = waves 4-7), the mean shader cycles per tile of
phase A (D: data-gradient MFMAs; W: DMA issue + remat), phase B (D: epilogue; W: weight-gradient MFMAs) and the
end-of-tile wait + barrier, for the last layer-2 launch.   usage: PCNERF_HIP_LIB=... python scripts/rb_clock.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pc-nerf_amd"))
from nof import _hip, synthetic as syn  # noqa: E402
from nof.criteria import nof_loss  # noqa: E402
from nof.networks import Embedding, NOF_coarse, NOF_fine  # noqa: E402
from nof.render import render_rays_train  # noqa: E402

dev = torch.device("cuda", 0)
rays = torch.from_numpy(syn.make_rays(16384, seed=0)).to(dev)
emb = Embedding(3, 10)
lf = nof_loss["smoothl1"]()
mc = syn.load_into(NOF_coarse(), syn.init_nof_params(42)).to(dev).train(True)
mf = syn.load_into(NOF_fine(), syn.init_nof_params(43)).to(dev).train(True)
r = render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=32, N_samples=128, N_importance=256, perturb=1,
                      noise_std=0, chunk=262144, issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0,
                      use_child_nerf_loss=1)
gt = rays[:, 14]
(1e-1 * lf(1e1 * r["depth"], 1e1 * gt) + 1e-1 * lf(1e1 * r["depth_fine"], 1e1 * gt)
 + 1e6 * r["child_free_loss_fine"] + 1e5 * r["child_depth_loss_fine"]).backward()
torch.cuda.synchronize()
L = _hip.lib()
buf = np.zeros((4096, 5), dtype=np.uint64)
fn = L.pcnerf_debug_rbclk
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
b = buf.reshape(512, 8, 5).astype(np.float64)
nk = b[:, :, 4]
ok = nk > 0
for role, ws in (("D", slice(0, 4)), ("W", slice(4, 8))):
    sel = b[:, ws, :]
    n = sel[:, :, 4]
    m = n > 0
    per = sel[:, :, :4][m] / n[m][:, None]
    print(f"{role}: cycles per tile  A {per[:, 0].mean():7.0f}  B {per[:, 1].mean():7.0f}  wait+barrier "
          f"{per[:, 2].mean():7.0f}  loop {per[:, 3].mean():7.0f}   (A+B {per[:, 0].mean() + per[:, 1].mean():7.0f};"
          f" spread of loop p10/p90 {np.percentile(per[:, 3], 10):.0f}/{np.percentile(per[:, 3], 90):.0f})")
print(f"tiles per workgroup: {nk[ok].min():.0f}..{nk[ok].max():.0f}")
