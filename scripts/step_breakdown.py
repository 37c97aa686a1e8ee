"""Wall-time breakdown of one training step of bench.py --mode train_step (synchronised phases): forward render,
losses, backward, optimizer, and the activation-store allocations inside the forward.  Diagnostic only."""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "pc-nerf_amd"), HERE]
from nof import _ops, synthetic as syn  # noqa: E402
from nof.criteria import nof_loss  # noqa: E402
from nof.networks import Embedding, NOF_coarse, NOF_fine  # noqa: E402
from nof.render import render_rays_train  # noqa: E402

dev = torch.device("cuda")
rays = torch.from_numpy(syn.make_rays(65536, n_children=32, seed=0)).to(dev)
mc = syn.load_into(NOF_coarse(), syn.init_nof_params(1234)).to(dev).train()
mf = syn.load_into(NOF_fine(), syn.init_nof_params(5678)).to(dev).train()
emb, loss_fn = Embedding(3, 10), nof_loss["smoothl1"]()
opt = torch.optim.Adam(list(mc.parameters()) + list(mf.parameters()), lr=5e-4, eps=1e-8, weight_decay=1e-3)
gt = rays[:, 14].contiguous()
alloc_t = []
_init = _ops.ActivationStore.__init__


def timed_init(self, *a, **k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _init(self, *a, **k)
    torch.cuda.synchronize()
    alloc_t.append((time.perf_counter() - t0) * 1e3)


_ops.ActivationStore.__init__ = timed_init


def tick():
    torch.cuda.synchronize()
    return time.perf_counter()


for it in range(4):
    alloc_t.clear()
    t0 = tick()
    opt.zero_grad(set_to_none=True)
    res = render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=32, N_samples=128, N_importance=256, perturb=1,
                            noise_std=0, chunk=262144, issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0,
                            use_child_nerf_loss=1)
    t1 = tick()
    loss = (1e-1 * loss_fn(1e1 * res["depth"], 1e1 * gt) + 1e-1 * loss_fn(1e1 * res["depth_fine"], 1e1 * gt)
            + 1e6 * res["child_free_loss_fine"] + 1e6 * res["child_free_loss"]
            + 1e5 * res["child_depth_loss_fine"] + 1e5 * res["child_depth_loss"])
    t2 = tick()
    loss.backward()
    t3 = tick()
    opt.step()
    t4 = tick()
    print(f"step {it}: fwd {1e3 * (t1 - t0):.1f} ms (store allocs {[round(x, 2) for x in alloc_t]} ms), "
          f"losses {1e3 * (t2 - t1):.1f}, backward {1e3 * (t3 - t2):.1f}, adam {1e3 * (t4 - t3):.1f}, "
          f"total {1e3 * (t4 - t0):.1f} ms", flush=True)
