"""Debug aid: run pcnerf_nof_forward_train through every variant library on the same embedded batch and report,
per layer, the max relative difference of the chunk statistics (workspace) vs the 'base' variant."""
import ctypes
import glob
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "pc-nerf_amd"), HERE]
from nof import _ops, synthetic as syn  # noqa: E402
from nof.networks import NOF_coarse  # noqa: E402
from variant_bench import load  # noqa: E402

n = int(os.environ.get("DBG_N", "4096"))
dev = torch.device("cuda")
m = syn.load_into(NOF_coarse(), syn.init_nof_params(1)).to(dev).train()
x = (torch.randn(n, 63, generator=torch.Generator().manual_seed(0))).to(dev)
s, keep = _ops._params(m)
res = {}
for path in sorted(glob.glob(os.path.join(HERE, "pc-nerf_amd", "lib", "variants", "*.so"))):
    name = os.path.basename(path)[10:-3]
    L = load(path)
    nb = L.pcnerf_nof_train_workspace_bytes(n)
    ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
    out = torch.empty(n, device=dev)
    rc = L.pcnerf_nof_forward_train(x.data_ptr(), n, ctypes.byref(s), 0.0, 1e-5, ws.data_ptr(), nb, out.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    tiles = (n + 31) // 32
    buf = tiles * 32 * 256 * 4
    rnd = lambda b: (b + 255) & ~255
    ost = 2 * rnd(buf) + rnd((2 * 8 * 64 * 4 * 8 + 7 * 32 * 8 * 64 * 4) * 4)  # approximate; located by search below
    res[name] = (ws.clone(), out.clone())
base_ws, base_out = res["base"]
for name, (w, o) in res.items():
    d = ((o - base_out).abs() / base_out.abs().clamp_min(1e-12)).max().item()
    # stats region = last 8*512 doubles of the carved workspace (before padding): compare bufA / bufB and stats
    tiles = (n + 31) // 32
    fb = tiles * 32 * 256 * 4
    A = w[:fb].view(torch.float32)
    B = w[((fb + 255) // 256) * 256:][:fb].view(torch.float32)
    bA = base_ws[:fb].view(torch.float32)
    bB = base_ws[((fb + 255) // 256) * 256:][:fb].view(torch.float32)
    dA = ((A - bA).abs() / bA.abs().clamp_min(1e-6)).max().item()
    dB = ((B - bB).abs() / bB.abs().clamp_min(1e-6)).max().item()
    badA = ((A - bA).abs() > 1e-3 * bA.abs().clamp_min(1e-3)).nonzero()
    first = badA[:8].flatten().tolist() if badA.numel() else []
    print(name, "p", d, "bufA", dA, "bufB", dB, "first bad A idx", first, "n bad", badA.numel())
