"""A/B timing of kernel variant libraries (pc-nerf_amd/lib/variants/*.so) in ONE process, interleaved rounds
(cdna_hip_programming.md 5.4 rule 24).  Times the train-mode query (all chunks) and the eval query on the same
inputs; prints per-variant median kernel times per tag."""
import ctypes
import glob
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "pc-nerf_amd"), HERE]
from nof import _hip as H  # noqa: E402
from nof import _ops, synthetic as syn  # noqa: E402
from nof.networks import NOF_coarse  # noqa: E402

TAGS = {0: "eval", 1: "hidden", 2: "first", 3: "skip", 4: "out", 5: "fold", 10: "wgrad", 11: "dgrad",
        12: "bwd_other", 14: "wgrad_b3", 15: "h1"}


def load(path):
    L = ctypes.CDLL(path)
    for name, (res, args) in H._SIGS.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


def read(L, tag):
    t, n, f, b = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
    L.pcnerf_prof_read(tag, ctypes.byref(t), ctypes.byref(n), ctypes.byref(f), ctypes.byref(b))
    return t.value, n.value, f.value


def main():
    rays_n = int(os.environ.get("VB_RAYS", "16384"))
    S = int(os.environ.get("VB_S", "384"))
    chunk = int(os.environ.get("VB_CHUNK", "262144"))
    libs = sorted(glob.glob(os.path.join(HERE, "pc-nerf_amd", "lib", "variants", "*.so")))
    only = os.environ.get("VB_ONLY")
    if only:
        libs = [l for l in libs if os.path.basename(l)[10:-3] in only.split(",")]
    dev = torch.device("cuda")
    rays = torch.from_numpy(syn.make_rays(rays_n, seed=0)).to(dev)
    z = (torch.linspace(0, 1, S, device=dev)[None] * rays[:, 7:8]).contiguous()
    m = syn.load_into(NOF_coarse(), syn.init_nof_params(1)).to(dev).train()
    s, keep = _ops._params(m)
    p = torch.empty_like(z)
    Ls = {os.path.basename(l)[10:-3]: load(l) for l in libs}
    ws = torch.empty(max(L.pcnerf_nof_train_workspace_bytes(chunk) for L in Ls.values()), dtype=torch.uint8, device=dev)
    packed = torch.empty(Ls[next(iter(Ls))].pcnerf_nof_eval_packed_floats(), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    res = {k: {t: [] for t in TAGS} for k in Ls}
    qt = {}
    outs, gouts, eouts = {}, {}, {}
    bwd = os.environ.get("VB_BWD", "1") == "1"
    if bwd:   # backward on a quarter of the rays (its workspace holds all 8 layers of a chunk)
        rays_b, z_b = rays[: rays_n // 4].contiguous(), z[: rays_n // 4].contiguous()
        g_logit = torch.randn(z_b.shape, generator=torch.Generator().manual_seed(3)).to(dev) * 1e-3
        wsb = torch.empty(max(L.pcnerf_nof_backward_workspace_bytes(chunk) for L in Ls.values()), dtype=torch.uint8,
                          device=dev)
    for rnd in range(4):
        for name, L in Ls.items():
            L.pcnerf_prof_enable(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = L.pcnerf_nof_query_train(rays.data_ptr(), rays_n, 15, z.data_ptr(), S, chunk, ctypes.byref(s),
                                          0.0, 1e-5, ws.data_ptr(), ws.numel(), p.data_ptr(), st)
            assert rc == 0, L.pcnerf_last_error()
            e1.record()
            if rnd == 0:
                outs[name] = p.clone()   # train-mode query output of this variant (checked against 'base')
            if bwd:
                gs, gout = _ops._grads_struct(m, dev)
                rc = L.pcnerf_nof_query_train_backward(rays_b.data_ptr(), rays_b.shape[0], 15, z_b.data_ptr(), S,
                                                       chunk, ctypes.byref(s), 1e-5, g_logit.data_ptr(),
                                                       wsb.data_ptr(), wsb.numel(), ctypes.byref(gs), st)
                assert rc == 0, L.pcnerf_last_error()
                if rnd == 0:
                    gouts[name] = gout[3].clone()   # weight gradient of a hidden layer
            m.eval()
            L.pcnerf_nof_pack_eval(ctypes.byref(s), packed.data_ptr(), st)
            L.pcnerf_nof_query_eval(rays.data_ptr(), rays_n, 15, z.data_ptr(), S, packed.data_ptr(), p.data_ptr(), st)
            if rnd == 0:
                eouts[name] = p.clone()   # eval-mode query output of this variant
            m.train()
            torch.cuda.synchronize()
            if rnd == 0:
                continue  # warm-up round
            qt.setdefault(name, []).append(e0.elapsed_time(e1) * 1e3)   # whole train query (us)
            for t in TAGS:
                tm, n, f = read(L, t)
                if n:
                    res[name][t].append((tm / n * 1e3, f / (tm * 1e-3) / 1e12))
            L.pcnerf_prof_enable(0)
    out = {}
    clk = {}
    for name, L in Ls.items():
        try:
            f = L.pcnerf_debug_clock
        except AttributeError:
            continue
        f.restype, f.argtypes = ctypes.c_int, [ctypes.POINTER(ctypes.c_double)]
        buf = (ctypes.c_double * 8)()
        if f(buf) == 0:
            clk[name] = [round(x, 1) for x in buf]
    for name in Ls:
        out[name] = {TAGS[t]: {"us": round(sorted(v)[len(v) // 2][0], 1), "TF": round(sorted(v)[len(v) // 2][1], 1)}
                     for t, v in res[name].items() if v}
        if name in qt:
            out[name]["query_train_us"] = round(sorted(qt[name])[len(qt[name]) // 2], 1)
    ref = outs.get("base")
    if ref is not None:
        for name in Ls:
            d = (outs[name] - ref).abs() / ref.abs().clamp_min(1e-12)
            out[name]["max_rel_diff_vs_base"] = float(d.max())
            if name in eouts and "base" in eouts:
                er = eouts["base"]
                out[name]["eval_max_rel_diff_vs_base"] = float(((eouts[name] - er).abs() / er.abs().clamp_min(1e-12)).max())
            if name in gouts:
                gr = gouts["base"]
                out[name]["grad_max_rel_diff_vs_base"] = float(((gouts[name] - gr).abs().max() / gr.abs().max()))
    for name, c in clk.items():
        out[name]["clock_stamps"] = dict(zip(["MHz", "span_us", "prologue_us", "loop_us", "epilogue_us",
                                              "entry_spread_us", "exit_spread_us", "loopend_spread_us"], c))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
