"""A/B timing of the fused train-mode query (pcnerf_nof_query_train_fused, k_nof_eval_h3<true>) and the split eval
query (k_nof_eval_h3<false>) across variant libraries (pc-nerf_amd/lib/variants/*.so) in ONE process, interleaved
rounds on the same inputs (cdna_hip_programming.md 5.4 rule 24).  Prints per-variant median times and the max
relative output difference against the 'base' variant.   env: FA_RAYS, FA_S, FA_CHUNK, FA_ROUNDS, VB_ONLY, FA_STORE
(1: the train query writes the activation store of every chunk, pcnerf_nof_query_train_fused_store)."""
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


def load(path):
    L = ctypes.CDLL(path)
    for name, (res, args) in H._SIGS.items():
        f = getattr(L, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return L


def main():
    n = int(os.environ.get("FA_RAYS", "16384"))
    S = int(os.environ.get("FA_S", "384"))
    chunk = int(os.environ.get("FA_CHUNK", "262144"))
    rounds = int(os.environ.get("FA_ROUNDS", "6"))
    libs = sorted(glob.glob(os.path.join(HERE, "pc-nerf_amd", "lib", "variants", "*.so")))
    only = os.environ.get("VB_ONLY")
    if only:
        libs = [l for l in libs if os.path.basename(l)[10:-3] in only.split(",")]
    Ls = {os.path.basename(l)[10:-3]: load(l) for l in libs}
    dev = torch.device("cuda")
    rays = torch.from_numpy(syn.make_rays(n, seed=0)).to(dev)
    z = (torch.linspace(0, 1, S, device=dev)[None] * rays[:, 7:8]).contiguous()
    m = syn.load_into(NOF_coarse(), syn.init_nof_params(1)).to(dev)
    st = torch.cuda.current_stream().cuda_stream
    p = torch.empty_like(z)
    first = next(iter(Ls.values()))
    def need(L):   # the fused query's state: the fold's full layout when the store is written (the backward reads
        # it), else pcnerf_nof_train_fused_bytes where the library has it
        f = None if os.environ.get("FA_STORE") == "1" else getattr(L, "pcnerf_nof_train_fused_bytes", None)
        f = f or L.pcnerf_nof_train_fold_bytes
        f.restype, f.argtypes = ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int64]
        return f(n * S, chunk)
    ws = torch.empty(max(need(L) for L in Ls.values()), dtype=torch.uint8, device=dev)
    nst = (n * S + chunk - 1) // chunk if os.environ.get("FA_STORE") == "1" else 0   # activation store: all chunks
    store = torch.empty(nst * first.pcnerf_nof_store_bytes(chunk), dtype=torch.uint8, device=dev) if nst else None
    packed = torch.empty(first.pcnerf_nof_eval_packed_floats(), device=dev)
    times = {k: {"train": [], "eval": []} for k in Ls}
    tags = {16: "moments", 17: "algebra", 18: "train_query"}   # prof.h: per-kernel HIP events of the train query
    ktimes = {k: {v: [] for v in tags.values()} for k in Ls}
    outs = {}
    for rnd in range(rounds):
        for name, L in Ls.items():
            for mode in ("train", "eval"):
                if mode == "train":
                    m.train()
                    s, keep = _ops._params(m)
                else:
                    m.eval()
                    s, keep = _ops._params(m)
                    assert L.pcnerf_nof_pack_eval(ctypes.byref(s), packed.data_ptr(), st) == 0
                torch.cuda.synchronize()
                L.pcnerf_prof_enable(1 if mode == "train" else 0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if mode == "train" and nst:
                    rc = L.pcnerf_nof_query_train_fused_store(rays.data_ptr(), n, rays.shape[1], z.data_ptr(), S,
                                                              chunk, ctypes.byref(s), 0.0, 1e-5, ws.data_ptr(),
                                                              ws.numel(), p.data_ptr(), store.data_ptr(), nst, st)
                elif mode == "train":
                    rc = L.pcnerf_nof_query_train_fused(rays.data_ptr(), n, rays.shape[1], z.data_ptr(), S, chunk,
                                                        ctypes.byref(s), 0.0, 1e-5, ws.data_ptr(), ws.numel(),
                                                        p.data_ptr(), st)
                else:
                    rc = L.pcnerf_nof_query_eval(rays.data_ptr(), n, rays.shape[1], z.data_ptr(), S,
                                                 packed.data_ptr(), p.data_ptr(), st)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, L.pcnerf_last_error()
                if rnd == 0:
                    outs[(name, mode)] = p.clone()
                else:
                    times[name][mode].append(e0.elapsed_time(e1))
                    if mode == "train":
                        for tg, nm in tags.items():
                            tm, nn, fl, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
                            L.pcnerf_prof_read(tg, ctypes.byref(tm), ctypes.byref(nn), ctypes.byref(fl), ctypes.byref(by))
                            if nn.value:
                                ktimes[name][nm].append(tm.value)
                L.pcnerf_prof_enable(0)
    res = {}
    for name in Ls:
        r = {}
        for mode in ("train", "eval"):
            v = sorted(times[name][mode])
            r[mode + "_ms"] = round(v[len(v) // 2], 3)
            if ("base", mode) in outs:
                ref = outs[("base", mode)]
                d = (outs[(name, mode)] - ref).abs() / ref.abs().clamp_min(1e-12)
                r[mode + "_max_rel_vs_base"] = float(d.max())
        for nm, v in ktimes[name].items():
            if v:
                r[nm + "_ms"] = round(sorted(v)[len(v) // 2], 3)
        res[name] = r
    print(json.dumps({"rays": n, "S": S, "chunk": chunk, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
