"""Diagnostic: phase stamps of the split eval query k_nof_eval_h2 (variant library built with -DPCN_EH2_STAMP=1,
`make variants VARIANTS="stamp:-DPCN_EH2_STAMP=1" VARIANT_SRCS=csrc/nof_eval.hip`), or plain timing of any library.
Eval query over EH_RAYS rays x EH_S samples after ~2 s of back-to-back launches (steady clock), then one stamped
launch; prints a JSON line: median in-kernel clock, per-phase cycles (prologue, layers 0-7, occ_out), kernel ms."""
import ctypes
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "pc-nerf_amd"), HERE]
from nof import _hip as H  # noqa: E402
from nof import _ops, synthetic as syn  # noqa: E402
from nof.networks import NOF_coarse  # noqa: E402


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "pc-nerf_amd", "lib", "libpcnerf_hip.so")
    L = ctypes.CDLL(lib)
    for name, (res, args) in H._SIGS.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    dev = torch.device("cuda")
    n, S = int(os.environ.get("EH_RAYS", "16384")), int(os.environ.get("EH_S", "384"))
    rays = torch.from_numpy(syn.make_rays(n, seed=0)).to(dev)
    z = (torch.linspace(0, 1, S, device=dev)[None] * rays[:, 7:8]).contiguous()
    m = syn.load_into(NOF_coarse(), syn.init_nof_params(1)).to(dev).eval()
    s, keep = _ops._params(m)
    packed = torch.empty(L.pcnerf_nof_eval_packed_floats(), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    assert L.pcnerf_nof_pack_eval(ctypes.byref(s), packed.data_ptr(), st) == 0
    p = torch.empty_like(z)

    train = os.environ.get("EH_TRAIN", "0") == "1"
    if train:   # the fused train-mode query (chunk 262,144), stamps from chunk 0's blocks
        m.train()
        s, keep = _ops._params(m)
        chunk = int(os.environ.get("EH_CHUNK", "262144"))
        ws = torch.empty((getattr(L, 'pcnerf_nof_train_fused_bytes', None) or L.pcnerf_nof_train_fold_bytes)(n * S, chunk), dtype=torch.uint8, device=dev)

    def run():
        if train:
            assert L.pcnerf_nof_query_train_fused(rays.data_ptr(), n, rays.shape[1], z.data_ptr(), S, chunk,
                                                  ctypes.byref(s), 0.1, 1e-5, ws.data_ptr(), ws.numel(),
                                                  p.data_ptr(), st) == 0
            return
        assert L.pcnerf_nof_query_eval(rays.data_ptr(), n, rays.shape[1], z.data_ptr(), S, packed.data_ptr(),
                                       p.data_ptr(), st) == 0
    t0 = time.time()
    k = 0
    warm = float(os.environ.get("EH_WARM", "2.0"))
    while time.time() - t0 < warm:
        run()
        k += 1
        if k % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    reps = int(os.environ.get("EH_REPS", "5"))
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    out = {"lib": os.path.basename(lib), "train": train, "samples": n * S, "ms": e0.elapsed_time(e1) / reps}
    if hasattr(L, "pcnerf_debug_eh2_clock"):
        buf = (ctypes.c_double * 15)()
        L.pcnerf_debug_eh2_clock.restype = ctypes.c_int
        rc = L.pcnerf_debug_eh2_clock(buf)
        names = ["clock_MHz", "prologue", "L0", "L1", "L2", "L3", "L4", "L5", "L6", "L7", "occ_out", "L2_kloop",
                 "L2_epi_barrier", "L2_split", "blocks"]
        out["rc"] = rc
        out["phases_cycles"] = {nm: round(v, 1) for nm, v in zip(names, buf)}
        tot = sum(buf[i] for i in range(1, 11))
        out["block_cycles"] = tot
        # MFMA cycles per block at 32 cyc per v_mfma_f32_32x32x16_f16 per SIMD: 120 k-steps x 18 per wave
        out["mfma_cycles_per_block"] = 120 * 18 * 32
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
