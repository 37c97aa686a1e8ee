"""Tensor-level wrappers over the C ABI (include/pcnerf_hip.h).

Every function takes ROCm device tensors, allocates its outputs with torch (memory only), and enqueues the HIP
kernels on the current stream.  Nothing here computes on the host.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _hip as H

# ----------------------------------------------------------------------------------------------- utilities
_ws_cache: dict = {}


def _workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """Grow-only scratch buffer per device (torch caching allocator memory)."""
    key = (device.type, device.index)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf


def _f32(t: torch.Tensor) -> torch.Tensor:
    H.require_device(t)
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _bn_config(model):
    norms = model.norms()
    mom, eps = norms[0].momentum, norms[0].eps
    for bn in norms:
        if bn.momentum != mom or bn.eps != eps or not bn.track_running_stats or not bn.affine:
            raise NotImplementedError("HIP NOF kernels need identical affine BatchNorm1d layers with running stats")
    if mom is None:
        raise NotImplementedError("BatchNorm1d(momentum=None) (cumulative averaging) is not supported")
    return float(mom), float(eps)


def _params(model) -> tuple[H.NofParams, list]:
    """Device pointers of a NOF module's parameters in reference state_dict order."""
    keep = []
    s = H.NofParams()

    def p(t):
        H.require_device(t)
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError("NOF parameters must be contiguous float32 device tensors")
        keep.append(t)
        return t.data_ptr()

    for i, lin in enumerate(model.linears()):
        s.lin_w[i] = p(lin.weight)
        s.lin_b[i] = p(lin.bias)
    for i, bn in enumerate(model.norms()):
        s.bn_w[i] = p(bn.weight)
        s.bn_b[i] = p(bn.bias)
        s.bn_rm[i] = p(bn.running_mean)
        s.bn_rv[i] = p(bn.running_var)
    s.out_w = p(model.occ_out[0].weight)
    s.out_b = p(model.occ_out[0].bias)
    return s, keep


def _stream(t: torch.Tensor):
    return H.stream_of(t)


# ----------------------------------------------------------------------------------------------- network
def pack_eval(model, device) -> torch.Tensor:
    """Eval-mode network image (BN folded, MFMA operand order); rebuilt per call (weights may change)."""
    L = H.lib()
    out = torch.empty(L.pcnerf_nof_eval_packed_floats(), dtype=torch.float32, device=device)
    s, keep = _params(model)
    _bn_config(model)
    H.check(L.pcnerf_nof_pack_eval(ctypes.byref(s), out.data_ptr(), _stream(out)))
    return out


# Exact affine fold of the eval network (opt-in; SURVEY fact 1: every LeakyReLU(True) is the identity, so the
# eval-mode NOF is sigmoid(a . emb + c)).  Off by default: the drop-in evaluates the module as written.
_EVAL_FOLD = os.environ.get("PCNERF_EVAL_FOLD", "0") == "1"


def set_eval_fold(enabled: bool) -> bool:
    """Route eval-mode NOF queries through the exact affine fold (True) or the full network (False, default).
    Returns the previous setting."""
    global _EVAL_FOLD
    prev, _EVAL_FOLD = _EVAL_FOLD, bool(enabled)
    return prev


def eval_fold_enabled() -> bool:
    return _EVAL_FOLD


def fold_eval(model, device) -> torch.Tensor:
    """(a, c) of the eval network as 64 float64 (a = fold[:63], c = fold[63]); rebuilt per call."""
    L = H.lib()
    out = torch.empty(64, dtype=torch.float64, device=device)
    s, keep = _params(model)
    _bn_config(model)
    H.check(L.pcnerf_nof_fold_eval(ctypes.byref(s), out.data_ptr(), _stream(out)))
    return out


# Arithmetic of the train-mode MLP, forward and backward (pcnerf_set_train_math): fp32 operands split into two fp16
# parts (22 significant bits) with exact products on the fp16 matrix pipe and fp32 accumulation, "f16x2_3"
# (hi*hi + hi*mid + mid*hi) or "f16x2_4" (+ mid*mid) -- the weight gradients under either as f16x2 / three bf16
# parts -- or "fp32" (fp32 MFMA throughout).  "f16x2_3_fused" (default): f16x2_3, except that a train-mode query
# whose layer outputs no backward reads (the render+loss forward, NOF.forward without autograd) runs as ONE fused
# per-sample kernel with each chunk's BatchNorm batch statistics taken from the chunk's encoding moments
# (pcnerf_nof_query_train_fused) instead of layer by layer through HBM.
TRAIN_MATH = {"fp32": 0, "f16x2_3": 1, "f16x2_4": 2, "f16x2_3_fused": 1}
_TRAIN_FUSED = True   # the library's own default is mode 1 (f16x2_3)


def set_remat_version(version: int) -> int:
    """Select the default training backward's layer kernel (4: k_bwd_remat3 with the BatchNorm-backward epilogue on
    the W waves, the default; 3: k_bwd_remat3 with it on the D waves; 2: k_bwd_remat2); returns the previous one
    (pcnerf_set_remat_version)."""
    prev = H.lib().pcnerf_set_remat_version(int(version))
    if prev < 0:
        raise RuntimeError(H.lib().pcnerf_last_error().decode())
    return prev


def get_remat_version() -> int:
    v = set_remat_version(4)
    set_remat_version(v)
    return v


def set_composite_group(group: int) -> int:
    """The compositing kernels' ray group: 0 automatic (default), 64 a wave per ray, 256 a workgroup per ray
    (pcnerf_set_composite_group); returns the previous setting."""
    prev = H.lib().pcnerf_set_composite_group(int(group))
    if prev < 0:
        raise RuntimeError(H.lib().pcnerf_last_error().decode())
    return prev


def set_train_math(mode: str) -> str:
    """Select the train-mode layer arithmetic; returns the previous mode's name."""
    global _TRAIN_FUSED
    if mode not in TRAIN_MATH:
        raise ValueError(f"train math must be one of {sorted(TRAIN_MATH)}")
    prev = H.lib().pcnerf_set_train_math(TRAIN_MATH[mode])
    if prev < 0:
        raise RuntimeError(H.lib().pcnerf_last_error().decode())
    prev_name = "f16x2_3_fused" if (prev == 1 and _TRAIN_FUSED) else {0: "fp32", 1: "f16x2_3", 2: "f16x2_4"}[prev]
    _TRAIN_FUSED = mode == "f16x2_3_fused"
    return prev_name


def get_train_math() -> str:
    prev = set_train_math("fp32")
    set_train_math(prev)
    return prev


if os.environ.get("PCNERF_TRAIN_MATH"):
    set_train_math(os.environ["PCNERF_TRAIN_MATH"])

# Arithmetic of the fused eval-mode query (pcnerf_set_eval_math): "f16x2_3" (default; the split products of the
# train math, weights scaled per layer and activations per sample) or "fp32" (fp32 MFMA).
EVAL_MATH = {"fp32": 0, "f16x2_3": 1}


def set_eval_math(mode: str) -> str:
    """Select the eval-mode query arithmetic; returns the previous mode's name."""
    if mode not in EVAL_MATH:
        raise ValueError(f"eval math must be one of {sorted(EVAL_MATH)}")
    prev = H.lib().pcnerf_set_eval_math(EVAL_MATH[mode])
    if prev < 0:
        raise RuntimeError(H.lib().pcnerf_last_error().decode())
    return {v: k for k, v in EVAL_MATH.items()}[prev]


def get_eval_math() -> str:
    prev = set_eval_math("fp32")
    set_eval_math(prev)
    return prev


if os.environ.get("PCNERF_EVAL_MATH"):
    set_eval_math(os.environ["PCNERF_EVAL_MATH"])


# render_rays' depth2 (render.py:598-600) ranks the last sample in argsort(weights, descending=True); where weights
# tie exactly (every weight after an opaque sample is 0) the order of equal keys decides.  "stable" (default): the
# order torch's sort gives on the GPU, where the reference runs render_rays (it moves the draws to cuda:0,
# render.py:397) -- rows longer than 32 go through torch's merge / radix sort, which are stable.  "cpu": torch CPU's
# std::sort (introsort) order, for comparing with CPU runs of the reference (the committed goldens).
_DEPTH2_ORDER = {"stable": 0, "cpu": 1}
_depth2_order = "stable"


def set_depth2_order(order: str) -> str:
    """Select depth2's order of equal weights; returns the previous one.  A process-wide setting (the library keeps
    one static): every thread and stream of the process renders with it.  For rows of at most 32 samples torch's GPU
    sort is a bitonic network, which does NOT keep equal keys in index order, so for S <= 32 neither setting is
    the order a GPU run of the reference would give there: depth2's tie order is parity-unpinned for such rows
    (no reference GPU output exists to pin either order; the goldens pin "cpu")."""
    global _depth2_order
    if order not in _DEPTH2_ORDER:
        raise ValueError(f"depth2 order must be one of {sorted(_DEPTH2_ORDER)}")
    H.check(H.lib().pcnerf_set_depth2_order(_DEPTH2_ORDER[order]))
    prev, _depth2_order = _depth2_order, order
    return prev


# Exact affine fold of the TRAIN-mode network (opt-in): every layer's BatchNorm batch statistics
# follow from the chunk's encoding mean and covariance, so each chunk's network is sigmoid(a_c . emb + c_c)
# (csrc/nof_fold.hip).  Off by default: the drop-in evaluates the module as written.
_TRAIN_FOLD = os.environ.get("PCNERF_TRAIN_FOLD", "0") == "1"


def set_train_fold(enabled: bool) -> bool:
    """Route train-mode NOF queries (forward and backward) through the exact affine fold (True) or the full
    network (False, default).  Returns the previous setting."""
    global _TRAIN_FOLD
    prev, _TRAIN_FOLD = _TRAIN_FOLD, bool(enabled)
    return prev


def train_fold_enabled() -> bool:
    return _TRAIN_FOLD


def fold_state(device, total_samples: int, chunk: int) -> torch.Tensor:
    """Device buffer of the train fold's per-chunk moments and layer maps (forward -> backward)."""
    n = int(H.lib().pcnerf_nof_train_fold_bytes(int(total_samples), int(chunk)))
    return torch.empty((max(n, 1),), dtype=torch.uint8, device=device)


# The active data-parallel BatchNorm recorder (nof.bn_sync.BnSync.record), or None: train-mode queries hand it their
# per-chunk batch statistics.
_BN_REC = None


def _bn_before(model):
    if _BN_REC is not None:
        _BN_REC.before(model)


def _bn_after(model, state: torch.Tensor, total: int, chunk: int):
    if _BN_REC is not None:
        _BN_REC.after(model, state, total, chunk)


def _bn_unsupported():
    """A train-mode query under a layered train math (f16x2_3, f16x2_4, fp32): it keeps no per-chunk statistics
    record, so the active recorder is told, and its sync() leaves every rank's running statistics as that rank's own
    forward set them (the per-rank behaviour of Lightning's DDP without sync_batchnorm), with a one-time warning."""
    if _BN_REC is not None:
        _BN_REC.mark_unsupported()


def bn_chunk_stats(state: torch.Tensor, total: int, chunk: int) -> torch.Tensor:
    """(C, 8, 2, 256) float64: each BatchNorm chunk's mean of h_L (bias included) and biased variance, read from a
    fused / fold train query's state right after its forward (pcnerf_nof_train_bn_stats)."""
    chunk = max(1, min(int(chunk), int(total)))
    C = -(-int(total) // chunk)
    out = torch.empty((C, 8, 2, 256), dtype=torch.float64, device=state.device)
    H.check(H.lib().pcnerf_nof_train_bn_stats(state.data_ptr(), state.numel(), int(total), chunk, out.data_ptr(),
                                              _stream(state)))
    return out


def bn_running_replay(model, stats: torch.Tensor, ns: torch.Tensor) -> None:
    """Advance the model's running_mean / running_var over the chunks' statistics ``stats`` (n, 8, 2, 256) float64
    in order, ``ns`` (n,) int64 their sample counts (pcnerf_bn_running_replay: the forward's own arithmetic)."""
    stats = stats.contiguous()
    ns = ns.to(device=stats.device, dtype=torch.int64).contiguous()
    if stats.dim() != 4 or tuple(stats.shape[1:]) != (8, 2, 256) or ns.numel() != stats.shape[0]:
        raise ValueError("stats must be (n, 8, 2, 256) with one sample count per chunk")
    mom, _ = _bn_config(model)
    s, keep = _params(model)
    H.check(H.lib().pcnerf_bn_running_replay(ctypes.byref(s), mom, stats.data_ptr(), ns.data_ptr(), stats.shape[0],
                                             _stream(stats)))


def _track_batches(model, n_chunks: int) -> None:
    for bn in model.norms():
        if bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(n_chunks)


# The training backward under the default train math ("f16x2_3_fused"): "remat" (default since round 5) keeps no
# activations -- the forward keeps only its fold state and the backward rematerialises each layer's input per tile
# from the chunk's encoding (pcnerf_nof_query_train_backward_remat); "store" is round 4's activation store (the
# forward writes the layer outputs of the chunks its budget holds, the rest are recomputed layer by layer).
_TRAIN_BACKWARD = os.environ.get("PCNERF_TRAIN_BACKWARD", "remat")


def set_train_backward(mode: str) -> str:
    """Select the default train math's backward ("remat" or "store"); returns the previous one."""
    global _TRAIN_BACKWARD
    if mode not in ("remat", "store"):
        raise ValueError("train backward must be 'remat' or 'store'")
    prev, _TRAIN_BACKWARD = _TRAIN_BACKWARD, mode
    return prev


def remat_enabled() -> bool:
    """True when a train-mode render pass keeps no activations (default train math, remat backward)."""
    return _TRAIN_FUSED and _TRAIN_BACKWARD == "remat" and not _TRAIN_FOLD


def query(model, rays: torch.Tensor, z: torch.Tensor, chunk: int, store=None, fold=None, keep=None) -> torch.Tensor:
    """Occupancy p (R, S) of the samples o + d*z through Embedding + NOF (render.py:18-25 / 44-51).
    ``store`` (train mode): an ActivationStore whose chunks keep the layer outputs for the backward.
    ``fold`` (train mode): a fold_state buffer -- the query runs through the train fold and keeps its state there
    (also taken, with a temporary buffer, when set_train_fold(True)).
    ``keep`` (train mode, default math): a fold_state buffer the fused query keeps its state in for
    nof_query_backward_remat."""
    L = H.lib()
    R, S = z.shape
    p = torch.empty((R, S), dtype=torch.float32, device=z.device)
    st = _stream(z)
    if model.training and keep is not None:
        if not _TRAIN_FUSED:
            raise RuntimeError("query(keep=...) needs the default train math (f16x2_3_fused)")
        chunk = max(1, min(int(chunk), R * S))
        mom, eps = _bn_config(model)
        s, keep_params = _params(model)
        _bn_before(model)
        H.check(L.pcnerf_nof_query_train_fused_state(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, int(chunk),
                                                     ctypes.byref(s), mom, eps, keep.data_ptr(), keep.numel(),
                                                     p.data_ptr(), st))
        _bn_after(model, keep, R * S, chunk)
        _track_batches(model, -(-R * S // int(chunk)))
    elif model.training and (fold is not None or _TRAIN_FOLD):
        chunk = max(1, min(int(chunk), R * S))
        mom, eps = _bn_config(model)
        s, keep = _params(model)
        if fold is None:
            fold = fold_state(z.device, R * S, chunk)
        _bn_before(model)
        H.check(L.pcnerf_nof_query_train_fold(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, int(chunk),
                                              ctypes.byref(s), mom, eps, fold.data_ptr(), fold.numel(),
                                              p.data_ptr(), st))
        _bn_after(model, fold, R * S, chunk)
        _track_batches(model, -(-R * S // int(chunk)))
    elif model.training and _TRAIN_FUSED:
        # the network per sample in one fused kernel; with an activation store it also writes the stored chunks'
        # raw layer outputs and BatchNorm sums for the backward (the layered store forward's layout)
        chunk = max(1, min(int(chunk), R * S))
        mom, eps = _bn_config(model)
        s, keep = _params(model)
        _bn_before(model)
        if store is not None and store.n_chunks > 0:
            # the state (the chunks' encoding moments and layer maps) is the backward's too: kept with the store
            store.fstate = fold_state(z.device, R * S, chunk)
            H.check(L.pcnerf_nof_query_train_fused_store(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S,
                                                         int(chunk), ctypes.byref(s), mom, eps,
                                                         store.fstate.data_ptr(), store.fstate.numel(), p.data_ptr(),
                                                         store.buf.data_ptr(), store.n_chunks, st))
            _bn_after(model, store.fstate, R * S, chunk)
        else:
            ws = _workspace(z.device, int(L.pcnerf_nof_train_fused_bytes(R * S, chunk)))
            H.check(L.pcnerf_nof_query_train_fused(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, int(chunk),
                                                   ctypes.byref(s), mom, eps, ws.data_ptr(), ws.numel(),
                                                   p.data_ptr(), st))
            _bn_after(model, ws, R * S, chunk)
        _track_batches(model, -(-R * S // int(chunk)))
    elif model.training:
        _bn_unsupported()
        chunk = max(1, min(int(chunk), R * S))   # a larger chunk is the same single BatchNorm chunk
        mom, eps = _bn_config(model)
        s, keep = _params(model)
        nbytes = L.pcnerf_nof_train_workspace_bytes(int(chunk))
        ws = _workspace(z.device, nbytes)
        if store is not None and store.n_chunks > 0:
            H.check(L.pcnerf_nof_query_train_store(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, int(chunk),
                                                   ctypes.byref(s), mom, eps, ws.data_ptr(), ws.numel(),
                                                   p.data_ptr(), store.buf.data_ptr(), store.n_chunks, st))
        else:
            H.check(L.pcnerf_nof_query_train(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, int(chunk),
                                             ctypes.byref(s), mom, eps, ws.data_ptr(), ws.numel(), p.data_ptr(), st))
        _track_batches(model, -(-R * S // int(chunk)))
    elif _EVAL_FOLD:
        fold = fold_eval(model, z.device)
        H.check(L.pcnerf_nof_query_eval_fold(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, fold.data_ptr(),
                                             p.data_ptr(), st))
    else:
        packed = pack_eval(model, z.device)
        H.check(L.pcnerf_nof_query_eval(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, packed.data_ptr(),
                                        p.data_ptr(), st))
    return p


def nof_forward_embedded(model, x: torch.Tensor, with_fold_state: bool = False):
    """NOF.forward on a (B, 63) embedded batch (one BatchNorm batch in train mode).  ``with_fold_state``: return
    (p, fold state or None) -- the state the train fold's backward needs when set_train_fold(True)."""
    L = H.lib()
    x = _f32(x)
    if x.dim() != 2 or x.shape[1] != 63:
        raise RuntimeError(f"expected (B, 63) embedded input, got {tuple(x.shape)}")
    B = x.shape[0]
    out = torch.empty((B, 1), dtype=torch.float32, device=x.device)
    st = _stream(x)
    fold = None
    if model.training and _TRAIN_FOLD:
        if B <= 1:
            raise ValueError("Expected more than 1 value per channel when training")
        mom, eps = _bn_config(model)
        s, keep = _params(model)
        fold = fold_state(x.device, B, B)
        _bn_before(model)
        H.check(L.pcnerf_nof_forward_train_fold(x.data_ptr(), B, ctypes.byref(s), mom, eps, fold.data_ptr(),
                                                fold.numel(), out.data_ptr(), st))
        _bn_after(model, fold, B, B)
        _track_batches(model, 1)
    elif model.training and _TRAIN_FUSED:
        if B <= 1:
            raise ValueError("Expected more than 1 value per channel when training")
        mom, eps = _bn_config(model)
        s, keep = _params(model)
        ws = _workspace(x.device, int(L.pcnerf_nof_train_fused_bytes(B, B)))
        _bn_before(model)
        H.check(L.pcnerf_nof_forward_train_fused(x.data_ptr(), B, ctypes.byref(s), mom, eps, ws.data_ptr(),
                                                 ws.numel(), out.data_ptr(), st))
        _bn_after(model, ws, B, B)
        _track_batches(model, 1)
    elif model.training:
        if B <= 1:
            raise ValueError("Expected more than 1 value per channel when training")
        _bn_unsupported()
        mom, eps = _bn_config(model)
        s, keep = _params(model)
        ws = _workspace(x.device, L.pcnerf_nof_train_workspace_bytes(B))
        H.check(L.pcnerf_nof_forward_train(x.data_ptr(), B, ctypes.byref(s), mom, eps, ws.data_ptr(), ws.numel(),
                                           out.data_ptr(), st))
        _track_batches(model, 1)
    elif _EVAL_FOLD:
        fold = fold_eval(model, x.device)
        H.check(L.pcnerf_nof_forward_eval_fold(x.data_ptr(), B, fold.data_ptr(), out.data_ptr(), st))
    else:
        packed = pack_eval(model, x.device)
        H.check(L.pcnerf_nof_forward_eval(x.data_ptr(), B, packed.data_ptr(), out.data_ptr(), st))
    return (out, fold) if with_fold_state else out


def embed(x: torch.Tensor) -> torch.Tensor:
    x = _f32(x)
    if x.shape[-1] != 3:
        raise RuntimeError("Embedding(3, 10) expects (..., 3) input")
    flat = x.reshape(-1, 3)
    out = torch.empty((flat.shape[0], 63), dtype=torch.float32, device=x.device)
    H.check(H.lib().pcnerf_embed(flat.data_ptr(), flat.shape[0], out.data_ptr(), _stream(x)))
    return out.reshape(*x.shape[:-1], 63)


# ----------------------------------------------------------------------------------------------- render stages
def sample_coarse(rays, n_samples, n_parent, near_col, far_col, cn_col=0, cf_col=0, disparity=False) -> torch.Tensor:
    R = rays.shape[0]
    z = torch.empty((R, n_samples), dtype=torch.float32, device=rays.device)
    H.check(H.lib().pcnerf_sample_coarse(rays.data_ptr(), R, rays.shape[1], near_col, far_col, cn_col, cf_col,
                                         n_samples, n_parent, int(bool(disparity)), z.data_ptr(), _stream(rays)))
    return z


def perturb(z, amount: float, rand: torch.Tensor) -> torch.Tensor:
    rand = _f32(rand)
    if rand.shape != z.shape:
        raise RuntimeError(f"perturbation draws {tuple(rand.shape)} != z {tuple(z.shape)}")
    out = torch.empty_like(z)
    H.check(H.lib().pcnerf_perturb(z.data_ptr(), z.shape[0], z.shape[1], float(amount), rand.data_ptr(),
                                   out.data_ptr(), _stream(z)))
    return out


def composite(p, z, noise=None, noise_std=0.0, eps=1e-10, rays=None, cn_col=10, cf_col=11, range_col=14,
              want_weights=True, extras=False):
    """-> (weights or None, depth (R,), free_ray (R,) or None, sl1_ray (R,) or None)
    [+ (opacity mean (), depth2 (R,)) when ``extras``]."""
    R, S = z.shape
    dev = z.device
    w = torch.empty((R, S), dtype=torch.float32, device=dev) if want_weights else None
    depth = torch.empty((R,), dtype=torch.float32, device=dev)
    fr = sl = None
    if rays is not None:
        fr = torch.empty((R,), dtype=torch.float32, device=dev)
        sl = torch.empty((R,), dtype=torch.float32, device=dev)
    if noise is not None:
        noise = _f32(noise)
        if noise.shape != z.shape:
            raise RuntimeError("noise draws must have the shape of the samples")
    opac = depth2 = None
    if extras:
        opac = torch.empty((R,), dtype=torch.float64, device=dev)
        depth2 = torch.empty((R,), dtype=torch.float32, device=dev)
    H.check(H.lib().pcnerf_composite(p.data_ptr(), z.data_ptr(), R, S, H.ptr(noise), float(noise_std), float(eps),
                                     H.ptr(rays), rays.shape[1] if rays is not None else 0, cn_col, cf_col, range_col,
                                     H.ptr(w), depth.data_ptr(), H.ptr(fr), H.ptr(sl), H.ptr(opac), H.ptr(depth2),
                                     _stream(z)))
    if not extras:
        return w, depth, fr, sl
    om = torch.empty((), dtype=torch.float32, device=dev)
    H.check(H.lib().pcnerf_mean_f64(opac.data_ptr(), R, float(R * S), om.data_ptr(), _stream(z)))
    return w, depth, fr, sl, om, depth2


def resample(z, w, n_importance: int, u=None) -> torch.Tensor:
    R, S = z.shape
    if u is not None:
        u = _f32(u)
        if u.shape != (R, n_importance):
            raise RuntimeError(f"u draws {tuple(u.shape)} != ({R}, {n_importance})")
    zf = torch.empty((R, S + n_importance), dtype=torch.float32, device=z.device)
    H.check(H.lib().pcnerf_resample(z.data_ptr(), w.data_ptr(), R, S, int(n_importance), H.ptr(u), zf.data_ptr(),
                                    _stream(z)))
    return zf


def sample_pdf_standalone(bins, weights, n_samples: int, det: bool, u=None) -> torch.Tensor:
    bins, weights = _f32(bins), _f32(weights)
    R, nb = bins.shape
    if weights.shape != (R, nb - 1):
        raise RuntimeError(f"weights {tuple(weights.shape)} must be (R, n_bins - 1) = ({R}, {nb - 1})")
    if not det and u is None:
        u = torch.rand((R, n_samples), device=bins.device)
    if u is not None:
        u = _f32(u)
    out = torch.empty((R, n_samples), dtype=torch.float32, device=bins.device)
    H.check(H.lib().pcnerf_sample_pdf(bins.data_ptr(), weights.data_ptr(), R, nb, int(n_samples),
                                      H.ptr(None if det else u), out.data_ptr(), _stream(bins)))
    return out


def child_losses(free_ray, sl1_ray, rays, divide: bool, sub_nerf_test_num: int):
    """-> (child_free_loss, child_depth_loss) device tensors; shape (1,) in the divide branch (render.py:109,138
    start from torch.tensor([0])), () otherwise."""
    L = H.lib()
    R = free_ray.shape[0]
    out = torch.empty((2,), dtype=torch.float32, device=free_ray.device)
    n = int(sub_nerf_test_num) if divide else 0
    ws = _workspace(free_ray.device, L.pcnerf_child_loss_workspace_bytes(n)) if n > 0 else None
    H.check(L.pcnerf_child_loss_reduce(free_ray.data_ptr(), sl1_ray.data_ptr(), R,
                                       rays.data_ptr() + 9 * 4 if n > 0 else None, rays.shape[1], n,
                                       H.ptr(ws), out.data_ptr(), _stream(free_ray)))
    if n > 0:
        return out[0:1], out[1:2]
    return out[0], out[1]


_GAUSS = {}


def _gauss_taps(device, sigma=5.0, truncate=4.0):
    """scipy.ndimage.gaussian_filter's kernel (render.py:306, sigma 5): radius int(truncate*sigma + 0.5),
    exp(-0.5 x^2 / sigma^2) normalised by its float64 sum -- a 41-entry host-side constant table."""
    key = (device.type, device.index, sigma, truncate)
    if key not in _GAUSS:
        import numpy as np
        radius = int(truncate * float(sigma) + 0.5)
        x = np.arange(-radius, radius + 1)
        phi = np.exp(-0.5 / (sigma * sigma) * x ** 2)
        phi = phi / phi.sum()
        _GAUSS[key] = (torch.from_numpy(phi[::-1].copy()).to(device), radius)
    return _GAUSS[key]


def view_rows(p, z, rows, method: int, eps: float, want_points=True):
    """-> weights (R,S), depth (R,), at_peak (R,) uint8, child_sum (R,), opac_row (R,) float64, points (R,3)."""
    R, S = z.shape
    dev = z.device
    g, radius = _gauss_taps(dev)
    w = torch.empty((R, S), dtype=torch.float32, device=dev)
    depth = torch.empty((R,), dtype=torch.float32, device=dev)
    at_peak = torch.empty((R,), dtype=torch.uint8, device=dev)
    csum = torch.empty((R,), dtype=torch.float32, device=dev)
    opac = torch.empty((R,), dtype=torch.float64, device=dev)
    pts = torch.empty((R, 3), dtype=torch.float32, device=dev) if want_points else None
    H.check(H.lib().pcnerf_view_rows(p.data_ptr(), z.data_ptr(), R, S, rows.data_ptr(), rows.shape[1], 6, 7,
                                     int(method), float(eps), g.data_ptr(), radius, w.data_ptr(), depth.data_ptr(),
                                     at_peak.data_ptr(), csum.data_ptr(), opac.data_ptr(), H.ptr(pts), _stream(z)))
    return w, depth, at_peak, csum, opac, pts


def view_walk(other, at_peak, child_sum, opac_row, n_samples: int):
    """-> flags (R, 1) bool, opacity () float32."""
    L = H.lib()
    R = at_peak.shape[0]
    H.require_device(other)
    other = other.to(torch.int64).contiguous()
    if other.numel() != R:
        raise RuntimeError(f"other_interest_sub_nerf_number has {other.numel()} entries for {R} rows")
    flags = torch.empty((R, 1), dtype=torch.bool, device=at_peak.device)
    opacity = torch.empty((), dtype=torch.float32, device=at_peak.device)
    ws = _workspace(at_peak.device, L.pcnerf_view_walk_workspace_bytes(R))
    H.check(L.pcnerf_view_walk(other.data_ptr(), R, at_peak.data_ptr(), child_sum.data_ptr(), opac_row.data_ptr(),
                               int(n_samples), ws.data_ptr(), flags.data_ptr(), opacity.data_ptr(),
                               _stream(at_peak)))
    return flags, opacity


_KIND = {"mse": 0, "l1": 1, "smoothl1": 2}


def _loss_mask(pred, valid_mask):
    if valid_mask is None:
        return None
    H.require_device(valid_mask)
    m = valid_mask.to(torch.uint8).contiguous()
    if m.numel() != pred.numel():
        raise RuntimeError("valid_mask must match the loss inputs")
    return m


def pointwise_loss_backward(pred, target, kind: str, valid_mask, grad_out) -> torch.Tensor:
    pred, target = _f32(pred), _f32(target)
    m = _loss_mask(pred, valid_mask)
    g = torch.empty_like(pred)
    H.check(H.lib().pcnerf_pointwise_loss_backward(pred.data_ptr(), target.data_ptr(), H.ptr(m), pred.numel(),
                                                   _KIND[kind], _f32(grad_out).data_ptr(), g.data_ptr(),
                                                   _stream(pred)))
    return g


def pointwise_loss(pred, target, kind: str, valid_mask=None) -> torch.Tensor:
    pred, target = _f32(pred), _f32(target)
    if pred.shape != target.shape:
        raise RuntimeError(f"loss inputs differ in shape: {tuple(pred.shape)} vs {tuple(target.shape)}")
    m = None
    if valid_mask is not None:
        H.require_device(valid_mask)
        m = valid_mask.to(torch.uint8).contiguous()
        if m.numel() != pred.numel():
            raise RuntimeError("valid_mask must match the loss inputs")
    out = torch.empty((), dtype=torch.float32, device=pred.device)
    H.check(H.lib().pcnerf_pointwise_loss(pred.data_ptr(), target.data_ptr(), H.ptr(m), pred.numel(), _KIND[kind],
                                          out.data_ptr(), _stream(pred)))
    return out


def _child_ids(rays, n):
    H.require_device(rays)
    if rays.dtype != torch.float32 or rays.dim() != 2 or rays.shape[1] < 10 or rays.shape[0] != n \
            or rays.stride(1) != 1:
        raise RuntimeError("child range loss: rays must be a float32 (N, >=10) row-major table matching pred")
    return rays.data_ptr() + 9 * 4, rays.stride(0)


def child_range_loss(pred, target, rays, sub_nerf_test_num: int, kind: str, pre: float, post: float):
    """-> (loss (1,) device tensor, workspace holding per-child sums/counts for the backward)."""
    pred, target = _f32(pred).reshape(-1), _f32(target).reshape(-1)
    n = pred.numel()
    if target.numel() != n:
        raise RuntimeError("child range loss: pred and target differ in size")
    cid, stride = _child_ids(rays, n)
    L = H.lib()
    # its own buffer, not the shared scratch: the backward reads the per-child sums/counts from it, and any HIP op
    # running between this forward and backward() (another micro-batch, a logging render) reuses the scratch
    ws = torch.empty(max(1, int(L.pcnerf_child_range_loss_workspace_bytes(int(sub_nerf_test_num)))),
                     dtype=torch.uint8, device=pred.device)
    out = torch.empty((1,), dtype=torch.float32, device=pred.device)
    H.check(L.pcnerf_child_range_loss(pred.data_ptr(), target.data_ptr(), n, cid, stride, int(sub_nerf_test_num),
                                      _KIND[kind], float(pre), float(post), ws.data_ptr(), out.data_ptr(),
                                      _stream(pred)))
    return out, ws


def child_range_loss_backward(pred, target, rays, sub_nerf_test_num, kind, pre, post, ws, grad_out):
    pred, target = _f32(pred).reshape(-1), _f32(target).reshape(-1)
    cid, stride = _child_ids(rays, pred.numel())
    g = torch.empty_like(pred)
    H.check(H.lib().pcnerf_child_range_loss_backward(pred.data_ptr(), target.data_ptr(), pred.numel(), cid, stride,
                                                     int(sub_nerf_test_num), _KIND[kind], float(pre), float(post),
                                                     ws.data_ptr(), _f32(grad_out).data_ptr(), g.data_ptr(),
                                                     _stream(pred)))
    return g


# ----------------------------------------------------------------------------------------------- backward
def grad_params(model) -> list:
    """The 34 trainable tensors of a NOF in pcnerf_nof_grads order (lin_w, lin_b, bn_w, bn_b, out_w, out_b)."""
    lins, norms = model.linears(), model.norms()
    return ([l.weight for l in lins] + [l.bias for l in lins] + [b.weight for b in norms] + [b.bias for b in norms]
            + [model.occ_out[0].weight, model.occ_out[0].bias])


def _grads_struct(model, device):
    # one zeroed allocation for all 34 tensors (views at 256-byte aligned offsets): one fill kernel, not 34
    ps = grad_params(model)
    offs, o = [], 0
    for t in ps:
        offs.append(o)
        o += (t.numel() + 63) & ~63
    flat = torch.zeros(o, dtype=torch.float32, device=device)
    out = [flat[a:a + t.numel()].view(t.shape) for a, t in zip(offs, ps)]
    s = H.NofGrads()
    for i in range(8):
        s.lin_w[i] = out[i].data_ptr()
        s.lin_b[i] = out[8 + i].data_ptr()
        s.bn_w[i] = out[16 + i].data_ptr()
        s.bn_b[i] = out[24 + i].data_ptr()
    s.out_w = out[32].data_ptr()
    s.out_b = out[33].data_ptr()
    return s, out


def _opt_scalar(g):
    if g is None:
        return None
    g = _f32(g)
    if g.numel() != 1:
        raise RuntimeError("loss gradients must be scalars")
    return g


def composite_backward(p, z, noise, noise_std, eps, rays, sub_nerf_test_num, g_depth, g_free, g_dl,
                       cn_col=10, cf_col=11, range_col=14, cid_col=9) -> torch.Tensor:
    """dL/dlogit (R, S) of the compositing + child-loss terms (pcnerf_composite_backward)."""
    L = H.lib()
    R, S = z.shape
    out = torch.empty((R, S), dtype=torch.float32, device=z.device)
    gd = None if g_depth is None else _f32(g_depth).reshape(-1)
    if gd is not None and gd.numel() != R:
        raise RuntimeError("depth gradient must have one entry per ray")
    n = int(sub_nerf_test_num) if rays is not None else 0
    ws = _workspace(z.device, L.pcnerf_composite_backward_workspace_bytes(n)) if n > 0 else None
    H.check(L.pcnerf_composite_backward(p.data_ptr(), z.data_ptr(), R, S, H.ptr(noise), float(noise_std), float(eps),
                                        H.ptr(rays), rays.shape[1] if rays is not None else 0, cn_col, cf_col,
                                        range_col, cid_col, n, H.ptr(gd), H.ptr(_opt_scalar(g_free)),
                                        H.ptr(_opt_scalar(g_dl)), H.ptr(ws), out.data_ptr(), _stream(z)))
    return out


# Activation-store budget (bytes) of one train-mode pass; None = the default policy below.
_STORE_BUDGET = None
# The default cap when the caller set none: a bounded amount, so a drop-in caller that never asked for the store
# does not find most of the HBM held between its forward and backward (the reference holds only autograd's own
# tensors).  32 GiB keeps 14 chunks of 262,144 samples -- every chunk of the reference's shell setting (256 rays x
# 3072 samples = 3 chunks) -- and callers that want the whole step kept opt in (bench.py: free HBM - 4 GiB).
DEFAULT_STORE_CAP = 32 << 30


def set_activation_store_budget(nbytes):
    """Explicit cap for the training forward's activation store (bytes per TrainPass; 0 disables it; None restores
    the default).  Returns the previous setting.  The store lives from a pass's forward to its backward, so a
    caller that allocates a lot in between should cap it; the bench opts into ``free HBM - 4 GiB``."""
    global _STORE_BUDGET
    prev, _STORE_BUDGET = _STORE_BUDGET, (None if nbytes is None else max(0, int(nbytes)))
    return prev


def store_budget(device, reserve: int) -> int:
    """Bytes the activation store of one train-mode pass may take (ActivationStore's policy, below)."""
    import os
    if os.environ.get("PCNERF_ACT_STORE", "1") == "0":
        return 0
    free, _ = torch.cuda.mem_get_info(device)
    free += torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)
    avail = max(0, free - int(reserve))
    cap = os.environ.get("PCNERF_ACT_STORE_GB")
    if _STORE_BUDGET is not None:
        return min(avail, _STORE_BUDGET)
    if cap is not None:
        return min(avail, int(float(cap) * (1 << 30)))
    return min(avail // 2, DEFAULT_STORE_CAP)


class ActivationStore:
    """Device buffer for the first ``n_chunks`` chunks' layer outputs + BatchNorm statistics of one train-mode
    query (pcnerf_nof_store_bytes per chunk), so its backward skips their recomputation.

    Budget, in order: ``PCNERF_ACT_STORE=0`` disables it; ``set_activation_store_budget(n)`` or
    ``PCNERF_ACT_STORE_GB`` set an explicit cap; otherwise the DEFAULT is ``DEFAULT_STORE_CAP`` (32 GiB), and never
    more than half of the HBM free at the forward (driver-free + torch's cached-but-unused) after ``reserve``
    bytes -- the rest stays free for whatever the caller allocates between forward and backward (a drop-in under
    Lightning: logging, other modules).  The store never takes more than free HBM minus ``reserve``; chunks beyond
    the budget are recomputed in the backward (same gradients)."""

    def __init__(self, device, total_samples: int, chunk: int, reserve: int):
        L = H.lib()
        self.per_chunk = int(L.pcnerf_nof_store_bytes(int(chunk)))
        n_chunks = -(-int(total_samples) // int(chunk))
        self.budget = store_budget(device, reserve) if n_chunks > 0 else 0
        self.n_chunks = min(n_chunks, self.budget // self.per_chunk)
        # the fused query addresses a stored layer with a 32-bit byte offset: a chunk whose layer region reaches 4 GiB
        # (>= 4,194,304 samples) is not stored there, every chunk is recomputed instead (the layered maths' store
        # has no such limit)
        layer_bytes = (self.per_chunk - 8 * 512 * 8) // 8
        if _TRAIN_FUSED and layer_bytes >= 1 << 32:
            self.n_chunks = 0
        self.buf = None
        self.fstate = None   # the fused forward's state (query), read by the one-pass backward
        while self.n_chunks > 0:
            try:
                self.buf = torch.empty((self.n_chunks * self.per_chunk,), dtype=torch.uint8, device=device)
                break
            except torch.cuda.OutOfMemoryError:   # fragmented cache: keep fewer chunks (the rest is recomputed)
                self.n_chunks //= 2

    def release(self):
        self.buf = None
        self.fstate = None
        self.n_chunks = 0


def nof_query_backward(model, rays, z, chunk: int, g_logit, store=None) -> list:
    """Parameter gradients (grad_params order) of the train-mode query given dL/dlogit per sample; chunks held in
    ``store`` (the forward's layer outputs) are not recomputed."""
    L = H.lib()
    R, S = z.shape
    _, eps = _bn_config(model)
    s, keep = _params(model)
    gs, out = _grads_struct(model, z.device)
    ws = _workspace(z.device, L.pcnerf_nof_backward_workspace_bytes(int(chunk)))
    fstate = getattr(store, "fstate", None) if store is not None else None
    if store is not None and store.n_chunks > 0 and fstate is not None:
        # the fused forward's store: one pass per layer (pcnerf_nof_query_train_backward_fused)
        H.check(L.pcnerf_nof_query_train_backward_fused(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S,
                                                        int(chunk), ctypes.byref(s), eps, _f32(g_logit).data_ptr(),
                                                        fstate.data_ptr(), fstate.numel(), ws.data_ptr(), ws.numel(),
                                                        ctypes.byref(gs), store.buf.data_ptr(), store.n_chunks,
                                                        _stream(z)))
        # that backward wrote g_{L-1} over the stored h_{L-1}: the store is consumed, so a second backward on it
        # recomputes every chunk instead of reading gradients as activations
        store.fstate = None
        store.n_chunks = 0
    elif store is not None and store.n_chunks > 0:
        H.check(L.pcnerf_nof_query_train_backward_store(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S,
                                                        int(chunk), ctypes.byref(s), eps, _f32(g_logit).data_ptr(),
                                                        ws.data_ptr(), ws.numel(), ctypes.byref(gs),
                                                        store.buf.data_ptr(), store.n_chunks, _stream(z)))
    else:
        H.check(L.pcnerf_nof_query_train_backward(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, int(chunk),
                                                  ctypes.byref(s), eps, _f32(g_logit).data_ptr(), ws.data_ptr(),
                                                  ws.numel(), ctypes.byref(gs), _stream(z)))
    return out


def nof_query_backward_remat(model, rays, z, chunk: int, g_logit, state) -> list:
    """Parameter gradients (grad_params order) of the default train-mode query whose forward kept ``state``
    (query(..., keep=state)); the state is consumed."""
    L = H.lib()
    R, S = z.shape
    chunk = max(1, min(int(chunk), R * S))
    _, eps = _bn_config(model)
    s, keep = _params(model)
    gs, out = _grads_struct(model, z.device)
    ws = _workspace(z.device, L.pcnerf_nof_backward_workspace_bytes(int(chunk)))
    H.check(L.pcnerf_nof_query_train_backward_remat(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, int(chunk),
                                                    ctypes.byref(s), eps, _f32(g_logit).data_ptr(), state.data_ptr(),
                                                    state.numel(), ws.data_ptr(), ws.numel(), ctypes.byref(gs),
                                                    _stream(z)))
    return out


def nof_query_backward_fold(model, rays, z, chunk: int, g_logit, fold) -> list:
    """Parameter gradients of the train fold's query (state from query(..., fold=...)) given dL/dlogit."""
    L = H.lib()
    R, S = z.shape
    _, eps = _bn_config(model)
    s, keep = _params(model)
    gs, out = _grads_struct(model, z.device)
    H.check(L.pcnerf_nof_query_train_fold_backward(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, int(chunk),
                                                   ctypes.byref(s), eps, _f32(g_logit).data_ptr(), fold.data_ptr(),
                                                   fold.numel(), ctypes.byref(gs), _stream(z)))
    return out


def nof_forward_backward_fold(model, x, p, g_p, fold) -> list:
    """Parameter gradients of NOF.forward(x) through the train fold given dL/dp."""
    L = H.lib()
    B = x.shape[0]
    _, eps = _bn_config(model)
    s, keep = _params(model)
    gs, out = _grads_struct(model, x.device)
    H.check(L.pcnerf_nof_forward_train_fold_backward(x.data_ptr(), B, ctypes.byref(s), eps, _f32(p).data_ptr(),
                                                     _f32(g_p).data_ptr(), fold.data_ptr(), fold.numel(),
                                                     ctypes.byref(gs), _stream(x)))
    return out


def nof_forward_backward(model, x, p, g_p) -> list:
    """Parameter gradients of NOF.forward(x) (train mode, one batch) given dL/dp."""
    L = H.lib()
    B = x.shape[0]
    _, eps = _bn_config(model)
    s, keep = _params(model)
    gs, out = _grads_struct(model, x.device)
    ws = _workspace(x.device, L.pcnerf_nof_backward_workspace_bytes(B))
    H.check(L.pcnerf_nof_forward_train_backward(x.data_ptr(), B, ctypes.byref(s), eps, _f32(p).data_ptr(),
                                                _f32(g_p).data_ptr(), ws.data_ptr(), ws.numel(), ctypes.byref(gs),
                                                _stream(x)))
    return out
