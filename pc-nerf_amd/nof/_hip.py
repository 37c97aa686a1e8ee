"""ctypes binding of lib/libpcnerf_hip.so (C ABI declared in include/pcnerf_hip.h).

The library is the only compute backend of this package: there is no CPU or eager-PyTorch fallback.  If it is
missing, or a tensor is not on a ROCm device, the call raises.  PyTorch provides device memory, the current
HIP stream and RNG draws; every arithmetic step of the render path runs in the library's kernels.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PCNERF_HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libpcnerf_hip.so"))

_lib = None
_lock = threading.Lock()
vp = ctypes.c_void_p
i64 = ctypes.c_int64
c_int = ctypes.c_int
c_float = ctypes.c_float
c_size = ctypes.c_size_t


class NofParams(ctypes.Structure):
    _fields_ = [("lin_w", vp * 8), ("lin_b", vp * 8), ("bn_w", vp * 8), ("bn_b", vp * 8), ("bn_rm", vp * 8),
                ("bn_rv", vp * 8), ("out_w", vp), ("out_b", vp)]


class NofGrads(ctypes.Structure):
    _fields_ = [("lin_w", vp * 8), ("lin_b", vp * 8), ("bn_w", vp * 8), ("bn_b", vp * 8), ("out_w", vp),
                ("out_b", vp)]


# name -> (restype, argtypes)
_SIGS = {
    "pcnerf_abi_version": (c_int, []),
    "pcnerf_last_error": (ctypes.c_char_p, []),
    "pcnerf_nof_eval_packed_floats": (c_size, []),
    "pcnerf_nof_pack_eval": (c_int, [ctypes.POINTER(NofParams), vp, vp]),
    "pcnerf_nof_query_eval": (c_int, [vp, i64, c_int, vp, c_int, vp, vp, vp]),
    "pcnerf_nof_train_workspace_bytes": (c_size, [i64]),
    "pcnerf_set_train_math": (c_int, [c_int]),
    "pcnerf_set_remat_version": (c_int, [c_int]),
    "pcnerf_set_composite_group": (c_int, [c_int]),
    "pcnerf_set_eval_math": (c_int, [c_int]),
    "pcnerf_nof_query_train": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams), c_float, c_float,
                                       vp, c_size, vp, vp]),
    "pcnerf_sample_coarse": (c_int, [vp, i64, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, vp, vp]),
    "pcnerf_perturb": (c_int, [vp, i64, c_int, c_float, vp, vp, vp]),
    "pcnerf_composite": (c_int, [vp, vp, i64, c_int, vp, c_float, c_float, vp, c_int, c_int, c_int, c_int, vp, vp,
                                 vp, vp, vp, vp, vp]),
    "pcnerf_set_depth2_order": (c_int, [c_int]),
    "pcnerf_mean_f64": (c_int, [vp, i64, ctypes.c_double, vp, vp]),
    "pcnerf_resample": (c_int, [vp, vp, i64, c_int, c_int, vp, vp, vp]),
    "pcnerf_sample_pdf": (c_int, [vp, vp, i64, c_int, c_int, vp, vp, vp]),
    "pcnerf_child_loss_workspace_bytes": (c_size, [c_int]),
    "pcnerf_child_loss_reduce": (c_int, [vp, vp, i64, vp, c_int, c_int, vp, vp, vp]),
    "pcnerf_pointwise_loss": (c_int, [vp, vp, vp, i64, c_int, vp, vp]),
    "pcnerf_pointwise_loss_backward": (c_int, [vp, vp, vp, i64, c_int, vp, vp, vp]),
    "pcnerf_child_range_loss_workspace_bytes": (c_size, [c_int]),
    "pcnerf_child_range_loss": (c_int, [vp, vp, i64, vp, c_int, c_int, c_int, c_float, c_float, vp, vp, vp]),
    "pcnerf_child_range_loss_backward": (c_int, [vp, vp, i64, vp, c_int, c_int, c_int, c_float, c_float, vp, vp, vp,
                                                 vp]),
    "pcnerf_embed": (c_int, [vp, i64, vp, vp]),
    "pcnerf_view_rows": (c_int, [vp, vp, i64, c_int, vp, c_int, c_int, c_int, c_int, c_float, vp, c_int, vp, vp, vp,
                                 vp, vp, vp, vp]),
    "pcnerf_view_walk_workspace_bytes": (c_size, [i64]),
    "pcnerf_view_walk": (c_int, [vp, i64, vp, vp, vp, c_int, vp, vp, vp, vp]),
    "pcnerf_rays_workspace_bytes": (c_size, [i64]),
    "pcnerf_build_train_rays": (c_int, [vp, i64, vp, vp, vp, i64, vp, ctypes.c_double, c_int, vp, vp, vp, vp, vp]),
    "pcnerf_count_view_rows": (c_int, [vp, i64, vp, vp, i64, vp, c_int, c_int, vp, vp, vp]),
    "pcnerf_emit_view_rows": (c_int, [vp, i64, vp, vp, i64, vp, c_int, c_int, vp, vp, vp, vp, vp, vp]),
    "pcnerf_prof_enable": (c_int, [c_int]),
    "pcnerf_prof_read": (c_int, [c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64),
                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "pcnerf_mfma_ceiling": (c_int, [ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_double), vp]),
    "pcnerf_nof_forward_eval": (c_int, [vp, i64, vp, vp, vp]),
    "pcnerf_nof_fold_eval": (c_int, [ctypes.POINTER(NofParams), vp, vp]),
    "pcnerf_nof_query_eval_fold": (c_int, [vp, i64, c_int, vp, c_int, vp, vp, vp]),
    "pcnerf_nof_forward_eval_fold": (c_int, [vp, i64, vp, vp, vp]),
    "pcnerf_nof_forward_train": (c_int, [vp, i64, ctypes.POINTER(NofParams), c_float, c_float, vp, c_size, vp, vp]),
    "pcnerf_nof_backward_workspace_bytes": (c_size, [i64]),
    "pcnerf_nof_query_train_backward": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams), c_float,
                                                vp, vp, c_size, ctypes.POINTER(NofGrads), vp]),
    "pcnerf_nof_forward_train_backward": (c_int, [vp, i64, ctypes.POINTER(NofParams), c_float, vp, vp, vp, c_size,
                                                  ctypes.POINTER(NofGrads), vp]),
    "pcnerf_nof_store_bytes": (c_size, [i64]),
    "pcnerf_nof_query_train_store": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams), c_float,
                                             c_float, vp, c_size, vp, vp, i64, vp]),
    "pcnerf_nof_query_train_fused_store": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams),
                                                   c_float, c_float, vp, c_size, vp, vp, i64, vp]),
    "pcnerf_nof_query_train_backward_store": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams),
                                                      c_float, vp, vp, c_size, ctypes.POINTER(NofGrads), vp, i64,
                                                      vp]),
    "pcnerf_nof_query_train_backward_fused": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams),
                                                      c_float, vp, vp, c_size, vp, c_size, ctypes.POINTER(NofGrads),
                                                      vp, i64, vp]),
    "pcnerf_nof_query_train_fused_state": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams),
                                                   c_float, c_float, vp, c_size, vp, vp]),
    "pcnerf_nof_query_train_backward_remat": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams),
                                                      c_float, vp, vp, c_size, vp, c_size, ctypes.POINTER(NofGrads),
                                                      vp]),
    "pcnerf_nof_train_bn_stats": (c_int, [vp, c_size, i64, i64, vp, vp]),
    "pcnerf_bn_running_replay": (c_int, [ctypes.POINTER(NofParams), c_float, vp, vp, i64, vp]),
    "pcnerf_nof_train_fold_bytes": (c_size, [i64, i64]),
    "pcnerf_nof_train_fused_bytes": (c_size, [i64, i64]),
    "pcnerf_nof_query_train_fold": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams), c_float,
                                            c_float, vp, c_size, vp, vp]),
    "pcnerf_nof_forward_train_fold": (c_int, [vp, i64, ctypes.POINTER(NofParams), c_float, c_float, vp, c_size, vp,
                                              vp]),
    "pcnerf_nof_query_train_fold_backward": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams),
                                                     c_float, vp, vp, c_size, ctypes.POINTER(NofGrads), vp]),
    "pcnerf_nof_forward_train_fold_backward": (c_int, [vp, i64, ctypes.POINTER(NofParams), c_float, vp, vp, vp,
                                                       c_size, ctypes.POINTER(NofGrads), vp]),
    "pcnerf_nof_query_train_fused": (c_int, [vp, i64, c_int, vp, c_int, i64, ctypes.POINTER(NofParams), c_float,
                                             c_float, vp, c_size, vp, vp]),
    "pcnerf_nof_forward_train_fused": (c_int, [vp, i64, ctypes.POINTER(NofParams), c_float, c_float, vp, c_size,
                                               vp, vp]),
    "pcnerf_nn_distance": (c_int, [vp, i64, vp, i64, vp, vp]),
    "pcnerf_eval_pts_workspace_bytes": (c_size, [i64, i64]),
    "pcnerf_eval_pts": (c_int, [vp, i64, vp, i64, ctypes.c_double, vp, vp, vp]),
    "pcnerf_range_metrics": (c_int, [vp, vp, vp, i64, ctypes.c_double, vp, vp]),
    "pcnerf_composite_backward_workspace_bytes": (c_size, [c_int]),
    "pcnerf_composite_backward": (c_int, [vp, vp, i64, c_int, vp, c_float, c_float, vp, c_int, c_int, c_int, c_int,
                                          c_int, c_int, vp, vp, vp, vp, vp, vp]),
}


def lib():
    """Load the library once; raise loudly if it is absent (no fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"PC-NeRF HIP library not found at {LIB_PATH}; build it with "
                                   f"`make -C pc-nerf_amd` (or __graft_entry__.build()). There is no CPU fallback.")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                if not hasattr(L, name):
                    raise RuntimeError(f"{LIB_PATH} does not export {name}; rebuild it")
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError("pcnerf_hip: " + lib().pcnerf_last_error().decode())


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def require_device(*ts: torch.Tensor) -> None:
    for t in ts:
        if t is None:
            continue
        if not (t.is_cuda and t.dtype in (torch.float32, torch.float64, torch.uint8, torch.bool, torch.int64)):
            raise RuntimeError("pcnerf_hip kernels take ROCm device tensors (got %s on %s); this package has no "
                               "CPU path" % (t.dtype, t.device))


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
