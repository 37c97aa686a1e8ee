"""Ray tables on the GPU -- the ray/AABB intersection that feeds the render path.

``build_train_rays`` produces the 15-column training rays of one LiDAR frame (nof/dataset/ipb2dmapping.py:736-768,
819-824) and ``build_view_rows`` the 13-column two-step rows grouped per ray plus ranges,
``other_interest_sub_nerf_number`` and the true-in flags (eval_kitti_render.py:675-803, 866-868).  Inputs are
float64 device tensors in the parent block's frame; child boxes are ``bounds6`` rows [xmin, ymin, zmin, xmax, ymax,
zmax] already grown by 0.025 m (ipb2dmapping.py:606-614).  The kernels are lib/libpcnerf_hip.so's
``pcnerf_build_train_rays`` / ``pcnerf_count_view_rows`` / ``pcnerf_emit_view_rows``.
"""
from __future__ import annotations

import torch

from . import _hip as H
from ._ops import _workspace


def _f64(t):
    H.require_device(t)
    return t.to(torch.float64).contiguous()


FACE_RULES = {"0606": 0, "0406": 1}   # compute_far_bound0606 (KITTI) / compute_far_bound0406 (MaiCity)


def build_train_rays(points, origin, centers, bounds6, parent6, surface_expand=0.05, face_rule="0606") -> torch.Tensor:
    """15-column rows of one frame.  face_rule "0606" (kitti_dataload) drops rays that hit no face of their child
    box; "0406" (maicity_dataload) keeps every point in a child box and, like the reference's IndexError, raises
    when a ray hits fewer than two faces."""
    points, origin, centers, bounds6, parent6 = map(_f64, (points, origin, centers, bounds6, parent6))
    n, C = points.shape[0], bounds6.shape[0]
    L = H.lib()
    rows = torch.empty((n, 15), dtype=torch.float32, device=points.device)
    cnt = torch.empty((1,), dtype=torch.int64, device=points.device)
    short = torch.zeros((1,), dtype=torch.int32, device=points.device)
    ws = _workspace(points.device, L.pcnerf_rays_workspace_bytes(n))
    H.check(L.pcnerf_build_train_rays(points.data_ptr(), n, origin.data_ptr(), centers.data_ptr(), bounds6.data_ptr(),
                                      C, parent6.data_ptr(), float(surface_expand), FACE_RULES[face_rule],
                                      ws.data_ptr(), rows.data_ptr(), cnt.data_ptr(), short.data_ptr(),
                                      H.stream_of(points)))
    if face_rule == "0406" and int(short):
        raise IndexError(f"compute_far_bound0406: {int(short)} ray(s) hit fewer than two faces of their child box "
                         "(the reference raises IndexError here)")
    return rows[:int(cnt)]


VIEW_RULES = {"kitti": 0, "maicity": 1}


def build_view_rows(points, origin, bounds6, parent6, method=2, rule="kitti"):
    """-> (rows (M,13) float32, ranges (M,) float32, other (M,) int64, true_in (M,) bool).  rule "maicity":
    multi_frame_maicity's expansion step (0.005) and parent-far column."""
    points, origin, bounds6, parent6 = map(_f64, (points, origin, bounds6, parent6))
    n, C = points.shape[0], bounds6.shape[0]
    L = H.lib()
    dev = points.device
    cnt = torch.empty((1,), dtype=torch.int64, device=dev)
    ws = _workspace(dev, L.pcnerf_rays_workspace_bytes(n))
    st = H.stream_of(points)
    H.check(L.pcnerf_count_view_rows(points.data_ptr(), n, origin.data_ptr(), bounds6.data_ptr(), C,
                                     parent6.data_ptr(), int(method), VIEW_RULES[rule], ws.data_ptr(), cnt.data_ptr(),
                                     st))
    m = int(cnt)
    rows = torch.empty((m, 13), dtype=torch.float32, device=dev)
    ranges = torch.empty((m,), dtype=torch.float32, device=dev)
    other = torch.empty((m,), dtype=torch.int64, device=dev)
    tin = torch.empty((m,), dtype=torch.bool, device=dev)
    if m:
        H.check(L.pcnerf_emit_view_rows(points.data_ptr(), n, origin.data_ptr(), bounds6.data_ptr(), C,
                                        parent6.data_ptr(), int(method), VIEW_RULES[rule], ws.data_ptr(),
                                        rows.data_ptr(),
                                        ranges.data_ptr(), other.data_ptr(), tin.data_ptr(), st))
    return rows, ranges, other, tin
