"""Evaluation metrics on the GPU -- drop-in for ``nof/criteria/pointcloud_metrics.py`` (``eval_pts``,
``nn_correspondance``) and the per-frame arithmetic of ``logs/*/render_result/print_metrics.py:31-133``
(``abs_error``, ``acc_thres``, ``error_metrics``).

The nearest-neighbour search is the HIP kernel ``pcnerf_nn_distance`` (exhaustive, float64) instead of an open3d
KD-tree queried point by point from Python; the reductions are HIP kernels too.  Inputs are (N, 3) clouds on the
device (numpy arrays are moved to ``device``).
"""
from __future__ import annotations

import torch

from . import _hip as H
from . import _ops


def _cloud(x, device):
    t = torch.as_tensor(x)
    if t.device.type != "cuda":
        t = t.to(device)
    t = t.to(torch.float32).reshape(-1, 3).contiguous()
    H.require_device(t)
    return t


def nn_correspondance(verts1, verts2, device="cuda"):
    """pointcloud_metrics.py:5-32: for each vertex of verts2 the distance to its nearest vertex in verts1
    (float64 tensor; indices are not produced -- no caller uses them)."""
    a, b = _cloud(verts1, device), _cloud(verts2, device)
    d = torch.empty((b.shape[0],), dtype=torch.float64, device=b.device)
    if a.shape[0] == 0 or b.shape[0] == 0:
        return d[:0]
    H.check(H.lib().pcnerf_nn_distance(a.data_ptr(), a.shape[0], b.data_ptr(), b.shape[0], d.data_ptr(),
                                       _ops._stream(b)))
    return d


def eval_pts(pts1, pts2, threshold=0.2, device="cuda"):
    """pointcloud_metrics.py:37-49 / print_metrics.py:31-41 -> (cd, fscore) as Python floats.
    pts1: rendered cloud, pts2: reference cloud."""
    p, g = _cloud(pts1, device), _cloud(pts2, device)
    L = H.lib()
    ws = torch.empty((L.pcnerf_eval_pts_workspace_bytes(p.shape[0], g.shape[0]),), dtype=torch.uint8,
                     device=p.device)
    out = torch.empty((4,), dtype=torch.float64, device=p.device)
    H.check(L.pcnerf_eval_pts(p.data_ptr(), p.shape[0], g.data_ptr(), g.shape[0], float(threshold), ws.data_ptr(),
                              out.data_ptr(), _ops._stream(p)))
    o = out.cpu().tolist()
    return o[0], o[1]


def range_metrics(pred_pts, gt_pts, origin, threshold=0.2, device="cuda"):
    """print_metrics.py:44-52, 121-124 on aligned clouds -> (abs_error m, acc % within threshold)."""
    p, g = _cloud(pred_pts, device), _cloud(gt_pts, device)
    if p.shape != g.shape:
        raise RuntimeError("range_metrics needs aligned clouds of equal size")
    o = _cloud(origin, device)
    out = torch.empty((2,), dtype=torch.float64, device=p.device)
    H.check(H.lib().pcnerf_range_metrics(p.data_ptr(), g.data_ptr(), o.data_ptr(), p.shape[0], float(threshold),
                                         out.data_ptr(), _ops._stream(p)))
    s, c = out.cpu().tolist()
    n = p.shape[0]
    return s / n, c / n * 100


def frame_metrics(pred_pts, gt_pts, origin, threshold=0.2, device="cuda"):
    """One frame of print_metrics.error_metrics (:54-133): the clouds are truncated to the shorter one, then
    (abs_error, acc, cd, fscore)."""
    p, g = _cloud(pred_pts, device), _cloud(gt_pts, device)
    n = min(p.shape[0], g.shape[0])
    p, g = p[:n].contiguous(), g[:n].contiguous()
    cd, f = eval_pts(p, g, threshold, device)
    err, acc = range_metrics(p, g, origin, threshold, device)
    return err, acc, cd, f
