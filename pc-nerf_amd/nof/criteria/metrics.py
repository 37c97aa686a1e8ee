"""Training/validation metrics -- drop-in for ``nof/criteria/metrics.py`` (metrics.py:5-35).

``abs_error`` / ``acc_thres`` are the reference's range reductions (device tensors in, device tensors out);
``eval_points`` runs the Chamfer distance / F-score on the GPU (nof.metrics.eval_pts, HIP exhaustive float64
nearest neighbours) instead of moving both clouds to the host for an open3d KD-tree.
"""
import torch

from .. import metrics as _m


def abs_error(pred, gt, valid_mask=None):
    """metrics.py:5-10: mean |pred - gt| over the selected elements."""
    value = torch.abs(pred - gt)
    if valid_mask is not None:
        value = value[valid_mask.to(value.device)]
    return torch.mean(value)


def acc_thres(pred, gt, valid_mask=None):
    """metrics.py:13-22: percentage of |pred - gt| < 0.2 m."""
    error = torch.abs(pred - gt)
    if valid_mask is not None:
        error = error[valid_mask.to(error.device)]
    acc = error < 0.2
    return torch.sum(acc) / acc.shape[0] * 100


def eval_points(pred_pts, gt_pts, valid_mask=None):
    """metrics.py:25-33 -> (cd, fscore) floats, threshold 0.2 m (pointcloud_metrics.py:37)."""
    if valid_mask is not None:
        m = valid_mask.to(pred_pts.device)
        pred_pts, gt_pts = pred_pts[m], gt_pts[m]
    return _m.eval_pts(pred_pts, gt_pts, 0.2, device=pred_pts.device)
