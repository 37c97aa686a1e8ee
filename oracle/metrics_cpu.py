"""CPU oracle for the evaluation metrics -- TEST INFRASTRUCTURE ONLY.

Restates nof/criteria/pointcloud_metrics.py:5-49 and logs/*/render_result/print_metrics.py:31-133 with scipy's
cKDTree in place of open3d's KDTreeFlann (open3d is absent here; both return the exact nearest neighbour of
float64 coordinates).  Pinned by the reference's committed rendered/source PCDs: the per-version averages it
reproduces are the ones SURVEY.md records (KITTI PC-NeRF two-step CD 0.2239 m = the paper's figure value).
"""
from __future__ import annotations

import numpy as np
from scipy.spatial import cKDTree


def nn_dist(verts1, verts2):
    """pointcloud_metrics.py:5-32: distance from each vertex of verts2 to its nearest vertex of verts1."""
    tree = cKDTree(np.asarray(verts1, dtype=np.float64))
    d, _ = tree.query(np.asarray(verts2, dtype=np.float64), k=1)
    return d


def eval_pts(pts1, pts2, threshold=0.2):
    """pointcloud_metrics.py:37-49."""
    d1, d2 = nn_dist(pts1, pts2), nn_dist(pts2, pts1)
    precision = np.mean((d1 < threshold).astype(float))
    recall = np.mean((d2 < threshold).astype(float))
    return float(np.mean(d1) + np.mean(d2)), float(2 * precision * recall / (precision + recall))


def frame_metrics(pred, gt, origin, threshold=0.2):
    """print_metrics.py:79-124 for one frame -> (abs_error, acc %, cd, fscore)."""
    pred = np.asarray(pred, dtype=np.float64)
    gt = np.asarray(gt, dtype=np.float64)
    n = min(len(pred), len(gt))
    pred, gt = pred[:n], gt[:n]
    o = np.asarray(origin, dtype=np.float64).reshape(1, 3)
    cd, f = eval_pts(pred, gt, threshold)
    e = np.abs(np.linalg.norm(pred - o, axis=1) - np.linalg.norm(gt - o, axis=1))
    return float(np.mean(e)), float(np.sum(e < threshold) / e.shape[0] * 100), cd, f
