"""CPU oracle for the dataset stages around the ray tables -- TEST INFRASTRUCTURE ONLY.

Restates with the reference's per-point loops (numpy float64 / float32 as the reference's arrays are typed):
  * scan filter + block transform + interest region: nof/dataset/ipb2dmapping.py:650-690 and
    data_preprocess/scripts/pointcloud_fusion.py:64-103;
  * parent cloud fusion: pointcloud_fusion.py:58-117;
  * child cells: data_preprocess/scripts/split_child_nerf_xyz.py:6-49 (``huafen`` + ``split_pointcloud2``);
  * child boxes / centres: ipb2dmapping.py:598-626;
  * val sampling: ipb2dmapping.py:854-861.
open3d / python-pcl are absent, so these modules cannot be imported; this is a restatement from the source text,
"parity unpinned" by reference outputs (no ray cache or child cloud of the reference is shipped), and pinned only
through the ray-row builder (oracle/rays_cpu.py), whose primitives are checked against the reference's functions.
"""
from __future__ import annotations

import math

import numpy as np


def filter_scan(pts32, range_delete, over_height, over_low, strict_range=False):
    """ipb2dmapping.py:650-664 (dist <= 120); strict_range: eval_kitti_render.py:621-641 (dist < 120)."""
    out = []
    dx, dy, dz = range_delete
    for p in np.asarray(pts32, dtype=np.float32):
        if abs(p[0]) < dx and abs(p[1]) < dy and abs(p[2]) < dz:
            continue
        sq = p * p
        dist = np.sqrt((sq[0] + sq[1]) + sq[2])
        if dist > np.float32(120) or (strict_range and dist == np.float32(120)):
            continue
        if p[2] > over_height or p[2] < over_low:
            continue
        out.append(p)
    return np.asarray(out, dtype=np.float32).reshape(-1, 3)


def to_block(pts32, pose32):
    P = np.asarray(pose32, dtype=np.float64)
    h = np.vstack([np.asarray(pts32, dtype=np.float64).T, np.ones((1, len(pts32)))])
    return (P @ h).T[:, :3]


def interest_filter(pts, positions, ix, iy):
    keep = []
    for p in pts:
        for q in positions:
            if abs(p[0] - float(q[0])) > ix or abs(p[1] - float(q[1])) > iy:
                continue
            keep.append(p)
            break
    return np.asarray(keep, dtype=np.float64).reshape(-1, 3)


def huafen(length, t, lo, hi):
    if length > 2 * t:
        n = int(length / t) if length % t <= 0.5 * t else int(length / t) + 1
        n += 1
    else:
        n = 2
    s = np.zeros(n)
    for i in range(n):
        s[i] = lo + i * t
    s[-1] = hi + 0.05
    return s


def split_children(cloud, t_xy=1.0, t_z=1.0):
    """-> list of (min (3,), max (3,)) per non-empty cell in the script's z, y, x loop order."""
    c = np.asarray(cloud, dtype=np.float64)
    lo, hi = c.min(0), c.max(0)
    sx, sy, sz = (huafen(hi[a] - lo[a], t, lo[a], hi[a]) for a, t in ((0, t_xy), (1, t_xy), (2, t_z)))
    out = []
    for k in range(len(sz) - 1):
        mz = (c[:, 2] >= sz[k]) & (c[:, 2] < sz[k + 1])
        for j in range(len(sy) - 1):
            my = mz & (c[:, 1] >= sy[j]) & (c[:, 1] < sy[j + 1])
            for i in range(len(sx) - 1):
                m = my & (c[:, 0] >= sx[i]) & (c[:, 0] < sx[i + 1])
                if m.any():
                    out.append((c[m].min(0), c[m].max(0)))
    return out


def child_boxes(cells):
    mn = np.stack([a for a, _ in cells])
    mx = np.stack([b for _, b in cells])
    return np.concatenate([mn - 0.025, mx + 0.025], 1), (mn + mx) / 2.0


def val_index(n_rays, cloud_size_val):
    import torch
    sel = torch.linspace(1, n_rays - 2, steps=cloud_size_val, dtype=torch.float32)
    return np.array([math.floor(float(s)) for s in sel], dtype=np.int64)


def batch_slices(rows_last_col, batch_size_set):
    """eval_kitti_render.py:1120-1143, the reference's loop verbatim in structure (float column compared < -0.5)."""
    n = len(rows_last_col)
    out = []
    i = 0
    while i < n:
        if i == n - 1:
            break
        if i + batch_size_set < n - 0.5 * batch_size_set:
            other_ray_number = 0
            while rows_last_col[i + batch_size_set + other_ray_number] < -0.5:
                other_ray_number = other_ray_number + 1
                if i + batch_size_set + other_ray_number == n:
                    break
            out.append((i, i + batch_size_set + other_ray_number))
            i = i + batch_size_set + other_ray_number
        else:
            out.append((i, n))
            i = n
    return out


def filter_scan_maicity(pts32, range_delete):
    """ipb2dmapping.py:318-330 (MaiCity): ego box, norm < 120 (strict); no height filter."""
    out = []
    dx, dy, dz = range_delete
    for p in np.asarray(pts32, dtype=np.float32):
        if abs(p[0]) < dx and abs(p[1]) < dy and abs(p[2]) < dz:
            continue
        sq = p * p
        if not np.sqrt((sq[0] + sq[1]) + sq[2]) < np.float32(120):
            continue
        out.append(p)
    return np.asarray(out, dtype=np.float32).reshape(-1, 3)


def in_parent_box(pts, lo, hi):
    """ipb2dmapping.py:336-338 (MaiCity): inclusive box test."""
    keep = [p for p in pts if all(lo[a] <= p[a] <= hi[a] for a in range(3))]
    return np.asarray(keep, dtype=np.float64).reshape(-1, 3)
