"""Synthetic LiDAR ray tables and deterministic NOF parameters.

The reference builds its ray tables from KITTI/MaiCity point clouds plus child-AABB point clouds that are not
shipped (``.MISSING_LARGE_BLOBS``), so benchmarks and parity tests run on synthetic tables with the exact column
layout the reference's dataset writes:

* train/val layout, 15 columns (``nof/dataset/ipb2dmapping.py:819-824``, decoded at ``nof/render.py:420-427``)::

      o(0:3) d(3:6) parent_near(6)=0 parent_far(7) ray_class(8)=3 child_id(9, 1-based)
      child_near(10) child_far(11) point_near(12)=range-0.05 point_far(13)=child_far range(14)

* two-step eval layout, 13 columns (``eval_kitti_render.py:703-714,783-788``, decoded at ``nof/render.py:619-623``)::

      o(0:3) d(3:6) child_near(6) child_far(7) class(8) parent_near(9)=0 parent_far(10) hit_rank(11) group_other(12)

  plus the separate ``other_interest_sub_nerf_number`` vector (k-1 on the first row of a k-row group, 0 else).

The generator follows SURVEY.md section 8(d) config 2: one parent block ``[-4.5,25.5]x[-4.5,25.5]x[-2,0.5]``
(``logs/kitti00/1151_1200_view/version_1/hparams.yaml``), LiDAR origin at 0, child AABBs of side U[0.5,1.5] m,
child near/far = slab intersection of the box grown by 0.025 m (``ipb2dmapping.py:616-622``) and then widened by
``surface_expand`` = 0.05 m (``ipb2dmapping.py:757-758``), parent far = slab exit, ``max(parent_far, child_far)``
(``ipb2dmapping.py:763-766``).  All geometry is computed in float64 and stored as float32, like the reference.
"""
from __future__ import annotations

import numpy as np

PARENT_LO = np.array([-4.5, -4.5, -2.0])
PARENT_HI = np.array([25.5, 25.5, 0.5])
AABB_GROW = 0.025        # ipb2dmapping.py:616-622
SURFACE_EXPAND = 0.05    # shells/pretraining/KITTI00_pcnerf_train.bash --surface_expand


def _slab(o, d, lo, hi):
    """Ray/box slab test in float64. Returns (t_enter, t_exit) per ray (rows of o, d)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t1 = (lo - o) * inv
        t2 = (hi - o) * inv
    tmin = np.where(np.isnan(t1), -np.inf, np.minimum(t1, t2))
    tmax = np.where(np.isnan(t2), np.inf, np.maximum(t1, t2))
    return tmin.max(axis=-1), tmax.min(axis=-1)


def make_children(n_children=32, seed=0, lo=PARENT_LO, hi=PARENT_HI, min_center_dist=3.0, origin=(0.0, 0.0, 0.0)):
    """Child AABBs (n,2,3) fully inside the parent block, centres at least ``min_center_dist`` from the origin."""
    rng = np.random.default_rng(seed)
    lo, hi, origin = np.asarray(lo, np.float64), np.asarray(hi, np.float64), np.asarray(origin, np.float64)
    boxes = []
    while len(boxes) < n_children:
        half = rng.uniform(0.5, 1.5, size=3) / 2
        c = rng.uniform(lo + half, hi - half)
        if np.linalg.norm(c - origin) < min_center_dist:
            continue
        boxes.append(np.stack([c - half, c + half]))
    return np.asarray(boxes)


# MaiCity-00's parent box (shells/pretraining/MaiCity00_pcnerf_train.bash) split in x into parent blocks (config 4)
MAICITY_LO = np.array([-12.0, -12.0, -2.0])
MAICITY_HI = np.array([61.0, 12.0, 0.5])


def block_bounds(b, n_blocks, lo=MAICITY_LO, hi=MAICITY_HI):
    """Parent block b of ``n_blocks`` equal x-slices of [lo, hi], and a LiDAR origin at its centre (z = 0)."""
    xs = np.linspace(lo[0], hi[0], n_blocks + 1)
    blo, bhi = np.array([xs[b], lo[1], lo[2]]), np.array([xs[b + 1], hi[1], hi[2]])
    return blo, bhi, np.array([0.5 * (xs[b] + xs[b + 1]), 0.5 * (lo[1] + hi[1]), 0.0])


def make_rays(n_rays, n_children=32, seed=0, layout="train", lo=PARENT_LO, hi=PARENT_HI, origin=(0.0, 0.0, 0.0)):
    """Config-2 synthetic rays (default parent block and origin), or those of another parent block ``[lo, hi]``
    seen from ``origin`` (config 4's blocks).

    Returns ``rays`` float32 ``(n_rays, 15)`` for ``layout='train'``.  Every ray starts at the origin and ends at
    a uniformly drawn point of a uniformly drawn child box (its LiDAR return)."""
    assert layout == "train"
    origin = np.asarray(origin, np.float64)
    boxes = make_children(n_children, seed, lo, hi, origin=origin)
    rng = np.random.default_rng(seed + 1)
    cid = rng.integers(0, n_children, size=n_rays)
    blo, bhi = boxes[cid, 0], boxes[cid, 1]
    t = rng.uniform(blo, bhi) - origin
    rng_ = np.linalg.norm(t, axis=1)
    d = t / rng_[:, None]
    o = np.broadcast_to(origin, d.shape).copy()
    cn, cf = _slab(o, d, blo - AABB_GROW, bhi + AABB_GROW)
    cn = np.maximum(cn, 0.0) - SURFACE_EXPAND
    cf = cf + SURFACE_EXPAND
    _, pf = _slab(o, d, np.asarray(lo, np.float64), np.asarray(hi, np.float64))
    pf = np.maximum(pf, cf)
    rays = np.zeros((n_rays, 15), dtype=np.float64)
    rays[:, 0:3] = o
    rays[:, 3:6] = d
    rays[:, 6] = 0.0
    rays[:, 7] = pf
    rays[:, 8] = 3.0
    rays[:, 9] = cid + 1
    rays[:, 10] = cn
    rays[:, 11] = cf
    rays[:, 12] = rng_ - SURFACE_EXPAND
    rays[:, 13] = cf
    rays[:, 14] = rng_
    return rays.astype(np.float32)


# group-size histogram of logs/kitti00/1151_1200_view/two_step/*/other_interest_sub_nerf_number_child.npy
# (SURVEY.md 8(d) config 5): 1:14.5 %, 2:33.3 %, 3:24.0 %, 4:11.2 %, 5:5.9 %, >=6: 11.0 % (spread over 6..10)
GROUP_P = np.array([0.145, 0.333, 0.240, 0.112, 0.059, 0.033, 0.026, 0.021, 0.016, 0.015])


def make_view_rows(n_rays, n_children=32, seed=0, max_rows=None):
    """Two-step eval rows (13-col layout) with ray groups: every ray gets k child hits sorted by near bound.

    Returns (rows float32 (N,13), other int64 (N,), ranges float32 (N,)).  Each group's rows share o/d/parent
    bounds; row j of a group carries the j-th hit child's near/far (eval_kitti_render.py:783-788,866-868)."""
    boxes = make_children(n_children, seed)
    rng = np.random.default_rng(seed + 2)
    ks = rng.choice(np.arange(1, len(GROUP_P) + 1), size=n_rays, p=GROUP_P / GROUP_P.sum())
    rows, other, ranges = [], [], []
    for r in range(n_rays):
        k = int(ks[r])
        ci = int(rng.integers(0, n_children))
        t = rng.uniform(boxes[ci, 0], boxes[ci, 1])
        rg = float(np.linalg.norm(t))
        d = t / rg
        _, pf = _slab(np.zeros((1, 3)), d[None], PARENT_LO, PARENT_HI)
        # the true child plus k-1 other intervals along the same ray (synthetic "other hits")
        hits = [(*_slab(np.zeros((1, 3)), d[None], boxes[ci, 0] - AABB_GROW, boxes[ci, 1] + AABB_GROW),)]
        hits = [(float(max(hits[0][0][0], 0.0)), float(hits[0][1][0]))]
        for _ in range(k - 1):
            a = float(rng.uniform(0.5, pf[0] - 1.0))
            hits.append((a, a + float(rng.uniform(0.3, 1.5))))
        hits.sort()
        for j, (hn, hf) in enumerate(hits):
            row = np.zeros(13)
            row[3:6] = d
            row[6], row[7] = hn, hf
            row[8] = 3.0
            row[9], row[10] = 0.0, max(float(pf[0]), hf)
            row[11] = j + 1
            row[12] = (k - 1) if j == 0 else -1
            rows.append(row)
            other.append((k - 1) if j == 0 else 0)
            ranges.append(rg)
        if max_rows is not None and len(rows) >= max_rows:
            break
    return (np.asarray(rows, dtype=np.float32), np.asarray(other, dtype=np.int64),
            np.asarray(ranges, dtype=np.float32))


def nof_param_names(feature_size=256):
    """state_dict keys of the reference NOF family (nof/networks/models.py:44-123): layer1 Linear at 0,3,6,9 and
    BatchNorm at 1,4,7,10; layer2 Linear at 0,2,4,6 and BatchNorm at 1,3,5,7; occ_out.0 Linear."""
    lin = [f"layer1.{i}" for i in (0, 3, 6, 9)] + [f"layer2.{i}" for i in (0, 2, 4, 6)]
    bn = [f"layer1.{i}" for i in (1, 4, 7, 10)] + [f"layer2.{i}" for i in (1, 3, 5, 7)]
    return lin, bn


def init_nof_params(seed, feature_size=256, in_channels=63, occ_bias=-4.0):
    """Deterministic NOF parameters as float32 numpy arrays keyed like the reference state_dict.

    Linear weights/biases ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (torch's default init range); BatchNorm
    gamma ~ U(0.6,1.4), beta ~ U(-0.3,0.3), running_mean ~ U(-0.3,0.3), running_var ~ U(0.2,0.6).
    Checkpoints are absent from the reference (.MISSING_LARGE_BLOBS), so every parity test and the bench use
    these (numpy PCG64 streams are reproducible across machines).  ``occ_bias`` (the occ_out bias) defaults to
    -4 so occupancy is low in free space and the transmittance survives to the child interval, as it does for a
    trained field; with a zero bias a random net saturates every ray within its first few samples."""
    rng = np.random.default_rng(seed)
    lin, bn = nof_param_names(feature_size)
    fan_in = [in_channels, feature_size, feature_size, feature_size,
              in_channels + feature_size, feature_size, feature_size, feature_size]
    p = {}
    for name, fi in zip(lin, fan_in):
        k = 1.0 / np.sqrt(fi)
        p[name + ".weight"] = rng.uniform(-k, k, size=(feature_size, fi)).astype(np.float32)
        p[name + ".bias"] = rng.uniform(-k, k, size=(feature_size,)).astype(np.float32)
    for name in bn:
        p[name + ".weight"] = rng.uniform(0.6, 1.4, size=feature_size).astype(np.float32)
        p[name + ".bias"] = rng.uniform(-0.3, 0.3, size=feature_size).astype(np.float32)
        p[name + ".running_mean"] = rng.uniform(-0.3, 0.3, size=feature_size).astype(np.float32)
        p[name + ".running_var"] = rng.uniform(0.2, 0.6, size=feature_size).astype(np.float32)
        p[name + ".num_batches_tracked"] = np.array(0, dtype=np.int64)
    k = 1.0 / np.sqrt(feature_size)
    p["occ_out.0.weight"] = rng.uniform(-k, k, size=(1, feature_size)).astype(np.float32)
    p["occ_out.0.bias"] = (rng.uniform(-k, k, size=(1,)) + occ_bias).astype(np.float32)
    return p


def load_into(module, params):
    """Load numpy params into an nn.Module with the reference state_dict keys (ours or the reference's)."""
    import torch
    sd = {k: torch.from_numpy(np.array(v)) for k, v in params.items()}
    module.load_state_dict(sd, strict=True)
    return module
