"""CPU oracle for the ray-table construction (ray/AABB intersection) -- TEST INFRASTRUCTURE ONLY.

Restates, in float64 numpy with the reference's loop order, SURVEY.md 8(a) rows a3-a5:
  * train/val 15-column rays (nof/dataset/ipb2dmapping.py:736-768 per-point loop, find_aabb_box :174-197,
    compute_far_bound0606 :119-172, compute_far_bound :36-77);
  * two-step 13-column rows grouped per ray (eval_kitti_render.py:675-803 per-point loop,
    compute_far_bound0429 :170-211, ray_aabb_distances :213-235, distance_to_ray :237-244).
The geometric primitives are pinned against the reference's own functions (tests/golden/aabb_primitives.npz, made
by executing their source in tests/golden/make_golden.py); the per-point assembly loops live in modules that import
open3d/pcl (absent here) and are restated from the source text.
"""
from __future__ import annotations

import numpy as np
from sklearn.neighbors import KDTree


def face_hits(p, d, lo, hi):
    """The face loop shared by compute_far_bound0406/0606/0429: for each axis, the lower face then the upper face
    ahead of the ray; a hit counts when the hit point lies inside the other two slabs (inclusive)."""
    out = []
    for i in range(3):
        for b in (lo[i], hi[i]):
            if d[i] * (b - p[i]) > 0:
                dist = (b - p[i]) / d[i]
                pe = p + dist * d
                cnt = sum(1 for k in range(3) if k != i and lo[k] <= pe[k] <= hi[k])
                if cnt >= 2:
                    out.append(dist)
    return out


def far_bound_0606(p, d, lo, hi):
    """ipb2dmapping.py:119-172: (intersect, near = min hit, far = max hit); no hit -> (False, 0, 0)."""
    h = face_hits(p, d, lo, hi)
    if not h:
        return False, 0.0, 0.0
    return True, min(h), max(h)


def far_bound_0406(p, d, lo, hi):
    """ipb2dmapping.py:82-114 (MaiCity): the FIRST two face hits in face order, swapped if needed; fewer than
    two hits make the reference raise IndexError -> (False, 0, 0) here."""
    h = face_hits(p, d, lo, hi)
    if len(h) < 2:
        return False, 0.0, 0.0
    a, b = h[0], h[1]
    return True, min(a, b), max(a, b)


def far_bound_0429(p, d, lo, hi):
    """eval_kitti_render.py:170-211: exactly two face hits or no intersection."""
    h = face_hits(p, d, lo, hi)
    if len(h) != 2:
        return False, 0.0, 0.0
    return True, min(h), max(h)


def far_bound_parent(o, d, lo, hi):
    """ipb2dmapping.py:36-77: min over the 6 planes of the non-negative plane distance (d = 0 or t < 0 -> inf);
    all infinite -> None (stored as nan by the caller)."""
    ts = []
    for a in range(3):
        for b in (hi[a], lo[a]):
            if d[a] != 0:
                t = (b - o[a]) / d[a]
                ts.append(np.inf if t < 0 else t)
            else:
                ts.append(np.inf)
    t = min(ts)
    return None if t == np.inf else t


def find_child(tree, bounds6, q, k=10):
    """ipb2dmapping.py:174-197: the first of the k nearest child centres (KD-tree order) whose box holds q."""
    _, idx = tree.query(q.reshape(1, -1), k=k)
    for i in idx.squeeze().tolist():
        b = bounds6[i]
        if b[0] <= q[0] <= b[3] and b[1] <= q[1] <= b[4] and b[2] <= q[2] <= b[5]:
            return i
    return None


def slab_far(o, dirs, lo, hi):
    """eval_kitti_render.py:213-235 (vectorised over rays): slab exit distance, inf if the slabs miss."""
    with np.errstate(divide="ignore", invalid="ignore"):
        t1 = (lo[0] - o[0]) / dirs[:, 0]
        t2 = (hi[0] - o[0]) / dirs[:, 0]
        t3 = (lo[1] - o[1]) / dirs[:, 1]
        t4 = (hi[1] - o[1]) / dirs[:, 1]
        t5 = (lo[2] - o[2]) / dirs[:, 2]
        t6 = (hi[2] - o[2]) / dirs[:, 2]
        tmin = np.max(np.vstack((np.minimum(t1, t2), np.minimum(t3, t4), np.minimum(t5, t6))), axis=0)
        tmax = np.min(np.vstack((np.maximum(t1, t2), np.maximum(t3, t4), np.maximum(t5, t6))), axis=0)
        return np.where(tmax >= tmin, tmax, np.inf)


def distance_to_ray(o, d, pts):
    """eval_kitti_render.py:237-244."""
    v = pts - o
    dist = np.sqrt(np.sum(v ** 2, axis=1))
    with np.errstate(invalid="ignore"):
        cos = np.sum(v * d, axis=1) / dist
        return dist * np.sqrt(1 - cos ** 2)


def rays_of(points, origin):
    vec = points - origin
    rng = np.linalg.norm(vec, axis=1)
    dirs = vec / rng[:, None]
    return dirs, rng


def build_train_rays(points, origin, centers, bounds6, parent_lo, parent_hi, surface_expand=0.05, rule="0606"):
    """ipb2dmapping.py:736-768 + 819-824 for one frame: float32 (N', 15) rows of the points that fall in a
    child box (KD-tree lookup) whose box the ray enters.  rule "0406" (MaiCity, :383-395): every point in a child
    box yields a row, near/far from the first two face hits (a ray with fewer raises, as the reference does)."""
    tree = KDTree(centers)
    dirs, rng = rays_of(points, origin)
    rows = []
    for i in range(points.shape[0]):
        k = find_child(tree, bounds6, points[i])
        if k is None:
            continue
        d = dirs[i]
        if rule == "0406":
            hit, near, far = far_bound_0406(origin, d, bounds6[k][:3], bounds6[k][3:6])
            if not hit:
                raise IndexError("compute_far_bound0406: fewer than two face hits")
        else:
            hit, near, far = far_bound_0606(origin, d, bounds6[k][:3], bounds6[k][3:6])
            if not hit:
                continue
        near, far = near - surface_expand, far + surface_expand
        pf = far_bound_parent(origin, d, parent_lo, parent_hi)
        pf = np.nan if pf is None else pf
        if pf < far:
            pf = far
        rows.append([*origin, *d, 0.0, pf, 3.0, k + 1, near, far, rng[i] - surface_expand, far, rng[i]])
    return np.asarray(rows, dtype=np.float64).reshape(-1, 15).astype(np.float32)


def build_view_rows(points, origin, bounds6, parent_lo, parent_hi, method=2, radius=0.65, rule="kitti"):
    """eval_kitti_render.py:675-803 for one frame -> (rows (M, 13) float32, ranges (M,) float32,
    other (M,) int64, true_in (M,) bool).  rule "maicity" (multi_frame_maicity, :344-431): expansion step 0.005
    instead of 0.05 and column 10 the parent far bound itself (KITTI: max(parent far, child far))."""
    step = 0.005 if rule == "maicity" else 0.05
    dirs, rng = rays_of(points, origin)
    pfar_all = slab_far(origin, dirs, parent_lo, parent_hi)
    center = (bounds6[:, :3] + bounds6[:, 3:]) / 2
    rows, ranges, other, tin = [], [], [], []
    for i in range(points.shape[0]):
        d = dirs[i]
        pnear, pfar = 0.0, pfar_all[i]
        filt = bounds6[distance_to_ray(origin, d, center) <= radius].copy()
        hits = []  # [near, far, col7_parent_far, true_in]

        def scan():
            for k in range(filt.shape[0]):
                ok, a, b = far_bound_0429(origin, d, filt[k][:3], filt[k][3:6])
                if ok:
                    q = points[i]
                    inside = bool(filt[k][0] <= q[0] <= filt[k][3] and filt[k][1] <= q[1] <= filt[k][4]
                                  and filt[k][2] <= q[2] <= filt[k][5])
                    adj = pfar if rule == "maicity" else (b if pfar < b else pfar)
                    if method == 1:
                        hits.append([pnear, pfar, adj, inside])
                        return True
                    hits.append([a, b, adj, inside])
            return bool(hits)

        found = scan()
        ext, drop = 0.0, False
        while not found:
            if ext > 0.5:
                drop = True
                break
            ext = ext + step
            filt[:, :3] = filt[:, :3] - ext
            filt[:, 3:6] = filt[:, 3:6] + ext
            found = scan()
        if drop or not hits:
            continue
        h = np.asarray(hits, dtype=np.float64)
        order = np.argsort(h[:, 0], kind="stable")
        n = len(order)
        for j, t in enumerate(order):
            rows.append([*origin, *d, h[t, 0], h[t, 1], 3.0, pnear, h[t, 2], j + 1, (n - 1) if j == 0 else -1])
            ranges.append(rng[i])
            other.append((n - 1) if j == 0 else 0)
            tin.append(bool(h[t, 3]))
    return (np.asarray(rows, dtype=np.float64).reshape(-1, 13).astype(np.float32),
            np.asarray(ranges, dtype=np.float32), np.asarray(other, dtype=np.int64), np.asarray(tin, dtype=bool))
