"""Ray-table oracle (oracle/rays_cpu.py) vs the reference's own ray/AABB primitives (aabb_primitives.npz)."""
import numpy as np
from sklearn.neighbors import KDTree

from conftest import golden
from oracle import rays_cpu as RC


def test_primitives_match_reference():
    g = golden("aabb_primitives")
    o, pts, lo, hi = g["origin"], g["points"], g["lo"], g["hi"]
    dirs, _ = RC.rays_of(pts, o)
    bounds6 = np.concatenate([lo, hi], 1)
    tree = KDTree(g["centers"])
    for i in range(len(pts)):
        k = RC.find_child(tree, bounds6, pts[i])
        assert (k is not None) == bool(g["find_inside"][i]) and (k or -1) == (g["find_idx"][i] if k is not None else -1)
        pf = RC.far_bound_parent(o, dirs[i], *(np.asarray(x) for x in _parent()))
        np.testing.assert_array_equal(np.nan if pf is None else pf, g["parent_far"][i])
        row, row2 = [], []
        for b in (g["cid"][i], g["other_box"][i]):
            h, a, z = RC.far_bound_0606(o, dirs[i], lo[b], hi[b])
            row += [float(h), a, z]
            row2.append(list(map(float, RC.far_bound_0429(o, dirs[i], lo[b], hi[b]))))
        np.testing.assert_array_equal(np.array(row), g["f0606"][i])
        np.testing.assert_array_equal(np.array(list(map(float, RC.far_bound_0406(o, dirs[i], lo[g["cid"][i]],
                                                                                  hi[g["cid"][i]])))), g["f0406"][i])
        np.testing.assert_array_equal(np.array(row2), g["f0429"][2 * i:2 * i + 2])
    np.testing.assert_array_equal(RC.slab_far(o, dirs, *(np.asarray(x) for x in _parent())), g["slab"])
    d2r = np.stack([RC.distance_to_ray(o, dirs[i], g["centers"]) for i in range(0, len(pts), 37)])
    np.testing.assert_array_equal(d2r, g["d2r"])


def _parent():
    from nof import synthetic as syn
    return syn.PARENT_LO, syn.PARENT_HI


def test_row_builders_shapes_and_groups():
    g = golden("aabb_primitives")
    bounds6 = np.concatenate([g["lo"], g["hi"]], 1)
    rows = RC.build_train_rays(g["points"], g["origin"], g["centers"], bounds6, *_parent())
    assert rows.shape[1] == 15 and 0 < len(rows) <= len(g["points"])
    assert np.all(rows[:, 10] <= rows[:, 11]) and np.all(rows[:, 7] >= rows[:, 11])
    v, rng, other, tin = RC.build_view_rows(g["points"], g["origin"], bounds6, *_parent())
    assert v.shape[1] == 13 and len(v) == len(rng) == len(other) == len(tin)
    # every group: first row carries k-1, others -1 (col 12) / 0 (other); hit ranks 1..k; nears sorted
    i = 0
    while i < len(v):
        k = int(other[i]) + 1
        assert v[i, 12] == k - 1 and np.all(v[i + 1:i + k, 12] == -1) and np.all(other[i + 1:i + k] == 0)
        assert list(v[i:i + k, 11]) == list(range(1, k + 1))
        assert np.all(np.diff(v[i:i + k, 6]) >= 0)
        i += k
