"""Fixture: ray-group sizes of the reference's own two-step test rows (logs/kitti00/1151_1200_view/two_step/
<frame>pcd/childnerf_ray_intersect/other_interest_sub_nerf_number_child.npy: k-1 on the first row of a k-row group,
0 on the others -- eval_kitti_render.py:783-788) for frames 1153 and 1178, as uint8 group sizes in row order.  Data
only (no reference code): tests/test_dist_gloo.py partitions them over ranks.   usage: python make_group_sizes.py"""
import os

import numpy as np

REF = "/root/reference/logs/kitti00/1151_1200_view/two_step"
out = {}
for f in (1153, 1178):
    o = np.load(f"{REF}/{f}pcd/childnerf_ray_intersect/other_interest_sub_nerf_number_child.npy",
                allow_pickle=False).reshape(-1)
    sizes, i = [], 0
    while i < o.shape[0]:
        k = int(o[i]) + 1
        sizes.append(k)
        i += k
    assert i == o.shape[0]
    out[f"f{f}"] = np.asarray(sizes, dtype=np.uint8)
np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "view_group_sizes.npz"), **out)
print({k: (v.shape[0], int(v.sum()), int(v.max())) for k, v in out.items()})
