"""Scene datasets -- drop-in for ``nof/dataset`` (``nof_dataset`` registry: ``kitti_dataload``,
``maicity_dataload``), built on the GPU.

The reference builds its training rays in ``nof/dataset/ipb2dmapping.py`` with open3d / python-pcl and per-point
Python loops (minutes per frame).  Here every stage is a device tensor op or a HIP kernel:

  poses           ``read_poses`` / ``relative_poses``   ipb2dmapping.py:560-584 (P @ T_velo2cam, then T_start^-1 @ P
                                                         in float32, like the reference's torch tensors)
  frame split     ``frame_ids``                           ipb2dmapping.py:632-644 (sparsity rules of the comments)
  scan filter     ``filter_scan``                         ipb2dmapping.py:650-664
  to block frame  ``to_block``                            ipb2dmapping.py:666-669
  interest region ``interest_mask``                       ipb2dmapping.py:672-690
  parent cloud    ``fuse_frames``                         data_preprocess/scripts/pointcloud_fusion.py:58-117
  child boxes     ``split_children`` + ``child_boxes``    split_child_nerf_xyz.py:6-49, ipb2dmapping.py:598-626
  ray rows        ``nof.raytable.build_train_rays``       ipb2dmapping.py:736-824 (HIP kernel, float64)
  val sampling    ``kitti_dataload.__getitem__``          ipb2dmapping.py:850-866

Child point clouds (``split_child_nerf2/*.pcd``) are not shipped with the reference (.MISSING_LARGE_BLOBS), nor is
the ROS ground-filter / clustering step that produces ``child_nerf/*.pcd``; when ``subnerf_path`` does not hold
them, the children are the non-empty 1 m cells of the fused parent cloud, split exactly as
``split_child_nerf_xyz.split_pointcloud2`` splits one child.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import io as nio

# KITTI Velodyne -> camera calibration used by the reference (ipb2dmapping.py:561-564)
T_VELO2CAM = np.array([[4.276802385584e-04, -9.999672484946e-01, -8.084491683471e-03, -1.198459927713e-02],
                       [-7.210626507497e-03, 8.081198471645e-03, -9.999413164504e-01, -5.403984729748e-02],
                       [9.999738645903e-01, 4.859485810390e-04, -7.206933692422e-03, -2.921968648686e-01],
                       [0.0, 0.0, 0.0, 1.0]])

CHILD_GROW = 0.025   # ipb2dmapping.py:607, :616 (extend_tmp / extend_tmp2)

# train-frame rules of ipb2dmapping.py:632-640 keyed by frame sparsity (%): keep frame j (0-based loop index,
# file j+1) for training when rule(j, data_start) holds
SPARSITY_RULES = {
    20: lambda j, s: (j + 1 - 3 - s) % 5 != 0,
    25: lambda j, s: (j + 1 - s) % 4 != 0,
    33: lambda j, s: (j + 1 - s) % 3 != 0,
    50: lambda j, s: (j + 1 - s) % 2 != 0,
    67: lambda j, s: (j + 1 - 1 - s) % 3 == 0,
    75: lambda j, s: (j + 1 - 1 - s) % 4 == 0,
    80: lambda j, s: (j + 1 - 3 - s) % 5 == 0,
    90: lambda j, s: (j + 1 - 5 - s) % 10 == 0,
}


def read_poses(pose_path: str) -> np.ndarray:
    """KITTI poses.txt -> (N, 4, 4) float64, each row's 3x4 matrix completed and right-multiplied by T_velo2cam."""
    out = []
    with open(pose_path, "r", encoding="utf-8") as fh:
        for line in fh:
            s = line.strip()
            if not s:
                continue
            P = np.vstack([np.array([float(v) for v in s.split(" ")]).reshape(3, 4), [[0.0, 0.0, 0.0, 1.0]]])
            out.append(P @ T_VELO2CAM)
    return np.asarray(out)


def relative_poses(poses: np.ndarray, data_start: int) -> torch.Tensor:
    """Poses relative to frame data_start+1 as the reference holds them: float32 ``T_start^-1 @ P`` (torch CPU
    batched matmul of the float32-rounded inverse and poses, ipb2dmapping.py:577-584)."""
    T_start_inv = torch.from_numpy(np.linalg.inv(poses[data_start + 1])).float()
    return T_start_inv @ torch.tensor(poses, dtype=torch.float32)


def frame_ids(data_start: int, data_end: int, split: str, sparsity: int = 20) -> list[int]:
    """File numbers (j+1) of the frames a split reads (ipb2dmapping.py:632-644).  val: (j+1-3) % 5 == 0."""
    if split == "train":
        rule = SPARSITY_RULES[int(sparsity)]
        return [j + 1 for j in range(data_start, data_end) if rule(j, data_start)]
    if split == "val":
        return [j + 1 for j in range(data_start, data_end) if (j + 1 - 3) % 5 == 0]
    raise ValueError(f"split must be 'train' or 'val', got {split!r}")


def filter_scan(pts: torch.Tensor, range_delete=(3.0, 2.0, 1.25), over_height=0.168, over_low=-2.0,
                max_range=120.0, strict_range=False) -> torch.Tensor:
    """ipb2dmapping.py:650-664: drop the ego box (|x|<dx and |y|<dy and |z|<dz), points beyond 120 m (norm in
    float32, like np.linalg.norm of the float32 scan) and points outside [over_low, over_height] in z.
    ``strict_range``: the test-frame variant keeps only norms < 120 (eval_kitti_render.py:637)."""
    p = pts.to(torch.float32)
    dx, dy, dz = (float(v) for v in range_delete)
    keep = (p[:, 0].abs() >= dx) | (p[:, 1].abs() >= dy) | (p[:, 2].abs() >= dz)
    sq = p * p
    nrm = torch.sqrt((sq[:, 0] + sq[:, 1]) + sq[:, 2])
    keep &= (nrm < max_range) if strict_range else (nrm <= max_range)
    keep &= (p[:, 2] <= over_height) & (p[:, 2] >= over_low)
    return p[keep]


def to_block(pts: torch.Tensor, pose: torch.Tensor) -> torch.Tensor:
    """ipb2dmapping.py:666-669: the float32 pose (promoted to float64) applied to homogeneous float64 points
    (the reference's ``tensor @ ndarray`` runs in numpy float64; summation order may differ by 1 ulp of float64)."""
    P = pose.to(device=pts.device, dtype=torch.float64)
    h = pts.to(torch.float64)
    return h @ P[:3, :3].T + P[:3, 3]


def interest_mask(pts: torch.Tensor, positions: torch.Tensor, interest_x: float, interest_y: float) -> torch.Tensor:
    """ipb2dmapping.py:672-690: keep a point when some pose of the sequence lies within interest_x / interest_y of
    it in x and y (float64 differences)."""
    pos = positions.to(device=pts.device, dtype=torch.float64)
    keep = torch.zeros(pts.shape[0], dtype=torch.bool, device=pts.device)
    for s in range(0, pts.shape[0], 1 << 18):
        q = pts[s:s + (1 << 18), None, :2]
        near = ((q[..., 0] - pos[None, :, 0]).abs() <= interest_x) & ((q[..., 1] - pos[None, :, 1]).abs() <= interest_y)
        keep[s:s + q.shape[0]] = near.any(1)
    return keep


def load_frame(root_dir: str, file_no: int) -> np.ndarray:
    return nio.read_pcd(os.path.join(root_dir, f"{file_no}.pcd"))


def fuse_frames(root_dir: str, poses: torch.Tensor, data_start: int, data_end: int, device, range_delete=(3, 2, 1.25),
                over_height=0.168, over_low=-2.0, interest_x=20.0, interest_y=20.0) -> torch.Tensor:
    """pointcloud_fusion.py:58-117: the parent cloud ``source.pcd`` -- every train frame ((j+1-3) % 5 != 0),
    filtered, moved to the block frame, restricted to the interest region; rounded to float32 as the PCD stores it."""
    positions = poses[data_start + 1:data_end + 1, :3, 3]
    parts = []
    for j in range(data_start, data_end):
        if (j + 1 - 3) % 5 == 0:
            continue
        p = filter_scan(torch.from_numpy(load_frame(root_dir, j + 1)).to(device), range_delete, over_height, over_low)
        w = to_block(p, poses[j + 1])
        parts.append(w[interest_mask(w, positions, interest_x, interest_y)])
    return torch.cat(parts).to(torch.float32)


def _splits(length: float, t: float, lo: float, hi: float) -> np.ndarray:
    """split_child_nerf_xyz.py:6-20 (``huafen``): cell boundaries lo + i*t, the last moved to hi + 0.05."""
    if length > 2 * t:
        n = int(length / t) if length % t <= 0.5 * t else int(length / t) + 1
        n += 1
    else:
        n = 2
    s = np.array([lo + i * t for i in range(n)], dtype=np.float64)
    s[-1] = hi + 0.05
    return s


def _cell(x: torch.Tensor, splits: np.ndarray) -> torch.Tensor:
    """Index i with splits[i] <= x < splits[i+1] (exact: the comparisons run against the same float64 bounds)."""
    s = torch.as_tensor(splits, dtype=torch.float64, device=x.device)
    return (torch.searchsorted(s, x.contiguous(), right=True) - 1).clamp_(0, len(splits) - 2)


def split_children(cloud: torch.Tensor, xy_threshold=1.0, z_threshold=1.0):
    """split_child_nerf_xyz.py:22-49 on one cloud: the non-empty cells of the grid in (z, y, x) loop order ->
    (min (C,3), max (C,3)) float64 bounds of each cell's points (the AABB open3d reports for the written cell)."""
    c = cloud.to(torch.float64)
    lo, hi = c.min(0).values.cpu().numpy(), c.max(0).values.cpu().numpy()
    sx = _splits(hi[0] - lo[0], xy_threshold, lo[0], hi[0])
    sy = _splits(hi[1] - lo[1], xy_threshold, lo[1], hi[1])
    sz = _splits(hi[2] - lo[2], z_threshold, lo[2], hi[2])
    ix, iy, iz = _cell(c[:, 0], sx), _cell(c[:, 1], sy), _cell(c[:, 2], sz)
    key = (iz * (len(sy) - 1) + iy) * (len(sx) - 1) + ix
    uniq, inv = torch.unique(key, sorted=True, return_inverse=True)
    C = uniq.shape[0]
    mn = torch.full((C, 3), math.inf, dtype=torch.float64, device=c.device)
    mx = torch.full((C, 3), -math.inf, dtype=torch.float64, device=c.device)
    idx = inv[:, None].expand(-1, 3)
    mn.scatter_reduce_(0, idx, c, reduce="amin")
    mx.scatter_reduce_(0, idx, c, reduce="amax")
    return mn, mx


def child_boxes(mn: torch.Tensor, mx: torch.Tensor):
    """ipb2dmapping.py:598-626: (bounds6 (C,6) grown by 0.025, centres (C,3) of the raw boxes)."""
    bounds6 = torch.cat([mn - CHILD_GROW, mx + CHILD_GROW], 1)
    centers = (mn + mx) / 2.0
    return bounds6, centers


def load_children(subnerf_path, n_children, device):
    """Child boxes from ``subnerf_path/<i>.pcd`` (i = 1..n) when they exist (the reference's input)."""
    mn, mx = [], []
    for i in range(n_children):
        p = torch.from_numpy(nio.read_pcd(os.path.join(subnerf_path, f"{i + 1}.pcd"))).to(torch.float64)
        mn.append(p.min(0).values)
        mx.append(p.max(0).values)
    return torch.stack(mn).to(device), torch.stack(mx).to(device)


class kitti_dataload(torch.utils.data.Dataset):
    """ipb2dmapping.py:512-866 with the reference's constructor keywords.  ``rays`` (N, 15) and ``ranges`` (N,)
    are float32 tensors on ``device``; ``__getitem__`` returns ``{'rays', 'ranges'}`` like the reference (val:
    ``cloud_size_val`` rows picked at floor(linspace(1, N-2, cloud_size_val)), ipb2dmapping.py:854-861).

    Extra keywords: ``device`` (where rays are built and kept), ``sparsity`` (train-frame rule, default the active
    20 % line), ``parent_bounds`` ((lo, hi) overriding the parent cloud's AABB), ``children`` ((min, max) child
    boxes overriding ``subnerf_path``).  With ``re_loaddata=0`` the cached ``self_rays_<split>.npy`` under
    ``result_path/save_npy/split_child_nerf2_3`` are loaded; with 1 they are rebuilt and saved there."""

    def __init__(self, root_dir, split='train', data_start=1439, data_end=1510, cloud_size_val=2048,
                 range_delete_x=2, range_delete_y=1, range_delete_z=0.5, sub_nerf_test_num=3, surface_expand=0.1,
                 over_height=0.168, over_low=-2, interest_x=12, interest_y=12, pose_path=None, subnerf_path=None,
                 parentnerf_path=None, re_loaddata=0, result_path=None, *, device="cuda", sparsity=20,
                 parent_bounds=None, children=None):
        super().__init__()
        self.split, self.cloud_size_val = split, cloud_size_val
        self.device = torch.device(device)
        cache = os.path.join(result_path, "save_npy", "split_child_nerf2_3") if result_path else None
        if not re_loaddata:
            if cache is None:
                raise ValueError("re_loaddata=0 needs result_path holding save_npy/split_child_nerf2_3")
            rays, ranges = nio.load_rays(cache, split)
            self.rays = torch.from_numpy(rays).to(self.device)
            self.ranges = torch.from_numpy(ranges.reshape(-1)).to(self.device)
            return
        rd = (range_delete_x, range_delete_y, range_delete_z)
        poses = relative_poses(read_poses(pose_path), data_start)
        self.poses = poses
        positions = poses[data_start + 1:data_end + 1, :3, 3]
        if parent_bounds is None:
            if parentnerf_path and os.path.exists(parentnerf_path):
                parent = torch.from_numpy(nio.read_pcd(parentnerf_path)).to(self.device)
            else:
                parent = fuse_frames(root_dir, poses, data_start, data_end, self.device, rd, over_height, over_low,
                                     interest_x, interest_y)
            self.parent_cloud = parent
            p64 = parent.to(torch.float64)
            parent_bounds = (p64.min(0).values, p64.max(0).values)
        parent6 = torch.cat([torch.as_tensor(b, dtype=torch.float64).reshape(3) for b in parent_bounds]).to(self.device)
        if children is None:
            if subnerf_path and os.path.isdir(subnerf_path):
                children = load_children(subnerf_path, sub_nerf_test_num, self.device)
            else:
                children = split_children(self.parent_cloud)
        self.bounds6, self.centers = child_boxes(*(torch.as_tensor(c, dtype=torch.float64).to(self.device)
                                                   for c in children))
        self.sub_nerf_test_num = self.bounds6.shape[0]
        from .raytable import build_train_rays
        rays = []
        for f in frame_ids(data_start, data_end, split, sparsity):
            p = filter_scan(torch.from_numpy(load_frame(root_dir, f)).to(self.device), rd, over_height, over_low)
            w = to_block(p, poses[f])
            w = w[interest_mask(w, positions, interest_x, interest_y)]
            origin = poses[f][:3, 3].to(device=self.device, dtype=torch.float64)
            rays.append(build_train_rays(w, origin, self.centers, self.bounds6, parent6, surface_expand))
        self.rays = torch.cat(rays) if rays else torch.zeros((0, 15), device=self.device)
        self.ranges = self.rays[:, 14].clone()
        if cache is not None:
            nio.save_rays(cache, self.rays.cpu().numpy(), self.ranges.cpu().numpy(), split)

    def val_index(self) -> torch.Tensor:
        """floor(linspace(1, N-2, cloud_size_val)) in float32 (ipb2dmapping.py:856-859)."""
        sel = torch.linspace(1, self.rays.shape[0] - 2, steps=self.cloud_size_val, dtype=torch.float32)
        return torch.floor(sel).to(torch.int64).to(self.rays.device)

    def __len__(self):
        return self.rays.shape[0] if self.split == 'train' else self.cloud_size_val

    def __getitem__(self, index):
        if self.split == 'train':
            return {'rays': self.rays[index], 'ranges': self.ranges[index]}
        i = self.val_index()[index]
        return {'rays': self.rays[i], 'ranges': self.ranges[i]}


def read_poses_raw(pose_path: str) -> np.ndarray:
    """MaiCity poses.txt -> (N, 4, 4) float64 absolute poses, no calibration (ipb2dmapping.py:236-246)."""
    out = []
    with open(pose_path, "r", encoding="utf-8") as fh:
        for line in fh:
            s = line.strip()
            if s:
                out.append(np.vstack([np.array([float(v) for v in s.split(" ")]).reshape(3, 4), [[0.0, 0.0, 0.0, 1.0]]]))
    return np.asarray(out)


def filter_scan_maicity(pts: torch.Tensor, range_delete=(2.0, 1.0, 0.5), max_range=120.0) -> torch.Tensor:
    """ipb2dmapping.py:318-330: the ego box and norms >= 120 m (strict) go; no height filter."""
    p = pts.to(torch.float32)
    dx, dy, dz = (float(v) for v in range_delete)
    keep = (p[:, 0].abs() >= dx) | (p[:, 1].abs() >= dy) | (p[:, 2].abs() >= dz)
    sq = p * p
    keep &= torch.sqrt((sq[:, 0] + sq[:, 1]) + sq[:, 2]) < max_range
    return p[keep]


def in_box(pts: torch.Tensor, lo, hi) -> torch.Tensor:
    """ipb2dmapping.py:336-338: inclusive parent-box test in float64."""
    lo = torch.as_tensor(lo, dtype=torch.float64, device=pts.device)
    hi = torch.as_tensor(hi, dtype=torch.float64, device=pts.device)
    return ((pts >= lo) & (pts <= hi)).all(1)


class maicity_dataload(torch.utils.data.Dataset):
    """ipb2dmapping.py:200-507 with the reference's constructor keywords: absolute poses (pose j for file j+1, no
    calibration), the parent block given by nerf_{length,width,height}_{min,max}, scans cut to that block, child
    near/far by compute_far_bound0406 (face_rule "0406": every point in a child box yields a row; a ray with fewer
    than two face hits raises IndexError, as in the reference).  val frames: (j+1-3-data_start) % 5 == 0.
    Extra keywords as kitti_dataload (``device``, ``sparsity``, ``children``)."""

    def __init__(self, root_dir, split='train', data_start=0, data_end=36, cloud_size_val=2048, range_delete_x=2,
                 range_delete_y=1, range_delete_z=0.5, sub_nerf_test_num=3, surface_expand=0.1, nerf_length_min=-4.5,
                 nerf_length_max=25.5, nerf_width_min=-12, nerf_width_max=12, nerf_height_min=-2, nerf_height_max=0.5,
                 pose_path=None, subnerf_path=None, re_loaddata=0, result_path=None, *, device="cuda", sparsity=20,
                 children=None):
        super().__init__()
        self.split, self.cloud_size_val = split, cloud_size_val
        self.device = torch.device(device)
        cache = os.path.join(result_path, "save_npy", "split_child_nerf2_3") if result_path else None
        if not re_loaddata:
            if cache is None:
                raise ValueError("re_loaddata=0 needs result_path holding save_npy/split_child_nerf2_3")
            rays, ranges = nio.load_rays(cache, split)
            self.rays = torch.from_numpy(rays).to(self.device)
            self.ranges = torch.from_numpy(ranges.reshape(-1)).to(self.device)
            return
        rd = (range_delete_x, range_delete_y, range_delete_z)
        lo = (nerf_length_min, nerf_width_min, nerf_height_min)
        hi = (nerf_length_max, nerf_width_max, nerf_height_max)
        parent6 = torch.tensor([*lo, *hi], dtype=torch.float64, device=self.device)
        P64 = read_poses_raw(pose_path)
        self.poses = torch.tensor(P64, dtype=torch.float32)      # torch.Tensor(poses), ipb2dmapping.py:247
        positions = P64[:, :3, 3]                                 # float64 (numpy), ipb2dmapping.py:245

        def frame(j):
            p = filter_scan_maicity(torch.from_numpy(load_frame(root_dir, j + 1)).to(self.device), rd)
            w = to_block(p, self.poses[j])
            return w[in_box(w, lo, hi)]

        if split == "train":
            rule = SPARSITY_RULES[int(sparsity)]
            frames = [j for j in range(data_start, data_end) if rule(j, data_start)]
        elif split == "val":
            frames = [j for j in range(data_start, data_end) if (j + 1 - 3 - data_start) % 5 == 0]
        else:
            raise ValueError(f"split must be 'train' or 'val', got {split!r}")
        if children is None:
            if subnerf_path and os.path.isdir(subnerf_path):
                children = load_children(subnerf_path, sub_nerf_test_num, self.device)
            else:   # the block's training frames, split like split_child_nerf_xyz.py (child clouds not shipped)
                rule = SPARSITY_RULES[int(sparsity)]
                cloud = torch.cat([frame(j) for j in range(data_start, data_end) if rule(j, data_start)])
                self.parent_cloud = cloud.to(torch.float32)
                children = split_children(self.parent_cloud)
        self.bounds6, self.centers = child_boxes(*(torch.as_tensor(c, dtype=torch.float64).to(self.device)
                                                   for c in children))
        self.sub_nerf_test_num = self.bounds6.shape[0]
        from .raytable import build_train_rays
        rays = []
        for j in frames:
            origin = torch.tensor(positions[j], dtype=torch.float64, device=self.device)
            rays.append(build_train_rays(frame(j), origin, self.centers, self.bounds6, parent6, surface_expand,
                                         face_rule="0406"))
        self.rays = torch.cat(rays) if rays else torch.zeros((0, 15), device=self.device)
        self.ranges = self.rays[:, 14].clone()
        if cache is not None:
            nio.save_rays(cache, self.rays.cpu().numpy(), self.ranges.cpu().numpy(), split)

    val_index = kitti_dataload.val_index
    __len__ = kitti_dataload.__len__
    __getitem__ = kitti_dataload.__getitem__


nof_dataset = {'kitti_dataload': kitti_dataload, 'maicity_dataload': maicity_dataload}
