"""Evaluation driver -- the reference's ``eval_kitti_render.py`` (two-step / one-step depth inference of the test
frames, rendered point clouds written as PCD) on the GPU.

Per test frame ((j+1-3-data_start) % 5 == 0, eval_kitti_render.py:1025-1033):
  1. rows: ``test_data_create=1`` builds the 13-column rows grouped per ray with the HIP ray/AABB kernels
     (nof.raytable.build_view_rows; the scan filter of eval_kitti_render.py:621-641 -- note the strict < 120 m --
     block transform, interest region, parent AABB slab exit, 0.65 m child prefilter, exactly-two-face-hit
     children) and caches them as the reference does under ``result_path/{two,one}_step/<n>pcd/
     childnerf_ray_intersect/``; ``test_data_create=0`` loads that cache (nof.io.load_view_rows);
  2. batches: the reference's rule (eval_kitti_render.py:1120-1143) -- ``batch_rows`` rows extended so no ray group
     is split, the tail half-batch merged, and its quirk kept: a single last row is never rendered;
  3. render: ``render_rays_view_0525_2_2`` (eval BN, no autograd) per batch;
  4. output: ``points_inference_fine`` of the rows flagged effective, written to ``pcd_path<n>_two_step.pcd``
     (or ``_one_step``), float32 xyz binary PCD like open3d writes.
Rendering is per row in eval mode, so the batch size only bounds memory: results are identical for any
``batch_rows`` (tests/test_eval_driver.py checks this).

Multi-GPU (torchrun, one process per GPU; the reference has no multi-GPU path): every rank holds the block's
coarse/fine weights (replicated) and renders a contiguous share of WHOLE ray groups of the rows the reference renders
(its batching rule decides which rows that is), shares cut by row count (nof.blocks.split_groups); the effective
points are gathered to rank 0 in rank order (nof.blocks.gather_rows, RCCL over xGMI), which writes the same PCD a
single process writes.  Rank 0 alone writes the row cache.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch.distributed as dist  # noqa: E402

from nof import dataset as D  # noqa: E402
from nof.blocks import gather_rows, split_groups  # noqa: E402
from nof import io as nio  # noqa: E402
from nof.networks import Embedding, NOF_coarse, NOF_fine  # noqa: E402
from nof.raytable import build_view_rows  # noqa: E402
from nof.render import render_rays_view_0525_2_2  # noqa: E402


def get_opts(argv=None):
    """eval_kitti_render.py:19-132 (the options the KITTI / MaiCity eval shells pass)."""
    p = argparse.ArgumentParser()
    a = p.add_argument
    a('--result_path', type=str, default=None)
    a('--test_data_create', type=int, default=0)
    a('--depth_inference_method', type=int, default=2)
    a('--dataset', type=str, default='maicity')
    a('--root_dir', type=str, default='~/ir-mcl/data/ipblab')
    a('--subnerf_path', type=str, default=None)
    a('--parentnerf_path', type=str, default=None)
    a('--over_height', type=float, default=0.168)
    a('--over_low', type=float, default=0.168)
    a('--interest_x', type=float, default=12)
    a('--interest_y', type=float, default=10)
    a('--view_pcd_number', type=int, default=1178)
    a('--sub_nerf_test_num', type=int, default=3)
    for k, v in (('nerf_length_min', -4.5), ('nerf_length_max', 25.5), ('nerf_width_min', -4.5),
                 ('nerf_width_max', 25.5), ('nerf_height_min', -2.0), ('nerf_height_max', 0.5)):
        a(f'--{k}', type=float, default=v)
    a('--range_delete_x', type=float, default=2)
    a('--range_delete_y', type=float, default=1)
    a('--range_delete_z', type=float, default=0.5)
    a('--data_start', type=int, default=1)
    a('--data_end', type=int, default=2)
    a('--ckpt_path', type=str, default=None)
    a('--pcd_path', type=str, default=None)
    a('--metrics_path', type=str, default=None)
    a('--chunk', type=int, default=32 * 1024)
    a('--N_samples', type=int, default=64)
    a('--N_importance', type=int, default=128)
    a('--use_disp', default=False, action="store_true")
    a('--perturb', type=float, default=0.0)
    a('--noise_std', type=float, default=0.0)
    a('--L_pos', type=int, default=10)
    a('--pose_path', type=str, default=None)
    a('--feature_size', type=int, default=256)
    a('--use_skip', default=False, action="store_true")
    # this implementation only
    a('--device', type=str, default='cuda')
    a('--batch_rows', type=int, default=0, help="rows per render call (0: the reference's 4096 KITTI / 18432 MaiCity)")
    a('--dist_backend', type=str, default='nccl', help="collective backend under torchrun (nccl = RCCL)")
    a('--frame_sparsity', type=int, default=20,
      help="held-out frame rule of eval_kitti_render.py:1054-1062 (percent; 20 is the reference's active one)")
    return p.parse_args(argv)


# the rendered (held-out) frames per frame sparsity (%), eval_kitti_render.py:1054-1062 (20 % active, the others in
# its comments): frame j + 1 is rendered when rule(j + 1 - data_start) holds
EVAL_SPARSITY_RULES = {
    20: lambda k: (k - 3) % 5 == 0,
    25: lambda k: k % 4 == 0,
    33: lambda k: k % 3 == 0,
    50: lambda k: k % 2 == 0,
    67: lambda k: (k - 1) % 3 != 0,
    75: lambda k: (k - 1) % 4 != 0,
    80: lambda k: (k - 3) % 5 != 0,
    90: lambda k: (k - 5) % 10 != 0,
}


def test_frame_ids(data_start, data_end, sparsity=20):
    """eval_kitti_render.py:1053-1062: the held-out frames at a frame sparsity (20 %: the active rule)."""
    if int(sparsity) not in EVAL_SPARSITY_RULES:
        raise ValueError(f"frame sparsity {sparsity}: one of {sorted(EVAL_SPARSITY_RULES)}")
    rule = EVAL_SPARSITY_RULES[int(sparsity)]
    return [j + 1 for j in range(data_start, data_end) if rule(j + 1 - data_start)]


def batch_slices(group_col: np.ndarray, batch_rows: int):
    """eval_kitti_render.py:1120-1143 on column 12 of the rows (-1 marks a group's continuation rows) ->
    [(start, end)].  A batch never ends inside a group; once fewer than 1.5 batches remain the rest is one batch;
    a lone last row is dropped (the reference's ``if i == N-1: break``)."""
    n = group_col.shape[0]
    out, i = [], 0
    while i < n:
        if i == n - 1:
            break
        if i + batch_rows < n - 0.5 * batch_rows:
            o = 0
            while group_col[i + batch_rows + o] < -0.5:
                o += 1
                if i + batch_rows + o == n:
                    break
            out.append((i, i + batch_rows + o))
            i += batch_rows + o
        else:
            out.append((i, n))
            i = n
    return out


class Scene:
    """Parent box, child boxes and poses of one sequence.  KITTI (multi_frame_kitti, eval_kitti_render.py:538-881):
    relative calibrated poses, parent box of the parent cloud, raw child boxes (no growth, :590-603).  MaiCity
    (multi_frame_maicity, :246-535): absolute poses (pose j for file j+1), the parent box from the command line,
    child boxes grown by 0.025 (:277-291), scans cut to the parent box."""

    def __init__(self, h, device):
        self.h, self.device = h, torch.device(device)
        self.maicity = h.dataset == "maicity"
        if self.maicity:
            self._init_maicity(h)
            return
        self.poses = D.relative_poses(D.read_poses(h.pose_path), h.data_start)
        rd = (h.range_delete_x, h.range_delete_y, h.range_delete_z)
        if h.parentnerf_path and os.path.exists(h.parentnerf_path):
            parent = torch.from_numpy(nio.read_pcd(h.parentnerf_path)).to(self.device)
        else:
            parent = D.fuse_frames(h.root_dir, self.poses, h.data_start, h.data_end, self.device, rd, h.over_height,
                                   h.over_low, h.interest_x, h.interest_y)
        p64 = parent.to(torch.float64)
        self.parent6 = torch.cat([p64.min(0).values, p64.max(0).values])
        if h.subnerf_path and os.path.isdir(h.subnerf_path):
            mn, mx = D.load_children(h.subnerf_path, h.sub_nerf_test_num, self.device)
        else:
            mn, mx = D.split_children(parent)
        self.bounds6 = torch.cat([mn, mx], 1)

    def _init_maicity(self, h):
        self.lo = (h.nerf_length_min, h.nerf_width_min, h.nerf_height_min)
        self.hi = (h.nerf_length_max, h.nerf_width_max, h.nerf_height_max)
        self.parent6 = torch.tensor([*self.lo, *self.hi], dtype=torch.float64, device=self.device)
        self.poses = torch.tensor(D.read_poses_raw(h.pose_path), dtype=torch.float32)
        if h.subnerf_path and os.path.isdir(h.subnerf_path):
            mn, mx = D.load_children(h.subnerf_path, h.sub_nerf_test_num, self.device)
        else:   # the training frames' cells, as maicity_dataload builds them
            train = [f for f in range(h.data_start + 1, h.data_end + 1) if (f - 3 - h.data_start) % 5 != 0]
            mn, mx = D.split_children(torch.cat([self.frame_points(f) for f in train]).to(torch.float32))
        self.bounds6 = torch.cat([mn - D.CHILD_GROW, mx + D.CHILD_GROW], 1)

    def frame_points(self, f):
        """eval_kitti_render.py:621-660 (KITTI: filtered, strict < 120 m, interest region) or :315-340 (MaiCity: ego
        box, < 120 m, cut to the parent box) -- scan of file f in the block frame."""
        h = self.h
        if self.maicity:
            raw = torch.from_numpy(D.load_frame(h.root_dir, f)).to(self.device)
            p = D.filter_scan_maicity(raw, (h.range_delete_x, h.range_delete_y, h.range_delete_z))
            w = D.to_block(p, self.poses[f - 1])
            return w[D.in_box(w, self.lo, self.hi)]
        raw = torch.from_numpy(D.load_frame(h.root_dir, f)).to(self.device)
        p = D.filter_scan(raw, (h.range_delete_x, h.range_delete_y, h.range_delete_z), h.over_height, h.over_low,
                          strict_range=True)
        w = D.to_block(p, self.poses[f])
        pos = self.poses[h.data_start + 1:h.data_end + 1, :3, 3]
        return w[D.interest_mask(w, pos, h.interest_x, h.interest_y)]

    def view_rows(self, f, method):
        pose = self.poses[f - 1] if self.maicity else self.poses[f]
        origin = pose[:3, 3].to(device=self.device, dtype=torch.float64)
        return build_view_rows(self.frame_points(f), origin, self.bounds6, self.parent6, method=method,
                               rule="maicity" if self.maicity else "kitti")


def cache_dir(h, f):
    step = "two_step" if h.depth_inference_method == 2 else "one_step"
    return os.path.join(h.result_path, step, f"{f}pcd", "childnerf_ray_intersect")


def group_batches(group_col, s0: int, e0: int, batch_rows: int):
    """Rows [s0, e0) (whole groups) in batches of >= batch_rows rows that never end inside a group (the reference's
    rule without its end-of-table quirks: a rank's share is not the table's end)."""
    out, i = [], s0
    while i < e0:
        e = min(i + batch_rows, e0)
        while e < e0 and group_col[e] < -0.5:
            e += 1
        out.append((i, e))
        i = e
    return out


def render_frame(models, rows, other, h, batch_rows, rank=0, world=1):
    """Steps 2-3 for one frame -> (points (M,3) float32 of the effective rows, n_rows rendered).  With world > 1
    every rank renders its share of the rows the single-process run renders and rank 0 receives every rank's
    points in rank order (others get None)."""
    mc, mf, emb = models
    col = rows[:, 12].cpu().numpy()
    pts, done = [], 0
    slices = batch_slices(col, batch_rows)
    if world > 1:
        n_render = slices[-1][1] if slices else 0
        s0, e0 = split_groups(col, world, 0, n_render)[rank]
        slices = group_batches(col, s0, e0, batch_rows)
    with torch.no_grad():
        for s, e in slices:
            r = render_rays_view_0525_2_2(mc, mf, emb, rows[s:e], other[s:e], N_samples=h.N_samples,
                                          N_importance=h.N_importance, use_disp=h.use_disp, perturb=h.perturb,
                                          noise_std=h.noise_std, chunk=h.chunk,
                                          depth_inference_method=h.depth_inference_method)
            m = r['rays_effective_flag_fine'].reshape(-1).bool()
            pts.append(r['points_inference_fine'][m])
            done += e - s
    out = (torch.cat(pts) if pts else torch.zeros((0, 3), device=rows.device)).to(torch.float32)
    if world > 1:
        n = torch.tensor([done], dtype=torch.int64, device=rows.device)
        dist.all_reduce(n)
        return gather_rows(out.contiguous(), dst=0), int(n)
    return out, done


def load_models(h, device):
    cin = 3 + 3 * h.L_pos * 2
    mc = NOF_coarse(feature_size=h.feature_size, in_channels_xy=cin, use_skip=h.use_skip)
    mf = NOF_fine(feature_size=h.feature_size, in_channels_xy=cin, use_skip=h.use_skip)
    if h.ckpt_path:
        nio.load_ckpt(mc, h.ckpt_path, model_name='nof_coarse')
        nio.load_ckpt(mf, h.ckpt_path, model_name='nof_fine')
    return mc.to(device).eval(), mf.to(device).eval(), Embedding(3, h.L_pos)


def main(argv=None):
    h = get_opts(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    own_group = False
    if world > 1 and h.device == "cuda":
        # one GPU per rank whatever the backend and whoever made the group (a gloo group left every rank
        # on cuda:0); ranks that are meant to share a GPU say so through LOCAL_RANK (the 2-rank test: both 0)
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        h.device = f"cuda:{local}"
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(h.dist_backend)
        own_group = True
    try:
        return _run(h, rank, world)
    finally:
        if own_group:
            dist.destroy_process_group()


def _run(h, rank, world):
    dev = torch.device(h.device)
    models = load_models(h, dev)
    batch_rows = h.batch_rows or (18432 if h.dataset == "maicity" else 4096)
    scene = None
    report = []
    for f in test_frame_ids(h.data_start, h.data_end, h.frame_sparsity):
        t0 = time.perf_counter()
        cdir = cache_dir(h, f)
        if h.test_data_create:
            scene = scene or Scene(h, dev)
            rows, ranges, other, tin = scene.view_rows(f, h.depth_inference_method)
            if rank == 0:
                nio.save_view_rows(cdir, rows.cpu().numpy(), other.cpu().numpy(), ranges.cpu().numpy(),
                                   tin.cpu().numpy())
        else:
            r, o, g, _ = nio.load_view_rows(cdir)
            rows, other = torch.from_numpy(r).to(dev), torch.from_numpy(o).to(dev)
        pts, n = render_frame(models, rows, other, h, batch_rows, rank, world)
        if rank != 0:
            continue
        if h.pcd_path:
            os.makedirs(os.path.dirname(os.path.abspath(h.pcd_path + "x")), exist_ok=True)
            suffix = "_two_step.pcd" if h.depth_inference_method == 2 else "_one_step.pcd"
            nio.write_pcd(h.pcd_path + str(f) + suffix, pts.cpu().numpy())
        torch.cuda.synchronize(dev)
        report.append({"frame": f, "rows": n, "points": int(pts.shape[0]), "seconds": time.perf_counter() - t0})
    if rank == 0:
        print(json.dumps(report))
    return report


if __name__ == "__main__":
    main()
