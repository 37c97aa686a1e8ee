"""Ray tables of the reference's own scenes for the config-1 / config-4 parity fixtures (no reference import here).

    python tests/golden/make_scene_rays.py      -> tests/golden/scene_rays.npz

BASELINE.json config 1 renders KITTI-00 rays (frames 1151-1200, 4,096-ray batch, 64/128 samples) and config 4
MaiCity-00 rays split over 4 parent blocks.  The child AABB clouds are absent from the reference
(.MISSING_LARGE_BLOBS), so -- as nof.dataset does -- the scenes are the committed fixture frames
(tests/golden/kitti_frames.npz: KITTI-00 scans 1151..1156, every 40th point; maicity_frames.npz: MaiCity-00 scans
1..6) fused into a parent cloud and split into 1 m child cells.  The rows come from the CPU restatement of the
reference's dataset code (oracle/dataset_cpu.py + oracle/rays_cpu.py; the host stages shared with nof.dataset are
checked equal to it in tests/test_dataset.py), so the GPU tests can rebuild them with nof.dataset and check them
bit for bit before rendering.

Stored (small subsets, the rest is rebuilt on the GPU):
  kitti_train  (4096, 15)  a seeded batch of the train split (DataLoader(shuffle=True) analogue), with its indices;
  kitti_train_all          the whole train split (config 3 draws its 262,144-ray batch from it with replacement);
  kitti_val    (N, 15)     the whole val split;
  maicity_b{0..3}          up to 1024 rows of each of 4 parent blocks (MaiCity bounds [-12,61] split in x), with
                           the block bounds and each block's child count;
  kitti_view_*             the two-step test rows (13 columns), ranges and ray-group column of the first KITTI
                           fixture test frame (config 5's eval_kitti_render.py path).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "pc-nerf_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

from nof import dataset as D  # noqa: E402
from oracle import dataset_cpu as OD  # noqa: E402
from oracle import rays_cpu as RC  # noqa: E402

# the kitti_dataload / maicity_dataload settings the fixture tests use (tests/test_dataset.py)
DS, DE = 1150, 1155
KW = dict(range_delete=(3.0, 2.0, 1.25), over_height=0.168, over_low=-2.0)
INTEREST = 20.0
M_LO, M_HI = (-12.0, -12.0, -2.0), (61.0, 12.0, 0.5)
M_RD = (2.0, 1.0, 0.5)
N_BLOCKS = 4


def kitti_rays(tmp):
    from test_dataset import oracle_poses, write_scene
    root, pose_path, g = write_scene(tmp)
    rel = D.relative_poses(D.read_poses(pose_path), DS)
    cloud = D.fuse_frames(root, rel, DS, DE, "cpu", KW["range_delete"], KW["over_height"], KW["over_low"],
                          INTEREST, INTEREST).numpy()
    b6, cen = OD.child_boxes(OD.split_children(cloud))
    plo, phi = cloud.astype(np.float64).min(0), cloud.astype(np.float64).max(0)
    P = oracle_poses(g, pose_path)
    positions = np.stack([P[k + 1][:3, 3] for k in range(DS, DE)])
    out = {}
    for split in ("train", "val"):
        rows = []
        for f in D.frame_ids(DS, DE, split):
            p = OD.filter_scan(g[f"f{f}"], KW["range_delete"], KW["over_height"], KW["over_low"])
            w = OD.interest_filter(D.to_block(torch.from_numpy(p), torch.from_numpy(P[f])).numpy(), positions,
                                   INTEREST, INTEREST)
            rows.append(RC.build_train_rays(w, P[f][:3, 3].astype(np.float64), cen, b6, plo, phi, 0.05))
        out[split] = np.concatenate(rows)
    return out, len(cen)


def kitti_view(tmp):
    """The two-step test rows of the first KITTI fixture test frame (eval_kitti_render.py:675-803 via
    oracle/rays_cpu.build_view_rows, method 2), as tests/test_eval_driver.py builds its oracle rows: strict < 120 m
    scan filter, interest region, raw 1 m child cells of the fused cloud, parent box = the cloud's bounds."""
    from test_dataset import oracle_poses, write_scene
    root, pose_path, g = write_scene(tmp)
    rel = D.relative_poses(D.read_poses(pose_path), DS)
    cloud = D.fuse_frames(root, rel, DS, DE, "cpu", KW["range_delete"], KW["over_height"], KW["over_low"],
                          INTEREST, INTEREST).numpy()
    cells = OD.split_children(cloud)
    b6 = np.concatenate([np.stack([a for a, _ in cells]), np.stack([b for _, b in cells])], 1)
    c64 = cloud.astype(np.float64)
    plo, phi = c64.min(0), c64.max(0)
    P = oracle_poses(g, pose_path)
    positions = np.stack([P[k + 1][:3, 3] for k in range(DS, DE)])
    f = [j + 1 for j in range(DS, DE) if (j + 1 - 3) % 5 == 0][0]
    p = OD.filter_scan(g[f"f{f}"], KW["range_delete"], KW["over_height"], KW["over_low"], strict_range=True)
    w = OD.interest_filter(D.to_block(torch.from_numpy(p), torch.from_numpy(P[f])).numpy(), positions, INTEREST,
                           INTEREST)
    rows, rng, other, tin = RC.build_view_rows(w, P[f][:3, 3].astype(np.float64), b6, plo, phi, 2)
    return dict(kitti_view_rows=rows, kitti_view_ranges=rng, kitti_view_other=other, kitti_view_frame=f)


def maicity_blocks(tmp):
    from test_dataset import write_maicity
    _, pose_path, g = write_maicity(tmp)
    P = D.read_poses_raw(pose_path)
    P32 = torch.tensor(P, dtype=torch.float32)
    xs = np.linspace(M_LO[0], M_HI[0], N_BLOCKS + 1)
    frames = [j for j in range(6) if (j + 1 - 3) % 5 != 0]
    blocks = []
    for b in range(N_BLOCKS):
        lo, hi = (float(xs[b]), M_LO[1], M_LO[2]), (float(xs[b + 1]), M_HI[1], M_HI[2])

        def frame(j):
            p = OD.filter_scan_maicity(g[f"f{j + 1}"], M_RD)
            return OD.in_parent_box(D.to_block(torch.from_numpy(p), P32[j]).numpy(), lo, hi)

        cells = OD.split_children(np.concatenate([frame(j) for j in frames]).astype(np.float32))
        b6, cen = OD.child_boxes(cells)
        rows = np.concatenate([RC.build_train_rays(frame(j), P[j][:3, 3], cen, b6, np.array(lo), np.array(hi), 0.05,
                                                   rule="0406") for j in frames])
        blocks.append((lo, hi, rows, len(cen)))
    return blocks


def main():
    import tempfile
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        out.update(kitti_view(os.path.join(tmp, "kitti_view")))
        k, n_children = kitti_rays(os.path.join(tmp, "kitti"))
        idx = np.random.default_rng(0).permutation(len(k["train"]))[:4096]
        out.update(kitti_train=k["train"][idx], kitti_train_idx=idx, kitti_train_total=len(k["train"]),
                   kitti_train_all=k["train"],
                   kitti_val=k["val"], kitti_children=n_children)
        for b, (lo, hi, rows, nc) in enumerate(maicity_blocks(os.path.join(tmp, "maicity"))):
            out[f"maicity_b{b}"] = rows[:1024]
            out[f"maicity_b{b}_total"] = len(rows)
            out[f"maicity_b{b}_lo"] = np.array(lo)
            out[f"maicity_b{b}_hi"] = np.array(hi)
            out[f"maicity_b{b}_children"] = nc
    path = os.path.join(HERE, "scene_rays.npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in out.items()})
    print("wrote", path, {k: np.asarray(v).shape for k, v in out.items()})


if __name__ == "__main__":
    main()
