"""Dataset pipeline (nof/dataset.py) vs its CPU oracle (oracle/dataset_cpu.py + oracle/rays_cpu.py).

Fixture: tests/golden/kitti_frames.npz -- KITTI-00 scans 1151..1156 from the reference's data directory (every
40th point) and poses.txt rows 1150..1156 (make_golden.gen_kitti_frames).  The host stages (filter, block
transform, interest region, fusion, child cells) are device-agnostic tensor code and are checked here on CPU
tensors; the ray rows need the HIP kernel and are checked in the GPU test (bit-exact rows vs the oracle).
Tolerance: exact everywhere except the block transform, which the reference runs through numpy's BLAS (1 ulp of
float64 allowed, rtol 1e-15)."""
import os

import numpy as np
import pytest
import torch

from conftest import golden
from nof import dataset as D
from nof import io as nio
from oracle import dataset_cpu as OD
from oracle import rays_cpu as RC

DS, DE = 1150, 1155
KW = dict(range_delete=(3.0, 2.0, 1.25), over_height=0.168, over_low=-2.0)
INTEREST = 20.0


def write_scene(tmp, name="kitti_frames"):
    """The fixture as the reference's inputs: <tmp>/pcd/<n>.pcd and a poses.txt whose rows 1150..1156 are real
    (``kitti_frames_full``: scans 1151..1200, rows 1150..1200)."""
    g = golden(name)
    os.makedirs(os.path.join(tmp, "pcd"), exist_ok=True)
    for k, v in g.items():
        if k.startswith("f"):
            nio.write_pcd(os.path.join(tmp, "pcd", f"{k[1:]}.pcd"), v)
    ident = "1 0 0 0 0 1 0 0 0 0 1 0"
    first = int(g["pose_first"])
    with open(os.path.join(tmp, "poses.txt"), "w") as fh:
        for _ in range(first):
            fh.write(ident + "\n")
        for row in g["poses"]:
            fh.write(" ".join(repr(float(v)) for v in row) + "\n")
    return os.path.join(tmp, "pcd"), os.path.join(tmp, "poses.txt"), g


def oracle_poses(g, pose_path):
    """ipb2dmapping.py:566-584 restated: every row of the file, then one batched float32 T_start^-1 @ poses (the
    batched product's rounding depends on the batch, so the whole file goes through it, as in the reference)."""
    return oracle_poses_from(g, pose_path, DS)


def oracle_poses_from(g, pose_path, data_start):
    """oracle_poses relative to frame ``data_start`` + 1 (another block's start)."""
    P = np.asarray([np.vstack([np.loadtxt([ln]).reshape(3, 4), [[0, 0, 0, 1.0]]]) @ D.T_VELO2CAM
                    for ln in open(pose_path).read().splitlines()])
    rel = (torch.from_numpy(np.linalg.inv(P[data_start + 1])).float() @ torch.tensor(P, dtype=torch.float32)).numpy()
    return {int(g["pose_first"]) + i: rel[int(g["pose_first"]) + i] for i in range(len(g["poses"]))}


def test_frame_rules():
    assert D.frame_ids(1150, 1200, "val") == [1153 + 5 * i for i in range(10)]
    tr = D.frame_ids(1150, 1200, "train")
    assert len(tr) == 40 and not set(tr) & set(D.frame_ids(1150, 1200, "val"))
    for sp, n in ((25, 38), (33, 34), (50, 25), (67, 17), (75, 13), (80, 10), (90, 5)):
        assert len(D.frame_ids(1150, 1200, "train", sp)) == n, sp
    with pytest.raises(ValueError):
        D.frame_ids(0, 5, "test")


def test_poses_match_oracle(tmp_path):
    _, pose_path, g = write_scene(str(tmp_path))
    rel = D.relative_poses(D.read_poses(pose_path), DS)
    for f, p in oracle_poses(g, pose_path).items():
        np.testing.assert_array_equal(rel[f].numpy(), p)
    np.testing.assert_allclose(rel[DS + 1].numpy(), np.eye(4), atol=1e-4)  # float32 rounding of |t| ~ 165 m


def test_host_stages_match_oracle(tmp_path):
    _, pose_path, g = write_scene(str(tmp_path))
    rel = D.relative_poses(D.read_poses(pose_path), DS)
    P = oracle_poses(g, pose_path)
    positions = np.stack([P[k + 1][:3, 3] for k in range(DS, DE)])
    for f in (1151, 1153, 1155):
        raw = g[f"f{f}"]
        got = D.filter_scan(torch.from_numpy(raw), **KW)
        want = OD.filter_scan(raw, KW["range_delete"], KW["over_height"], KW["over_low"])
        np.testing.assert_array_equal(got.numpy(), want)
        w = D.to_block(got, rel[f])
        ow = OD.to_block(want, P[f])
        np.testing.assert_allclose(w.numpy(), ow, rtol=1e-15, atol=1e-13)
        m = D.interest_mask(w, rel[DS + 1:DE + 1, :3, 3], INTEREST, 8.0)
        np.testing.assert_array_equal(w[m].numpy(), OD.interest_filter(w.numpy(), positions, INTEREST, 8.0))
        assert 0 < int(m.sum()) < len(m)


def test_fusion_and_child_cells_match_oracle(tmp_path):
    root, pose_path, g = write_scene(str(tmp_path))
    rel = D.relative_poses(D.read_poses(pose_path), DS)
    cloud = D.fuse_frames(root, rel, DS, DE, "cpu", KW["range_delete"], KW["over_height"], KW["over_low"],
                          INTEREST, INTEREST)
    assert cloud.dtype == torch.float32 and cloud.shape[0] > 1000
    mn, mx = D.split_children(cloud)
    cells = OD.split_children(cloud.numpy())
    assert len(cells) == mn.shape[0]
    np.testing.assert_array_equal(mn.numpy(), np.stack([a for a, _ in cells]))
    np.testing.assert_array_equal(mx.numpy(), np.stack([b for _, b in cells]))
    b6, c = D.child_boxes(mn, mx)
    ob6, oc = OD.child_boxes(cells)
    np.testing.assert_array_equal(b6.numpy(), ob6)
    np.testing.assert_array_equal(c.numpy(), oc)
    assert np.all((mx - mn).numpy() <= 1.5 + 0.05 + 1e-9)


def test_val_index_rule():
    for n, k in ((10, 4), (1000, 37), (123457, 4096)):
        ds = D.kitti_dataload.__new__(D.kitti_dataload)
        ds.rays, ds.cloud_size_val = torch.zeros((n, 15)), k
        np.testing.assert_array_equal(ds.val_index().numpy(), OD.val_index(n, k))


@pytest.mark.gpu
def test_kitti_dataload_rays_match_oracle(tmp_path):
    root, pose_path, g = write_scene(str(tmp_path))
    kw = dict(data_start=DS, data_end=DE, cloud_size_val=64, range_delete_x=3, range_delete_y=2,
              range_delete_z=1.25, sub_nerf_test_num=0, surface_expand=0.05, over_height=0.168, over_low=-2.0,
              interest_x=INTEREST, interest_y=INTEREST, pose_path=pose_path, re_loaddata=1,
              result_path=str(tmp_path / "out"), device="cuda")
    tr = D.kitti_dataload(root, split="train", **kw)
    va = D.kitti_dataload(root, split="val", **kw)
    # oracle: same parent cloud (fusion is checked on CPU above), oracle child cells / rays per frame
    cloud = tr.parent_cloud.cpu().numpy()
    b6, cen = OD.child_boxes(OD.split_children(cloud))
    plo, phi = cloud.astype(np.float64).min(0), cloud.astype(np.float64).max(0)
    P = oracle_poses(g, pose_path)
    positions = np.stack([P[k + 1][:3, 3] for k in range(DS, DE)])
    for ds, split in ((tr, "train"), (va, "val")):
        want = []
        for f in D.frame_ids(DS, DE, split):
            p = OD.filter_scan(g[f"f{f}"], KW["range_delete"], KW["over_height"], KW["over_low"])
            w = OD.interest_filter(D.to_block(torch.from_numpy(p), torch.from_numpy(P[f])).numpy(), positions,
                                   INTEREST, INTEREST)
            want.append(RC.build_train_rays(w, P[f][:3, 3].astype(np.float64), cen, b6, plo, phi, 0.05))
        want = np.concatenate(want)
        got = ds.rays.cpu().numpy()
        assert got.shape == want.shape and len(got) > 100, (split, got.shape, want.shape)
        np.testing.assert_array_equal(got, want)
    # val sampling and the ray cache round trip (re_loaddata=0)
    b = va[torch.arange(64)]
    np.testing.assert_array_equal(b["rays"].cpu().numpy(), va.rays.cpu().numpy()[OD.val_index(len(va.rays), 64)])
    again = D.kitti_dataload(root, split="train", **{**kw, "re_loaddata": 0})
    assert torch.equal(again.rays, tr.rays)


# ----------------------------------------------------------------------------------------------- MaiCity
M_LO, M_HI = (-12.0, -12.0, -2.0), (61.0, 12.0, 0.5)     # shells/pretraining/MaiCity00_pcnerf_train.bash
M_RD = (2.0, 1.0, 0.5)


def write_maicity(tmp):
    g = golden("maicity_frames")
    os.makedirs(os.path.join(tmp, "pcd"), exist_ok=True)
    for k, v in g.items():
        if k.startswith("f"):
            nio.write_pcd(os.path.join(tmp, "pcd", f"{k[1:]}.pcd"), v)
    with open(os.path.join(tmp, "poses.txt"), "w") as fh:
        for row in g["poses"]:
            fh.write(" ".join(repr(float(v)) for v in row) + "\n")
    return os.path.join(tmp, "pcd"), os.path.join(tmp, "poses.txt"), g


def test_maicity_host_stages_match_oracle(tmp_path):
    _, pose_path, g = write_maicity(str(tmp_path))
    P = D.read_poses_raw(pose_path)
    np.testing.assert_array_equal(P[:, :3, :].reshape(len(P), 12), g["poses"])
    P32 = torch.tensor(P, dtype=torch.float32)
    for j in (0, 2, 4):
        raw = g[f"f{j + 1}"]
        got = D.filter_scan_maicity(torch.from_numpy(raw), M_RD)
        want = OD.filter_scan_maicity(raw, M_RD)
        np.testing.assert_array_equal(got.numpy(), want)
        w = D.to_block(got, P32[j])
        kept = w[D.in_box(w, M_LO, M_HI)].numpy()
        np.testing.assert_array_equal(kept, OD.in_parent_box(w.numpy(), M_LO, M_HI))
        assert 0 < len(kept) < len(got)


@pytest.mark.gpu
def test_maicity_dataload_rays_match_oracle(tmp_path):
    root, pose_path, g = write_maicity(str(tmp_path))
    kw = dict(data_start=0, data_end=6, cloud_size_val=32, range_delete_x=M_RD[0], range_delete_y=M_RD[1],
              range_delete_z=M_RD[2], sub_nerf_test_num=0, surface_expand=0.05, nerf_length_min=M_LO[0],
              nerf_length_max=M_HI[0], nerf_width_min=M_LO[1], nerf_width_max=M_HI[1], nerf_height_min=M_LO[2],
              nerf_height_max=M_HI[2], pose_path=pose_path, re_loaddata=1, result_path=str(tmp_path / "out"),
              device="cuda")
    P = D.read_poses_raw(pose_path)
    P32 = torch.tensor(P, dtype=torch.float32)

    def oracle_frame(j):
        p = OD.filter_scan_maicity(g[f"f{j + 1}"], M_RD)
        return OD.in_parent_box(D.to_block(torch.from_numpy(p), P32[j]).numpy(), M_LO, M_HI)

    frames = [j for j in range(6) if (j + 1 - 3) % 5 != 0]
    cells = OD.split_children(np.concatenate([oracle_frame(j) for j in frames]).astype(np.float32))
    b6, cen = OD.child_boxes(cells)
    want, err = [], None
    try:
        for j in frames:
            want.append(RC.build_train_rays(oracle_frame(j), P[j][:3, 3], cen, b6, np.array(M_LO), np.array(M_HI),
                                            0.05, rule="0406"))
    except IndexError as e:       # the reference raises here too; the GPU path must as well
        err = e
    if err is not None:
        with pytest.raises(IndexError):
            D.maicity_dataload(root, split="train", **kw)
        return
    tr = D.maicity_dataload(root, split="train", **kw)
    got = tr.rays.cpu().numpy()
    want = np.concatenate(want)
    assert got.shape == want.shape and len(got) > 100
    np.testing.assert_array_equal(got, want)
