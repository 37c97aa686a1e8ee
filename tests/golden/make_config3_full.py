"""BASELINE config 3's scene: KITTI-00 frames 1151-1200 at the 50 % frame-sparsity rule.

    python tests/golden/make_config3_full.py frames   -> kitti_frames_full.npz: scans 1151..1200 of the reference's
                                                         data/kitti/00/pcd_remove_dynamic (every 16th point, float32
                                                         as stored) and poses.txt rows 1150..1200
    python tests/golden/make_config3_full.py rays     -> config3_full_scene.npz: the train split's rows built by the
                                                         CPU restatement (oracle/dataset_cpu.py + rays_cpu.py) from
                                                         those frames -- count, sha256 of the float32 rows, children,
                                                         the first 4,096 rows -- and the whole table in
                                                         /tmp/config3_full_rows.npy for the next two steps
    python tests/golden/make_config3_full.py ref [threads] [name]
                                                      -> config3_full.npz (config3_full_alt.npz with 3 threads): the
                                                         reference's render_rays_train (imported from
                                                         /root/reference/nof, as make_golden.py does) on the
                                                         262,144-ray batch drawn with numpy seed 3
    python tests/golden/make_config3_full.py f64      -> config3_full_f64.npz: the float64 evaluation (make_f64.py's)

The scene: ipb2dmapping.py:647-660's train rule ``(j+1-data_start) % 2 != 0`` (frame sparsity 50 %) over
data_start 1150, data_end 1200 (25 train frames), the parent cloud fused from every train-rule frame of
pointcloud_fusion.py ((j+1-3) % 5 != 0), 1 m child cells, the KITTI shell's filters and a 20 m interest region --
the settings of the 6-scan fixture (make_scene_rays.py), on the whole 50-frame sequence.  Test infrastructure.
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
DS, DE, SPARSITY, STEP = 1150, 1200, 50, 16
N_RAYS, SEED = 262144, 3
ROWS_TMP = "/tmp/config3_full_rows.npy"


def sha(rows):
    return hashlib.sha256(np.ascontiguousarray(rows, dtype=np.float32).tobytes()).hexdigest()


def raw_pcd(path):
    """make_golden.py's minimal reader of the reference's binary xyz float32 PCDs (no reference import here)."""
    b = open(path, "rb").read()
    i = b.index(b"DATA binary\n") + len(b"DATA binary\n")
    n = int([ln for ln in b[:i].decode().splitlines() if ln.startswith("POINTS")][0].split()[1])
    return np.frombuffer(b[i:i + 12 * n], dtype="<f4").reshape(n, 3).copy()


def gen_frames():
    frames = {f"f{f}": raw_pcd(os.path.join(REF, f"data/kitti/00/pcd_remove_dynamic/{f}.pcd"))[::STEP]
              for f in range(DS + 1, DE + 1)}
    with open(os.path.join(REF, "data/kitti/00/poses.txt")) as fh:
        rows = [ln.strip() for ln in fh if ln.strip()]
    poses = np.array([[float(v) for v in rows[i].split(" ")] for i in range(DS, DE + 1)])
    path = os.path.join(HERE, "kitti_frames_full.npz")
    np.savez_compressed(path, poses=poses, pose_first=np.array(DS), **frames)
    print("wrote", path, sum(v.shape[0] for v in frames.values()), "points")


def build_rows():
    import tempfile
    import torch
    for p in (REPO, os.path.join(REPO, "pc-nerf_amd"), os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    from nof import dataset as D
    from oracle import dataset_cpu as OD
    from oracle import rays_cpu as RC
    from test_dataset import oracle_poses, write_scene
    from make_scene_rays import KW, INTEREST
    with tempfile.TemporaryDirectory() as tmp:
        root, pose_path, g = write_scene(tmp, "kitti_frames_full")
        rel = D.relative_poses(D.read_poses(pose_path), DS)
        cloud = D.fuse_frames(root, rel, DS, DE, "cpu", KW["range_delete"], KW["over_height"], KW["over_low"],
                              INTEREST, INTEREST).numpy()
        b6, cen = OD.child_boxes(OD.split_children(cloud))
        plo, phi = cloud.astype(np.float64).min(0), cloud.astype(np.float64).max(0)
        P = oracle_poses(g, pose_path)
        positions = np.stack([P[k + 1][:3, 3] for k in range(DS, DE)])
        rows = []
        for f in D.frame_ids(DS, DE, "train", SPARSITY):
            p = OD.filter_scan(g[f"f{f}"], KW["range_delete"], KW["over_height"], KW["over_low"])
            w = OD.interest_filter(D.to_block(torch.from_numpy(p), torch.from_numpy(P[f])).numpy(), positions,
                                   INTEREST, INTEREST)
            rows.append(RC.build_train_rays(w, P[f][:3, 3].astype(np.float64), cen, b6, plo, phi, 0.05))
            print("frame", f, rows[-1].shape[0], "rows", flush=True)
    rows = np.concatenate(rows).astype(np.float32)
    np.save(ROWS_TMP, rows)
    path = os.path.join(HERE, "config3_full_scene.npz")
    np.savez_compressed(path, n_rows=rows.shape[0], sha256=np.array(sha(rows)), children=len(cen),
                        head=rows[:4096], frames=np.array(D.frame_ids(DS, DE, "train", SPARSITY)),
                        data_start=DS, data_end=DE, sparsity=SPARSITY, step=STEP)
    print("wrote", path, rows.shape, "children", len(cen))


def batch():
    rows = np.load(ROWS_TMP)
    sc = dict(np.load(os.path.join(HERE, "config3_full_scene.npz"), allow_pickle=False))
    assert sha(rows) == str(sc["sha256"]), "rows in /tmp differ from the committed scene: rerun `rays`"
    idx = np.random.default_rng(SEED).integers(0, rows.shape[0], N_RAYS)
    return rows[idx], int(sc["children"])


def gen_ref(threads=None, name="config3_full"):
    """The reference's render_rays_train on the batch, train mode, the PC-NeRF KITTI shell's settings."""
    import time
    rays, n_child = batch()
    sys.argv = [sys.argv[0]]
    sys.path.insert(0, HERE)
    import make_golden as G   # imports the reference's nof (and applies its one device shim)
    import torch
    torch.set_num_threads(threads or os.cpu_count() or 1)
    emb, mc, mf = G.models(train=True)
    t0 = time.perf_counter()
    with torch.no_grad():
        res = G.R.render_rays_train(mc, mf, emb, torch.from_numpy(rays), sub_nerf_test_num=n_child, N_samples=64,
                                    N_importance=128, **G.PCNERF_TRAIN)
    print(name, time.perf_counter() - t0, "s")
    G.save(name, n_rays=rays.shape[0], seed=SEED, N_samples=64, N_importance=128, sub_nerf_test_num=n_child,
           threads=torch.get_num_threads(), **G.train_outputs(res, rays, mc, mf))


def gen_f64():
    import torch
    for p in (REPO, os.path.join(REPO, "pc-nerf_amd"), os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    sys.path.insert(0, HERE)
    from make_f64 import render64, stats
    from nof import synthetic as syn
    from oracle import ref_cpu as O
    torch.set_num_threads(os.cpu_count() or 1)
    rays, _ = batch()
    g = dict(np.load(os.path.join(HERE, "config3_full.npz"), allow_pickle=False))
    with torch.no_grad():
        d64, df64 = render64(O.params_from_numpy(syn.init_nof_params(1234)), O.params_from_numpy(
            syn.init_nof_params(5678)), torch.from_numpy(rays), 64, 128, 262144)
    stats("config3_full ref depth", g["depth"], d64)
    stats("config3_full ref depth_fine", g["depth_fine"], df64)
    path = os.path.join(HERE, "config3_full_f64.npz")
    np.savez_compressed(path, depth=d64, depth_fine=df64)
    print("wrote", path)


if __name__ == "__main__":
    what = sys.argv[1]
    if what == "frames":
        gen_frames()
    elif what == "rays":
        build_rows()
    elif what == "ref":
        gen_ref(int(sys.argv[2]) if len(sys.argv) > 2 else None, sys.argv[3] if len(sys.argv) > 3 else "config3_full")
    elif what == "f64":
        gen_f64()
    else:
        raise SystemExit(__doc__)
