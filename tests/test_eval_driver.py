"""Evaluation driver (pc-nerf_amd/eval_kitti_render.py): test-frame selection and the reference's batching rule on
CPU; on the GPU, the test rows of a fixture frame vs the oracle (bit-exact), batch-size independence of the
rendered cloud, and the PCD / row-cache round trip of main()."""
import os

import numpy as np
import pytest
import torch

import eval_kitti_render as E
from oracle import dataset_cpu as OD


def test_test_frames():
    assert E.test_frame_ids(1150, 1200) == [1153 + 5 * i for i in range(10)]
    assert E.test_frame_ids(0, 50)[:2] == [3, 8]
    # the commented rules of eval_kitti_render.py:1055-1062; 80 % renders exactly the frames 20 % trains on less
    t20, t80 = set(E.test_frame_ids(1150, 1200)), set(E.test_frame_ids(1150, 1200, 80))
    assert len(t80) == 40 and not t20 & t80 and t20 | t80 == set(range(1151, 1201))
    for sp, n in ((25, 12), (33, 16), (50, 25), (67, 33), (75, 37), (90, 45)):
        assert len(E.test_frame_ids(1150, 1200, sp)) == n, sp
    assert E.test_frame_ids(1150, 1156, 80) == [1151, 1152, 1154, 1155, 1156]   # config 5's 6-frame block
    with pytest.raises(ValueError):
        E.test_frame_ids(0, 10, 40)


def _groups(sizes):
    col = []
    for k in sizes:
        col += [k - 1] + [-1] * (k - 1)
    return np.asarray(col, dtype=np.float32)


@pytest.mark.parametrize("seed", range(6))
def test_batch_slices_match_reference_loop(seed):
    rng = np.random.default_rng(seed)
    col = _groups(rng.integers(1, 9, size=int(rng.integers(1, 3000))))
    for bs in (1, 7, 64, 4096):
        got = E.batch_slices(col, bs)
        assert got == OD.batch_slices(col, bs)
        for s, e in got:       # a batch never ends inside a group
            assert col[s] >= -0.5 and (e == len(col) or col[e] >= -0.5)


def test_batch_slices_edges():
    assert E.batch_slices(np.zeros(1, np.float32), 4) == []                 # lone last row dropped
    assert E.batch_slices(_groups([1, 1]), 4) == [(0, 2)]
    assert E.batch_slices(_groups([3, 1, 1, 1, 1, 1, 1]), 2) == [(0, 3), (3, 5), (5, 7), (7, 9)]


@pytest.mark.gpu
def test_view_rows_and_render_on_fixture(tmp_path):
    from test_dataset import write_scene, oracle_poses, DS, DE, KW, INTEREST
    from oracle import rays_cpu as RC
    from nof import io as nio
    from nof import synthetic as syn
    from nof.networks import NOF_coarse, NOF_fine
    root, pose_path, g = write_scene(str(tmp_path))
    ckpt = str(tmp_path / "seeded.ckpt")   # fixed weights for every main() call (a fresh NOF is randomly initialised)
    nio.save_ckpt(ckpt, nof_coarse=syn.load_into(NOF_coarse(), syn.init_nof_params(11)),
                  nof_fine=syn.load_into(NOF_fine(), syn.init_nof_params(12)))
    args = f"""--dataset kitti --root_dir {root} --pose_path {pose_path} --data_start {DS} --data_end {DE} --ckpt_path {ckpt}
     --test_data_create 1 --depth_inference_method 2 --result_path {tmp_path}/res --pcd_path {tmp_path}/pcd/v1_
     --N_samples 32 --N_importance 64 --chunk 8192 --range_delete_x 3 --range_delete_y 2 --range_delete_z 1.25
     --over_height 0.168 --over_low -2.0 --interest_x {INTEREST} --interest_y {INTEREST} --use_skip"""
    h = E.get_opts(args.split())
    scene = E.Scene(h, "cuda")
    f = E.test_frame_ids(DS, DE)[0]
    rows, ranges, other, tin = scene.view_rows(f, 2)
    # oracle: same parent cloud / raw child cells, oracle filter (strict < 120) and row builder
    P = oracle_poses(g, pose_path)
    positions = np.stack([P[k + 1][:3, 3] for k in range(DS, DE)])
    p = OD.filter_scan(g[f"f{f}"], KW["range_delete"], KW["over_height"], KW["over_low"], strict_range=True)
    import nof.dataset as D
    w = OD.interest_filter(D.to_block(torch.from_numpy(p), torch.from_numpy(P[f])).numpy(), positions, INTEREST,
                           INTEREST)
    cells = OD.split_children(D.fuse_frames(root, D.relative_poses(D.read_poses(pose_path), DS), DS, DE, "cpu",
                                            KW["range_delete"], KW["over_height"], KW["over_low"], INTEREST,
                                            INTEREST).numpy())
    b6 = np.concatenate([np.stack([a for a, _ in cells]), np.stack([b for _, b in cells])], 1)
    plo, phi = scene.parent6[:3].cpu().numpy(), scene.parent6[3:].cpu().numpy()
    orows, orng, ooth, otin = RC.build_view_rows(w, P[f][:3, 3].astype(np.float64), b6, plo, phi, 2)
    assert rows.shape[0] == orows.shape[0] > 50
    np.testing.assert_array_equal(rows.cpu().numpy(), orows)
    np.testing.assert_array_equal(other.cpu().numpy(), ooth)
    # batch-size independence (eval BN renders rows independently; groups never split)
    models = E.load_models(h, torch.device("cuda"))
    a, na = E.render_frame(models, rows, other, h, 64)
    b, nb = E.render_frame(models, rows, other, h, 1 << 20)
    assert na == nb and torch.equal(a, b) and a.shape[0] > 0
    # main(): build + cache + PCD, then the cached rows give the same cloud
    rep = E.main(args.split())
    h0 = args.replace("--test_data_create 1", "--test_data_create 0").replace("v1_", "v0_")
    rep0 = E.main(h0.split())
    assert [r["points"] for r in rep] == [r["points"] for r in rep0]
    for r in rep:
        x = nio.read_pcd(f"{tmp_path}/pcd/v1_{r['frame']}_two_step.pcd")
        y = nio.read_pcd(f"{tmp_path}/pcd/v0_{r['frame']}_two_step.pcd")
        assert x.shape == (r["points"], 3) and np.array_equal(x, y)


@pytest.mark.gpu
def test_view_rows_maicity_on_fixture(tmp_path):
    """MaiCity two-step rows (multi_frame_maicity): expansion step 0.005, parent-far column, boxes grown 0.025."""
    from test_dataset import write_maicity, M_LO, M_HI, M_RD
    from oracle import rays_cpu as RC
    import nof.dataset as D
    root, pose_path, g = write_maicity(str(tmp_path))
    args = f"""--dataset maicity --root_dir {root} --pose_path {pose_path} --data_start 0 --data_end 6
     --range_delete_x {M_RD[0]} --range_delete_y {M_RD[1]} --range_delete_z {M_RD[2]}
     --nerf_length_min {M_LO[0]} --nerf_length_max {M_HI[0]} --nerf_width_min {M_LO[1]} --nerf_width_max {M_HI[1]}
     --nerf_height_min {M_LO[2]} --nerf_height_max {M_HI[2]}"""
    h = E.get_opts(args.split())
    scene = E.Scene(h, "cuda")
    f = E.test_frame_ids(0, 6)[0]
    rows, ranges, other, tin = scene.view_rows(f, 2)
    P32 = torch.tensor(D.read_poses_raw(pose_path), dtype=torch.float32)
    pts = OD.in_parent_box(D.to_block(torch.from_numpy(OD.filter_scan_maicity(g[f"f{f}"], M_RD)),
                                      P32[f - 1]).numpy(), M_LO, M_HI)
    b6 = scene.bounds6.cpu().numpy()
    orows, orng, ooth, _ = RC.build_view_rows(pts, P32[f - 1][:3, 3].double().numpy(), b6, np.array(M_LO),
                                              np.array(M_HI), 2, rule="maicity")
    assert rows.shape[0] == orows.shape[0] > 50
    np.testing.assert_array_equal(rows.cpu().numpy(), orows)
    np.testing.assert_array_equal(other.cpu().numpy(), ooth)
    np.testing.assert_array_equal(ranges.cpu().numpy(), orng)


@pytest.mark.gpu
@pytest.mark.parametrize("method", [2, 0])
def test_two_step_render_kitti_rows_vs_reference(method):
    """Config 5's path on real rows: the two-step test rows of the first KITTI fixture frame
    (tests/golden/scene_rays.npz kitti_view_*, the oracle rows that test_view_rows_and_render_on_fixture checks the
    GPU row builder against bit for bit) through render_rays_view_0525_2_2, against the reference's own render of
    the same rows and weights (tests/golden/make_golden.py gen_view_kitti): effective-row flags bit-equal, depths
    and points within 1e-4 (the north star), opacities within 1e-5."""
    from conftest import golden
    from nof import synthetic as syn
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_view_0525_2_2
    g = golden("render_view_kitti")
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(11)).cuda().eval()
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(12)).cuda().eval()
    with torch.no_grad():
        res = render_rays_view_0525_2_2(mc, mf, Embedding(3, 10), torch.from_numpy(g["rows"]).cuda(),
                                        torch.from_numpy(g["other"]).cuda(), N_samples=64, N_importance=128,
                                        perturb=0, noise_std=0, chunk=262144, depth_inference_method=method)
    pre = f"m{method}_"
    for k in ("rays_effective_flag", "rays_effective_flag_fine"):
        np.testing.assert_array_equal(res[k].cpu().numpy(), g[pre + k], err_msg=k)
    for k in ("depth", "depth_fine", "points_inference", "points_inference_fine"):
        np.testing.assert_allclose(res[k].cpu().numpy(), g[pre + k], rtol=1e-4, atol=1e-5, err_msg=k)
    for k in ("opacity", "opacity_fine"):
        np.testing.assert_allclose(res[k].cpu().numpy(), g[pre + k], rtol=1e-5, err_msg=k)
    d, r = res["depth_fine"].cpu().numpy().astype(np.float64), g[pre + "depth_fine"].astype(np.float64)
    _report({"case": f"config5_kitti_rows_m{method}", "rows": int(len(r)),
             "depth_fine_max_rel": float(np.max(np.abs(d - r) / np.maximum(np.abs(r), 1e-6))),
             "flags_equal": True})


def _report(line):
    import json
    path = os.environ.get("PCNERF_PARITY_REPORT")
    if path:
        with open(path, "a") as fh:
            fh.write(json.dumps(line) + "\n")


def _eval_rank(rank, world, port, argv, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "pc-nerf_amd"), here):
        sys.path.insert(0, p)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import eval_kitti_render as E2
    rep = E2.main(argv)
    q.put((rank, rep))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_eval_driver_two_ranks_writes_the_same_pcd(tmp_path):
    """The eval driver under 2 ranks sharing the GPU (gloo carries the gather: RCCL needs one GPU per rank): each
    rank renders a row-balanced share of whole ray groups, rank 0 gathers the points and writes the PCD -- byte-
    identical to the single-process run's."""
    import socket
    import torch.multiprocessing as mp
    from test_dataset import write_scene, DS, DE, INTEREST
    from nof import io as nio
    from nof import synthetic as syn
    from nof.networks import NOF_coarse, NOF_fine
    root, pose_path, g = write_scene(str(tmp_path))
    ckpt = str(tmp_path / "seeded.ckpt")
    nio.save_ckpt(ckpt, nof_coarse=syn.load_into(NOF_coarse(), syn.init_nof_params(11)),
                  nof_fine=syn.load_into(NOF_fine(), syn.init_nof_params(12)))
    base = f"""--dataset kitti --root_dir {root} --pose_path {pose_path} --data_start {DS} --data_end {DE} --ckpt_path {ckpt}
     --test_data_create 1 --depth_inference_method 2 --N_samples 32 --N_importance 64 --chunk 8192
     --range_delete_x 3 --range_delete_y 2 --range_delete_z 1.25 --over_height 0.168 --over_low -2.0
     --interest_x {INTEREST} --interest_y {INTEREST} --use_skip --batch_rows 256"""
    one = (base + f" --result_path {tmp_path}/r1 --pcd_path {tmp_path}/pcd/w1_").split()
    two = (base + f" --result_path {tmp_path}/r2 --pcd_path {tmp_path}/pcd/w2_ --dist_backend gloo").split()
    rep1 = E.main(one)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_eval_rank, args=(r, 2, port, two, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, rep = q.get(timeout=240)
        got[r] = rep
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert [r["rows"] for r in got[0]] == [r["rows"] for r in rep1]
    assert [r["points"] for r in got[0]] == [r["points"] for r in rep1] and got[1] == []
    for r in rep1:
        a = open(f"{tmp_path}/pcd/w1_{r['frame']}_two_step.pcd", "rb").read()
        b = open(f"{tmp_path}/pcd/w2_{r['frame']}_two_step.pcd", "rb").read()
        assert r["points"] > 0 and a == b


@pytest.mark.gpu
def test_eval_driver_frame_sparsity_80(tmp_path):
    """--frame_sparsity 80 (eval_kitti_render.py:1060, BASELINE config 5's rule): main() renders exactly the frames
    the 80 % rule holds out -- the complement of the 20 % rule's -- and each frame's rendered row count is the one its
    two-step rows give (the reference's batching rule: all rows but a lone last one)."""
    from test_dataset import write_scene, DS, DE, INTEREST
    root, pose_path, g = write_scene(str(tmp_path))
    base = f"""--dataset kitti --root_dir {root} --pose_path {pose_path} --data_start {DS} --data_end {DE}
     --test_data_create 1 --depth_inference_method 2 --N_samples 32 --N_importance 64 --chunk 8192
     --range_delete_x 3 --range_delete_y 2 --range_delete_z 1.25 --over_height 0.168 --over_low -2.0
     --interest_x {INTEREST} --interest_y {INTEREST} --use_skip --result_path {tmp_path}/res
     --pcd_path {tmp_path}/pcd/s80_ --frame_sparsity 80"""
    rep = E.main(base.split())
    frames = [r["frame"] for r in rep]
    assert frames == E.test_frame_ids(DS, DE, 80) == [f for f in range(DS + 1, DE + 1)
                                                      if f not in E.test_frame_ids(DS, DE)]
    h = E.get_opts(base.split())
    scene = E.Scene(h, "cuda")
    for r in rep:
        rows, _, _, _ = scene.view_rows(r["frame"], 2)
        assert r["rows"] == sum(e - s for s, e in E.batch_slices(rows[:, 12].cpu().numpy(), 4096)) > 0
        assert os.path.exists(f"{tmp_path}/pcd/s80_{r['frame']}_two_step.pcd")
