"""BASELINE.json's configurations on the GPU, against the reference.

  config 1  KITTI-00 rays, 4,096-ray batch, 64/128 samples (train and val) -- rows rebuilt on the GPU by
            nof.dataset from the fixture frames, checked bit for bit against the fixture's rows, then rendered and
            compared with the reference's outputs on those rows (tests/golden/config1_kitti.npz);
  config 2  the headline workload at FULL size: 65,536 rays, 128/256 samples, chunk 262,144 (32 coarse + 96 fine
            BatchNorm chunks), child losses, against the reference run on the same rays (config2_full.npz);
  config 3  the KITTI training loop at 262,144 rays/iter (64/128 samples): the full-size step's forward against the
            reference run on the same rays (config3_full.npz: frames 1151-1200 at 50 % sparsity), then forward, losses, backward, Adam, properties;
  config 4  MaiCity-00 in 4 parent blocks, each with its own weights (config4_maicity.npz);
  the training driver: k steps of Adam + MultiStepLR through train_kitti.fit() against the oracle's autograd +
            torch.optim.Adam (parameters and per-step losses), once with BatchNorm inputs whose |mean|/std >> 1.

Tolerances: depths, losses, BatchNorm running stats rtol 1e-4 against the reference (the north star's bound),
atol 1e-6 for values near zero -- except depth_fine of the train-mode configs, which is ill-conditioned in the
reference itself: its float32 value moves by up to ~1e-4 (config 2) / ~8e-4 (config 1) when the reference is
rerun with another thread count, and sits as far from a float64 evaluation of the same function.  There the HIP
depth_fine must be within 1e-4 of the float64 evaluation for every ray (tests/golden/make_f64.py) and no farther
from the reference than the reference is from itself (check_fine_depth).  Every number is reported
(PCNERF_PARITY_REPORT=<path> appends one JSON line per case).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import golden
from nof import synthetic as syn
from nof.criteria import nof_loss
from nof.networks import Embedding, NOF_coarse, NOF_fine
from nof import render as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEED_C, SEED_F = 1234, 5678
RTOL = 1e-4
PCNERF_TRAIN = dict(use_child_nerf_loss=1, issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0, perturb=0,
                    noise_std=0, chunk=262144)


def models(train, sc=SEED_C, sf=SEED_F):
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(sc)).to(DEV).train(train)
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(sf)).to(DEV).train(train)
    return Embedding(3, 10), mc, mf


def running(m):
    return np.stack([np.stack([bn.running_mean.cpu().numpy(), bn.running_var.cpu().numpy()]) for bn in m.norms()])


def report(name, **vals):
    path = os.environ.get("PCNERF_PARITY_REPORT")
    if path:
        with open(path, "a") as fh:
            fh.write(json.dumps({"case": name, **{k: float(v) for k, v in vals.items()}}) + "\n")


def max_rel(a, b):
    a = a.detach().cpu().numpy().astype(np.float64) if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-6)))


def close(a, b, rtol=RTOL, atol=1e-6, what=""):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    np.testing.assert_allclose(a.astype(np.float64), b.astype(np.float64), rtol=rtol, atol=atol, err_msg=what)


def rel_err(a, b):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    a, b = a.astype(np.float64), np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), 1e-6)


def check_fine_depth(got, ref, f64, alt, what):
    """depth_fine, whose float32 value is ill-conditioned in the reference itself (tests/golden/make_f64.py): within
    1e-4 of the float64 evaluation of the same rays/weights for EVERY ray, and no farther from the reference than
    the reference is from itself rerun with another thread count (quantiles 50 / 99 / 99.9 / 100 %, 1.5x + 2e-5)."""
    e64, eref, eself = rel_err(got, f64), rel_err(got, ref), rel_err(alt, ref)
    qs = (0.5, 0.99, 0.999, 1.0)
    stats = {f"{what}_vs_f64_max": e64.max(), f"{what}_vs_ref_max": eref.max(),
             f"{what}_ref_self_spread_max": eself.max(), f"{what}_ref_vs_f64_max": rel_err(ref, f64).max(),
             f"{what}_vs_ref_frac_gt_1e-4": (eref > 1e-4).mean(), f"{what}_ref_self_frac_gt_1e-4": (eself > 1e-4).mean()}
    bad = []
    if e64.max() > RTOL:
        bad.append(f"{what}: {int((e64 > RTOL).sum())} rays beyond 1e-4 of the float64 evaluation (max {e64.max():.3e})")
    for q in qs:
        a, b = np.quantile(eref, q), np.quantile(eself, q)
        if a > 1.5 * b + 2e-5:
            bad.append(f"{what}: q{q} vs reference {a:.3e} > 1.5 x its self-spread {b:.3e} + 2e-5")
    return stats, bad


def check_train(res, g, rays, mc, mf, pre="", name="", f64=None, alt=None):
    """Depths, the four child losses, the range losses of train_kitti.py:144-146, the total, running stats:
    rtol 1e-4 against the reference; depth_fine as check_fine_depth says when the float64 evaluation and the
    reference's self-spread rerun are given (else rtol 1e-4 too).  Every number is reported before asserting."""
    loss = nof_loss["smoothl1"]()
    gt = rays[:, 14]
    lr = 1e-1 * loss(1e1 * res["depth"], 1e1 * gt)
    lrf = 1e-1 * loss(1e1 * res["depth_fine"], 1e1 * gt)
    tot = lr + lrf + 1e6 * res["child_free_loss_fine"] + 1e6 * res["child_free_loss"] + \
        1e5 * res["child_depth_loss_fine"] + 1e5 * res["child_depth_loss"]
    vals = {"depth": res["depth"], "child_free_loss": res["child_free_loss"],
            "child_depth_loss": res["child_depth_loss"], "child_free_loss_fine": res["child_free_loss_fine"],
            "child_depth_loss_fine": res["child_depth_loss_fine"], "loss_range": lr, "loss_range_fine": lrf,
            "loss_total": tot, "running_c": running(mc), "running_f": running(mf)}
    if f64 is None:
        vals["depth_fine"] = res["depth_fine"]
    stats, bad = {}, []
    for k, v in vals.items():
        e = rel_err(v, g[pre + k])
        stats[k + "_max_rel"] = e.max()
        atol = 1e-6 if k in ("depth", "depth_fine", "running_c", "running_f") else 1e-9
        if alt is not None and k in ("running_c", "running_f"):
            # a chunk's running mean sums 262,144 samples: entries near zero move by up to ~3e-5 absolute when the
            # reference itself reruns with another thread count -- twice that spread is the absolute floor
            spread = float(np.max(np.abs(np.asarray(alt[pre + k], np.float64) - np.asarray(g[pre + k], np.float64))))
            stats[k + "_ref_self_spread_abs"] = spread
            stats[k + "_max_abs"] = float(np.max(np.abs(np.asarray(v, np.float64) - np.asarray(g[pre + k], np.float64))))
            atol = max(atol, 2 * spread)
        if not np.all(np.abs(np.asarray(v.detach().cpu() if torch.is_tensor(v) else v, np.float64)
                             - np.asarray(g[pre + k], np.float64)) <= atol + RTOL * np.abs(g[pre + k])):
            bad.append(f"{k}: max rel {e.max():.3e} vs reference")
    if f64 is not None:
        st, b = check_fine_depth(res["depth_fine"], g[pre + "depth_fine"], f64[pre + "depth_fine"],
                                 alt[pre + "depth_fine"], "depth_fine")
        stats.update(st)
        bad += b
        stats["depth_vs_f64_max"] = rel_err(res["depth"], f64[pre + "depth"]).max()
    report(name, rays=rays.shape[0], **stats)
    assert not bad, "\n".join(bad)


# ----------------------------------------------------------------------------------------------- config 2
@pytest.fixture(params=["f16x2_3", "fp32", "f16x2_3_fused"])
def train_math(request):
    """The train-mode layer arithmetic (nof._ops.set_train_math): the default split-fp16 products and fp32 MFMA."""
    from nof import _ops
    prev = _ops.set_train_math(request.param)
    yield request.param
    _ops.set_train_math(prev)


def test_config2_full_size_vs_reference(train_math):
    """65,536 rays x (128 + 384) MLP samples in train-mode BatchNorm chunks of 262,144, vs the reference."""
    g = golden("config2_full")
    rays = torch.from_numpy(syn.make_rays(int(g["n_rays"]), n_children=32, seed=int(g["seed"]))).to(DEV)
    emb, mc, mf = models(True)
    with torch.no_grad():
        res = R.render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=32, N_samples=128, N_importance=256,
                                  **PCNERF_TRAIN)
    dump = os.environ.get("PCNERF_PARITY_DUMP")
    if dump:   # the HIP depths, for offline analysis against the reference / a float64 evaluation
        np.savez_compressed(dump, depth=res["depth"].cpu().numpy(), depth_fine=res["depth_fine"].cpu().numpy())
    check_train(res, g, rays, mc, mf, name=f"config2_full_{train_math}", f64=golden("config2_full_f64"),
                alt=golden("config2_full_alt"))
    assert int(mc.norms()[0].num_batches_tracked) == 32 and int(mf.norms()[0].num_batches_tracked) == 96


# ----------------------------------------------------------------------------------------------- config 1
def kitti_scene(tmp_path):
    from test_dataset import DS, DE, INTEREST, write_scene
    from nof import dataset as D
    root, pose_path, _ = write_scene(str(tmp_path))
    kw = dict(data_start=DS, data_end=DE, cloud_size_val=64, range_delete_x=3, range_delete_y=2,
              range_delete_z=1.25, sub_nerf_test_num=0, surface_expand=0.05, over_height=0.168, over_low=-2.0,
              interest_x=INTEREST, interest_y=INTEREST, pose_path=pose_path, re_loaddata=1,
              result_path=str(tmp_path / "out"), device=DEV)
    return D.kitti_dataload(root, split="train", **kw), D.kitti_dataload(root, split="val", **kw)


def test_config1_kitti_rays_train_and_val(tmp_path, train_math):
    """KITTI-00 rows built on the GPU (nof.dataset) == the fixture's rows; a 4,096-ray batch through
    render_rays_train (64/128, PC-NeRF KITTI settings) and the val split through render_rays_val."""
    sc, g = golden("scene_rays"), golden("config1_kitti")
    tr, va = kitti_scene(tmp_path)
    assert tr.rays.shape[0] == int(sc["kitti_train_total"])
    batch = tr.rays[torch.from_numpy(sc["kitti_train_idx"]).to(DEV)]
    np.testing.assert_array_equal(batch.cpu().numpy(), sc["kitti_train"])
    np.testing.assert_array_equal(va.rays.cpu().numpy(), sc["kitti_val"])
    emb, mc, mf = models(True)
    with torch.no_grad():
        res = R.render_rays_train(mc, mf, emb, batch, sub_nerf_test_num=int(g["sub_nerf_test_num"]), N_samples=64,
                                  N_importance=128, **PCNERF_TRAIN)
    check_train(res, g, batch, mc, mf, name=f"config1_kitti_train_{train_math}", f64=golden("config1_kitti_f64"),
                alt=golden("config1_kitti_alt"))
    emb, mc, mf = models(False)
    with torch.no_grad():
        rv = R.render_rays_val(mc, mf, emb, va.rays, N_samples=64, N_importance=128, perturb=0, noise_std=0,
                               chunk=262144)
    report("config1_kitti_val", max_rel_depth=max_rel(rv["depth"], g["val_depth"]),
           max_rel_depth_fine=max_rel(rv["depth_fine"], g["val_depth_fine"]), rays=va.rays.shape[0])
    close(rv["depth"], g["val_depth"], what="val depth")
    close(rv["depth_fine"], g["val_depth_fine"], what="val depth_fine")


# ----------------------------------------------------------------------------------------------- config 4
def test_config4_maicity_blocks(tmp_path):
    """MaiCity-00 in 4 parent blocks (x split of [-12, 61]): each block's rows built on the GPU (maicity_dataload,
    0406 face rule) == the fixture's; each block rendered with its own coarse/fine weights (128/256)."""
    from test_dataset import M_RD, write_maicity
    from nof import dataset as D
    sc, g = golden("scene_rays"), golden("config4_maicity")
    root, pose_path, _ = write_maicity(str(tmp_path))
    for b in range(4):
        lo, hi = sc[f"maicity_b{b}_lo"], sc[f"maicity_b{b}_hi"]
        ds = D.maicity_dataload(root, split="train", data_start=0, data_end=6, cloud_size_val=16,
                                range_delete_x=M_RD[0], range_delete_y=M_RD[1], range_delete_z=M_RD[2],
                                sub_nerf_test_num=0, surface_expand=0.05, nerf_length_min=float(lo[0]),
                                nerf_length_max=float(hi[0]), nerf_width_min=float(lo[1]), nerf_width_max=float(hi[1]),
                                nerf_height_min=float(lo[2]), nerf_height_max=float(hi[2]), pose_path=pose_path,
                                re_loaddata=1, result_path=str(tmp_path / f"out{b}"), device=DEV)
        assert ds.rays.shape[0] == int(sc[f"maicity_b{b}_total"]), b
        want = sc[f"maicity_b{b}"]
        rays = ds.rays[:want.shape[0]].contiguous()
        np.testing.assert_array_equal(rays.cpu().numpy(), want)
        emb, mc, mf = models(True, SEED_C + b, SEED_F + b)
        with torch.no_grad():
            res = R.render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=int(sc[f"maicity_b{b}_children"]),
                                      N_samples=128, N_importance=256, **PCNERF_TRAIN)
        check_train(res, g, rays, mc, mf, pre=f"b{b}_", name=f"config4_maicity_b{b}",
                    f64=golden("config4_maicity_f64"), alt=golden("config4_maicity_alt"))


# ----------------------------------------------------------------------------------------------- config 5
def test_config5_kitti_blocks_two_step(tmp_path):
    """BASELINE config 5 at its shape on the fixture's one sequence: KITTI-00 frames 1150..1198 as 8 contiguous
    6-frame parent blocks (bench.kitti_view_blocks: each block's own parent cloud and child boxes, eval_kitti_render
    .Scene), the two-step rows of every block's held-out frames at 80 % frame sparsity (eval_kitti_render.py:1060).
    Per block: the rows of its first held-out frame bit for bit against the oracle's row builder (oracle/rays_cpu.py:
    the scan filter, block transform and interest region of eval_kitti_render.py:621-660 on the oracle's float32
    relative poses; child boxes from the same parent cloud), the row table's group structure, and a 256-group slice
    rendered two-step (render.py:614-699) against the oracle on the same rows and weights: effective flags equal,
    depths / points within 1e-4."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import eval_kitti_render as E
    import nof.dataset as D
    from test_dataset import oracle_poses_from
    from oracle import dataset_cpu as OD, ref_cpu as O, rays_cpu as RC
    from nof.render import render_rays_view_0525_2_2
    blocks = bench.kitti_view_blocks(DEV)
    assert [b["block"] for b in blocks] == list(range(8))
    g = golden("kitti_frames_full")
    root, pose_path = bench.write_kitti_fixture(str(tmp_path))
    rd, interest = (2.0, 1.0, 0.5), 20.0
    for kb in blocks:
        ds = bench.C5_START + bench.C5_FRAMES * kb["block"]
        de = ds + bench.C5_FRAMES
        assert kb["frames"] == [ds + k for k in range(1, bench.C5_FRAMES + 1) if (k - 3) % 5 != 0]   # 80 %: 5 of 6
        rows = kb["rows"].cpu().numpy()
        starts = np.nonzero(rows[:, 12] >= -0.5)[0]
        assert kb["groups"] == len(starts) > 1000 and starts[0] == 0
        # a group's head row carries its row count - 1, its continuation rows -1
        assert np.array_equal(np.diff(np.append(starts, len(rows))) - 1, rows[starts, 12].astype(np.int64))
        # the first held-out frame's rows vs the oracle
        f = kb["frames"][0]
        P = oracle_poses_from(g, pose_path, ds)
        positions = np.stack([P[k + 1][:3, 3] for k in range(ds, de)])
        pts = OD.filter_scan(g[f"f{f}"], rd, 0.168, -2.0, strict_range=True)
        w = OD.interest_filter(D.to_block(torch.from_numpy(pts), torch.from_numpy(P[f])).numpy(), positions,
                               interest, interest)
        parent = D.fuse_frames(root, D.relative_poses(D.read_poses(pose_path), ds), ds, de, "cpu", rd, 0.168, -2.0,
                               interest, interest)
        cells = OD.split_children(parent.numpy())
        b6 = np.concatenate([np.stack([a for a, _ in cells]), np.stack([b for _, b in cells])], 1)
        p6 = kb["parent6"].cpu().numpy()
        orows, orng, ooth, _ = RC.build_view_rows(w, P[f][:3, 3].astype(np.float64), b6, p6[:3], p6[3:], 2)
        n0 = orows.shape[0]
        assert kb["children"] == b6.shape[0]
        np.testing.assert_array_equal(rows[:n0], orows, err_msg=f"block {kb['block']} frame {f}")
        np.testing.assert_array_equal(kb["other"][:n0].cpu().numpy(), ooth)
        np.testing.assert_array_equal(kb["ranges"][:n0].cpu().numpy(), orng)
        report(f"config5_kitti_b{kb['block']}_rows", frames=len(kb["frames"]), rows=len(rows), groups=kb["groups"],
               children=kb["children"])
    # two-step render of block 3's first 256 groups vs the oracle (seeded block weights, as the bench)
    kb = blocks[3]
    starts = torch.nonzero(kb["rows"][:, 12] >= -0.5).reshape(-1)
    end = int(starts[256])
    rows, other = kb["rows"][:end], kb["other"][:end]
    seeds = (1234 + 3, 5678 + 3)
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(seeds[0])).to(DEV).eval()
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(seeds[1])).to(DEV).eval()
    Pc, Pf = (O.params_from_numpy(syn.init_nof_params(sd)) for sd in seeds)
    P64 = [{k: (v.double() if v.is_floating_point() else v) for k, v in P.items()} for P in (Pc, Pf)]
    with torch.no_grad():
        res = render_rays_view_0525_2_2(mc, mf, Embedding(3, 10), rows, other, N_samples=128, N_importance=256,
                                        perturb=0, noise_std=0, chunk=262144, depth_inference_method=2)
        ref = O.render_rays_view(Pc, Pf, rows.cpu(), other.cpu(), 128, 256, 262144, method=2)
        f64 = O.render_rays_view(P64[0], P64[1], rows.cpu().double(), other.cpu(), 128, 256, 262144, method=2)
    for k in ("rays_effective_flag", "rays_effective_flag_fine"):
        assert torch.equal(res[k].reshape(-1).cpu().bool(), ref[k].reshape(-1).bool()), k
    for k in ("depth", "points_inference"):
        close(res[k].cpu(), ref[k], what=k)
    # the fine depths go through sample_pdf's fine positions, which one float32 ulp of a coarse weight moves (the
    # train-mode configs' depth_fine, above; here the float32 oracle itself sits up to ~1.4e-4 from the float64
    # evaluation of the same rows and weights): the target is that float64 evaluation, and this path's relative
    # error distribution must be no wider than the float32 oracle's -- quantiles 50 / 90 / 99 / 100 %, 1.5x + 2e-5
    for k in ("depth_fine",):
        eh, er = rel_err(res[k], f64[k].numpy()), rel_err(ref[k], f64[k].numpy())
        for q in (0.5, 0.9, 0.99, 1.0):
            a, b = np.quantile(eh, q), np.quantile(er, q)
            assert a <= 1.5 * b + 2e-5, (k, q, a, b)
    report("config5_kitti_b3_render", rows=end,
           depth_fine_vs_f64_max_rel=max_rel(res["depth_fine"].cpu(), f64["depth_fine"]),
           depth_fine_vs_ref_max_rel=max_rel(res["depth_fine"].cpu(), ref["depth_fine"]),
           ref_vs_f64_max_rel=max_rel(ref["depth_fine"], f64["depth_fine"]))


# ----------------------------------------------------------------------------------------------- config 3
def kitti_scene_full(tmp_path):
    """BASELINE config 3's scene: KITTI-00 scans 1151..1200 (tests/golden/kitti_frames_full.npz, every 16th point)
    at the 50 % frame-sparsity rule (ipb2dmapping.py:647-660: 25 train frames), built on the GPU by nof.dataset."""
    from test_dataset import INTEREST, write_scene
    from nof import dataset as D
    sc = golden("config3_full_scene")
    root, pose_path, _ = write_scene(str(tmp_path), "kitti_frames_full")
    return D.kitti_dataload(root, split="train", data_start=int(sc["data_start"]), data_end=int(sc["data_end"]),
                            cloud_size_val=64, range_delete_x=3, range_delete_y=2, range_delete_z=1.25,
                            sub_nerf_test_num=0, surface_expand=0.05, over_height=0.168, over_low=-2.0,
                            interest_x=INTEREST, interest_y=INTEREST, pose_path=pose_path, re_loaddata=1,
                            result_path=str(tmp_path / "out"), device=DEV, sparsity=int(sc["sparsity"])), sc


def test_config3_training_step_262144_rays(tmp_path):
    """The KITTI training loop's step at 262,144 rays/iter (64/128 samples, chunk 262,144: 64 coarse + 192 fine
    BatchNorm chunks) on BASELINE config 3's scene -- KITTI-00 frames 1151-1200 at 50 % frame sparsity (25 train
    frames, 157,108 rows, 3,362 child cells; tests/golden/make_config3_full.py): the train split rebuilt on the GPU
    by nof.dataset and checked bit for bit against the CPU restatement's (sha256 of all rows, the first 4,096 rows),
    a batch drawn from it with replacement (numpy seed 3).  The first step's forward (depths, child and range losses,
    total, running statistics) against the reference run on the same 262,144 rays (config3_full.npz) with
    check_train's tolerances -- depth_fine against the float64 evaluation and the reference's own spread
    (config3_full_f64.npz, _alt.npz); then three steps of forward, losses, backward, Adam: finite losses that
    decrease on the repeated batch, finite non-zero gradients on both networks, running statistics and parameters
    updated."""
    import hashlib
    tr, sc = kitti_scene_full(tmp_path)
    g3 = golden("config3_full")
    got = tr.rays.cpu().numpy()
    assert got.shape[0] == int(sc["n_rows"])
    np.testing.assert_array_equal(got[:4096], sc["head"])
    assert hashlib.sha256(np.ascontiguousarray(got, dtype=np.float32).tobytes()).hexdigest() == str(sc["sha256"])
    assert int(g3["sub_nerf_test_num"]) == int(sc["children"])
    idx = np.random.default_rng(int(g3["seed"])).integers(0, tr.rays.shape[0], int(g3["n_rays"]))
    rays = tr.rays[torch.from_numpy(idx).to(DEV)].contiguous()
    emb, mc, mf = models(True)
    params = list(mc.parameters()) + list(mf.parameters())
    opt = torch.optim.Adam(params, lr=5e-4, eps=1e-8, weight_decay=1e-3)
    w0 = mc.layer2[6].weight.detach().clone()
    loss_fn = nof_loss["smoothl1"]()
    losses = []
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        res = R.render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=int(g3["sub_nerf_test_num"]), N_samples=64,
                                  N_importance=128, **PCNERF_TRAIN)
        for k in ("depth", "depth_fine"):
            assert torch.isfinite(res[k]).all()
        if not losses:   # the first step's forward against the reference
            check_train({k: v.detach() for k, v in res.items()}, g3, rays, mc, mf, name="config3_full",
                        f64=golden("config3_full_f64"), alt=golden("config3_full_alt"))
        gt = rays[:, 14]
        loss = (1e-1 * loss_fn(1e1 * res["depth"], 1e1 * gt) + 1e-1 * loss_fn(1e1 * res["depth_fine"], 1e1 * gt)
                + 1e6 * (res["child_free_loss"] + res["child_free_loss_fine"])
                + 1e5 * (res["child_depth_loss"] + res["child_depth_loss_fine"]))
        loss.backward()
        for m in (mc, mf):
            g = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
            assert torch.isfinite(g).all() and float(g.abs().max()) > 0
        opt.step()
        losses.append(float(loss))
    assert all(np.isfinite(losses)) and losses[2] < losses[0], losses
    assert int(mc.norms()[0].num_batches_tracked) == 3 * 64 and int(mf.norms()[0].num_batches_tracked) == 3 * 192
    assert not torch.equal(w0, mc.layer2[6].weight.detach())
    report("config3_train_step", loss0=losses[0], loss2=losses[2], rays=rays.shape[0])


# ----------------------------------------------------------------------------------------------- driver trajectory
class RayTable(torch.utils.data.Dataset):
    def __init__(self, rays):
        self.rays, self.ranges = rays, rays[:, 14].clone()

    def __len__(self):
        return self.rays.shape[0]

    def __getitem__(self, index):
        return {'rays': self.rays[index], 'ranges': self.ranges[index]}


def _stress_bn(params: dict, scale: float) -> dict:
    """Shift every BatchNorm's input mean far from zero relative to its spread: the BN shifts (and the Linear
    biases) scaled by ``scale`` make each next layer's pre-BN activations |mean|/std >> 1."""
    out = dict(params)
    for k in out:
        if k.endswith(".bias") and not k.startswith("occ_out"):
            out[k] = (out[k] * scale).astype(np.float32)
    return out


@pytest.mark.parametrize("stress", [1.0, 30.0])
def test_fit_trajectory_vs_oracle(tmp_path, stress):
    """train_kitti.fit(): 6 epochs of one 256-ray batch (64/128 samples, chunk 8192: 2 coarse + 6 fine BatchNorm
    chunks, perturb 0), Adam(lr 5e-4, eps 1e-8, wd 1e-3) + MultiStepLR([5, 120, 256], 0.2) (nof_utils.py:158-173,
    train_kitti.py:108-115) -- the LR drops after epoch 5 -- against the oracle: same batches in the same
    (device randperm) order through oracle autograd + torch.optim.Adam + MultiStepLR.  Losses every step and
    the final parameters (see the comment before the parameter checks for Adam's normalised steps)."""
    import train_kitti as T
    from gradcheck import noise_level_grads
    from nof.nof_utils import get_opts
    from oracle import ref_cpu as O
    n, epochs = 256, 6
    rays_np = syn.make_rays(n, seed=77)
    args = f"""--N_samples 64 --N_importance 128 --perturb 0 --noise_std 0 --chunk 8192 --batch_size {n}
     --num_epochs {epochs} --optimizer adam --lr 5e-4 --weight_decay 1e-3 --decay_gamma 0.2 --use_child_nerf_divide 0
     --use_child_nerf_loss 1 --use_segmentated_sample 1 --segmentated_child_nerf_ratio 0.1 --lambda_loss 1
     --lambda_loss_fine 1 --lambda_child_free_loss 1000000 --lambda_child_depth_loss 100000 --sub_nerf_test_num 32
     --seed 3 --visualize 0 --device cuda"""
    h = get_opts(args.split())
    pc_np = _stress_bn(syn.init_nof_params(SEED_C), stress)
    pf_np = _stress_bn(syn.init_nof_params(SEED_F), stress)
    system = T.NOFSystem(h, train_dataset=RayTable(torch.from_numpy(rays_np).to(DEV)),
                         val_dataset=RayTable(torch.zeros((0, 15), device=DEV)))
    syn.load_into(system.nof_coarse, pc_np)
    syn.load_into(system.nof_fine, pf_np)
    log = str(tmp_path / "log.jsonl")
    T.fit(system, log_path=log)
    hip_losses = [r["train/loss"] for r in map(json.loads, open(log)) if "train/loss" in r]
    assert len(hip_losses) == epochs

    # the oracle, fed the same batches in fit()'s order -- in float32 (the reference's arithmetic) and in float64
    # (the same trajectory evaluated exactly, from the same float32 coarse positions)
    def oracle_fit(f64):
        gen = torch.Generator(device=DEV).manual_seed(int(h.seed))
        Pc, Pf = O.params_from_numpy(pc_np), O.params_from_numpy(pf_np)
        if f64:
            Pc, Pf = ({k: (v.double() if v.is_floating_point() else v) for k, v in P.items()} for P in (Pc, Pf))
        leaves = [P[k].requires_grad_(True) for P in (Pc, Pf) for k in P if k.endswith((".weight", ".bias"))]
        opt = torch.optim.Adam(leaves, lr=5e-4, eps=1e-8, weight_decay=1e-3)
        sched = torch.optim.lr_scheduler.MultiStepLR(opt, milestones=[5, 120, 256], gamma=0.2)
        rays_c = torch.from_numpy(rays_np)
        ref_losses = []
        for _ in range(epochs):
            perm = torch.randperm(n, device=DEV, generator=gen).cpu()
            r = rays_c[perm]
            opt.zero_grad()
            res = O.render_rays_train(Pc, Pf, r, sub_nerf_test_num=32, N_samples=64, N_importance=128, perturb=0,
                                      noise_std=0, chunk=8192, issegmentated=1, childnerf_ratio=0.1,
                                      use_child_nerf_divide=0, use_child_nerf_loss=1, f64=f64)
            rr = r.double() if f64 else r
            lr, lrf = O.range_losses(res["depth"], res["depth_fine"], rr[:, 14])
            loss = O.total_loss(res, lr, lrf)
            loss.backward()
            opt.step()
            sched.step()
            ref_losses.append(float(loss))
        return Pc, Pf, ref_losses

    Pc, Pf, ref_losses = oracle_fit(False)
    Pc64, Pf64, _ = oracle_fit(True)
    np.testing.assert_allclose(hip_losses, ref_losses, rtol=RTOL)
    # Adam normalises every element's step (lr * m / sqrt(v)): an element whose gradient is at rounding-noise level
    # -- the mathematically-zero gradients of noise_level_grads, or single weights with a near-zero gradient --
    # moves by up to ~3 lr per step in a direction set by that noise, in either implementation.  So: every element
    # within Adam's largest possible movement; each tensor's update (final - initial) matching the reference's
    # to 1 % in norm (the trajectory); a running mean follows the
    # bias / previous BN shift feeding its Linear, so it gets that drift through the Linear as tolerance; running
    # variances of the drifted network within 5e-3.  A tensor whose update the reference's own float32 rounding
    # moves by more than 1 % (its float64 trajectory's distance: the occ_out bias under the x30 BatchNorm stress,
    # whose Adam steps nearly cancel, 1.5 %) is held to 1.5 x that distance instead.
    nz = noise_level_grads()
    adam_max = 2 * 3.2 * 5e-4 * epochs
    init = {("c", k): v for k, v in pc_np.items()}
    init.update({("f", k): v for k, v in pf_np.items()})
    worst, worst_nz, worst_rm, worst_rv = 0.0, 0.0, 0.0, 0.0
    for tag, m, P, P64 in (("c", system.nof_coarse, Pc, Pc64), ("f", system.nof_fine, Pf, Pf64)):
        sd = m.state_dict()
        for k, v in sd.items():
            if k.endswith("num_batches_tracked"):
                continue
            got, want = v.cpu().numpy().astype(np.float64), P[k].detach().numpy().astype(np.float64)
            err = got - want
            if k.endswith("running_var"):
                # the statistics of the updated network: its parameters carry the Adam drift described above, and
                # the fine network's statistics the fine-sample spread the reference shows against itself
                # (running stats of the config fixtures move by ~2e-3 between its own thread counts)
                np.testing.assert_allclose(got, want, rtol=5e-3, atol=1e-7, err_msg=tag + k)
                worst_rv = max(worst_rv, float(np.max(np.abs(err) / np.abs(want))))
            elif k.endswith("running_mean"):
                lin = O.LIN[O.BN.index(k[:-len(".running_mean")])]
                w = sd[lin + ".weight"].abs().sum(1).cpu().numpy().astype(np.float64)
                drift = 1.01 * adam_max * (1 + w)
                np.testing.assert_array_less(np.abs(err), 1e-6 * np.abs(want).max() + drift, err_msg=tag + k)
                worst_rm = max(worst_rm, float(np.max(np.abs(err))))
            else:
                np.testing.assert_array_less(np.abs(err), adam_max, err_msg=tag + k)
                if k in nz:
                    worst_nz = max(worst_nz, float(np.max(np.abs(err))))
                    continue
                upd = np.linalg.norm(want - init[(tag, k)].astype(np.float64))
                ratio = float(np.linalg.norm(err) / upd)
                spread = float(np.linalg.norm(want - P64[k].detach().numpy()) / upd)
                assert ratio <= max(1e-2, 1.5 * spread), (tag + k, ratio, spread)
                worst = max(worst, ratio)
    report(f"fit_trajectory_stress{stress:g}", max_update_err_rel_norm=worst, max_noise_param_drift=worst_nz,
           max_running_mean_err=worst_rm, max_running_var_rel=worst_rv,
           loss_rel=max_rel(np.array(hip_losses), np.array(ref_losses)))
