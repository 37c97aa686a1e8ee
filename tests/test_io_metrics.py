"""On-disk formats (nof/io.py) and the metrics oracle, on CPU.

The metrics oracle (oracle/metrics_cpu.py) is pinned by the reference's committed rendered/source PCDs: its
per-version averages over the test frames (tests/golden/metrics_reference.json, made by make_golden.gen_metrics)
are the values SURVEY.md records from print_metrics.py's logic, e.g. KITTI PC-NeRF two-step CD 0.2239 m (the
paper's figure value)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN as GOLDEN_DIR, golden
from nof import io as nio
from nof.networks import NOF_coarse, NOF_fine
from nof import synthetic as syn

REF = "/root/reference"

# SURVEY.md section 6 (perf/quality baselines): AvgErr m, Acc %, CD m, F
RECORDED = {"kitti/version_1/two_step": (0.488, 66.65, 0.2239, 0.891),
            "kitti/version_0/two_step": (0.511, 65.23, 0.2201, 0.890),
            "maicity/version_1/two_step": (None, None, 0.1718, 0.956),
            "maicity/version_0/two_step": (None, None, 0.2973, 0.923),
            "kitti/version_1/one_step": (None, None, 1.62, None),
            "kitti/version_0/one_step": (None, None, 3.55, None)}


def test_metrics_oracle_reproduces_recorded_values():
    with open(os.path.join(GOLDEN_DIR, "metrics_reference.json")) as fh:
        ref = json.load(fh)
    for key, vals in RECORDED.items():
        got = ref[key]["mean"]
        for g, v in zip(got, vals):
            if v is not None:
                # within one unit of the last digit SURVEY.md printed
                assert abs(g - v) <= 1.01 * 10 ** -(len(str(v).split(".")[1])), (key, got, vals)


def test_metrics_oracle_on_fixture_frame():
    from oracle import metrics_cpu as M
    g = golden("metrics_frame")
    got = M.frame_metrics(g["pred"], g["gt"], g["origin"], 0.2)
    np.testing.assert_allclose(got, g["expected"], rtol=1e-12)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference data not present")
def test_read_pcd_reference_files():
    g = golden("metrics_frame")
    base = os.path.join(REF, "logs/kitti00/1151_1200_view/render_result")
    np.testing.assert_array_equal(nio.read_pcd(f"{base}/source/1153_source.pcd"), g["gt"])
    np.testing.assert_array_equal(nio.read_pcd(f"{base}/infer/version_1_1153_two_step.pcd"), g["pred"])
    np.testing.assert_array_equal(nio.read_pcd(f"{base}/source/1153_pose.pcd").reshape(-1), g["origin"])
    pts = nio.read_pcd(os.path.join(REF, "data/kitti/00/pcd_remove_dynamic/1151.pcd"))
    assert pts.ndim == 2 and pts.shape[1] == 3 and pts.shape[0] > 1000 and np.isfinite(pts).all()


def test_pcd_roundtrip_binary_and_ascii(tmp_path):
    rng = np.random.default_rng(0)
    pts = rng.normal(size=(1234, 3)).astype(np.float32)
    p = str(tmp_path / "a.pcd")
    nio.write_pcd(p, pts)
    np.testing.assert_array_equal(nio.read_pcd(p), pts)
    q = str(tmp_path / "b.pcd")
    with open(q, "w") as fh:
        fh.write("# .PCD v0.7\nVERSION 0.7\nFIELDS x y z intensity\nSIZE 4 4 4 4\nTYPE F F F F\nCOUNT 1 1 1 1\n"
                 f"WIDTH {len(pts)}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {len(pts)}\nDATA ascii\n")
        for r in pts:
            fh.write(f"{float(r[0])!r} {float(r[1])!r} {float(r[2])!r} 7\n")
    np.testing.assert_array_equal(nio.read_pcd(q), pts)


def test_ray_cache_roundtrip(tmp_path):
    rays = syn.make_rays(300, seed=3)
    nio.save_rays(str(tmp_path), rays, split="train")
    r, rg = nio.load_rays(str(tmp_path), "train")
    np.testing.assert_array_equal(r, rays)
    np.testing.assert_array_equal(rg[:, 0], rays[:, 14])
    rows = np.zeros((5, 13), np.float32)
    nio.save_view_rows(str(tmp_path / "v"), rows, [1, 0, 2, 0, 0], np.arange(5), [1, 0, 1, 1, 0])
    rw, other, rng_, tin = nio.load_view_rows(str(tmp_path / "v"))
    assert rw.shape == (5, 13) and other.tolist() == [1, 0, 2, 0, 0] and tin.tolist() == [1, 0, 1, 1, 0]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference data not present")
def test_reference_two_step_side_files_load():
    d = os.path.join(REF, "logs/kitti00/1151_1200_view/two_step/1153pcd/childnerf_ray_intersect")
    other = np.load(os.path.join(d, "other_interest_sub_nerf_number_child.npy"), allow_pickle=False).reshape(-1)
    # group structure of the committed rows: first row of a group holds k-1, the rest 0 (a2)
    i, n = 0, len(other)
    while i < n:
        k = int(other[i]) + 1
        assert k >= 1 and (other[i + 1:i + k] == 0).all()
        i += k
    assert i == n


def test_lightning_ckpt_roundtrip(tmp_path):
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(1))
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(2))
    p = str(tmp_path / "last.ckpt")
    nio.save_ckpt(p, nof_coarse=mc, nof_fine=mf)
    a, b = NOF_coarse(), NOF_fine()
    nio.load_ckpt(a, p, model_name="nof_coarse")    # train_kitti.py:35-36
    nio.load_ckpt(b, p, model_name="nof_fine")
    for x, y in ((a, mc), (b, mf)):
        for (k, v), (k2, v2) in zip(x.state_dict().items(), y.state_dict().items()):
            assert k == k2 and torch.equal(v, v2)
    sd = nio.extract_model_state_dict(p, "nof_coarse", prefixes_to_ignore=["occ_out"])
    assert not any(k.startswith("occ_out") for k in sd) and "layer1.0.weight" in sd


def _lightning_like_ckpt(path, mc, mf, hparams_kind):
    """A checkpoint with the top-level keys and value types a Lightning (1.x/2.x) ModelCheckpoint writes for the
    reference's NOFSystem (Lightning itself is not importable here): hyper_parameters from save_hyperparameters(
    argparse.Namespace) -- a Namespace, or Lightning's AttributeDict (a dict subclass living in a Lightning module:
    emulated by a class registered under that module path while saving) --, Adam + MultiStepLR states (a Counter
    of milestones), ModelCheckpoint callback state, loops, version."""
    import argparse
    import collections
    import sys
    import types
    hp = dict(N_samples=768, N_importance=1536, lr=5e-4, decay_step=[2], use_skip=True, ckpt_path=None,
              exp_name="kitti00/1151_1200_view")
    saved_mod = None
    if hparams_kind == "namespace":
        hyper = argparse.Namespace(**hp)
    else:
        names = ("pytorch_lightning", "pytorch_lightning.utilities", "pytorch_lightning.utilities.parsing")
        saved_mod = {n: sys.modules.get(n) for n in names}
        mods = [types.ModuleType(n) for n in names]
        AttributeDict = type("AttributeDict", (dict,), {"__module__": names[-1]})
        mods[-1].AttributeDict = AttributeDict
        mods[0].utilities, mods[1].parsing = mods[1], mods[2]
        for m in mods:
            sys.modules[m.__name__] = m
        hyper = AttributeDict(hp)
    sd = {f"nof_coarse.{k}": v for k, v in mc.state_dict().items()}
    sd.update({f"nof_fine.{k}": v for k, v in mf.state_dict().items()})
    params = list(mc.parameters()) + list(mf.parameters())
    opt = torch.optim.Adam(params, lr=5e-4, eps=1e-8, weight_decay=1e-3)
    for p in params:
        p.grad = torch.ones_like(p)
    opt.step()
    sched = torch.optim.lr_scheduler.MultiStepLR(opt, milestones=[5, 120, 256], gamma=0.2)
    ck = {"epoch": 3, "global_step": 15759, "pytorch-lightning_version": "1.9.0", "state_dict": sd,
          "loops": {"fit_loop": {"state_dict": {}, "epoch_progress": {"total": {"ready": 4, "completed": 3}}}},
          "callbacks": {"ModelCheckpoint{'monitor': 'train/loss', 'mode': 'min'}": {
              "monitor": "train/loss", "best_model_score": torch.tensor(0.42), "best_model_path": "/x/best.ckpt",
              "best_k_models": {"/x/a.ckpt": torch.tensor(0.5)}, "last_model_path": "/x/last.ckpt"}},
          "optimizer_states": [opt.state_dict()], "lr_schedulers": [sched.state_dict()],
          "hparams_name": "hparams", "hyper_parameters": hyper}
    assert isinstance(ck["lr_schedulers"][0]["milestones"], collections.Counter)
    try:
        torch.save(ck, path)
    finally:
        if hparams_kind != "namespace":
            for n, m in saved_mod.items():
                if m is None:
                    del sys.modules[n]
                else:
                    sys.modules[n] = m


@pytest.mark.parametrize("hparams_kind", ["namespace", "attributedict"])
def test_lightning_full_checkpoint_loads_weights_only(tmp_path, hparams_kind):
    """load_ckpt on a full Lightning-layout checkpoint: the plain weights_only load refuses the Namespace /
    AttributeDict globals, the loader retries with those data containers allowed (still weights_only: nothing in
    the file executes) and reads the nof_coarse. / nof_fine. weights."""
    import pickle
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(3))
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(4))
    p = str(tmp_path / "epoch=3.ckpt")
    _lightning_like_ckpt(p, mc, mf, hparams_kind)
    with pytest.raises(pickle.UnpicklingError):
        torch.load(p, map_location="cpu", weights_only=True)
    a, b = NOF_coarse(), NOF_fine()
    nio.load_ckpt(a, p, model_name="nof_coarse")
    nio.load_ckpt(b, p, model_name="nof_fine")
    for x, y in ((a, mc), (b, mf)):
        for (k, v), (k2, v2) in zip(x.state_dict().items(), y.state_dict().items()):
            assert k == k2 and torch.equal(v, v2)
    ck = nio.load_checkpoint(p)
    assert ck["hyper_parameters"]["N_samples"] if hparams_kind != "namespace" else ck["hyper_parameters"].N_samples
