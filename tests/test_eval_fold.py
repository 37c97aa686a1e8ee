"""Opt-in exact affine fold of the eval network (every LeakyReLU(True) in nof/networks/models.py
is the identity, so eval-mode NOF(e) = sigmoid(a . e + c)).

CPU: the algebra, restated in float64 numpy from the module's parameters, against the reference's own eval
forward (golden nof_eval, made by importing /root/reference/nof).  GPU: the HIP fold path
(``nof._ops.set_eval_fold(True)``: k_fold_eval + k_nof_eval_fold) against the same goldens and against the full
network.  Tolerances: network output 2e-5 relative (as the full-network test), depths 1e-4 (the north star).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from nof import synthetic as syn

SEED_C, SEED_F = 1234, 5678
RTOL = 1e-4


def fold_np(p):
    """(a, c) with NOF_eval(e) = sigmoid(a . e + c), composed backwards from occ_out (models.py:44-123)."""
    lin, bn = syn.nof_param_names()
    v = p["occ_out.0.weight"][0].astype(np.float64)
    c = float(p["occ_out.0.bias"][0])
    a = np.zeros(63)
    for L in range(7, -1, -1):
        g, b = p[bn[L] + ".weight"].astype(np.float64), p[bn[L] + ".bias"].astype(np.float64)
        rm, rv = p[bn[L] + ".running_mean"].astype(np.float64), p[bn[L] + ".running_var"].astype(np.float64)
        alpha = g / np.sqrt(rv + 1e-5)
        beta = b - rm * alpha
        W, bl = p[lin[L] + ".weight"].astype(np.float64), p[lin[L] + ".bias"].astype(np.float64)
        c += float(v @ (alpha * bl + beta))
        va = v * alpha
        if L == 0:
            a += va @ W
        elif L == 4:
            a += va @ W[:, :63]
            v = va @ W[:, 63:]
        else:
            v = va @ W
    return a, c


def test_fold_algebra_vs_reference_eval_forward():
    g = golden("nof_eval")
    a, c = fold_np(syn.init_nof_params(SEED_C))
    p = 1.0 / (1.0 + np.exp(-(g["embedding"].astype(np.float64) @ a + c)))
    np.testing.assert_allclose(p, g["p"][:, 0], rtol=2e-5, atol=1e-7)


@pytest.fixture
def fold_on():
    from nof import _ops
    prev = _ops.set_eval_fold(True)
    yield
    _ops.set_eval_fold(prev)


def _models():
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(SEED_C)).cuda().eval()
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(SEED_F)).cuda().eval()
    return Embedding(3, 10), mc, mf


def _close(a, b, rtol, atol, what):
    np.testing.assert_allclose(a.detach().cpu().numpy().astype(np.float64), np.asarray(b, np.float64), rtol=rtol,
                               atol=atol, err_msg=what)


@pytest.mark.gpu
def test_fold_coefficients_on_gpu(fold_on):
    from nof import _ops
    _, mc, _ = _models()
    f = _ops.fold_eval(mc, torch.device("cuda")).cpu().numpy()
    a, c = fold_np(syn.init_nof_params(SEED_C))
    np.testing.assert_allclose(f[:63], a, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(f[63], c, rtol=1e-9)


@pytest.mark.gpu
def test_fold_nof_forward(fold_on):
    g = golden("nof_eval")
    _, mc, _ = _models()
    with torch.no_grad():
        p = mc(torch.from_numpy(g["embedding"]).cuda())
    _close(p, g["p"], 2e-5, 1e-7, "p eval (fold)")


@pytest.mark.gpu
@pytest.mark.parametrize("S", [64, 128])
def test_fold_render_val(fold_on, S):
    from nof import render as R
    g = golden(f"render_val_s{S}")
    emb, mc, mf = _models()
    with torch.no_grad():
        res = R.render_rays_val(mc, mf, emb, torch.from_numpy(g["rays"]).cuda(), N_samples=S,
                                N_importance=int(g["N_importance"]), perturb=0, noise_std=0, chunk=int(g["chunk"]))
    _close(res["depth"], g["depth"], RTOL, 1e-6, "depth (fold)")
    _close(res["depth_fine"], g["depth_fine"], RTOL, 1e-6, "depth_fine (fold)")


@pytest.mark.gpu
@pytest.mark.parametrize("method", [0, 2])
def test_fold_render_view(fold_on, method):
    from nof import render as R
    g = golden(f"render_view_m{method}")
    emb, mc, mf = _models()
    with torch.no_grad():
        res = R.render_rays_view_0525_2_2(mc, mf, emb, torch.from_numpy(g["rows"]).cuda(),
                                          torch.from_numpy(g["other"]).cuda(), N_samples=int(g["N_samples"]),
                                          N_importance=int(g["N_importance"]), perturb=0, noise_std=0, chunk=4096,
                                          depth_inference_method=method)
    for k in ("depth", "depth_fine", "points_inference", "points_inference_fine"):
        _close(res[k], g[k], RTOL, 1e-6, k + " (fold)")
    for k in ("rays_effective_flag", "rays_effective_flag_fine"):
        assert np.array_equal(res[k].cpu().numpy(), g[k]), k


@pytest.mark.gpu
def test_fold_matches_full_network_config2():
    from nof import _ops, render as R
    emb, mc, mf = _models()
    rays = torch.from_numpy(syn.make_rays(2048, seed=3)).cuda()
    kw = dict(N_samples=128, N_importance=256, perturb=0, noise_std=0, chunk=262144)
    with torch.no_grad():
        prev = _ops.set_eval_fold(False)
        full = R.render_rays_val(mc, mf, emb, rays, **kw)
        _ops.set_eval_fold(True)
        fold = R.render_rays_val(mc, mf, emb, rays, **kw)
        _ops.set_eval_fold(prev)
    for k in ("depth", "depth_fine"):
        _close(fold[k], full[k].cpu().numpy(), RTOL, 1e-6, k)
