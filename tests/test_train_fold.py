"""Opt-in exact affine fold of the TRAIN-mode network (nof._ops.set_train_fold; csrc/nof_fold.hip).

Within one BatchNorm chunk the reference NOF (nof/networks/models.py:183-203, identity activations:
models.py:72,152,232) is sigmoid(a_c . e + c_c), with every layer's batch statistics exact functions of the chunk's
encoding mean and covariance.  Pinned three ways:
  CPU: the float64 numpy restatement (train_fold_np.py: forward, running stats and the hand-derived backward the
       kernels implement) against torch float64 autograd of the layer-by-layer network (1e-9), and against the
       reference's own train-mode forward (golden nof_train: p 2e-5, running stats 1e-4);
  GPU: the HIP fold against that restatement on the same fp32 encodings (p 1e-6, gradients 1e-6 of each tensor's
       largest entry), and end to end with the fold switched on: the render / gradient / full-size config-2
       parity tests of the default path, at their tolerances (depths 1e-4, gradients 2e-4).
"""
import numpy as np
import pytest
import torch

import train_fold_np as TF
from conftest import golden
from nof import synthetic as syn
from oracle import ref_cpu as O

SEED_C = 1234


def _torch_params(seed):
    P = {k: torch.from_numpy(np.array(v, dtype=np.float64)) for k, v in syn.init_nof_params(seed).items()}
    for k in P:
        if k.endswith(".weight") or k.endswith(".bias"):
            P[k].requires_grad_(True)
    return P


def test_fold_algebra_matches_layerwise_network_float64():
    """Forward, running-stat update and every parameter gradient of one chunk, fold vs torch float64 autograd."""
    torch.manual_seed(2)
    x = (torch.rand(700, 3, dtype=torch.float64) * 30 - 15)
    e = O.embed(x.float()).double()
    wgt = torch.randn(700, dtype=torch.float64)
    P = _torch_params(SEED_C)
    p_ref = O.nof_forward(P, e, True)[:, 0]
    (p_ref * wgt).sum().backward()

    params = syn.init_nof_params(SEED_C)
    a, c, st = TF.fold_forward(params, e.numpy())
    logit = e.numpy() @ a + c
    p = 1.0 / (1.0 + np.exp(-logit))
    np.testing.assert_allclose(p, p_ref.detach().numpy(), rtol=1e-9, atol=1e-12)

    TF.running_update(params, st)
    lin, bn = syn.nof_param_names()
    for b in bn:
        for k in (".running_mean", ".running_var"):
            np.testing.assert_allclose(params[b + k], P[b + k].numpy().astype(np.float32), rtol=1e-6, atol=1e-7)

    g = TF.fold_backward(params, e.numpy(), wgt.numpy() * p * (1 - p), st)
    zero = {b + ".bias" for b in lin} | {b + ".bias" for b in bn[:7]}
    gamma_scale = np.abs(P[bn[0] + ".weight"].grad.numpy()).max()
    for k, t in P.items():
        if t.grad is None:
            continue
        ref = t.grad.numpy()
        if k in zero:   # mathematically zero (the next BatchNorm removes the mean): autograd's float64 noise only
            assert np.abs(ref).max() <= 1e-9 * gamma_scale and np.abs(g[k]).max() == 0.0, k
            continue
        scale = max(np.abs(ref).max(), 1e-30)
        np.testing.assert_allclose(g[k].reshape(ref.shape), ref, rtol=1e-8, atol=1e-9 * scale, err_msg=k)


def test_fold_algebra_vs_reference_train_forward():
    """The reference's own train-mode NOF forward over chunks (golden nof_train): p and running stats."""
    g = golden("nof_train")
    e = O.embed(torch.from_numpy(g["points"])).double().numpy()
    c = int(g["chunk"])
    params = syn.init_nof_params(SEED_C)
    ps = []
    for i in range(0, len(e), c):
        a, cc, st = TF.fold_forward(params, e[i:i + c])
        ps.append(1.0 / (1.0 + np.exp(-(e[i:i + c] @ a + cc))))
        TF.running_update(params, st)
    np.testing.assert_allclose(np.concatenate(ps), g["p"][:, 0], rtol=2e-5, atol=1e-7)
    _, bn = syn.nof_param_names()
    run = np.stack([np.stack([params[b + ".running_mean"], params[b + ".running_var"]]) for b in bn])
    np.testing.assert_allclose(run, g["running"], rtol=1e-4, atol=1e-7)


# ----------------------------------------------------------------------------------------------- GPU
DEV = "cuda"


@pytest.fixture
def fold_on():
    from nof import _ops
    prev = _ops.set_train_fold(True)
    yield "fold"
    _ops.set_train_fold(prev)


def _model(seed=SEED_C):
    from nof.networks import NOF_coarse
    return syn.load_into(NOF_coarse(), syn.init_nof_params(seed)).to(DEV).train(True)


@pytest.mark.gpu
@pytest.mark.parametrize("n,chunk", [(4096, 1000), (3000, 3000), (70000, 65536)])
def test_fold_gpu_matches_restatement(n, chunk, fold_on):
    """NOF.forward(emb) in train mode through the HIP fold, chunk by chunk (ragged last chunk; 64-sample tiles
    past the chunk end), vs the float64 restatement on the same fp32 encodings: p, running stats, gradients."""
    from nof.networks import Embedding
    torch.manual_seed(4)
    x = (torch.rand(n, 3) * 30 - 15).to(DEV)
    e = Embedding(3, 10)(x)
    wgt = torch.randn(n, device=DEV)
    m = _model()
    params = syn.init_nof_params(SEED_C)
    en = e.double().cpu().numpy()
    for i in range(0, n, chunk):   # one BatchNorm chunk per call; gradients compared per chunk (no fp32 .grad sums)
        m.zero_grad(set_to_none=True)
        pg = m(e[i:i + chunk])[:, 0]
        (pg * wgt[i:i + chunk]).sum().backward()
        a, c, st = TF.fold_forward(params, en[i:i + chunk])
        pc = 1.0 / (1.0 + np.exp(-(en[i:i + chunk] @ a + c)))
        np.testing.assert_allclose(pg.detach().cpu().numpy(), pc, rtol=1e-6, atol=1e-9)
        # dL/dlogit as the kernels form it from the fp32 p (g (1 - p) p): a sum over mixed-sign terms amplifies
        # the last bits of p, so the restatement takes the same fp32 values
        pd = pg.detach()
        gl = (wgt[i:i + chunk] * (1.0 - pd) * pd).double().cpu().numpy()
        grads = TF.fold_backward(params, en[i:i + chunk], gl, st)
        for k, t in m.named_parameters():
            ref = np.asarray(grads[k]).reshape(t.shape)
            scale = max(float(np.abs(ref).max()), 1e-30)
            np.testing.assert_allclose(t.grad.cpu().numpy(), ref, rtol=1e-5, atol=1e-6 * scale, err_msg=k)
        TF.running_update(params, st)
    _, bn = syn.nof_param_names()
    for b in bn:
        for k in (".running_mean", ".running_var"):
            np.testing.assert_allclose(dict(m.named_buffers())[b + k].cpu().numpy(), params[b + k], rtol=1e-6,
                                       atol=1e-7, err_msg=b + k)


@pytest.mark.gpu
def test_fold_nof_train_golden(fold_on):
    import test_parity_gpu as PG
    PG.test_nof_train_forward_chunks_and_running_stats(fold_on)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["original", "pcnerf", "pcnerf_divide", "pcnerf_perturb"])
def test_fold_render_train_golden(name, fold_on):
    import test_parity_gpu as PG
    PG.test_render_train(name, fold_on)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["pcnerf", "divide", "original"])
def test_fold_train_grads_vs_reference(name, fold_on):
    import test_backward_gpu as BG
    BG.test_train_grads_vs_reference(name, fold_on)


@pytest.mark.gpu
@pytest.mark.parametrize("divide,noise_std", [(0, 0.0), (1, 1e-3)])
def test_fold_train_grads_vs_oracle_ragged_chunks(divide, noise_std, monkeypatch, fold_on):
    import test_backward_gpu as BG
    BG.test_train_grads_vs_oracle_ragged_chunks_with_draws(divide, noise_std, "all", monkeypatch, fold_on)


@pytest.mark.gpu
def test_fold_nof_forward_backward_embedded(fold_on):
    import test_backward_gpu as BG
    BG.test_nof_forward_backward_embedded()


@pytest.mark.gpu
def test_fold_grad_accumulates_and_running_stats_once(fold_on):
    import test_backward_gpu as BG
    BG.test_grad_accumulates_and_running_stats_once()


@pytest.mark.gpu
def test_fold_config2_full_size_vs_reference(fold_on):
    """65,536 rays x (128 + 384) samples, chunks of 262,144 (32 coarse + 96 fine folds), vs the reference and the
    float64 evaluation (depth_fine within 1e-4 of it for every ray)."""
    import test_configs_gpu as CG
    CG.test_config2_full_size_vs_reference(fold_on)
