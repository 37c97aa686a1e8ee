"""Pin the CPU oracle (oracle/ref_cpu.py) against golden vectors made by importing the reference."""
import numpy as np
import pytest
import torch

from conftest import golden
from gradcheck import check_grads
from nof import synthetic as syn
from oracle import ref_cpu as O

SEED_C, SEED_F = 1234, 5678
torch.set_num_threads(1)  # goldens were made single-threaded: keep reduction orders identical


def P(seed):
    return O.params_from_numpy(syn.init_nof_params(seed))


def close(a, b, rtol=1e-6, atol=1e-7):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def running(Pm):
    return np.stack([np.stack([Pm[b + ".running_mean"].numpy(), Pm[b + ".running_var"].numpy()]) for b in O.BN])


def test_embedding_and_nof_eval():
    g = golden("nof_eval")
    x = torch.from_numpy(g["points"])
    e = O.embed(x)
    close(e, g["embedding"], 0, 0)
    close(O.nof_forward(P(SEED_C), e, False), g["p"])


def test_nof_train_chunks_and_running_stats():
    g = golden("nof_train")
    Pm = P(SEED_C)
    x = torch.from_numpy(g["points"])
    c = int(g["chunk"])
    p = torch.cat([O.nof_forward(Pm, O.embed(x[i:i + c]), True) for i in range(0, len(x), c)])
    close(p, g["p"])
    close(running(Pm), g["running"])


def test_sample_pdf():
    g = golden("sample_pdf")
    b, w = torch.from_numpy(g["bins"]), torch.from_numpy(g["weights"])
    close(O.sample_pdf(b, w, 96, det=True), g["samples_det"], 0, 0)
    close(O.sample_pdf(b, w, 96, det=False, u=torch.from_numpy(g["u"])), g["samples_rand"], 0, 0)


@pytest.mark.parametrize("S", [64, 128])
def test_render_val(S):
    g = golden(f"render_val_s{S}")
    res = O.render_rays_val(P(SEED_C), P(SEED_F), torch.from_numpy(g["rays"]), N_samples=S,
                            N_importance=int(g["N_importance"]), perturb=0, noise_std=0, chunk=int(g["chunk"]))
    close(res["depth"], g["depth"])
    close(res["depth_fine"], g["depth_fine"])


TRAIN = ["pcnerf", "pcnerf_noseg", "pcnerf_divide", "original", "pcnerf_perturb", "pcnerf_s128"]


@pytest.mark.parametrize("name", TRAIN)
def test_render_train(name):
    g = golden(f"render_train_{name}")
    rays = torch.from_numpy(g["rays"])
    Pc, Pf = P(SEED_C), P(SEED_F)
    draws = {k: torch.from_numpy(g[k]) for k in ("perturb_rand", "u") if k in g}
    res = O.render_rays_train(Pc, Pf, rays, sub_nerf_test_num=int(g["sub_nerf_test_num"]),
                              N_samples=int(g["N_samples"]), N_importance=int(g["N_importance"]),
                              perturb=int(g["perturb"]), noise_std=0, chunk=int(g["chunk"]),
                              issegmentated=int(g["issegmentated"]), childnerf_ratio=float(g["childnerf_ratio"]),
                              use_child_nerf_divide=int(g["use_child_nerf_divide"]),
                              use_child_nerf_loss=int(g["use_child_nerf_loss"]), draws=draws)
    for k in ("depth", "depth_fine", "child_free_loss", "child_depth_loss", "child_free_loss_fine",
              "child_depth_loss_fine"):
        close(res[k], g[k], 1e-5, 1e-9)
    lr, lrf = O.range_losses(res["depth"], res["depth_fine"], rays[:, 14], rays,
                             int(g["use_child_nerf_divide"]), int(g["sub_nerf_test_num"]))
    close(lr, g["loss_range"], 1e-5)
    close(lrf, g["loss_range_fine"], 1e-5)
    close(O.total_loss(res, lr, lrf), g["loss_total"], 1e-5)
    close(running(Pc), g["running_c"])
    close(running(Pf), g["running_f"])


@pytest.mark.parametrize("method", [0, 2])
def test_render_view(method):
    g = golden(f"render_view_m{method}")
    res = O.render_rays_view(P(SEED_C), P(SEED_F), torch.from_numpy(g["rows"]), torch.from_numpy(g["other"]),
                             N_samples=int(g["N_samples"]), N_importance=int(g["N_importance"]), chunk=4096,
                             method=method)
    for k in ("depth", "depth_fine", "weights", "z_vals", "opacity", "opacity_fine", "points_inference",
              "points_inference_fine"):
        close(res[k], g[k], 1e-5, 1e-9)
    for k in ("rays_effective_flag", "rays_effective_flag_fine"):
        assert np.array_equal(res[k].numpy(), g[k])


@pytest.mark.parametrize("isval", [0, 1])
def test_render_rays(isval):
    g = golden(f"render_rays_isval{isval}")
    res = O.render_rays(P(SEED_C), P(SEED_F), torch.from_numpy(g["rays"]), N_samples=int(g["N_samples"]),
                        N_importance=int(g["N_importance"]), perturb=0, noise_std=0, chunk=4096, isval=bool(isval))
    for k in ("depth", "depth_fine", "weights", "z_vals", "depth2", "opacity", "opacity_fine"):
        close(res[k], g[k], 1e-5, 1e-9)


def grad_leaves(Pm):
    keys = [k for k in Pm if k.endswith(".weight") or k.endswith(".bias")]
    for k in keys:
        Pm[k].requires_grad_(True)
    return keys


@pytest.mark.parametrize("name", ["pcnerf", "divide", "original"])
def test_train_grads(name):
    """loss.backward() of train_kitti.py:117-155 through render_rays_train: oracle autograd == reference."""
    g = golden(f"grads_{name}")
    Pc, Pf = P(SEED_C), P(SEED_F)
    kc, kf = grad_leaves(Pc), grad_leaves(Pf)
    rays = torch.from_numpy(g["rays"])
    div = int(g["use_child_nerf_divide"])
    res = O.render_rays_train(Pc, Pf, rays, sub_nerf_test_num=32, N_samples=64, N_importance=128, perturb=0,
                              noise_std=0, chunk=4096, issegmentated=int(g["issegmentated"]), childnerf_ratio=0.1,
                              use_child_nerf_divide=div, use_child_nerf_loss=int(g["use_child_nerf_loss"]))
    lr, lrf = O.range_losses(res["depth"], res["depth_fine"], rays[:, 14], rays, div, 32)
    tot = O.total_loss(res, lr, lrf)
    close(tot.detach().reshape(-1), g["loss_total"].reshape(-1), 1e-6, 0)
    tot.sum().backward()
    check_grads(lambda k: Pc[k].grad.numpy(), kc, g, "c:", 1e-5)
    check_grads(lambda k: Pf[k].grad.numpy(), kf, g, "f:", 1e-5)


def test_sample_pdf_pytest_hook():
    """render.py:386-394 (pytest=True): np.random.seed(0) draws, det (numpy linspace) and random."""
    g = golden("sample_pdf_pytest")
    b, w = torch.from_numpy(g["bins"]), torch.from_numpy(g["weights"])
    R, n = b.shape[0], 96
    np.random.seed(0)
    u_det = torch.from_numpy(np.broadcast_to(np.linspace(0., 1., n), (R, n)).astype(np.float32))
    close(O.sample_pdf(b, w, n, det=False, u=u_det), g["samples_det"], 0, 0)
    np.random.seed(0)
    u_rnd = torch.from_numpy(np.random.rand(R, n).astype(np.float32))
    close(O.sample_pdf(b, w, n, det=False, u=u_rnd), g["samples_rand"], 0, 0)


PCNERF_TRAIN = dict(use_child_nerf_loss=1, issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0, perturb=0,
                    noise_std=0, chunk=262144)


def check_train(res, g, rays, Pc, Pf, pre=""):
    for k in ("depth", "depth_fine", "child_free_loss", "child_depth_loss", "child_free_loss_fine",
              "child_depth_loss_fine"):
        close(res[k], g[pre + k], 1e-5, 1e-9)
    lr, lrf = O.range_losses(res["depth"], res["depth_fine"], rays[:, 14])
    close(lr, g[pre + "loss_range"], 1e-5)
    close(lrf, g[pre + "loss_range_fine"], 1e-5)
    close(O.total_loss(res, lr, lrf), g[pre + "loss_total"], 1e-5)
    close(running(Pc), g[pre + "running_c"], 1e-5)
    close(running(Pf), g[pre + "running_f"], 1e-5)


def test_config1_kitti():
    """Config 1: KITTI-00 4,096-ray batch (64/128, one 262,144-sample coarse chunk) and the val split (eval)."""
    sc, g = golden("scene_rays"), golden("config1_kitti")
    rays = torch.from_numpy(sc["kitti_train"])
    Pc, Pf = P(SEED_C), P(SEED_F)
    res = O.render_rays_train(Pc, Pf, rays, sub_nerf_test_num=int(g["sub_nerf_test_num"]), N_samples=64,
                              N_importance=128, **PCNERF_TRAIN)
    check_train(res, g, rays, Pc, Pf)
    rv = O.render_rays_val(P(SEED_C), P(SEED_F), torch.from_numpy(sc["kitti_val"]), N_samples=64, N_importance=128,
                           perturb=0, noise_std=0, chunk=262144)
    close(rv["depth"], g["val_depth"], 1e-5, 1e-9)
    close(rv["depth_fine"], g["val_depth_fine"], 1e-5, 1e-9)


@pytest.mark.parametrize("b", [0, 1, 2, 3])
def test_config4_maicity_block(b):
    """Config 4: MaiCity-00 parent block b with its own coarse/fine weights (128/256 samples)."""
    sc, g = golden("scene_rays"), golden("config4_maicity")
    rays = torch.from_numpy(sc[f"maicity_b{b}"])
    Pc, Pf = P(SEED_C + b), P(SEED_F + b)
    res = O.render_rays_train(Pc, Pf, rays, sub_nerf_test_num=int(sc[f"maicity_b{b}_children"]), N_samples=128,
                              N_importance=256, **PCNERF_TRAIN)
    check_train(res, g, rays, Pc, Pf, pre=f"b{b}_")
