"""PC-NeRF LiDAR volume rendering -- drop-in for ``nof/render.py`` of the reference, on MI355X HIP kernels.

Same function names, signatures, result keys, shapes and dtypes as the reference.  Each stage is a kernel of
lib/libpcnerf_hip.so (see include/pcnerf_hip.h):

    coarse z sampling (+segmented merge)  pcnerf_sample_coarse      render.py:429-442
    stratified perturbation               pcnerf_perturb            render.py:449-454
    Embedding + NOF query (chunked BN)    pcnerf_nof_query_*        render.py:18-25 / 44-51, models.py
    compositing, child masks, loss terms  pcnerf_composite          render.py:51-61, 75-159
    sample_pdf + sort(cat(z, samples))    pcnerf_resample           render.py:371-412, 463-467
    child loss reductions                 pcnerf_child_loss_reduce  render.py:102-159

Differences from the reference, all deliberate:
  * everything stays on ``rays.device`` (the reference pins ``u`` to ``cuda:0``, render.py:397);
  * RNG: draws are taken from torch's generator on the device, and only when used (the reference also draws
    ``randn`` noise when ``noise_std == 0``).  Parity tests inject the draws with the keyword-only ``rng``
    dict: ``perturb_rand`` (R,S), ``noise`` (R,S), ``u`` (R,I), ``noise_fine`` (R,S+I);
  * gradients: ``render_rays_train`` is differentiable (train-mode networks): with autograd enabled and
    parameters requiring grad, each pass runs as ``nof._autograd.TrainPass`` whose backward is the HIP
    compositing backward + the NOF backward (chunks recomputed), so ``loss.backward()`` of train_kitti.py:155
    fills ``.grad`` of both networks.  The inference renderers stay forward-only (they raise under autograd).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _autograd, _ops
from . import _torch_ops
from .networks import NOF, Embedding, NOF_coarse, NOF_fine, NOF_plusfine  # noqa: F401  (reference exports)

__all__ = ['render_rays']

EPSILON = 1e-10  # render.py:456, :514, :656
# the tensor-level stages go through the registered operators (nof._torch_ops): torch's dispatcher, FakeTensor
# tracing and torch.compile see them as graph nodes
P = torch.ops.pcnerf


def _query(model, rays, z, chunk):
    """The NOF query of one pass: eval mode through pcnerf::pack_eval + pcnerf::query_eval (the module's tensors
    are operator inputs); train mode and the opt-in eval fold through nof._ops.query (module-level state: BatchNorm
    running statistics, chunk moments)."""
    if not model.training and not _ops.eval_fold_enabled():
        _ops._bn_config(model)
        return P.query_eval(rays, z, P.pack_eval(_torch_ops.eval_params(model)))
    return _ops.query(model, rays, z, chunk)


def _check_inputs(model, model_fine, embedding_xy, rays, n_cols, differentiable=False):
    if not rays.is_cuda:
        raise RuntimeError("nof.render (HIP) renders device-resident rays; move them with rays.to('cuda') -- there "
                           "is no CPU path")
    if rays.dim() != 2 or rays.shape[1] < n_cols:
        raise RuntimeError(f"rays must be (N_rays, >={n_cols}); got {tuple(rays.shape)}")
    if embedding_xy is not None and not embedding_xy.supported():
        raise NotImplementedError("HIP render supports Embedding(3, 10) (L_pos = 10)")
    for m in (model, model_fine):
        if not m.supported():
            raise NotImplementedError("HIP render supports NOF(feature_size=256, in_channels_xy=63, use_skip=True)")
        if _autograd.needs_grad(m):
            if not differentiable:
                raise NotImplementedError("this HIP renderer is forward-only (inference); call it under "
                                          "torch.no_grad()")
            _autograd.check_trainable(m)
    return rays.float().contiguous()


def _draw(rng, key, shape, device, fn):
    if rng is not None and key in rng:
        t = rng[key]
        return t.to(device=device, dtype=torch.float32).contiguous()
    return fn(shape, device=device)


def _coarse(rays, N_samples, segmented, ratio, perturb, rng):
    """render.py:429-454."""
    R = rays.shape[0]
    n_parent = int(N_samples * (1 - ratio)) if segmented else N_samples
    z = P.sample_coarse(rays, N_samples, n_parent, 6, 7, 10, 11, False)
    if perturb > 0:
        z = P.perturb(z, float(perturb), _draw(rng, "perturb_rand", (R, N_samples), rays.device, torch.rand))
    return z


def _noise(rng, key, z, noise_std):
    if noise_std == 0:
        return None
    return _draw(rng, key, tuple(z.shape), z.device, torch.randn)


def sample_pdf(bins, weights, N_samples, det=False, pytest=False, *, u=None):
    """render.py:371-412: inverse-CDF samples, unsorted, ``bins`` (R, B), ``weights`` (R, B-1) -> (R, N).
    ``u`` (keyword-only) injects the uniform draws when ``det`` is False.

    ``pytest=True`` is the reference's test hook (render.py:386-394): ``np.random.seed(0)`` (numpy's global
    generator, as the reference seeds it), then ``u`` = float32 of ``np.linspace(0, 1, N)`` (det) or of
    ``np.random.rand(R, N)``; the draws are made on the host and uploaded, the sampling itself runs on the device.
    With ``det`` False the reference first draws (and discards) ``torch.rand`` from torch's CPU generator
    (render.py:383); that draw is made here too, so torch's global RNG state afterwards is the reference's."""
    if pytest:
        R = bins.shape[0]
        if not det:   # render.py:383 draws u from torch's CPU generator before the numpy overwrite: consume it too
            torch.rand((R, N_samples))
        np.random.seed(0)
        if det:
            hu = np.broadcast_to(np.linspace(0., 1., N_samples), (R, N_samples))
        else:
            hu = np.random.rand(R, N_samples)
        u = torch.from_numpy(np.ascontiguousarray(hu, dtype=np.float32)).to(bins.device)
        det = False   # the uploaded draws are used as given (the linspace is numpy's, float64 rounded to float32)
    return P.sample_pdf(bins, weights, int(N_samples), bool(det), u)


def render_rays_train(model: NOF, model_fine: NOF, embedding_xy: Embedding, rays: torch.Tensor, sub_nerf_test_num=4,
                      N_samples=64, N_importance=128, use_disp=False, perturb=0, noise_std=1, chunk=1024 * 3,
                      isval=False, issegmentated=0, childnerf_ratio=0.5, use_child_nerf_divide=0,
                      use_child_nerf_loss=0, *, rng=None):
    """render.py:416-482 -> {'child_free_loss_fine', 'child_depth_loss_fine', 'depth_fine', 'child_free_loss',
    'child_depth_loss', 'depth'}."""
    rays = _check_inputs(model, model_fine, embedding_xy, rays, 15, differentiable=True)
    R = rays.shape[0]
    z = _coarse(rays, N_samples, issegmentated, childnerf_ratio, perturb, rng)
    with_losses = use_child_nerf_loss == 1

    def one_pass(m, z, noise_key):
        if _autograd.needs_grad(m):
            noise = _noise(rng, noise_key, z, noise_std)
            sub = int(sub_nerf_test_num) if use_child_nerf_divide == 1 else 0
            w, depth, free, dl = _autograd.TrainPass.apply(m, rays, z, noise, float(noise_std), EPSILON, int(chunk),
                                                           with_losses, sub, *_ops.grad_params(m))
            if not with_losses:
                free, dl = torch.tensor(0.0), torch.tensor(0.0)
            return w, depth, free, dl
        p = _query(m, rays, z, chunk)
        w, depth, fr, sl = P.composite(p, z, _noise(rng, noise_key, z, noise_std), float(noise_std), EPSILON,
                                       rays if with_losses else None, 10, 11, 14, True)
        if with_losses:
            free, dl = P.child_losses(fr, sl, rays, use_child_nerf_divide == 1, int(sub_nerf_test_num))
        else:
            free, dl = torch.tensor(0.0), torch.tensor(0.0)   # render.py:123-125, 157-159 (CPU scalars)
        return w, depth, free, dl

    w, depth, free, dl = one_pass(model, z, "noise")
    u = None if perturb == 0 else _draw(rng, "u", (R, N_importance), rays.device, torch.rand)
    zf = P.resample(z, w, int(N_importance), u)
    _, depth_f, free_f, dl_f = one_pass(model_fine, zf, "noise_fine")
    return {'child_free_loss_fine': free_f, 'child_depth_loss_fine': dl_f, "depth_fine": depth_f,
            'child_free_loss': free, 'child_depth_loss': dl, 'depth': depth}


def render_rays_val(model: NOF, model_fine: NOF, embedding_xy: Embedding, rays: torch.Tensor, sub_nerf_test_num=4,
                    N_samples=64, N_importance=128, use_disp=False, perturb=0, noise_std=1, chunk=1024 * 3,
                    isval=False, *, rng=None):
    """render.py:485-536 -> {'depth_fine', 'depth'}."""
    rays = _check_inputs(model, model_fine, embedding_xy, rays, 8)
    R = rays.shape[0]
    z = _coarse(rays, N_samples, False, 0.0, perturb, rng)
    p = _query(model, rays, z, chunk)
    w, depth, _, _ = P.composite(p, z, _noise(rng, "noise", z, noise_std), float(noise_std), EPSILON, None, 10, 11,
                                 14, True)
    u = None if perturb == 0 else _draw(rng, "u", (R, N_importance), rays.device, torch.rand)
    zf = P.resample(z, w, int(N_importance), u)
    pf = _query(model_fine, rays, zf, chunk)
    _, depth_f, _, _ = P.composite(pf, zf, _noise(rng, "noise_fine", zf, noise_std), float(noise_std), EPSILON,
                                   None, 10, 11, 14, False)
    return {"depth_fine": depth_f, 'depth': depth}


def render_rays(model: NOF, model_fine: NOF, embedding_xy: Embedding, rays: torch.Tensor, N_samples=64,
                N_importance=128, use_disp=False, perturb=0, noise_std=1, chunk=1024 * 3, isval=False, *, rng=None):
    """render.py:538-611 (the generic NOF renderer, exported in the reference's __all__).  Reproduces the
    reference's call ``inference(..., chunk, noise_std, isval)``, which lands ``isval`` in inference's
    ``epsilon`` slot: weights are always normalised, by sum(w) + float(isval).  Returns {'depth_fine',
    'weights', 'opacity', 'z_vals', 'depth', 'depth2', 'opacity_fine'}; depth2 is the z at the position where
    the last sample falls in the descending weight order (render.py:598-600; ties broken stably)."""
    rays = _check_inputs(model, model_fine, embedding_xy, rays, 8)
    R = rays.shape[0]
    z = P.sample_coarse(rays, N_samples, N_samples, 6, 7, 0, 0, bool(use_disp))
    if perturb > 0:
        z = P.perturb(z, float(perturb), _draw(rng, "perturb_rand", (R, N_samples), rays.device, torch.rand))
    eps = float(isval)
    p = _query(model, rays, z, chunk)
    w, depth, opac, _ = P.composite_extras(p, z, _noise(rng, "noise", z, noise_std), float(noise_std), eps)
    u = None if perturb == 0 else _draw(rng, "u", (R, N_importance), rays.device, torch.rand)
    zf = P.resample(z, w, int(N_importance), u)
    pf = _query(model_fine, rays, zf, chunk)
    wf, depth_f, opac_f, depth2 = P.composite_extras(pf, zf, _noise(rng, "noise_fine", zf, noise_std),
                                                     float(noise_std), eps)
    return {'depth_fine': depth_f, 'weights': wf, 'opacity': opac, 'z_vals': zf, "depth": depth, "depth2": depth2,
            "opacity_fine": opac_f}


def _inference_view(model, rays, z, other, chunk, method):
    """inference_0525_2 (render.py:229-368) on the HIP kernels: query, per-row compositing / peak / child sums,
    then the ray-group walk."""
    p = _query(model, rays, z, chunk)
    w, depth, at_peak, csum, opac_row, pts = P.view_rows(p, z, rays, int(method), EPSILON)
    flags, opacity = P.view_walk(other, at_peak, csum, opac_row, int(z.shape[1]))
    return depth, w, opacity, flags, pts


def render_rays_view_0525_2_2(model: NOF, model_fine: NOF, embedding_xy: Embedding, rays: torch.Tensor,
                              other_interest_sub_nerf_number: torch.Tensor, N_samples=64, N_importance=128,
                              use_disp=False, perturb=0, noise_std=1, chunk=1024 * 3, isval=False,
                              depth_inference_method=0, *, rng=None):
    """render.py:614-699: two-step inference on 13-column rows grouped per ray.  Returns {'depth_fine', 'weights',
    'opacity', 'z_vals', 'depth', 'opacity_fine', 'points_inference_fine', 'points_inference',
    'rays_effective_flag', 'rays_effective_flag_fine'} (the reference's debug prints are not reproduced)."""
    rays = _check_inputs(model, model_fine, embedding_xy, rays, 11)
    other = other_interest_sub_nerf_number
    if not torch.is_tensor(other):
        other = torch.as_tensor(other)
    other = other.to(rays.device)
    R = rays.shape[0]
    z = P.sample_coarse(rays, N_samples, N_samples, 9, 10, 0, 0, False)   # parent bounds, render.py:622-628
    if perturb > 0:
        z = P.perturb(z, float(perturb), _draw(rng, "perturb_rand", (R, N_samples), rays.device, torch.rand))
    method = int(depth_inference_method)
    depth, w, opacity, flags, pts = _inference_view(model, rays, z, other, chunk, method)
    u = None if perturb == 0 else _draw(rng, "u", (R, N_importance), rays.device, torch.rand)
    zf = P.resample(z, w, int(N_importance), u)
    depth_f, wf, opacity_f, flags_f, pts_f = _inference_view(model_fine, rays, zf, other, chunk, method)
    return {'depth_fine': depth_f, 'weights': wf, 'opacity': opacity, 'z_vals': zf, "depth": depth,
            "opacity_fine": opacity_f, "points_inference_fine": pts_f, "points_inference": pts,
            "rays_effective_flag": flags, "rays_effective_flag_fine": flags_f}
