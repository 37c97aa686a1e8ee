"""Autograd bindings of the training path: loss.backward() of the reference's training step
(train_kitti.py:117-155, returned to Lightning) through the HIP kernels.

Two torch.autograd.Functions, each owning one forward kernel chain and its hand-written backward:
  * TrainPass -- one render pass of render_rays_train (render.py:38-163, 416-482): train-mode query + compositing
    + child losses.  Outputs (weights [non-differentiable], depth, child_free_loss, child_depth_loss); backward =
    pcnerf_composite_backward (dL/dlogit) -> pcnerf_nof_query_train_backward (parameter gradients, chunks
    recomputed).  The fine samples are detached from the coarse weights exactly as render.py:466 does.
  * NofForward -- NOF.forward on an embedded batch in train mode (models.py:183-203).
Gradients flow to the 34 trainable tensors of the network; inputs (rays, positions) get none, as in the
reference where they never require grad.
"""
from __future__ import annotations

import torch

from . import _ops


class TrainPass(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, rays, z, noise, noise_std, eps, chunk, with_losses, sub_num, *params):
        # a chunk larger than the pass is the same single BatchNorm chunk: size workspaces and store by the pass
        chunk = max(1, min(int(chunk), z.numel()))
        ctx.store = ctx.fold = ctx.state = None
        if _ops.train_fold_enabled():   # opt-in exact affine fold: per-chunk moments + layer maps, no activations
            ctx.fold = _ops.fold_state(z.device, z.numel(), chunk)
            p = _ops.query(model, rays, z, chunk, fold=ctx.fold)
        elif _ops.remat_enabled():
            # default: no activations kept -- the fused query's state (moments + layer maps, ~3 MB per chunk) only;
            # the backward rematerialises every layer input from the encoding
            ctx.state = _ops.fold_state(z.device, z.numel(), chunk)
            p = _ops.query(model, rays, z, chunk, keep=ctx.state)
        else:
            # keep the chunks' layer outputs for the backward in the HBM left after its workspace (+ 4 GiB margin)
            L = _ops.H.lib()
            reserve = int(L.pcnerf_nof_backward_workspace_bytes(int(chunk))) + (4 << 30)
            ctx.store = _ops.ActivationStore(z.device, z.numel(), chunk, reserve)
            p = _ops.query(model, rays, z, chunk, ctx.store)
        w, depth, fr, sl = _ops.composite(p, z, noise, noise_std, eps, rays if with_losses else None)
        if with_losses:
            free, dl = _ops.child_losses(fr, sl, rays, sub_num > 0, sub_num)
        else:
            free = dl = torch.zeros((), dtype=torch.float32, device=z.device)
        ctx.model, ctx.noise_std, ctx.eps, ctx.chunk = model, noise_std, eps, chunk
        ctx.with_losses, ctx.sub_num = with_losses, sub_num
        ctx.save_for_backward(rays, z, p, noise)
        ctx.mark_non_differentiable(w)
        return w, depth, free, dl

    @staticmethod
    def backward(ctx, g_w, g_depth, g_free, g_dl):
        rays, z, p, noise = ctx.saved_tensors
        if not ctx.with_losses:
            g_free = g_dl = None
        g_logit = _ops.composite_backward(p, z, noise, ctx.noise_std, ctx.eps, rays if ctx.with_losses else None,
                                          ctx.sub_num, g_depth, g_free, g_dl)
        if ctx.fold is not None:
            grads = _ops.nof_query_backward_fold(ctx.model, rays, z, ctx.chunk, g_logit, ctx.fold)
            ctx.fold = None
        elif ctx.state is not None:
            grads = _ops.nof_query_backward_remat(ctx.model, rays, z, ctx.chunk, g_logit, ctx.state)
            ctx.state = None
        else:
            grads = _ops.nof_query_backward(ctx.model, rays, z, ctx.chunk, g_logit, ctx.store)
            ctx.store.release()
        return (None,) * 9 + tuple(grads)


class NofForward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, x, *params):
        p, ctx.fold = _ops.nof_forward_embedded(model, x, with_fold_state=True)
        ctx.model = model
        ctx.save_for_backward(x, p)
        return p

    @staticmethod
    def backward(ctx, g_p):
        x, p = ctx.saved_tensors
        if ctx.fold is not None:
            grads = _ops.nof_forward_backward_fold(ctx.model, x, p.reshape(-1), g_p.contiguous().reshape(-1),
                                                   ctx.fold)
            ctx.fold = None
        else:
            grads = _ops.nof_forward_backward(ctx.model, x, p.reshape(-1), g_p.contiguous().reshape(-1))
        return (None, None) + tuple(grads)


class ChildRangeLoss(torch.autograd.Function):
    """Per-child range loss of train_kitti.py:125-142 (divide branch) with d/dpred."""

    @staticmethod
    def forward(ctx, pred, target, rays, sub_num, kind, pre, post):
        out, ws = _ops.child_range_loss(pred, target, rays, sub_num, kind, pre, post)
        ctx.args = (sub_num, kind, pre, post)
        ctx.save_for_backward(pred, target, rays, ws)
        return out

    @staticmethod
    def backward(ctx, g):
        pred, target, rays, ws = ctx.saved_tensors
        gp = _ops.child_range_loss_backward(pred, target, rays, *ctx.args, ws, g.contiguous())
        return (gp.reshape(pred.shape),) + (None,) * 6


def needs_grad(model) -> bool:
    return torch.is_grad_enabled() and any(t.requires_grad for t in model.parameters())


def check_trainable(model) -> None:
    if not model.training:
        raise NotImplementedError("gradients through the HIP NOF kernels are implemented for train-mode BatchNorm "
                                  "(the reference trains with model.train()); call model.train() or use no_grad")
