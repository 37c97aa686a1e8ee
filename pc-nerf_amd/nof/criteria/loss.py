"""Range losses -- drop-in for ``nof/criteria/loss.py`` (NOFLoss family, loss.py:7-50).

``forward(pred, target, valid_mask=None)`` returns the mean element loss over the selected elements, computed by
the ``pcnerf_pointwise_loss`` kernel (MSE, L1, SmoothL1 with beta 1; nn.*Loss(reduction='mean') semantics);
differentiable in ``pred`` (``pcnerf_pointwise_loss_backward``) for the training step.
"""
from torch import nn

import torch

from .. import _autograd, _ops, _torch_ops  # noqa: F401  (_torch_ops registers torch.ops.pcnerf)

__all__ = ["NOFLoss", "NOFMSELoss", "NOFL1Loss", "NOFSmoothL1Loss", "child_range_loss"]


class NOFLoss(nn.Module):
    kind = None

    def __init__(self):
        super().__init__()

    def forward(self, pred, target, valid_mask=None):
        # pcnerf::pointwise_loss: its backward (pcnerf::pointwise_loss_backward) is registered with the operator
        return torch.ops.pcnerf.pointwise_loss(pred, target, self.kind, valid_mask)


class NOFMSELoss(NOFLoss):
    """Mean squared error between predicted and measured ranges."""
    kind = "mse"


class NOFL1Loss(NOFLoss):
    """Mean absolute error between predicted and measured ranges."""
    kind = "l1"


class NOFSmoothL1Loss(NOFLoss):
    """SmoothL1 (beta 1): squared below 1, absolute above."""
    kind = "smoothl1"


def child_range_loss(pred, target, rays, sub_nerf_test_num, lambda_loss=1.0, kind="smoothl1", pre=1e1, post=None):
    """The use_child_nerf_divide == 1 range loss of train_kitti.py:125-142 in one kernel pair instead of a Python
    loop over sub_nerf_test_num children: sum over child ids c = 1..N (ray column 9) that own >= 1 ray of
    ``0.1 * lambda_loss * loss(10 * pred_c, 10 * target_c)`` (mean over the child's rays).  Shape (1,) like the
    reference's ``torch.tensor([0]) + ...`` accumulator; differentiable in ``pred``."""
    post = 1e-1 * lambda_loss if post is None else post
    if torch.is_grad_enabled() and pred.requires_grad:
        return _autograd.ChildRangeLoss.apply(pred, target, rays, int(sub_nerf_test_num), kind, pre, post)
    return _ops.child_range_loss(pred, target, rays, int(sub_nerf_test_num), kind, pre, post)[0]
