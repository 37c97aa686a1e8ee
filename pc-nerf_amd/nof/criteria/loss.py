"""Range losses -- drop-in for ``nof/criteria/loss.py`` (NOFLoss family, loss.py:7-50).

``forward(pred, target, valid_mask=None)`` returns the mean element loss over the selected elements, computed by
the ``pcnerf_pointwise_loss`` kernel (MSE, L1, SmoothL1 with beta 1; nn.*Loss(reduction='mean') semantics);
differentiable in ``pred`` (``pcnerf_pointwise_loss_backward``) for the training step.
"""
from torch import nn

import torch

from .. import _autograd, _ops

__all__ = ["NOFLoss", "NOFMSELoss", "NOFL1Loss", "NOFSmoothL1Loss"]


class NOFLoss(nn.Module):
    kind = None

    def __init__(self):
        super().__init__()

    def forward(self, pred, target, valid_mask=None):
        if torch.is_grad_enabled() and pred.requires_grad:
            return _autograd.PointwiseLoss.apply(pred, target, self.kind, valid_mask)
        return _ops.pointwise_loss(pred, target, self.kind, valid_mask)


class NOFMSELoss(NOFLoss):
    """Mean squared error between predicted and measured ranges."""
    kind = "mse"


class NOFL1Loss(NOFLoss):
    """Mean absolute error between predicted and measured ranges."""
    kind = "l1"


class NOFSmoothL1Loss(NOFLoss):
    """SmoothL1 (beta 1): squared below 1, absolute above."""
    kind = "smoothl1"
