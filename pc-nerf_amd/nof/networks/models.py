"""NOF occupancy networks and positional encoding -- drop-in for ``nof/networks/models.py`` of the reference.

The module layout (and therefore every state_dict key) is the reference's: ``layer1`` is a Sequential of
Linear / BatchNorm1d / LeakyReLU(True) triples for the first four layers followed by four more LeakyReLU(True)
(the reference appends the second block's activations to ``layer1``, models.py:72,92), ``layer2`` holds
Linear / BatchNorm1d pairs (the skip input is [x, layer1(x)], 63 + 256 wide), ``occ_out`` is Linear + Sigmoid.
``LeakyReLU(True)`` sets ``negative_slope = True == 1``: an identity.  Checkpoints written by the reference
(``nof_utils.load_ckpt``) therefore load unchanged.

Compute: ``forward`` does not run the PyTorch layers.  It hands the parameters to the HIP kernels
(``pcnerf_nof_query_*``), which evaluate the same network on MFMA: eval mode with BatchNorm folded into each
Linear, train mode with batch statistics over the whole call (one chunk) and running-stat updates, exactly
like ``nn.BatchNorm1d``.  The render functions in ``nof.render`` call the kernels directly on sample positions
(encoding fused), so they never materialise the 63-wide embedding.
"""
from __future__ import annotations

import torch
from torch import nn

from .. import _autograd, _ops


class Embedding(nn.Module):
    """models.py:4-41: x -> (x, sin(2^k x), cos(2^k x), ...) for k < N_freq (log scale) -- 63 channels for
    in_channels=3, N_freq=10.  The HIP kernels implement exactly this configuration."""

    def __init__(self, in_channels, N_freq, logscale=True):
        super().__init__()
        self.N_freq = N_freq
        self.in_channels = in_channels
        self.funcs = [torch.sin, torch.cos]
        if logscale:
            self.freq_bands = 2 ** torch.linspace(0, N_freq - 1, N_freq)
        else:
            self.freq_bands = torch.linspace(1, 3 ** (N_freq - 1), N_freq)
        self.logscale = logscale

    def supported(self) -> bool:
        return self.in_channels == 3 and self.N_freq == 10 and self.logscale

    def forward(self, x):
        if not self.supported():
            raise NotImplementedError("HIP Embedding supports in_channels=3, N_freq=10, logscale=True "
                                      "(the configuration of every reference script)")
        return _ops.embed(x)


class _NOFBase(nn.Module):
    """Shared body of NOF / NOF_coarse / NOF_fine / NOF_plusfine (models.py:44-359 are four identical copies)."""

    def __init__(self, feature_size=256, in_channels_xy=63, use_skip=True):
        super().__init__()
        self.feature_size = feature_size
        self.in_channels_xy = in_channels_xy
        self.use_skip = use_skip
        first = []
        for i in range(4):
            first += [nn.Linear(in_channels_xy if i == 0 else feature_size, feature_size),
                      nn.BatchNorm1d(feature_size), nn.LeakyReLU(True)]
        second = []
        for i in range(4):
            fan_in = (in_channels_xy + feature_size if use_skip else feature_size) if i == 0 else feature_size
            second += [nn.Linear(fan_in, feature_size), nn.BatchNorm1d(feature_size)]
            first.append(nn.LeakyReLU(True))   # models.py:92: the second block's activations land in layer1
        self.layer1 = nn.Sequential(*first)
        self.layer2 = nn.Sequential(*second)
        self.occ_out = nn.Sequential(nn.Linear(feature_size, 1), nn.Sigmoid())

    # ------------------------------------------------------------------ kernel plumbing
    def supported(self) -> bool:
        # the kernels evaluate every LeakyReLU(True) as the identity it is (negative_slope = True = 1); a module
        # whose activations were changed is not this network
        slopes_one = all(m.negative_slope == 1.0 for m in self.modules() if isinstance(m, nn.LeakyReLU))
        return self.feature_size == 256 and self.in_channels_xy == 63 and self.use_skip and slopes_one

    def linears(self):
        return [self.layer1[i] for i in (0, 3, 6, 9)] + [self.layer2[i] for i in (0, 2, 4, 6)]

    def norms(self):
        return [self.layer1[i] for i in (1, 4, 7, 10)] + [self.layer2[i] for i in (1, 3, 5, 7)]

    def forward(self, x):
        """x: (B, 63) embedded positions -> (B, 1) occupancy probability (models.py:183-203)."""
        if not self.supported():
            raise NotImplementedError("HIP NOF kernels support feature_size=256, in_channels_xy=63, use_skip=True")
        if _autograd.needs_grad(self):
            _autograd.check_trainable(self)
            return _autograd.NofForward.apply(self, x, *_ops.grad_params(self))
        return _ops.nof_forward_embedded(self, x)


class NOF(_NOFBase):
    pass


class NOF_coarse(_NOFBase):
    pass


class NOF_fine(_NOFBase):
    pass


class NOF_plusfine(_NOFBase):
    pass
