"""The render path's C-ABI entries as PyTorch custom operators (``torch.ops.pcnerf.*``).

Each operator is a ``torch.library.custom_op`` whose implementation is the ctypes launcher in ``nof._ops`` (the
``extern "C"`` kernels of lib/libpcnerf_hip.so, enqueued on the current HIP stream), with a fake (meta)
implementation giving the output shapes and dtypes, so torch's dispatcher, FakeTensor tracing and ``torch.compile``
see the path as graph nodes instead of opaque Python.  The loss operator carries its backward through
``register_autograd``.  ``nof.render`` calls the tensor-level stages through these operators; the stages that take a
whole ``nn.Module`` (the train-mode queries and their backward, ``nof._autograd``) stay autograd Functions, since an
operator schema holds tensors, not modules -- the eval query is an operator on the packed weight image instead.

Reference boundary replaced: render.py:416 (render_rays_train), :485 (render_rays_val), :614
(render_rays_view_0525_2_2) and their helpers -- same arguments, the operators are an implementation layer below.
"""
from typing import Optional

import torch
from torch import Tensor

from . import _hip as H
from . import _ops

NS = "pcnerf"
_PACKED = []


def _packed_floats() -> int:
    if not _PACKED:
        _PACKED.append(int(H.lib().pcnerf_nof_eval_packed_floats()))
    return _PACKED[0]


def _need(op: str, name: str, t: Optional[Tensor], shape: tuple, dtype=torch.float32) -> None:
    """Host-side check of one operand against the layout its kernel's grid and reads assume: a contiguous ``dtype``
    device tensor of ``shape`` (None: any size, ``('min', k)``: at least k)."""
    if t is None:
        return
    H.require_device(t)
    if t.dtype != dtype or not t.is_contiguous():
        raise RuntimeError(f"pcnerf::{op}: {name} must be a contiguous {dtype} device tensor")
    ok = t.dim() == len(shape)
    for have, want in zip(t.shape, shape):
        if want is None:
            continue
        if isinstance(want, tuple):
            ok = ok and have >= want[1]
        else:
            ok = ok and have == want
    if not ok:
        raise RuntimeError(f"pcnerf::{op}: {name} has shape {tuple(t.shape)}, expected {shape}")


# ----------------------------------------------------------------------------------------------- embedding
@torch.library.custom_op(f"{NS}::embed", mutates_args=())
def embed(x: Tensor) -> Tensor:
    """Embedding(3, 10) (models.py:27-41)."""
    return _ops.embed(x)


@embed.register_fake
def _(x):
    return x.new_empty((*x.shape[:-1], 63), dtype=torch.float32)


# ----------------------------------------------------------------------------------------------- sampling
@torch.library.custom_op(f"{NS}::sample_coarse", mutates_args=())
def sample_coarse(rays: Tensor, n_samples: int, n_parent: int, near_col: int, far_col: int, cn_col: int,
                  cf_col: int, disparity: bool) -> Tensor:
    """Coarse z (render.py:429-442; the segmented merge when n_parent < n_samples)."""
    _need("sample_coarse", "rays", rays, (None, None))
    return _ops.sample_coarse(rays, n_samples, n_parent, near_col, far_col, cn_col, cf_col, disparity)


@sample_coarse.register_fake
def _(rays, n_samples, n_parent, near_col, far_col, cn_col, cf_col, disparity):
    return rays.new_empty((rays.shape[0], n_samples), dtype=torch.float32)


@torch.library.custom_op(f"{NS}::perturb", mutates_args=())
def perturb(z: Tensor, amount: float, rand: Tensor) -> Tensor:
    """Stratified perturbation (render.py:449-454)."""
    _need("perturb", "z", z, (None, None))
    _need("perturb", "rand", rand, tuple(z.shape))
    return _ops.perturb(z, amount, rand)


@perturb.register_fake
def _(z, amount, rand):
    return torch.empty_like(z)


@torch.library.custom_op(f"{NS}::resample", mutates_args=())
def resample(z: Tensor, w: Tensor, n_importance: int, u: Optional[Tensor]) -> Tensor:
    """sample_pdf + sort(cat(z, samples)) (render.py:371-412, 463-467)."""
    _need("resample", "z", z, (None, None))
    _need("resample", "w", w, tuple(z.shape))
    return _ops.resample(z, w, n_importance, u)


@resample.register_fake
def _(z, w, n_importance, u):
    return z.new_empty((z.shape[0], z.shape[1] + n_importance), dtype=torch.float32)


@torch.library.custom_op(f"{NS}::sample_pdf", mutates_args=())
def sample_pdf(bins: Tensor, weights: Tensor, n_samples: int, det: bool, u: Optional[Tensor]) -> Tensor:
    """sample_pdf (render.py:371-412), unsorted draws."""
    return _ops.sample_pdf_standalone(bins, weights, n_samples, det, u)


@sample_pdf.register_fake
def _(bins, weights, n_samples, det, u):
    return bins.new_empty((bins.shape[0], n_samples), dtype=torch.float32)


# ----------------------------------------------------------------------------------------------- network (eval)
# pcnerf_nof_params' tensor shapes (models.py: 4 + 4 Linear/BatchNorm1d layers of 256, the skip layer's input
# [x, h_3] 63 + 256 wide, occ_out 256 -> 1): the kernels index them at these sizes, so the operator checks them
_LIN_IN = (63, 256, 256, 256, 319, 256, 256, 256)


def _param_shapes() -> list:
    return ([(256, k) for k in _LIN_IN] + [(256,)] * 40 + [(1, 256), (1,)])


def _check_query(rays: Tensor, z: Tensor, packed: Tensor) -> None:
    """The host-side checks before pcnerf_nof_query_eval's launch: its grid and reads assume these layouts."""
    H.require_device(rays, z, packed)
    for name, t in (("rays", rays), ("z", z), ("packed", packed)):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError(f"pcnerf::query_eval: {name} must be a contiguous float32 device tensor")
    if z.dim() != 2 or rays.dim() != 2 or rays.shape[0] != z.shape[0] or rays.shape[1] < 6:
        raise RuntimeError(f"pcnerf::query_eval: rays (R, >=6) and z (R, S) expected, got {tuple(rays.shape)} and "
                           f"{tuple(z.shape)}")
    if packed.numel() != _packed_floats():
        raise RuntimeError(f"pcnerf::query_eval: packed must be pcnerf::pack_eval's image ({_packed_floats()} floats), "
                           f"got {packed.numel()}")
    if not (rays.device == z.device == packed.device):
        raise RuntimeError("pcnerf::query_eval: rays, z and packed must be on one device")


@torch.library.custom_op(f"{NS}::pack_eval", mutates_args=())
def pack_eval(params: list[Tensor]) -> Tensor:
    """The eval network image (BatchNorm folded, MFMA operand order) from the module's 50 tensors in
    pcnerf_nof_params order: lin_w[8], lin_b[8], bn_w[8], bn_b[8], bn_rm[8], bn_rv[8], out_w, out_b."""
    if len(params) != 50:
        raise RuntimeError(f"pcnerf::pack_eval takes 50 parameter tensors, got {len(params)}")
    s = H.NofParams()
    for i, (t, shp) in enumerate(zip(params, _param_shapes())):
        H.require_device(t)
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError("NOF parameters must be contiguous float32 device tensors")
        if tuple(t.shape) != shp:
            raise RuntimeError(f"pcnerf::pack_eval: parameter {i} has shape {tuple(t.shape)}, expected {shp} "
                               "(NOF(feature_size=256, in_channels_xy=63, use_skip=True))")
    for i in range(8):
        s.lin_w[i], s.lin_b[i] = params[i].data_ptr(), params[8 + i].data_ptr()
        s.bn_w[i], s.bn_b[i] = params[16 + i].data_ptr(), params[24 + i].data_ptr()
        s.bn_rm[i], s.bn_rv[i] = params[32 + i].data_ptr(), params[40 + i].data_ptr()
    s.out_w, s.out_b = params[48].data_ptr(), params[49].data_ptr()
    import ctypes
    out = torch.empty(_packed_floats(), dtype=torch.float32, device=params[0].device)
    H.check(H.lib().pcnerf_nof_pack_eval(ctypes.byref(s), out.data_ptr(), H.stream_of(out)))
    return out


@pack_eval.register_fake
def _(params):
    return params[0].new_empty((_packed_floats(),), dtype=torch.float32)


def eval_params(model) -> list:
    """A NOF module's tensors in pcnerf::pack_eval's order."""
    lins, norms = model.linears(), model.norms()
    return ([l.weight for l in lins] + [l.bias for l in lins] + [b.weight for b in norms] + [b.bias for b in norms]
            + [b.running_mean for b in norms] + [b.running_var for b in norms]
            + [model.occ_out[0].weight, model.occ_out[0].bias])


@torch.library.custom_op(f"{NS}::query_eval", mutates_args=())
def query_eval(rays: Tensor, z: Tensor, packed: Tensor) -> Tensor:
    """Eval-mode occupancy p (R, S) of o + d z through Embedding + NOF (render.py:18-25, models.py:183-203)."""
    _check_query(rays, z, packed)
    R, S = z.shape
    p = torch.empty((R, S), dtype=torch.float32, device=z.device)
    H.check(H.lib().pcnerf_nof_query_eval(rays.data_ptr(), R, rays.shape[1], z.data_ptr(), S, packed.data_ptr(),
                                          p.data_ptr(), H.stream_of(z)))
    return p


@query_eval.register_fake
def _(rays, z, packed):
    return torch.empty_like(z)


# ----------------------------------------------------------------------------------------------- compositing
@torch.library.custom_op(f"{NS}::composite", mutates_args=())
def composite(p: Tensor, z: Tensor, noise: Optional[Tensor], noise_std: float, eps: float, rays: Optional[Tensor],
              cn_col: int, cf_col: int, range_col: int, want_weights: bool) -> tuple[Tensor, Tensor, Tensor, Tensor]:
    """(weights (R,S) or (0,), depth (R,), free_ray (R,) or (0,), sl1_ray (R,) or (0,)): render.py:51-61, 75-159."""
    _need("composite", "z", z, (None, None))
    _need("composite", "p", p, tuple(z.shape))
    _need("composite", "rays", rays, (z.shape[0], None))
    w, d, fr, sl = _ops.composite(p, z, noise, noise_std, eps, rays, cn_col, cf_col, range_col, want_weights)
    e = z.new_empty((0,))
    return (w if w is not None else e), d, (fr if fr is not None else e.clone()), (sl if sl is not None else e.clone())


@composite.register_fake
def _(p, z, noise, noise_std, eps, rays, cn_col, cf_col, range_col, want_weights):
    R, S = z.shape
    w = z.new_empty((R, S) if want_weights else (0,))
    r = (R,) if rays is not None else (0,)
    return w, z.new_empty((R,)), z.new_empty(r), z.new_empty(r)


@torch.library.custom_op(f"{NS}::composite_extras", mutates_args=())
def composite_extras(p: Tensor, z: Tensor, noise: Optional[Tensor], noise_std: float,
                     eps: float) -> tuple[Tensor, Tensor, Tensor, Tensor]:
    """render_rays's compositing (render.py:538-611): (weights, depth, opacity mean (), depth2 (R,))."""
    _need("composite_extras", "z", z, (None, None))
    _need("composite_extras", "p", p, tuple(z.shape))
    w, d, _, _, om, d2 = _ops.composite(p, z, noise, noise_std, eps, extras=True)
    return w, d, om, d2


@composite_extras.register_fake
def _(p, z, noise, noise_std, eps):
    R, S = z.shape
    return z.new_empty((R, S)), z.new_empty((R,)), z.new_empty(()), z.new_empty((R,))


@torch.library.custom_op(f"{NS}::child_losses", mutates_args=())
def child_losses(free_ray: Tensor, sl1_ray: Tensor, rays: Tensor, divide: bool,
                 sub_nerf_test_num: int) -> tuple[Tensor, Tensor]:
    """(child_free_loss, child_depth_loss): (1,) each in the divide branch, () otherwise (render.py:102-159)."""
    _need("child_losses", "free_ray", free_ray, (None,))
    _need("child_losses", "sl1_ray", sl1_ray, tuple(free_ray.shape))
    _need("child_losses", "rays", rays, (free_ray.shape[0], ("min", 10)))
    a, b = _ops.child_losses(free_ray, sl1_ray, rays, divide, sub_nerf_test_num)
    return a.clone(), b.clone()


@child_losses.register_fake
def _(free_ray, sl1_ray, rays, divide, sub_nerf_test_num):
    shp = (1,) if (divide and sub_nerf_test_num > 0) else ()
    return free_ray.new_empty(shp), free_ray.new_empty(shp)


# ----------------------------------------------------------------------------------------------- two-step view
@torch.library.custom_op(f"{NS}::view_rows", mutates_args=())
def view_rows(p: Tensor, z: Tensor, rows: Tensor, method: int,
              eps: float) -> tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """inference_0525_2's per-row stage (render.py:229-330): weights, depth, at_peak (uint8), child sum, per-row
    opacity terms (float64), points (R, 3)."""
    _need("view_rows", "z", z, (None, None))
    _need("view_rows", "p", p, tuple(z.shape))
    _need("view_rows", "rows", rows, (z.shape[0], ("min", 8)))
    return _ops.view_rows(p, z, rows, method, eps)


@view_rows.register_fake
def _(p, z, rows, method, eps):
    R, S = z.shape
    return (z.new_empty((R, S)), z.new_empty((R,)), z.new_empty((R,), dtype=torch.uint8), z.new_empty((R,)),
            z.new_empty((R,), dtype=torch.float64), z.new_empty((R, 3)))


@torch.library.custom_op(f"{NS}::view_walk", mutates_args=())
def view_walk(other: Tensor, at_peak: Tensor, child_sum: Tensor, opac_row: Tensor,
              n_samples: int) -> tuple[Tensor, Tensor]:
    """inference_0525_2's ray-group walk (render.py:331-368): effective-row flags (R, 1) bool, opacity ()."""
    return _ops.view_walk(other, at_peak, child_sum, opac_row, n_samples)


@view_walk.register_fake
def _(other, at_peak, child_sum, opac_row, n_samples):
    R = at_peak.shape[0]
    return at_peak.new_empty((R, 1), dtype=torch.bool), at_peak.new_empty((), dtype=torch.float32)


# ----------------------------------------------------------------------------------------------- losses
@torch.library.custom_op(f"{NS}::pointwise_loss", mutates_args=())
def pointwise_loss(pred: Tensor, target: Tensor, kind: str, valid_mask: Optional[Tensor]) -> Tensor:
    """mean(loss(pred, target)) of nof/criteria/loss.py (MSE / L1 / SmoothL1)."""
    return _ops.pointwise_loss(pred, target, kind, valid_mask)


@pointwise_loss.register_fake
def _(pred, target, kind, valid_mask):
    return pred.new_empty((), dtype=torch.float32)


@torch.library.custom_op(f"{NS}::pointwise_loss_backward", mutates_args=())
def pointwise_loss_backward(pred: Tensor, target: Tensor, kind: str, valid_mask: Optional[Tensor],
                            grad_out: Tensor) -> Tensor:
    return _ops.pointwise_loss_backward(pred, target, kind, valid_mask, grad_out).reshape(pred.shape)


@pointwise_loss_backward.register_fake
def _(pred, target, kind, valid_mask, grad_out):
    return torch.empty_like(pred, dtype=torch.float32)


def _pl_setup(ctx, inputs, output):
    pred, target, kind, valid_mask = inputs
    ctx.kind = kind
    ctx.save_for_backward(pred, target, valid_mask)


def _pl_backward(ctx, g):
    pred, target, m = ctx.saved_tensors
    return torch.ops.pcnerf.pointwise_loss_backward(pred, target, ctx.kind, m, g.contiguous()), None, None, None


pointwise_loss.register_autograd(_pl_backward, setup_context=_pl_setup)


def op_names() -> list:
    """The registered operator names (tests)."""
    return ["embed", "sample_coarse", "perturb", "resample", "sample_pdf", "pack_eval", "query_eval", "composite",
            "composite_extras", "child_losses", "view_rows", "view_walk", "pointwise_loss",
            "pointwise_loss_backward"]
