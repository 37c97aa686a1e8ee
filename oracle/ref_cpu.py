"""CPU oracle for the PC-NeRF render + loss hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity checker.  Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it; the product path (``pc-nerf_amd/nof``) never does and fails loudly when its HIP
library is missing.

It restates, vectorised, the reference's PyTorch arithmetic on CPU (torch CPU is the reference's own arithmetic
library, so each op here is the op the reference runs).  Every function cites the reference lines it follows.
The restatement is pinned against golden vectors produced by importing the reference itself
(``tests/golden/make_golden.py``; checked by ``tests/test_oracle_golden.py``).

Numerics it preserves on purpose (all verified against the reference in this container):
* ``torch.linspace`` values; z = near*(1-s)+far*s and p = o + d*z rounded op by op (no FMA);
* ``cumprod``/``cumsum`` accumulate in float64 on CPU and round each prefix to float32;
* child-mask expansion: ``thr`` grows by 0.01 in Python float64, each bound is ``fl32(bound -/+ fl32(thr))``;
* BatchNorm statistics per ``chunk`` of flattened ray-major samples (train mode), running-stat updates per chunk.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as Fn

EPS_BN = 1e-5
MOMENTUM = 0.1


# ----------------------------------------------------------------------------------------------- network
def embed(x: torch.Tensor, n_freq: int = 10) -> torch.Tensor:
    """models.py:27-41 -- [x, sin(2^k x), cos(2^k x)] for k = 0..n_freq-1 (freq_bands at models.py:23)."""
    feats = [x]
    for f in (2.0 ** torch.linspace(0, n_freq - 1, n_freq)).tolist():
        feats.append(torch.sin(f * x))
        feats.append(torch.cos(f * x))
    return torch.cat(feats, -1)


LIN = ["layer1.0", "layer1.3", "layer1.6", "layer1.9", "layer2.0", "layer2.2", "layer2.4", "layer2.6"]
BN = ["layer1.1", "layer1.4", "layer1.7", "layer1.10", "layer2.1", "layer2.3", "layer2.5", "layer2.7"]


def params_from_numpy(p: dict) -> dict:
    return {k: torch.from_numpy(np.array(v)).clone() for k, v in p.items()}


def nof_forward(P: dict, e: torch.Tensor, training: bool) -> torch.Tensor:
    """models.py:183-203 on one chunk: 4 x (Linear, BatchNorm1d, identity) -> cat(e, .) -> 4 x (Linear,
    BatchNorm1d) -> Linear(256,1) -> sigmoid.  LeakyReLU(True) has negative_slope == 1 (models.py:72,152): an
    identity, so it is not applied.  In training mode BatchNorm uses the chunk's statistics and updates the
    running stats in ``P`` in place (momentum 0.1, unbiased variance), exactly like nn.BatchNorm1d."""
    h = e
    for i in range(8):
        if i == 4:
            h = torch.cat([e, h], 1)  # models.py:196-197 skip
        h = Fn.linear(h, P[LIN[i] + ".weight"], P[LIN[i] + ".bias"])
        b = BN[i]
        if training and h.shape[0] <= 1:
            raise ValueError("Expected more than 1 value per channel when training")
        h = Fn.batch_norm(h, P[b + ".running_mean"], P[b + ".running_var"], P[b + ".weight"], P[b + ".bias"],
                          training=training, momentum=MOMENTUM, eps=EPS_BN)
        if training:
            P[b + ".num_batches_tracked"] += 1
    return torch.sigmoid(Fn.linear(h, P["occ_out.0.weight"], P["occ_out.0.bias"]))


def query(P: dict, pts: torch.Tensor, training: bool, chunk: int) -> torch.Tensor:
    """render.py:18-25 / 44-51 chunk loop: flatten ray-major samples, run embed + NOF per chunk, reshape."""
    R, S = pts.shape[:2]
    flat = pts.reshape(-1, 3)
    out = [nof_forward(P, embed(flat[i:i + chunk]), training) for i in range(0, flat.shape[0], chunk)]
    return torch.cat(out, 0).view(R, S)


# ----------------------------------------------------------------------------------------------- sampling
def lin_z(near: torch.Tensor, far: torch.Tensor, n: int) -> torch.Tensor:
    """render.py:430-432: z = near*(1-s) + far*s with s = linspace(0,1,n)."""
    s = torch.linspace(0, 1, n).expand(near.shape[0], n)
    return near * (1 - s) + far * s


def coarse_z(rays, S, segmented, ratio, near_col=6, far_col=7, cn_col=10, cf_col=11):
    """render.py:429-442: uniform z in [near, far]; segmented: int(S*(1-ratio)) parent samples plus the rest in
    [child_near, child_far], merged by sort."""
    near, far = rays[:, near_col:near_col + 1], rays[:, far_col:far_col + 1]
    if not segmented:
        return lin_z(near, far, S)
    sp = int(S * (1 - ratio))
    zp = lin_z(near, far, sp)
    zc = lin_z(rays[:, cn_col:cn_col + 1], rays[:, cf_col:cf_col + 1], S - sp)
    return torch.sort(torch.cat([zp, zc], -1), -1)[0]


def perturb_z(z, perturb, rand):
    """render.py:449-454: stratified jitter between midpoints."""
    mid = 0.5 * (z[:, :-1] + z[:, 1:])
    upper = torch.cat([mid, z[:, -1:]], -1)
    lower = torch.cat([z[:, :1], mid], -1)
    return lower + (upper - lower) * (perturb * rand)


def points(rays, z):
    """render.py:458: p = o + d*z (op by op)."""
    return rays[:, None, 0:3] + rays[:, None, 3:6] * z[..., None]


def sample_pdf(bins, weights, n, det, u=None):
    """render.py:371-412 (nerf-pytorch inverse-CDF sampling); ``u`` may be injected when ``det`` is False."""
    weights = weights + 1e-5
    pdf = weights / torch.sum(weights, -1, keepdim=True)
    cdf = torch.cumsum(pdf, -1)
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], -1)
    if det:
        u = torch.linspace(0., 1., steps=n).expand(list(cdf.shape[:-1]) + [n])
    elif u is None:
        u = torch.rand(list(cdf.shape[:-1]) + [n])
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    below = torch.clamp(inds - 1, min=0)
    above = torch.clamp(inds, max=cdf.shape[-1] - 1)
    cdf_lo, cdf_hi = torch.gather(cdf, 1, below), torch.gather(cdf, 1, above)
    b_lo, b_hi = torch.gather(bins, 1, below), torch.gather(bins, 1, above)
    denom = cdf_hi - cdf_lo
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    t = (u - cdf_lo) / denom
    return b_lo + t * (b_hi - b_lo)


# ----------------------------------------------------------------------------------------------- compositing
def composite(p, z, eps=1e-10, noise=None):
    """render.py:51-61 (== :25-34, :241-246): w_i = p_i * prod_{j<i}(1-p_j); (+noise); w /= sum(w)+eps; depth."""
    free = 1 - p
    trans = torch.cumprod(torch.cat([torch.ones_like(free[:, :1]), free], -1), -1)[:, :-1]
    w = trans * p
    if noise is not None:
        w = w + noise
    w = w / (torch.sum(w, -1).reshape(-1, 1) + eps)
    return w, torch.sum(w * z, -1)


def expand_mask(z, near, far, thr0, strict=False):
    """render.py:77-84 / 91-97 (inclusive, thr0 = 0 and 2) and :252-263 (strict, thr0 = 0.01): per ray, the
    smallest thr = thr0 + k*0.01 (accumulated in float64) for which some sample lies in
    [fl32(near - fl32(thr)), fl32(far + fl32(thr))]."""
    R = z.shape[0]
    thr = np.full(R, float(thr0))
    todo = np.ones(R, dtype=bool)
    mask = torch.zeros_like(z, dtype=torch.bool)
    it = 0
    while todo.any():
        idx = torch.from_numpy(np.nonzero(todo)[0])
        t32 = torch.from_numpy(thr[todo].astype(np.float32))[:, None]
        lo, hi = near[idx][:, None] - t32, far[idx][:, None] + t32
        zz = z[idx]
        m = ((lo < zz) & (zz < hi)) if strict else ((lo <= zz) & (zz <= hi))
        mask[idx] = m
        ok = m.any(1).numpy()
        done = np.nonzero(todo)[0][ok]
        todo[done] = False
        rest = todo.copy()
        thr[rest] = thr[rest] + 0.01
        it += 1
        if it > 1_000_000:
            raise RuntimeError("child mask expansion did not terminate")
    return mask


def child_losses(w, z, rays, near_far_child, ranges, divide, sub_num, eps=1e-10):
    """render.py:75-159: free-space loss on weights outside the child interval (M0, exact bounds) and the
    child depth loss on weights re-normalised inside the interval grown by 2 m (M2)."""
    R, S = w.shape
    m0 = expand_mask(z, near_far_child[:, 0], near_far_child[:, 1], 0.0)
    m2 = expand_mask(z, near_far_child[:, 0], near_far_child[:, 1], 2)
    w_free = w * (~m0).float()
    wc = w * m2.float()
    zc = z * m2.float()
    wc = wc / (torch.sum(wc, -1).reshape(-1, 1) + eps)
    dc = torch.sum(wc * zc, -1)
    sl1 = torch.nn.SmoothL1Loss(reduction="mean")
    rr = ranges.reshape(-1)
    if not divide:
        free = torch.sum(torch.square(w_free)) / R
        depth = 1 / R * 0.1 * sl1(1e1 * dc, 1e1 * rr)
        return free, depth
    sub = rays[:, 9]
    free = torch.tensor([0.0])
    depth = torch.tensor([0.0])
    for i in range(sub_num):                                     # render.py:111-119, 140-152
        m = (sub > (i + 0.5)) & (sub < (i + 1.5))
        c = m.float().sum()                                      # float32 count, as sub_nerf_tmp.sum()
        if c >= 1:
            free = free + torch.sum(torch.square(w_free[m])) / c
            depth = depth + 1 / c * 0.1 * sl1(1e1 * dc[m], 1e1 * rr[m])
    return free, depth


# ----------------------------------------------------------------------------------------------- render paths
def render_rays_train(Pc, Pf, rays, sub_nerf_test_num=4, N_samples=64, N_importance=128, perturb=0, noise_std=1,
                      chunk=3072, issegmentated=0, childnerf_ratio=0.5, use_child_nerf_divide=0,
                      use_child_nerf_loss=0, training=True, draws=None, f64=False):
    """render.py:416-482 with inference_train (:38-163).  ``draws`` may carry the RNG tensors the reference
    would consume: ``perturb_rand`` (R,S), ``noise`` (R,S), ``u`` (R,I), ``noise_fine`` (R,S+I).
    ``f64``: the float64 evaluation of tests/golden/make_f64.py -- coarse z and points rounded in float32 exactly as
    the reference rounds them (float32 ``rays``), everything after them (network with float64 ``Pc``/``Pf``,
    BatchNorm, compositing, losses, sample_pdf, fine points) in float64."""
    draws = draws or {}
    R = rays.shape[0]
    z = coarse_z(rays, N_samples, issegmentated, childnerf_ratio)
    if perturb > 0:
        z = perturb_z(z, perturb, draws["perturb_rand"] if "perturb_rand" in draws else torch.rand(z.shape))
    pts_c = points(rays, z)
    if f64:
        pts_c, z, rays = pts_c.double(), z.double(), rays.double()
    nfc, ranges = rays[:, 10:12], rays[:, 14]

    def pass_(P, z, noise, pts=None):
        p = query(P, points(rays, z) if pts is None else pts, training, chunk)
        nz = None if noise_std == 0 else noise * noise_std
        w, depth = composite(p, z, 1e-10, nz)
        if use_child_nerf_loss:
            fl, dl = child_losses(w, z, rays, nfc, ranges, use_child_nerf_divide, sub_nerf_test_num)
        else:
            fl, dl = torch.tensor(0.0), torch.tensor(0.0)
        return w, depth, fl, dl

    w, depth, fl, dl = pass_(Pc, z, draws.get("noise"), pts_c)
    zmid = .5 * (z[..., 1:] + z[..., :-1])
    zs = sample_pdf(zmid, w[..., 1:-1], N_importance, det=(perturb == 0.), u=draws.get("u")).detach()  # :466
    zf = torch.sort(torch.cat([z, zs], -1), -1)[0]
    wf, depth_f, flf, dlf = pass_(Pf, zf, draws.get("noise_fine"))
    return {"child_free_loss_fine": flf, "child_depth_loss_fine": dlf, "depth_fine": depth_f,
            "child_free_loss": fl, "child_depth_loss": dl, "depth": depth}


def render_rays_val(Pc, Pf, rays, N_samples=64, N_importance=128, perturb=0, noise_std=1, chunk=3072,
                    training=False, draws=None):
    """render.py:485-536 with inference_val (:13-36)."""
    draws = draws or {}
    z = lin_z(rays[:, 6:7], rays[:, 7:8], N_samples)
    if perturb > 0:
        z = perturb_z(z, perturb, draws["perturb_rand"] if "perturb_rand" in draws else torch.rand(z.shape))
    p = query(Pc, points(rays, z), training, chunk)
    w, depth = composite(p, z, 1e-10, None if noise_std == 0 else draws["noise"] * noise_std)
    zmid = .5 * (z[..., 1:] + z[..., :-1])
    zs = sample_pdf(zmid, w[..., 1:-1], N_importance, det=(perturb == 0.), u=draws.get("u"))
    zf = torch.sort(torch.cat([z, zs], -1), -1)[0]
    pf = query(Pf, points(rays, zf), training, chunk)
    _, depth_f = composite(pf, zf, 1e-10, None if noise_std == 0 else draws["noise_fine"] * noise_std)
    return {"depth_fine": depth_f, "depth": depth}


def gaussian_smooth(w: torch.Tensor, sigma=5.0, truncate=4.0) -> torch.Tensor:
    """scipy.ndimage.gaussian_filter(row, sigma=5) as used at render.py:306 (mode 'reflect', radius
    int(truncate*sigma+0.5) = 20, float64 accumulation, float32 result)."""
    from scipy.ndimage import gaussian_filter1d
    out = gaussian_filter1d(w.numpy().astype(np.float32), sigma=sigma, axis=-1, mode="reflect", truncate=truncate)
    return torch.from_numpy(out.astype(np.float32))


def inference_view(p, z, other, near_far_child, method, eps=1e-10):
    """render.py:229-368 after the network query: composite, strict child mask (thr 0.01 + 0.01 steps),
    Gaussian-smoothed peak, group walk (render.py:317-340) and the method-2 child re-normalised depth."""
    w, _ = composite(p, z, eps)
    R = w.shape[0]
    mask_child = expand_mask(z, near_far_child[:, 0], near_far_child[:, 1], 0.01, strict=True)
    peak = torch.argmax(gaussian_smooth(w), dim=1)
    at_peak = mask_child[torch.arange(R), peak]
    wsum_child = torch.sum(w * mask_child.float(), -1)
    flag = torch.zeros((R, 1), dtype=torch.bool)
    oth = [int(v) for v in other.tolist()]
    i = 0
    while i < R:
        o = oth[i]
        if abs(o) < 0.5:
            flag[i] = True
            i += 1
        elif o > 0.5:
            pick = i
            if not bool(at_peak[i]):
                found = False
                for j in range(o):
                    if bool(at_peak[i + j + 1]):
                        pick, found = i + j + 1, True
                        break
                if not found:
                    for j in range(o):
                        if wsum_child[i + j + 1] > wsum_child[pick]:
                            pick = i + j + 1
            flag[pick] = True
            i += o + 1
        else:
            i += 1
    if method == 2:
        wc = w * mask_child.float()
        wc = wc / (torch.sum(wc, -1).reshape(-1, 1) + eps)
        depth = torch.sum(wc * z, -1)
    else:
        depth = torch.sum(w * z, -1)
    opacity = torch.mean(torch.log(0.1 + p) + torch.log(0.1 + (1 - p)) + 2.20727)
    return depth, w, opacity, flag


def render_rays(Pc, Pf, rays, N_samples=64, N_importance=128, use_disp=False, perturb=0, noise_std=1, chunk=3072,
                isval=False, draws=None):
    """render.py:538-611 with inference (:166-226).  The call at render.py:585/596 passes ``isval`` positionally
    into inference's ``epsilon`` slot, so weights are always normalised, by sum + float(isval), and inference's
    own ``isval`` stays False.  depth2 = z at the position where sample F-1 appears in the descending argsort of
    the fine weights (render.py:598-600)."""
    draws = draws or {}
    near, far = rays[:, 6:7], rays[:, 7:8]
    s = torch.linspace(0, 1, N_samples).expand(rays.shape[0], N_samples)
    z = 1 / (1 / near * (1 - s) + 1 / far * s) if use_disp else near * (1 - s) + far * s
    if perturb > 0:
        z = perturb_z(z, perturb, draws["perturb_rand"] if "perturb_rand" in draws else torch.rand(z.shape))
    eps = float(isval)

    def inf(P, z, noise):
        p = query(P, points(rays, z), False, chunk)
        w, depth = composite(p, z, eps, None if noise_std == 0 else noise * noise_std)
        opac = torch.mean(torch.log(0.1 + p) + torch.log(0.1 + (1 - p)) + 2.20727)
        return depth, w, opac

    depth, w, opac = inf(Pc, z, draws.get("noise"))
    zmid = .5 * (z[..., 1:] + z[..., :-1])
    zs = sample_pdf(zmid, w[..., 1:-1], N_importance, det=(perturb == 0.), u=draws.get("u"))
    zf = torch.sort(torch.cat([z, zs], -1), -1)[0]
    depth_f, wf, opac_f = inf(Pf, zf, draws.get("noise_fine"))
    mask = wf.argsort(dim=-1, descending=True).eq(wf.shape[1] - 1)
    return {"depth_fine": depth_f, "weights": wf, "opacity": opac, "z_vals": zf, "depth": depth,
            "depth2": zf[mask], "opacity_fine": opac_f}


def render_rays_view(Pc, Pf, rows, other, N_samples=64, N_importance=128, chunk=3072, method=0):
    """render.py:614-699: parent bounds from cols 9/10, child bounds cols 6:8, coarse + fine inference_view,
    points o + depth*d."""
    nfc = rows[:, 6:8]
    z = lin_z(rows[:, 9:10], rows[:, 10:11], N_samples)
    p = query(Pc, points(rows, z), False, chunk)
    depth, w, opac, flag = inference_view(p, z, other, nfc, method)
    zmid = .5 * (z[..., 1:] + z[..., :-1])
    zs = sample_pdf(zmid, w[..., 1:-1], N_importance, det=True)
    zf = torch.sort(torch.cat([z, zs], -1), -1)[0]
    pf = query(Pf, points(rows, zf), False, chunk)
    depth_f, wf, opac_f, flag_f = inference_view(pf, zf, other, nfc, method)
    o, d = rows[:, 0:3], rows[:, 3:6]
    return {"depth_fine": depth_f, "weights": wf, "opacity": opac, "z_vals": zf, "depth": depth,
            "opacity_fine": opac_f, "points_inference_fine": o + depth_f[:, None] * d,
            "points_inference": o + depth[:, None] * d, "rays_effective_flag": flag,
            "rays_effective_flag_fine": flag_f}


# ----------------------------------------------------------------------------------------------- losses
def range_losses(depth, depth_fine, gt, rays=None, divide=0, sub_num=4, lam=1.0, lam_fine=1.0):
    """train_kitti.py:121-146 (SmoothL1 from nof/criteria/loss.py:42-50): 0.1*lambda*SmoothL1(10 d, 10 gt);
    the non-divide branch uses lambda_loss for both coarse and fine (train_kitti.py:145-146)."""
    sl1 = torch.nn.SmoothL1Loss(reduction="mean")
    if not divide:
        return 1e-1 * lam * sl1(1e1 * depth, 1e1 * gt), 1e-1 * lam * sl1(1e1 * depth_fine, 1e1 * gt)
    lr, lrf = torch.tensor([0.0]), torch.tensor([0.0])
    sub = rays[:, 9]
    for i in range(sub_num):
        m = (sub > (i + 0.5)) & (sub < (i + 1.5))
        if int(m.sum()) >= 1:
            lr = lr + 1e-1 * lam * sl1(1e1 * depth[m], 1e1 * gt[m])
            lrf = lrf + 1e-1 * lam_fine * sl1(1e1 * depth_fine[m], 1e1 * gt[m])
    return lr, lrf


def total_loss(res, lr, lrf, lam_free=1e6, lam_depth=1e5):
    """train_kitti.py:153-155."""
    return (lr + lrf + lam_free * res["child_free_loss_fine"] + lam_free * res["child_free_loss"]
            + lam_depth * res["child_depth_loss_fine"] + lam_depth * res["child_depth_loss"])
