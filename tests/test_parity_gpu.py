"""HIP path vs the reference: golden vectors (made by importing the reference) and the CPU oracle.

Tolerances (north star: depth and losses within 1e-4 relative fp32 of the reference PyTorch path):
  depth / depth_fine / losses: rtol 1e-4 (atol 1e-6 for values near zero);
  network outputs p: rtol 2e-5; embeddings: atol 2e-6 (sinf/cosf differ from torch CPU by <= 1-2 ulp);
  BatchNorm running stats: rtol 1e-4.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from gradcheck import _report
from nof import synthetic as syn
from nof.networks import Embedding, NOF_coarse, NOF_fine
from nof import render as R
from oracle import ref_cpu as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEED_C, SEED_F = 1234, 5678
RTOL = 1e-4


def models(train):
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(SEED_C)).to(DEV).train(train)
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(SEED_F)).to(DEV).train(train)
    return Embedding(3, 10), mc, mf


def close(a, b, rtol=RTOL, atol=1e-6, what=""):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    np.testing.assert_allclose(a.astype(np.float64), b.astype(np.float64), rtol=rtol, atol=atol, err_msg=what)


def running(m):
    return np.stack([np.stack([bn.running_mean.cpu().numpy(), bn.running_var.cpu().numpy()]) for bn in m.norms()])


def test_embedding():
    g = golden("nof_eval")
    e = Embedding(3, 10)(torch.from_numpy(g["points"]).to(DEV))
    close(e, g["embedding"], 0, 2e-6, "embedding")


@pytest.fixture(params=["f16x2_3", "fp32"])
def eval_math(request):
    """The fused eval query's arithmetic (nof._ops.set_eval_math): the default split-fp16 products and fp32 MFMA."""
    from nof import _ops
    prev = _ops.set_eval_math(request.param)
    yield request.param
    _ops.set_eval_math(prev)


def test_nof_eval_forward(eval_math):
    g = golden("nof_eval")
    _, mc, _ = models(False)
    with torch.no_grad():
        p = mc(torch.from_numpy(g["embedding"]).to(DEV))
    close(p, g["p"], 2e-5, 1e-7, "p eval")


def test_nof_train_forward_chunks_and_running_stats(train_math):
    g = golden("nof_train")
    _, mc, _ = models(True)
    emb = Embedding(3, 10)
    x = torch.from_numpy(g["points"]).to(DEV)
    c = int(g["chunk"])
    with torch.no_grad():
        p = torch.cat([mc(emb(x[i:i + c])) for i in range(0, len(x), c)])
    close(p, g["p"], 2e-5, 1e-7, "p train")
    close(running(mc), g["running"], RTOL, 1e-7, "running stats")
    assert int(mc.norms()[0].num_batches_tracked) == -(-len(x) // c)


def test_nof_train_forward_far_positions(train_math):
    """Train-mode NOF.forward on embeddings whose position features spread over 80 km (|e - e0| > 2^15): the
    split forward's layer-0 moments (k_enc_gram) take their per-unit power-of-two range guard.  Against the float64
    oracle forward of the same parameters (p within 1e-4, running statistics within 1e-4)."""
    from oracle import ref_cpu as O
    gen = torch.Generator().manual_seed(11)
    e = torch.rand(6000, 63, generator=gen) * 2 - 1
    e[:, :3] = (torch.rand(6000, 3, generator=gen) * 2 - 1) * 4.0e4
    _, mc, _ = models(True)
    with torch.no_grad():
        p = mc(e.to(DEV))
    P = {k: v.double() if v.is_floating_point() else v.clone() for k, v in
         O.params_from_numpy(syn.init_nof_params(SEED_C)).items()}
    ref = O.nof_forward(P, e.double(), True)
    close(p, ref.squeeze(-1).numpy() if p.dim() == 1 else ref.numpy(), 1e-4, 1e-6, "p far positions")
    rs = np.stack([np.stack([P[b + ".running_mean"].numpy(), P[b + ".running_var"].numpy()]) for b in O.BN])
    close(running(mc), rs, 1e-4, 1e-6, "running stats far positions")


def test_layered_split_range_guard():
    """Positions at or beyond fp16's 65,504 from the block origin: the layered split train math (its encoding operand
    is split without a scale) raises instead of returning NaN; the fused default and fp32 MFMA evaluate them
    (p within 1e-4 of the float64 oracle)."""
    from nof import _ops as ops
    gen = torch.Generator().manual_seed(12)
    e = torch.rand(3000, 63, generator=gen) * 2 - 1
    e[:, :3] = (torch.rand(3000, 3, generator=gen) * 2 - 1) * 6.0e4
    e[7, 1] = 7.0e4
    P = {k: v.double() if v.is_floating_point() else v.clone() for k, v in
         O.params_from_numpy(syn.init_nof_params(SEED_C)).items()}
    ref = O.nof_forward(P, e.double(), True).reshape(-1).numpy()
    prev = ops.get_train_math()
    try:
        for m in ("f16x2_3", "f16x2_4"):
            ops.set_train_math(m)
            _, mc, _ = models(True)
            with torch.no_grad(), pytest.raises(RuntimeError, match="fp16's range"):
                mc(e.to(DEV))
        for m in ("f16x2_3_fused", "fp32"):
            ops.set_train_math(m)
            _, mc, _ = models(True)
            with torch.no_grad():
                p = mc(e.to(DEV))
            close(p.reshape(-1), ref, 1e-4, 1e-6, f"p beyond fp16 range ({m})")
    finally:
        ops.set_train_math(prev)


def knife_edge(bins, weights, u):
    """Samples whose bin has cdf_hi - cdf_lo within 4 ulp of the reference's 1e-5 threshold (render.py:408): there
    the branch depends on the last bit of the normaliser sum, whose order torch CPU fixes per ISA."""
    w = weights + 1e-5
    cdf = torch.cat([torch.zeros_like(w[:, :1]), torch.cumsum(w / w.sum(-1, keepdim=True), -1)], -1)
    inds = torch.searchsorted(cdf, u, right=True)
    lo = torch.gather(cdf, 1, torch.clamp(inds - 1, min=0))
    hi = torch.gather(cdf, 1, torch.clamp(inds, max=cdf.shape[-1] - 1))
    ulp = torch.finfo(torch.float32).eps * torch.maximum(hi.abs(), torch.tensor(1e-30))
    near = ((hi - lo) - 1e-5).abs() <= 4 * ulp
    # a neighbouring cdf entry within an ulp of u can also move the bin
    return near | ((u - lo).abs() <= 2 * ulp) | ((hi - u).abs() <= 2 * ulp)


def test_sample_pdf():
    g = golden("sample_pdf")
    bc, wc = torch.from_numpy(g["bins"]), torch.from_numpy(g["weights"])
    b, w = bc.to(DEV), wc.to(DEV)
    for det, key in ((True, "samples_det"), (False, "samples_rand")):
        u = torch.linspace(0, 1, 96).expand(64, 96) if det else torch.from_numpy(g["u"])
        got = R.sample_pdf(b, w, 96, det=det, u=None if det else u.to(DEV)).cpu()
        edge = knife_edge(bc, wc, u.contiguous())
        ok = ~edge
        assert edge.float().mean() < 0.05, "too many knife-edge samples in the fixture"  # flat runs are built in
        close(got[ok], g[key][ok.numpy()], RTOL, 1e-5, key)


@pytest.mark.parametrize("S", [64, 128])
def test_render_val(S, eval_math):
    g = golden(f"render_val_s{S}")
    emb, mc, mf = models(False)
    with torch.no_grad():
        res = R.render_rays_val(mc, mf, emb, torch.from_numpy(g["rays"]).to(DEV), N_samples=S,
                                N_importance=int(g["N_importance"]), perturb=0, noise_std=0, chunk=int(g["chunk"]))
    assert set(res) == {"depth", "depth_fine"}
    close(res["depth"], g["depth"], what="depth")
    close(res["depth_fine"], g["depth_fine"], what="depth_fine")


TRAIN = ["pcnerf", "pcnerf_noseg", "pcnerf_divide", "original", "pcnerf_perturb", "pcnerf_s128"]


@pytest.fixture(params=["f16x2_3", "fp32", "f16x2_3_fused"])
def train_math(request):
    """The train-mode layer arithmetic (nof._ops.set_train_math): the default split-fp16 products and fp32 MFMA."""
    from nof import _ops
    prev = _ops.set_train_math(request.param)
    yield request.param
    _ops.set_train_math(prev)


@pytest.mark.parametrize("name", TRAIN)
def test_render_train(name, train_math):
    g = golden(f"render_train_{name}")
    emb, mc, mf = models(True)
    rng = {k: torch.from_numpy(g[k]).to(DEV) for k in ("perturb_rand", "u") if k in g}
    rays = torch.from_numpy(g["rays"]).to(DEV)
    with torch.no_grad():
        res = R.render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=int(g["sub_nerf_test_num"]),
                                  N_samples=int(g["N_samples"]), N_importance=int(g["N_importance"]),
                                  perturb=int(g["perturb"]), noise_std=0, chunk=int(g["chunk"]),
                                  issegmentated=int(g["issegmentated"]),
                                  childnerf_ratio=float(g["childnerf_ratio"]),
                                  use_child_nerf_divide=int(g["use_child_nerf_divide"]),
                                  use_child_nerf_loss=int(g["use_child_nerf_loss"]), rng=rng)
    assert set(res) == {"child_free_loss_fine", "child_depth_loss_fine", "depth_fine", "child_free_loss",
                        "child_depth_loss", "depth"}
    close(res["depth"], g["depth"], what="depth")
    close(res["depth_fine"], g["depth_fine"], what="depth_fine")
    for k in ("child_free_loss", "child_depth_loss", "child_free_loss_fine", "child_depth_loss_fine"):
        close(res[k], g[k], RTOL, 1e-9, k)
    # range losses through the drop-in criteria (train_kitti.py:121-155)
    from nof.criteria import nof_loss
    loss = nof_loss["smoothl1"]()
    gt = rays[:, 14]
    if int(g["use_child_nerf_divide"]):
        lr = torch.zeros(1, device=DEV)
        lrf = torch.zeros(1, device=DEV)
        sub = rays[:, 9]
        for i in range(int(g["sub_nerf_test_num"])):
            m = torch.logical_and(sub > (i + 0.5), sub < (i + 1.5))
            if int(m.sum()) >= 1:
                lr = lr + 1e-1 * loss(1e1 * res["depth"][m], 1e1 * gt[m])
                lrf = lrf + 1e-1 * loss(1e1 * res["depth_fine"][m], 1e1 * gt[m])
    else:
        lr = 1e-1 * loss(1e1 * res["depth"], 1e1 * gt)
        lrf = 1e-1 * loss(1e1 * res["depth_fine"], 1e1 * gt)
    close(lr, g["loss_range"], what="loss_range")
    close(lrf, g["loss_range_fine"], what="loss_range_fine")
    total = lr + lrf + 1e6 * res["child_free_loss_fine"].to(DEV) + 1e6 * res["child_free_loss"].to(DEV) + \
        1e5 * res["child_depth_loss_fine"].to(DEV) + 1e5 * res["child_depth_loss"].to(DEV)
    close(total, g["loss_total"], what="loss_total")
    close(running(mc), g["running_c"], RTOL, 1e-6, "running coarse")
    close(running(mf), g["running_f"], RTOL, 1e-6, "running fine")


def check_weights64(got_w, got_z, g, rows, seed, eps, what):
    """Fine weights against the float64 evaluation of the SAME fine sample positions: each path's float32 z_vals and
    points (o + d*z rounded in float32, as render.py computes them), then embedding, eval-mode network and
    compositing (w / (sum + eps)) in float64 by the oracle.  The reference's own float32 weights sit <= 5e-6 relative
    from that evaluation of its z_vals (asserted below as the fixture's sanity); this path's weights must sit within
    1e-4 relative (north-star tolerance; floor 1e-6 on |w|) of the evaluation of ITS z_vals, for every sample -- a
    fine sample moved by sample_pdf's knife edge (see test_sample_pdf) moves both sides alike."""
    P = {k: v.double() if v.is_floating_point() else v.clone() for k, v in
         O.params_from_numpy(syn.init_nof_params(seed)).items()}
    r32 = torch.from_numpy(rows)

    def w64(z32):
        z32 = torch.as_tensor(z32, dtype=torch.float32)
        p = O.query(P, O.points(r32, z32).double(), False, 1 << 20)
        return O.composite(p, z32.double(), eps)[0].numpy()

    def rel(w, ref):
        return np.abs(np.asarray(w, np.float64) - ref) / np.maximum(np.abs(ref), 1e-6)

    e_ref = rel(g["weights"], w64(g["z_vals"]))
    e_got = rel(got_w.cpu().numpy(), w64(got_z.cpu().numpy()))
    _report({"case": f"{what}_weights", "vs_f64_max": float(e_got.max()), "ref_vs_f64_max": float(e_ref.max())})
    assert e_ref.max() <= 5e-6, (what, "fixture's reference weights vs float64", e_ref.max())
    assert e_got.max() <= RTOL, (what, "weights vs float64 of the same z", e_got.max(), int((e_got > RTOL).sum()))


@pytest.mark.parametrize("method", [0, 2])
def test_render_view(method, eval_math):
    g = golden(f"render_view_m{method}")
    emb, mc, mf = models(False)
    with torch.no_grad():
        res = R.render_rays_view_0525_2_2(mc, mf, emb, torch.from_numpy(g["rows"]).to(DEV),
                                          torch.from_numpy(g["other"]).to(DEV), N_samples=int(g["N_samples"]),
                                          N_importance=int(g["N_importance"]), perturb=0, noise_std=0, chunk=4096,
                                          depth_inference_method=method)
    assert set(res) == {"depth_fine", "weights", "opacity", "z_vals", "depth", "opacity_fine",
                        "points_inference_fine", "points_inference", "rays_effective_flag",
                        "rays_effective_flag_fine"}
    for k in ("depth", "depth_fine", "points_inference", "points_inference_fine", "opacity", "opacity_fine"):
        close(res[k], g[k], RTOL, 1e-6, k)
    close(res["z_vals"], g["z_vals"], RTOL, 1e-5, "z_vals")
    check_weights64(res["weights"], res["z_vals"], g, g["rows"], SEED_F, 1e-10, f"view_m{method}_{eval_math}")
    for k in ("rays_effective_flag", "rays_effective_flag_fine"):
        got = res[k].cpu().numpy()
        assert got.dtype == np.bool_ and got.shape == g[k].shape
        assert np.array_equal(got, g[k]), k


@pytest.mark.parametrize("isval", [0, 1])
def test_render_rays(isval, eval_math):
    from nof import _ops
    g = golden(f"render_rays_isval{isval}")
    emb, mc, mf = models(False)
    prev = _ops.set_depth2_order("cpu")   # the goldens are the reference on torch CPU: its tie order
    try:
        with torch.no_grad():
            res = R.render_rays(mc, mf, emb, torch.from_numpy(g["rays"]).to(DEV), N_samples=int(g["N_samples"]),
                                N_importance=int(g["N_importance"]), perturb=0, noise_std=0, chunk=4096,
                                isval=bool(isval))
    finally:
        _ops.set_depth2_order(prev)
    assert set(res) == {"depth_fine", "weights", "opacity", "z_vals", "depth", "depth2", "opacity_fine"}
    for k in ("depth", "depth_fine", "opacity", "opacity_fine"):
        close(res[k], g[k], RTOL, 1e-6, k)
    close(res["z_vals"], g["z_vals"], RTOL, 1e-5, "z_vals")
    # render.py:585/596 normalise by sum + float(isval) (see oracle/ref_cpu.py::render_rays)
    check_weights64(res["weights"], res["z_vals"], g, g["rays"], SEED_F, float(isval), f"rays_isval{isval}_{eval_math}")
    # depth2 = z at the position of sample S-1 in argsort(weights, descending=True) (render.py:598-600), torch CPU's
    # order of equal keys (set_depth2_order("cpu")):
    # (1) exactly the reference's rule applied to this path's own weights, every row (torch's argsort on the CPU);
    # (2) exactly the reference's depth2 on every row whose weights compare with w[S-1] exactly as the reference's
    #     do (the same <, = or > for every sample: the same samples ranked before it) and, on rows where w[S-1]
    #     ties another weight, compare pairwise exactly as the reference's (then the sort takes the same steps and
    #     leaves the tied samples in the same order); rows where a weight difference of ~1e-7 flips a comparison
    #     with w[S-1] (a fine sample moved by sample_pdf's knife edge) are the ones left out, and they must be few
    d2 = res["depth2"].cpu().numpy()
    wh, zh = res["weights"].cpu(), res["z_vals"].cpu().numpy()
    S = wh.shape[1]
    own = zh[wh.argsort(dim=-1, descending=True).eq(S - 1).numpy()]
    np.testing.assert_array_equal(d2, own)
    wr = torch.from_numpy(g["weights"])
    tied = (wr[:, :-1] == wr[:, -1:]).any(-1).numpy()
    last = (torch.sign(wh - wh[:, -1:]) == torch.sign(wr - wr[:, -1:])).all(-1).numpy()
    full = (torch.sign(wh[:, :, None] - wh[:, None, :]) == torch.sign(wr[:, :, None] - wr[:, None, :])).all(-1).all(-1)
    ok = last & (~tied | full.numpy())
    _report({"case": f"render_rays_isval{isval}_depth2_{eval_math}", "rows": int(ok.size),
             "same_order_rows": float(ok.mean()), "tied_rows": int(tied.sum()),
             "tied_same_order": int((ok & tied).sum())})
    assert ok.mean() >= 0.98, ok.mean()   # (measured: every row, both maths)
    rank_h = wh.argsort(dim=-1, descending=True).eq(S - 1).int().argmax(-1).numpy()
    rank_r = wr.argsort(dim=-1, descending=True).eq(S - 1).int().argmax(-1).numpy()
    np.testing.assert_array_equal(rank_h[ok], rank_r[ok])                  # the same sample selected, exactly
    close(d2[ok], g["depth2"][ok], 1e-5, 1e-5, "depth2")                     # its z within z_vals' tolerance


@pytest.mark.parametrize("order", ["stable", "cpu"])
def test_depth2_tie_order(order):
    """render.py:598's argsort(descending=True) on rows where w[S-1] ties other weights exactly (p = 0 samples and
    a p = 1 sample zero every weight after it).  "stable" (default): the order torch's sort gives on the GPU, where
    the reference runs render_rays (rows > 32 long: stable merge / radix sort; parity unpinned -- no GPU run of the
    reference exists here) -- torch's stable argsort; "cpu": torch CPU's std::sort order, restated by
    k_depth2_ties -- torch's own CPU argsort.  The HIP depth2 must equal z at that position on every row."""
    from nof import _ops
    g = torch.Generator().manual_seed(23)
    prev = _ops.set_depth2_order(order)
    try:
        for S in (64, 192, 384, 1000) + ((4000,) if order == "stable" else ()):
            R = 128
            p = torch.rand(R, S, generator=g)
            p[torch.rand(R, S, generator=g) < 0.3] = 0.0
            stop = torch.randint(S // 4, S, (R,), generator=g)
            for r in range(0, R, 2):
                p[r, stop[r]] = 1.0                      # every later weight exactly 0, w[S-1] among them
            p[1::4] = torch.rand(R // 4, S, generator=g) * 0.1 + 1e-3   # rows without ties
            z = torch.sort(torch.rand(R, S, generator=g) * 30, dim=1).values
            w, depth, _, _, _, d2 = _ops.composite(p.to(DEV), z.to(DEV), eps=1e-10, extras=True)
            w = w.cpu()
            idx = w.argsort(dim=-1, descending=True, stable=(order == "stable"))
            expect = z.numpy()[idx.eq(S - 1).numpy()]
            np.testing.assert_array_equal(d2.cpu().numpy(), expect, err_msg=f"S={S}")
        if order == "cpu":   # refused before any launch beyond the restatement's LDS row
            with pytest.raises(RuntimeError, match="2048"):
                _ops.composite(torch.rand(4, 3000, device=DEV), torch.rand(4, 3000, device=DEV), extras=True)
    finally:
        _ops.set_depth2_order(prev)


def test_view_walk_fallback_matches_parallel():
    """Malformed group lists take the literal sequential walk; well-formed ones the parallel path."""
    from nof import _ops
    R = 12
    at_peak = torch.tensor([0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0, 0], dtype=torch.uint8, device=DEV)
    csum = torch.arange(R, dtype=torch.float32, device=DEV).flip(0)
    op = torch.ones(R, dtype=torch.float64, device=DEV)
    good = torch.tensor([2, 0, 0, 0, 3, 0, 0, 0, 1, 0, 0, 0], device=DEV)
    flags, opac = _ops.view_walk(good, at_peak, csum, op, 4)
    assert flags[:, 0].nonzero().flatten().tolist() == [2, 3, 6, 8, 10, 11]
    assert abs(float(opac) - 0.25) < 1e-7
    bad = torch.tensor([2, 1, 0, 0, 3, 0, -1, 0, 0, 0, 0, 0], device=DEV)   # nested head + negative inner row
    flags, _ = _ops.view_walk(bad, at_peak, csum, op, 4)
    assert flags[:, 0].nonzero().flatten().tolist() == [2, 3, 6, 8, 9, 10, 11]


@pytest.mark.parametrize("ratio", [0.1, 0.5])
def test_segmented_coarse_z_bitexact(ratio):
    """k_sample_coarse (render.py:429-442) against the oracle's sort of the two linspaces, bit for bit: the
    binary-search merge (both lists non-decreasing) and, with every other ray's child interval reversed
    (child_near > child_far: a decreasing list), the all-pairs rank fallback."""
    from nof import _ops
    rays = torch.from_numpy(syn.make_rays(512, seed=21))
    rev = rays.clone()
    rev[::2, 10], rev[::2, 11] = rays[::2, 11], rays[::2, 10]
    for S in (64, 128, 200):
        sp = int(S * (1 - ratio))
        for r in (rays, rev):
            got = _ops.sample_coarse(r.to(DEV), S, sp, 6, 7, 10, 11).cpu()
            want = O.coarse_z(r, S, True, ratio)
            assert torch.equal(got, want), (S, ratio)


@pytest.mark.parametrize("R,S,I,sorted_u", [(256, 128, 256, True), (256, 128, 256, False), (64, 200, 500, False),
                                             (32, 300, 1000, False), (16, 768, 1536, False),
                                             (4, 4096, 8192, True), (4, 4096, 8192, False)])
def test_resample_merge_exact(R, S, I, sorted_u):
    """k_resample's sort(cat(z, z_samples)) (render.py:463-467): bit for bit the sort of the coarse z and the
    fine samples the same pdf code draws (pcnerf_sample_pdf), for sorted coarse rows (fine sort + binary-search
    merge) and with every third row unsorted (the ray falls back to the bitonic sort of the concatenation); sorted
    (perturb=0) and unsorted (perturb: torch.rand) uniforms; workgroup sizes 64..512 (fine lists of 256..2048
    slots, the reference shell's 768 / 1536 last); and the fine samples against the oracle."""
    from nof import _ops
    gen = torch.Generator().manual_seed(7)
    z = torch.sort(torch.rand(R, S, generator=gen) * 30, -1)[0]
    w = torch.rand(R, S, generator=gen)
    u = torch.rand(R, I, generator=gen)
    if sorted_u:
        u = torch.sort(u, -1)[0]
    zr = z.clone()
    zr[::3, 40], zr[::3, 41] = z[::3, 41], z[::3, 40]
    for zz in (z, zr):
        got = _ops.resample(zz.to(DEV), w.to(DEV), I, u.to(DEV)).cpu()
        mid = 0.5 * (zz[:, 1:] + zz[:, :-1])
        fine = _ops.sample_pdf_standalone(mid.to(DEV), w[:, 1:-1].to(DEV), I, False, u.to(DEV)).cpu()
        assert torch.equal(got, torch.sort(torch.cat([zz, fine], -1), -1)[0])
        close(fine, O.sample_pdf(mid, w[:, 1:-1], I, False, u).numpy(), 1e-5, 1e-6, "fine samples")


def test_render_val_eval_shell_setting():
    """The reference eval shells' sampling (shells/pretraining/*_eval.bash: N_samples 4096, N_importance 8192, chunk
    184320): k_resample's largest fine list (8,192 draws, 12,288-value merge) fits one workgroup's LDS and the
    rendered depths match the oracle (the launch used to exceed the 160 KiB cap)."""
    rays = syn.make_rays(6, seed=29)
    emb, mc, mf = models(False)
    kw = dict(N_samples=4096, N_importance=8192, perturb=0, noise_std=0, chunk=184320)
    with torch.no_grad():
        res = R.render_rays_val(mc, mf, emb, torch.from_numpy(rays).to(DEV), **kw)
    Pc, Pf = O.params_from_numpy(syn.init_nof_params(SEED_C)), O.params_from_numpy(syn.init_nof_params(SEED_F))
    ref = O.render_rays_val(Pc, Pf, torch.from_numpy(rays), **kw)
    for k in ("depth", "depth_fine"):
        close(res[k], ref[k].numpy(), RTOL, 1e-9, k)


@pytest.mark.parametrize("method", [1, 2])
def test_render_view_eval_shell_setting(method):
    """The two-step inference at the reference eval shells' sampling (N_samples 4096, N_importance 8192, chunk
    184320; eval_kitti_render.py renders through render_rays_view_0525_2_2 at exactly this): 12,288 fine samples per
    row -- k_view_rows' largest per-row buffers (48 KiB, one wave per workgroup) and its widest template -- and the
    ray-group walk, against the oracle on a few synthetic groups."""
    rows, other, _ = syn.make_view_rows(5, seed=41)
    # occupancy bias -9: per-sample occupancy ~1e-4, so transmittance survives 12,288 samples and the depths land
    # inside the rays (at the default -4 a random net's weights pile up in the first few hundred samples)
    pc_np, pf_np = syn.init_nof_params(SEED_C, occ_bias=-9.0), syn.init_nof_params(SEED_F, occ_bias=-9.0)
    mc = syn.load_into(NOF_coarse(), pc_np).to(DEV).eval()
    mf = syn.load_into(NOF_fine(), pf_np).to(DEV).eval()
    emb = Embedding(3, 10)
    kw = dict(N_samples=4096, N_importance=8192, perturb=0, noise_std=0, chunk=184320)
    with torch.no_grad():
        res = R.render_rays_view_0525_2_2(mc, mf, emb, torch.from_numpy(rows).to(DEV), torch.from_numpy(other).to(DEV),
                                          depth_inference_method=method, **kw)
    Pc, Pf = O.params_from_numpy(pc_np), O.params_from_numpy(pf_np)
    ref = O.render_rays_view(Pc, Pf, torch.from_numpy(rows), torch.from_numpy(other), N_samples=4096,
                             N_importance=8192, chunk=184320, method=method)
    for k in ("rays_effective_flag", "rays_effective_flag_fine"):
        assert np.array_equal(res[k].cpu().numpy(), ref[k].numpy().reshape(res[k].shape)), k
    for k in ("depth", "depth_fine", "points_inference", "points_inference_fine"):
        close(res[k], ref[k].numpy(), RTOL, 1e-6, k)


def test_empty_rays_raise_like_the_reference():
    """Zero rays: the reference's chunk loop collects nothing and torch.cat([]) raises (render.py:18-25, 44-51);
    the HIP path refuses the empty input with an exception too, never a silent empty result."""
    emb, mc, mf = models(False)
    rays = torch.zeros((0, 15), device=DEV)
    with torch.no_grad(), pytest.raises((RuntimeError, ValueError)):
        R.render_rays_val(mc, mf, emb, rays, N_samples=64, N_importance=128, perturb=0, noise_std=0, chunk=4096)
    with pytest.raises((RuntimeError, ValueError)):
        O.render_rays_val(O.params_from_numpy(syn.init_nof_params(SEED_C)),
                          O.params_from_numpy(syn.init_nof_params(SEED_F)), rays.cpu(), N_samples=64,
                          N_importance=128, perturb=0, noise_std=0, chunk=4096)
    emb, mc, mf = models(True)
    with torch.no_grad(), pytest.raises((RuntimeError, ValueError)):
        R.render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=4, N_samples=64, N_importance=128, perturb=0,
                            noise_std=0, chunk=4096, issegmentated=1, childnerf_ratio=0.1, use_child_nerf_loss=1)


def test_render_train_vs_oracle_config2_subset(train_math):
    """Config-2 rays at S=128/I=256 with several BatchNorm chunks, against the CPU oracle."""
    rays = syn.make_rays(192, seed=3)
    emb, mc, mf = models(True)
    kw = dict(sub_nerf_test_num=32, N_samples=128, N_importance=256, perturb=0, noise_std=0, chunk=16384,
              issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0, use_child_nerf_loss=1)
    with torch.no_grad():
        res = R.render_rays_train(mc, mf, emb, torch.from_numpy(rays).to(DEV), **kw)
    ref = O.render_rays_train(O.params_from_numpy(syn.init_nof_params(SEED_C)),
                              O.params_from_numpy(syn.init_nof_params(SEED_F)), torch.from_numpy(rays), **kw)
    for k in ("depth", "depth_fine", "child_free_loss", "child_depth_loss", "child_free_loss_fine",
              "child_depth_loss_fine"):
        close(res[k], ref[k].numpy(), RTOL, 1e-9, k)


def test_render_train_reference_shell_setting():
    """The reference's training shells' sampling (shells/pretraining/*_train.bash: 256 rays, N_samples 768,
    N_importance 1536, chunk 262144, segmented 0.1, child losses): one coarse BatchNorm chunk of 196,608 samples and
    fine chunks of 262,144 + 262,144 + 65,536 (default train math).  At 2,304 samples per ray the float32 oracle's
    own rounding moves depth_fine by ~2e-4 with its thread count, so the reference value is the oracle's float64
    evaluation (make_f64.py's): every entry within 1e-4 of it, or within 1.5 x the float32 oracle's own largest
    error; the running statistics of both networks after every chunk's update within 1e-4.  Occupancy bias -7.5:
    with 768 + 2304 samples per ray the default -4 puts every ray's weight in its first samples."""
    rays = syn.make_rays(256, seed=13)
    pc_np, pf_np = syn.init_nof_params(SEED_C, occ_bias=-7.5), syn.init_nof_params(SEED_F, occ_bias=-7.5)
    mc = syn.load_into(NOF_coarse(), pc_np).to(DEV).train(True)
    mf = syn.load_into(NOF_fine(), pf_np).to(DEV).train(True)
    emb = Embedding(3, 10)
    kw = dict(sub_nerf_test_num=32, N_samples=768, N_importance=1536, perturb=0, noise_std=0, chunk=262144,
              issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0, use_child_nerf_loss=1)
    with torch.no_grad():
        res = R.render_rays_train(mc, mf, emb, torch.from_numpy(rays).to(DEV), **kw)
        ref = O.render_rays_train(O.params_from_numpy(pc_np), O.params_from_numpy(pf_np), torch.from_numpy(rays),
                                  **kw)
        P64 = [{k: (v.double() if v.is_floating_point() else v) for k, v in O.params_from_numpy(q).items()}
               for q in (pc_np, pf_np)]
        r64 = O.render_rays_train(P64[0], P64[1], torch.from_numpy(rays), **kw, f64=True)
    for k in ("depth", "depth_fine", "child_free_loss", "child_depth_loss", "child_free_loss_fine",
              "child_depth_loss_fine"):
        want = r64[k].numpy().astype(np.float64)
        e_hip = np.abs(res[k].cpu().numpy().astype(np.float64) - want) / np.maximum(np.abs(want), 1e-30)
        e_ref = np.abs(ref[k].numpy().astype(np.float64) - want) / np.maximum(np.abs(want), 1e-30)
        _report({"case": f"train_shell_{k}", "vs_f64_max": float(e_hip.max()), "ref_vs_f64_max": float(e_ref.max())})
        assert e_hip.max() <= max(RTOL, 1.5 * e_ref.max()), (k, float(e_hip.max()), float(e_ref.max()))
    for m, P in ((mc, P64[0]), (mf, P64[1])):
        want = np.stack([np.stack([P[b + ".running_mean"].numpy(), P[b + ".running_var"].numpy()]) for b in O.BN])
        close(running(m), want, RTOL, 1e-7, "running stats")


@pytest.mark.parametrize("chunk", [50, 1000, 262144])
def test_render_train_tiny_and_odd_chunks(chunk, train_math):
    """BatchNorm chunks of 50 samples (two 32-sample tiles, the second partial: a 2-workgroup grid), 1000 and one
    chunk covering everything, against the CPU oracle -- the train kernels' grid, tail-tile and statistics paths.
    Checked on the coarse pass and its running statistics: with 16 coarse samples the fine pass's resampling is
    ill-conditioned (the fp32 oracle itself differs from a float64 run of it by up to 1.5e-3 on depth_fine here)."""
    rays = syn.make_rays(24, seed=11)
    emb, mc, mf = models(True)
    kw = dict(sub_nerf_test_num=32, N_samples=16, N_importance=32, perturb=0, noise_std=0, chunk=chunk,
              issegmentated=1, childnerf_ratio=0.25, use_child_nerf_divide=0, use_child_nerf_loss=1)
    with torch.no_grad():
        res = R.render_rays_train(mc, mf, emb, torch.from_numpy(rays).to(DEV), **kw)
    Pc, Pf = O.params_from_numpy(syn.init_nof_params(SEED_C)), O.params_from_numpy(syn.init_nof_params(SEED_F))
    ref = O.render_rays_train(Pc, Pf, torch.from_numpy(rays), **kw)
    for k in ("depth", "child_free_loss", "child_depth_loss"):
        close(res[k], ref[k].numpy(), RTOL, 1e-9, k)
    # the coarse network's running statistics after every chunk's update, in chunk order
    want = np.stack([np.stack([Pc[b + ".running_mean"].numpy(), Pc[b + ".running_var"].numpy()]) for b in O.BN])
    close(running(mc), want, RTOL, 1e-7, "running stats")


def test_eval_query_is_per_sample(eval_math):
    """Eval mode: a ray rendered alone equals the same ray rendered inside a large batch (bitwise)."""
    rays = torch.from_numpy(syn.make_rays(4096, seed=5)).to(DEV)
    emb, mc, mf = models(False)
    with torch.no_grad():
        full = R.render_rays_val(mc, mf, emb, rays, N_samples=128, N_importance=256, perturb=0, noise_std=0)
        part = R.render_rays_val(mc, mf, emb, rays[1000:1037], N_samples=128, N_importance=256, perturb=0,
                                 noise_std=0)
    assert torch.equal(full["depth"][1000:1037], part["depth"])
    assert torch.equal(full["depth_fine"][1000:1037], part["depth_fine"])


def test_full_size_properties():
    """Config 2 at full size (65,536 rays, 128/256 samples, train mode, chunk 262,144): every depth is finite
    and lies in [0, parent far]; losses are finite and non-negative; train-mode BatchNorm stats moved."""
    rays = torch.from_numpy(syn.make_rays(65536, seed=0)).to(DEV)
    emb, mc, mf = models(True)
    rm0 = mc.norms()[0].running_mean.clone()
    with torch.no_grad():
        res = R.render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=32, N_samples=128, N_importance=256,
                                  perturb=1, noise_std=0, chunk=262144, issegmentated=1, childnerf_ratio=0.1,
                                  use_child_nerf_loss=1)
    far = rays[:, 7]
    for k in ("depth", "depth_fine"):
        d = res[k]
        assert torch.isfinite(d).all()
        assert (d >= -1e-4).all() and (d <= far * (1 + 1e-5) + 1e-4).all()
    for k in ("child_free_loss", "child_depth_loss", "child_free_loss_fine", "child_depth_loss_fine"):
        v = float(res[k])
        assert np.isfinite(v) and v >= 0
    assert not torch.equal(rm0, mc.norms()[0].running_mean)


def _aabb_scene():
    g = golden("aabb_primitives")
    bounds6 = np.concatenate([g["lo"], g["hi"]], 1)
    parent6 = np.concatenate([syn.PARENT_LO, syn.PARENT_HI])
    return g, bounds6, parent6


def test_build_train_rays_vs_oracle():
    from nof.raytable import build_train_rays
    from oracle import rays_cpu as RC
    g, bounds6, parent6 = _aabb_scene()
    ref = RC.build_train_rays(g["points"], g["origin"], g["centers"], bounds6, syn.PARENT_LO, syn.PARENT_HI)
    t = lambda a: torch.from_numpy(np.asarray(a, dtype=np.float64)).to(DEV)
    got = build_train_rays(t(g["points"]), t(g["origin"]), t(g["centers"]), t(bounds6), t(parent6)).cpu().numpy()
    assert got.shape == ref.shape
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("method", [2, 1])
def test_build_view_rows_vs_oracle(method):
    from nof.raytable import build_view_rows
    from oracle import rays_cpu as RC
    g, bounds6, parent6 = _aabb_scene()
    rows, rng, other, tin = RC.build_view_rows(g["points"], g["origin"], bounds6, syn.PARENT_LO, syn.PARENT_HI,
                                               method=method)
    t = lambda a: torch.from_numpy(np.asarray(a, dtype=np.float64)).to(DEV)
    r2, g2, o2, t2 = build_view_rows(t(g["points"]), t(g["origin"]), t(bounds6), t(parent6), method=method)
    assert r2.shape == rows.shape
    np.testing.assert_array_equal(r2.cpu().numpy(), rows)
    np.testing.assert_array_equal(g2.cpu().numpy(), rng)
    np.testing.assert_array_equal(o2.cpu().numpy(), other)
    np.testing.assert_array_equal(t2.cpu().numpy(), tin)


def test_sample_pdf_pytest_hook():
    """sample_pdf(pytest=True) (render.py:386-394): numpy-seeded draws, det and random, vs the reference."""
    g = golden("sample_pdf_pytest")
    bc, wc = torch.from_numpy(g["bins"]), torch.from_numpy(g["weights"])
    b, w = bc.to(DEV), wc.to(DEV)
    R_ = bc.shape[0]
    for det, key in ((True, "samples_det"), (False, "samples_rand")):
        got = R.sample_pdf(b, w, 96, det=det, pytest=True).cpu()
        np.random.seed(0)
        u = np.broadcast_to(np.linspace(0., 1., 96), (R_, 96)) if det else np.random.rand(R_, 96)
        ok = ~knife_edge(bc, wc, torch.from_numpy(np.ascontiguousarray(u, dtype=np.float32)))   # see test_sample_pdf
        assert (~ok).float().mean() < 0.05
        close(got[ok], g[key][ok.numpy()], RTOL, 1e-5, key)
    # torch's global CPU generator ends where the reference leaves it: one torch.rand(R, N) per det=False call
    # (render.py:383), none for det=True
    for det in (True, False):
        torch.manual_seed(77)
        R.sample_pdf(b, w, 96, det=det, pytest=True)
        after = torch.rand(4)
        torch.manual_seed(77)
        if not det:
            torch.rand((R_, 96))
        np.testing.assert_array_equal(after.numpy(), torch.rand(4).numpy())


def test_nan_bounds_sort_like_torch():
    """Rays with NaN child bounds / NaN coarse weights: the segmented coarse z and the fine merge hold every value
    once with the NaNs last (torch.sort's order), never an unwritten slot (both kernels take their rank / bitonic
    path when a list holds a NaN)."""
    from nof import _ops
    rays = torch.from_numpy(syn.make_rays(64, seed=23))
    rays[::4, 10] = float("nan")
    rays[1::4, 11] = float("nan")
    got = _ops.sample_coarse(rays.to(DEV), 64, 57, 6, 7, 10, 11).cpu()
    want = O.coarse_z(rays, 64, True, 0.1)
    np.testing.assert_array_equal(got.numpy(), want.numpy())
    gen = torch.Generator().manual_seed(4)
    R_, S, I = 64, 64, 128
    z = torch.sort(torch.rand(R_, S, generator=gen) * 30, -1)[0]
    w = torch.rand(R_, S, generator=gen)
    w[::5, 7] = float("nan")
    z[2::5, 30] = float("nan")     # a NaN coarse depth: NaN bins and fine samples, NaNs in both merged lists
    u = torch.sort(torch.rand(R_, I, generator=gen), -1)[0]
    zf = _ops.resample(z.to(DEV), w.to(DEV), I, u.to(DEV)).cpu()
    mid = 0.5 * (z[:, 1:] + z[:, :-1])
    fine = _ops.sample_pdf_standalone(mid.to(DEV), w[:, 1:-1].contiguous().to(DEV), I, False, u.to(DEV)).cpu()
    np.testing.assert_array_equal(zf.numpy(), torch.sort(torch.cat([z, fine], -1), -1)[0].numpy())


@pytest.mark.parametrize("R_,S", [(256, 768), (256, 2304), (40, 4096)])
def test_composite_workgroup_per_ray(R_, S):
    """The reference shell's shape (256 rays x 768 coarse / 2,304 fine samples) and 4,096-sample rows: k_composite /
    k_composite_bwd with a 256-thread workgroup per ray (Grp<256>, the automatic choice here) against a wave per ray
    (Grp<64>) on the same inputs -- weights, depth, child-loss terms, opacity sums, depth2 and dL/dlogit -- and
    the forward against the oracle's compositing (render.py:51-61; depth rtol 1e-5).  Every sum and scan is float64
    rounded once, so the two groupings agree to float64 association noise."""
    from nof import _ops
    gen = torch.Generator().manual_seed(S)
    rays = torch.from_numpy(syn.make_rays(R_, seed=S))
    z = torch.sort(rays[:, 6:7] + (rays[:, 7:8] - rays[:, 6:7]) * torch.rand(R_, S, generator=gen), -1)[0]
    p = torch.rand(R_, S, generator=gen) ** 8   # mostly transparent, a few occupied samples per ray
    rd, zd, pd = rays.to(DEV), z.to(DEV), p.to(DEV)
    gdep = torch.randn(R_, generator=gen).to(DEV)
    gfree, gdl = torch.tensor(0.3, device=DEV), torch.tensor(-0.7, device=DEV)
    outs = {}
    prev = _ops.set_composite_group(0)
    try:
        for grp in (64, 256):
            _ops.set_composite_group(grp)
            w, d, fr, sl = _ops.composite(pd, zd, None, 0.0, 1e-10, rd)
            w2, d2, _, _, om, dep2 = _ops.composite(pd, zd, None, 0.0, 1e-10, extras=True)
            g = _ops.composite_backward(pd, zd, None, 0.0, 1e-10, rd, 0, gdep, gfree, gdl)
            outs[grp] = [t.cpu().double() for t in (w, d, fr, sl, om, dep2, g)]
    finally:
        _ops.set_composite_group(prev)
    names = ("weights", "depth", "free_ray", "sl1_ray", "opacity", "depth2", "g_logit")
    for n, a, b in zip(names, outs[64], outs[256]):
        scale = float(b.abs().max()) or 1.0
        assert float((a - b).abs().max()) <= 2e-6 * scale, n
    wr, dr = O.composite(p, z)
    close(outs[256][1], dr.numpy(), 1e-5, 1e-6, "depth vs oracle")
    close(outs[256][0], wr.numpy(), 1e-5, 1e-7, "weights vs oracle")
