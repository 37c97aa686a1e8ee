"""The render path as torch custom operators (torch.ops.pcnerf.*, nof/_torch_ops.py).

CPU: every operator is registered with a schema and its fake (meta) implementation gives the shapes the HIP
implementation returns.  GPU: the operators are what nof.render runs (the parity tests go through them), the loss's
backward is the operator's registered autograd, and torch.compile (non-fullgraph, the aot_eager backend: FakeTensor
tracing through the fake implementations, no code generation) renders render_rays_val with the pcnerf operators as
graph nodes and the eager result bit for bit.
"""
import pytest
import torch

from nof import _torch_ops as T


def test_ops_registered_with_schemas():
    for name in T.op_names():
        op = getattr(torch.ops.pcnerf, name)
        assert str(op.default._schema).startswith(f"pcnerf::{name}(")


def test_fake_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode
    P = torch.ops.pcnerf
    with FakeTensorMode():
        rays = torch.empty(5, 15, device="meta")
        z = P.sample_coarse(rays, 64, 57, 6, 7, 10, 11, False)
        assert z.shape == (5, 64)
        assert P.perturb(z, 1.0, torch.empty(5, 64, device="meta")).shape == (5, 64)
        p = torch.empty(5, 64, device="meta")
        w, d, fr, sl = P.composite(p, z, None, 0.0, 1e-10, rays, 10, 11, 14, True)
        assert (w.shape, d.shape, fr.shape, sl.shape) == ((5, 64), (5,), (5,), (5,))
        w, d, fr, sl = P.composite(p, z, None, 0.0, 1e-10, None, 10, 11, 14, False)
        assert (w.shape, fr.shape) == ((0,), (0,))
        assert P.resample(z, w, 128, None).shape == (5, 192)
        a, b = P.child_losses(d, d, rays, True, 4)
        assert a.shape == (1,) and b.shape == (1,)
        a, b = P.child_losses(d, d, rays, False, 4)
        assert a.shape == () and b.shape == ()
        outs = P.view_rows(p, z, torch.empty(5, 13, device="meta"), 2, 1e-10)
        assert [o.shape for o in outs] == [(5, 64), (5,), (5,), (5,), (5,), (5, 3)]
        assert outs[2].dtype == torch.uint8 and outs[4].dtype == torch.float64
        f, o = P.view_walk(torch.empty(5, dtype=torch.int64, device="meta"), outs[2], outs[3], outs[4], 64)
        assert f.shape == (5, 1) and f.dtype == torch.bool and o.shape == ()
        assert P.embed(torch.empty(7, 3, device="meta")).shape == (7, 63)
        assert P.pointwise_loss(d, d, "smoothl1", None).shape == ()


@pytest.mark.gpu
def test_loss_autograd_through_operator():
    """nof.criteria's loss is pcnerf::pointwise_loss; d/dpred comes from its registered backward and equals the
    kernel's own backward entry."""
    from nof import _ops
    from nof.criteria import nof_loss
    g = torch.Generator().manual_seed(3)
    pred = (torch.rand(1000, generator=g) * 40).cuda().requires_grad_(True)
    tgt = (torch.rand(1000, generator=g) * 40).cuda()
    loss = nof_loss["smoothl1"]()(10 * pred, 10 * tgt)
    loss.backward()
    ref = 10 * _ops.pointwise_loss_backward((10 * pred).detach(), 10 * tgt, "smoothl1", None,
                                            torch.ones((), device="cuda"))
    assert torch.equal(pred.grad, ref.reshape(pred.shape))


@pytest.mark.gpu
def test_torch_compile_render_rays_val():
    """torch.compile(render_rays_val) with the aot_eager backend: every pcnerf stage appears as a graph node (no
    fallback to untraced Python for them) and the depths equal the eager call's bit for bit."""
    from nof import synthetic as syn
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_val
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(1234)).cuda().eval()
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(5678)).cuda().eval()
    emb = Embedding(3, 10)
    rays = torch.from_numpy(syn.make_rays(300, seed=5)).cuda()
    seen = []

    def backend(gm, example_inputs):
        seen.extend(str(n.target) for n in gm.graph.nodes if n.op == "call_function")
        return torch._dynamo.lookup_backend("aot_eager")(gm, example_inputs)

    def fn(r):
        return render_rays_val(mc, mf, emb, r, N_samples=64, N_importance=128, perturb=0, noise_std=0, chunk=32768)

    torch._dynamo.reset()
    with torch.no_grad():
        want = fn(rays)
        got = torch.compile(fn, backend=backend)(rays)
    for k in ("depth", "depth_fine"):
        assert torch.equal(got[k], want[k]), k
    for op in ("sample_coarse", "pack_eval", "query_eval", "composite", "resample"):
        assert any(f"pcnerf.{op}" in s for s in seen), (op, sorted(set(seen)))


def test_param_shapes_match_module():
    """pcnerf::pack_eval's shape check is the module's own layout (models.py), tensor for tensor."""
    from nof.networks import NOF_coarse
    got = [tuple(t.shape) for t in T.eval_params(NOF_coarse())]
    assert got == T._param_shapes() and len(got) == 50


@pytest.mark.gpu
def test_operators_reject_bad_layouts():
    """The public operators check on the host what their kernels' grids and reads assume: wrong shapes, strides,
    dtypes or image sizes raise before any launch."""
    from nof import synthetic as syn
    from nof.networks import NOF_coarse
    P = torch.ops.pcnerf
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(7)).cuda().eval()
    params = T.eval_params(mc)
    packed = P.pack_eval(params)
    rays = torch.from_numpy(syn.make_rays(64, seed=3)).cuda()
    z = torch.linspace(1, 20, 32, device="cuda").expand(64, 32).contiguous()
    assert P.query_eval(rays, z, packed).shape == (64, 32)
    with pytest.raises(RuntimeError, match="contiguous"):
        P.query_eval(rays, z.t().contiguous().t(), packed)
    with pytest.raises(RuntimeError, match="expected"):
        P.query_eval(rays[:63].contiguous(), z, packed)
    with pytest.raises(RuntimeError, match="pack_eval's image"):
        P.query_eval(rays, z, packed[:-1].contiguous())
    bad = list(params)
    bad[4] = torch.zeros(256, 256, device="cuda")   # the skip layer takes 319 inputs
    with pytest.raises(RuntimeError, match="expected"):
        P.pack_eval(bad)


@pytest.mark.gpu
def test_tensor_operators_reject_mismatched_operands():
    """Each tensor-level operator checks its operands' rows / shapes / contiguity on the host before the launch."""
    P = torch.ops.pcnerf
    dev = "cuda"
    rays = torch.rand(32, 15, device=dev) + 1.0
    z = torch.sort(torch.rand(32, 16, device=dev) * 10 + 1, dim=1).values.contiguous()
    p = torch.rand(32, 16, device=dev)
    with pytest.raises(RuntimeError, match="expected"):
        P.perturb(z, 1.0, torch.rand(32, 15, device=dev))
    with pytest.raises(RuntimeError, match="expected"):
        P.resample(z, p[:, :15].contiguous(), 8, None)
    with pytest.raises(RuntimeError, match="expected"):
        P.composite(p[:31].contiguous(), z, None, 0.0, 1e-10, rays, 10, 11, 14, True)
    with pytest.raises(RuntimeError, match="expected"):
        P.composite(p, z, None, 0.0, 1e-10, rays[:31].contiguous(), 10, 11, 14, True)
    with pytest.raises(RuntimeError, match="contiguous"):
        P.composite(p.t().contiguous().t(), z, None, 0.0, 1e-10, rays, 10, 11, 14, True)
    with pytest.raises(RuntimeError, match="expected"):
        P.view_rows(p, z, rays[:, :7].contiguous(), 2, 1e-10)
    w, d, fr, sl = P.composite(p, z, None, 0.0, 1e-10, rays, 10, 11, 14, True)
    with pytest.raises(RuntimeError, match="expected"):
        P.child_losses(fr, sl[:31].contiguous(), rays, False, 4)
    assert P.resample(z, w, 8, None).shape == (32, 24)
