"""Generate the golden vectors under tests/golden/ by importing the reference (``/root/reference/nof``) on CPU.

Run in the build container only (the reference does not travel to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it pins: Embedding + NOF eval/train forward, render_rays_val, render_rays_train in the
PC-NeRF / OriginalNeRF configurations (child losses on/off, segmented sampling on/off, per-child divide on/off,
perturbation with recorded RNG draws), sample_pdf incl. the denom<1e-5 branch, the two-step
render_rays_view_0525_2_2 (methods 0 and 2), and the range loss of ``train_kitti.py:121-155`` computed with the
reference's own ``nof.criteria`` loss classes.

Only one shim is applied: ``nof/render.py:397`` moves ``u`` to ``"cuda:0"``; on this CPU-only container that
device move is turned into a no-op so the identical arithmetic runs on CPU.

Inputs are synthetic (checkpoints and child-AABB clouds are absent from the reference): weights come from
``nof.synthetic.init_nof_params(seed)`` and rays from ``nof.synthetic.make_rays`` -- both reproducible from the
seeds stored in each fixture; the rays themselves are also stored so the fixtures stand alone.
"""
import importlib.util
import os
import sys

import json
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

# our synthetic-data module, loaded by path (our package is also called ``nof``)
_spec = importlib.util.spec_from_file_location("pcnerf_synthetic", os.path.join(REPO, "pc-nerf_amd", "nof", "synthetic.py"))
syn = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(syn)

sys.path.insert(0, REF)
import nof.render as R  # noqa: E402  (the reference)
from nof.networks import Embedding, NOF_coarse, NOF_fine  # noqa: E402
from nof.criteria import nof_loss  # noqa: E402

_orig_to = torch.Tensor.to


def _to_shim(self, *a, **k):  # render.py:397 ``u.to("cuda:0")`` -> stay on CPU
    if a and isinstance(a[0], str) and a[0].startswith("cuda"):
        return self
    return _orig_to(self, *a, **k)


torch.Tensor.to = _to_shim
torch.set_num_threads(1)

SEED_C, SEED_F = 1234, 5678


def models(train):
    emb = Embedding(3, 10)
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(SEED_C))
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(SEED_F))
    mc.train(train)
    mf.train(train)
    return emb, mc, mf


def running_stats(m):
    out = []
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            out.append(torch.stack([mod.running_mean, mod.running_var]))
    return torch.stack(out).numpy()


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print("wrote", path, sum(np.asarray(v).nbytes for v in arrs.values()), "bytes raw")


def t(x):
    return x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)


def gen_nof():
    rng = np.random.default_rng(7)
    pts = rng.uniform(syn.PARENT_LO, syn.PARENT_HI, size=(2048, 3)).astype(np.float32)
    emb, mc, _ = models(train=False)
    with torch.no_grad():
        e = emb(torch.from_numpy(pts))
        p = mc(e)
    save("nof_eval", points=pts, embedding=t(e), p=t(p), seed=SEED_C)

    pts = rng.uniform(syn.PARENT_LO, syn.PARENT_HI, size=(4096, 3)).astype(np.float32)
    emb, mc, _ = models(train=True)
    chunk = 1000
    out = []
    with torch.no_grad():
        for i in range(0, len(pts), chunk):  # render.py:47-50 chunk loop
            out.append(mc(emb(torch.from_numpy(pts[i:i + chunk]))))
    save("nof_train", points=pts, p=t(torch.cat(out)), chunk=chunk, running=running_stats(mc), seed=SEED_C)


def gen_val():
    for S, I, nr in ((64, 128, 256), (128, 256, 96)):
        rays = syn.make_rays(nr, seed=11)
        emb, mc, mf = models(train=False)
        with torch.no_grad():
            res = R.render_rays_val(mc, mf, emb, torch.from_numpy(rays), N_samples=S, N_importance=I,
                                    perturb=0, noise_std=0, chunk=4096)
        save(f"render_val_s{S}", rays=rays, N_samples=S, N_importance=I, chunk=4096,
             depth=t(res["depth"]), depth_fine=t(res["depth_fine"]))


TRAIN_CASES = {
    # name: (use_child_nerf_loss, issegmentated, use_child_nerf_divide, perturb, S, I, ratio)
    "pcnerf": (1, 1, 0, 0, 64, 128, 0.1),
    "pcnerf_noseg": (1, 0, 0, 0, 64, 128, 0.1),
    "pcnerf_divide": (1, 1, 1, 0, 64, 128, 0.1),
    "original": (0, 0, 0, 0, 64, 128, 0.1),
    "pcnerf_perturb": (1, 1, 0, 1, 64, 128, 0.1),
    "pcnerf_s128": (1, 1, 0, 0, 128, 256, 0.1),
}


def range_losses(depth, depth_fine, gt, rays, divide, sub_num, lam=1.0, lam_fine=1.0):
    """train_kitti.py:121-146 restated with the reference's own loss class (nof/criteria/loss.py:42-50)."""
    loss = nof_loss["smoothl1"]()
    if divide:
        lr = torch.tensor([0])
        lrf = torch.tensor([0])
        sub = rays[:, 9]
        for i in range(sub_num):
            m = torch.logical_and(sub > (i + 0.5), sub < (i + 1.5))
            if m.sum() >= 1:
                lr = lr + 1e-1 * lam * loss(1e1 * depth[m], 1e1 * gt[m])
                lrf = lrf + 1e-1 * lam_fine * loss(1e1 * depth_fine[m], 1e1 * gt[m])
        return lr, lrf
    return 1e-1 * lam * loss(1e1 * depth, 1e1 * gt), 1e-1 * lam * loss(1e1 * depth_fine, 1e1 * gt)


def gen_train():
    for name, (cl, seg, div, pert, S, I, ratio) in TRAIN_CASES.items():
        nr = 256 if S == 64 else 64
        rays = syn.make_rays(nr, seed=21)
        if name == "pcnerf_noseg":
            # shrink child intervals so some contain no coarse sample: exercises render.py:82-84 expand loop
            mid = 0.5 * (rays[:, 10] + rays[:, 11])
            rays[::3, 10] = mid[::3] - 0.02
            rays[::3, 11] = mid[::3] + 0.02
        emb, mc, mf = models(train=True)
        torch.manual_seed(99)
        # record the RNG draws in the order the reference consumes them (render.py:453,57,383,57)
        F = S + I
        g = torch.Generator().manual_seed(99)
        draws = {}
        if pert > 0:
            draws["perturb_rand"] = torch.rand((nr, S), generator=g).numpy()
            torch.randn((nr, S), generator=g)
            draws["u"] = torch.rand((nr, I), generator=g).numpy()
            torch.randn((nr, F), generator=g)
        with torch.no_grad():
            res = R.render_rays_train(mc, mf, emb, torch.from_numpy(rays), sub_nerf_test_num=32, N_samples=S,
                                      N_importance=I, perturb=pert, noise_std=0, chunk=4096, issegmentated=seg,
                                      childnerf_ratio=ratio, use_child_nerf_divide=div, use_child_nerf_loss=cl)
            gt = torch.from_numpy(rays[:, 14])
            lr, lrf = range_losses(res["depth"], res["depth_fine"], gt, torch.from_numpy(rays), div, 32)
            total = lr + lrf + 1e6 * res["child_free_loss_fine"] + 1e6 * res["child_free_loss"] + \
                1e5 * res["child_depth_loss_fine"] + 1e5 * res["child_depth_loss"]
        save(f"render_train_{name}", rays=rays, N_samples=S, N_importance=I, chunk=4096, sub_nerf_test_num=32,
             use_child_nerf_loss=cl, issegmentated=seg, use_child_nerf_divide=div, perturb=pert,
             childnerf_ratio=ratio, depth=t(res["depth"]), depth_fine=t(res["depth_fine"]),
             child_free_loss=t(res["child_free_loss"]), child_depth_loss=t(res["child_depth_loss"]),
             child_free_loss_fine=t(res["child_free_loss_fine"]),
             child_depth_loss_fine=t(res["child_depth_loss_fine"]),
             loss_range=t(lr), loss_range_fine=t(lrf), loss_total=t(total),
             running_c=running_stats(mc), running_f=running_stats(mf), **draws)


def gen_pdf():
    rng = np.random.default_rng(31)
    nr, nb = 64, 33
    bins = np.sort(rng.uniform(0, 30, size=(nr, nb)), axis=1).astype(np.float32)
    w = rng.uniform(0, 1, size=(nr, nb - 1)).astype(np.float32) ** 8
    w[::4, 5:20] = 0.0      # flat cdf runs: denom < 1e-5 branch (render.py:408)
    w[1::8] = 0.0           # all-zero rows
    w = (w / (w.sum(1, keepdims=True) + 1e-10)).astype(np.float32)
    with torch.no_grad():
        det = R.sample_pdf(torch.from_numpy(bins), torch.from_numpy(w), 96, det=True)
        torch.manual_seed(5)
        u = torch.rand((nr, 96))
        torch.manual_seed(5)
        rnd = R.sample_pdf(torch.from_numpy(bins), torch.from_numpy(w), 96, det=False)
    save("sample_pdf", bins=bins, weights=w, samples_det=t(det), u=t(u), samples_rand=t(rnd))


def gen_view():
    rows, other, ranges = syn.make_view_rows(48, seed=41)
    for method in (0, 2):
        emb, mc, mf = models(train=False)
        with torch.no_grad():
            res = R.render_rays_view_0525_2_2(mc, mf, emb, torch.from_numpy(rows), torch.from_numpy(other),
                                              N_samples=64, N_importance=128, perturb=0, noise_std=0,
                                              chunk=4096, depth_inference_method=method)
        save(f"render_view_m{method}", rows=rows, other=other, ranges=ranges, N_samples=64, N_importance=128,
             depth_inference_method=method,
             **{k: t(v) for k, v in res.items()})


def gen_view_kitti():
    """Config 5's path on real rows: the reference's render_rays_view_0525_2_2 (render.py:614-699, as
    eval_kitti_render.py:1148-1161 calls it) on the two-step test rows of the first KITTI fixture test frame
    (scene_rays.npz kitti_view_*, rebuilt bit for bit by nof.dataset on the GPU side), seeded eval-mode weights
    (the fixture checkpoint's seeds 11 / 12), 64/128 samples, methods 2 and 0; each run again at 4 torch threads
    (``alt_`` keys: the reference's own spread)."""
    sc = scene_rays()
    rows, other = sc["kitti_view_rows"], sc["kitti_view_other"]
    out = {"rows": rows, "other": other, "N_samples": 64, "N_importance": 128}
    for method in (2, 0):
        for threads, pre in ((1, ""), (4, "alt_")):
            torch.set_num_threads(threads)
            emb = Embedding(3, 10)
            mc = syn.load_into(NOF_coarse(), syn.init_nof_params(11)).eval()
            mf = syn.load_into(NOF_fine(), syn.init_nof_params(12)).eval()
            with torch.no_grad():
                res = R.render_rays_view_0525_2_2(mc, mf, emb, torch.from_numpy(rows), torch.from_numpy(other),
                                                  N_samples=64, N_importance=128, perturb=0, noise_std=0,
                                                  chunk=262144, depth_inference_method=method)
            for k in ("depth", "depth_fine", "points_inference", "points_inference_fine", "rays_effective_flag",
                      "rays_effective_flag_fine", "opacity", "opacity_fine"):
                out[f"{pre}m{method}_{k}"] = t(res[k])
    torch.set_num_threads(1)
    save("render_view_kitti", **out)


def gen_render_rays():
    rays = syn.make_rays(128, seed=51)
    for isval in (False, True):
        emb, mc, mf = models(train=False)
        with torch.no_grad():
            res = R.render_rays(mc, mf, emb, torch.from_numpy(rays[:, :8].copy()), N_samples=64, N_importance=128,
                                perturb=0, noise_std=0, chunk=4096, isval=isval)
        save(f"render_rays_isval{int(isval)}", rays=rays[:, :8].copy(), N_samples=64, N_importance=128,
             **{k: t(v) for k, v in res.items()})


def reference_functions():
    """The reference's ray/AABB primitives, executed from its own source text: the modules that define them
    (nof/dataset/ipb2dmapping.py, eval_kitti_render.py) import open3d/pcl at top level, which this image lacks,
    but the functions themselves only use numpy and sklearn's KDTree."""
    import ast
    from sklearn.neighbors import KDTree
    ns = {"np": np, "KDTree": KDTree}
    want = {"nof/dataset/ipb2dmapping.py": ("compute_far_bound", "compute_far_bound0406", "compute_far_bound0606",
                                            "find_aabb_box"),
            "eval_kitti_render.py": ("compute_far_bound0429", "ray_aabb_distances", "distance_to_ray")}
    for rel, names in want.items():
        src = open(os.path.join(REF, rel)).read()
        for node in ast.parse(src).body:
            if isinstance(node, ast.FunctionDef) and node.name in names:
                code = ast.get_source_segment(src, node).replace('    print("here")\n', "")
                exec(compile(code, rel, "exec"), ns)
    return ns


def gen_aabb():
    """Ray/AABB primitives on synthetic scenes: points on/inside child boxes seen from an origin, plus boxes the
    rays graze (edge/corner hits, the eval path's exactly-two-hits rule) and misses."""
    F = reference_functions()
    rng = np.random.default_rng(61)
    boxes = syn.make_children(200, seed=62, min_center_dist=2.0)
    lo = boxes[:, 0] - syn.AABB_GROW
    hi = boxes[:, 1] + syn.AABB_GROW
    centers = 0.5 * (boxes[:, 0] + boxes[:, 1])
    origin = np.array([0.3, -0.2, 0.1])
    n = 600
    cid = rng.integers(0, len(boxes), size=n)
    pts = rng.uniform(boxes[cid, 0] - 0.3, boxes[cid, 1] + 0.3)          # some outside every box
    pts[::7] = np.where(rng.random((len(pts[::7]), 3)) < 0.5, boxes[cid[::7], 0], boxes[cid[::7], 1])  # corners
    vec = pts - origin
    rng_ = np.linalg.norm(vec, axis=1)
    dirs = vec / rng_[:, None]
    bounds6 = np.concatenate([lo, hi], 1)
    inside, idx = [], []
    for q in pts:
        ok, k = F["find_aabb_box"](centers, bounds6, q)
        inside.append(ok)
        idx.append(-1 if k is None else k)
    pb = (syn.PARENT_LO, syn.PARENT_HI)
    parent_far = []
    for d in dirs:
        t = F["compute_far_bound"](origin, d, pb[1][0], pb[0][0], pb[1][1], pb[0][1], pb[1][2], pb[0][2])
        parent_far.append(np.nan if t is None else t)
    # face-hit tests against the point's own box and a random box
    other_box = rng.integers(0, len(boxes), size=n)
    f0606, f0429, f0406 = [], [], []
    for i in range(n):
        try:   # MaiCity's rule: the first two face hits; fewer than two raise IndexError in the reference
            a4, z4 = F["compute_far_bound0406"](origin, dirs[i], lo[cid[i]], hi[cid[i]])
            f0406.append([1.0, a4, z4])
        except IndexError:
            f0406.append([0.0, 0.0, 0.0])
        row = []
        for b in (cid[i], other_box[i]):
            hit, a, z = F["compute_far_bound0606"](origin, dirs[i], lo[b], hi[b])
            row += [float(hit), a, z]
            hit2, a2, z2 = F["compute_far_bound0429"](origin, dirs[i], lo[b], hi[b])
            f0429.append([float(hit2), a2, z2])
        f0606.append(row)
    slab = F["ray_aabb_distances"](origin, dirs, np.array(syn.PARENT_LO), np.array(syn.PARENT_HI))
    d2r = np.stack([F["distance_to_ray"](torch.from_numpy(origin), dirs[i], centers) for i in range(0, n, 37)])
    save("aabb_primitives", boxes=boxes, lo=lo, hi=hi, centers=centers, origin=origin, points=pts, cid=cid,
         other_box=other_box, find_inside=np.array(inside), find_idx=np.array(idx), parent_far=np.array(parent_far),
         f0606=np.array(f0606), f0429=np.array(f0429), f0406=np.array(f0406), slab=slab, d2r=d2r)


GRAD_CASES = {"pcnerf": (1, 1, 0), "divide": (1, 1, 1), "original": (0, 0, 0)}


def grad_summary(m, seed):
    """Full gradients of the small tensors; norm + 2048 fixed entries of each weight matrix."""
    out = {}
    rng = np.random.default_rng(seed)
    for k, p_ in m.named_parameters():
        gr = p_.grad.detach().numpy()
        if gr.size <= 512:
            out[k] = gr
        else:
            idx = rng.choice(gr.size, size=2048, replace=False)
            out[k + "@idx"] = idx
            out[k + "@val"] = gr.reshape(-1)[idx]
            out[k + "@norm"] = np.linalg.norm(gr.astype(np.float64))
    return out


def gen_grads():
    """Parameter gradients of the train_kitti.py:117-155 loss through render_rays_train (train-mode BN, several
    chunks), i.e. what loss.backward() produces in the reference's training step.  Each case is run at 1 torch
    thread and again at 4 (``alt:`` prefix): the reference's own spread under another summation order."""
    for name, (cl, seg, div) in GRAD_CASES.items():
        rays = syn.make_rays(96, seed=71)
        runs = []
        for threads in (1, 4):
            torch.set_num_threads(threads)
            emb, mc, mf = models(train=True)
            res = R.render_rays_train(mc, mf, emb, torch.from_numpy(rays), sub_nerf_test_num=32, N_samples=64,
                                      N_importance=128, perturb=0, noise_std=0, chunk=4096, issegmentated=seg,
                                      childnerf_ratio=0.1, use_child_nerf_divide=div, use_child_nerf_loss=cl)
            gt = torch.from_numpy(rays[:, 14])
            lr, lrf = range_losses(res["depth"], res["depth_fine"], gt, torch.from_numpy(rays), div, 32)
            total = lr + lrf + 1e6 * res["child_free_loss_fine"] + 1e6 * res["child_free_loss"] + \
                1e5 * res["child_depth_loss_fine"] + 1e5 * res["child_depth_loss"]
            total.sum().backward()
            out = {"c:" + k: v for k, v in grad_summary(mc, 81).items()}
            out.update({"f:" + k: v for k, v in grad_summary(mf, 82).items()})
            out["loss_total"] = t(total)
            runs.append(out)
        torch.set_num_threads(1)
        save(f"grads_{name}", rays=rays, use_child_nerf_loss=cl, issegmentated=seg, use_child_nerf_divide=div,
             **runs[0], **{"alt:" + k: v for k, v in runs[1].items() if not k.endswith("@idx")})


def grad_sample(m, seed, n=8192):
    """Every gradient of a NOF: tensors of <= 512 entries in full, each weight matrix by ``n`` fixed entries (the
    same indices for every run with the same seed) plus its float64 norm."""
    out = {}
    rng = np.random.default_rng(seed)
    for k, p_ in m.named_parameters():
        gr = p_.grad.detach().numpy()
        if gr.size <= 512:
            out[k] = gr
        else:
            idx = np.sort(rng.choice(gr.size, size=n, replace=False))
            out[k + "@idx"] = idx
            out[k + "@val"] = gr.reshape(-1)[idx]
            out[k + "@norm"] = np.linalg.norm(gr.astype(np.float64))
    return out


def _grads_chunk(rays, n_child, threads):
    """loss.backward() of train_kitti.py:117-155 (PC-NeRF shell settings, render.py:38-163 with the production
    chunk=262,144: one full coarse BatchNorm chunk and three fine ones at 64/128 samples) on torch CPU."""
    import time
    torch.set_num_threads(threads)
    emb, mc, mf = models(train=True)
    t0 = time.perf_counter()
    res = R.render_rays_train(mc, mf, emb, torch.from_numpy(rays), sub_nerf_test_num=n_child, N_samples=64,
                              N_importance=128, **PCNERF_TRAIN)
    gt = torch.from_numpy(rays[:, 14])
    lr, lrf = range_losses(res["depth"], res["depth_fine"], gt, torch.from_numpy(rays), 0, 0)
    total = lr + lrf + 1e6 * res["child_free_loss_fine"] + 1e6 * res["child_free_loss"] + \
        1e5 * res["child_depth_loss_fine"] + 1e5 * res["child_depth_loss"]
    total.sum().backward()
    print(f"grads at chunk 262144 ({threads} threads): {time.perf_counter() - t0:.1f} s")
    out = {"c:" + k: v for k, v in grad_sample(mc, 91).items()}
    out.update({"f:" + k: v for k, v in grad_sample(mf, 92).items()})
    out.update(loss_total=t(total), loss_range=t(lr), loss_range_fine=t(lrf), depth=t(res["depth"]),
               depth_fine=t(res["depth_fine"]), child_free_loss=t(res["child_free_loss"]),
               child_depth_loss=t(res["child_depth_loss"]), child_free_loss_fine=t(res["child_free_loss_fine"]),
               child_depth_loss_fine=t(res["child_depth_loss_fine"]))
    del res, total, mc, mf
    torch.set_num_threads(1)
    return out


def gen_grads_chunk():
    """Training-step gradients at the PRODUCTION BatchNorm chunk: 4,096 rays, 64/128 samples,
    chunk 262,144 -- config 2's synthetic rays (make_rays(4096, seed=73)) and config 3's KITTI fixture rays
    (scene_rays.npz kitti_train).  Each is run twice, at 8 and at 3 torch threads (the reference's own spread under
    a different summation order), and both runs are stored (``alt:`` prefix for the second)."""
    sc = scene_rays()
    cases = {"grads_chunk_config2": (syn.make_rays(4096, seed=73), 32),
             "grads_chunk_kitti": (sc["kitti_train"], int(sc["kitti_children"]))}
    for name, (rays, n_child) in cases.items():
        a = _grads_chunk(rays, n_child, 8)
        b = _grads_chunk(rays, n_child, 3)
        save(name, rays=rays, sub_nerf_test_num=n_child, N_samples=64, N_importance=128, chunk=262144, **a,
             **{"alt:" + k: v for k, v in b.items() if not k.endswith("@idx")})


METRIC_SCENES = {"kitti":("logs/kitti00/1151_1200_view/render_result", range(1150, 1200)),
                 "maicity": ("logs/maicity00/maicity_00_1/render_result", range(0, 50))}


def raw_pcd(path):
    """Independent minimal reader for the reference's binary xyz float32 PCDs (checks nof.io.read_pcd)."""
    b = open(path, "rb").read()
    i = b.index(b"DATA binary\n") + len(b"DATA binary\n")
    n = int([ln for ln in b[:i].decode().splitlines() if ln.startswith("POINTS")][0].split()[1])
    return np.frombuffer(b[i:i + 12 * n], dtype="<f4").reshape(n, 3).copy()


def gen_metrics():
    """print_metrics.py:54-133 over the reference's committed rendered / source PCDs (two versions x one/two-step
    x every test frame, both scenes), computed by the cKDTree oracle; plus one KITTI frame's clouds as the GPU
    fixture."""
    sys.path.append(REPO)
    from oracle import metrics_cpu as M
    out = {}
    for scene, (rel, frames) in METRIC_SCENES.items():
        base = os.path.join(REF, rel)
        for ver in ("version_0", "version_1"):
            for kind in ("one_step", "two_step"):
                rows = {}
                for j in frames:
                    if (j + 1 - 3) % 5 != 0:
                        continue
                    f = j + 1
                    gt = raw_pcd(f"{base}/source/{f}_source.pcd")
                    org = raw_pcd(f"{base}/source/{f}_pose.pcd").reshape(-1)
                    pred = raw_pcd(f"{base}/infer/{ver}_{f}_{kind}.pcd")
                    rows[str(f)] = M.frame_metrics(pred, gt, org, 0.2)
                avg = np.mean(np.array(list(rows.values())), 0).tolist()
                out[f"{scene}/{ver}/{kind}"] = {"frames": rows, "mean": avg}
    with open(os.path.join(HERE, "metrics_reference.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    base = os.path.join(REF, METRIC_SCENES["kitti"][0])
    save("metrics_frame", gt=raw_pcd(f"{base}/source/1153_source.pcd"),
         origin=raw_pcd(f"{base}/source/1153_pose.pcd").reshape(-1),
         pred=raw_pcd(f"{base}/infer/version_1_1153_two_step.pcd"),
         expected=np.array(out["kitti/version_1/two_step"]["frames"]["1153"]))
    print("metrics", {k: [round(x, 4) for x in v["mean"]] for k, v in out.items()})


def gen_kitti_frames(step=40):
    """Scene fixture for the dataset pipeline (nof/dataset.py): KITTI-00 scans 1151..1156 of the reference's
    data/kitti/00/pcd_remove_dynamic (every ``step``-th point, float32 as stored) and poses.txt rows 1150..1156."""
    frames = {f"f{f}": raw_pcd(os.path.join(REF, f"data/kitti/00/pcd_remove_dynamic/{f}.pcd"))[::step]
              for f in range(1151, 1157)}
    with open(os.path.join(REF, "data/kitti/00/poses.txt")) as fh:
        rows = [ln.strip() for ln in fh if ln.strip()]
    poses = np.array([[float(v) for v in rows[i].split(" ")] for i in range(1150, 1157)])
    save("kitti_frames", poses=poses, pose_first=np.array(1150), **frames)


def gen_maicity_frames(step=40):
    """MaiCity-00 scans 1..6 of the reference's data/maicity/00/pcd (every ``step``-th point) and poses.txt rows
    0..6, for maicity_dataload."""
    frames = {f"f{f}": raw_pcd(os.path.join(REF, f"data/maicity/00/pcd/{f}.pcd"))[::step] for f in range(1, 7)}
    with open(os.path.join(REF, "data/maicity/00/poses.txt")) as fh:
        rows = [ln.strip() for ln in fh if ln.strip()]
    poses = np.array([[float(v) for v in rows[i].split(" ")] for i in range(0, 7)])
    save("maicity_frames", poses=poses, **frames)


def gen_pdf_pytest():
    """sample_pdf(..., pytest=True) (render.py:386-394): numpy-seeded u, det and random, on gen_pdf's inputs."""
    rng = np.random.default_rng(31)
    nr, nb = 64, 33
    bins = np.sort(rng.uniform(0, 30, size=(nr, nb)), axis=1).astype(np.float32)
    w = rng.uniform(0, 1, size=(nr, nb - 1)).astype(np.float32) ** 8
    w = (w / (w.sum(1, keepdims=True) + 1e-10)).astype(np.float32)
    with torch.no_grad():
        det = R.sample_pdf(torch.from_numpy(bins), torch.from_numpy(w), 96, det=True, pytest=True)
        rnd = R.sample_pdf(torch.from_numpy(bins), torch.from_numpy(w), 96, det=False, pytest=True)
    save("sample_pdf_pytest", bins=bins, weights=w, samples_det=t(det), samples_rand=t(rnd))


PCNERF_TRAIN = dict(use_child_nerf_loss=1, issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0, perturb=0,
                    noise_std=0, chunk=262144)   # shells/pretraining/*_pcnerf_train.bash (perturb 0: deterministic)


def train_outputs(res, rays, mc, mf):
    gt = torch.from_numpy(rays[:, 14])
    lr, lrf = range_losses(res["depth"], res["depth_fine"], gt, torch.from_numpy(rays), 0, 0)
    total = lr + lrf + 1e6 * res["child_free_loss_fine"] + 1e6 * res["child_free_loss"] + \
        1e5 * res["child_depth_loss_fine"] + 1e5 * res["child_depth_loss"]
    return dict(depth=t(res["depth"]), depth_fine=t(res["depth_fine"]), child_free_loss=t(res["child_free_loss"]),
                child_depth_loss=t(res["child_depth_loss"]), child_free_loss_fine=t(res["child_free_loss_fine"]),
                child_depth_loss_fine=t(res["child_depth_loss_fine"]), loss_range=t(lr), loss_range_fine=t(lrf),
                loss_total=t(total), running_c=running_stats(mc), running_f=running_stats(mf))


def gen_config2_full(threads=None, name="config2_full"):
    """BASELINE config 2 at its full size: 65,536 rays of nof.synthetic.make_rays(65536, seed=0) (regenerated from the
    seed by the test; only outputs are stored), 128/256 samples, train-mode BatchNorm over 262,144-sample chunks
    (32 coarse + 96 fine chunks), child losses, segmented sampling 0.1, perturb 0."""
    import time
    torch.set_num_threads(threads or os.cpu_count() or 1)
    rays = syn.make_rays(65536, seed=0)
    emb, mc, mf = models(train=True)
    t0 = time.perf_counter()
    with torch.no_grad():
        res = R.render_rays_train(mc, mf, emb, torch.from_numpy(rays), sub_nerf_test_num=32, N_samples=128,
                                  N_importance=256, **PCNERF_TRAIN)
    print("config2 full:", time.perf_counter() - t0, "s")
    save(name, n_rays=65536, seed=0, N_samples=128, N_importance=256, threads=torch.get_num_threads(),
         **train_outputs(res, rays, mc, mf))
    torch.set_num_threads(1)


def scene_rays():
    return dict(np.load(os.path.join(HERE, "scene_rays.npz"), allow_pickle=False))


def gen_config1_kitti(threads=1, name="config1_kitti"):
    """BASELINE config 1: a 4,096-ray batch of KITTI-00 rays (scene_rays.npz, made by make_scene_rays.py from the
    fixture frames) through render_rays_train at 64/128 samples with the PC-NeRF KITTI shell's settings (one
    262,144-sample coarse chunk, three fine chunks), and the val split through render_rays_val (eval mode)."""
    sc = scene_rays()
    rays = sc["kitti_train"]
    n_child = int(sc["kitti_children"])
    torch.set_num_threads(threads)
    emb, mc, mf = models(train=True)
    with torch.no_grad():
        res = R.render_rays_train(mc, mf, emb, torch.from_numpy(rays), sub_nerf_test_num=n_child, N_samples=64,
                                  N_importance=128, **PCNERF_TRAIN)
    out = train_outputs(res, rays, mc, mf)
    emb, mc, mf = models(train=False)
    val = sc["kitti_val"]
    with torch.no_grad():
        rv = R.render_rays_val(mc, mf, emb, torch.from_numpy(val), N_samples=64, N_importance=128, perturb=0,
                               noise_std=0, chunk=262144)
    save(name, N_samples=64, N_importance=128, sub_nerf_test_num=n_child, threads=threads, **out,
         val_depth=t(rv["depth"]), val_depth_fine=t(rv["depth_fine"]))
    torch.set_num_threads(1)


# BASELINE config 3 (KITTI-00 frames 1151-1200 at 50 % frame sparsity, 262,144 rays): tests/golden/make_config3_full.py
# (its ``ref`` step imports this module for the reference's render_rays_train and these helpers)


def gen_config4_maicity(threads=1, name="config4_maicity"):
    """BASELINE config 4: MaiCity-00 split into 4 parent blocks, each with its own coarse/fine NOF (seeds
    1234+b / 5678+b), up to 1,024 rows per block through render_rays_train at 128/256 samples."""
    sc = scene_rays()
    out = {}
    torch.set_num_threads(threads)
    for b in range(4):
        rays = sc[f"maicity_b{b}"]
        emb = Embedding(3, 10)
        mc = syn.load_into(NOF_coarse(), syn.init_nof_params(SEED_C + b)).train()
        mf = syn.load_into(NOF_fine(), syn.init_nof_params(SEED_F + b)).train()
        with torch.no_grad():
            res = R.render_rays_train(mc, mf, emb, torch.from_numpy(rays), sub_nerf_test_num=int(sc[f"maicity_b{b}_children"]),
                                      N_samples=128, N_importance=256, **PCNERF_TRAIN)
        out.update({f"b{b}_{k}": v for k, v in train_outputs(res, rays, mc, mf).items()})
    save(name, N_samples=128, N_importance=256, threads=threads, **out)
    torch.set_num_threads(1)


def gen_self_spread():
    """The reference against ITSELF: configs 1, 4 and 2 rerun with another torch thread count (different BLAS
    blocking, so different float32 rounding; same inputs and weights).  Its fine depths move by up to ~7e-4
    relative at KITTI ranges (render.py's fine samples sit where the high-frequency encoding turns an ulp of
    position into ~1e-4 of occupancy), which is the floor any float32 reimplementation's parity sits on; the GPU
    tests hold the HIP path to that spread (tests/test_configs_gpu.py)."""
    gen_config1_kitti(threads=8, name="config1_kitti_alt")
    gen_config4_maicity(threads=8, name="config4_maicity_alt")
    gen_config2_full(threads=3, name="config2_full_alt")


GENERATORS = [gen_maicity_frames, gen_kitti_frames, gen_metrics, gen_grads, gen_aabb, gen_render_rays, gen_nof,
              gen_pdf, gen_val, gen_train, gen_view, gen_pdf_pytest, gen_config1_kitti, gen_config4_maicity,
              gen_config2_full, gen_self_spread, gen_grads_chunk, gen_view_kitti]

if __name__ == "__main__":
    # python make_golden.py [name ...]  (names without the gen_ prefix; default: all)
    want = set(sys.argv[1:])
    for fn in GENERATORS:
        if not want or fn.__name__[4:] in want:
            fn()
