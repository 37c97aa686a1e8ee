"""Benchmark: LiDAR rays/s (render + loss) at 128 samples/ray on MI355X -- BASELINE.json config 2 by default.

Default (--config 2, --mode train_fwd): one step = the reference training step's forward on one batch
(train_kitti.py:117-155 without backward): ``render_rays_train`` (train-mode BatchNorm over 262,144-sample chunks,
segmented sampling ratio 0.1, child free/depth losses, perturb 1, noise_std 0) over 65,536 synthetic rays of one
parent block with 32 child AABBs at N_samples=128 / N_importance=256 (512 MLP samples per ray), plus the SmoothL1
range losses and the weighted total loss.  Inputs are resident in HBM before timing starts.
--mode train_step adds what Lightning does with that loss: loss.backward() through the HIP backward kernels and
the reference's optimizer step (Adam lr 5e-4, eps 1e-8, weight_decay 1e-3 over both networks, nof_utils.py:162-173).
--mode val: render_rays_val (eval BN).  --mode view: two-step inference (render_rays_view_0525_2_2, method 2) on
13-column rows grouped per LiDAR ray; value counts LiDAR rays (groups).

The other BASELINE configs (--config):
  3  KITTI-00 training loop: train_step at 262,144 rays/iter and 64/128 samples on frames 1151-1200 at 50 % frame
     sparsity (nof.dataset on tests/golden/kitti_frames_full.npz, batch drawn with replacement); with N GPUs each rank takes
     262,144 rays of a data-parallel step and the gradients are averaged over RCCL (nof.blocks.allreduce_grads);
  4  MaiCity-00 bounds split into 4 parent blocks (own weights, 262,144 rays each, 128/256 samples), train_fwd,
     blocks dealt over the ranks, every block's depths gathered to rank 0 over RCCL (strong scaling: 1M rays/iter);
  5  8 parent blocks of two-step rows (view mode, 16,384 ray groups each), gathered to rank 0 (strong scaling).

Multi-GPU: ``python bench.py --gpus N`` (no WORLD_SIZE in the environment) starts
``python -m torch.distributed.run --nproc-per-node N`` on this same command line before anything touches the GPU
and relays rank 0's line; under an external torchrun ``--gpus`` must equal WORLD_SIZE.  One process per GPU over
RCCL; the timed region is bracketed by barriers and the time is the max over ranks.  ``--dry-run`` exercises the
launcher and the distributed timing on CPU (gloo), with no GPU.

The default run (N=1, config 2, train_fwd) also times, in the same process and as extra keys of its one line, the
training step (``train_step``: config 2 with backward + Adam), the reference's own shell setting of it
(``train_step_refcfg``: 256 rays at 768 + 1536 samples, chunk 262,144, shells/pretraining/KITTI00_pcnerf_train.bash),
BASELINE configs 3 (``config3``) and 4 (``config4``, all four MaiCity blocks on the one GPU), ``val`` and the
two-step ``view``, each with its own ms_per_step, roofline, cpu_baseline and cd_vs_ref (--no-extra
skips them), and measures what the fp16 matrix pipe sustains on the board (``mfma_ceiling_measured``, 1 s).

Prints ONE compact JSON line (rank 0, the last stdout line, <= 4 KB) with the throughput, the dominant kernel's
roofline (HIP events over the timed region, on the kernels' own stream; ``achieved`` = the algorithmic fp32 FLOP rate,
``frac_issued`` the split products' rate), a CPU baseline (the CPU oracle on a 2,048-ray sample, rank 0 at N=1 only),
a one-line summary per extra line and, at N > 1, the rank report (backend, ranks seen, per-rank rays / ms /
collective ms).  Every line in full (per-kernel tables, fp32-MFMA comparison) goes to ``--detail``.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "pc-nerf_amd"))
sys.path.insert(0, HERE)

FP32_MFMA_PEAK_TFLOPS = 157.3  # /opt/skills/guides/MI355X_MICROARCH.md (F32 MFMA = vector peak, no xf32)
HBM_PEAK_GBS = 8000.0          # same guide (spec)
MODE_OF_CONFIG = {2: "train_fwd", 3: "train_step", 4: "train_fwd", 5: "view"}
# one CPU-baseline sample size for every ray line (256- and 4,096-ray samples of the same per-ray
# workload measured 3.1x apart); the whole line when it is smaller (the reference shell's 256 rays)
CPU_SAMPLE_RAYS = 2048


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=2)
    ap.add_argument("--mode", choices=["train_fwd", "train_step", "val", "view"], default=None,
                    help="default: the config's workload (2: train_fwd, 3: train_step, 4: train_fwd, 5: view)")
    ap.add_argument("--rays", type=int, default=None,
                    help="LiDAR rays per block (default 65,536; config 3: 262,144 per GPU; config 4: 262,144; "
                         "view: 16,384 ray groups = ~52k two-step rows)")
    ap.add_argument("--samples", type=int, default=None, help="N_samples (default 128; config 3: 64)")
    ap.add_argument("--importance", type=int, default=None, help="N_importance (default 2 x N_samples)")
    ap.add_argument("--chunk", type=int, default=262144)
    ap.add_argument("--cpu-rays", type=int, default=None,
                    help="bounded CPU-baseline sample (rays; default %d on every line, or the whole line when "
                         "smaller; ray groups for view)" % CPU_SAMPLE_RAYS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32-line", action="store_true",
                    help="skip the comparison run of the train lines under the fp32 MFMA train math (profiling)")
    ap.add_argument("--fold", action="store_true",
                    help="the opt-in exact affine fold (SURVEY fact 1): eval modes fold the eval network, train modes "
                         "the train-mode network per BatchNorm chunk (forward and backward); reported as its own "
                         "line, never the headline")
    ap.add_argument("--gather", action="store_true",
                    help="gather every block's depth_fine to rank 0 inside each step (eval-driver output path; on "
                         "by default for configs 4 and 5)")
    ap.add_argument("--no-extra", action="store_true",
                    help="default run only: skip the extra lines (train_step, train_step_refcfg, val, view)")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the measured fp16 MFMA ceiling (1 s)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / distributed-timing check on CPU (gloo): no GPU, no render")
    ap.add_argument("--detail", default=os.path.join(HERE, "gpurun_out", "bench_detail.json"),
                    help="file for every line in full (kernel tables, fp32-MFMA comparison); '' for none. stdout "
                         "carries only the compact line (<= 4 KB)")
    a = ap.parse_args(argv)
    a.mode = a.mode or MODE_OF_CONFIG[a.config]
    if a.samples is None:
        a.samples = 64 if a.config == 3 else 128
    if a.importance is None:
        a.importance = 2 * a.samples
    if a.rays is None:
        a.rays = 16384 if a.mode == "view" else 262144 if a.config in (3, 4) else 65536
    if a.config in (4, 5):
        a.gather = True
    return a


# ----------------------------------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n: int, argv: list) -> int:
    """One process per GPU: torch.distributed.run as a CHILD process (this process has not touched the GPU and
    is not replaced); rank 0's JSON line reaches our stdout through the inherited descriptor."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def dry_run(a, world, rank):
    """The distributed skeleton of main() on CPU: gloo group, warmup, barrier-bracketed timed steps, max over
    ranks, rank 0's line -- what the launcher test checks without a GPU."""
    import torch.distributed as tdist
    from nof.blocks import blocks_of_rank, max_over_ranks
    dist = world > 1
    if dist:
        tdist.init_process_group("gloo")
    blocks = (list(range(8)) if a.config == 5 else    # config 5: every block, a row-balanced share of each
              blocks_of_rank(rank, world, world if a.config in (2, 3) else 4))
    x = torch.randn(256, 256)
    coll = [0.0, False]

    def step():
        y = (x @ x).sum().reshape(1)
        if dist and coll[1]:   # the step's collective, timed as the GPU run times its gather / all-reduce
            t = time.perf_counter()
            tdist.all_reduce(y)
            coll[0] += time.perf_counter() - t
        return y

    for _ in range(a.warmup):
        step()
    if dist:
        tdist.barrier()
    coll[1] = True
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    local = time.perf_counter() - t0
    if dist:
        tdist.barrier()
    elapsed = max_over_ranks(local)
    info = None
    if dist:
        info = rank_report(tdist, torch.device("cpu"), 256 * len(blocks), local, 1e3 * coll[0], a.steps)
    if rank == 0:
        print(json.dumps({"metric": "launcher dry run", "value": a.steps / elapsed, "unit": "steps/s",
                          "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "dry_run": True,
                          "rank0_blocks": blocks, "dist": info,
                          "config": {"workload": f"config {a.config} dry run"}}), flush=True)
    if dist:
        tdist.destroy_process_group()


# ----------------------------------------------------------------------------------------------- profiling
def prof_read(L, tag):
    t, n, f, b = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
    rc = L.pcnerf_prof_read(tag, ctypes.byref(t), ctypes.byref(n), ctypes.byref(f), ctypes.byref(b))
    if rc:
        raise RuntimeError(L.pcnerf_last_error().decode())
    return t.value, n.value, f.value, b.value


def pmc_traffic(kernel_name: str, line: str = None):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json) and
    where they come from (profile file + the commit it was measured at), or (None, None).  ``line``: the bench line
    whose profile to prefer (``<kernel>@<line>`` entries: the same kernel moves different bytes in different lines,
    e.g. the train query with and without the activation store)."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None
    ks = d.get("kernels", d)
    # a line with its own name (train_step_refcfg, config3) takes only its own profile's entry; the mode-named lines
    # the kernel's entry
    if line in EXTRA_LINES and EXTRA_LINES[line].get("line") == line:
        v = ks.get(f"{kernel_name}@{line}", {})
    else:
        v = ks.get(f"{kernel_name}@{line}") or ks.get(kernel_name, {}) if line else ks.get(kernel_name, {})
    meta = d.get("_meta", {})
    return v.get("hbm_bytes_per_launch"), ({"file": "profiles/pmc_traffic.json", "head": v.get("head", meta.get("head")),
                                            "profile": v.get("profile", meta.get("profile"))} if v else None)


# ----------------------------------------------------------------------------------------------- workloads
def write_kitti_fixture(tmp):
    """tests/golden/kitti_frames_full.npz (KITTI-00 scans 1151..1200, every 16th point, and their poses) as the
    reference's on-disk layout under ``tmp``: pcd/<frame>.pcd and poses.txt (identity rows before frame 1150)."""
    from nof import io as nio
    g = dict(np.load(os.path.join(HERE, "tests", "golden", "kitti_frames_full.npz"), allow_pickle=False))
    os.makedirs(os.path.join(tmp, "pcd"), exist_ok=True)
    for k, v in g.items():
        if k.startswith("f"):
            nio.write_pcd(os.path.join(tmp, "pcd", f"{k[1:]}.pcd"), v)
    with open(os.path.join(tmp, "poses.txt"), "w") as fh:
        for _ in range(int(g["pose_first"])):
            fh.write("1 0 0 0 0 1 0 0 0 0 1 0\n")
        for row in g["poses"]:
            fh.write(" ".join(repr(float(v)) for v in row) + "\n")
    return os.path.join(tmp, "pcd"), os.path.join(tmp, "poses.txt")


# BASELINE config 5: KITTI-00 frames 1150..1198 as 8 contiguous parent blocks of 6 frames (the fixture holds one
# 50-frame sequence), each with its own parent box and child boxes; the held-out frames at 80 % frame sparsity
# (eval_kitti_render.py:1060) rendered by the two-step path
C5_START, C5_FRAMES, C5_BLOCKS, C5_SPARSITY = 1150, 6, 8, 80


def eval_opts(root, pose_path, ds, de, samples=128, importance=256, chunk=262144, extra=""):
    """eval_kitti_render.get_opts with the KITTI eval shell's settings (shells/pretraining/KITTI00_pcnerf_eval.bash:
    range_delete 2/1/0.5, over_height 0.168, over_low -2, interest 20 x 20, skip connection, method 2)."""
    import eval_kitti_render as E
    return E.get_opts(f"""--dataset kitti --root_dir {root} --pose_path {pose_path} --data_start {ds} --data_end {de}
        --depth_inference_method 2 --test_data_create 1 --N_samples {samples} --N_importance {importance}
        --chunk {chunk} --range_delete_x 2 --range_delete_y 1 --range_delete_z 0.5 --over_height 0.168
        --over_low -2 --interest_x 20 --interest_y 20 --use_skip {extra}""".split())


def kitti_view_blocks(dev, blocks=None):
    """Config 5's rows: for each parent block b (frames C5_START + 6 b + 1 .. + 6) the eval driver's scene (parent
    cloud of the block's frames, its child boxes, eval_kitti_render.Scene) and the two-step rows (method 2) of the
    block's held-out frames at 80 % sparsity, built on the GPU (nof.raytable) and concatenated frame after frame
    (whole ray groups).  -> [{block, rows, other, ranges, frames, groups}]."""
    import tempfile
    import eval_kitti_render as E
    out = []
    with tempfile.TemporaryDirectory() as tmp:
        root, poses = write_kitti_fixture(tmp)
        for b in (range(C5_BLOCKS) if blocks is None else blocks):
            ds = C5_START + C5_FRAMES * b
            h = eval_opts(root, poses, ds, ds + C5_FRAMES)
            scene = E.Scene(h, dev)
            frames = E.test_frame_ids(ds, ds + C5_FRAMES, C5_SPARSITY)
            parts = [scene.view_rows(f, 2) for f in frames]
            rows = torch.cat([p[0] for p in parts])
            out.append(dict(block=b, rows=rows, ranges=torch.cat([p[1] for p in parts]),
                            other=torch.cat([p[2] for p in parts]), frames=frames,
                            groups=int((rows[:, 12] >= -0.5).sum()), children=int(scene.bounds6.shape[0]),
                            parent6=scene.parent6))
    return out


def kitti_fixture_rays(dev):
    """BASELINE config 3's scene: KITTI-00 scans 1151..1200 (tests/golden/kitti_frames_full.npz, every 16th point)
    at the 50 % frame-sparsity rule (25 train frames, 157,108 rows), its train rays built on the GPU by nof.dataset
    exactly as the parity test builds them (tests/golden/make_config3_full.py)."""
    import tempfile
    from nof import dataset as D
    sc = dict(np.load(os.path.join(HERE, "tests", "golden", "config3_full_scene.npz"), allow_pickle=False))
    with tempfile.TemporaryDirectory() as tmp:
        write_kitti_fixture(tmp)
        ds = D.kitti_dataload(os.path.join(tmp, "pcd"), split="train", data_start=int(sc["data_start"]),
                              data_end=int(sc["data_end"]), cloud_size_val=64, range_delete_x=3, range_delete_y=2,
                              range_delete_z=1.25, sub_nerf_test_num=0, surface_expand=0.05, over_height=0.168,
                              over_low=-2.0, interest_x=20.0, interest_y=20.0, pose_path=os.path.join(tmp, "poses.txt"),
                              re_loaddata=1, result_path=os.path.join(tmp, "out"), device=dev,
                              sparsity=int(sc["sparsity"]))
    return ds.rays, int(sc["children"])


def make_blocks(a, rank, world, dev, syn):
    """This rank's work: a list of parent blocks, each {rays, other, gt, seeds, sub_num}.  Config 5 (the two-step
    inference over 8 parent blocks): every rank holds all 8 blocks' weights (replicated) and renders a row-balanced
    share of WHOLE ray groups of each block (nof.blocks.split_groups), so no rank waits on a larger block."""
    from nof.blocks import blocks_of_rank, split_groups
    out = []
    if a.config == 5 and a.mode == "view":
        for kb in kitti_view_blocks(dev):
            b, vr = kb["block"], kb["rows"]
            s, e = split_groups(vr[:, 12].cpu().numpy(), world)[rank]
            out.append(dict(block=b, rays=vr[s:e].contiguous(), other=kb["other"][s:e].contiguous(),
                            gt=kb["ranges"][s:e].contiguous(), seeds=(1234 + b, 5678 + b),
                            sub_num=kb["children"], groups=int((vr[s:e, 12] >= -0.5).sum()), frames=kb["frames"]))
        return out
    if a.config == 3:
        scene, n_child = kitti_fixture_rays(dev)
        gen = torch.Generator(device=dev).manual_seed(rank)
        idx = torch.randint(0, scene.shape[0], (a.rays,), device=dev, generator=gen)
        rays = scene[idx].contiguous()
        return [dict(block=0, rays=rays, other=None, gt=rays[:, 14].contiguous(), seeds=(1234, 5678),
                     sub_num=n_child, scene=scene)]
    n_blocks = {2: world, 4: 4, 5: 8}[a.config]
    for b in blocks_of_rank(rank, world, n_blocks):
        seeds = (1234 + b, 5678 + b)
        if a.mode == "view":
            vr, vo, vg = syn.make_view_rows(a.rays, n_children=32, seed=1000 * b)
            out.append(dict(block=b, rays=torch.from_numpy(vr).to(dev), other=torch.from_numpy(vo).to(dev),
                            gt=torch.from_numpy(vg).to(dev), seeds=seeds, sub_num=32))
            continue
        if a.config == 4:
            lo, hi, origin = syn.block_bounds(b, 4)
            r = syn.make_rays(a.rays, n_children=256, seed=1000 * b, lo=lo, hi=hi, origin=origin)
            sub = 256
        else:
            r = syn.make_rays(a.rays, n_children=32, seed=1000 * b)
            sub = 32
        rays = torch.from_numpy(r).to(dev)
        out.append(dict(block=b, rays=rays, other=None, gt=rays[:, 14].contiguous(), seeds=seeds, sub_num=sub))
    return out


# The default N=1 run also times these lines in the same process, as extra keys of the one JSON line (the headline
# value stays the render+loss forward): the whole training step at config 2 and at the reference's own shell setting
# (shells/pretraining/KITTI00_pcnerf_train.bash:8-10: 256 rays, 768 + 1536 samples, chunk 262,144 -- the setting of
# the reference's published 779 rays/s), render_rays_val and the two-step inference.
EXTRA_LINES = {
    "train_step": dict(mode="train_step", rays=65536, samples=128, importance=256, cpu_rays=None),
    "train_step_refcfg": dict(mode="train_step", rays=256, samples=768, importance=1536, cpu_rays=None,
                              line="train_step_refcfg"),
    # BASELINE config 3: one training step of 262,144 KITTI-fixture rays at 64/128 (train_kitti.py:117-155; 256
    # BatchNorm chunks of 262,144 samples -- the reference's shell chunk)
    "config3": dict(config=3, mode="train_step", rays=262144, samples=64, importance=128, cpu_rays=None,
                    line="config3"),
    # BASELINE config 4: the MaiCity-00 split, 4 parent blocks with their own weights, 262,144 rays each at 128/256,
    # train_fwd -- on one GPU all four blocks, 1,048,576 rays per step
    "config4": dict(config=4, mode="train_fwd", rays=262144, samples=128, importance=256, cpu_rays=None,
                    line="config4"),
    # BASELINE config 5: the two-step inference of 8 KITTI parent blocks' held-out frames (80 % frame sparsity), all
    # eight on the one GPU (kitti_view_blocks)
    "config5": dict(config=5, mode="view", rays=16384, samples=128, importance=256, cpu_rays=None, line="config5"),
    "val": dict(mode="val", rays=65536, samples=128, importance=256, cpu_rays=None),
    "view": dict(mode="view", rays=16384, samples=128, importance=256, cpu_rays=None),
}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and a.gpus > 1:
        sys.exit(launch(a.gpus, argv))
    world = int(world_env or "1")
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} does not match WORLD_SIZE={world} of the launcher")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_run:
        return dry_run(a, world, rank)
    dist = dist_on(world)
    # test-only: PCNERF_BENCH_SHARE_GPU=1 puts every rank on cuda:0 with the gloo backend (RCCL needs one GPU per
    # rank), so the N-rank path runs on a one-GPU box (tests/test_dist_gpu.py); the driver's runs never set it
    share = os.environ.get("PCNERF_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        if share:
            tdist.init_process_group("gloo")
        else:
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    from nof import _hip
    L = _hip.lib()

    head = run_line(a, L, dev, rank, world)

    # what the fp16 matrix pipe sustains on this board, measured in this process
    ceiling = None
    if not a.no_ceiling:
        tf, mhz = ctypes.c_double(), ctypes.c_double()
        _hip.check(L.pcnerf_mfma_ceiling(1.0, ctypes.byref(tf), ctypes.byref(mhz),
                                         torch.cuda.current_stream(dev).cuda_stream))
        ceiling = {"TFLOPs": round(tf.value, 1), "clock_MHz": round(mhz.value), "seconds": 1.0,
                   "kernel": "bare v_mfma_f32_16x16x32_f16 loop, B from LDS, random fp16 operands, 1 wave/SIMD"}
    extras = {}
    if world == 1 and a.config == 2 and a.mode == "train_fwd" and not a.fold and not a.no_extra:
        for name, over in EXTRA_LINES.items():
            b = argparse.Namespace(**{**vars(a), **over, "no_fp32_line": True, "gather": False})
            extras[name] = run_line(b, L, dev, rank, world)
    if rank != 0:
        if dist:
            tdist.destroy_process_group()
        return
    line, detail = assemble(a, world, head, extras, ceiling, head.get("dist"))
    emit(line, detail, a.detail)
    if dist:
        tdist.destroy_process_group()


# ----------------------------------------------------------------------------------------------- the one line
LINE_MAX_BYTES = 4096   # the driver parses the LAST stdout line; round 5's 24.5 KB line was not parsed
REQUIRED_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                 "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "cd_vs_ref")
ROOF_KEYS = ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "avg_launch_us", "frac_issued",
             "frac_of_measured_ceiling")
CONFIG_KEYS = ("workload", "baseline_config", "rays_per_step", "N_samples", "N_importance", "chunk", "parallelism")


def _pick(d, keys):
    return None if d is None else {k: d[k] for k in keys if k in d}


def assemble(a, world, head, extras, ceiling, dist_info=None):
    """(compact line, detail): the compact line is what stdout carries (every key the contract names, each extra
    line summarised to value / ms / dominant kernel's frac / CPU baseline); the detail object holds every line in
    full -- per-kernel tables, fp32-MFMA comparison, PMC sources -- and goes to a file, never to stdout."""
    for ln in [head] + list(extras.values()):
        add_ceiling(ln["roofline"], ceiling)
        if ln.get("fp32_mfma"):
            add_ceiling(ln["fp32_mfma"]["roofline"], ceiling)
    full = line_json(a, world, head)
    full["mfma_ceiling_measured"] = ceiling
    if dist_info is not None:
        full["dist"] = dist_info
    detail = {"headline": full}
    for name, ln in extras.items():
        b = argparse.Namespace(**{**vars(a), **EXTRA_LINES[name]})
        detail[name] = line_json(b, world, ln)
    line = {k: full[k] for k in REQUIRED_KEYS}
    line["config"] = _pick(full["config"], CONFIG_KEYS)
    line["roofline"] = _pick(full["roofline"], ROOF_KEYS)
    line["cpu_baseline"] = _pick(full["cpu_baseline"], ("value", "unit", "cores", "kind", "sample"))
    line["cd_vs_ref"] = _pick(full["cd_vs_ref"], ("cd_m", "fscore", "max_rel_depth_err", "flags_equal", "rays"))
    if dist_info is not None:
        line["dist"] = dist_info
    line["loss"] = full["loss"]
    if ceiling:
        line["mfma_ceiling_TFLOPs"] = ceiling["TFLOPs"]
    # the last step carries two HIP events per launch: its kernel sum exceeds a plain step by their cost
    line["kernels_step_ms_instrumented"] = full["kernels_step_ms"]
    if extras:
        line["extras"] = {}
        for name, e in detail.items():
            if name == "headline":
                continue
            r, cb = e["roofline"] or {}, e["cpu_baseline"]
            line["extras"][name] = {"value": e["value"], "ms_per_step": e["ms_per_step"],
                                    "rays_per_step": e["config"]["rays_per_step"], "kernel": r.get("kernel"),
                                    "bound": r.get("bound"), "frac": r.get("frac"),
                                    "cpu": None if cb is None else cb["value"],
                                    "cpu_rays": None if cb is None else cb.get("rays")}
    return line, detail


def emit(line, detail, detail_path):
    """Write the detail file (when a path is given), a short per-line summary to stderr, and the compact line as
    the LAST line of stdout."""
    if detail_path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail_path)), exist_ok=True)
            with open(detail_path, "w") as fh:
                json.dump(detail, fh, indent=1)
            line["detail"] = os.path.relpath(os.path.abspath(detail_path), HERE)
        except OSError as e:   # a read-only tree: the detail is lost, the line is not
            log(f"detail file not written: {e}")
    for name, e in detail.items():
        r = e.get("roofline") or {}
        log(f"{name}: {e['value']} rays/s, {e['ms_per_step']} ms/step, {r.get('kernel')} frac {r.get('frac')}, "
            f"cpu {(e.get('cpu_baseline') or {}).get('value')}")
    s = json.dumps(line, separators=(",", ":"))
    if len(s) > LINE_MAX_BYTES:   # never again an unparseable line: drop the summaries before the contract keys
        line.pop("extras", None)
        s = json.dumps(line, separators=(",", ":"))
    print(s, flush=True)


def log(msg):
    """Progress on stderr (a long default run keeps showing signs of life)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def add_ceiling(roof, ceiling):
    """The algorithmic fraction (fp32-equivalent FLOP of the network as written / the fp16 dense peak the split
    products run on) beside the issued-products ``frac``, and the issued rate against the measured ceiling."""
    if roof is None or roof.get("unit") != "TFLOP/s":
        return
    fp32eq = roof.get("fp32_equivalent_TFLOPs")
    if fp32eq is not None:
        roof["frac_algorithmic"] = round(fp32eq / FP16_MFMA_PEAK_TFLOPS, 4)
    if ceiling and roof.get("issued_TFLOPs"):
        roof["ceiling_measured_TFLOPs"] = ceiling["TFLOPs"]
        roof["frac_of_measured_ceiling"] = round(roof["issued_TFLOPs"] / ceiling["TFLOPs"], 4)


def dist_on(world):
    """Whether this run goes through torch.distributed: N > 1, or (test-only, PCNERF_BENCH_FORCE_DIST=1 under a
    one-process torchrun) N = 1 over a one-rank RCCL group, so every collective of the N-rank path runs through RCCL
    on a one-GPU box (tests/test_dist_gpu.py); the driver's runs never set it."""
    return world > 1 or os.environ.get("PCNERF_BENCH_FORCE_DIST") == "1"


def run_line(a, L, dev, rank, world):
    """One bench line: ``a.warmup`` untimed + ``a.steps`` timed steps of ``a.mode`` on this rank's blocks, the
    kernel breakdown / roofline of the last step, the fp32-MFMA comparison and (rank 0, N=1) the CPU baseline."""
    import gc
    from nof import _ops, synthetic as syn
    from nof.blocks import allreduce_grads, gather_rows, max_over_ranks
    from nof.criteria import nof_loss
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_train, render_rays_val, render_rays_view_0525_2_2
    dist = dist_on(world)
    if dist:
        import torch.distributed as tdist

    view = a.mode == "view"
    train = a.mode in ("train_fwd", "train_step")
    grad = a.mode == "train_step"
    if a.fold:
        if train:
            _ops.set_train_fold(True)
        else:
            _ops.set_eval_fold(True)
    # (the default training backward keeps no activation store; under set_train_backward("store") this caller, which
    # allocates nothing between forward and backward, lets the store take the free HBM)
    prev_budget = _ops.set_activation_store_budget(1 << 62) if grad and not _ops.remat_enabled() else None
    blocks = make_blocks(a, rank, world, dev, syn)
    for blk in blocks:
        blk["mc"] = syn.load_into(NOF_coarse(), syn.init_nof_params(blk["seeds"][0])).to(dev).train(train)
        blk["mf"] = syn.load_into(NOF_fine(), syn.init_nof_params(blk["seeds"][1])).to(dev).train(train)
    emb = Embedding(3, 10)
    loss_fn = nof_loss["smoothl1"]()
    opt = None
    if grad:
        params = [p for blk in blocks for m in (blk["mc"], blk["mf"]) for p in m.parameters()]
        opt = torch.optim.Adam(params, lr=5e-4, eps=1e-8, weight_decay=1e-3)   # nof_utils.py:167-169
    dp = grad and dist and a.config == 3   # one block trained data-parallel: average gradients over ranks

    def block_step(blk):
        mc, mf, rays, gt = blk["mc"], blk["mf"], blk["rays"], blk["gt"]
        if train:
            res = render_rays_train(mc, mf, emb, rays, sub_nerf_test_num=blk["sub_num"], N_samples=a.samples,
                                    N_importance=a.importance, perturb=1, noise_std=0, chunk=a.chunk,
                                    issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0,
                                    use_child_nerf_loss=1)
            lr = 1e-1 * loss_fn(1e1 * res["depth"], 1e1 * gt)           # train_kitti.py:145-146
            lrf = 1e-1 * loss_fn(1e1 * res["depth_fine"], 1e1 * gt)
            loss = (lr + lrf + 1e6 * res["child_free_loss_fine"] + 1e6 * res["child_free_loss"]
                    + 1e5 * res["child_depth_loss_fine"] + 1e5 * res["child_depth_loss"])
        elif view:   # eval_kitti_render.py:1147-1161: two-step inference, effective rows' points kept
            res = render_rays_view_0525_2_2(mc, mf, emb, rays, blk["other"], N_samples=a.samples,
                                            N_importance=a.importance, perturb=0, noise_std=0, chunk=a.chunk,
                                            depth_inference_method=2)
            keep = res["rays_effective_flag_fine"].reshape(-1)
            loss = res["points_inference_fine"][keep].abs().mean()
        else:
            res = render_rays_val(mc, mf, emb, rays, N_samples=a.samples, N_importance=a.importance, perturb=0,
                                  noise_std=0, chunk=a.chunk)
            loss = 1e-1 * loss_fn(1e1 * res["depth_fine"], 1e1 * gt)
        return loss, res["depth_fine"]

    def step():
        if grad:
            opt.zero_grad(set_to_none=True)
        losses, depths = [], []
        for blk in blocks:
            loss, d = block_step(blk)
            if grad:
                loss.backward()
            losses.append(loss.detach().reshape(()))
            depths.append(d.detach().reshape(-1, 1))
        ev = None
        if coll["on"] and (a.gather or dp):   # the step's collectives, timed with events on torch's stream
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if a.gather:   # every block's per-ray depth to rank 0 (RCCL all_gather over xGMI)
            gather_rows(torch.cat(depths) if depths else torch.zeros((0, 1), device=dev), dst=0)
        if grad and dp:
            allreduce_grads(opt.param_groups[0]["params"])
        if ev is not None:
            ev[1].record()
            coll["events"].append(ev)
        if grad:
            opt.step()
        return torch.stack(losses).sum() if losses else torch.zeros((), device=dev)

    breakdown = {}   # wall time of the instrumented (last) step, the one the kernel breakdown comes from
    coll = {"on": False, "events": []}   # collective events of the timed steps (N > 1)

    def timed(steps, warmup):
        """warmup, barrier, ``steps`` timed steps (HIP events on the last), barrier; max over ranks."""
        with (torch.enable_grad() if grad else torch.no_grad()):
            for _ in range(warmup):
                loss = step()
            torch.cuda.synchronize(dev)
            if dist:
                tdist.barrier()
            torch.cuda.synchronize(dev)
            coll["on"], coll["events"] = dist, []
            t0 = time.perf_counter()
            eb0 = eb1 = None
            for i in range(steps):
                # per-kernel HIP events (kernel breakdown + roofline) around every launch of the LAST timed step
                # only: their own cost (two hipEventRecord per launch) then weighs 1/steps on the timed region
                if i == steps - 1:
                    L.pcnerf_prof_enable(1)
                    eb0 = torch.cuda.Event(enable_timing=True)
                    eb0.record()
                loss = step()
            if eb0 is not None:
                eb1 = torch.cuda.Event(enable_timing=True)
                eb1.record()
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            coll["on"] = False
            coll["ms"] = sum(e0.elapsed_time(e1) for e0, e1 in coll["events"])
            coll["local_s"] = el
            if eb0 is not None:
                breakdown["ms"] = eb0.elapsed_time(eb1)
            if dist:
                tdist.barrier()
            lv = float(loss)
        if not np.isfinite(lv):
            raise RuntimeError(f"non-finite loss {lv}")
        return max_over_ranks(el, device=dev), lv

    train_math = (("fold" if a.fold else _ops.get_train_math()) if train else None)
    eval_math = None if (train or a.fold) else _ops.get_eval_math()
    log(f"{a.mode} ({a.rays} rays, {a.samples}/{a.importance}): {a.warmup} + {a.steps} steps")
    elapsed, loss_val = timed(a.steps, a.warmup)
    dist_info = None
    if dist:   # the self-proving N-rank record: who ran, over which backend, each rank's work and time
        n_loc = (sum(blk.get("groups", a.rays) for blk in blocks) if view
                 else sum(blk["rays"].shape[0] for blk in blocks))
        dist_info = rank_report(tdist, dev, n_loc, coll["local_s"], coll["ms"], a.steps)
    log(f"{a.mode}: {1e3 * elapsed / a.steps:.2f} ms/step")
    kstep_ms = breakdown.get("ms", 0.0)
    roof, kernels = kernel_report(L, a, train_math, eval_math, getattr(a, "line", None) or a.mode)

    # the same workload with the MLP on the fp32 MFMA pipe (train / eval math "fp32"), for comparison
    fp32_line = None
    if train and train_math != "fp32" and not a.no_fp32_line and not a.fold:
        _ops.set_train_math("fp32")
        el32, _ = timed(a.steps, 1)
        roof32, k32 = kernel_report(L, a, "fp32", line="fp32")
        _ops.set_train_math(train_math)
        fp32_line = {"value": None, "ms_per_step": round(1e3 * el32 / a.steps, 3), "roofline": roof32,
                     "kernels": {k: v for k, v in k32.items() if k.startswith("train")},
                     "note": "the same timed steps with the train-mode Linear layers as fp32 MFMA (v_mfma_f32_32x32x2_f32)"}
        fp32_elapsed = el32
    if eval_math not in (None, "fp32") and not a.no_fp32_line:
        _ops.set_eval_math("fp32")
        el32, _ = timed(a.steps, 1)
        roof32, k32 = kernel_report(L, a, None, "fp32", line="fp32")
        _ops.set_eval_math(eval_math)
        fp32_line = {"value": None, "ms_per_step": round(1e3 * el32 / a.steps, 3), "roofline": roof32,
                     "kernels": {k: v for k, v in k32.items() if k.startswith("eval")},
                     "note": "the same timed steps with the fused eval network as fp32 MFMA (k_nof_eval, v_mfma_f32_32x32x2_f32)"}
        fp32_elapsed = el32

    # rays processed per step by the whole job (weak scaling: every rank its own blocks / batch)
    # (view: LiDAR rays = ray groups, a.rays per block; otherwise the rays of the block's batch)
    n_local = (sum(blk.get("groups", a.rays) for blk in blocks) if view
               else sum(blk["rays"].shape[0] for blk in blocks))
    blocks_rank0 = [blk["block"] for blk in blocks]
    sample = {k: blocks[0][k] for k in ("block", "rays", "seeds", "sub_num", "other") if k in blocks[0]}
    del blocks, opt, step, block_step
    gc.collect()
    torch.cuda.empty_cache()
    if prev_budget is not None or (grad and not _ops.remat_enabled()):
        _ops.set_activation_store_budget(prev_budget)
    if a.fold:
        _ops.set_train_fold(False)
        _ops.set_eval_fold(False)

    cpu = cdref = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:   # the CPU baseline belongs to the N=1 line only
        if a.cpu_rays is None:
            a.cpu_rays = min(CPU_SAMPLE_RAYS, a.rays)
        if a.fold:
            (_ops.set_train_fold if train else _ops.set_eval_fold)(True)
        log(f"{a.mode}: CPU baseline on {a.cpu_rays} rays")
        cpu, ext = cpu_baseline(a, syn, sample)
        cdref = (cd_vs_ref_view if view else cd_vs_ref)(a, syn, ext, dev, sample)
        log(f"{a.mode}: CPU baseline {cpu['value']} rays/s")
        if a.fold:
            _ops.set_train_fold(False)
            _ops.set_eval_fold(False)
        del ext
        gc.collect()
        torch.cuda.empty_cache()

    n_tot = torch.tensor([float(n_local)], dtype=torch.float64, device=dev)
    if dist:
        tdist.all_reduce(n_tot)
    rays_per_step = float(n_tot)
    value = rays_per_step * a.steps / elapsed
    if fp32_line is not None:
        fp32_line["value"] = round(rays_per_step * a.steps / fp32_elapsed, 1)
    return {"value": value, "elapsed": elapsed, "rays_per_step": rays_per_step, "roofline": roof,
            "kernels": kernels, "kstep_ms": kstep_ms, "fp32_mfma": fp32_line, "cpu_baseline": cpu,
            "cd_vs_ref": cdref, "loss": loss_val, "train_math": train_math, "eval_math": eval_math,
            "blocks_rank0": blocks_rank0, "dist": dist_info,
            "backward": (None if not grad else
                         "remat: no activation store, no memory budget set -- the drop-in's default training path "
                         "(nof._ops.set_train_backward)" if _ops.remat_enabled() else
                         "store: activation store, budget free HBM - 4 GiB (opt-in)")}


def rank_report(tdist, dev, n_local, local_s, coll_ms, steps):
    """backend, ranks seen, and per rank: rays per step, ms per step, ms per step inside the step's collectives
    (the depth gather / gradient all-reduce, HIP events) -- all-gathered so rank 0's line can prove that N ranks ran
    over RCCL and how the work was dealt."""
    v = torch.tensor([float(n_local), 1e3 * local_s / steps, coll_ms / steps], dtype=torch.float64, device=dev)
    allv = [torch.zeros_like(v) for _ in range(tdist.get_world_size())]
    tdist.all_gather(allv, v)
    m = torch.stack(allv).cpu().numpy()
    return {"backend": tdist.get_backend(), "ranks_seen": tdist.get_world_size(),
            "rays_per_rank": [int(x) for x in m[:, 0]], "ms_per_step_per_rank": [round(float(x), 3) for x in m[:, 1]],
            "collective_ms_per_step_per_rank": [round(float(x), 3) for x in m[:, 2]]}


def line_json(a, world, ln):
    """The JSON object of one bench line."""
    view = a.mode == "view"
    train = a.mode in ("train_fwd", "train_step")
    scaling = "strong" if a.config in (4, 5) else "weak"
    return {
        "metric": "LiDAR rays/s (render+loss) at 128 samples/ray; CD vs ref depth",
        "value": round(ln["value"], 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1e3 * ln["elapsed"] / a.steps, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        # every tensor and every accumulation is fp32; the Linear layers' products as the selected math forms them
        "dtype": dtype_label(ln["train_math"], ln["eval_math"], a.fold),
        "data": {2: "synthetic (config-2 parent block, 32 child AABBs; seeded NOF weights -- checkpoints absent)",
                 3: "KITTI-00 frames 1151-1200 at 50% frame sparsity (every 16th point) rays built by "
                    "nof.dataset, 262,144-ray batches drawn with replacement; seeded NOF weights",
                 4: "synthetic MaiCity-00 parent blocks (x-split of [-12,61]x[-12,12]x[-2,0.5], 256 child AABBs "
                    "each); seeded per-block NOF weights",
                 5: "KITTI-00 frames 1151-1198 (every 16th point) as 8 contiguous 6-frame parent blocks, two-step "
                    "rows of each block's held-out frames at 80% frame sparsity built by nof.raytable; seeded "
                    "per-block NOF weights"}[a.config]
                + ("; ray groups with the group-size histogram of the reference's KITTI test frames"
                   if view and a.config == 2 else ""),
        "config": {"workload": {"train_fwd": "render_rays_train fwd + range/child losses",
                                "train_step": "render_rays_train fwd + losses + backward + Adam step",
                                "val": "render_rays_val fwd",
                                "view": "render_rays_view_0525_2_2 two-step inference (method 2) + effective points"
                                }[a.mode] + ((" -- exact affine fold of the train-mode network per BatchNorm chunk "
                                              "(opt-in)" if train else " -- exact affine fold of the eval network "
                                              "(opt-in)") if a.fold else ""),
                   "baseline_config": a.config,
                   "rays_per_step": int(ln["rays_per_step"]),
                   "rays_per_block": None if (view and a.config == 5) else a.rays,
                   "blocks_rank0": ln["blocks_rank0"],
                   "N_samples": a.samples, "N_importance": a.importance,
                   "mlp_samples_per_ray": a.samples + a.samples + a.importance, "chunk": a.chunk,
                   "batchnorm": "train (batch stats per chunk)" if train else "eval (folded)",
                   "network": "affine fold (sigmoid(a.e + c))" if a.fold else "9 Linear layers as written",
                   "segmented_ratio": 0.1 if train else None, "perturb": 1 if train else 0,
                   "parallelism": (f"dp{world}" if a.config == 3 else f"blocks{world}"), "gather": bool(a.gather),
                   "backward": ln.get("backward")},
        "roofline": ln["roofline"],
        "train_math": ln["train_math"],
        "eval_math": ln["eval_math"],
        "fp32_mfma": ln["fp32_mfma"],
        "cpu_baseline": ln["cpu_baseline"],
        "cd_vs_ref": ln["cd_vs_ref"],
        "loss": ln["loss"],
        "kernels": ln["kernels"],
        "kernels_step_ms": round(ln["kstep_ms"], 3),   # the instrumented last step's own time (the kernels' step)
        "dist": ln.get("dist"),
    }


def dtype_label(train_math, eval_math, fold=False):
    """The arithmetic of the path: fp32 tensors and accumulation, and how the Linear layers' fp32 products are
    formed (DESIGN.md 'The split train math')."""
    split = "fp32 (Linear products: fp16 hi/mid split, {} MFMA products, fp32 accumulate)"
    if train_math in ("f16x2_3", "f16x2_3_fused") or (train_math is None and eval_math == "f16x2_3"):
        return split.format(3)
    if train_math == "f16x2_4":
        return split.format(4)
    if fold:
        return "fp32 (float64 {}layer algebra + float64 63-term dot per sample)".format(
            "per-chunk " if train_math == "fold" else "")
    return "fp32 (fp32 MFMA)"


# ----------------------------------------------------------------------------------------------- roofline
FP16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: ~2.5 PF dense BF16/FP16 MFMA


def split_layer_bound(bytes_per_launch, flop_per_launch, products):
    """The roof of a split-fp16 layer kernel: the one whose floor for the launch's algorithmic work is longer --
    ``products`` fp16 MFMA products per fp32 FLOP against the dense fp16 peak, or the bytes against HBM."""
    t_mfma = products * flop_per_launch / (FP16_MFMA_PEAK_TFLOPS * 1e12)
    t_hbm = bytes_per_launch / (HBM_PEAK_GBS * 1e9)
    return "mfma" if t_mfma > t_hbm else "hbm"


def kernel_report(L, a, train_math, eval_math=None, line=None):
    """Kernel breakdown of the last timed step (library HIP events) and the dominant kernel's roofline; ``line``
    selects the PMC traffic entries (pmc_traffic)."""
    from nof import _ops
    line = line or a.mode
    remat = a.mode == "train_step" and train_math == "f16x2_3_fused" and _ops.remat_enabled()
    rver = _ops.get_remat_version() if remat else None
    split = train_math in ("f16x2_3", "f16x2_4", "f16x2_3_fused")
    esplit = eval_math == "f16x2_3"
    nterm = 3 if (train_math in ("f16x2_3", "f16x2_3_fused") or esplit) else 4
    hid = f"k_train_h<0,true,{nterm}>" if split else "k_train_ws<0,true>"
    knames = {0: "k_nof_eval_h3<false,false>" if esplit else "k_nof_eval", 1: hid, 2: f"k_train_h<8,false,{nterm}>" if split else "k_train_ws<8,false>",
              3: f"k_train_h<8,true,{nterm}>" if split else "k_train_ws<8,true>",
              10: "k_wgrad<2>+k_wgrad<1>" if split else "k_wgrad<0>", 11: f"k_dgrad_h<{nterm}>" if split else "k_dgrad_ws",
              # (the encoding columns of layers 0 and 4: k_wgrad_enc in the remat backward, k_wgrad_b3 MODE 3 in the
              # store backward; the layered split backward launches several modes, named by its hidden-layer one)
              13: "k_nof_eval_fold", 15: f"k_train_h1<{nterm}>",
              14: ("k_wgrad_enc" if remat else f"k_wgrad_b3<1,3,1,true,{nterm}>") if train_math == "f16x2_3_fused"
              else f"k_wgrad_b3<1,0,0,true,{nterm}>",
              16: "k_tf_moments", 17: "k_tf_layer+k_tf_bwd_layer+k_tf_dw",
              # (the train query writing the activation store is its own instantiation)
              18: "k_nof_eval_h3<true,true>" if a.mode == "train_step" and not remat else "k_nof_eval_h3<true,false>",
              19: ({3: "k_bwd_remat3<false,false,4>", 4: "k_bwd_remat3<true,false,4>"}.get(rver, "k_bwd_remat2<0>") if remat
                   else "k_bwd_fused<0,false>")}
    pmc_names = {**knames, 4: "k_train_out", 7: "k_resample", 9: "k_composite_bwd", 20: "k_g7",
                 21: "k_bwd_remat3<true,true,4>"}
    tag = max(knames, key=lambda t: prof_read(L, t)[0])
    kname = knames[tag]
    ktime_ms, klaunch, kflops, kbytes = prof_read(L, tag)
    kernels = {}
    for t, nm in ((0, "eval_query"), (1, "train_hidden"), (2, "train_first"), (3, "train_skip"), (4, "train_out"),
                  (5, "bn_fold"), (6, "composite"), (7, "resample"), (8, "sample"), (9, "composite_bwd"),
                  (10, "wgrad"), (11, "dgrad"), (12, "bwd_other"), (13, "eval_fold"), (14, "wgrad_b3"),
                  (15, "train_h1"), (16, "fold_moments"), (17, "fold_algebra"), (18, "train_query"),
                  (19, "bwd_fused"), (20, "bwd_remat_operands"), (21, "bwd_fused_layer1")):
        tm, n, f, b = prof_read(L, t)
        if n:
            tr, src = pmc_traffic(pmc_names.get(t, ""), line)
            kernels[nm] = {"kernel": pmc_names.get(t), "ms_per_step": round(tm, 3), "launches_per_step": n,
                           "avg_us": round(1e3 * tm / n, 2),
                           "TFLOP/s": round(f / (tm * 1e-3) / 1e12, 2) if f else None,
                           "GB/s": round(b / (tm * 1e-3) / 1e9, 1) if b else None,
                           "hbm_bytes_per_launch_pmc": tr}
    L.pcnerf_prof_enable(0)
    avg_s = ktime_ms * 1e-3 / max(klaunch, 1)
    achieved = (kflops / max(klaunch, 1)) / avg_s / 1e12
    gbs = kbytes / max(klaunch, 1) / avg_s / 1e9
    traffic, traffic_src = pmc_traffic(kname, line)
    nprod = nterm   # k_wgrad_b3 too: f16x2 parts, nterm products (the six-product bf16x3 form is a build option)
    if tag == 19 and rver in (3, 4):
        # k_bwd_remat3 issues 3 products of (2.256.256 + 2.256.64 + 2.256.64) per sample against the algorithmic
        # 2.2.256.256 (its weight gradient contracts the 64 encoding columns; the rematerialised x is extra work)
        nprod = 3.0 * (131072 + 32768 + 32768) / 262144
    if a.fold:   # no MLP left: the query moves 8 B per sample (+ ray rows) and is bound by its sincos (VALU)
        roof = {"kernel": kname, "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                "avg_launch_us": round(avg_s * 1e6, 2), "algorithmic_bytes_per_launch": kbytes / max(klaunch, 1),
                "note": ("VALU-bound (the encoding's 30 sincosf per sample, recomputed by the moment, query and "
                         "gradient-moment passes; the per-chunk layer algebra is float64 MFMA); HBM fraction "
                         "reported as the contract asks") if a.mode in ("train_fwd", "train_step") else
                        "VALU-bound (60 sincosf per sample); HBM fraction reported as the contract asks"}
    elif (esplit and tag == 0) or tag == 18:
        # split-fp16 fused network (eval query, or the train-mode query with per-chunk BatchNorm coefficients):
        # nterm fp16 MFMA products per fp32 product, weights streamed from L2
        # achieved = the ALGORITHMIC rate (fp32 FLOP of the network as written / launch time) against the dense fp16
        # peak of the pipe the products run on; the issued-products rate (x nprod) beside it as frac_issued
        roof = {"kernel": kname, "bound": "mfma", "achieved": round(achieved, 1), "peak": FP16_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / FP16_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                "avg_launch_us": round(avg_s * 1e6, 2), "algorithmic_flop_per_launch": kflops / max(klaunch, 1),
                "products_per_fp32_product": nprod, "fp32_equivalent_TFLOPs": round(achieved, 2),
                "issued_TFLOPs": round(nprod * achieved, 1),
                "frac_issued": round(nprod * achieved / FP16_MFMA_PEAK_TFLOPS, 4)}
    elif split and tag in (1, 2, 3, 11, 14, 15, 19):
        # split-fp16 layer kernel: nterm fp16 MFMA products per fp32 product.  The bound is the roof with the longer
        # floor for the launch's algorithmic work: the layered kernels' 2 KiB/sample stream outlasts their MFMA
        # work (hbm); the rematerialised layer's 3 x 294,912 fp16 FLOP/sample outlast its 2.25 KiB (mfma)
        per_b, per_f = kbytes / max(klaunch, 1), kflops / max(klaunch, 1)
        mfma_bound = split_layer_bound(per_b, per_f, nprod) == "mfma"
        hbm = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
        mf = {"achieved": round(achieved, 1), "peak": FP16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
              "frac": round(achieved / FP16_MFMA_PEAK_TFLOPS, 4), "issued_TFLOPs": round(nprod * achieved, 1),
              "frac_issued": round(nprod * achieved / FP16_MFMA_PEAK_TFLOPS, 4)}
        roof = {"kernel": kname, "bound": "mfma" if mfma_bound else "hbm", **(mf if mfma_bound else hbm),
                "traffic": traffic, "avg_launch_us": round(avg_s * 1e6, 2),
                "algorithmic_bytes_per_launch": per_b, "algorithmic_flop_per_launch": per_f,
                "products_per_fp32_product": nprod, "fp32_equivalent_TFLOPs": round(achieved, 2),
                "other_roof": {"bound": "hbm" if mfma_bound else "mfma", **(hbm if mfma_bound else mf)}}
    else:
        roof = {"kernel": kname, "bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                "avg_launch_us": round(avg_s * 1e6, 2), "algorithmic_flop_per_launch": kflops / max(klaunch, 1)}
    if tag == 19 and remat:
        # one launch per layer and chunk: the per-sample bytes (g_L + encoding in, g_{L-1} out) are the algorithmic
        # count; each launch also writes its 128 pair partials of the weight gradient (the split-K over tiles) and
        # reads the previous layer's
        per_launch = kbytes / max(klaunch, 1)
        partials = 2.0 * 128 * (256 * (64 if rver in (3, 4) else 256) + 256) * 4
        roof["note"] = (("k_bwd_remat3 (weight gradient over the 64 encoding columns, projected by P'^T per chunk)"
                         if rver in (3, 4) else "layer launches k_bwd_remat2<0|2> averaged") +
                        "; the weight-gradient partial round trip is outside the algorithmic bytes")
        roof["partials_bytes_per_launch"] = partials
        if traffic:
            roof["traffic_over_algorithmic"] = round(traffic / per_launch, 3)
            roof["traffic_over_algorithmic_with_partials"] = round(traffic / (per_launch + partials), 3)
    roof["traffic_source"] = traffic_src
    return roof, kernels


# ----------------------------------------------------------------------------------------------- CPU baseline
def available_cores() -> int:
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU quota when one is set (a GPU box's
    share of the host)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def _best_of(fn, reps=3, long_s=8.0):
    """Warm-up is done by the caller; best wall time of ``reps`` runs (warm-up 1, best of 3), or of
    one run when that run alone takes longer than ``long_s`` (a 2,048-ray training step on the host: its spread is
    small next to its length, and three would stretch the default bench past a few minutes).  Returns (best, output,
    runs)."""
    best, out, n = float("inf"), None, 0
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        n += 1
        best = min(best, time.perf_counter() - t0)
        if best > long_s:
            break
    return best, out, n


def cpu_baseline(a, syn, blk):
    """The CPU oracle (oracle/ref_cpu.py, the reference's arithmetic on torch CPU) on a bounded sample of the
    same workload: ``--cpu-rays`` rays of rank 0's first block, same settings, forward + losses (+ backward + Adam
    in train_step mode), warm-up + best of 3.  The RNG draws are generated here and returned with the oracle's
    depths, so the HIP path can be run on the identical inputs for the "CD vs ref depth" half of the metric."""
    from oracle import ref_cpu as O
    threads = available_cores()
    torch.set_num_threads(threads)
    if a.mode == "view":
        return cpu_baseline_view(a, syn, O, threads, blk)
    rays = blk["rays"][:a.cpu_rays].cpu()
    Pc = O.params_from_numpy(syn.init_nof_params(blk["seeds"][0]))
    Pf = O.params_from_numpy(syn.init_nof_params(blk["seeds"][1]))
    train = a.mode in ("train_fwd", "train_step")
    grad = a.mode == "train_step"
    gen = torch.Generator().manual_seed(7)
    R = rays.shape[0]
    draws = {"perturb_rand": torch.rand(R, a.samples, generator=gen),
             "u": torch.rand(R, a.importance, generator=gen)} if train else {}
    leaves = []
    init = [{k: v.detach().clone() for k, v in P.items()} for P in (Pc, Pf)]
    if grad:
        for P in (Pc, Pf):
            for k in P:
                if k.endswith(".weight") or k.endswith(".bias"):
                    leaves.append(P[k].requires_grad_(True))
        opt = torch.optim.Adam(leaves, lr=5e-4, eps=1e-8, weight_decay=1e-3)

    def run(r, dr, step):
        if train:
            res = O.render_rays_train(Pc, Pf, r, sub_nerf_test_num=blk["sub_num"], N_samples=a.samples,
                                      N_importance=a.importance, perturb=1, noise_std=0, chunk=a.chunk,
                                      issegmentated=1, childnerf_ratio=0.1, use_child_nerf_loss=1, training=True,
                                      draws=dr)
            lr, lrf = O.range_losses(res["depth"], res["depth_fine"], r[:, 14])
            loss = O.total_loss(res, lr, lrf)
            if grad and step:
                opt.zero_grad()
                loss.backward()
                opt.step()
            return res
        return O.render_rays_val(Pc, Pf, r, N_samples=a.samples, N_importance=a.importance, perturb=0, noise_std=0,
                                 chunk=a.chunk)

    with (torch.enable_grad() if grad else torch.no_grad()):
        run(rays[:64], {k: v[:64] for k, v in draws.items()}, False)  # warm-up (no parameter update)
        dt, _, nrun = _best_of(lambda: run(rays, draws, True))
        # the depths the HIP path is compared with: the oracle's forward from the INITIAL weights
        for P, P0 in zip((Pc, Pf), init):
            for k in P:
                P[k] = P0[k].clone()
        with torch.no_grad():
            res = run(rays, draws, False)
    R = int(rays.shape[0])
    base = {"value": round(R / dt, 2), "unit": "rays/s", "cores": threads, "kind": "port", "rays": R,
            "sample": f"{R} rays, same workload, oracle/ref_cpu.py on torch CPU, {threads} threads; "
                      f"warm-up + best of {nrun} = {dt:.1f} s"}
    return base, {"rays": rays, "draws": draws, "depth_fine": res["depth_fine"].detach()}


def cpu_baseline_view(a, syn, O, threads, blk):
    """Two-step inference (render.py:614-699 restated in oracle/ref_cpu.py) on ``--cpu-rays`` ray groups."""
    if blk.get("other") is not None and a.config == 5:   # the first --cpu-rays ray groups of the block's own rows
        starts = torch.nonzero(blk["rays"][:, 12] >= -0.5).reshape(-1).cpu()
        end = int(starts[a.cpu_rays]) if a.cpu_rays < starts.numel() else int(blk["rays"].shape[0])
        rows, other = blk["rays"][:end].cpu(), blk["other"][:end].cpu()
        a.cpu_rays = min(a.cpu_rays, int(starts.numel()))
    else:
        vr, vo, _ = syn.make_view_rows(a.cpu_rays, n_children=32, seed=1000 * blk["block"])
        rows, other = torch.from_numpy(vr), torch.from_numpy(vo)
    Pc = O.params_from_numpy(syn.init_nof_params(blk["seeds"][0]))
    Pf = O.params_from_numpy(syn.init_nof_params(blk["seeds"][1]))
    with torch.no_grad():
        O.render_rays_view(Pc, Pf, rows[:16], torch.zeros(16, dtype=torch.int64), a.samples, a.importance, a.chunk,
                           method=2)   # warm-up
        dt, res, nrun = _best_of(lambda: O.render_rays_view(Pc, Pf, rows, other, a.samples, a.importance,
                                                            a.chunk, method=2))
    base = {"value": round(a.cpu_rays / dt, 2), "unit": "rays/s", "cores": threads, "kind": "port",
            "rays": a.cpu_rays,
            "sample": f"{a.cpu_rays} ray groups ({rows.shape[0]} two-step rows), oracle/ref_cpu.py on torch CPU, "
                      f"{threads} threads; warm-up + best of {nrun} = {dt:.1f} s"}
    return base, {"rows": rows, "other": other, "res": res}


def cd_vs_ref_view(a, syn, ext, dev, blk):
    """HIP two-step inference on the CPU sample's rows vs the oracle: effective-row flags must agree; CD / F-score
    of the effective rows' fine points (what eval_kitti_render.py writes to the PCD)."""
    from nof import metrics as NM
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_view_0525_2_2
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(blk["seeds"][0])).to(dev).eval()
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(blk["seeds"][1])).to(dev).eval()
    rows, other, ref = ext["rows"].to(dev), ext["other"].to(dev), ext["res"]
    with torch.no_grad():
        res = render_rays_view_0525_2_2(mc, mf, Embedding(3, 10), rows, other, N_samples=a.samples,
                                        N_importance=a.importance, perturb=0, noise_std=0, chunk=a.chunk,
                                        depth_inference_method=2)
    fh = res["rays_effective_flag_fine"].reshape(-1).cpu()
    fr = ref["rays_effective_flag_fine"].reshape(-1)
    p_hip = res["points_inference_fine"][fh.to(dev)]
    p_ref = ref["points_inference_fine"][fr].to(dev)
    cd, f = NM.eval_pts(p_hip, p_ref, 0.2)
    d_hip, d_ref = res["depth_fine"].cpu(), ref["depth_fine"]
    rel = float(((d_hip - d_ref).abs() / d_ref.abs().clamp_min(1e-6)).max())
    return {"cd_m": cd, "fscore": f, "max_rel_depth_err": rel, "flags_equal": bool(torch.equal(fh, fr)),
            "rays": int(rows.shape[0]), "vs": "oracle two-step points of the effective rows (same rows and weights)"}


def cd_vs_ref(a, syn, ext, dev, blk):
    """The HIP path on the CPU sample's rays and draws (fresh weights of the same seeds) vs the oracle's depths:
    Chamfer distance / F-score (0.2 m) of the rendered points o + d * depth_fine (nof.metrics on the GPU) and the
    largest relative depth error."""
    from nof import metrics as NM
    from nof.networks import Embedding, NOF_coarse, NOF_fine
    from nof.render import render_rays_train, render_rays_val
    train = a.mode in ("train_fwd", "train_step")
    mc = syn.load_into(NOF_coarse(), syn.init_nof_params(blk["seeds"][0])).to(dev).train(train)
    mf = syn.load_into(NOF_fine(), syn.init_nof_params(blk["seeds"][1])).to(dev).train(train)
    rays = ext["rays"].to(dev)
    with torch.no_grad():
        if train:
            res = render_rays_train(mc, mf, Embedding(3, 10), rays, sub_nerf_test_num=blk["sub_num"],
                                    N_samples=a.samples, N_importance=a.importance, perturb=1, noise_std=0,
                                    chunk=a.chunk, issegmentated=1, childnerf_ratio=0.1, use_child_nerf_divide=0,
                                    use_child_nerf_loss=1, rng={k: v.to(dev) for k, v in ext["draws"].items()})
        else:
            res = render_rays_val(mc, mf, Embedding(3, 10), rays, N_samples=a.samples, N_importance=a.importance,
                                  perturb=0, noise_std=0, chunk=a.chunk)
    d_hip, d_ref = res["depth_fine"], ext["depth_fine"].to(dev)
    p_hip = rays[:, 0:3] + rays[:, 3:6] * d_hip[:, None]
    p_ref = rays[:, 0:3] + rays[:, 3:6] * d_ref[:, None]
    cd, f = NM.eval_pts(p_hip, p_ref, 0.2)
    rel = ((d_hip - d_ref).abs() / d_ref.abs().clamp_min(1e-6)).double()
    return {"cd_m": cd, "fscore": f, "max_rel_depth_err": float(rel.max()),
            "frac_rel_err_gt_1e-4": float((rel > 1e-4).double().mean()), "rays": int(rays.shape[0]),
            "vs": "oracle depth_fine on the cpu_baseline sample (same rays, draws and initial weights)"}


if __name__ == "__main__":
    main()
