"""DESIGN.md's measured table from the bench lines of one tag: python3 scripts/measured_table.py r03n
(profiles/<tag>_bench_<line>.json, as scripts/gpu_bench_all.sh writes them under gpurun_out/bench/)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINES = [
    ("train_fwd", "`train_fwd` (headline; config 2, 65,536 rays, 128/256, train BN per chunk 262,144, child losses; "
                  "default `f16x2_3_fused`)"),
    ("train_step", "`train_step` (forward writing the activation store + losses + backward + Adam)"),
    ("config3", "`config3` (one training step of 262,144 rays, 64/128)"),
    ("config4", "`config4` (train_fwd, 1,048,576 rays)"),
    ("val", "`val` (`render_rays_val`, eval BN)"),
    ("view", "`view` (two-step inference, method 2, 16,384 ray groups)"),
    ("config5", "`config5` (two-step inference, 8 blocks)"),
    ("view_frame", "`view_frame` (one KITTI frame per step)"),
    ("val_fold", "`val --fold` (opt-in exact affine fold)"),
    ("view_fold", "`view --fold`"),
    ("train_fwd_fold", "`train_fwd --fold` (opt-in fold of the train-mode network)"),
    ("train_step_fold", "`train_step --fold`"),
    ("train_step_refcfg", "`train_step`, the reference's own shell config (256 rays/step, 768+1536 samples)"),
]


def roof(r):
    if r["unit"] == "TFLOP/s":
        return f"`{r['kernel']}` {r['achieved']:.0f} TFLOP/s fp16 = **{100 * r['frac']:.1f} %** of the dense fp16 peak"
    return f"`{r['kernel']}` {100 * r['frac']:.1f} % of HBM"


def main(tag):
    rows = []
    for line, label in LINES:
        path = os.path.join(HERE, "profiles", f"{tag}_bench_{line}.json")
        if not os.path.exists(path):
            continue
        d = json.loads(open(path).read().strip().splitlines()[-1])
        fp = d.get("fp32_mfma")
        cb = d.get("cpu_baseline") or {}
        cd = d.get("cd_vs_ref") or {}
        par = (f"CD {cd['cd_m']:.1e} m, max rel depth err {cd['max_rel_depth_err']:.1e}"
               + (", flags equal" if cd.get("flags_equal") else "")) if cd else "—"
        rows.append(f"| {label} | **{d['value']:,.0f}** | {d['ms_per_step']:.1f} | "
                    f"{fp['value']:,.0f} | " if fp else f"| {label} | **{d['value']:,.0f}** | {d['ms_per_step']:.1f} | — | ")
        rows[-1] += f"{roof(d['roofline'])} | {cb.get('value', 0):,.0f} rays/s | {par} |"
    print("\n".join(rows))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r03n")
