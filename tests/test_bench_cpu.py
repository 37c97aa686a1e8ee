"""bench.py's accounting helpers on the CPU (no GPU, no library call)."""
import importlib.util
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(HERE, "..", "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_split_layer_bound(bench):
    """The rematerialised layer kernel is priced on the matrix pipe, the layered split kernels on HBM (DESIGN.md
    kernel table): per sample 3 x 294,912 fp16 FLOP vs 2.25 KiB, and 3 x 131,072 vs 2 KiB."""
    n = 262144
    assert bench.split_layer_bound(2304 * n, 294912 * n, 3) == "mfma"
    assert bench.split_layer_bound(2048 * n, 2 * 256 * 256 * n, 3) == "hbm"
    # the floors themselves: 92.8 us on the matrix pipe against 75.5 us of HBM for the rematerialised layer
    assert 3 * 294912 * n / (bench.FP16_MFMA_PEAK_TFLOPS * 1e12) == pytest.approx(92.8e-6, rel=1e-3)
    assert 2304 * n / (bench.HBM_PEAK_GBS * 1e9) == pytest.approx(75.5e-6, rel=1e-3)


def test_pmc_traffic_line_keys(bench):
    """A line with its own profile (config3, config4, the reference's shell setting) takes only its own
    ``<kernel>@<line>`` entry; the mode-named lines fall back to the kernel's entry."""
    for line in ("config3", "config4", "train_step_refcfg"):
        assert bench.EXTRA_LINES[line]["line"] == line
    tr, src = bench.pmc_traffic("k_bwd_remat2<0>", "train_step")
    assert tr is None or (tr > 0 and src["file"] == "profiles/pmc_traffic.json")
    assert bench.pmc_traffic("no_such_kernel", "config4") == (None, None)


def _canned_line(bench, name, kernel, n_kernels=21):
    """A run_line() result shaped like a real one, with a full per-kernel table (the part that made round 5's
    line 24.5 KB)."""
    kernels = {f"kernel_{i}": {"kernel": f"k_some_kernel<{i},true,3>", "ms_per_step": 12.345, "launches_per_step": 1792,
                               "avg_us": 205.11, "TFLOP/s": 376.9, "GB/s": 3456.7, "hbm_bytes_per_launch_pmc": 678000000}
               for i in range(n_kernels)}
    roof = {"kernel": kernel, "bound": "mfma", "achieved": 397.1, "peak": 2500.0, "unit": "TFLOP/s", "frac": 0.1588,
            "issued_TFLOPs": 1191.3, "frac_issued": 0.4765,
            "traffic": 236000000.0, "avg_launch_us": 40017.97, "algorithmic_flop_per_launch": 1.648e13,
            "products_per_fp32_product": 3, "fp32_equivalent_TFLOPs": 397.1,
            "traffic_source": {"file": "profiles/pmc_traffic.json", "head": "bd9e60a", "profile": "r05h_x"}}
    return {"value": 794712.3, "elapsed": 1.649, "rays_per_step": 65536.0, "roofline": roof, "kernels": kernels,
            "kstep_ms": 84.1, "fp32_mfma": {"value": 123.4, "ms_per_step": 400.0, "roofline": dict(roof),
                                             "kernels": kernels, "note": "x" * 120},
            "cpu_baseline": {"value": 434.6, "unit": "rays/s", "cores": 16, "kind": "port", "rays": 2048,
                             "sample": "2048 rays, same workload, oracle/ref_cpu.py on torch CPU, 16 threads; "
                                       "warm-up + best of 3 = 4.7 s"},
            "cd_vs_ref": {"cd_m": 5.6e-06, "fscore": 1.0, "max_rel_depth_err": 3.2e-06, "flags_equal": True,
                          "rays": 2048, "vs": "y" * 90},
            "loss": 0.123, "train_math": "f16x2_3_fused", "eval_math": None, "blocks_rank0": [0, 1, 2, 3],
            "dist": None, "backward": "z" * 150}


def test_bench_line_compact_and_parseable(bench, tmp_path, capsys):
    """the driver parses the LAST stdout line.  With the headline and all six extra lines carrying
    full kernel tables, that line is valid JSON, at most 4 KB, and holds every key the contract names (roofline and
    cpu_baseline included); the full tables go to the detail file."""
    import argparse
    import json
    a = bench.parse([])
    head = _canned_line(bench, "headline", "k_nof_eval_h3<true,false>")
    extras = {n: _canned_line(bench, n, "k_bwd_remat2<0>") for n in bench.EXTRA_LINES}
    ceiling = {"TFLOPs": 1887.2, "clock_MHz": 2100, "seconds": 1.0, "kernel": "bare loop"}
    line, detail = bench.assemble(a, 1, head, extras, ceiling)
    path = tmp_path / "detail.json"
    print("noise before the line")
    bench.emit(line, detail, str(path))
    out = capsys.readouterr().out.splitlines()
    last = out[-1]
    assert len(last.encode()) <= bench.LINE_MAX_BYTES, len(last)
    got = json.loads(last)
    for k in bench.REQUIRED_KEYS:
        assert k in got, k
    for k in ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in got["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in got["cpu_baseline"], k
    assert set(got["extras"]) == set(bench.EXTRA_LINES)
    for e in got["extras"].values():
        assert {"value", "ms_per_step", "frac", "cpu", "kernel"} <= set(e)
    assert "kernels" not in got and "fp32_mfma" not in got
    full = json.loads(path.read_text())
    assert set(full) == {"headline", *bench.EXTRA_LINES}
    assert full["headline"]["kernels"] and full["config4"]["fp32_mfma"]["kernels"]


def test_bench_line_n_ranks_keys(bench):
    """An N-rank line carries the rank report (backend, ranks seen, per-rank rays / ms / collective ms) and still
    fits; the CPU baseline is absent at N > 1."""
    import json
    a = bench.parse(["--gpus", "8", "--config", "4"])
    head = _canned_line(bench, "headline", "k_nof_eval_h3<true,false>")
    head["cpu_baseline"] = head["cd_vs_ref"] = None
    head["dist"] = {"backend": "nccl", "ranks_seen": 8, "rays_per_rank": [262144] * 8,
                    "ms_per_step_per_rank": [1300.123] * 8, "collective_ms_per_step_per_rank": [0.456] * 8}
    line, _ = bench.assemble(a, 8, head, {}, None, head["dist"])
    s = json.dumps(line, separators=(",", ":"))
    assert len(s) <= bench.LINE_MAX_BYTES
    assert line["dist"]["ranks_seen"] == 8 and line["cpu_baseline"] is None and line["n_gpus"] == 8


def test_cpu_baseline_sample_is_fixed(bench):
    """every ray line's CPU baseline runs on the same sample size (the whole line when it is
    smaller), so lines of the same per-ray workload are comparable."""
    assert bench.CPU_SAMPLE_RAYS >= 2048
    for over in bench.EXTRA_LINES.values():
        assert over["cpu_rays"] is None          # the rule in run_line decides, not a per-line constant
    t = [0]

    def fn():
        t[0] += 1
        return t[0]
    best, out, n = bench._best_of(fn, reps=3, long_s=1e9)
    assert n == 3 and out == 3


def test_dist_on_only_for_n_ranks_or_the_test_switch(bench, monkeypatch):
    """The N-rank path runs for world > 1, and at world 1 only under the test-only PCNERF_BENCH_FORCE_DIST=1 (the
    one-rank RCCL test); the driver's default N = 1 run never initialises a process group."""
    monkeypatch.delenv("PCNERF_BENCH_FORCE_DIST", raising=False)
    assert not bench.dist_on(1) and bench.dist_on(2) and bench.dist_on(8)
    monkeypatch.setenv("PCNERF_BENCH_FORCE_DIST", "1")
    assert bench.dist_on(1)
