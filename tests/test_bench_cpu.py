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
