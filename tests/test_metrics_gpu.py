"""GPU evaluation metrics (nof/metrics.py -> pcnerf_nn_distance / pcnerf_eval_pts / pcnerf_range_metrics) vs the
cKDTree oracle and the reference's committed KITTI frame 1153 (PC-NeRF two-step render vs source cloud).
Exhaustive float64 search: nearest distances equal the KD-tree's to rounding (rtol 1e-12); counts at the 0.2 m
threshold are exact."""
import numpy as np
import pytest

from conftest import golden
from nof import metrics as NM
from oracle import metrics_cpu as M

pytestmark = pytest.mark.gpu


def test_nn_distance_vs_kdtree():
    rng = np.random.default_rng(1)
    a = rng.uniform(-20, 20, size=(5003, 3)).astype(np.float32)
    b = rng.uniform(-20, 20, size=(777, 3)).astype(np.float32)
    d = NM.nn_correspondance(a, b).cpu().numpy()
    np.testing.assert_allclose(d, M.nn_dist(a, b), rtol=1e-12, atol=0)


def test_eval_pts_random_clouds():
    rng = np.random.default_rng(2)
    a = rng.uniform(-5, 5, size=(3000, 3)).astype(np.float32)
    b = (a[:2500] + rng.normal(scale=0.15, size=(2500, 3))).astype(np.float32)
    cd, f = NM.eval_pts(a, b, 0.2)
    cd_r, f_r = M.eval_pts(a, b, 0.2)
    np.testing.assert_allclose([cd, f], [cd_r, f_r], rtol=1e-12)


def test_reference_frame_metrics():
    g = golden("metrics_frame")
    got = NM.frame_metrics(g["pred"], g["gt"], g["origin"], 0.2)
    np.testing.assert_allclose(got, g["expected"], rtol=1e-10)
