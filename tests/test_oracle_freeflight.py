"""CPU checks of the oracle's free-flight restatement (FreeFlightGaussians integrator.h:300-408,
MultiScatterGaussians integrator.h:532-717). The reference holds no free-flight render, so the
restatement is pinned in expectation: single-scattering free-flight sampling and the analytic
ray-march (RayMarchingGaussians, pinned against the reference's own renders in
test_oracle_golden.py) estimate the same single-scattered radiance, so at high sample counts the
two images agree up to Monte-Carlo noise and the 0.01 march-step discretisation.
"""
import numpy as np
import pytest

import pyoracle as O
from helpers import CAM_POS, FOV, main_view_dir, scene_path


@pytest.mark.parametrize("name", ["2_gaussian.txt", "many_gaussians.txt"])
def test_single_scatter_free_flight_converges_to_raymarch(name):
    s = O.OracleScene.load_gmm(scene_path(name))
    W = 24
    ff = O.render_ff(s, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, W, multi=False, num_samples=1024)
    rm = O.render(s, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, W, O.RAYMARCH_GAUSSIANS, 0.01, 64)
    rel = abs(ff.mean() - rm.mean()) / rm.mean()
    assert rel < 5e-3, rel
    assert np.abs(ff - rm).mean() < 1e-2


def test_multi_scatter_adds_energy_and_is_deterministic():
    s = O.OracleScene.load_gmm(scene_path("many_gaussians.txt"))
    W = 20
    args = (s, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, W)
    ss = O.render_ff(*args, multi=False, num_samples=256)
    ms = O.render_ff(*args, multi=True, num_samples=256)
    assert ms.mean() > ss.mean()
    assert np.array_equal(O.render_ff(*args, multi=True, num_samples=4), O.render_ff(*args, multi=True, num_samples=4))


def test_free_flight_miss_pixels_are_env():
    s = O.OracleScene.load_gmm(scene_path("1_gaussian.txt"))
    img = O.render_ff(s, O.PINHOLE, CAM_POS, main_view_dir(), FOV, 16, 16, multi=True, num_samples=4)
    env = np.float32([0.53, 0.81, 0.92])
    acc = np.zeros(3, np.float32)
    for _ in range(4):
        acc = (acc + env).astype(np.float32)
    assert np.array_equal(img[0, 0], (acc / np.float32(4)).astype(np.float32))
