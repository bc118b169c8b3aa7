"""Pin the oracle's free-flight restatement (FreeFlightGaussians integrator.h:300-408,
MultiScatterGaussians integrator.h:532-717, distance_solvers.h:25-187) to the reference's own
free-flight renders (tests/renders, copied to tests/golden/renders):

  FreeFlightGaussians    2g_freeflight (2_gaussian.txt with the light x70, as baseline_2),
                         7g_freeflight (many_gaussians.txt), 50_rand_ss, 250_rand_ss
  MultiScatterGaussians  50_rand_ms, 250_rand_ms (ANALYTIC_PLUS_NEWTON, the compiled-in solver),
                         250_rand_{newton,bisection,uniform}_big (the solver the file is named after)

Finding (measured here): the goldens are not path-exact reproductions of the
current source at any spp. They are unbiased Monte-Carlo images: each golden agrees with the
reference's own RayMarchingGaussians render of the same scene to 0.01 % in mean, but the current
source's PCG32 (rng.h:43 rotates by (-rot + 1) & 31 instead of (-rot) & 31) ORs overlapping halves
whenever rot <= 1 and so draws biased uniforms (E[-log(1 - u)] = 1.08 instead of 1). That makes
the as-written integrators 0.5-1.4 % brighter than the goldens. The oracle keeps the reference's
PCG32 (the device path matches it path for path, tests/test_gpu_freeflight.py); with the textbook
rotation switched on (a test-only oracle switch) the same restatement reproduces every golden
within Monte-Carlo noise and without bias, which pins the rest of the free-flight algorithm:
event sweep, analytic/Newton/bisection/uniform solvers, albedo, NEE, Russian roulette.
"""
import ctypes
import os

import numpy as np
import pytest

import pyoracle as O
from helpers import CAM_POS, FOV, RENDERS, SCENES, main_view_dir, read_ppm, scene_path, to8

SOLVER = {"analytic_newton": 0, "bisection": 1, "newton": 2, "analytic_bisection": 3, "uniform": 4}


def _lib():
    L = O.lib()
    L.orc_set_solver.argtypes = [ctypes.c_int]
    L.orc_set_pcg_textbook.argtypes = [ctypes.c_int]
    return L


@pytest.fixture
def oracle_modes():
    L = _lib()
    yield L
    L.orc_set_solver(SOLVER["analytic_newton"])
    L.orc_set_pcg_textbook(0)


def _pixels(n, seed=0, W=512, H=512):
    rng = np.random.default_rng(seed)
    idx = rng.choice(W * H, size=n, replace=False)
    return np.stack([idx % W, idx // W], 1).astype(np.int32)


def _scene(name, tmp_path):
    if name == "2_gaussian_x70":  # baseline_2 / 2g_freeflight: light intensity 70 (file edited later)
        txt = open(scene_path("2_gaussian.txt")).read().replace("1.0  1.0  1.0", "70.0  70.0  70.0", 1)
        p = tmp_path / "2g_x70.txt"
        p.write_text(txt)
        return O.OracleScene.load_gmm(str(p))
    return O.OracleScene.load_gmm(scene_path(name))


def test_reference_pcg32_rotation_is_biased():
    """rng.h:43's rotation quirk, measured on the streams the integrators use (third draw of
    PCG32(derive_path_seed(x, y, si), 1), the free-flight target optical depth)."""
    n = 8192
    third = np.array([O.pcg32(O.derive_path_seed(256, 300, si), 1, 3)[2] for si in range(n)], np.uint64)
    u = (third >> np.uint64(8)).astype(np.float64) / 16777216.0
    e = -np.log1p(-u)
    assert e.mean() > 1.04, e.mean()  # Exp(1) would be 1 +- 0.011 (1 sigma)
    assert u.mean() > 0.5, u.mean()


# (golden, scene, multi, solver, max mean |diff| (8-bit), max |signed mean diff|)
# Measured with textbook PCG at 256 spp on these 2048 pixels: |signed| <= 0.14, mean |diff| 1.0-5.5
# (the goldens' own Monte-Carlo noise plus ours).
GOLDENS = [
    ("2g_freeflight.ppm", "2_gaussian_x70", False, "analytic_newton", 1.4, 0.3),
    ("7g_freeflight.ppm", "many_gaussians.txt", False, "analytic_newton", 2.5, 0.3),
    ("50_rand_ss.ppm", "50_random.txt", False, "analytic_newton", 5.0, 0.35),
    ("250_rand_ss.ppm", "250_random.txt", False, "analytic_newton", 5.3, 0.35),
    ("50_rand_ms.ppm", "50_random.txt", True, "analytic_newton", 5.2, 0.35),
    ("250_rand_ms.ppm", "250_random.txt", True, "analytic_newton", 6.2, 0.35),
    ("250_rand_newton_big.ppm", "250_random.txt", True, "newton", 6.0, 0.35),
    ("250_rand_bisection_big.ppm", "250_random.txt", True, "bisection", 6.0, 0.35),
    ("250_rand_uniform_big.ppm", "250_random.txt", True, "uniform", 6.0, 0.35),
]


@pytest.mark.parametrize("golden,scene,multi,solver,mean_tol,bias_tol", GOLDENS)
def test_free_flight_matches_reference_render(oracle_modes, tmp_path, golden, scene, multi, solver, mean_tol, bias_tol):
    L = oracle_modes
    L.orc_set_solver(SOLVER[solver])
    L.orc_set_pcg_textbook(1)
    s = _scene(scene, tmp_path)
    pix = _pixels(2048)
    g = read_ppm(os.path.join(RENDERS, golden))[pix[:, 1], pix[:, 0]].astype(int)
    out = O.render_ff(s, O.PINHOLE, CAM_POS, main_view_dir(), FOV, 512, 512, multi=multi, num_samples=256, pixels=pix)
    d = to8(out).astype(int) - g
    print(f"{golden}: mean|d| {np.abs(d).mean():.3f} signed {d.mean():+.3f} p99 {np.percentile(np.abs(d), 99):.0f}")
    assert np.abs(d).mean() < mean_tol, np.abs(d).mean()
    assert abs(d.mean()) < bias_tol, d.mean()


@pytest.mark.parametrize("golden,scene", [("50_rand_ss.ppm", "50_random.txt"), ("250_rand_ss.ppm", "250_random.txt")])
def test_as_written_pcg_is_brighter_than_the_goldens(oracle_modes, golden, scene):
    """The same renders with the reference's PCG32 as written (the oracle default, and what the
    device reproduces): a systematic +0.5..+2 % brightness, the rotation quirk's bias."""
    s = O.OracleScene.load_gmm(scene_path(scene))
    pix = _pixels(2048)
    g = read_ppm(os.path.join(RENDERS, golden))[pix[:, 1], pix[:, 0]].astype(float)
    out = O.render_ff(s, O.PINHOLE, CAM_POS, main_view_dir(), FOV, 512, 512, multi=False, num_samples=256, pixels=pix)
    ratio = to8(out).astype(float).mean() / g.mean()
    assert 1.004 < ratio < 1.02, ratio


def test_free_flight_goldens_agree_with_raymarch_goldens():
    """Cross-check between the reference's own renders: the single-scattering free-flight image and
    the analytic ray-march image of a scene estimate the same radiance (means within 0.05 %)."""
    for a, b in [("50_rand_baseline.ppm", "50_rand_ss.ppm"), ("250_rand_baseline.ppm", "250_rand_ss.ppm"),
                 ("baseline_7.ppm", "7g_freeflight.ppm"), ("2_gaussian_ref.ppm", "2g_freeflight.ppm")]:
        A = read_ppm(os.path.join(RENDERS, a)).astype(float)
        B = read_ppm(os.path.join(RENDERS, b)).astype(float)
        assert abs(B.mean() / A.mean() - 1.0) < 5e-4, (a, b)


@pytest.mark.parametrize("name", ["2_gaussian.txt", "many_gaussians.txt"])
def test_single_scatter_free_flight_converges_to_raymarch(oracle_modes, name):
    """Unbiased (textbook-PCG) single-scattering free flight and the analytic ray-march estimate
    the same single-scattered radiance."""
    oracle_modes.orc_set_pcg_textbook(1)
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
