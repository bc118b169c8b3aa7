"""GPU: RECORD_PIXEL_GAUSSIANS recording (integrator.h:616-644) and the stochastic finite-difference
inverse loop (inverse_integrator.h:61-246) on the device, through the C ABI, vs the oracle."""
import numpy as np
import pytest

import pyoracle as O
import vr_amd as vr
from vr_amd import inverse as inv
from helpers import CAM_POS, FOV, main_view_dir, scene_path

pytestmark = pytest.mark.gpu


def _cam():
    return vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)


@pytest.mark.parametrize("name,W,spp", [("50_random.txt", 32, 4), ("many_gaussians.txt", 32, 4),
                                        ("2_gaussian.txt", 24, 16)])
def test_recorded_pixel_gaussians_match_oracle(name, W, spp):
    path = scene_path(name)
    integ = vr.MultiScatterGaussians(_cam(), spp)
    img = vr.Image(W, W)
    integ.record(vr.Scene.load_GMM(path), img, slot=0)
    bits = integ.pixel_gaussian_bits(0)
    oimg, obits = O.render_ms_record(O.OracleScene.load_gmm(path), O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, W, spp)
    assert bits.shape == obits.shape
    same = np.all(bits == obits, axis=0)
    print(f"pixels with identical Gaussian sets: {same.mean():.4f}, set bits {int(np.unpackbits(bits.view(np.uint8)).sum())}")
    assert same.mean() >= 0.99
    assert np.abs(img.pixels - oimg).max(axis=-1).mean() < 1e-4


def test_per_pixel_lists_and_plain_render_agree():
    path = scene_path("50_random.txt")
    scene = vr.Scene.load_GMM(path)
    integ = vr.MultiScatterGaussians(_cam(), 4)
    a, b = vr.Image(16, 16), vr.Image(16, 16)
    lists = []
    integ.render(scene, a, per_pixel_gaussians=lists)
    integ.render(scene, b)
    assert np.array_equal(a.pixels, b.pixels)  # recording does not change the image
    assert len(lists) == 256 and all(l == sorted(set(l)) for l in lists)
    assert any(len(l) for l in lists)


def test_sfd_loss_diff_matches_host_union_sum():
    path = scene_path("50_random.txt")
    scene = vr.Scene.load_GMM(path)
    n = scene.get_num_primitives()
    W = 32
    integ = vr.MultiScatterGaussians(_cam(), 4)
    ia, ib = vr.Image(W, W), vr.Image(W, W)
    integ.record(scene, ia, slot=0)
    b0 = integ.pixel_gaussian_bits(0)
    params = inv.pack_parameters(scene.gaussians())
    params[0::11] += 0.05
    integ.record(inv.apply_params(params, scene.lights, scene.env_color), ib, slot=1)
    b1 = integ.pixel_gaussian_bits(1)
    rng = np.random.default_rng(3)
    lb = rng.random(W * W).astype(np.float32)
    lp = rng.random(W * W).astype(np.float32)
    out = np.zeros(n, np.float64)
    import ctypes
    vr.check(vr.lib().vr_sfd_loss_diff(vr.Device.get(0)._h, lb.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                       lp.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), W, W,
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n))
    u = np.unpackbits((b0 | b1).T.copy().view(np.uint8), axis=1, bitorder="little")[:, :n].astype(bool)  # (npix, n)
    ref = (u * (lp.astype(np.float64) - lb.astype(np.float64))[:, None]).sum(axis=0)
    np.testing.assert_allclose(out, ref, rtol=1e-9, atol=1e-9)


def test_sfd_optimize_runs_and_is_reproducible():
    path = scene_path("2_gaussian.txt")
    target = vr.Scene.load_GMM(path)
    W = 24
    I_ref = vr.Image(W, W)
    vr.MultiScatterGaussians(_cam(), 16).render(target, I_ref)
    p = inv.pack_parameters(target.gaussians())
    p[9::11] -= 0.7  # start from thinner Gaussians
    start = inv.apply_params(p, target.lights, target.env_color)
    runs = []
    for _ in range(2):
        opt = inv.StochasticFiniteDiffInverseIntegrator(_cam(), vr.MultiScatterGaussians(_cam(), 4),
                                                        inv.SFDConfig(max_iters=6, num_stoch_samples=2, lr=0.05, seed=1))
        assert opt.optimize(start, I_ref)
        assert np.all(np.isfinite(opt.history)) and np.all(np.isfinite(opt.params))
        runs.append(opt.params.copy())
    assert np.array_equal(runs[0], runs[1])
    assert not np.array_equal(runs[0], p)
