"""GPU: the binned primary march (VR_OPT_MARCH_BINNED, kernels/vr_gauss.hip march_binned_kernel) against
the BVH window-query march (march_kernel).

Both marches decide every entry with the same exact intersect and evaluate every step with the same
march_step, so the scatter records (positions, steps, active lists, T) are the same and the frames must
be bit-identical — on the reference's scenes, a dense scene whose pixels overflow the binned march's
per-lane lists (they re-run in the BVH fallback), an orthographic camera, PureRayMarching, multi-GPU
tile shares and the full-size benchmark frame. The oracle parity of the BVH march is test_gpu_parity.py.
"""
import numpy as np
import pytest

import vr_amd as vr
from helpers import CAM_POS, FOV, main_view_dir, scene_path

pytestmark = pytest.mark.gpu


def _render(scene, cam, W, H, binned, integrator=vr.RayMarchingGaussians, **kw):
    dev = vr.Device.get(0)
    saved = dev.get_option("march_binned")
    dev.set_option("march_binned", binned)
    try:
        img = vr.Image(W, H)
        integ = integrator(cam, **kw)
        integ.render(scene, img)
        return img.pixels.copy(), dict(integ.last_stats)
    finally:
        dev.set_option("march_binned", saved)


def _pinhole():
    return vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)


@pytest.mark.parametrize("name,W,H", [
    ("1_gaussian.txt", 96, 96),
    ("2g_altered.txt", 64, 64),
    ("god_ray.txt", 80, 72),
    ("50_random.txt", 128, 96),
    ("1000_random.txt", 192, 192),
    ("many_gaussians.txt", 96, 96),
    ("20k_bias.txt", 160, 128),
])
def test_binned_march_equals_bvh_march(name, W, H):
    scene = vr.Scene.load_GMM(scene_path(name))
    a, sa = _render(scene, _pinhole(), W, H, 0)
    b, sb = _render(scene, _pinhole(), W, H, 1)
    assert sa["error_pixels"] == 0 and sb["error_pixels"] == 0
    assert sa["scatter_records"] == sb["scatter_records"] or sb["fallback_pixels"] > 0
    assert np.array_equal(a, b, equal_nan=True)


def test_binned_march_orthographic_and_other_step():
    scene = vr.Scene.load_GMM(scene_path("50_random.txt"))
    cam = vr.Orthographic_Camera(CAM_POS, main_view_dir())
    a, _ = _render(scene, cam, 96, 96, 0, step_size=0.02)
    b, _ = _render(scene, cam, 96, 96, 1, step_size=0.02)
    assert np.array_equal(a, b, equal_nan=True)


def test_binned_march_pure_raymarching():
    scene = vr.Scene.load_GMM(scene_path("250_random.txt"))
    a, _ = _render(scene, _pinhole(), 96, 96, 0, integrator=vr.PureRayMarching)
    b, _ = _render(scene, _pinhole(), 96, 96, 1, integrator=vr.PureRayMarching)
    assert np.array_equal(a, b, equal_nan=True)


def test_binned_march_dense_overlaps_take_the_fallback():
    """Nested Gaussians: more than the binned march's 16 pending / 16 active entries per pixel; those
    pixels re-run in the BVH fallback passes and the frame stays identical."""
    rng = np.random.default_rng(3)
    n = 40
    mean = np.zeros((n, 3), np.float32) + np.array([0.0, 1.0, 0.0], np.float32)
    mean += rng.normal(0.0, 0.02, (n, 3)).astype(np.float32)
    s = np.linspace(0.05, 0.5, n).astype(np.float32)
    cov = np.zeros((n, 6), np.float32)
    cov[:, 0] = cov[:, 3] = cov[:, 5] = s * s
    scene = vr.Scene.from_gaussians(mean, cov, np.full(n, 0.3, np.float32), np.full(n, 0.8, np.float32),
                                    [vr.Light([0.0, 4.0, 1.0], [20.0, 20.0, 20.0])])
    a, sa = _render(scene, _pinhole(), 64, 64, 0, env_samples=4)
    b, sb = _render(scene, _pinhole(), 64, 64, 1, env_samples=4)
    assert sb["fallback_pixels"] > 0
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.timeout(600)
def test_binned_march_full_size_c4():
    """The benchmark frame (4096^2, 1 M make_random Gaussians, t_eps 1e-6): identical frames."""
    scene = vr.Scene(vr.Scene.GAUSSIANS)
    scene.add_random_gaussians(1_000_000, seed=2025, variant=0)
    for p, i in [((0.0, 5.0, 0.1), (50.0, 0.0, 0.0)), ((-3.0, 3.0, 0.3), (0.0, 30.0, 0.0)),
                 ((3.0, 3.0, -0.2), (0.0, 0.0, 30.0))]:
        scene.add_light(vr.Light(p, i))
    a, sa = _render(scene, _pinhole(), 4096, 4096, 0, t_eps=1e-6)
    b, sb = _render(scene, _pinhole(), 4096, 4096, 1, t_eps=1e-6)
    print(f"C4 records {sa['scatter_records']} / {sb['scatter_records']}, fallback pixels {sa['fallback_pixels']} / "
          f"{sb['fallback_pixels']}, march {sa['stage_ms']['march']:.2f} / {sb['stage_ms']['march']:.2f} ms")
    assert sb["error_pixels"] == 0
    assert np.array_equal(a, b, equal_nan=True)
