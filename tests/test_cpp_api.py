"""C++ host API (3dg-vol-renderer_amd/include/vr/*.h, the reference's class surface over the C ABI)
driven through tools/vol_render, the counterpart of the reference's tests/main.cpp.

CPU: the driver builds against the headers and its primary rays equal the oracle's bit for bit;
errors surface as std::runtime_error with the library's message. GPU: a render through the C++
classes equals the Python/ctypes render of the same scene bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest

import pyoracle as O
from helpers import CAM_POS, FOV, ROOT, main_view_dir, read_ppm, scene_path

TOOLS = os.path.join(ROOT, "tools")
EXE = os.path.join(TOOLS, "vol_render")


@pytest.fixture(scope="module")
def exe():
    r = subprocess.run(["make", "-C", TOOLS], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return EXE


def _run(exe, *args, check=True):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300)
    if check:
        assert r.returncode == 0, r.stdout + r.stderr
    return r


def _rays(out):
    rows = [ln.split()[1:] for ln in out.splitlines() if ln.startswith("ray ")]
    xy = np.array([[int(a), int(b)] for a, b, *_ in rows])
    od = np.array([[float(v) for v in r[2:]] for r in rows], np.float32)
    return xy, od


@pytest.mark.parametrize("W,H", [(512, 512), (37, 19)])
def test_pinhole_rays_match_oracle(exe, W, H):
    r = _run(exe, "--scene", scene_path("many_gaussians.txt"), "--size", f"{W}x{H}", "--dump-rays", "300")
    assert "scene: 7 primitives, 3 lights" in r.stdout
    xy, od = _rays(r.stdout)
    ref = np.array([O.primary_ray(O.PINHOLE, CAM_POS, main_view_dir(), FOV, int(x), int(y), W, H) for x, y in xy],
                   np.float32)
    assert np.array_equal(od.view(np.uint32), ref.view(np.uint32))


def test_xml_sensor_rays_match_oracle(exe):
    r = _run(exe, "--scene", scene_path("env_one_sphere_test_ortho.xml"), "--xml", "--dump-rays", "200")
    assert "scene: 1 primitives, 1 lights" in r.stdout
    xy, od = _rays(r.stdout)
    ref = np.array([O.primary_ray(O.ORTHO, np.float32([0, 1, 6]), np.float32([0, 0, -1]), 0.0, int(x), int(y), 512,
                                  512) for x, y in xy], np.float32)
    assert np.array_equal(od.view(np.uint32), ref.view(np.uint32))


def test_errors_are_runtime_errors(exe, tmp_path):
    r = _run(exe, "--scene", str(tmp_path / "missing.txt"), check=False)
    assert r.returncode == 1 and "vol_render:" in r.stderr and "missing.txt" in r.stderr


def test_render_without_gpu_fails_loudly(exe, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = _run(exe, "--scene", scene_path("1_gaussian.txt"), "--size", "8x8", "--out", str(tmp_path / "o.ppm"),
             check=False)
    assert r.returncode == 1 and "no HIP device" in r.stderr
    assert not (tmp_path / "o.ppm").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("scene,extra", [("many_gaussians.txt", []), ("2g_altered.txt", ["--env", "8"]),
                                         ("sph_2_spheres.txt", ["--spheres", "--integrator", "spheres"])])
def test_cpp_render_equals_python_render(exe, tmp_path, scene, extra):
    import vr_amd as vr
    out = tmp_path / "cpp.ppm"
    _run(exe, "--scene", scene_path(scene), "--size", "96x64", "--out", str(out), *extra)
    spheres = "--spheres" in extra
    s = vr.Scene.load_SMM(scene_path(scene)) if spheres else vr.Scene.load_GMM(scene_path(scene))
    cam = vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)
    env = int(extra[extra.index("--env") + 1]) if "--env" in extra else (5 if spheres else 20)
    integ = vr.RayMarchingSpheres(cam, 0.01, env) if spheres else vr.RayMarchingGaussians(cam, 0.01, env)
    img = vr.Image(96, 64)
    integ.render(s, img)
    py = tmp_path / "py.ppm"
    img.make_PPM(str(py))
    assert np.array_equal(read_ppm(str(out)), read_ppm(str(py)))


@pytest.mark.gpu
def test_cpp_record_render_equals_python(exe, tmp_path):
    """MultiScatterGaussians::render(scene, image, &per_pixel_gaussians) (integrator.h:532-536) through the
    C++ mirror records the same (pixel, Gaussian) pairs as the Python mirror."""
    import vr_amd as vr
    r = _run(exe, "--scene", scene_path("50_random.txt"), "--size", "32x32", "--integrator", "multiscatter", "--spp",
             "4", "--record", "--out", str(tmp_path / "r.ppm"))
    pairs = int([ln for ln in r.stdout.splitlines() if ln.startswith("recorded pairs")][0].split()[-1])
    integ = vr.MultiScatterGaussians(vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV), 4)
    lists = []
    integ.render(vr.Scene.load_GMM(scene_path("50_random.txt")), vr.Image(32, 32), per_pixel_gaussians=lists)
    assert pairs == sum(len(l) for l in lists) > 0


@pytest.mark.gpu
def test_cpp_inverse_loop_equals_python(exe, tmp_path):
    """StochasticFiniteDiffInverseIntegrator through the C++ mirror and through the Python mirror (both
    over vr_sfd_optimize) give the same loss history bit for bit on the same inputs."""
    import vr_amd as vr
    from vr_amd import inverse as inv
    cam = vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)
    ref = vr.Image(24, 24)
    vr.MultiScatterGaussians(cam, 16).render(vr.Scene.load_GMM(scene_path("2g_altered.txt")), ref)
    ref_path = tmp_path / "ref.ppm"
    ref.make_PPM(str(ref_path))
    r = _run(exe, "--scene", scene_path("2_gaussian.txt"), "--size", "24x24", "--integrator", "multiscatter", "--spp",
             "4", "--inverse", "3", "--ref", str(ref_path), "--seed", "5", "--stoch", "2", "--lr", "0.05",
             "--final-spp", "8")
    cpp = [float(ln.split()[-1]) for ln in r.stdout.splitlines() if ln.startswith("sfd iter")]
    cpp_final = float([ln for ln in r.stdout.splitlines() if ln.startswith("sfd final")][0].split()[-1])
    opt = inv.StochasticFiniteDiffInverseIntegrator(cam, vr.MultiScatterGaussians(cam, 4),
                                                    inv.SFDConfig(max_iters=3, num_stoch_samples=2, lr=0.05, seed=5,
                                                                  final_samples=8))
    assert opt.optimize(vr.Scene.load_GMM(scene_path("2_gaussian.txt")), vr.Image(str(ref_path)))
    assert len(cpp) == 3 and cpp == opt.history
    assert cpp_final == opt.final_loss
    assert np.all(np.isfinite(opt.history)) and not np.array_equal(opt.params, inv.pack_parameters(
        vr.Scene.load_GMM(scene_path("2_gaussian.txt"))))
