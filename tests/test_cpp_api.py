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
