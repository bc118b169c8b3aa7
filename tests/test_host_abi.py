"""CPU-only tests of libvr_hip.so's host side and C ABI (no GPU calls).

* the library loads and exports every function include/vr_hip.h declares;
* the Gaussian precompute (the 48-B HBM records) is bit-identical to the oracle's restatement of
  gaussian.h:52-55 — so device-vs-oracle parity is never polluted by input differences;
* camera bases and primary rays are bit-identical to the oracle (camera.h, ray.h);
* loaders reproduce scene.h's parsing quirks; the XML subset maps onto 1_spheres.txt; PPM I/O
  truncates like image.h:66;
* device entry points fail loudly (VR_ERR_HIP / VR_ERR_NOSCENE), never silently.
"""
import os
import re

import numpy as np
import pytest

import pyoracle as O
import vr_amd as vr
from vr_amd import _lib as L
from helpers import CAM_POS, FOV, ROOT, main_view_dir, scene_path


def _declared_functions():
    text = open(os.path.join(ROOT, "include", "vr_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vr_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = L.lib()
    declared = _declared_functions()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(L.SIGNATURES), set(declared) ^ set(L.SIGNATURES)
    assert b"gfx950" in lib.vr_version()


@pytest.mark.parametrize("name", ["1_gaussian.txt", "2_gaussian.txt", "many_gaussians.txt", "50_random.txt",
                                  "250_random.txt", "1000_random.txt", "god_ray.txt", "1_gaussian_rotated.txt"])
def test_records_bit_identical_to_oracle(name):
    s = vr.Scene.load_GMM(scene_path(name))
    o = O.OracleScene.load_gmm(scene_path(name))
    a, b = s.records(), o.records()
    assert a.shape == b.shape
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert len(s.lights) == o.num_lights


def test_records_from_arrays_match_oracle():
    rng = np.random.default_rng(1)
    n = 500
    mean = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    cov = []
    for _ in range(n):
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        c = q @ np.diag(rng.uniform(0.005, 0.0175, 3) ** 2) @ q.T
        cov.append([c[0, 0], c[0, 1], c[0, 2], c[1, 1], c[1, 2], c[2, 2]])
    cov = np.asarray(cov, np.float32)
    dens = rng.uniform(0.2, 0.5, n).astype(np.float32)
    alb = rng.uniform(0.25, 0.95, n).astype(np.float32)
    s = vr.Scene.from_gaussians(mean, cov, dens, alb)
    o = O.OracleScene.from_gaussians(mean, cov, dens, alb, np.zeros((0, 3)), np.zeros((0, 3)))
    assert np.array_equal(s.records().view(np.uint32), o.records().view(np.uint32))


@pytest.mark.parametrize("cam_type,pos,vd,fov", [
    (0, CAM_POS, None, FOV),
    (1, CAM_POS, None, 0.0),
    (0, [0.3, 2.0, 5.0], [-0.1, -0.3, -1.0], 0.7),
    (1, [-2.0, 1.0, 4.0], [0.5, 0.1, -0.8], 0.0),
])
def test_camera_and_primary_rays_bit_identical(cam_type, pos, vd, fov):
    pos = np.asarray(pos, np.float32)
    vd = main_view_dir() if vd is None else np.asarray(vd, np.float32)
    cam = vr.Pinhole_Camera(pos, vd, fov) if cam_type == 0 else vr.Orthographic_Camera(pos, vd)
    ref = O.camera(cam_type, pos, vd, fov)
    b = cam.basis()
    got = np.concatenate([[cam.struct.type], b["position"], b["view_dir"], b["right"], b["up"], b["pinhole"] if
                          cam_type == 0 else ref[13:16], [cam.struct.focal_length if cam_type == 0 else ref[16]]])
    assert np.array_equal(got.astype(np.float32).view(np.uint32), ref.view(np.uint32))
    W, H = 37, 23
    for x, y in [(0, 0), (36, 22), (18, 11), (5, 17)]:
        r = cam.sample_ray(((x + np.float32(0.5)) / np.float32(W), (y + np.float32(0.5)) / np.float32(H)))
        ro = O.primary_ray(cam_type, pos, vd, fov, x, y, W, H)
        assert np.array_equal(np.concatenate([r.origin, r.direction]).view(np.uint32), ro.view(np.uint32))


def test_load_gmm_quirks(tmp_path):
    # comment tokens are skipped one at a time; emission optional; trailing blank on the last line ok
    p = tmp_path / "q.txt"
    p.write_text("// a comment line with words\n"
                 "l 0 5 0 1 2 3\n"
                 "g 0 1 0 0.1 0 0 0.1 0 0.1 1.0 0.5 0.2 0.3 0.4\n"
                 "g 0 1 1 0.2 0 0 0.2 0 0.2 2.0 0.25\n"
                 "g 1 1 1 0.3 0 0 0.3 0 0.3 3.0 0.75 \n")
    s = vr.Scene.load_GMM(p)
    g = s.gaussians()
    assert g.shape == (3, 14)
    np.testing.assert_array_equal(g[0, 11:14], np.float32([0.2, 0.3, 0.4]))
    np.testing.assert_array_equal(g[1, 11:14], 0)
    assert s.lights[0].intensity.tolist() == [1.0, 2.0, 3.0]
    # scene.h:99-106: trailing blank + no emission swallows the next line's tag
    q = tmp_path / "q2.txt"
    q.write_text("g 0 1 0 0.1 0 0 0.1 0 0.1 1.0 0.5 \ng 0 1 1 0.2 0 0 0.2 0 0.2 2.0 0.25\n")
    s2 = vr.Scene.load_GMM(q)
    assert s2.get_num_primitives() == O.OracleScene.load_gmm(q).num == 1


def test_load_smm_crlf_and_missing_file():
    s = vr.Scene.load_SMM(scene_path("sph_1_spheres.txt"))
    sp = s.spheres()
    np.testing.assert_array_equal(sp, np.float32([[0, 1, 0, 1, 0.1, 0.7]]))
    assert s.lights[0].position.tolist() == [0.0, 4.0, 0.0]
    with pytest.raises(vr.VRError) as e:
        vr.Scene.load_GMM("/nonexistent/scene.txt")
    assert e.value.status == 2 and "Failed to open scene file" in str(e.value)


def test_xml_subset_maps_to_reference_scene():
    scene, cam, (W, H), kw = vr.Scene.load_XML(scene_path("env_one_sphere_test_ortho.xml"))
    ref = vr.Scene.load_SMM(scene_path("sph_1_spheres.txt"))
    assert (W, H) == (512, 512)
    assert kw == {"step_size": np.float32(0.01), "env_samples": 5}
    assert np.array_equal(scene.spheres(), ref.spheres())
    assert scene.lights[0].position.tolist() == ref.lights[0].position.tolist()
    assert scene.lights[0].intensity.tolist() == ref.lights[0].intensity.tolist()
    np.testing.assert_array_equal(scene.env_color, np.float32([0.53, 0.81, 0.92]))
    assert cam.struct.type == 1
    o = O.camera(1, np.float32([0, 1, 6]), np.float32([0, 0, -1]))
    b = cam.basis()
    assert np.array_equal(np.concatenate([b["position"], b["view_dir"], b["right"], b["up"]]), o[1:13])


def test_xml_errors(tmp_path):
    p = tmp_path / "bad.xml"
    p.write_text("<scene><shape type='sphere'><float name='radius' value='1'/></shape>")
    with pytest.raises(vr.VRError) as e:
        vr.Scene.load_XML(p)
    assert e.value.status == 3


def test_ppm_roundtrip_truncates_like_reference(tmp_path):
    img = vr.Image(3, 2)
    img.pixels[...] = np.float32([[[0.0, 0.5, 1.0], [1.5, -0.2, 0.999], [0.1, 0.2, 0.3]],
                                  [[0.53, 0.81, 0.92], [0.00392, 0.00393, 0.9999], [1, 1, 1]]])
    p = tmp_path / "a.ppm"
    img.make_PPM(p)
    raw = open(p, "rb").read()
    assert raw.startswith(b"P6\n3 2\n255\n")
    px = np.frombuffer(raw[len(b"P6\n3 2\n255\n"):], np.uint8).reshape(2, 3, 3)
    assert np.array_equal(px, img.to_uint8())
    assert px[1, 0].tolist() == [135, 206, 234]  # env colour, truncated (SURVEY §4 miss-mask KAT)
    back = vr.Image(p)
    assert back.get_width() == 3 and back.get_height() == 2
    np.testing.assert_array_equal(back.pixels, px.astype(np.float32) / np.float32(255.0))


def test_device_entry_points_fail_loudly_without_scene_or_gpu():
    try:
        dev = vr.Device(0)
    except vr.VRError as e:  # no GPU in this container: must be a HIP error, not a fallback
        assert e.status == 4
        return
    cam = vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)
    integ = vr.RayMarchingGaussians(cam)
    import ctypes
    out = np.zeros((4, 4, 3), np.float32)
    st = L.lib().vr_render(dev._h, ctypes.byref(cam.struct), ctypes.byref(integ.params), 4, 4, L.fptr(out))
    assert st == 5


def test_option_table_mirrors_the_header():
    """Every vr_option of include/vr_hip.h has the same value in vr_amd._lib and a Device.set_option name
    (the Python mirror cannot drift from the ABI's option numbers)."""
    header = open(os.path.join(ROOT, "include", "vr_hip.h")).read()
    enum = header[header.index("typedef enum vr_option"):]
    enum = enum[:enum.index("} vr_option;")]
    declared = {m.group(1): int(m.group(2)) for m in re.finditer(r"(VR_OPT_[A-Z0-9_]+)\s*=\s*(\d+)", enum)}
    assert len(declared) >= 11
    for name, value in declared.items():
        assert getattr(L, name) == value, name
    assert sorted(vr.Device.OPTIONS.values()) == sorted(declared.values())


def test_num_tiles():
    assert vr.num_tiles(16, 16) == 1
    assert vr.num_tiles(17, 16) == 2
    assert vr.num_tiles(4096, 4096) == 65536
    assert vr.num_tiles(1920, 1080) == 120 * 68
