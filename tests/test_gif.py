"""Animated GIF writer (vr_gif_*; the role of gif-h in tests/main.cpp:81-114's turntable mode). CPU:
frames written by the library decode (Pillow) to the frames given, within the per-frame 256-colour
palette's quantisation error, with the delay and looping of the reference's GifBegin call."""
import ctypes

import numpy as np
import pytest

import vr_amd as vr
from vr_amd._lib import check, lib

PIL = pytest.importorskip("PIL.Image")


def _write(path, frames, delay):
    h = ctypes.c_void_p()
    H, W = frames[0].shape[:2]
    check(lib().vr_gif_begin(str(path).encode(), W, H, delay, ctypes.byref(h)))
    for f in frames:
        rgba = np.ascontiguousarray(f, np.uint8)
        check(lib().vr_gif_write_frame(h, rgba.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), delay))
    check(lib().vr_gif_end(h))


def test_gif_frames_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    W, H = 97, 61
    yy, xx = np.mgrid[0:H, 0:W]
    frames = []
    for k in range(4):  # smooth gradients + a few flat regions + noise: many distinct colours
        f = np.zeros((H, W, 4), np.uint8)
        f[..., 0] = (xx * 255 // (W - 1) + 40 * k) % 256
        f[..., 1] = yy * 255 // (H - 1)
        f[..., 2] = ((xx + yy) * 3 + rng.integers(0, 8, (H, W))) % 256
        f[10:20, 10:30, :3] = (135, 206, 234)
        f[..., 3] = 255
        frames.append(f)
    p = tmp_path / "a.gif"
    _write(p, frames, 3)
    im = PIL.open(p)
    assert im.n_frames == 4 and im.size == (W, H)
    assert im.info.get("loop") == 0 and im.info.get("duration") == 30
    for k in range(4):
        im.seek(k)
        got = np.asarray(im.convert("RGB"), np.int32)
        ref = frames[k][..., :3].astype(np.int32)
        err = np.abs(got - ref)
        assert err.mean() < 6 and np.percentile(err, 99) < 24, (k, err.mean(), err.max())
        assert np.array_equal(got[10:20, 10:30], np.broadcast_to(np.array([135, 206, 234]), (10, 20, 3))) or \
            np.abs(got[10:20, 10:30] - np.array([135, 206, 234])).max() <= 8


def test_gif_large_frame_exercises_code_table_resets(tmp_path):
    """A 512x512 noise frame overflows the 4096-entry LZW table many times."""
    rng = np.random.default_rng(1)
    f = np.zeros((512, 512, 4), np.uint8)
    f[..., :3] = rng.integers(0, 256, (512, 512, 3))
    f[..., 3] = 255
    p = tmp_path / "n.gif"
    _write(p, [f], 4)
    got = np.asarray(PIL.open(p).convert("RGB"), np.int32)
    assert got.shape == (512, 512, 3)
    assert np.abs(got - f[..., :3]).mean() < 40  # 256 colours for uniform noise: coarse but decodable
    assert np.array_equal(np.asarray(PIL.open(p).convert("P")), np.asarray(PIL.open(p).convert("P")))


def test_gif_errors(tmp_path):
    h = ctypes.c_void_p()
    with pytest.raises(vr.VRError):
        check(lib().vr_gif_begin(str(tmp_path / "nodir" / "x.gif").encode(), 4, 4, 3, ctypes.byref(h)))
    with pytest.raises(vr.VRError):
        check(lib().vr_gif_begin(str(tmp_path / "x.gif").encode(), 0, 4, 3, ctypes.byref(h)))


@pytest.mark.gpu
def test_turntable_gif_from_the_cpp_driver(tmp_path):
    """tools/vol_render --gif: the reference driver's turntable (main.cpp:81-114) — frames of an
    orthographic camera orbiting (0, 1, 0) at radius 6, height +1, RayMarchingGaussians; frame k
    decodes to the Python render of the same camera within the palette's quantisation error."""
    import os
    import subprocess
    from helpers import ROOT, scene_path
    tools = os.path.join(ROOT, "tools")
    assert subprocess.run(["make", "-C", tools], capture_output=True).returncode == 0
    out = tmp_path / "t.gif"
    r = subprocess.run([os.path.join(tools, "vol_render"), "--scene", scene_path("2g_altered.txt"), "--size", "64x48",
                        "--gif", str(out), "--frames", "4", "--env", "4"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    im = PIL.open(out)
    assert im.n_frames == 4 and im.info.get("duration") == 30 and im.info.get("loop") == 0
    scene = vr.Scene.load_GMM(scene_path("2g_altered.txt"))
    for k in (0, 3):
        a = np.float32(2.0 * np.pi * (k / 4.0))
        pos = np.array([0, 1, 0], np.float32) + np.array([6 * np.sin(a), 1.0, 6 * np.cos(a)], np.float32)
        vd = np.array([0, 1, 0], np.float32) - pos
        vd = vd / np.sqrt(np.dot(vd, vd))
        img = vr.Image(64, 48)
        vr.RayMarchingGaussians(vr.Orthographic_Camera(pos, vd), env_samples=4).render(scene, img)
        im.seek(k)
        got = np.asarray(im.convert("RGB"), np.int32)
        err = np.abs(got - img.to_uint8().astype(np.int32))
        assert err.mean() < 4 and err.max() <= 40, (k, err.mean(), err.max())
