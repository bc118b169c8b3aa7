"""Shared test helpers (camera setups of the reference driver, PPM reading, scene paths)."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
RENDERS = os.path.join(ROOT, "tests", "golden", "renders")

# tests/main.cpp:18-34 — camera (0,1,6) looking at (0,1,0), FOV pi/4
CAM_POS = np.array([0.0, 1.0, 6.0], np.float32)
CAM_LOOKAT = np.array([0.0, 1.0, 0.0], np.float32)
FOV = np.float32(0.25 * np.pi)


def main_view_dir():
    d = CAM_LOOKAT - CAM_POS
    return (d / np.sqrt(np.float32(np.dot(d, d)))).astype(np.float32)


def scene_path(name):
    return os.path.join(SCENES, name)


def read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(maxsplit=4)
    assert parts[0] == b"P6"
    W, H = int(parts[1]), int(parts[2])
    px = np.frombuffer(parts[4][: W * H * 3], np.uint8)
    return px.reshape(H, W, 3)


def to8(img):
    return np.clip(np.asarray(img, np.float32) * np.float32(255.0), 0.0, 255.0).astype(np.uint8)


def tie_aware_linf(got, pixels, render, tol):
    """Per-pixel L-inf of device pixels `got` ((n, 3)) against the oracle `render(pixels)` run with the
    reference's std::sort event order (on the reference's own BVH) and f32 arithmetic. A pixel over `tol` is
    re-rendered with stable tie order (pyoracle.stable_ties): it is tie-dependent only if the two oracle
    orders disagree there (a tangent hit whose entry and exit keys are equal), and is then held to the same
    bar against the stable order (the device's rule). Returns (max error, number of tie-dependent pixels,
    number of NaN mismatches, pixels over the bar that are not tie-dependent, the reference-order oracle
    pixels)."""
    import pyoracle as O
    got = np.asarray(got, np.float64)
    ref = np.asarray(render(pixels), np.float64)
    nan_mismatch = int(np.sum(np.isnan(got) != np.isnan(ref)))
    d = np.abs(got - ref)
    d[np.isnan(got) & np.isnan(ref)] = 0.0
    d = np.nanmax(d, axis=-1) if d.size else np.zeros(0)
    bad = np.nonzero(d >= tol)[0]
    explained = 0
    if bad.size:
        with O.stable_ties():
            ref_s = np.asarray(render(pixels[bad]), np.float64)
        tie = np.any(ref_s != ref[bad], axis=-1)
        d_s = np.nanmax(np.abs(got[bad] - ref_s), axis=-1)
        ok = tie & (d_s < tol)
        d[bad] = np.where(tie, d_s, d[bad])
        explained = int(ok.sum())
    return float(d.max()) if d.size else 0.0, explained, nan_mismatch, int(bad.size - explained), ref
