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
