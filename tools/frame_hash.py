"""Renders the bench's C4 scene at 1024x1024 (RayMarchingGaussians, bench settings) and prints a hash
of the frame bytes: A/B builds that must not change results (VR_LIB_PATH) print the same hash."""
import hashlib
import sys

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import bench
import vr_amd as vr

# (argument "pure": PureRayMarching at 256x256, 4 environment samples, instead)
pure = len(sys.argv) > 1 and sys.argv[1] == "pure"
scene, _, _ = bench.build_scene("c4", 2025)
cam = vr.Pinhole_Camera(bench.CAM_POS, bench.CAM_VIEW, bench.FOV)
img = vr.Image(256, 256) if pure else vr.Image(1024, 1024)
if pure:
    vr.PureRayMarching(cam, step_size=0.01, env_samples=4).render(scene, img)
else:
    vr.RayMarchingGaussians(cam, step_size=0.01, env_samples=20, t_eps=1e-6).render(scene, img)
print(hashlib.sha256(np.ascontiguousarray(img.pixels).tobytes()).hexdigest()[:16], float(img.pixels.mean()))
