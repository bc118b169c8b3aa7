"""Renders the bench's free-flight frames (bench scene and camera, full size) and prints a hash of each
frame's bytes: A/B builds that must not change results (VR_LIB_PATH) print the same hashes.
    python3 tools/ff_frame_hash.py [cfg:integrator:spp ...]   (default c2:multiscatter:4 c3:freeflight:1)"""
import hashlib
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import numpy as np
import torch  # noqa: F401

import bench
import vr_amd as vr

cases = sys.argv[1:] or ["c2:multiscatter:4", "c3:freeflight:1"]
cam = vr.Pinhole_Camera(bench.CAM_POS, bench.CAM_VIEW, bench.FOV)
for c in cases:
    cfg, integ, spp = c.split(":")
    scene, W, H = bench.build_scene(cfg, 2025)
    img = vr.Image(W, H)
    I = vr.MultiScatterGaussians(cam, int(spp), 5) if integ == "multiscatter" else vr.FreeFlightGaussians(cam, int(spp))
    I.render(scene, img)
    px = np.ascontiguousarray(img.pixels)
    if os.environ.get("FRAME_SAVE"):  # FRAME_SAVE=prefix: the frames as .npy for a pixel-level comparison
        np.save(f"{os.environ['FRAME_SAVE']}_{cfg}_{integ}_{spp}.npy", px)
    print(c, hashlib.sha256(px.tobytes()).hexdigest()[:16], float(np.nanmean(px)), int(np.isnan(px).any(axis=-1).sum()), flush=True)
