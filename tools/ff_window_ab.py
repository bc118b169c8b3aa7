"""A/B of VR_OPT_FF_WINDOW0 (first hit-window capacity of the free-flight event sweep) on the bench's
free-flight lines: frame time of the path kernel (HIP events) per setting. Results do not depend on it."""
import sys
import time

import numpy as np
import torch

import bench
import vr_amd as vr

for cfg, integ_name, spp in (("c2", "multiscatter", 16), ("c5", "multiscatter", 16), ("c4", "multiscatter", 1),
                             ("c3", "freeflight", 4)):
    scene, W, H = bench.build_scene(cfg, 2025)
    cam = vr.Pinhole_Camera(bench.CAM_POS, bench.CAM_VIEW, bench.FOV)
    integ = vr.MultiScatterGaussians(cam, spp, 5) if integ_name == "multiscatter" else vr.FreeFlightGaussians(cam, spp)
    dev = vr.Device.get(0)
    dev.upload(scene)
    img = vr.Image(W, H)
    for w0 in (0, 2, 4, 8, 16, 32):
        dev.set_option("ff_window0", w0)
        integ.render(scene, img)
        ts = []
        for _ in range(3):
            integ.render(scene, img)
            ts.append(dev.stats()["stage_ms"]["march"])
        print(cfg, "window0", w0, "path kernel ms", round(float(np.mean(ts)), 2), flush=True)
    dev.set_option("ff_window0", 0)
