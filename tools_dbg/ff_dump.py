import sys, os
sys.path[:0] = ['3dg-vol-renderer_amd', 'tests']
import numpy as np, vr_amd as vr
from helpers import CAM_POS, FOV, main_view_dir, scene_path
os.makedirs('gpurun_out', exist_ok=True)
for name in ["1_gaussian.txt", "many_gaussians.txt"]:
    for multi in (False, True):
        for spp in (1, 4):
            cam = vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)
            integ = vr.MultiScatterGaussians(cam, spp) if multi else vr.FreeFlightGaussians(cam, spp)
            img = vr.Image(48, 48)
            integ.render(vr.Scene.load_GMM(scene_path(name)), img)
            np.save(f"gpurun_out/ff_{name[:-4]}_{int(multi)}_{spp}.npy", img.pixels)
print("ok")
