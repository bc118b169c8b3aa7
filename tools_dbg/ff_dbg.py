import sys, os
sys.path[:0] = ['3dg-vol-renderer_amd', 'tests']
os.makedirs('gpurun_out', exist_ok=True)
os.environ["VR_FF_DEBUG"] = "gpurun_out/ff_dbg_1g.bin"
import numpy as np, vr_amd as vr
from helpers import CAM_POS, FOV, main_view_dir, scene_path
cam = vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)
img = vr.Image(48, 48)
vr.FreeFlightGaussians(cam, 1).render(vr.Scene.load_GMM(scene_path("1_gaussian.txt")), img)
np.save("gpurun_out/ff_dbg_img.npy", img.pixels)
print("ok")
