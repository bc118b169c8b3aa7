import sys, os, numpy as np
sys.path[:0] = ['3dg-vol-renderer_amd', 'oracle', 'tests']
import vr_amd as vr
from helpers import CAM_POS, FOV, main_view_dir, scene_path
for name, W in [('50_random.txt', 256), ('250_random.txt', 128)]:
    scene = vr.Scene.load_GMM(scene_path(name))
    img = vr.Image(W, W)
    integ = vr.RayMarchingGaussians(vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV))
    integ.render(scene, img)
    np.save(f'gpurun_out/{name}_{W}.npy', img.pixels)
    print(name, integ.last_stats)
