# Render C3 (exact settings) and save the frame + fallback pixels for offline oracle comparison.
import os, sys
import numpy as np
sys.path[:0] = ['3dg-vol-renderer_amd', 'oracle', 'tests', '.']
import vr_amd as vr
from test_gpu_parity import _synthetic_scene
from helpers import CAM_POS, FOV, main_view_dir
W, H, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
teps = float(sys.argv[4])
scene, osc = _synthetic_scene(n)
img = vr.Image(W, H)
integ = vr.RayMarchingGaussians(vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV), t_eps=teps)
integ.render(scene, img)
print(integ.last_stats)
np.save(f'gpurun_out/frame_{W}_{n}_{teps}.npy', img.pixels)
