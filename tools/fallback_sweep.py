"""Oracle sweep of the fallback pixels of the C4 frame at exact settings (t_eps = 0): every k-th pixel of
the sorted fallback list against the CPU restatement (16 threads), the worst pixels printed and those over
1e-4 re-checked with the stable tie order.  python3 tools/fallback_sweep.py [k]  (GPU box)"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dg-vol-renderer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np
import torch  # noqa
import vr_amd as vr
import pyoracle as O
from test_gpu_parity import _synthetic_scene
from helpers import CAM_POS, FOV, main_view_dir
scene, osc = _synthetic_scene(1_000_000)
cam = vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)
img = vr.Image(4096, 4096)
integ = vr.RayMarchingGaussians(cam, t_eps=0.0)
integ.render(scene, img)
fb = vr.Device.get(0).fallback_pixels()
order = np.lexsort((fb[:, 0], fb[:, 1]))
fb = fb[order]
step = int(sys.argv[1]) if len(sys.argv) > 1 else 40
pix = fb[::step].astype(np.int32)
print("fallback", len(fb), "sampled", len(pix), flush=True)
t = time.time()
ref = O.render(osc, O.PINHOLE, CAM_POS, main_view_dir(), FOV, 4096, 4096, O.RAYMARCH_GAUSSIANS_LISTS, 0.01, 20, pixels=pix, nthreads=16)
print("oracle", round(time.time() - t, 1), "s", flush=True)
got = img.pixels[pix[:, 1], pix[:, 0]].astype(np.float64)
d = np.abs(got - ref).max(axis=1)
idx = np.argsort(d)[::-1][:12]
print("over 1e-4:", int((d >= 1e-4).sum()), flush=True)
for i in idx:
    print(pix[i].tolist(), "dev", got[i].tolist(), "orc", ref[i].tolist(), "d", d[i], flush=True)
bad = pix[d >= 1e-4]
if len(bad):
    with O.stable_ties():
        ref_s = O.render(osc, O.PINHOLE, CAM_POS, main_view_dir(), FOV, 4096, 4096, O.RAYMARCH_GAUSSIANS_LISTS, 0.01, 20, pixels=bad, nthreads=16)
    gb = img.pixels[bad[:, 1], bad[:, 0]].astype(np.float64)
    print("stable-ties d:", np.abs(gb - ref_s).max(axis=1).tolist()[:12], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", "fallback_sweep_bad.npy"), bad)
