"""GPU side of a per-pixel record comparison: render C4 (t_eps 0 unless --t-eps) and dump the scatter records of
the given pixels (vr_debug_pixel_records) to gpurun_out/<tag>_records.npz; tools/pixel_records_cmp.py compares
them with the oracle's.  python3 tools/pixel_records_dump.py TAG x,y [x,y ...]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dg-vol-renderer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
import numpy as np
import vr_amd as vr
from helpers import CAM_POS, FOV, main_view_dir
from c4_exact_dump import c4_scene

tag = sys.argv[1]
pix = [tuple(int(v) for v in a.split(",")) for a in sys.argv[2:]]
scene = c4_scene()
cam = vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)
img = vr.Image(4096, 4096)
integ = vr.RayMarchingGaussians(cam, t_eps=0.0)
integ.render(scene, img)
dev = vr.Device.get(0)
out = {}
for x, y in pix:
    out[f"{x}_{y}"] = dev.debug_pixel_records(x, y)
    out[f"{x}_{y}_px"] = img.pixels[y, x]
    print((x, y), "records", len(out[f"{x}_{y}"]), "pixel", img.pixels[y, x].tolist(), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"{tag}_records.npz"), **out)
