# render the C4 frame with the current secondary variant and save it (argv[1]) / compare two saves
import os, sys
import numpy as np
if sys.argv[1] == "cmp":
    a = np.load(sys.argv[2]); b = np.load(sys.argv[3])
    d = np.abs(a.astype(np.float64) - b)
    print("nan a/b:", int(np.isnan(a).sum()), int(np.isnan(b).sum()), "max|d|:", float(np.nanmax(d)),
          "n>1e-5:", int((d > 1e-5).sum()), "n>1e-4:", int((d > 1e-4).sum()), "mean:", float(np.nanmean(d)))
    idx = np.unravel_index(np.nanargmax(d), d.shape); print("worst", idx, a[idx[:2]], b[idx[:2]])
    sys.exit(0)
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
import bench
import vr_amd as vr
scene, W, H = bench.build_scene(os.environ.get("CFG", "c4"), 2025)
cam = vr.Pinhole_Camera(bench.CAM_POS, bench.CAM_VIEW, bench.FOV)
img = vr.Image(W, H)
vr.RayMarchingGaussians(cam, env_samples=20, t_eps=float(os.environ.get("TEPS", "1e-6"))).render(scene, img)
np.save(sys.argv[1], img.pixels)
print("saved", sys.argv[1], float(np.nanmax(img.pixels)))
