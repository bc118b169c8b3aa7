"""C4 ray-march diagnostics for A/B builds: frame / stage times of the product schedule plus the
instrumented counters of one frame (VR_LIB_PATH picks the library; diagnostic builds reuse the
secondary counter slots, see VR_DIAG_CYCLES / VR_DIAG_WAVE_UTIL in kernels/vr_gauss.hip).

  python3 tools/diag_c4.py [--size 4096] [--frames 3] [--counts 1]
Prints one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dg-vol-renderer_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
import vr_amd as vr  # noqa: E402
from vr_amd import tiles  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=4096)
ap.add_argument("--frames", type=int, default=3)
ap.add_argument("--counts", type=int, default=1)
ap.add_argument("--config", default="c4")
ap.add_argument("--opt", action="append", default=[], help="name=value device option (vr_set_option)")
args = ap.parse_args()

scene, W, H = bench.build_scene(args.config, 2025)
if args.size > 0:  # (0: the config's own frame size)
    W = H = args.size
cam = vr.Pinhole_Camera(bench.CAM_POS, bench.CAM_VIEW, bench.FOV)
integ = vr.RayMarchingGaussians(cam, step_size=0.01, env_samples=20, t_eps=1e-6)
dev = vr.Device.get(0)
for o in args.opt:
    k, v = o.split("=")
    dev.set_option(k, int(v))
dev.upload(scene)
frame = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
stats = []
for i in range(args.frames + 1):
    tiles.render_local(dev, cam, integ.params, W, H, 0, 1, None, frame, sp)
    if i:
        stats.append(dev.stats())
out = {"lib": os.environ.get("VR_LIB_PATH", "product"), "opt": args.opt,
       "kernel_ms": float(np.mean([s["kernel_ms"] for s in stats])),
       "stage_ms": {k: round(float(np.mean([s["stage_ms"][k] for s in stats])), 3) for k in vr.Device.STAGES},
       "mean": float(frame.mean()), "slow_rays": stats[-1]["slow_rays"], "band_rays": stats[-1]["band_rays"], "fallback_pixels": stats[-1]["fallback_pixels"],
       "scatter_records": stats[-1]["scatter_records"]}
if args.counts:
    out["work"] = dev.count_work(cam, integ.params, W, H)
print(json.dumps(out), flush=True)
