#!/usr/bin/env python3
"""One C4 frame share (tiles r, r+R, ...) rendered --reps times, for rocprofv3 --kernel-trace: the
per-kernel cost of a share against the full frame (tools/rocpd_stats.py or the csv of each run).
    rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- python3 tools/share_prof.py --ranks 8
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dg-vol-renderer_amd")]

import torch  # noqa: E402,F401
import bench  # noqa: E402
import vr_amd as vr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
scene, W, H = bench.build_scene("c4", 2025)
cam = vr.Pinhole_Camera(bench.CAM_POS, bench.CAM_VIEW, bench.FOV)
integ = vr.RayMarchingGaussians(cam, step_size=0.01, env_samples=20, t_eps=1e-6)
dev = vr.Device.get(0)
dev.upload(scene)
nt = vr.num_tiles(W, H)
out = torch.empty((nt * 256 * 3,), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
count = len(range(a.rank, nt, a.ranks))
for i in range(a.reps + 1):
    dev.render_tiles_device(cam, integ.params, W, H, a.rank, a.ranks, count, True, out.data_ptr(), stream)
    dev.synchronize()
    s = dev.stats()
    print(f"share {a.rank}/{a.ranks}: {s['kernel_ms']:.2f} ms {s['stage_ms']}", flush=True)
