#!/usr/bin/env python3
"""Predicts the tile-split scaling on one GPU: renders each of the R interleaved
rank shares of a frame (tiles r, r+R, r+2R, ...) on its own and times it with the library's HIP
events (vr_get_stats kernel_ms). Predicted speed-up at R GPUs = full-frame time / slowest share
and, with the gather modelled, full-frame time / (slowest share + gather + root unshuffle): the root
renders its own tiles straight into the frame; every other rank's slab (its tiles x 256 px x 12 B)
reaches the root over its own xGMI link at --xgmi-gbs GB/s (the links run in parallel), then the root's
unshuffle reads and writes the other ranks' (R - 1) / R of the frame at --hbm-gbs.
Prints one JSON object.

    python tools/share_balance.py [--config c4|bias20k] [--ranks 2,4,8]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dg-vol-renderer_amd")]

import torch  # noqa: E402,F401  (its HIP runtime first, see vr_amd/_lib.py)
import bench  # noqa: E402
import vr_amd as vr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4", choices=["c4", "bias20k"])
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--t-eps", type=float, default=1e-6)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--xgmi-gbs", type=float, default=50.0, help="effective per-link xGMI rate of the gather")
    ap.add_argument("--hbm-gbs", type=float, default=4000.0, help="effective HBM rate of the root's unshuffle")
    a = ap.parse_args()
    if a.config == "c4":
        scene, W, H = bench.build_scene("c4", 2025)
        desc = bench.CONFIGS["c4"][3]
    else:
        scene = vr.Scene.load_GMM(os.path.join(ROOT, "tests", "golden", "scenes", "20k_bias.txt"))
        W = H = 4096
        desc = "4096x4096, scenes/gaussians/20k_bias.txt (y-skewed density)"
    cam = vr.Pinhole_Camera(bench.CAM_POS, bench.CAM_VIEW, bench.FOV)
    integ = vr.RayMarchingGaussians(cam, step_size=0.01, env_samples=20, t_eps=a.t_eps)
    dev = vr.Device.get(0)
    dev.upload(scene)
    nt = vr.num_tiles(W, H)
    out = torch.empty((nt * 256 * 3,), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    stages = {}

    def share(first, stride, count):
        times, st = [], []
        for _ in range(a.reps + 1):  # the first is a warm-up (sizes the record buffers)
            dev.render_tiles_device(cam, integ.params, W, H, first, stride, count, True, out.data_ptr(), stream)
            dev.synchronize()
            s = dev.stats()
            times.append(s["kernel_ms"])
            st.append(s["stage_ms"])
        stages[(first, stride)] = {k: float(np.median([x[k] for x in st[1:]])) for k in st[0]}
        return float(np.median(times[1:]))

    full = share(0, 1, nt)
    res = {"workload": desc, "width": W, "height": H, "tiles": nt, "full_frame_ms": full,
           "full_frame_stage_ms": stages[(0, 1)], "ranks": {}}
    for R in [int(x) for x in a.ranks.split(",")]:
        t = [share(r, R, len(range(r, nt, R))) for r in range(R)]
        slab = len(range(0, nt, R)) * 256 * 12  # bytes of the largest share's slab
        gather_ms = slab / (a.xgmi_gbs * 1e9) * 1e3
        unshuffle_ms = 2.0 * (nt - len(range(0, nt, R))) * 256 * 12 / (a.hbm_gbs * 1e9) * 1e3
        with_gather = max(t) + gather_ms + unshuffle_ms
        res["ranks"][R] = {"share_ms": t, "max_ms": max(t), "sum_ms": sum(t),
                           "stage_ms_of_slowest": stages[(int(np.argmax(t)), R)],
                           "imbalance_max_over_mean": max(t) / (sum(t) / R),
                           "predicted_speedup": full / max(t), "predicted_efficiency": full / max(t) / R,
                           "gather": {"slab_bytes": slab, "xgmi_gbs": a.xgmi_gbs, "gather_ms": gather_ms,
                                      "unshuffle_ms": unshuffle_ms, "hbm_gbs": a.hbm_gbs},
                           "predicted_speedup_with_gather": full / with_gather,
                           "predicted_efficiency_with_gather": full / with_gather / R}
        print(f"[share_balance] R={R}: max {max(t):.1f} ms, mean {sum(t) / R:.1f} ms, predicted speed-up "
              f"{full / max(t):.2f} ({full / with_gather:.2f} with the gather)", file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
