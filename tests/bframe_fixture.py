#!/usr/bin/env python3
"""Generates tests/golden/bframe_<config>.json: SURVEY.md §8(d)'s algorithmic bytes of one bench.py frame,
    B_frame = 48 sum_t n_t + 4 sum_t n_t + 12 W H,
n_t = the Gaussians whose conservative 3-sigma box overlaps 16x16 tile t's frustum up to the tile's
termination depth D_t (largest termination distance of its primary rays: the end of the step after
which T <= t_eps, or the last event). Termination depths come from the CPU restatement's primary
march (oracle orc_primary_depths), n_t from its tile binning (orc_tile_bins) — measurement
infrastructure, not the kernel. bench.py reads the JSON for its HBM line (it never runs the oracle).

    python tests/bframe_fixture.py [--config c4] [--t-eps 1e-6]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "3dg-vol-renderer_amd")]

import pyoracle as O  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--t-eps", type=float, default=1e-6)
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    scene, W, H = bench.build_scene(a.config, a.seed)
    g = scene.gaussians()
    lights = scene.lights
    osc = O.OracleScene.from_gaussians(g[:, 0:3], g[:, 3:9], g[:, 9], g[:, 10],
                                       np.array([l.position for l in lights], np.float32),
                                       np.array([l.intensity for l in lights], np.float32))
    t0 = time.time()
    depth = O.primary_depths(osc, O.PINHOLE, bench.CAM_POS, bench.CAM_VIEW, bench.FOV, W, H, 0.01, a.t_eps,
                             nthreads=a.threads)
    t1 = time.time()
    nt = O.tile_bins(osc, bench.CAM_POS, bench.CAM_VIEW, bench.FOV, W, H, depth, nthreads=a.threads)
    t2 = time.time()
    s = int(nt.astype(np.int64).sum())
    out = {"config": a.config, "width": W, "height": H, "gaussians": int(len(g)), "seed": a.seed, "t_eps": a.t_eps,
           "step_size": 0.01, "tiles": int(nt.size), "sum_n_t": s, "mean_n_t": float(nt.mean()), "max_n_t": int(nt.max()),
           "B_frame": 48 * s + 4 * s + 12 * W * H, "hit_fraction": float((depth >= 0).mean()),
           "mean_depth_of_hits": float(depth[depth >= 0].mean()) if (depth >= 0).any() else None,
           "seconds": {"depths": t1 - t0, "binning": t2 - t1},
           "generator": "tests/bframe_fixture.py (oracle orc_primary_depths + orc_tile_bins)"}
    path = os.path.join(HERE, "golden", f"bframe_{a.config}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
