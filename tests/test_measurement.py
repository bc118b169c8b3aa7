"""CPU checks of the measurement tools behind bench.py's HBM line (SURVEY.md §8(d) B_frame):
oracle/vr_oracle.cpp orc_primary_depths (termination distances) and orc_tile_bins (n_t)."""
import numpy as np

import pyoracle as O
from helpers import CAM_POS, FOV, main_view_dir, scene_path


def test_tile_bins_cover_every_gaussian_the_tile_rays_meet():
    """n_t is conservative: it counts at least every Gaussian that some pixel-centre ray of the tile
    enters before that tile's termination depth D_t."""
    osc = O.OracleScene.load_gmm(scene_path("50_random.txt"))
    W = H = 48
    depth = O.primary_depths(osc, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, H)
    nt = O.tile_bins(osc, CAM_POS, main_view_dir(), FOV, W, H, depth)
    tx = (W + 15) // 16
    hits = [set() for _ in range(nt.size)]
    for y in range(H):
        for x in range(W):
            t = (y // 16) * tx + x // 16
            D = depth[(y // 16) * 16:(y // 16) * 16 + 16, (x // 16) * 16:(x // 16) * 16 + 16].max()
            r = O.primary_ray(O.PINHOLE, CAM_POS, main_view_dir(), FOV, x, y, W, H)
            for i in range(osc.num):
                p = osc.probe(i, r[:3], r[3:])
                if p[0] and p[1] <= D:
                    hits[t].add(i)
    need = np.array([len(h) for h in hits])
    assert need.sum() > 0
    assert np.all(nt >= need), (nt, need)
    assert nt.sum() <= osc.num * nt.size  # sanity


def test_primary_depths_stop_at_t_eps():
    """A ray's depth is the end of the step after which T <= t_eps: smaller t_eps, deeper rays; rays
    without events are -1 and t_eps = 0 runs to the last event."""
    osc = O.OracleScene.load_gmm(scene_path("50_random.txt"))
    W = H = 32
    d6 = O.primary_depths(osc, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, H, t_eps=1e-6)
    d2 = O.primary_depths(osc, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, H, t_eps=1e-2)
    d0 = O.primary_depths(osc, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, H, t_eps=0.0)
    miss = d0 < 0
    assert np.array_equal(miss, d6 < 0) and miss.any() and (~miss).any()
    assert np.all(d2[~miss] <= d6[~miss]) and np.all(d6[~miss] <= d0[~miss])


def test_free_flight_roofline_from_work_counts():
    """bench.ff_roofline: the path kernel's executed flops are its counted node steps, ray-Gaussian
    tests and erf evaluations times FF_FLOP_WEIGHTS over its HIP-event time; the shadow-ray kernel is
    reported beside it; the algorithmic part leaves out tree steps."""
    import bench
    work = {"path": {"paths": 10, "bounces": 20, "node4_steps": 1000, "node2_steps": 10, "gaussian_tests": 500,
                     "erf_evals": 800, "nee_inline": 0, "nee_queued": 15},
            "nee": {"rays": 15, "node4_steps": 300, "gaussian_tests": 200, "optical_depths": 50, "unused4": 0,
                    "unused5": 0, "unused6": 0, "unused7": 0}}
    stage_ms = {"march": 2.0, "sizing": 0.0, "secondary": 1.0, "accumulate": 0.1}
    r = bench.ff_roofline(work, stage_ms, "nonexistent-config")
    w = bench.FF_FLOP_WEIGHTS
    path = 1000 * w["node4"] + 10 * w["node2"] + 500 * w["prim"] + 800 * w["erf"]
    assert r["executed_flops"] == path
    assert r["alg_flops"] == 500 * w["prim"] + 800 * w["erf"]
    assert abs(r["achieved"] - path / 2e-3 / 1e12) < 1e-15
    assert abs(r["frac"] - r["achieved"] / bench.FP32_PEAK_TFLOPS) < 1e-15
    assert r["nee_kernel"]["executed_flops"] == 300 * w["node4"] + 200 * w["prim"] + 50 * w["od"]
    assert r["bound"] == "valu" and r["traffic"] is None
