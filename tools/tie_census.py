"""Tie-order census (gmm.h:508-514): on a config's parity-test pixel sample, how many pixels
depend on the order std::sort leaves tangent-hit ties in (t0 == t1 in float: a ray grazing a 3-sigma
ellipsoid), and by how much. Both orders come from the oracle (the reference's libstdc++ std::sort order and
the stable emission order the device uses); a pixel is tie-dependent iff they differ. CPU only.
    python3 tools/tie_census.py c2|c3|c4 [threads] [extra.npz (xy: more pixels, e.g. every fallback pixel)]
Writes profiles/r05_tie_census_<cfg>.json."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dg-vol-renderer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np
import pyoracle as O
from helpers import CAM_POS, FOV, main_view_dir, scene_path


def tile_stratified(W, H, stride, seed):  # tests/test_gpu_parity.py _tile_stratified
    rng = np.random.default_rng(seed)
    tx, ty = (W + 15) // 16, (H + 15) // 16
    tiles = np.arange(0, tx * ty, stride)
    x = (tiles % tx) * 16 + rng.integers(0, 16, tiles.size)
    y = (tiles // tx) * 16 + rng.integers(0, 16, tiles.size)
    keep = (x < W) & (y < H)
    return np.stack([x[keep], y[keep]], 1).astype(np.int32)


def synthetic(n):
    import vr_amd as vr
    from test_gpu_parity import LIGHTS_1000 as L
    scene = vr.Scene(vr.Scene.GAUSSIANS)
    scene.add_random_gaussians(n, seed=2025, variant=0)
    g = scene.gaussians()
    return O.OracleScene.from_gaussians(g[:, 0:3], g[:, 3:9], g[:, 9], g[:, 10], np.array([l[0] for l in L], np.float32),
                                        np.array([l[1] for l in L], np.float32))


def main():
    cfg = sys.argv[1]
    nthreads = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 8)
    if cfg == "c2":
        W = H = 512
        osc = O.OracleScene.load_gmm(scene_path("1000_random.txt"))
        pix = tile_stratified(W, H, 1, seed=2)
        sample = "one pixel in every 16x16 tile (test_c2_tile_stratified_matches_list_oracle)"
    elif cfg == "c3":
        W, H = 1920, 1080
        osc = synthetic(100_000)
        pix = tile_stratified(W, H, 3, seed=11)
        sample = "one pixel in every 3rd tile (_check_full_size stratified part)"
    else:
        W = H = 4096
        osc = synthetic(1_000_000)
        pix = tile_stratified(W, H, 32, seed=11)
        sample = "one pixel in every 32nd tile (_check_full_size stratified part)"
    n_strat = len(pix)
    known_ref = None  # reference-order values of the extra pixels already computed (fallback_sweep_local.py)
    if len(sys.argv) > 3:
        extra = np.load(sys.argv[3])["xy"].astype(np.int32)
        pix = np.concatenate([pix, extra])
        sample += f" + {len(extra)} pixels of {os.path.basename(sys.argv[3])}"
        ref_path = sys.argv[3].replace("_fallback.npz", "_fallback_oracle.npy")
        if ref_path != sys.argv[3] and os.path.exists(ref_path):
            known_ref = np.load(ref_path).astype(np.float32)
    render = lambda p: O.render(osc, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, H, O.RAYMARCH_GAUSSIANS_LISTS, 0.01, 20,
                                pixels=p, nthreads=nthreads)
    out = {}
    for order in ("reference", "stable"):
        t0 = time.time()
        vals = np.zeros((len(pix), 3), np.float32)
        B = 4096
        todo = len(pix)
        if order == "reference" and known_ref is not None:
            vals[n_strat:] = known_ref
            todo = n_strat
        for i in range(0, todo, B):
            j = min(i + B, todo)
            if order == "stable":
                with O.stable_ties():
                    vals[i:j] = render(pix[i:j])
            else:
                vals[i:j] = render(pix[i:j])
            print(f"{cfg} {order}: {j}/{todo} {time.time() - t0:.0f} s", flush=True)
        out[order] = vals
    d = np.abs(out["reference"].astype(np.float64) - out["stable"]).max(axis=1)
    tie = d > 0.0
    res = {"config": cfg, "frame": [W, H], "sample": sample, "pixels": int(len(pix)), "stratified_pixels": n_strat,
           "tie_dependent_pixels": int(tie.sum()), "tie_dependent_stratified": int(tie[:n_strat].sum()),
           "fraction": float(tie.mean()), "fraction_stratified": float(tie[:n_strat].mean()),
           "estimated_frame_pixels": float(tie[:n_strat].mean()) * W * H,
           "max_effect": float(d.max()), "over_1e-4": int((d >= 1e-4).sum()),
           "worst": [[int(v) for v in pix[i]] + [float(d[i])] for i in np.argsort(d)[::-1][:10] if d[i] > 0]}
    print(json.dumps(res, indent=1), flush=True)
    with open(os.path.join(ROOT, "profiles", f"r05_tie_census_{cfg}.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
