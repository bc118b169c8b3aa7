"""Tie-order census (gmm.h:457-515) against the reference's own BVH: on a config's parity-test
pixel sample, how many pixels depend on the order std::sort leaves tangent-hit ties in (t0 == t1 in float: a ray
grazing a 3-sigma ellipsoid), and by how much. The oracle builds the reference's midpoint BVH on the reference's
get_aabb boxes (gaussian.h:304-319, the oracle's default since round 6), so its pre-sort event arrays and the
libstdc++ std::sort outcome are the reference's, up to the bits of Eigen's f32 eigensolver (restated from Eigen
3.4.0's algorithm). Per pixel:
  * reference order: the oracle's default render, with the pixel's count of tangent ties (rays on which some
    Gaussian's entry and exit keys are equal);
  * stable order (the device's rule, tree-independent): rendered again only where the count is > 0 (elsewhere
    the two orders are the same array);
  * a pixel is tie-dependent iff the two differ.
Also checked: whether the reference's tighter-or-looser boxes change the event set itself (a box only culls, and
the f32 quadratic accepts fringe points outside the exact ellipsoid): the stratified sample is rendered in stable
order on a tree over the padded tight boxes (every fringe hit kept, what the device does) too; a pixel that differs
there lost or gained a fringe hit through the reference's boxes. For extra pixels whose reference-order values on
the padded tree are already known (<tag>_fallback_oracle.npy, tools/fallback_sweep_local.py) the same comparison
runs on the pixels without ties. CPU only.
    python3 tools/tie_census.py c2|c3|c4 [threads] [extra.npz (xy: more pixels, e.g. every fallback pixel)]
Writes profiles/r06_tie_census_<cfg>.json."""
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
    return lambda: O.OracleScene.from_gaussians(g[:, 0:3], g[:, 3:9], g[:, 9], g[:, 10],
                                                np.array([l[0] for l in L], np.float32),
                                                np.array([l[1] for l in L], np.float32))


def main():
    cfg = sys.argv[1]
    nthreads = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 8)
    if cfg == "c2":
        W = H = 512
        make = lambda: O.OracleScene.load_gmm(scene_path("1000_random.txt"))
        pix = tile_stratified(W, H, 1, seed=2)
        sample = "one pixel in every 16x16 tile (test_c2_tile_stratified_matches_list_oracle)"
    elif cfg == "c3":
        W, H = 1920, 1080
        make = synthetic(100_000)
        pix = tile_stratified(W, H, 3, seed=11)
        sample = "one pixel in every 3rd tile (_check_full_size stratified part)"
    else:
        W = H = 4096
        make = synthetic(1_000_000)
        pix = tile_stratified(W, H, 32, seed=11)
        sample = "one pixel in every 32nd tile (_check_full_size stratified part)"
    osc = make()
    with O.padded_boxes():
        osc_pad = make()
    n_strat = len(pix)
    old_ref = None  # reference-order values of the extra pixels on the padded tree (fallback_sweep_local.py)
    if len(sys.argv) > 3:
        extra = np.load(sys.argv[3])["xy"].astype(np.int32)
        pix = np.concatenate([pix, extra])
        sample += f" + {len(extra)} pixels of {os.path.basename(sys.argv[3])}"
        p = sys.argv[3].replace("_fallback.npz", "_fallback_oracle.npy")
        if p != sys.argv[3] and os.path.exists(p):
            old_ref = np.load(p).astype(np.float32)
    render = lambda sc, p, **kw: O.render(sc, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, H, O.RAYMARCH_GAUSSIANS_LISTS,
                                          0.01, 20, pixels=p, nthreads=nthreads, **kw)

    def batched(sc, p, ties=None, stable=False, what=""):
        vals = np.zeros((len(p), 3), np.float32)
        t0 = time.time()
        B = 4096
        for i in range(0, len(p), B):
            j = min(i + B, len(p))
            tb = np.zeros(j - i, np.int32) if ties is not None else None
            if stable:
                with O.stable_ties():
                    vals[i:j] = render(sc, p[i:j], ties=tb)
            else:
                vals[i:j] = render(sc, p[i:j], ties=tb)
            if ties is not None:
                ties[i:j] = tb
            print(f"{cfg} {what}: {j}/{len(p)} {time.time() - t0:.0f} s", flush=True)
        return vals

    ties = np.zeros(len(pix), np.int32)
    ref = batched(osc, pix, ties=ties, what="reference order")
    tp = np.nonzero(ties > 0)[0]
    st = ref.copy()
    if tp.size:
        st[tp] = batched(osc, pix[tp], stable=True, what="stable order (pixels with ties)")
    d = np.abs(ref.astype(np.float64) - st).max(axis=1)
    tie = d > 0.0
    # the event set: stable order on the padded-box tree (what the device keeps) vs the reference's tree
    pad = batched(osc_pad, pix[:n_strat], stable=True, what="stable order, padded-box tree (stratified)")
    dset = np.abs(pad.astype(np.float64) - st[:n_strat]).max(axis=1)
    res = {"config": cfg, "frame": [W, H], "tree": "the reference's midpoint BVH on get_aabb boxes (gaussian.h:304-319)",
           "sample": sample, "pixels": int(len(pix)), "stratified_pixels": n_strat,
           "pixels_with_tangent_ties": int((ties > 0).sum()), "tangent_ties": int(ties.sum()),
           "tie_dependent_pixels": int(tie.sum()), "tie_dependent_stratified": int(tie[:n_strat].sum()),
           "fraction": float(tie.mean()), "fraction_stratified": float(tie[:n_strat].mean()),
           "estimated_frame_pixels": float(tie[:n_strat].mean()) * W * H,
           "max_effect": float(d.max()), "over_1e-4": int((d >= 1e-4).sum()),
           "worst": [[int(v) for v in pix[i]] + [float(d[i])] for i in np.argsort(d)[::-1][:10] if d[i] > 0],
           "event_set_vs_padded_tree": {"pixels": n_strat, "differ": int((dset > 0).sum()),
                                        "over_1e-4": int((dset >= 1e-4).sum()), "max": float(dset.max()) if n_strat else 0.0}}
    if old_ref is not None:
        e = np.arange(n_strat, len(pix))
        no_tie = ties[e] == 0
        dold = np.abs(old_ref.astype(np.float64) - ref[e]).max(axis=1)
        res["extra_vs_padded_tree_reference_order"] = {
            "pixels": int(len(e)), "without_ties": int(no_tie.sum()), "differ_without_ties": int((dold[no_tie] > 0).sum()),
            "over_1e-4_without_ties": int((dold[no_tie] >= 1e-4).sum()),
            "max_without_ties": float(dold[no_tie].max()) if no_tie.any() else 0.0,
            "worst_without_ties": [[int(v) for v in pix[e][i]] + [float(dold[i])] for i in np.argsort(np.where(no_tie, dold, 0))[::-1][:10]
                                   if no_tie[i] and dold[i] > 0]}
        np.save(os.path.join(ROOT, "gpurun_out", f"r06_census_{cfg}_extra_reference.npy"), ref[e])
    print(json.dumps(res, indent=1), flush=True)
    with open(os.path.join(ROOT, "profiles", f"r06_tie_census_{cfg}.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
