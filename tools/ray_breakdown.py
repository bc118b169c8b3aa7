"""Per-Gaussian breakdown of one secondary ray of the C4 frame (t_eps 0): the oracle's segment loop
(orc_debug_secondary_ray: what each Gaussian contributes over the reference's segments) against a numpy model
of the device's whitened per-Gaussian intervals (vr_gauss.hip wtest / sec_finish), to find the Gaussian
whose treatment differs.  python3 tools/ray_breakdown.py x y k sample"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dg-vol-renderer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tools")]
import numpy as np
from scipy.special import erf
import pyoracle as O
import vr_amd as vr
from helpers import CAM_POS, FOV, main_view_dir
from test_gpu_parity import LIGHTS_1000

M64 = (1 << 64) - 1


def pcg_env_xi(seed, e):
    inc = (1 << 1) | 1
    st = 0
    st = (st * 6364136223846793005 + inc) & M64
    st = (st + seed) & M64
    st = (st * 6364136223846793005 + inc) & M64
    def nxt():
        nonlocal st
        old = st
        st = (old * 6364136223846793005 + inc) & M64
        sh = (((old >> 18) ^ old) >> 27) & 0xffffffff
        rot = old >> 59
        v = ((sh >> rot) | (sh << ((-rot) & 31))) & 0xffffffff
        return np.float32((v >> 8) * (1.0 / 16777216.0))
    for _ in range(2 * e):
        nxt()
    return nxt(), nxt()


def main():
    x, y, k, s = (int(v) for v in sys.argv[1:5])
    scene = vr.Scene(vr.Scene.GAUSSIANS)
    scene.add_random_gaussians(1_000_000, seed=2025, variant=0)
    g = scene.gaussians()
    osc = O.OracleScene.from_gaussians(g[:, 0:3], g[:, 3:9], g[:, 9], g[:, 10], np.array([l[0] for l in LIGHTS_1000], np.float32),
                                       np.array([l[1] for l in LIGHTS_1000], np.float32))
    rows = O.debug_pixel_records(osc, CAM_POS, main_view_dir(), FOV, x, y, 4096, 4096)
    row = rows[rows[:, 0] == k][0]
    pos = row[1:4].astype(np.float32)
    L = O.lib()
    L.orc_debug_record_active.restype = ctypes.c_int64
    L.orc_debug_record_active.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float), ctypes.c_float,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_int64), ctypes.c_int64]
    cp = np.ascontiguousarray(CAM_POS, np.float32)
    vd = np.ascontiguousarray(main_view_dir(), np.float32)
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    act = np.zeros(4096, np.int64)
    na = L.orc_debug_record_active(osc.h, fp(cp), fp(vd), float(FOV), x, y, 4096, 4096, 0.01, 20, k, act.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), 4096)
    act = act[:na]
    print(f"pixel ({x}, {y}) step {k}: pos {pos.tolist()} Ts {row[4]:.6g}, active {act.tolist()}")
    nl = 3
    if s < nl:
        lp = np.array(LIGHTS_1000[s][0], np.float32)
        dvec = lp - pos
        dist = np.float32(np.sqrt(np.float32(np.dot(dvec, dvec))))
        d = (dvec / dist).astype(np.float32)
        is_light = 1
    else:
        seed = int(O.lib().orc_derive_path_seed(x, y, k))
        xi1, xi2 = pcg_env_xi(seed, s - nl)
        d = np.zeros(3, np.float32)
        O.lib().orc_env_dir(ctypes.c_float(xi1), ctypes.c_float(xi2), fp(d))
        dist = np.float32(0)
        is_light = 0
    L.orc_debug_secondary_ray.restype = ctypes.c_int64
    L.orc_debug_secondary_ray.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                          ctypes.c_float, ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, ctypes.POINTER(ctypes.c_float),
                                          ctypes.c_int64, ctypes.POINTER(ctypes.c_float)]
    out = np.zeros((20000, 6), np.float32)
    tr = np.zeros(1, np.float32)
    n = L.orc_debug_secondary_ray(osc.h, fp(pos), fp(d), is_light, float(dist), act.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(act),
                                  fp(out), 20000, fp(tr))
    out = out[:n]
    print(f"ray {s} dir {d.tolist()} oracle Tr {tr[0]:.6f} (tau {-np.log(max(tr[0], 1e-30)):.5f}), {n} Gaussians active on it")
    # device model: whitened forms for every Gaussian (double here: the model, not the device's f32 bits)
    mean = g[:, 0:3].astype(np.float64)
    c6 = g[:, 3:9].astype(np.float64)
    cov = np.zeros((len(g), 3, 3))
    cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2], cov[:, 2, 2] = c6.T
    cov[:, 1, 0], cov[:, 2, 0], cov[:, 2, 1] = cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 2]
    Minv = np.linalg.inv(cov)
    Lc = np.linalg.cholesky(Minv)  # lower: M = Lc Lc^T; the device's upper L = Lc^T
    U = np.transpose(Lc, (0, 2, 1))
    p = np.einsum("nij,nj->ni", U, pos.astype(np.float64)[None] - mean)
    dd = np.einsum("nij,j->ni", U, d.astype(np.float64))
    a = (dd * dd).sum(1)
    h = (p * dd).sum(1)
    cq = (p * p).sum(1)
    r = 1 / np.sqrt(a)
    hr = h * r
    e2 = ((p - (h / a)[:, None] * dd) ** 2).sum(1)
    D = 9 - e2
    hit = D >= 0
    sd = np.sqrt(np.maximum(D, 0))
    t1 = r * (sd - hr)
    t0 = r * (-hr - sd)
    hit &= t1 >= 0
    det = np.linalg.det(cov)
    norm = (2 * np.pi) ** -1.5 * det ** -0.5
    dn = g[:, 9].astype(np.float64) * norm * np.sqrt(np.pi / 2)
    members = set(act.tolist())
    cmax = max(cq[i] for i in act) if len(act) else -np.inf
    lim = t1[hit].max() if hit.any() else 0.0
    rows_m = []
    for i in np.nonzero(hit | np.isin(np.arange(len(g)), act))[0]:
        mem = i in members
        if hit[i]:
            inside = hr[i] > -sd[i]
            lo_u = hr[i] if (mem or inside) else -sd[i]
            od = dn[i] * r[i] * np.exp(-e2[i] / 2) * (erf(sd[i] / np.sqrt(2)) - erf(lo_u / np.sqrt(2)))
        else:  # a member the ray misses: active to the last event
            od = dn[i] * r[i] * np.exp(-e2[i] / 2) * (erf((a[i] ** 0.5 * lim + hr[i]) / np.sqrt(2)) - erf(hr[i] / np.sqrt(2)))
        rows_m.append((i, mem, hit[i], t0[i], t1[i], od, cq[i]))
    model = {int(rw[0]): rw for rw in rows_m}
    orc = {int(rw[0]): rw for rw in out}
    tau_m = sum(rw[5] for rw in rows_m)
    print(f"device model tau {tau_m:.5f} Tr {np.exp(-tau_m):.6f}; cmax {cmax:.5f}; last event {lim:.5f}")
    print(" gauss   member  Mhit  whit   t0        t1        c        e2        od_oracle    od_model")
    for i in sorted(set(model) | set(orc), key=lambda i: -abs(model.get(i, (0,) * 7)[5] - (orc[i][5] if i in orc else 0))):
        om = orc[i][5] if i in orc else 0.0
        mm = model[i][5] if i in model else 0.0
        if abs(om - mm) < 1e-4 * max(1, abs(om)) and not (i in members or len(orc) < 8):
            continue
        mh = int(orc[i][2]) if i in orc else -1
        wh = int(model[i][2]) if i in model else -1
        ab = f" oracle f32 [{orc[i][3]:.7f}, {orc[i][4]:.7f}]" if i in orc else ""
        print(f" {i:7d}  {int(i in members):3d}    {mh:3d}  {wh:3d}  {t0[i]:9.5f} {t1[i]:9.5f} {cq[i]:8.5f} {e2[i]:8.5f} {om:11.6f}  {mm:11.6f}  dens {g[i, 9]:.4g}{ab}")


if __name__ == "__main__":
    main()
