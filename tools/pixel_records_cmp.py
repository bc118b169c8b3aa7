"""CPU side of tools/pixel_records_dump.py: the oracle's scattering steps of each dumped pixel against the
device's records, step by step (position, T sigma_s, Li + Le, every secondary ray's Tr).
    python3 tools/pixel_records_cmp.py TAG [threshold]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dg-vol-renderer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tools")]
import numpy as np
import pyoracle as O
from helpers import CAM_POS, FOV, main_view_dir
from fallback_sweep_local import c4_oracle_scene

tag = sys.argv[1]
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-4
d = np.load(os.path.join(ROOT, "gpurun_out", f"{tag}_records.npz"))
osc = c4_oracle_scene()
for key in d.files:
    if key.endswith("_px"):
        continue
    x, y = (int(v) for v in key.split("_"))
    dev = d[key].astype(np.float64)
    orc = O.debug_pixel_records(osc, CAM_POS, main_view_dir(), FOV, x, y, 4096, 4096).astype(np.float64)
    print(f"== pixel ({x}, {y}): device {len(dev)} records, oracle {len(orc)}; pixel dev {d[key + '_px'].tolist()}")
    ko = {int(r[0]): r for r in orc}
    kd = {int(r[0]): r for r in dev}
    only_d = sorted(set(kd) - set(ko))
    only_o = sorted(set(ko) - set(kd))
    if only_d or only_o:
        print("  steps only on the device:", only_d[:20], " only in the oracle:", only_o[:20])
    for k in sorted(set(kd) & set(ko)):
        a, b = kd[k], ko[k]
        dpos = np.abs(a[1:4] - b[1:4]).max()
        dts = abs(a[4] - b[4]) / max(abs(b[4]), 1e-30)
        drad = np.abs(a[5:8] - b[5:8]).max()
        dtr = np.abs(a[9:] - b[9:])
        bad = np.nonzero(dtr > thr)[0]
        if dpos > 0 or dts > 1e-5 or drad > thr or len(bad) or a[8] != b[8]:
            print(f"  k {k}: dpos {dpos:.2e} Ts dev {a[4]:.6e} orc {b[4]:.6e} (rel {dts:.1e}) act dev {int(a[8])} orc {int(b[8])} "
                  f"rad dev {a[5]:.5f} orc {b[5]:.5f}")
            for s in bad:
                print(f"      ray {s} ({'light' if s < 3 else 'env ' + str(s - 3)}): Tr dev {a[9 + s]:.6f} orc {b[9 + s]:.6f}")
