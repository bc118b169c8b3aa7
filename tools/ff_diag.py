"""Raw work counters of one instrumented free-flight frame (vr_count_work) on the bench scene, for
diagnostic builds whose counters hold other statistics (VR_DIAG_FF_CYCLES, VR_DIAG_FFSM).
    python3 tools/ff_diag.py [cfg] [integrator] [spp]      (default c2 multiscatter 16)"""
import json
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import torch  # noqa: F401

import bench
import vr_amd as vr

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
integ = sys.argv[2] if len(sys.argv) > 2 else "multiscatter"
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 16
scene, W, H = bench.build_scene(cfg, 2025)
cam = vr.Pinhole_Camera(bench.CAM_POS, bench.CAM_VIEW, bench.FOV)
I = vr.MultiScatterGaussians(cam, spp, 5) if integ == "multiscatter" else vr.FreeFlightGaussians(cam, spp)
dev = vr.Device.get(0)
dev.upload(scene)
w = dev.count_work(cam, I.params, W, H)
raw = [w["path"][k] for k in vr.Device.WORK_NAMES["path"]]
out = {"config": cfg, "integrator": integ, "spp": spp, "path_raw": raw, "nee": w["nee"]}
if os.environ.get("DIAG_KIND") == "ffsm":
    cyc = raw[0:3]
    it = raw[3:6]
    out["ffsm"] = {
        "phase_cycles16": dict(zip(("collect", "sweep", "shade"), cyc)),
        "phase_share": {k: round(c / max(1, sum(cyc)), 4) for k, c in zip(("collect", "sweep", "shade"), cyc)},
        "iterations": dict(zip(("collect", "sweep", "shade"), it)),
        "lanes_per_iteration": {"collect": round(raw[6] / max(1, it[0]), 2), "sweep": round(raw[7] / max(1, it[1]), 2)},
        "cycles_per_iteration": {k: round(16 * c / max(1, n), 1) for k, c, n in zip(("collect", "sweep", "shade"), cyc, it)},
    }
if os.environ.get("DIAG_KIND") == "ffsm2":
    names = ("node", "prim", "sweep", "shade")
    cyc, it = raw[0:4], raw[4:8]
    out["ffsm2"] = {"phase_share": {k: round(c / max(1, sum(cyc)), 4) for k, c in zip(names, cyc)},
                    "iterations": dict(zip(names, it)),
                    "cycles_per_iteration": {k: round(16 * c / max(1, n), 1) for k, c, n in zip(names, cyc, it)}}
print(json.dumps(out))
