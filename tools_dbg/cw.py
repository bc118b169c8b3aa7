# work counters of one C4 frame for the current secondary variant (VR_SECONDARY env)
import os, sys, json
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
import bench
import vr_amd as vr
import torch
scene, W, H = bench.build_scene(os.environ.get("CFG", "c4"), 2025)
cam = vr.Pinhole_Camera(bench.CAM_POS, bench.CAM_VIEW, bench.FOV)
integ = vr.RayMarchingGaussians(cam, env_samples=20, t_eps=1e-6)
dev = vr.Device.get(0)
dev.upload(scene)
w = dev.count_work(cam, integ.params, W, H)
print(os.environ.get("VR_SECONDARY", "ww"), json.dumps(w["secondary"]))
if os.environ.get("VR_WW_PROF") in ("1", "2"):
    v = [w["secondary"][k] for k in vr.Device.WORK_NAMES]
    clk = os.environ["VR_WW_PROF"] == "2"
    names = ["node_iters", "prim_iters", "node_lanes", "prim_lanes"] + (
        ["node_cyc", "prim_cyc", "refill_cyc"] if clk else ["live_lanes", "queue_blocked", "either"]) + ["refills"]
    d = dict(zip(names, v))
    it = d["node_iters"] + d["prim_iters"]
    print("PROF", json.dumps(d))
    print("PROF per iteration: node lanes %.1f prim lanes %.1f" % (d["node_lanes"] / max(1, d["node_iters"]),
          d["prim_lanes"] / max(1, d["prim_iters"])))
    if clk:
        tot = d["node_cyc"] + d["prim_cyc"] + d["refill_cyc"]
        print("PROF cycles: node %.1f%% prim %.1f%% refill+finish %.1f%%" % (100 * d["node_cyc"] / tot, 100 * d["prim_cyc"] / tot,
              100 * d["refill_cyc"] / tot))
    else:
        print("PROF per iteration: live %.1f queue-blocked %.1f either %.1f" % (d["live_lanes"] / it, d["queue_blocked"] / it,
              d["either"] / it))
