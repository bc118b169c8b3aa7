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
