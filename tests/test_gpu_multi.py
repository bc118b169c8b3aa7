"""Multi-GPU context through the C ABI (vr_init_multi): the frame's 16x16 tiles are
dealt round-robin over the ranks, gathered to the first device (RCCL ncclSend/ncclRecv when every
rank has its own GPU, device copies when ranks share one) and unshuffled there; the root renders its
own tiles straight into the frame. On the one-GPU test box groups that list GPU 0 several times
exercise the split, the gather and the unshuffle (a one-rank group holds an RCCL communicator but,
with no other rank, sends nothing). Every result must equal the
single-device render bit for bit (pixels are independent; env and path RNG are keyed by pixel)."""
import os
import subprocess

import numpy as np
import pytest

import vr_amd as vr
from helpers import CAM_POS, FOV, ROOT, main_view_dir, read_ppm, scene_path

pytestmark = pytest.mark.gpu


def _cam():
    return vr.Pinhole_Camera(CAM_POS, main_view_dir(), FOV)


def _render(integ_cls, scene, W, H, device, **kw):
    img = vr.Image(W, H)
    integ = integ_cls(_cam(), device=device, **kw)
    integ.render(scene, img)
    return img.pixels.copy(), integ.last_stats


@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0), (0, 0, 0, 0, 0, 0, 0, 0)])
def test_group_render_equals_single_device(devices):
    scene = vr.Scene.load_GMM(scene_path("50_random.txt"))
    W, H = 100, 70
    ref, _ = _render(vr.RayMarchingGaussians, scene, W, H, 0)
    got, st = _render(vr.RayMarchingGaussians, scene, W, H, devices)
    dev = vr.Device.get(devices)
    assert dev.num_devices == len(devices)
    assert dev.uses_rccl == (len(set(devices)) == len(devices))
    assert np.array_equal(got, ref)
    nt = vr.num_tiles(W, H)
    per_rank = [dev.rank_stats(r)["pixels"] for r in range(len(devices))]
    assert per_rank == [len(range(r, nt, len(devices))) * 256 for r in range(len(devices))]
    assert st["pixels"] == nt * 256


def test_group_with_more_ranks_than_tiles():
    scene = vr.Scene.load_GMM(scene_path("2_gaussian.txt"))
    ref, _ = _render(vr.RayMarchingGaussians, scene, 20, 12, 0)  # 2 tiles
    got, _ = _render(vr.RayMarchingGaussians, scene, 20, 12, (0, 0, 0))
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("integ,kw", [(vr.MultiScatterGaussians, {"samples": 4}),
                                      (vr.PureRayMarching, {"env_samples": 4})])
def test_group_other_integrators(integ, kw):
    scene = vr.Scene.load_GMM(scene_path("many_gaussians.txt"))
    ref, _ = _render(integ, scene, 48, 40, 0, **kw)
    got, _ = _render(integ, scene, 48, 40, (0, 0), **kw)
    assert np.array_equal(got, ref)


def _nested(n, density):
    mean = np.tile(np.array([[0.0, 1.0, 0.0]], np.float32), (n, 1))
    sig = np.linspace(0.3, 0.4, n)
    cov = np.stack([sig ** 2, 0 * sig, 0 * sig, sig ** 2, 0 * sig, sig ** 2], 1).astype(np.float32)
    return vr.Scene.from_gaussians(mean, cov, np.full(n, density, np.float32), np.full(n, 0.5, np.float32),
                                   [vr.Light([0, 5, 0], [1, 1, 1])])


def test_group_deep_active_sets_equal_single_device():
    # 80 nested Gaussians: the deep march pass (active sets > 64) on every rank of the group
    scene = _nested(80, 1e-4)
    a, _ = _render(vr.RayMarchingGaussians, scene, 16, 16, 0, env_samples=1)
    b, st = _render(vr.RayMarchingGaussians, scene, 16, 16, (0, 0), env_samples=1)
    assert np.array_equal(a, b) and st["error_pixels"] == 0


def test_group_overflow_fails_loudly():
    # more Gaussians overlapping one point than every capacity holds (kActDeep = 2048)
    with pytest.raises(vr.VRError) as e:
        _render(vr.RayMarchingGaussians, _nested(2100, 1e-6), 4, 4, (0, 0), env_samples=1)
    assert e.value.status == 6


@pytest.mark.parametrize("devices", ["0", "0,0,0"])
def test_cpp_driver_on_a_group(tmp_path, devices):
    tools = os.path.join(ROOT, "tools")
    r = subprocess.run(["make", "-C", tools], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    outs = {}
    for tag, extra in (("single", []), ("group", ["--devices", devices])):
        out = tmp_path / f"{tag}.ppm"
        r = subprocess.run([os.path.join(tools, "vol_render"), "--scene", scene_path("many_gaussians.txt"), "--size",
                            "96x64", "--out", str(out), *extra], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        outs[tag] = (read_ppm(str(out)), r.stdout)
    ndev = len(devices.split(","))
    assert f"{ndev} device(s)" in outs["group"][1]
    # a group of distinct GPUs holds RCCL communicators; on this one-GPU box that is the one-rank group,
    # which has nothing to gather (the N > 1 ncclSend / ncclRecv branch runs only on a multi-GPU node)
    assert ("RCCL communicator (one rank" in outs["group"][1]) == (ndev == 1)
    assert "RCCL gather" not in outs["group"][1]
    assert np.array_equal(outs["single"][0], outs["group"][0])


def test_group_stats_sum_the_ranks():
    """vr_get_stats on a group: counts are the sum over the ranks (vr_get_rank_stats), times the slowest
    rank's, and stage_ms keeps its four stages (the group reduction once ran past the array)."""
    scene = vr.Scene.load_GMM(scene_path("50_random.txt"))
    devices = (0, 0, 0)
    _, st = _render(vr.RayMarchingGaussians, scene, 100, 70, devices)
    dev = vr.Device.get(devices)
    ranks = [dev.rank_stats(r) for r in range(len(devices))]
    assert len(st["stage_ms"]) == 4
    for key in ("pixels", "scatter_records", "secondary_rays", "fallback_pixels", "error_pixels", "deep_pixels", "slow_rays", "band_rays"):
        assert st[key] == sum(r[key] for r in ranks), key
    assert st["scatter_records"] > 0
    for stage, ms in st["stage_ms"].items():
        assert ms == max(r["stage_ms"][stage] for r in ranks), stage


@pytest.mark.timeout(600)
def test_c4_eight_way_split_equals_single_device():
    """BASELINE config 4 at full size (4096^2, 1M make_random Gaussians, the bench settings: 20 env
    samples, t_eps 1e-6) through vr_init_multi with eight ranks on GPU 0: every rank renders its
    interleaved 1/8 of the 65536 tiles (the root straight into the frame, the others into packed slabs
    gathered and unshuffled on the root). The reference's pixel loop is what the split shards
    (test_integrators.h:164): the frame must equal the one-device frame bit for bit."""
    scene = vr.Scene(vr.Scene.GAUSSIANS)
    scene.add_random_gaussians(1_000_000, seed=2025, variant=0)
    for p, i in [((0.0, 5.0, 0.1), (50.0, 0.0, 0.0)), ((-3.0, 3.0, 0.3), (0.0, 30.0, 0.0)),
                 ((3.0, 3.0, -0.2), (0.0, 0.0, 30.0))]:
        scene.add_light(vr.Light(p, i))
    W = H = 4096
    ref, st1 = _render(vr.RayMarchingGaussians, scene, W, H, 0, t_eps=1e-6)
    devices = (0,) * 8
    got, st8 = _render(vr.RayMarchingGaussians, scene, W, H, devices, t_eps=1e-6)
    assert st1["error_pixels"] == 0 and st8["error_pixels"] == 0
    assert st8["scatter_records"] == st1["scatter_records"]
    assert np.array_equal(got, ref)
    vr.Device._cache.pop(devices, None)  # release the eight full-size rank contexts


# ---- groups of distinct GPUs: RCCL between devices (runs itself on any multi-GPU box, skips on one GPU) ----

def _distinct_devices():
    n = vr.Device.count()
    if n < 2:
        pytest.skip(f"{n} GPU(s): the RCCL send/receive branch needs at least two distinct devices")
    return tuple(range(min(8, n)))


@pytest.mark.timeout(600)
def test_c4_split_over_distinct_gpus_equals_single_device():
    """BASELINE config 4 (4096^2, 1M make_random Gaussians, bench settings) through vr_init_multi over up to
    eight distinct GPUs: every rank renders its interleaved tiles on its own device, ranks 1 .. N-1 ncclSend
    their packed slabs to the root, which ncclRecvs them in one group and unshuffles them
    (vr_multi.cpp group_frame). The reference's pixel loop is what the split shards (test_integrators.h:164):
    the frame must equal the one-device frame bit for bit."""
    devices = _distinct_devices()
    scene = vr.Scene(vr.Scene.GAUSSIANS)
    scene.add_random_gaussians(1_000_000, seed=2025, variant=0)
    for p, i in [((0.0, 5.0, 0.1), (50.0, 0.0, 0.0)), ((-3.0, 3.0, 0.3), (0.0, 30.0, 0.0)),
                 ((3.0, 3.0, -0.2), (0.0, 0.0, 30.0))]:
        scene.add_light(vr.Light(p, i))
    W = H = 4096
    ref, st1 = _render(vr.RayMarchingGaussians, scene, W, H, 0, t_eps=1e-6)
    got, stn = _render(vr.RayMarchingGaussians, scene, W, H, devices, t_eps=1e-6)
    dev = vr.Device.get(devices)
    assert dev.uses_rccl and dev.num_devices == len(devices)
    assert st1["error_pixels"] == 0 and stn["error_pixels"] == 0
    assert stn["scatter_records"] == st1["scatter_records"]
    assert np.array_equal(got, ref)
    vr.Device._cache.pop(devices, None)


@pytest.mark.parametrize("integ,kw", [(vr.RayMarchingGaussians, {}), (vr.MultiScatterGaussians, {"samples": 4})])
def test_group_over_distinct_gpus_equals_single_device(integ, kw):
    """50_random.txt through a group of distinct GPUs (RCCL gather) for the ray-march and the free-flight
    integrators, and the group statistics summed over the ranks."""
    devices = _distinct_devices()
    scene = vr.Scene.load_GMM(scene_path("50_random.txt"))
    ref, _ = _render(integ, scene, 200, 150, 0, **kw)
    got, st = _render(integ, scene, 200, 150, devices, **kw)
    dev = vr.Device.get(devices)
    assert dev.uses_rccl
    assert np.array_equal(got, ref)
    assert st["pixels"] == sum(dev.rank_stats(r)["pixels"] for r in range(len(devices)))


@pytest.mark.timeout(600)
def test_bench_torchrun_over_distinct_gpus_equals_one_gpu(tmp_path):
    """bench.py --gpus N under torch.distributed.run (one process per GPU, nccl = RCCL): every rank renders
    its interleaved tiles, the slabs reach rank 0 in one batch_isend_irecv and are unshuffled there
    (vr_amd/tiles.py). Config 3 (1920x1080, 100k Gaussians): the gathered frame equals bench.py's one-GPU
    frame bit for bit, and the JSON line reports N GPUs."""
    import json
    import socket
    import sys
    devices = _distinct_devices()
    n = len(devices)
    common = ["--config", "c3", "--steps", "1", "--warmup", "1", "--cpu-budget", "0", "--flops", "0"]
    one = tmp_path / "one.npy"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", *common, "--dump-frame", str(one)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    many = tmp_path / "many.npy"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", str(n), *common, "--dump-frame", str(many)],
                       capture_output=True, text=True, timeout=420, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == n and line["value"] > 0
    assert np.array_equal(np.load(many), np.load(one))


def test_group_first_frame_queue_grows_to_its_bound_then_inline():
    """A fresh group sizes its first frame's shadow-ray queue as one context does (one ray per bounce up to
    min_bounces + 1) and renders the frame again while it is outgrown: with VR_OPT_FF_NEE_QUEUE = 16 a
    MultiScatter frame with min_bounces = 1 doubles its queue up to the bound and then traces inline, about
    five renders. The group follows the same attempt schedule as vr_render on one context (kFrameAttempts;
    it used to give up after four) and equals that context's frame bit for bit."""
    import ctypes
    scene = vr.Scene.load_GMM(scene_path("50_random.txt"))
    integ = vr.MultiScatterGaussians(_cam(), 16, 1)
    frames = []
    for devices in (0, (0, 0)):
        dev = vr.Device(devices)
        dev.set_option("ff_nee_queue", 16)
        dev.upload(scene)
        out = np.empty((40, 48, 3), np.float32)
        vr.check(vr.lib().vr_render(dev._h, ctypes.byref(integ.camera.struct), ctypes.byref(integ.params), 48, 40,
                                    vr.fptr(out)))
        frames.append(out)
    assert np.array_equal(frames[0], frames[1])
