"""vr_amd — Python mirror of the reference's forward-render API over libvr_hip.so.

Names, argument meaning and error behaviour follow wantonsushi/3DG-vol-renderer:

    scene = Scene.load_GMM("scenes/gaussians/many_gaussians.txt")      # scene.h:72-120
    camera = Pinhole_Camera(position, view_dir, fov)                    # camera.h:31-54
    image = Image(512, 512)                                             # image.h:9-20
    RayMarchingGaussians(camera).render(scene, image)                   # test_integrators.h:143-297
    image.make_PPM("output.ppm")                                        # image.h:62-84

Everything runs through the C ABI (include/vr_hip.h); rendering happens on the GPU only. Errors
are raised as VRError (a RuntimeError), as the reference raises std::runtime_error.
"""
import ctypes
import os

import numpy as np

from . import _lib as L
from ._lib import VRError, check, fptr, lib

__all__ = [
    "VRError", "Light", "Scene", "Camera", "Pinhole_Camera", "Orthographic_Camera", "Ray", "Image",
    "Integrator", "RayMarchingGaussians", "PureRayMarching", "RayMarchingSpheres", "FreeFlightGaussians",
    "MultiScatterGaussians", "bits_to_lists", "TestIntegrator", "Device",
    "load_xml",
    "num_tiles",
]


def _v3(x):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32).reshape(3))
    return a


class Light:
    """scene.h:12-15"""

    def __init__(self, position, intensity):
        self.position = _v3(position)
        self.intensity = _v3(intensity)

    def __repr__(self):
        return f"Light(position={self.position.tolist()}, intensity={self.intensity.tolist()})"


class Scene:
    """Scene (scene.h:17-205). Owns a native vr_scene handle.

    volume_type: "GAUSSIANS" or "SPHERES". Mutations (add_*, env_color) bump `version` so a
    device context re-uploads before the next render.
    """

    GAUSSIANS = L.VR_VOLUME_GAUSSIANS
    SPHERES = L.VR_VOLUME_SPHERES

    def __init__(self, volume_type=GAUSSIANS, _handle=None):
        if _handle is None:
            h = ctypes.c_void_p()
            check(lib().vr_scene_create(int(volume_type), ctypes.byref(h)))
            _handle = h
        self._h = _handle
        self.version = 0

    # ---- loaders ----
    @classmethod
    def load_GMM(cls, filename):
        h = ctypes.c_void_p()
        check(lib().vr_scene_load_gmm(os.fsencode(str(filename)), ctypes.byref(h)))
        return cls(_handle=h)

    @classmethod
    def load_SMM(cls, filename):
        h = ctypes.c_void_p()
        check(lib().vr_scene_load_smm(os.fsencode(str(filename)), ctypes.byref(h)))
        return cls(_handle=h)

    @classmethod
    def load_XML(cls, filename):
        """Mitsuba-subset XML -> (scene, camera, (width, height), integrator_kwargs)."""
        h = ctypes.c_void_p()
        cam = L.vr_camera()
        w, hh = ctypes.c_uint32(), ctypes.c_uint32()
        p = L.vr_render_params()
        check(lib().vr_scene_load_xml(os.fsencode(str(filename)), ctypes.byref(h), ctypes.byref(cam),
                                      ctypes.byref(w), ctypes.byref(hh), ctypes.byref(p)))
        scene = cls(_handle=h)
        camera = Camera._from_struct(cam)
        kw = {"step_size": p.step_size, "env_samples": p.env_samples}
        return scene, camera, (w.value, hh.value), kw

    @classmethod
    def from_gaussians(cls, mean, cov6, density, albedo, lights=(), env_color=None, emission=None):
        """Build a Gaussian scene from arrays (n,3), (n,6) [xx xy xz yy yz zz], (n,), (n,)."""
        s = cls(cls.GAUSSIANS)
        s.add_gaussians(mean, cov6, density, albedo, emission)
        for l in lights:
            s.add_light(l)
        if env_color is not None:
            s.env_color = env_color
        return s

    # ---- mutation ----
    def add_gaussians(self, mean, cov6, density, albedo, emission=None):
        mean = np.asarray(mean, np.float32).reshape(-1, 3)
        n = mean.shape[0]
        cov6 = np.asarray(cov6, np.float32).reshape(n, 6)
        arr = (L.vr_gaussian * max(n, 1))()
        buf = np.frombuffer(arr, dtype=np.float32).reshape(max(n, 1), 14)
        if n:
            buf[:n, 0:3] = mean
            buf[:n, 3:9] = cov6
            buf[:n, 9] = np.asarray(density, np.float32).reshape(n)
            buf[:n, 10] = np.asarray(albedo, np.float32).reshape(n)
            buf[:n, 11:14] = 0.0 if emission is None else np.asarray(emission, np.float32).reshape(n, 3)
        check(lib().vr_scene_add_gaussians(self._h, arr, n))
        self.version += 1

    def add_random_gaussians(self, n, seed=0, variant=0):
        """Synthetic Gaussians with make_random.py's (variant 0) or make_nonuniform_random.py's
        (variant 1) distribution, generated natively (vr_scene_add_random_gaussians)."""
        check(lib().vr_scene_add_random_gaussians(self._h, int(n), int(seed), int(variant)))
        self.version += 1

    def add_spheres(self, center, radius, sigma_a, sigma_s):
        center = np.asarray(center, np.float32).reshape(-1, 3)
        n = center.shape[0]
        arr = (L.vr_sphere * max(n, 1))()
        buf = np.frombuffer(arr, dtype=np.float32).reshape(max(n, 1), 6)
        if n:
            buf[:n, 0:3] = center
            buf[:n, 3] = np.asarray(radius, np.float32).reshape(n)
            buf[:n, 4] = np.asarray(sigma_a, np.float32).reshape(n)
            buf[:n, 5] = np.asarray(sigma_s, np.float32).reshape(n)
        check(lib().vr_scene_add_spheres(self._h, arr, n))
        self.version += 1

    def add_light(self, light):
        l = L.vr_light()
        l.position[:] = [float(v) for v in light.position]
        l.intensity[:] = [float(v) for v in light.intensity]
        check(lib().vr_scene_add_lights(self._h, ctypes.byref(l), 1))
        self.version += 1

    # ---- queries ----
    def info(self):
        i = L.vr_scene_info()
        check(lib().vr_scene_get_info(self._h, ctypes.byref(i)))
        return i

    @property
    def volume_type(self):
        return self.info().volume_type

    def get_num_primitives(self):
        return int(self.info().num_primitives)

    @property
    def lights(self):
        n = int(self.info().num_lights)
        arr = (L.vr_light * max(n, 1))()
        check(lib().vr_scene_get_lights(self._h, arr, n))
        return [Light(list(arr[i].position), list(arr[i].intensity)) for i in range(n)]

    @property
    def env_color(self):
        return np.array(list(self.info().env_color), np.float32)

    @env_color.setter
    def env_color(self, rgb):
        a = _v3(rgb)
        check(lib().vr_scene_set_env_color(self._h, fptr(a)))
        self.version += 1

    def records(self):
        """Precomputed Gaussian records (n, 12): mean3, density, inv_cov 00 01 02 11 12 22, norm, albedo."""
        n = self.get_num_primitives()
        out = np.zeros((n, 12), np.float32)
        check(lib().vr_scene_get_records(self._h, fptr(out), n))
        return out

    def gaussians(self):
        n = self.get_num_primitives()
        arr = (L.vr_gaussian * max(n, 1))()
        check(lib().vr_scene_get_gaussians(self._h, arr, n))
        return np.frombuffer(arr, dtype=np.float32).reshape(max(n, 1), 14)[:n].copy()

    def spheres(self):
        n = self.get_num_primitives()
        arr = (L.vr_sphere * max(n, 1))()
        check(lib().vr_scene_get_spheres(self._h, arr, n))
        return np.frombuffer(arr, dtype=np.float32).reshape(max(n, 1), 6)[:n].copy()

    def unshuffle_tiles_part_device(self, slabs_ptr, first, nslabs, stride, tiles_per_slab, width, height, image_ptr,
                                    stream_ptr=0):
        """Slabs of ranks first .. first + nslabs - 1 of a stride-way split into the frame
        (vr_unshuffle_tiles_part_device)."""
        check(lib().vr_unshuffle_tiles_part_device(self._h, ctypes.c_void_p(slabs_ptr), first, nslabs, stride,
                                                   tiles_per_slab, width, height, ctypes.c_void_p(image_ptr),
                                                   ctypes.c_void_p(stream_ptr)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and L is not None and L._lib is not None:  # (L is None during interpreter teardown)
            L._lib.vr_scene_destroy(h)
            self._h = None


def load_xml(filename):
    return Scene.load_XML(filename)


class Ray:
    """ray.h:7-16 (direction normalised)."""

    def __init__(self, origin, direction):
        self.origin = _v3(origin)
        self.direction = _v3(direction)

    def __call__(self, t):
        return self.origin + np.float32(t) * self.direction


class Camera:
    """camera.h:7-27; the state a constructor leaves behind is a vr_camera struct."""

    def __init__(self):
        self._c = L.vr_camera()

    @classmethod
    def _from_struct(cls, c):
        obj = Pinhole_Camera.__new__(Pinhole_Camera) if c.type == L.VR_CAMERA_PINHOLE else \
            Orthographic_Camera.__new__(Orthographic_Camera)
        obj._c = c
        return obj

    @property
    def struct(self):
        return self._c

    def sample_ray(self, uv):
        o = np.zeros(3, np.float32)
        d = np.zeros(3, np.float32)
        check(lib().vr_camera_sample_ray(ctypes.byref(self._c), float(uv[0]), float(uv[1]), fptr(o), fptr(d)))
        return Ray(o, d)

    def basis(self):
        c = self._c
        return {k: np.array(list(getattr(c, k)), np.float32) for k in ("position", "view_dir", "right", "up", "pinhole")}


class Pinhole_Camera(Camera):
    """camera.h:31-54: Pinhole_Camera(position, view_dir, fov [radians])."""

    def __init__(self, position, view_dir, fov):
        super().__init__()
        p, v = _v3(position), _v3(view_dir)
        check(lib().vr_camera_pinhole(fptr(p), fptr(v), float(fov), ctypes.byref(self._c)))


class Orthographic_Camera(Camera):
    """camera.h:58-74: Orthographic_Camera(position, forward)."""

    def __init__(self, position, forward):
        super().__init__()
        p, v = _v3(position), _v3(forward)
        check(lib().vr_camera_orthographic(fptr(p), fptr(v), ctypes.byref(self._c)))


class Image:
    """image.h:9-106: float RGB framebuffer, row-major, pixel (i, j) at pixels[j, i]."""

    def __init__(self, width, height=None):
        if isinstance(width, (str, os.PathLike)):  # Image(const std::string&) — P6 reader
            w, h = ctypes.c_uint32(), ctypes.c_uint32()
            path = os.fsencode(str(width))
            check(lib().vr_image_read_ppm(path, None, ctypes.byref(w), ctypes.byref(h)))
            self.pixels = np.zeros((h.value, w.value, 3), np.float32)
            check(lib().vr_image_read_ppm(path, fptr(self.pixels), ctypes.byref(w), ctypes.byref(h)))
        else:
            self.pixels = np.zeros((int(height), int(width), 3), np.float32)

    def get_width(self):
        return self.pixels.shape[1]

    def get_height(self):
        return self.pixels.shape[0]

    def get_pixel(self, i, j):
        return self.pixels[j, i].copy()

    def set_pixel(self, i, j, rgb):
        self.pixels[j, i] = rgb

    def make_PPM(self, filename):
        check(lib().vr_image_write_ppm(os.fsencode(str(filename)), fptr(np.ascontiguousarray(self.pixels)),
                                       self.get_width(), self.get_height()))

    def to_uint8(self):
        """Same quantisation as make_PPM: clamp(v * 255, 0, 255) then truncate (image.h:66)."""
        return np.clip(self.pixels * np.float32(255.0), 0.0, 255.0).astype(np.uint8)

    def get_rgba_buffer(self):
        rgb = self.to_uint8()
        return np.concatenate([rgb, np.full(rgb.shape[:2] + (1,), 255, np.uint8)], axis=2)


class Device:
    """A device context (vr_ctx). `device` is a GPU index (vr_init) or a tuple of GPU indices: a
    multi-GPU context (vr_init_multi) that splits every frame's tiles over those GPUs and gathers
    them over RCCL (a GPU listed twice rehearses the split on one GPU, gathering with device copies).
    Scenes are uploaded lazily and re-uploaded when they change."""

    _cache = {}

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        if isinstance(device, (tuple, list)):
            devs = (ctypes.c_int32 * len(device))(*[int(d) for d in device])
            check(lib().vr_init_multi(len(device), devs, ctypes.byref(h)))
            device = tuple(int(d) for d in device)
        else:
            check(lib().vr_init(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device
        self._scene_key = None

    @staticmethod
    def count():
        n = ctypes.c_int32()
        check(lib().vr_device_count(ctypes.byref(n)))
        return int(n.value)

    @property
    def num_devices(self):
        return int(lib().vr_ctx_num_devices(self._h))

    @property
    def uses_rccl(self):
        return bool(lib().vr_ctx_uses_rccl(self._h))

    def rank_stats(self, rank):
        """vr_get_rank_stats: one rank's statistics of the last frame (same keys as stats())."""
        s = L.vr_render_stats()
        check(lib().vr_get_rank_stats(self._h, int(rank), ctypes.byref(s)))
        return self._stats_dict(s)

    @classmethod
    def get(cls, device=0):
        if isinstance(device, list):
            device = tuple(device)
        d = cls._cache.get(device)
        if d is None:
            d = cls._cache[device] = cls(device)
        return d

    def upload(self, scene, force=False):
        key = (id(scene), scene.version)
        if force or key != self._scene_key:
            check(lib().vr_upload_scene(self._h, scene._h))
            self._scene_key = key
            self._scene_ref = scene

    def stats(self):
        s = L.vr_render_stats()
        check(lib().vr_get_stats(self._h, ctypes.byref(s)))
        return self._stats_dict(s)

    def _stats_dict(self, s):
        return {"kernel_ms": s.kernel_ms, "pixels": s.pixels, "fallback_pixels": s.fallback_pixels,
                "error_pixels": s.error_pixels, "stage_ms": dict(zip(self.STAGES, list(s.stage_ms))),
                "scatter_records": s.scatter_records, "secondary_rays": s.secondary_rays,
                "record_overflow": bool(s.record_overflow), "deep_pixels": s.deep_pixels,
                "slow_rays": s.slow_rays, "band_rays": s.band_rays}

    def fallback_pixels(self):
        """(n, 2) int array of the (x, y) pixels of the last ray-march frame that were re-run on the
        large-capacity fallback path (vr_get_fallback_pixels)."""
        n = ctypes.c_size_t()
        check(lib().vr_get_fallback_pixels(self._h, None, 0, ctypes.byref(n)))
        xy = np.zeros((max(n.value, 1), 2), np.uint32)
        check(lib().vr_get_fallback_pixels(self._h, xy.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n.value,
                                           ctypes.byref(n)))
        return xy[:n.value].astype(np.int32)

    def debug_pixel_records(self, x, y):
        """vr_debug_pixel_records: the scatter records of pixel (x, y) of the last ray-march frame, (n, 9 + S)
        rows (S = lights + env_samples, the row width the context reports): step k, position xyz,
        T * sigma_s, Li + Le rgb, active-list length, then each secondary ray's Tr (lights, then
        environment samples)."""
        n, row = ctypes.c_size_t(), ctypes.c_size_t()
        check(lib().vr_debug_pixel_records(self._h, int(x), int(y), None, 0, 0, ctypes.byref(n), ctypes.byref(row)))
        out = np.zeros((max(n.value, 1), row.value), np.float32)
        check(lib().vr_debug_pixel_records(self._h, int(x), int(y), fptr(out), n.value, row.value, ctypes.byref(n), None))
        return out[:n.value]

    OPTIONS = {"half_nodes": L.VR_OPT_HALF_NODES, "secondary_budget": L.VR_OPT_SECONDARY_BUDGET,
               "ff_window0": L.VR_OPT_FF_WINDOW0, "record_capacity": L.VR_OPT_RECORD_CAPACITY,
               "device_bvh": L.VR_OPT_DEVICE_BVH, "ff_nee_queue": L.VR_OPT_FF_NEE_QUEUE,
               "march_binned": L.VR_OPT_MARCH_BINNED, "ff_solver": L.VR_OPT_FF_SOLVER,
               "start_subtree": L.VR_OPT_START_SUBTREE, "ff_kernel": L.VR_OPT_FF_KERNEL,
               "sec_tight": L.VR_OPT_SEC_TIGHT, "march_wide_min": L.VR_OPT_MARCH_WIDE_MIN}

    def set_option(self, name, value):
        """vr_set_option (include/vr_hip.h): explicit per-context tuning (half_nodes applies at the
        next upload, so the scene is re-uploaded)."""
        check(lib().vr_set_option(self._h, self.OPTIONS[name], int(value)))
        if name in ("half_nodes", "device_bvh", "sec_tight"):
            self._scene_key = None

    def get_option(self, name):
        v = ctypes.c_int64()
        check(lib().vr_get_option(self._h, self.OPTIONS[name], ctypes.byref(v)))
        return int(v.value)

    # vr_render_stats.stage_ms (include/vr_hip.h)
    STAGES = ("march", "sizing", "secondary", "accumulate")

    def synchronize(self):
        """Waits for the device; raises VRError(VR_ERR_OVERFLOW) if the last frame is invalid."""
        check(lib().vr_synchronize(self._h))

    def render_tiles_device(self, camera, params, width, height, first_tile, tile_stride, num_tiles, packed,
                            out_ptr, stream_ptr=0):
        check(lib().vr_render_tiles_device(self._h, ctypes.byref(camera.struct), ctypes.byref(params), width,
                                           height, first_tile, tile_stride, num_tiles, int(packed),
                                           ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream_ptr)))

    # Work counters of the instrumented build (include/vr_hip.h vr_count_work), per stage.
    WORK_NAMES = {
        "march": ("node_tests", "gaussian_tests", "optical_depths", "densities", "unused", "active_steps",
                  "primary_queries", "pixels"),
        # secondary stage = the persistent kernel's own schedule (+ the exact slow path)
        "secondary": ("node_tests", "gaussian_tests", "optical_depths", "list_tests", "secondary_rays",
                      "cut_rays", "cut_ray_node_steps", "repeat_depths"),
        # free-flight integrators: the path kernel and the shadow-ray (deferred NEE) kernel
        "path": ("paths", "bounces", "node4_steps", "node2_steps", "gaussian_tests", "erf_evals", "nee_inline",
                 "nee_queued"),
        "nee": ("rays", "node4_steps", "gaussian_tests", "optical_depths", "unused4", "unused5", "unused6", "unused7"),
    }

    def count_work(self, camera, params, width, height, first_tile=0, tile_stride=1, num_tiles=None):
        """Instrumented (untimed) render of the given tiles; returns the raw counts per stage."""
        if num_tiles is None:
            num_tiles = len(range(first_tile, num_tiles_of(width, height), tile_stride))
        arr = (ctypes.c_uint64 * 16)()
        check(lib().vr_count_work(self._h, ctypes.byref(camera.struct), ctypes.byref(params), width, height,
                                  first_tile, tile_stride, num_tiles, arr))
        stages = ("path", "nee") if params.integrator in (L.VR_FREE_FLIGHT, L.VR_MULTI_SCATTER) else ("march", "secondary")
        out = {stage: {k: int(arr[8 * s + i]) for i, k in enumerate(self.WORK_NAMES[stage])}
               for s, stage in enumerate(stages)}
        sec = out.get("secondary")
        if sec is not None:  # node steps of the rays that ran to the end of the tree
            sec["full_ray_node_steps"] = sec["node_tests"] - sec["cut_ray_node_steps"]
        return out

    def unshuffle_tiles_device(self, slabs_ptr, nslabs, tiles_per_slab, width, height, image_ptr, stream_ptr=0):
        check(lib().vr_unshuffle_tiles_device(self._h, ctypes.c_void_p(slabs_ptr), nslabs, tiles_per_slab, width,
                                              height, ctypes.c_void_p(image_ptr), ctypes.c_void_p(stream_ptr)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and L is not None and L._lib is not None:  # (L is None during interpreter teardown)
            L._lib.vr_destroy(h)
            self._h = None


def num_tiles(width, height):
    return int(lib().vr_num_tiles(width, height))


num_tiles_of = num_tiles


class Integrator:
    """integrator.h:49-57: Integrator(camera); render(scene, image) fills `image` in place."""

    integrator_id = None

    def __init__(self, camera, step_size=0.01, env_samples=20, t_eps=0.0, device=0):
        self.camera = camera
        self.params = L.vr_render_params()
        self.params.integrator = self.integrator_id
        self.params.step_size = float(step_size)
        self.params.env_samples = int(env_samples)
        self.params.t_eps = float(t_eps)
        self.params.flags = 0
        self.device = device
        self.last_stats = None

    solver = None  # free-flight integrators: a SOLVERS key (VR_OPT_FF_SOLVER), set on the device per render

    def _device(self, scene):
        dev = Device.get(self.device)
        dev.upload(scene)
        if self.solver is not None:
            dev.set_option("ff_solver", SOLVERS[self.solver])
        return dev

    def render(self, scene, image):
        dev = self._device(scene)
        W, H = image.get_width(), image.get_height()
        out = np.empty((H, W, 3), np.float32)
        check(lib().vr_render(dev._h, ctypes.byref(self.camera.struct), ctypes.byref(self.params), W, H, fptr(out)))
        image.pixels[...] = out
        self.last_stats = dev.stats()
        return image


class RayMarchingGaussians(Integrator):
    """test_integrators.h:143-297: RayMarchingGaussians(camera, step_size=0.01, env_samples=20)."""

    integrator_id = L.VR_RAYMARCH_GAUSSIANS

    def __init__(self, camera, step_size=0.01, env_samples=20, t_eps=0.0, device=0):
        super().__init__(camera, step_size, env_samples, t_eps, device)


class PureRayMarching(Integrator):
    """integrator.h:100-267: PureRayMarching(camera, step_size=0.01, env_samples=20) — primary and
    shadow/environment transmittance marched at step_size (T *= exp(-sigma_t dt))."""

    integrator_id = L.VR_PURE_RAYMARCH

    def __init__(self, camera, step_size=0.01, env_samples=20, t_eps=0.0, device=0):
        super().__init__(camera, step_size, env_samples, t_eps, device)


# distance_solvers.h:143-147 (compile-time #defines in the reference) -> VR_OPT_FF_SOLVER values
SOLVERS = {"analytic_newton": 0, "bisection": 1, "newton": 2, "analytic_bisection": 3, "uniform": 4}


class FreeFlightGaussians(Integrator):
    """integrator.h:273-408: FreeFlightGaussians(camera, num_samples=256) — single scattering by
    free-flight sampling, one NEE sample (a light or the environment) per path. `solver`: the
    distance solver (SOLVERS; the reference's compiled-in ANALYTIC_PLUS_NEWTON by default)."""

    integrator_id = L.VR_FREE_FLIGHT

    def __init__(self, camera, num_samples=256, device=0, solver="analytic_newton"):
        super().__init__(camera, 0.01, 0, 0.0, device)
        self.params.num_samples = int(num_samples)
        self.solver = solver

    def set_num_samples(self, n):
        self.params.num_samples = int(n)


class MultiScatterGaussians(Integrator):
    """integrator.h:416-720: MultiScatterGaussians(camera, samples=16, min_bounces=5) — free-flight
    paths with NEE at every scattering event and Russian roulette after min_bounces."""

    integrator_id = L.VR_MULTI_SCATTER

    def __init__(self, camera, samples=16, min_bounces=5, device=0, solver="analytic_newton"):
        super().__init__(camera, 0.01, 0, 0.0, device)
        self.params.num_samples = int(samples)
        self.params.min_bounces = int(min_bounces)
        self.solver = solver

    def set_num_samples(self, n):  # integrator.h:719
        self.params.num_samples = int(n)

    def render(self, scene, image, per_pixel_gaussians=None, slot=0):
        """render(scene, image[, per_pixel_gaussians]) (integrator.h:525-536). With RECORD_PIXEL_GAUSSIANS
        semantics when `per_pixel_gaussians` is a list: it is filled with one sorted list of Gaussian
        indices per row-major pixel (integrator.h:616-644, 700-705). The device keeps the recording
        in `slot` (0/1) for vr_sfd_loss_diff; record() skips the host decode."""
        if per_pixel_gaussians is None:
            return super().render(scene, image)
        self.record(scene, image, slot)
        bits = self.pixel_gaussian_bits(slot)
        per_pixel_gaussians[:] = bits_to_lists(bits, scene.get_num_primitives())
        return image

    def record(self, scene, image, slot=0):
        dev = self._device(scene)
        W, H = image.get_width(), image.get_height()
        out = np.empty((H, W, 3), np.float32)
        check(lib().vr_render_record(dev._h, ctypes.byref(self.camera.struct), ctypes.byref(self.params), W, H,
                                     fptr(out), int(slot)))
        image.pixels[...] = out
        self._rec_shape = (scene.get_num_primitives(), W * H)
        self.last_stats = dev.stats()
        return image

    def pixel_gaussian_bits(self, slot=0):
        """(ceil(N/32), W*H) uint32: bit b of word w at pixel p <=> Gaussian 32w+b recorded at p."""
        n, npix = self._rec_shape
        bits = np.zeros(((n + 31) // 32, npix), np.uint32)
        check(lib().vr_get_pixel_gaussians(Device.get(self.device)._h, int(slot),
                                          bits.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), bits.size))
        return bits


def bits_to_lists(bits, n):
    """Decode a (words, npix) recording bitset into per-pixel sorted Gaussian index lists."""
    words, npix = bits.shape
    unpacked = np.unpackbits(bits.T.copy().view(np.uint8), axis=1, bitorder="little")[:, :n]
    return [np.nonzero(row)[0].astype(np.uint32).tolist() for row in unpacked]


class RayMarchingSpheres(Integrator):
    """test_integrators.h:11-136: RayMarchingSpheres(camera, step_size=0.01, env_samples=5)."""

    integrator_id = L.VR_RAYMARCH_SPHERES

    def __init__(self, camera, step_size=0.01, env_samples=5, t_eps=0.0, device=0):
        super().__init__(camera, step_size, env_samples, t_eps, device)


class TestIntegrator(Integrator):
    """integrator.h:65-94: magenta where the primary ray hits anything, env colour elsewhere."""

    __test__ = False  # not a pytest class
    integrator_id = L.VR_TEST_HITMASK

    def __init__(self, camera, device=0):
        super().__init__(camera, 0.01, 0, 0.0, device)
