"""TEST INFRASTRUCTURE ONLY — ctypes wrapper around oracle/build/liboracle_vr.so.

The oracle is the CPU restatement of the reference ray-march path (see vr_oracle.cpp header).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product (vr_amd / libvr_hip.so) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle_vr.so")
_lib = None

RAYMARCH_GAUSSIANS = 0
RAYMARCH_SPHERES = 1
RAYMARCH_GAUSSIANS_LISTS = 2  # same algorithm, sparse active sets + stop at T == 0 (bit-identical)
PURE_RAYMARCH = 3  # PureRayMarching (integrator.h:100-267): marched primary and shadow transmittance
PINHOLE = 0
ORTHO = 1


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_SO):
        build()
    L = ctypes.CDLL(_SO)
    P = ctypes.c_void_p
    fp = ctypes.POINTER(ctypes.c_float)
    ip = ctypes.POINTER(ctypes.c_int)
    L.orc_last_error.restype = ctypes.c_char_p
    L.orc_load_gmm.restype = P
    L.orc_load_gmm.argtypes = [ctypes.c_char_p]
    L.orc_load_smm.restype = P
    L.orc_load_smm.argtypes = [ctypes.c_char_p]
    L.orc_scene_from_gaussians.restype = P
    L.orc_scene_from_gaussians.argtypes = [ctypes.c_int64, fp, fp, fp, fp, ctypes.c_int64, fp, fp]
    L.orc_scene_free.argtypes = [P]
    L.orc_scene_set_env.argtypes = [P, ctypes.c_float, ctypes.c_float, ctypes.c_float]
    L.orc_scene_num.restype = ctypes.c_int64
    L.orc_scene_num.argtypes = [P]
    L.orc_scene_num_lights.restype = ctypes.c_int64
    L.orc_scene_num_lights.argtypes = [P]
    L.orc_scene_type.argtypes = [P]
    L.orc_scene_records.argtypes = [P, fp]
    L.orc_camera.argtypes = [ctypes.c_int, fp, fp, ctypes.c_float, fp]
    L.orc_primary_ray.argtypes = [ctypes.c_int, fp, fp, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, fp]
    L.orc_gaussian_probe.argtypes = [P, ctypes.c_int64, fp, fp, fp]
    L.orc_derive_path_seed.restype = ctypes.c_uint64
    L.orc_derive_path_seed.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.orc_pcg32.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
    L.orc_env_dir.argtypes = [ctypes.c_float, ctypes.c_float, fp]
    L.orc_render.restype = ctypes.c_int
    L.orc_render_ff.argtypes = [P, ctypes.c_int, fp, fp, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int64, fp,
                                ctypes.c_int]
    L.orc_render_ms_record.argtypes = [P, ctypes.c_int, fp, fp, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, fp, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
    L.orc_render.argtypes = [P, ctypes.c_int, fp, fp, ctypes.c_float, ctypes.c_int, ctypes.c_float,
                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ip, ctypes.c_int64, fp, ctypes.c_int]
    L.orc_primary_depths.argtypes = [P, ctypes.c_int, fp, fp, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_float, ctypes.c_float, fp, ctypes.c_int]
    L.orc_tile_bins.restype = ctypes.c_int64
    L.orc_tile_bins.argtypes = [P, fp, fp, ctypes.c_float, ctypes.c_int, ctypes.c_int, fp,
                                ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
    L.orc_set_stable_ties.argtypes = [ctypes.c_int]
    L.orc_set_stable_ties.restype = ctypes.c_int
    _lib = L
    return L


def debug_pixel_records(scene, pos, view_dir, fov, x, y, W, H, step_size=0.01, env_samples=20):
    """orc_debug_pixel_records (pinhole, RAYMARCH_GAUSSIANS_LISTS): the scattering steps of pixel (x, y), one
    row of 9 + lights + env_samples floats each (the layout of vr_debug_pixel_records). Test tooling only."""
    pos, pp = _f(pos)
    vd, pv = _f(view_dir)
    L = lib()
    L.orc_debug_pixel_records.restype = ctypes.c_int64
    L.orc_debug_pixel_records.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                          ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_float, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.c_int64]
    row = 9 + scene.num_lights + int(env_samples)
    out = np.zeros((4096, row), np.float32)
    n = L.orc_debug_pixel_records(scene.h, pp, pv, float(fov), int(x), int(y), int(W), int(H), float(step_size),
                                  int(env_samples), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), out.shape[0])
    return out[:min(n, out.shape[0])]


def primary_depths(scene, cam_type, pos, view_dir, fov, W, H, step_size=0.01, t_eps=1e-6, nthreads=0):
    """(H, W) termination distance of every primary ray (-1: no events); see orc_primary_depths."""
    pos, pp = _f(pos)
    vd, pv = _f(view_dir)
    out = np.zeros((H, W), np.float32)
    lib().orc_primary_depths(scene.h, cam_type, pp, pv, float(fov), W, H, float(step_size), float(t_eps),
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), int(nthreads))
    return out


def tile_bins(scene, pos, view_dir, fov, W, H, depth, nthreads=0):
    """Per 16x16 tile (row-major) the Gaussians overlapping its frustum up to its termination depth
    (SURVEY §8(d) n_t); see orc_tile_bins. Pinhole camera."""
    pos, pp = _f(pos)
    vd, pv = _f(view_dir)
    d, pd = _f(depth)
    nt = np.zeros(((W + 15) // 16) * ((H + 15) // 16), np.uint32)
    lib().orc_tile_bins(scene.h, pp, pv, float(fov), W, H, pd, nt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                        int(nthreads))
    return nt


class stable_ties:
    """Context manager: the oracle resolves event-sort ties (a ray grazing a 3-sigma ellipsoid with
    t0 == t1 in float) in emission order instead of the reference's unstable std::sort (see
    g_stable_ties in vr_oracle.cpp)."""

    def __enter__(self):
        self._old = lib().orc_set_stable_ties(1)
        return self

    def __exit__(self, *exc):
        lib().orc_set_stable_ties(self._old)
        return False


class accurate_chords:
    """Context manager: the sparse-list restatement computes secondary-ray chords (intersect and optical
    depth) in double instead of the reference's f32 forms (see g_accurate_chords in vr_oracle.cpp)."""

    def __enter__(self):
        L = lib()
        L.orc_set_accurate_chords.argtypes = [ctypes.c_int]
        L.orc_set_accurate_chords.restype = ctypes.c_int
        self._old = L.orc_set_accurate_chords(1)
        return self

    def __exit__(self, *exc):
        lib().orc_set_accurate_chords(self._old)
        return False


class padded_boxes:
    """Context manager: scenes built inside it get their BVH on the padded tight 3-sigma boxes instead of the
    reference's eigen-derived get_aabb boxes (gaussian.h:304-319; see g_padded_boxes in vr_oracle.cpp).
    Read when a scene is built, not when it renders."""

    def __enter__(self):
        L = lib()
        L.orc_set_padded_boxes.argtypes = [ctypes.c_int]
        L.orc_set_padded_boxes.restype = ctypes.c_int
        self._old = L.orc_set_padded_boxes(1)
        return self

    def __exit__(self, *exc):
        lib().orc_set_padded_boxes(self._old)
        return False


def _f(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class OracleScene:
    """Oracle-side scene (restatement of Scene::load_GMM / load_SMM, scene.h:38-120)."""

    def __init__(self, handle):
        if not handle:
            raise RuntimeError(lib().orc_last_error().decode())
        self.h = handle

    @classmethod
    def load_gmm(cls, path):
        return cls(lib().orc_load_gmm(os.fsencode(path)))

    @classmethod
    def load_smm(cls, path):
        return cls(lib().orc_load_smm(os.fsencode(path)))

    @classmethod
    def from_gaussians(cls, mean, cov6, density, albedo, light_pos, light_int):
        mean, pm = _f(mean)
        cov6, pc = _f(cov6)
        density, pd = _f(density)
        albedo, pa = _f(albedo)
        light_pos, plp = _f(np.asarray(light_pos).reshape(-1, 3))
        light_int, pli = _f(np.asarray(light_int).reshape(-1, 3))
        n = density.shape[0]
        return cls(lib().orc_scene_from_gaussians(n, pm, pc, pd, pa, light_pos.shape[0], plp, pli))

    def set_env(self, rgb):
        lib().orc_scene_set_env(self.h, float(rgb[0]), float(rgb[1]), float(rgb[2]))

    @property
    def num(self):
        return int(lib().orc_scene_num(self.h))

    @property
    def num_lights(self):
        return int(lib().orc_scene_num_lights(self.h))

    def records(self):
        out = np.zeros((self.num, 12), np.float32)
        lib().orc_scene_records(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        return out

    def probe(self, i, origin, direction):
        o, po = _f(origin)
        d, pd = _f(direction)
        out = np.zeros(4, np.float32)
        lib().orc_gaussian_probe(self.h, int(i), po, pd, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        return out

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().orc_scene_free(self.h)
                self.h = None
        except Exception:
            pass


def camera(cam_type, pos, view_dir, fov=0.0):
    pos, pp = _f(pos)
    vd, pv = _f(view_dir)
    out = np.zeros(17, np.float32)
    lib().orc_camera(cam_type, pp, pv, float(fov), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return out


def primary_ray(cam_type, pos, view_dir, fov, x, y, W, H):
    pos, pp = _f(pos)
    vd, pv = _f(view_dir)
    out = np.zeros(6, np.float32)
    lib().orc_primary_ray(cam_type, pp, pv, float(fov), x, y, W, H, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return out


def render(scene, cam_type, pos, view_dir, fov, W, H, integrator=RAYMARCH_GAUSSIANS, step_size=0.01,
           env_samples=20, pixels=None, nthreads=0, ties=None):
    """Render the full W x H frame (returns H x W x 3) or only `pixels` ((n,2) int x,y; returns n x 3).
    ties: an int32 array of one entry per rendered pixel that receives the pixel's count of tangent-hit ties
    (rays on which a Gaussian's entry and exit keys are equal, so std::sort decides their order)."""
    pos, pp = _f(pos)
    vd, pv = _f(view_dir)
    if pixels is not None:
        pix = np.ascontiguousarray(np.asarray(pixels, dtype=np.int32).reshape(-1, 2))
        out = np.zeros((pix.shape[0], 3), np.float32)
        pix_p = pix.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
        npix = pix.shape[0]
    else:
        out = np.zeros((H, W, 3), np.float32)
        pix_p = None
        npix = 0
    L = lib()
    if ties is not None:
        assert ties.dtype == np.int32 and ties.flags.c_contiguous and ties.size == (npix if pixels is not None else W * H)
        L.orc_tie_flags.argtypes = [ctypes.POINTER(ctypes.c_int32)]
        L.orc_tie_flags(ties.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    try:
        rc = L.orc_render(scene.h, cam_type, pp, pv, float(fov), integrator, float(step_size), int(env_samples),
                          int(W), int(H), pix_p, npix, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                          int(nthreads))
    finally:
        if ties is not None:
            L.orc_tie_flags(None)
    if rc != 0:
        raise RuntimeError("oracle render failed: " + lib().orc_last_error().decode())
    return out


def render_ff(scene, cam_type, pos, view_dir, fov, W, H, multi=True, num_samples=16, min_bounces=5, pixels=None,
              nthreads=0):
    """FreeFlightGaussians (multi=False) / MultiScatterGaussians (multi=True); output as render()."""
    pos, pp = _f(pos)
    vd, pv = _f(view_dir)
    if pixels is not None:
        pix = np.ascontiguousarray(np.asarray(pixels, dtype=np.int32).reshape(-1, 2))
        out = np.zeros((pix.shape[0], 3), np.float32)
        pix_p = pix.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
        npix = pix.shape[0]
    else:
        out = np.zeros((H, W, 3), np.float32)
        pix_p = None
        npix = 0
    rc = lib().orc_render_ff(scene.h, cam_type, pp, pv, float(fov), int(bool(multi)), int(num_samples),
                             int(min_bounces), int(W), int(H), pix_p, npix,
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), int(nthreads))
    if rc != 0:
        raise RuntimeError("oracle render failed: " + lib().orc_last_error().decode())
    return out


def render_ms_record(scene, cam_type, pos, view_dir, fov, W, H, num_samples=16, min_bounces=5, nthreads=0,
                     pixels=None):
    """MultiScatterGaussians with RECORD_PIXEL_GAUSSIANS: (image H x W x 3, bits (ceil(N/32), W*H)); with
    `pixels` ((n, 2) x, y) only those: (n x 3, bits (ceil(N/32), n))."""
    pos, pp = _f(pos)
    vd, pv = _f(view_dir)
    if pixels is not None:
        pix = np.ascontiguousarray(np.asarray(pixels, dtype=np.int32).reshape(-1, 2))
        out = np.zeros((pix.shape[0], 3), np.float32)
        bits = np.zeros(((scene.num + 31) // 32, pix.shape[0]), np.uint32)
        L = lib()
        L.orc_render_ms_record_px.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                              ctypes.POINTER(ctypes.c_float), ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int64,
                                              ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
        rc = L.orc_render_ms_record_px(scene.h, cam_type, pp, pv, float(fov), int(num_samples), int(min_bounces), int(W),
                                       int(H), pix.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), pix.shape[0],
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                       bits.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), int(nthreads))
        if rc != 0:
            raise RuntimeError("oracle render failed: " + lib().orc_last_error().decode())
        return out, bits
    out = np.zeros((H, W, 3), np.float32)
    bits = np.zeros(((scene.num + 31) // 32, W * H), np.uint32)
    rc = lib().orc_render_ms_record(scene.h, cam_type, pp, pv, float(fov), int(num_samples), int(min_bounces), int(W),
                                    int(H), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                    bits.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), int(nthreads))
    if rc != 0:
        raise RuntimeError("oracle render failed: " + lib().orc_last_error().decode())
    return out, bits


def derive_path_seed(x, y, si):
    return int(lib().orc_derive_path_seed(x, y, si))


def pcg32(seed, seq, n):
    out = np.zeros(n, np.uint32)
    lib().orc_pcg32(seed, seq, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    return out


def env_dir(xi1, xi2):
    out = np.zeros(3, np.float32)
    lib().orc_env_dir(float(xi1), float(xi2), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return out
