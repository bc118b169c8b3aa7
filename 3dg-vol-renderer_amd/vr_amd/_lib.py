"""ctypes binding of libvr_hip.so (the C ABI declared in include/vr_hip.h).

Loading fails loudly when the native library is missing: there is no CPU fallback anywhere in
this package.
"""
import ctypes
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("VR_LIB_PATH") or os.path.join(_PKG_ROOT, "libvr_hip.so")  # override: A/B builds

VR_OK = 0
VR_ERR_OVERFLOW, VR_ERR_RETRY = 6, 8
STATUS_NAMES = {
    0: "VR_OK", 1: "VR_ERR_INVALID", 2: "VR_ERR_IO", 3: "VR_ERR_PARSE", 4: "VR_ERR_HIP",
    5: "VR_ERR_NOSCENE", 6: "VR_ERR_OVERFLOW", 7: "VR_ERR_UNSUPPORTED", 8: "VR_ERR_RETRY",
}
VR_VOLUME_GAUSSIANS, VR_VOLUME_SPHERES = 0, 1
VR_CAMERA_PINHOLE, VR_CAMERA_ORTHOGRAPHIC = 0, 1
VR_RAYMARCH_GAUSSIANS, VR_RAYMARCH_SPHERES, VR_TEST_HITMASK, VR_PURE_RAYMARCH = 0, 1, 2, 3
VR_FREE_FLIGHT, VR_MULTI_SCATTER = 4, 5
VR_OPT_HALF_NODES, VR_OPT_SECONDARY_BUDGET, VR_OPT_FF_WINDOW0, VR_OPT_RECORD_CAPACITY, VR_OPT_DEVICE_BVH = 1, 2, 3, 4, 5
VR_OPT_FF_NEE_QUEUE = 6
VR_OPT_MARCH_BINNED = 7
VR_OPT_FF_SOLVER = 8
VR_OPT_START_SUBTREE = 9
VR_OPT_SEC_TIGHT = 11
VR_OPT_MARCH_WIDE_MIN = 12
VR_OPT_FF_KERNEL = 13

f3 = ctypes.c_float * 3


class vr_light(ctypes.Structure):
    _fields_ = [("position", f3), ("intensity", f3)]


class vr_gaussian(ctypes.Structure):
    _fields_ = [("mean", f3), ("cov", ctypes.c_float * 6), ("density", ctypes.c_float),
                ("albedo", ctypes.c_float), ("emission", f3)]


class vr_sphere(ctypes.Structure):
    _fields_ = [("center", f3), ("radius", ctypes.c_float), ("sigma_a", ctypes.c_float),
                ("sigma_s", ctypes.c_float)]


class vr_camera(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("position", f3), ("view_dir", f3), ("right", f3), ("up", f3),
                ("pinhole", f3), ("fov", ctypes.c_float), ("focal_length", ctypes.c_float)]


class vr_render_params(ctypes.Structure):
    _fields_ = [("integrator", ctypes.c_int32), ("step_size", ctypes.c_float), ("env_samples", ctypes.c_int32),
                ("t_eps", ctypes.c_float), ("flags", ctypes.c_uint32), ("num_samples", ctypes.c_int32),
                ("min_bounces", ctypes.c_int32)]


class vr_scene_info(ctypes.Structure):
    _fields_ = [("volume_type", ctypes.c_int32), ("num_primitives", ctypes.c_int64),
                ("num_lights", ctypes.c_int64), ("env_color", f3), ("bounds_min", f3), ("bounds_max", f3)]


class vr_render_stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("pixels", ctypes.c_int64), ("fallback_pixels", ctypes.c_int64),
                ("error_pixels", ctypes.c_int64), ("stage_ms", ctypes.c_double * 4),
                ("scatter_records", ctypes.c_int64), ("secondary_rays", ctypes.c_int64),
                ("record_overflow", ctypes.c_int64), ("deep_pixels", ctypes.c_int64), ("slow_rays", ctypes.c_int64),
                ("band_rays", ctypes.c_int64)]


class vr_sfd_config(ctypes.Structure):
    _fields_ = [("max_iters", ctypes.c_int32), ("save_every", ctypes.c_int32), ("num_stoch_samples", ctypes.c_int32),
                ("lr", ctypes.c_float), ("seed", ctypes.c_uint64), ("final_samples", ctypes.c_int32),
                ("out_dir", ctypes.c_char_p)]


class vr_sfd_result(ctypes.Structure):
    _fields_ = [("params", ctypes.POINTER(ctypes.c_float)), ("loss_history", ctypes.POINTER(ctypes.c_double)),
                ("last_grads", ctypes.POINTER(ctypes.c_double)), ("final_image", ctypes.POINTER(ctypes.c_float)),
                ("final_loss", ctypes.c_double)]


# name -> (restype, argtypes). Every symbol declared in include/vr_hip.h.
P = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)
FP = ctypes.POINTER(ctypes.c_float)
U32P = ctypes.POINTER(ctypes.c_uint32)
ST = ctypes.c_int
SIGNATURES = {
    "vr_version": (ctypes.c_char_p, []),
    "vr_last_error": (ctypes.c_char_p, []),
    "vr_scene_create": (ST, [ctypes.c_int32, PP]),
    "vr_scene_load_gmm": (ST, [ctypes.c_char_p, PP]),
    "vr_scene_load_smm": (ST, [ctypes.c_char_p, PP]),
    "vr_scene_load_xml": (ST, [ctypes.c_char_p, PP, ctypes.POINTER(vr_camera), U32P, U32P,
                               ctypes.POINTER(vr_render_params)]),
    "vr_scene_add_gaussians": (ST, [P, ctypes.POINTER(vr_gaussian), ctypes.c_size_t]),
    "vr_scene_add_random_gaussians": (ST, [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32]),
    "vr_scene_add_spheres": (ST, [P, ctypes.POINTER(vr_sphere), ctypes.c_size_t]),
    "vr_scene_add_lights": (ST, [P, ctypes.POINTER(vr_light), ctypes.c_size_t]),
    "vr_scene_set_env_color": (ST, [P, FP]),
    "vr_scene_get_info": (ST, [P, ctypes.POINTER(vr_scene_info)]),
    "vr_scene_get_records": (ST, [P, FP, ctypes.c_size_t]),
    "vr_scene_get_lights": (ST, [P, ctypes.POINTER(vr_light), ctypes.c_size_t]),
    "vr_scene_get_gaussians": (ST, [P, ctypes.POINTER(vr_gaussian), ctypes.c_size_t]),
    "vr_scene_get_spheres": (ST, [P, ctypes.POINTER(vr_sphere), ctypes.c_size_t]),
    "vr_scene_destroy": (None, [P]),
    "vr_camera_pinhole": (ST, [FP, FP, ctypes.c_float, ctypes.POINTER(vr_camera)]),
    "vr_camera_orthographic": (ST, [FP, FP, ctypes.POINTER(vr_camera)]),
    "vr_camera_sample_ray": (ST, [ctypes.POINTER(vr_camera), ctypes.c_double, ctypes.c_double, FP, FP]),
    "vr_image_write_ppm": (ST, [ctypes.c_char_p, FP, ctypes.c_uint32, ctypes.c_uint32]),
    "vr_image_read_ppm": (ST, [ctypes.c_char_p, FP, U32P, U32P]),
    "vr_init": (ST, [ctypes.c_int, PP]),
    "vr_gif_begin": (ST, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, PP]),
    "vr_gif_write_frame": (ST, [P, ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint32]),
    "vr_gif_end": (ST, [P]),
    "vr_gmm_pack_parameters": (ST, [P, FP, ctypes.c_size_t]),
    "vr_gmm_apply_parameters": (ST, [P, FP, ctypes.c_size_t, PP]),
    "vr_gmm_default_eps": (ST, [FP, ctypes.c_size_t]),
    "vr_adam_step": (ST, [FP, FP, FP, FP, ctypes.c_size_t, ctypes.c_int32, ctypes.c_float, ctypes.c_float,
                          ctypes.c_float, ctypes.c_float]),
    "vr_sfd_sign_vector": (ST, [ctypes.c_uint64, ctypes.c_uint64, FP, ctypes.c_size_t]),
    "vr_sfd_optimize": (ST, [P, ctypes.POINTER(vr_camera), ctypes.POINTER(vr_render_params), P, FP, ctypes.c_uint32,
                             ctypes.c_uint32, ctypes.POINTER(vr_sfd_config), ctypes.POINTER(vr_sfd_result)]),
    "vr_device_count": (ST, [ctypes.POINTER(ctypes.c_int32)]),
    "vr_init_multi": (ST, [ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), PP]),
    "vr_ctx_num_devices": (ctypes.c_int32, [P]),
    "vr_ctx_uses_rccl": (ctypes.c_int32, [P]),
    "vr_get_rank_stats": (ST, [P, ctypes.c_int32, ctypes.POINTER(vr_render_stats)]),
    "vr_destroy": (None, [P]),
    "vr_upload_scene": (ST, [P, P]),
    "vr_render": (ST, [P, ctypes.POINTER(vr_camera), ctypes.POINTER(vr_render_params), ctypes.c_uint32,
                       ctypes.c_uint32, FP]),
    "vr_render_tiles_device": (ST, [P, ctypes.POINTER(vr_camera), ctypes.POINTER(vr_render_params),
                                    ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.c_int32, P, P]),
    "vr_unshuffle_tiles_device": (ST, [P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       P, P]),
    "vr_unshuffle_tiles_part_device": (ST, [P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, P, P]),
    "vr_count_work": (ST, [P, ctypes.POINTER(vr_camera), ctypes.POINTER(vr_render_params), ctypes.c_uint32,
                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.POINTER(ctypes.c_uint64)]),
    "vr_render_record": (ST, [P, ctypes.POINTER(vr_camera), ctypes.POINTER(vr_render_params), ctypes.c_uint32,
                              ctypes.c_uint32, ctypes.POINTER(ctypes.c_float), ctypes.c_int32]),
    "vr_get_pixel_gaussians": (ST, [P, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t]),
    "vr_sfd_loss_diff": (ST, [P, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float), ctypes.c_uint32,
                              ctypes.c_uint32, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t]),
    "vr_num_tiles": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32]),
    "vr_set_option": (ST, [P, ctypes.c_int32, ctypes.c_int64]),
    "vr_get_option": (ST, [P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]),
    "vr_synchronize": (ST, [P]),
    "vr_get_stats": (ST, [P, ctypes.POINTER(vr_render_stats)]),
    "vr_get_fallback_pixels": (ST, [P, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "vr_debug_pixel_records": (ST, [P, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_float), ctypes.c_size_t,
                                    ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]),
}

_lib = None


class VRError(RuntimeError):
    """Raised for a non-zero vr_status (the reference raises std::runtime_error)."""

    def __init__(self, status, msg):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


def _single_hip_runtime():
    """Exactly one HIP runtime may live in a process. torch ships its own libamdhip64.so.7 (same
    SONAME as /opt/rocm's); if libvr_hip.so were loaded first, torch would bind to the system
    runtime and fail to see the GPU. So when torch is importable, load it first: libvr_hip.so then
    resolves libamdhip64.so.7 to torch's copy and both share one runtime, one device context and
    one stream namespace (bench.py hands torch streams/tensors straight to the kernels)."""
    if os.environ.get("VR_NO_TORCH_RUNTIME") == "1":
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                              "(there is no CPU fallback)")
        _single_hip_runtime()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status):
    if status != VR_OK:
        raise VRError(status, lib().vr_last_error().decode(errors="replace"))


def fptr(a):
    return a.ctypes.data_as(FP)
