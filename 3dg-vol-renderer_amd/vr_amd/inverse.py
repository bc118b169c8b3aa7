"""Inverse rendering by stochastic finite differences: Python mirror of
StochasticFiniteDiffInverseIntegrator (include/inverse_integrator.h:50-246), AdamOptimizer
(include/optimizer.h:13-55) and the GMM <-> feature-vector maps (include/gmm.h:583-706).

Everything runs natively in libvr_hip.so (host/vr_inverse.cpp): the parameter maps, Adam, and the
loop itself (vr_sfd_optimize), whose forward renders (1 + num_stoch_samples MultiScatterGaussians
renders with per-pixel Gaussian recording per iteration), per-pixel L1 losses and per-Gaussian
union-of-pixels loss statistic run on the device, with the BVH of every re-uploaded scene built on
the device. The C++ mirror (include/vr/inverse_integrator.h) calls the same entry points.

Deviations: the sign vectors come from a seeded PCG32 stream (vr_sfd_sign_vector)
instead of mt19937(random_device) (:101-103, not reproducible in the reference); the eigenbasis of
pack_parameters comes from a Jacobi solver (Eigen's SelfAdjointEigenSolver signs are unpinned) and is
made right-handed before the AngleAxis conversion: the reference converts a possibly left-handed
eigenvector matrix (det -1) to AngleAxis, which is not a rotation and changes the covariance on the
first apply_params_to_gmm_local; here pack -> apply reproduces the covariance.
"""
import ctypes
import os

import numpy as np

from . import MultiScatterGaussians, Scene, Device, Image, check, lib  # noqa: F401
from . import _lib as L

PER = 11  # parameters per Gaussian (inverse_integrator.h:108)
_fp = ctypes.POINTER(ctypes.c_float)
_dp = ctypes.POINTER(ctypes.c_double)


# ---- gmm.h:18-32 ----
def sigmoidf_safe(x):
    x = np.asarray(x, np.float32)
    z = np.exp(-np.abs(x)).astype(np.float32)
    return np.where(x >= 0, np.float32(1) / (np.float32(1) + z), z / (np.float32(1) + z)).astype(np.float32)


def inv_sigmoidf(y):
    yy = np.clip(np.asarray(y, np.float32), np.float32(1e-7), np.float32(1 - 1e-7))
    return np.log(yy / (np.float32(1) - yy)).astype(np.float32)


def _as_scene(gaussians_or_scene):
    if isinstance(gaussians_or_scene, Scene):
        return gaussians_or_scene
    g = np.asarray(gaussians_or_scene, np.float32)
    return Scene.from_gaussians(g[:, 0:3], g[:, 3:9], g[:, 9], g[:, 10])


def pack_parameters(gaussians):
    """GaussianMixtureModel::pack_parameters (gmm.h:583-628), native (vr_gmm_pack_parameters): per
    Gaussian mean(3), Rodrigues rotation(3), log scale(3), log density, logit albedo. `gaussians`: a
    Scene or an (N, >=11) array as returned by Scene.gaussians() (mean, cov6, density, albedo)."""
    s = _as_scene(gaussians)
    out = np.zeros(s.get_num_primitives() * PER, np.float32)
    check(lib().vr_gmm_pack_parameters(s._h, out.ctypes.data_as(_fp), out.size))
    return out


def apply_params(params, lights, env_color, base=None):
    """apply_params_to_gmm_local (gmm.h:634-674), native (vr_gmm_apply_parameters): a new Scene with
    every Gaussian rebuilt from params (covariance R S S^T R^T); lights and environment as given."""
    p = np.ascontiguousarray(params, np.float32).reshape(-1)
    n = p.size // PER
    if base is None:
        base = Scene.from_gaussians(np.zeros((n, 3)), np.tile([1, 0, 0, 1, 0, 1], (n, 1)), np.ones(n), np.ones(n),
                                    lights=lights, env_color=env_color)
    h = ctypes.c_void_p()
    check(lib().vr_gmm_apply_parameters(base._h, p.ctypes.data_as(_fp), p.size, ctypes.byref(h)))
    return Scene(_handle=h)


def make_default_eps_for_params(params):
    """gmm.h:678-706 (vr_gmm_default_eps)"""
    eps = np.zeros(np.asarray(params).size, np.float32)
    check(lib().vr_gmm_default_eps(eps.ctypes.data_as(_fp), eps.size))
    return eps


def sign_vector(seed, k, n):
    """Sign vector k of a vr_sfd_optimize run (+1 / -1 per parameter; vr_sfd_sign_vector)."""
    s = np.zeros(n, np.float32)
    check(lib().vr_sfd_sign_vector(int(seed), int(k), s.ctypes.data_as(_fp), n))
    return s


class AdamOptimizer:
    """optimizer.h:13-55 (float32 state; the step is the native vr_adam_step)."""

    def __init__(self, ndim, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8):
        self.lr, self.beta1, self.beta2, self.eps = float(lr), float(beta1), float(beta2), float(eps)
        self.m = np.zeros(ndim, np.float32)
        self.v = np.zeros(ndim, np.float32)
        self.t = 0

    def step(self, params, grads):
        if params.shape != grads.shape or params.shape != self.m.shape:
            return False
        self.t += 1
        g = np.ascontiguousarray(grads, np.float32)
        check(lib().vr_adam_step(params.ctypes.data_as(_fp), g.ctypes.data_as(_fp), self.m.ctypes.data_as(_fp),
                                 self.v.ctypes.data_as(_fp), params.size, self.t, self.lr, self.beta1, self.beta2,
                                 self.eps))
        return True

    def reset_state(self):
        self.m[:] = 0
        self.v[:] = 0
        self.t = 0


def compute_pixel_losses(I, I_ref):
    """inverse_integrator.h:21-30: per-pixel L1 over RGB, row-major (|d0| + (|d1| + |d2|), Eigen's order)."""
    d = np.abs(I.pixels - I_ref.pixels)
    return (d[..., 0] + (d[..., 1] + d[..., 2])).reshape(-1).astype(np.float32)


class SFDConfig:
    """inverse_integrator.h:52-57 (SFDDConfig) + seed, output directory and final render samples."""

    def __init__(self, max_iters=1000, save_every=25, num_stoch_samples=4, lr=1e-2, seed=0, out_dir=None,
                 final_samples=16384):
        self.max_iters, self.save_every, self.num_stoch_samples, self.lr = max_iters, save_every, num_stoch_samples, lr
        self.seed, self.out_dir, self.final_samples = seed, out_dir, final_samples


class StochasticFiniteDiffInverseIntegrator:
    """inverse_integrator.h:61-246 — optimize(scene_initial, I_ref) -> bool, on the device
    (vr_sfd_optimize). `history` holds the mean L1 loss of every base render, `last_grads` the last
    SFD gradient estimate (float64), `params` / `scene` the optimised GMM, `final_loss` /
    `final_image` the final render at cfg.final_samples paths/pixel (:229-238; 0 skips it). As in the
    reference, the forward integrator is left at final_samples paths per pixel afterwards."""

    def __init__(self, camera, forward_integrator, cfg=None):
        if not isinstance(forward_integrator, MultiScatterGaussians):
            raise TypeError("the forward integrator must be MultiScatterGaussians (inverse_integrator.h:64)")
        self.camera, self.fwd, self.cfg = camera, forward_integrator, cfg or SFDConfig()
        self.history = []
        self.params = None
        self.last_grads = None
        self.final_loss = None
        self.final_image = None
        self.scene = None

    def optimize(self, scene_initial, I_ref):
        cfg = self.cfg
        n = scene_initial.get_num_primitives()
        if n == 0:
            return False
        W, H = I_ref.get_width(), I_ref.get_height()
        params = np.zeros(n * PER, np.float32)
        hist = np.zeros(max(cfg.max_iters, 1), np.float64)
        grads = np.zeros(n * PER, np.float64)
        final = Image(W, H)
        res = L.vr_sfd_result(params.ctypes.data_as(_fp), hist.ctypes.data_as(_dp), grads.ctypes.data_as(_dp),
                              final.pixels.ctypes.data_as(_fp), 0.0)
        out_dir = cfg.out_dir or ""
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
        c = L.vr_sfd_config(int(cfg.max_iters), int(cfg.save_every), int(cfg.num_stoch_samples), float(cfg.lr),
                            int(cfg.seed), int(cfg.final_samples), os.fsencode(out_dir))
        ref = np.ascontiguousarray(I_ref.pixels, np.float32)
        dev = Device.get(self.fwd.device)
        check(lib().vr_sfd_optimize(dev._h, ctypes.byref(self.camera.struct), ctypes.byref(self.fwd.params),
                                    scene_initial._h, ref.ctypes.data_as(_fp), W, H, ctypes.byref(c),
                                    ctypes.byref(res)))
        dev._scene_key = None  # the device now holds the last uploaded parameter set
        self.history = hist[:cfg.max_iters].tolist()
        self.params = params
        self.last_grads = grads if cfg.max_iters > 0 else None
        self.scene = apply_params(params, scene_initial.lights, scene_initial.env_color, base=scene_initial)
        if cfg.final_samples > 0:
            self.fwd.set_num_samples(cfg.final_samples)
            self.final_loss = float(res.final_loss)
            self.final_image = final
        return True
