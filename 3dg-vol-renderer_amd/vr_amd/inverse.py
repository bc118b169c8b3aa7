"""Inverse rendering by stochastic finite differences, host side of
StochasticFiniteDiffInverseIntegrator (include/inverse_integrator.h:50-246), AdamOptimizer
(include/optimizer.h:13-55) and the GMM <-> feature-vector maps (include/gmm.h:583-706).

The forward renders (1 + num_stoch_samples MultiScatterGaussians renders with per-pixel Gaussian
recording per iteration) and the per-Gaussian union-of-pixels loss statistic run on the device
(vr_render_record, vr_sfd_loss_diff: the recordings stay in HBM as W*H x N bitsets, the statistic
is one bandwidth-bound pass over them). Parameter bookkeeping, Adam and the BVH rebuild of each
re-uploaded scene stay on the host, as in the reference.

Deviations (documented in DESIGN.md): the sign vectors come from a seeded numpy generator instead
of mt19937(random_device) (:101-103, not reproducible in the reference); eigenvector signs of the
3x3 eigen-decomposition (pack_parameters, gmm.h:599) follow LAPACK, not Eigen's solver (unpinned),
and the eigenbasis is made right-handed before the AngleAxis conversion: the reference converts a
possibly left-handed eigenvector matrix (det -1) to AngleAxis, which is not a rotation and changes
the covariance on the first apply_params_to_gmm_local; here pack -> apply reproduces the covariance.
"""
import os

import numpy as np

from . import MultiScatterGaussians, Scene, Light, Device, Image, check, lib  # noqa: F401

PER = 11  # parameters per Gaussian (inverse_integrator.h:108)


# ---- gmm.h:18-32 ----
def sigmoidf_safe(x):
    x = np.asarray(x, np.float32)
    z = np.exp(-np.abs(x)).astype(np.float32)
    return np.where(x >= 0, np.float32(1) / (np.float32(1) + z), z / (np.float32(1) + z)).astype(np.float32)


def inv_sigmoidf(y):
    yy = np.clip(np.asarray(y, np.float32), np.float32(1e-7), np.float32(1 - 1e-7))
    return np.log(yy / (np.float32(1) - yy)).astype(np.float32)


def _cov_matrix(cov6):
    c = np.asarray(cov6, np.float64)
    return np.array([[c[0], c[1], c[2]], [c[1], c[3], c[4]], [c[2], c[4], c[5]]])


def _angle_axis_from_matrix(R):
    """Eigen AngleAxis(const Matrix3&): quaternion from the matrix (Eigen's branch on the trace /
    largest diagonal), then angle = 2 atan2(|v|, |w|), axis = v / |v| (sign of w folded in)."""
    m = R
    t = m[0, 0] + m[1, 1] + m[2, 2]
    q = np.zeros(4)  # x y z w
    if t > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (m[2, 1] - m[1, 2]) * t
        q[1] = (m[0, 2] - m[2, 0]) * t
        q[2] = (m[1, 0] - m[0, 1]) * t
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k, j] - m[j, k]) * t
        q[j] = (m[j, i] + m[i, j]) * t
        q[k] = (m[k, i] + m[i, k]) * t
    n = np.linalg.norm(q[:3])
    if n < 1e-12:
        return np.zeros(3)
    angle = 2.0 * np.arctan2(n, abs(q[3]))
    if q[3] < 0:
        n = -n
    return q[:3] / n * angle


def _rotation_from_rodrigues(rod):
    angle = float(np.linalg.norm(rod))
    if not angle > 1e-12:
        return np.eye(3)
    a = rod / angle
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(angle) * K + (1 - np.cos(angle)) * (K @ K)  # AngleAxis::toRotationMatrix


def pack_parameters(gaussians):
    """GaussianMixtureModel::pack_parameters (gmm.h:583-628): per Gaussian mean(3), Rodrigues
    rotation(3), log scale(3), log density, logit albedo. `gaussians`: (N, >=11) array as returned by
    Scene.gaussians() (mean, cov6, density, albedo)."""
    g = np.asarray(gaussians, np.float32)
    out = np.zeros((g.shape[0], PER), np.float32)
    for i, row in enumerate(g):
        lam, U = np.linalg.eigh(_cov_matrix(row[3:9]))  # ascending, like SelfAdjointEigenSolver
        if np.linalg.det(U) < 0:  # right-handed eigenbasis (see module docstring)
            U[:, 2] = -U[:, 2]
        rod = _angle_axis_from_matrix(U)
        if not np.all(np.isfinite(rod)):
            rod = np.zeros(3)
        sd = np.sqrt(np.maximum(lam, 0.0))
        out[i, 0:3] = row[0:3]
        out[i, 3:6] = rod
        out[i, 6:9] = np.log(np.maximum(sd, 1e-12))
        out[i, 9] = np.log(max(float(row[9]), 1e-12))
        out[i, 10] = inv_sigmoidf(np.clip(row[10], 0.0, 1.0))
    return out.reshape(-1)


def apply_params(params, lights, env_color):
    """apply_params_to_gmm_local (gmm.h:634-674): rebuild every Gaussian from (mean, R, S) with
    covariance R S S^T R^T; returns a new Scene (the device BVH is rebuilt at upload, gmm.h:673)."""
    p = np.asarray(params, np.float32).reshape(-1, PER)
    n = p.shape[0]
    rod = p[:, 3:6].astype(np.float64)
    angle = np.linalg.norm(rod, axis=1)
    ok = angle > 1e-12
    ax = np.where(ok[:, None], rod / np.where(ok, angle, 1.0)[:, None], 0.0)
    K = np.zeros((n, 3, 3))
    K[:, 0, 1], K[:, 0, 2], K[:, 1, 2] = -ax[:, 2], ax[:, 1], -ax[:, 0]
    K[:, 1, 0], K[:, 2, 0], K[:, 2, 1] = ax[:, 2], -ax[:, 1], ax[:, 0]
    R = np.eye(3)[None] + np.sin(angle)[:, None, None] * K + (1 - np.cos(angle))[:, None, None] * np.einsum("nij,njk->nik", K, K)
    s2 = np.exp(p[:, 6:9].astype(np.float32)).astype(np.float64) ** 2
    C = np.einsum("nij,nj,nkj->nik", R, s2, R)  # R S S^T R^T (AngleAxis::toRotationMatrix)
    cov6 = np.stack([C[:, 0, 0], C[:, 0, 1], C[:, 0, 2], C[:, 1, 1], C[:, 1, 2], C[:, 2, 2]], 1).astype(np.float32)
    density = np.exp(p[:, 9]).astype(np.float32)
    albedo = np.clip(sigmoidf_safe(p[:, 10]), 0.0, 1.0)
    return Scene.from_gaussians(p[:, 0:3], cov6, density, albedo, lights=lights, env_color=env_color)


def make_default_eps_for_params(params):
    """gmm.h:678-706"""
    one = np.array([0.02] * 3 + [0.10] * 3 + [0.05] * 3 + [0.25, 0.5], np.float32)
    return np.tile(one, len(params) // PER)


class AdamOptimizer:
    """optimizer.h:13-55 (float32 state, bias-corrected step size a = lr sqrt(1-b2^t) / (1-b1^t))."""

    def __init__(self, ndim, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8):
        self.lr, self.beta1, self.beta2, self.eps = np.float32(lr), np.float32(beta1), np.float32(beta2), np.float32(eps)
        self.m = np.zeros(ndim, np.float32)
        self.v = np.zeros(ndim, np.float32)
        self.t = 0

    def step(self, params, grads):
        if params.shape != grads.shape or params.shape != self.m.shape:
            return False
        self.t += 1
        one = np.float32(1)
        a = self.lr * np.sqrt(one - self.beta2 ** np.float32(self.t)) / (one - self.beta1 ** np.float32(self.t))
        g = grads.astype(np.float32)
        self.m[:] = self.beta1 * self.m + (one - self.beta1) * g
        self.v[:] = self.beta2 * self.v + (one - self.beta2) * g * g
        params -= (a * (self.m / (np.sqrt(self.v) + self.eps))).astype(np.float32)
        return True

    def reset_state(self):
        self.m[:] = 0
        self.v[:] = 0
        self.t = 0


def compute_pixel_losses(I, I_ref):
    """inverse_integrator.h:21-30: per-pixel L1 over RGB, row-major."""
    return np.abs(I.pixels - I_ref.pixels).sum(axis=2).reshape(-1).astype(np.float32)


class SFDConfig:
    """inverse_integrator.h:54-59"""

    def __init__(self, max_iters=1000, save_every=25, num_stoch_samples=4, lr=1e-2, seed=0, out_dir=None,
                 final_samples=16384):
        self.max_iters, self.save_every, self.num_stoch_samples, self.lr = max_iters, save_every, num_stoch_samples, lr
        self.seed, self.out_dir, self.final_samples = seed, out_dir, final_samples


class StochasticFiniteDiffInverseIntegrator:
    """inverse_integrator.h:61-246 — optimize(scene_initial, I_ref) -> bool. `history` holds the
    mean L1 loss of every base render, `last_grads` the last SFD gradient estimate (float64),
    `final_loss` / `final_image` the final render at cfg.final_samples paths/pixel (:229-238;
    final_samples = 0 skips it)."""

    def __init__(self, camera, forward_integrator, cfg=None):
        if not isinstance(forward_integrator, MultiScatterGaussians):
            raise TypeError("the forward integrator must be MultiScatterGaussians (inverse_integrator.h:64)")
        self.camera, self.fwd, self.cfg = camera, forward_integrator, cfg or SFDConfig()
        self.history = []
        self.params = None
        self.last_grads = None
        self.final_loss = None
        self.final_image = None

    def optimize(self, scene_initial, I_ref):
        cfg = self.cfg
        g0 = scene_initial.gaussians()
        if len(g0) == 0:
            return False
        lights, env = scene_initial.lights, scene_initial.env_color
        params = pack_parameters(g0)
        eps = make_default_eps_for_params(params)
        adam = AdamOptimizer(params.size, cfg.lr)
        rng = np.random.default_rng(cfg.seed)
        W, H = I_ref.get_width(), I_ref.get_height()
        I_base, I_plus = Image(W, H), Image(W, H)
        n = len(g0)
        dev = Device.get(self.fwd.device)
        if cfg.out_dir:
            os.makedirs(cfg.out_dir, exist_ok=True)
        scene_opt = scene_initial  # the reference renders the initial GMM first (:84-88)
        for it in range(cfg.max_iters):
            self.fwd.record(scene_opt, I_base, slot=0)  # 1) base render + recording
            loss_base = compute_pixel_losses(I_base, I_ref)
            self.history.append(float(loss_base.mean()))
            grads = np.zeros(params.size, np.float64)
            for _ in range(cfg.num_stoch_samples):  # 3) stochastic sign vectors
                s = np.where(rng.random(params.size) < 0.5, 1.0, -1.0).astype(np.float32)
                params_plus = (params + s * eps).astype(np.float32)
                self.fwd.record(apply_params(params_plus, lights, env), I_plus, slot=1)
                loss_plus = compute_pixel_losses(I_plus, I_ref)
                fdiff = np.zeros(n, np.float64)
                check(lib().vr_sfd_loss_diff(dev._h, loss_base.ctypes.data_as(_fp), loss_plus.ctypes.data_as(_fp), W, H,
                                             fdiff.ctypes.data_as(_dp), n))
                grads += np.repeat(fdiff, PER) * s.astype(np.float64) / eps.astype(np.float64)
            grads /= cfg.num_stoch_samples
            self.last_grads = grads.copy()
            if not adam.step(params, grads.astype(np.float32)):
                return False
            scene_opt = apply_params(params, lights, env)
            if cfg.out_dir and it % cfg.save_every == 0:
                self.fwd.render(scene_opt, I_base)
                I_base.make_PPM(os.path.join(cfg.out_dir, f"iter_{it:04d}.ppm"))
        self.params = params
        self.scene = scene_opt
        if cfg.final_samples > 0:  # final save (:229-238): the optimised GMM at final_samples paths/pixel
            self.fwd.set_num_samples(cfg.final_samples)  # left set, as the reference leaves it
            self.fwd.render(scene_opt, I_base)
            self.final_loss = float(compute_pixel_losses(I_base, I_ref).astype(np.float64).mean())
            self.final_image = I_base
            if cfg.out_dir:
                I_base.make_PPM(os.path.join(cfg.out_dir, f"iter_{cfg.max_iters - 1:04d}.ppm"))
        return True


import ctypes  # noqa: E402

_fp = ctypes.POINTER(ctypes.c_float)
_dp = ctypes.POINTER(ctypes.c_double)
