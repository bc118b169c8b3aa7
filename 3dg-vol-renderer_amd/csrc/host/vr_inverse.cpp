// Inverse rendering by stochastic finite differences, natively:
//   * the GMM <-> feature-vector maps of gmm.h:583-706 (pack_parameters, apply_params_to_gmm_local,
//     make_default_eps_for_params) as host C++ on the library's scenes;
//   * AdamOptimizer (optimizer.h:13-55);
//   * StochasticFiniteDiffInverseIntegrator::optimize (inverse_integrator.h:61-238) as vr_sfd_optimize:
//     every forward render is a device MultiScatterGaussians render with RECORD_PIXEL_GAUSSIANS
//     bitsets kept in HBM, the per-pixel L1 losses are computed on the device next to the frame, the
//     per-Gaussian union-of-pixels statistic is one device pass over the two bitsets, and each
//     re-upload after a parameter update builds its BVH on the device (VR_OPT_DEVICE_BVH). The host
//     keeps the O(N) parameter bookkeeping and Adam, as the reference does.
// Deviations: the sign vectors come from a seeded PCG32 stream per (seed, vector index)
// instead of mt19937(random_device) (inverse_integrator.h:101-103); the eigen-decomposition of
// pack_parameters is a double-precision Jacobi solver with the eigenbasis made right-handed (Eigen's
// SelfAdjointEigenSolver may return det -1, which AngleAxisf silently turns into a different rotation).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "vr_common.h"

using namespace vr;

namespace {

constexpr size_t kPer = 11;  // parameters per Gaussian (inverse_integrator.h:108)

// gmm.h:18-32
float sigmoidf_safe(float x) {
    if (x >= 0.0f) {
        const float z = std::exp(-x);
        return 1.0f / (1.0f + z);
    }
    const float z = std::exp(x);
    return z / (1.0f + z);
}
float inv_sigmoidf(float y) {
    y = std::clamp(y, 1e-7f, 1.0f - 1e-7f);
    return std::log(y / (1.0f - y));
}

// Symmetric 3x3 eigen-decomposition (cyclic Jacobi, double): ascending eigenvalues, eigenvectors as
// columns of V, made right-handed.
void eigen_sym3(const double A_in[3][3], double w[3], double V[3][3]) {
    double A[3][3];
    std::memcpy(A, A_in, sizeof(A));
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) V[i][j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 64; ++sweep) {
        const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
        if (off < 1e-300) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                if (A[p][q] == 0.0) continue;
                const double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 3; ++k) {  // A <- J^T A J
                    const double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    const double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
    int idx[3] = {0, 1, 2};
    std::sort(idx, idx + 3, [&](int a, int b) { return A[a][a] < A[b][b]; });
    double W2[3][3];
    for (int j = 0; j < 3; ++j) {
        w[j] = A[idx[j]][idx[j]];
        for (int i = 0; i < 3; ++i) W2[i][j] = V[i][idx[j]];
    }
    std::memcpy(V, W2, sizeof(W2));
    const double det = V[0][0] * (V[1][1] * V[2][2] - V[1][2] * V[2][1]) - V[0][1] * (V[1][0] * V[2][2] - V[1][2] * V[2][0]) +
                       V[0][2] * (V[1][0] * V[2][1] - V[1][1] * V[2][0]);
    if (det < 0)
        for (int i = 0; i < 3; ++i) V[i][2] = -V[i][2];
}

// Eigen AngleAxis<float>(const Matrix3f&): quaternion from the matrix (branch on the trace / the
// largest diagonal entry), then angle = 2 atan2(|v|, |w|), axis = v / |v| with w's sign folded in.
void angle_axis_from_matrix(const float m[3][3], float rod[3]) {
    float q[4];  // x y z w
    float t = m[0][0] + m[1][1] + m[2][2];
    if (t > 0.0f) {
        t = std::sqrt(t + 1.0f);
        q[3] = 0.5f * t;
        t = 0.5f / t;
        q[0] = (m[2][1] - m[1][2]) * t;
        q[1] = (m[0][2] - m[2][0]) * t;
        q[2] = (m[1][0] - m[0][1]) * t;
    } else {
        int i = 0;
        if (m[1][1] > m[0][0]) i = 1;
        if (m[2][2] > m[i][i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0f);
        q[i] = 0.5f * t;
        t = 0.5f / t;
        q[3] = (m[k][j] - m[j][k]) * t;
        q[j] = (m[j][i] + m[i][j]) * t;
        q[k] = (m[k][i] + m[i][k]) * t;
    }
    float n = std::sqrt(q[0] * q[0] + (q[1] * q[1] + q[2] * q[2]));
    if (!(n > 0.0f)) {
        rod[0] = rod[1] = rod[2] = 0.0f;
        return;
    }
    const float angle = 2.0f * std::atan2(n, std::fabs(q[3]));
    if (q[3] < 0.0f) n = -n;
    for (int k = 0; k < 3; ++k) rod[k] = (q[k] / n) * angle;
}

// Eigen AngleAxis<float>::toRotationMatrix.
void rotation_from_angle_axis(float angle, const float a[3], float R[3][3]) {
    const float s = std::sin(angle), c = std::cos(angle);
    const float sa[3] = {s * a[0], s * a[1], s * a[2]};
    const float ca[3] = {(1.0f - c) * a[0], (1.0f - c) * a[1], (1.0f - c) * a[2]};
    float tmp = ca[0] * a[1];
    R[0][1] = tmp - sa[2];
    R[1][0] = tmp + sa[2];
    tmp = ca[0] * a[2];
    R[0][2] = tmp + sa[1];
    R[2][0] = tmp - sa[1];
    tmp = ca[1] * a[2];
    R[1][2] = tmp - sa[0];
    R[2][1] = tmp + sa[0];
    for (int k = 0; k < 3; ++k) R[k][k] = ca[k] * a[k] + c;
}

// 3x3 product with Eigen's per-coefficient order a_i0 b_0j + (a_i1 b_1j + a_i2 b_2j).
void mul3(const float A[3][3], const float B[3][3], float C[3][3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i][j] = A[i][0] * B[0][j] + (A[i][1] * B[1][j] + A[i][2] * B[2][j]);
}

// apply_params_to_gmm_local, one Gaussian (gmm.h:640-672): mean, R from the Rodrigues vector,
// S = diag(exp(log scale)), covariance R S S^T R^T (Gaussian's rotation+scale constructor,
// gaussian.h:95-108), density exp, albedo sigmoid clamped.
vr_gaussian gaussian_from_params(const float* p, const vr_gaussian& like) {
    vr_gaussian g = like;
    g.mean[0] = p[0];
    g.mean[1] = p[1];
    g.mean[2] = p[2];
    const float rod[3] = {p[3], p[4], p[5]};
    const float angle = std::sqrt(rod[0] * rod[0] + (rod[1] * rod[1] + rod[2] * rod[2]));
    float R[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    if (angle > 1e-12f) {
        const float axis[3] = {rod[0] / angle, rod[1] / angle, rod[2] / angle};
        rotation_from_angle_axis(angle, axis, R);
    }
    const float S[3][3] = {{std::exp(p[6]), 0, 0}, {0, std::exp(p[7]), 0}, {0, 0, std::exp(p[8])}};
    float St[3][3], Rt[3][3], RS[3][3], RSS[3][3], C[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            St[i][j] = S[j][i];
            Rt[i][j] = R[j][i];
        }
    mul3(R, S, RS);
    mul3(RS, St, RSS);
    mul3(RSS, Rt, C);
    g.cov[0] = C[0][0];
    g.cov[1] = C[0][1];
    g.cov[2] = C[0][2];
    g.cov[3] = C[1][1];
    g.cov[4] = C[1][2];
    g.cov[5] = C[2][2];
    g.density = std::exp(p[9]);
    g.albedo = std::clamp(sigmoidf_safe(p[10]), 0.0f, 1.0f);
    return g;
}

// Sign vector k of a run: PCG32 (rng.h) seeded by splitmix64 of (seed, k); +1 where the uniform < 0.5.
void sign_vector(uint64_t seed, uint64_t k, float* s, size_t n) {
    auto splitmix = [](uint64_t x) {
        x += 0x9e3779b97f4a7c15ULL;
        x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
        x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
        return x ^ (x >> 31);
    };
    uint64_t inc = (splitmix(k) << 1u) | 1u, state = 0;
    auto next = [&]() {
        const uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        const uint32_t x = (uint32_t)(((old >> 18u) ^ old) >> 27u), rot = (uint32_t)(old >> 59u);
        return (x >> rot) | (x << ((0u - rot) & 31u));
    };
    next();
    state += splitmix(seed);
    next();
    for (size_t i = 0; i < n; ++i) s[i] = ((next() >> 8) * (1.0f / 16777216.0f)) < 0.5f ? 1.0f : -1.0f;
}

}  // namespace

extern "C" {

vr_status vr_gmm_pack_parameters(const vr_scene* sc, float* out, size_t n_params) {
    if (!sc || (n_params && !out)) return fail(VR_ERR_INVALID, "vr_gmm_pack_parameters: NULL argument");
    const HostScene& s = sc->s;
    if (s.type != VR_VOLUME_GAUSSIANS) return fail(VR_ERR_INVALID, "vr_gmm_pack_parameters: not a Gaussian scene");
    if (n_params != s.gaussians.size() * kPer)
        return fail(VR_ERR_INVALID, "vr_gmm_pack_parameters: n_params must be 11 * N = " + std::to_string(s.gaussians.size() * kPer));
    for (size_t i = 0; i < s.gaussians.size(); ++i) {  // gmm.h:583-628
        const vr_gaussian& g = s.gaussians[i];
        float* p = out + i * kPer;
        p[0] = g.mean[0];
        p[1] = g.mean[1];
        p[2] = g.mean[2];
        const double A[3][3] = {{g.cov[0], g.cov[1], g.cov[2]}, {g.cov[1], g.cov[3], g.cov[4]}, {g.cov[2], g.cov[4], g.cov[5]}};
        double w[3], V[3][3];
        eigen_sym3(A, w, V);
        float R[3][3];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) R[a][b] = (float)V[a][b];
        float rod[3];
        angle_axis_from_matrix(R, rod);
        if (!std::isfinite(rod[0]) || !std::isfinite(rod[1]) || !std::isfinite(rod[2])) rod[0] = rod[1] = rod[2] = 0.0f;
        p[3] = rod[0];
        p[4] = rod[1];
        p[5] = rod[2];
        for (int k = 0; k < 3; ++k) {  // scale = sqrt(max(eigenvalue, 0)) (gaussian.h:87-90), guarded at 1e-12
            const float sd = std::sqrt(std::max((float)w[k], 0.0f));
            p[6 + k] = std::log(std::max(sd, 1e-12f));
        }
        p[9] = std::log(std::max(g.density, 1e-12f));
        p[10] = inv_sigmoidf(std::clamp(g.albedo, 0.0f, 1.0f));
    }
    return VR_OK;
}

vr_status vr_gmm_apply_parameters(const vr_scene* base, const float* params, size_t n_params, vr_scene** out) {
    if (!base || !out || (n_params && !params)) return fail(VR_ERR_INVALID, "vr_gmm_apply_parameters: NULL argument");
    const HostScene& b = base->s;
    if (b.type != VR_VOLUME_GAUSSIANS) return fail(VR_ERR_INVALID, "vr_gmm_apply_parameters: not a Gaussian scene");
    if (n_params != b.gaussians.size() * kPer) return fail(VR_ERR_INVALID, "apply params size mismatch");  // gmm.h:637
    auto* s = new vr_scene();
    s->s.type = VR_VOLUME_GAUSSIANS;
    s->s.lights = b.lights;
    std::memcpy(s->s.env, b.env, sizeof(s->s.env));
    s->s.gaussians.resize(b.gaussians.size());
    s->s.pre.resize(b.gaussians.size());
    for (size_t i = 0; i < b.gaussians.size(); ++i) {
        s->s.gaussians[i] = gaussian_from_params(params + i * kPer, b.gaussians[i]);
        s->s.pre[i] = precompute_gaussian(s->s.gaussians[i]);
    }
    *out = s;
    return VR_OK;
}

vr_status vr_gmm_default_eps(float* eps, size_t n_params) {  // gmm.h:678-706
    if (n_params % kPer != 0 || (n_params && !eps)) return fail(VR_ERR_INVALID, "vr_gmm_default_eps: n_params must be 11 * N");
    const float one[kPer] = {0.02f, 0.02f, 0.02f, 0.10f, 0.10f, 0.10f, 0.05f, 0.05f, 0.05f, 0.25f, 0.5f};
    for (size_t i = 0; i < n_params; ++i) eps[i] = one[i % kPer];
    return VR_OK;
}

vr_status vr_sfd_sign_vector(uint64_t seed, uint64_t k, float* s, size_t n) {
    if (n && !s) return fail(VR_ERR_INVALID, "vr_sfd_sign_vector: NULL argument");
    sign_vector(seed, k, s, n);
    return VR_OK;
}

vr_status vr_adam_step(float* params, const float* grads, float* m, float* v, size_t n, int32_t t, float lr, float beta1,
                       float beta2, float eps) {  // optimizer.h:31-44, step t >= 1
    if (n && (!params || !grads || !m || !v)) return fail(VR_ERR_INVALID, "vr_adam_step: NULL argument");
    if (t < 1) return fail(VR_ERR_INVALID, "vr_adam_step: t must be >= 1");
    const float a = lr * std::sqrt(1.0f - std::pow(beta2, (float)t)) / (1.0f - std::pow(beta1, (float)t));
    for (size_t i = 0; i < n; ++i) {
        const float g = grads[i];
        m[i] = beta1 * m[i] + (1.0f - beta1) * g;
        v[i] = beta2 * v[i] + (1.0f - beta2) * g * g;
        params[i] -= a * (m[i] / (std::sqrt(v[i]) + eps));
    }
    return VR_OK;
}

vr_status vr_sfd_optimize(vr_ctx* c, const vr_camera* cam, const vr_render_params* fwd, const vr_scene* initial,
                          const float* I_ref, uint32_t W, uint32_t H, const vr_sfd_config* cfg, vr_sfd_result* res) {
    if (!c || !cam || !fwd || !initial || !I_ref || !cfg || !res) return fail(VR_ERR_INVALID, "vr_sfd_optimize: NULL argument");
    if (fwd->integrator != VR_MULTI_SCATTER)
        return fail(VR_ERR_INVALID, "vr_sfd_optimize: the forward integrator must be MultiScatterGaussians (inverse_integrator.h:64)");
    if (cfg->max_iters < 0 || cfg->num_stoch_samples < 1) return fail(VR_ERR_INVALID, "vr_sfd_optimize: bad config");
    if (!res->params || (cfg->max_iters > 0 && !res->loss_history))
        return fail(VR_ERR_INVALID, "vr_sfd_optimize: result buffers missing");
    const HostScene& s0 = initial->s;
    const size_t N = s0.gaussians.size();
    if (s0.type != VR_VOLUME_GAUSSIANS || N == 0) return fail(VR_ERR_INVALID, "Scene has no GMM.");  // :71-74
    const size_t D = N * kPer;
    std::vector<float> params(D), eps(D), m(D, 0.0f), v(D, 0.0f), sgn(D), grads_f(D);
    std::vector<double> grads(D);
    vr_status st;
    if ((st = vr_gmm_pack_parameters(initial, params.data(), D)) != VR_OK) return st;
    vr_gmm_default_eps(eps.data(), D);
    const uint32_t npix = W * H;
    std::vector<float> loss(npix);
    // A multi-GPU context (vr_init_multi) spreads the perturbed renders of an iteration over its
    // ranks: rank r renders samples r, r + R, ... after a base render of its own (every rank holds
    // the same GMM, the render is deterministic, so each rank's base recording and losses are the
    // ones rank 0 would make). Sample k's difference vector lands in slot k and the gradient sums
    // them in sample order: the result does not depend on the number of ranks.
    const int R = std::max(1, std::min(ctx_ranks(c), cfg->num_stoch_samples));
    auto rank_label = [](int r) { return "vr_sfd_optimize rank " + std::to_string(r); };
    std::vector<std::vector<float>> rloss(R, std::vector<float>(npix));
    std::vector<std::vector<double>> fd((size_t)cfg->num_stoch_samples, std::vector<double>(N));
    int64_t old_bvh = 0;
    vr_get_option(c, VR_OPT_DEVICE_BVH, &old_bvh);
    if ((st = vr_set_option(c, VR_OPT_DEVICE_BVH, 1)) != VR_OK) return st;  // every re-upload builds on the device
    auto done = [&](vr_status r) {
        vr_set_option(c, VR_OPT_DEVICE_BVH, old_bvh);
        return r;
    };
    st = run_parallel(R, [&](int r) { return sfd_set_reference(ctx_rank(c, r), I_ref, W, H); }, rank_label);
    if (st != VR_OK) return done(st);
    auto mean = [&](const std::vector<float>& l) {  // :222-225: double sum in pixel order
        double a = 0.0;
        for (float x : l) a += x;
        return a / (double)l.size();
    };
    auto upload_params = [&](vr_ctx* ctx, const float* p) -> vr_status {  // ctx: one rank, or the whole group
        vr_scene* sc = nullptr;
        vr_status r = vr_gmm_apply_parameters(initial, p, D, &sc);
        if (r != VR_OK) return r;
        r = vr_upload_scene(ctx, sc);
        vr_scene_destroy(sc);
        return r;
    };
    if ((st = vr_upload_scene(c, initial)) != VR_OK) return done(st);  // the initial GMM first (:84-88)
    for (int it = 0; it < cfg->max_iters; ++it) {
        // 1) base render + recording, base losses (:114-122); 2-3) stochastic sign vectors, perturbed
        // recorded renders, union statistic (:135-190)
        const uint64_t draw0 = (uint64_t)it * (uint64_t)cfg->num_stoch_samples;
        st = run_parallel(
            R,
            [&](int r) -> vr_status {
                vr_ctx* cr = ctx_rank(c, r);
                vr_status e = sfd_render(cr, cam, fwd, W, H, 0, 0, rloss[r].data(), nullptr);
                std::vector<float> sg(D), pl(D), lplus(npix);
                for (int k = r; e == VR_OK && k < cfg->num_stoch_samples; k += R) {
                    sign_vector(cfg->seed, draw0 + (uint64_t)k, sg.data(), D);
                    for (size_t i = 0; i < D; ++i) pl[i] = params[i] + sg[i] * eps[i];
                    if ((e = upload_params(cr, pl.data())) != VR_OK) break;
                    if ((e = sfd_render(cr, cam, fwd, W, H, 1, 1, lplus.data(), nullptr)) != VR_OK) break;
                    e = sfd_loss_diff_device(cr, npix, fd[k].data(), N);
                }
                return e;
            },
            rank_label);
        if (st != VR_OK) return done(st);
        res->loss_history[it] = mean(rloss[0]);
        std::fill(grads.begin(), grads.end(), 0.0);
        for (int k = 0; k < cfg->num_stoch_samples; ++k) {
            sign_vector(cfg->seed, draw0 + (uint64_t)k, sgn.data(), D);
            for (size_t i = 0; i < D; ++i) {
                const double denom = (double)eps[i];
                if (std::fabs(denom) < 1e-12) continue;
                grads[i] += fd[k][i / kPer] * (double)sgn[i] / denom;
            }
        }
        for (size_t i = 0; i < D; ++i) grads_f[i] = (float)(grads[i] / (double)cfg->num_stoch_samples);
        if (res->last_grads)
            for (size_t i = 0; i < D; ++i) res->last_grads[i] = grads[i] / (double)cfg->num_stoch_samples;
        // Adam (:201-205), then the updated GMM on every rank (:208)
        if ((st = vr_adam_step(params.data(), grads_f.data(), m.data(), v.data(), D, it + 1, cfg->lr, 0.9f, 0.999f, 1e-8f)) != VR_OK)
            return done(st);
        if ((st = upload_params(c, params.data())) != VR_OK) return done(st);
        if (cfg->save_every > 0 && cfg->out_dir && cfg->out_dir[0] && it % cfg->save_every == 0) {  // :211-227
            std::vector<float> rgb((size_t)npix * 3);
            if ((st = sfd_render(c, cam, fwd, W, H, -1, 0, loss.data(), rgb.data())) != VR_OK) return done(st);
            char fn[4096];
            std::snprintf(fn, sizeof(fn), "%s/iter_%04d.ppm", cfg->out_dir, it);
            if ((st = vr_image_write_ppm(fn, rgb.data(), W, H)) != VR_OK) return done(st);
        }
    }
    std::memcpy(res->params, params.data(), D * sizeof(float));
    res->final_loss = -1.0;
    if (cfg->final_samples > 0) {  // final save (:229-238) at final_samples paths per pixel
        vr_render_params fp = *fwd;
        fp.num_samples = cfg->final_samples;
        std::vector<float> rgb(res->final_image ? 0 : (size_t)npix * 3);
        float* img = res->final_image ? res->final_image : rgb.data();
        if ((st = sfd_render(c, cam, &fp, W, H, -1, 0, loss.data(), img)) != VR_OK) return done(st);
        res->final_loss = mean(loss);
        if (cfg->out_dir && cfg->out_dir[0]) {
            char fn[4096];
            std::snprintf(fn, sizeof(fn), "%s/iter_%04d.ppm", cfg->out_dir, std::max(cfg->max_iters - 1, 0));
            if ((st = vr_image_write_ppm(fn, img, W, H)) != VR_OK) return done(st);
        }
    }
    return done(VR_OK);
}

}  // extern "C"
