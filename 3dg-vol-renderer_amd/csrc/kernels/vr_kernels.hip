// Ray-march kernels for gfx950 (MI355X).
//
// rm_gaussians_kernel: the north-star loop, RayMarchingGaussians::render
// (test_integrators.h:160-296), one thread per pixel, one 256-thread workgroup per 16x16 tile
// (each wave64 an 8x8 quadrant, so a wave's rays are spatially coherent).
//
// The reference gathers every ellipsoid event of a ray, sorts them and walks a float step
// sequence, re-scanning an O(N) mask at every step. Here no event list is ever built:
//   * the step sequence t_k is the reference's own iterated float sum, precomputed once per
//     step size (RenderArgs::tsteps), so empty stretches are skipped by index;
//   * the active set at step k is {i : a_i <= t_k < b_i}; it is kept as a short sorted list of
//     Gaussian indices in LDS and extended by BVH queries on the primary ray restricted to the
//     window (t_{k-1}, t_k] ("segment query"), or by a closest-entry query when it runs empty;
//   * secondary (light / environment) transmittance telescopes the reference's segment loop
//     into one sum of per-Gaussian optical depths over each Gaussian's active interval on the
//     secondary ray, reproducing its quirks exactly: Gaussians active on the primary ray are
//     pre-activated at t = 0 (test_integrators.h:209-211), a light's final segment runs to the
//     first event at or past the light (:220-235), environment rays run to their last event
//     (:258-271);
//   * a ray stops when its transmittance reaches t_eps (exactly 0 by default, which changes no
//     output bit: every later contribution is multiplied by T).
// Pixels whose active set outgrows the fast path's LDS list are pushed to a queue and re-run by
// rm_gaussians_fallback_kernel (larger list, same code), so results never depend on capacity.
#include <hip/hip_runtime.h>

#include "../../../include/vr_hip.h"
#include "vr_march.h"

namespace vr {
namespace dev {

constexpr float kInv4Pi = (float)(1.0 / (4.0 * 3.14159265358979323846));  // Vector3f * double -> float
constexpr float k4Pi = (float)(4.0 * 3.14159265358979323846);
constexpr float kTPad = 1e-5f;

struct ActList {
    int* act;    // LDS, element i at act[i * stride]
    int stride;
    int n;
    uint64_t bloom;
    __device__ __forceinline__ int get(int i) const { return act[i * stride]; }
    __device__ __forceinline__ void set(int i, int v) { act[i * stride] = v; }
    __device__ __forceinline__ void rebuild_bloom() {
        bloom = 0;
        for (int i = 0; i < n; ++i) bloom |= 1ull << (get(i) & 63);
    }
    // slot of Gaussian j in the list, or -1
    __device__ __forceinline__ int find(int j) const {
        if (!((bloom >> (j & 63)) & 1ull)) return -1;
        for (int i = 0; i < n; ++i)
            if (get(i) == j) return i;
        return -1;
    }
};

// Transmittance from `pos` towards a point light at distance `dist` along shadow ray `sr`
// (test_integrators.h:202-237).
__device__ float light_transmittance(const RenderArgs& A, const Ray& sr, float dist, const ActList& act, int* stack,
                                     int stride) {
    if (!(dist > 0.0f)) return 1.0f;  // `while (t_prev < dist)` never runs
    const GaussianRecord* __restrict__ G = A.gauss;
    float tau = 0.0f;
    bool needs_stop = false;
    uint64_t hitmask = 0;
    traverse(A.nodes, sr, stack, stride, [&](float tmin, float) { return tmin <= dist + kTPad * (1.0f + dist); },
             [&](uint32_t first, uint32_t count) {
                 for (uint32_t j = first; j < first + count; ++j) {
                     GRec g = load_rec(G, j);
                     Quad q = quad(g, sr);
                     float a, b;
                     if (!intersect(q, a, b)) continue;
                     int slot = act.find((int)j);
                     float lo = a;
                     if (slot >= 0) {
                         lo = 0.0f;
                         hitmask |= 1ull << slot;
                     }
                     if (b < dist) tau += optical_depth(g, q, lo, b);
                     else if (lo < dist) needs_stop = true;
                 }
             });
    uint64_t all = act.n >= 64 ? ~0ull : ((1ull << act.n) - 1ull);
    uint64_t missed = all & ~hitmask;
    if (needs_stop || missed) {
        // first event at or beyond the light: where the reference's last segment ends
        float tstop = INFINITY;
        traverse(A.nodes, sr, stack, stride,
                 [&](float tmin, float tmax) {
                     return tmax >= dist - kTPad * (1.0f + dist) && tmin <= tstop + kTPad * (1.0f + tstop);
                 },
                 [&](uint32_t first, uint32_t count) {
                     for (uint32_t j = first; j < first + count; ++j) {
                         GRec g = load_rec(G, j);
                         Quad q = quad(g, sr);
                         float a, b;
                         if (!intersect(q, a, b)) continue;
                         if (b >= dist) {
                             float e = (a >= dist) ? a : b;
                             tstop = fminf(tstop, e);
                         }
                     }
                 });
        if (tstop == INFINITY) tstop = dist;
        if (needs_stop) {
            traverse(A.nodes, sr, stack, stride,
                     [&](float tmin, float tmax) {
                         return tmin <= dist + kTPad * (1.0f + dist) && tmax >= dist - kTPad * (1.0f + dist);
                     },
                     [&](uint32_t first, uint32_t count) {
                         for (uint32_t j = first; j < first + count; ++j) {
                             GRec g = load_rec(G, j);
                             Quad q = quad(g, sr);
                             float a, b;
                             if (!intersect(q, a, b)) continue;
                             float lo = act.find((int)j) >= 0 ? 0.0f : a;
                             if (lo < dist && b >= dist) tau += optical_depth(g, q, lo, tstop);
                         }
                     });
        }
        while (missed) {
            int s = __ffsll((unsigned long long)missed) - 1;
            missed &= missed - 1;
            int j = act.get(s);
            GRec g = load_rec(G, j);
            Quad q = quad(g, sr);
            tau += optical_depth(g, q, 0.0f, tstop);
        }
    }
    return expf(-tau);
}

// Transmittance along an environment ray to its last event (test_integrators.h:241-273).
__device__ float env_transmittance(const RenderArgs& A, const Ray& er, const ActList& act, int* stack, int stride) {
    const GaussianRecord* __restrict__ G = A.gauss;
    float tau = 0.0f, tlast = 0.0f;
    uint64_t hitmask = 0;
    traverse(A.nodes, er, stack, stride, [&](float, float) { return true; },
             [&](uint32_t first, uint32_t count) {
                 for (uint32_t j = first; j < first + count; ++j) {
                     GRec g = load_rec(G, j);
                     Quad q = quad(g, er);
                     float a, b;
                     if (!intersect(q, a, b)) continue;
                     int slot = act.find((int)j);
                     float lo = a;
                     if (slot >= 0) {
                         lo = 0.0f;
                         hitmask |= 1ull << slot;
                     }
                     tau += optical_depth(g, q, lo, b);
                     tlast = fmaxf(tlast, b);
                 }
             });
    uint64_t all = act.n >= 64 ? ~0ull : ((1ull << act.n) - 1ull);
    uint64_t missed = all & ~hitmask;
    while (missed) {
        int s = __ffsll((unsigned long long)missed) - 1;
        missed &= missed - 1;
        int j = act.get(s);
        GRec g = load_rec(G, j);
        Quad q = quad(g, er);
        tau += optical_depth(g, q, 0.0f, tlast);
    }
    return expf(-tau);
}

enum { kOK = 0, kOverflow = 1, kError = 2 };

// One pixel of RayMarchingGaussians. Returns kOK / kOverflow (active list full) / kError.
template <int ACT>
__device__ int march_gaussians(const RenderArgs& A, int px, int py, int* act_base, int* stack, int stride, float& R0,
                               float& R1, float& R2) {
    const Ray ray = primary_ray(A, px, py);
    const GaussianRecord* __restrict__ G = A.gauss;
    const float* __restrict__ ts = A.tsteps;
    const int nts = A.num_tsteps;
    const float step = A.step_size;
    float T = 1.0f, L0 = 0.0f, L1 = 0.0f, L2 = 0.0f;
    ActList act{act_base, stride, 0, 0};
    int kq = 0;
    for (;;) {
        const float t_lo = (kq == 0) ? -1.0f : ts[kq - 1];
        int k;
        if (act.n == 0) {
            // closest entry strictly after t_lo
            float best = INFINITY;
            traverse(A.nodes, ray, stack, stride,
                     [&](float tmin, float tmax) {
                         return tmax >= t_lo - kTPad * (1.0f + fabsf(t_lo)) && tmin <= best + kTPad * (1.0f + best);
                     },
                     [&](uint32_t first, uint32_t count) {
                         for (uint32_t j = first; j < first + count; ++j) {
                             GRec g = load_rec(G, j);
                             Quad q = quad(g, ray);
                             float a, b;
                             if (intersect(q, a, b) && a > t_lo && a < best) best = a;
                         }
                     });
            if (best == INFINITY) break;
            k = kfirst(ts, nts, step, best);
        } else {
            k = kq;
        }
        if (k >= nts - 1) return kError;  // step table too short (host sizes it from scene bounds)
        const float t_k = ts[k];
        // entrants: t_lo < a <= t_k and still inside at t_k (b > t_k)
        bool ovf = false;
        traverse(A.nodes, ray, stack, stride,
                 [&](float tmin, float tmax) {
                     return tmax >= t_lo - kTPad * (1.0f + fabsf(t_lo)) && tmin <= t_k + kTPad * (1.0f + t_k);
                 },
                 [&](uint32_t first, uint32_t count) {
                     for (uint32_t j = first; j < first + count; ++j) {
                         GRec g = load_rec(G, j);
                         Quad q = quad(g, ray);
                         float a, b;
                         if (!intersect(q, a, b) || !(a > t_lo) || !(a <= t_k) || !(b > t_k)) continue;
                         if (act.n >= ACT) {
                             ovf = true;
                             continue;
                         }
                         int i = act.n;  // sorted insert
                         while (i > 0 && act.get(i - 1) > (int)j) {
                             act.set(i, act.get(i - 1));
                             --i;
                         }
                         act.set(i, (int)j);
                         act.n++;
                     }
                 });
        if (ovf) return kOverflow;
        kq = k + 1;
        // retire (b <= t_k), evaluate sigma at pos (gmm.h:98-126) and the step's optical depth
        const float px_ = ray.ox + t_k * ray.dx;
        const float py_ = ray.oy + t_k * ray.dy;
        const float pz_ = ray.oz + t_k * ray.dz;
        const float t_k1 = t_k + step;  // `t + step_size` (test_integrators.h:286)
        float smu = 0.0f, smua = 0.0f, tau_seg = 0.0f;
        int w = 0;
        for (int i = 0; i < act.n; ++i) {
            int j = act.get(i);
            GRec g = load_rec(G, j);
            Quad q = quad(g, ray);
            float a, b;
            bool hit = intersect(q, a, b);
            if (!hit || b <= t_k) continue;
            act.set(w++, j);
            float m = mu_t(g, px_, py_, pz_);
            smu += m;
            smua += m * g.albedo;
            tau_seg += optical_depth(g, q, t_k, t_k1);
        }
        act.n = w;
        if (w == 0) continue;
        float sigma_s = 0.0f;
        if (smu > 0.0f) {
            float a_mix = smua / smu;
            sigma_s = a_mix * smu;
        }
        if (sigma_s > 0.0f) {
            act.rebuild_bloom();
            float Li0 = 0.0f, Li1 = 0.0f, Li2 = 0.0f;
            for (int l = 0; l < A.num_lights; ++l) {
                const LightRecord& lr = A.lights[l];
                float dx = lr.px - px_, dy = lr.py - py_, dz = lr.pz - pz_;
                float sq = dot3(dx, dy, dz, dx, dy, dz);
                float dist = sqrtf(sq);
                float wx = dx, wy = dy, wz = dz;
                normalize3(wx, wy, wz);
                Ray sr = make_ray(px_, py_, pz_, wx, wy, wz);
                float Tr = light_transmittance(A, sr, dist, act, stack, stride);
                float d2 = dist * dist;
                Li0 += __fdiv_rn(Tr * lr.ix, d2);
                Li1 += __fdiv_rn(Tr * lr.iy, d2);
                Li2 += __fdiv_rn(Tr * lr.iz, d2);
            }
            float Le0 = 0.0f, Le1 = 0.0f, Le2 = 0.0f;
            PCG32 rng(derive_path_seed(px, py, k), 1);
            for (int s = 0; s < A.env_samples; ++s) {
                float xi1 = rng.uniform();
                float xi2 = rng.uniform();
                float wx, wy, wz;
                env_dir(xi1, xi2, wx, wy, wz);
                Ray er = make_ray(px_, py_, pz_, wx, wy, wz);
                float Tr = env_transmittance(A, er, act, stack, stride);
                Le0 += Tr * A.env[0];
                Le1 += Tr * A.env[1];
                Le2 += Tr * A.env[2];
            }
            const float fs = (float)A.env_samples;
            Le0 = __fdiv_rn(Le0, fs) * k4Pi;
            Le1 = __fdiv_rn(Le1, fs) * k4Pi;
            Le2 = __fdiv_rn(Le2, fs) * k4Pi;
            const float Ts = T * sigma_s;
            L0 += ((Ts * (Li0 + Le0)) * step) * kInv4Pi;
            L1 += ((Ts * (Li1 + Le1)) * step) * kInv4Pi;
            L2 += ((Ts * (Li2 + Le2)) * step) * kInv4Pi;
        }
        T *= expf(-tau_seg);
        if (T <= A.t_eps) break;
    }
    R0 = L0 + T * A.env[0];
    R1 = L1 + T * A.env[1];
    R2 = L2 + T * A.env[2];
    return kOK;
}

// ---- output addressing ----
__device__ __forceinline__ void store_px(const RenderArgs& A, uint32_t tile_local, int lx, int ly, int x, int y, float r,
                                         float g, float b) {
    if (A.packed) {
        size_t o = ((size_t)tile_local * 256u + (size_t)(ly * kTile + lx)) * 3u;
        A.out[o] = r;
        A.out[o + 1] = g;
        A.out[o + 2] = b;
    } else if (x < (int)A.width && y < (int)A.height) {
        size_t o = ((size_t)y * A.width + (size_t)x) * 3u;
        A.out[o] = r;
        A.out[o + 1] = g;
        A.out[o + 2] = b;
    }
}

__device__ __forceinline__ void tile_pixel(const RenderArgs& A, uint32_t tile_local, int lane_id, int& lx, int& ly, int& x,
                                           int& y) {
    // 256 threads: wave w covers the 8x8 quadrant (w & 1, w >> 1) of the 16x16 tile
    int wv = lane_id >> 6, ln = lane_id & 63;
    lx = (wv & 1) * 8 + (ln & 7);
    ly = (wv >> 1) * 8 + (ln >> 3);
    uint32_t tile = A.first_tile + tile_local * A.tile_stride;
    x = (int)((tile % A.tiles_x) * kTile) + lx;
    y = (int)((tile / A.tiles_x) * kTile) + ly;
}

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so give each XCD a
// contiguous run of tiles (neighbouring tiles share BVH paths and records in that XCD's L2).
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    if (nb % 8u != 0u) return b;
    return (b % 8u) * (nb / 8u) + b / 8u;
}

template <int ACT, int BLOCK>
__global__ __launch_bounds__(BLOCK) void rm_gaussians_kernel(RenderArgs A) {
    __shared__ int s_act[ACT * BLOCK];
    __shared__ int s_stack[kStackSize * BLOCK];
    const int tid = threadIdx.x;
    const uint32_t tile_local = xcd_tile(blockIdx.x, gridDim.x);
    int lx, ly, x, y;
    tile_pixel(A, tile_local, tid, lx, ly, x, y);
    if (x >= (int)A.width || y >= (int)A.height) {
        store_px(A, tile_local, lx, ly, x, y, 0.0f, 0.0f, 0.0f);
        return;
    }
    float r = 0.0f, g = 0.0f, b = 0.0f;
    int st = A.num_prims > 0 ? march_gaussians<ACT>(A, x, y, s_act + tid, s_stack + tid, BLOCK, r, g, b)
                             : (r = A.env[0], g = A.env[1], b = A.env[2], (int)kOK);
    if (st == kOverflow) {
        uint32_t slot = atomicAdd(A.queue, 1u);
        if (slot < A.queue_cap) {
            A.queue[1 + slot] = (tile_local << 8) | (uint32_t)(ly * kTile + lx);
            return;
        }
        st = kError;
    }
    if (st == kError) {
        atomicAdd(A.counters, 1u);
        r = g = b = __builtin_nanf("");
    }
    store_px(A, tile_local, lx, ly, x, y, r, g, b);
}

template <int ACT, int BLOCK>
__global__ __launch_bounds__(BLOCK) void rm_gaussians_fallback_kernel(RenderArgs A) {
    __shared__ int s_act[ACT * BLOCK];
    __shared__ int s_stack[kStackSize * BLOCK];
    const int tid = threadIdx.x;
    const uint32_t n = min(A.queue[0], A.queue_cap);
    for (uint32_t q = blockIdx.x * BLOCK + tid; q < n; q += gridDim.x * BLOCK) {
        uint32_t id = A.queue[1 + q];
        uint32_t tile_local = id >> 8;
        int lx = (int)(id & 255u) % kTile, ly = (int)(id & 255u) / kTile;
        uint32_t tile = A.first_tile + tile_local * A.tile_stride;
        int x = (int)((tile % A.tiles_x) * kTile) + lx;
        int y = (int)((tile / A.tiles_x) * kTile) + ly;
        float r, g, b;
        int st = march_gaussians<ACT>(A, x, y, s_act + tid, s_stack + tid, BLOCK, r, g, b);
        if (st != kOK) {
            atomicAdd(A.counters, 1u);
            r = g = b = __builtin_nanf("");
        }
        store_px(A, tile_local, lx, ly, x, y, r, g, b);
    }
}

// =============================================================================================
// RayMarchingSpheres (test_integrators.h:23-135) and TestIntegrator (integrator.h:65-94).
// Sphere scenes are tiny (<= kMaxSpheresDev); events are emulated exactly as the reference
// builds them: sorted per-ray lists with the primary-active spheres inserted in front.
// =============================================================================================
constexpr int kMaxSpheresDev = 16;

struct SEvt {
    float t;
    int idx;
    int enter;
};

// Sphere::intersect (smm.h:29-39)
__device__ __forceinline__ bool sphere_hit(const SphereRecord& s, const Ray& r, float& te, float& tx) {
    float Lx = s.cx - r.ox, Ly = s.cy - r.oy, Lz = s.cz - r.oz;
    float tca = dot3(Lx, Ly, Lz, r.dx, r.dy, r.dz);
    float d2 = dot3(Lx, Ly, Lz, Lx, Ly, Lz) - tca * tca;
    float r2 = s.radius * s.radius;
    if (d2 > r2) return false;
    float thc = sqrtf(r2 - d2);
    te = tca - thc;
    tx = tca + thc;
    return tx >= 0.0f;
}

// SphereMixtureModel::intersect_events (smm.h:54-63): stable insertion sort by t (what
// std::sort does on lists this short).
__device__ __forceinline__ int sphere_events(const RenderArgs& A, const Ray& r, SEvt* ev) {
    int n = 0;
    for (int i = 0; i < A.num_prims; ++i) {
        float te, tx;
        if (!sphere_hit(A.spheres[i], r, te, tx)) continue;
        if (te >= 0.0f) ev[n++] = SEvt{te, i, 1};
        if (tx >= 0.0f) ev[n++] = SEvt{tx, i, 0};
    }
    for (int i = 1; i < n; ++i) {
        SEvt e = ev[i];
        int j = i;
        while (j > 0 && e.t < ev[j - 1].t) {
            ev[j] = ev[j - 1];
            --j;
        }
        ev[j] = e;
    }
    return n;
}

// SphereMixtureModel::transmittance_from_events (smm.h:79-103) with the primary-active spheres
// pre-inserted at t = 0 (test_integrators.h:80-85).
__device__ float sphere_transmittance(const RenderArgs& A, const Ray& r, uint32_t active, float tmax) {
    SEvt ev[2 * kMaxSpheresDev];
    int n = sphere_events(A, r, ev);
    float T = 1.0f, t_prev = 0.0f;
    uint32_t act = 0;
    // inserted events (t = 0, entering): dt = 0 -> factor exp(-0) = 1, then active
    for (int i = kMaxSpheresDev - 1; i >= 0; --i)
        if ((active >> i) & 1u) {
            if (0.0f > tmax) return T;
            float sig = 0.0f;
            for (int s = 0; s < A.num_prims; ++s)
                if ((act >> s) & 1u) sig += A.spheres[s].sigma_a + A.spheres[s].sigma_s;
            T *= expf(-sig * (0.0f - t_prev));
            act |= 1u << i;
            t_prev = 0.0f;
        }
    for (int e = 0; e < n; ++e) {
        if (ev[e].t > tmax) break;
        float dt = ev[e].t - t_prev;
        float sig = 0.0f;
        for (int s = 0; s < A.num_prims; ++s)
            if ((act >> s) & 1u) sig += A.spheres[s].sigma_a + A.spheres[s].sigma_s;
        T *= expf(-sig * dt);
        if (ev[e].enter) act |= 1u << ev[e].idx;
        else act &= ~(1u << ev[e].idx);
        t_prev = ev[e].t;
    }
    return T;
}

__device__ void march_spheres(const RenderArgs& A, int px, int py, float& R0, float& R1, float& R2) {
    const Ray ray = primary_ray(A, px, py);
    SEvt ev[2 * kMaxSpheresDev];
    int n = sphere_events(A, ray, ev);
    if (n == 0) {
        R0 = A.env[0];
        R1 = A.env[1];
        R2 = A.env[2];
        return;
    }
    const float* __restrict__ ts = A.tsteps;
    const float t_end = ev[n - 1].t;
    float T = 1.0f, L0 = 0.0f, L1 = 0.0f, L2 = 0.0f;
    uint32_t active = 0;
    int ce = 0;
    // first step that can see an active sphere: kfirst(first event)
    int k = kfirst(ts, A.num_tsteps, A.step_size, ev[0].t);
    if (k > 0) --k;
    for (; k < A.num_tsteps - 1; ++k) {
        const float t = ts[k];
        if (!(t < t_end)) break;
        while (ce < n && ev[ce].t <= t) {
            if (ev[ce].enter) active |= 1u << ev[ce].idx;
            else active &= ~(1u << ev[ce].idx);
            ++ce;
        }
        if (active == 0) continue;  // sigma = 0: no scattering, T *= exp(-0) = 1
        float sa = 0.0f, ss = 0.0f;  // smm.h:66-76
        for (int i = 0; i < A.num_prims; ++i)
            if ((active >> i) & 1u) {
                sa += A.spheres[i].sigma_a;
                ss += A.spheres[i].sigma_s;
            }
        const float px_ = ray.ox + t * ray.dx, py_ = ray.oy + t * ray.dy, pz_ = ray.oz + t * ray.dz;
        if (ss > 0.0f) {
            float Li0 = 0.0f, Li1 = 0.0f, Li2 = 0.0f;
            for (int l = 0; l < A.num_lights; ++l) {
                const LightRecord& lr = A.lights[l];
                float dx = lr.px - px_, dy = lr.py - py_, dz = lr.pz - pz_;
                float dist = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
                normalize3(dx, dy, dz);
                Ray sr = make_ray(px_, py_, pz_, dx, dy, dz);
                float Tr = sphere_transmittance(A, sr, active, dist);
                float d2 = dist * dist;
                Li0 += __fdiv_rn(Tr * lr.ix, d2);
                Li1 += __fdiv_rn(Tr * lr.iy, d2);
                Li2 += __fdiv_rn(Tr * lr.iz, d2);
            }
            float Le0 = 0.0f, Le1 = 0.0f, Le2 = 0.0f;
            PCG32 rng(derive_path_seed(px, py, k), 1);
            for (int s = 0; s < A.env_samples; ++s) {
                float xi1 = rng.uniform();
                float xi2 = rng.uniform();
                float wx, wy, wz;
                env_dir(xi1, xi2, wx, wy, wz);
                Ray er = make_ray(px_, py_, pz_, wx, wy, wz);
                float Tr = sphere_transmittance(A, er, active, INFINITY);
                Le0 += Tr * A.env[0];
                Le1 += Tr * A.env[1];
                Le2 += Tr * A.env[2];
            }
            const float fs = (float)A.env_samples;
            Le0 = __fdiv_rn(Le0, fs) * k4Pi;
            Le1 = __fdiv_rn(Le1, fs) * k4Pi;
            Le2 = __fdiv_rn(Le2, fs) * k4Pi;
            const float Ts = T * ss;
            L0 += ((Ts * (Li0 + Le0)) * A.step_size) * kInv4Pi;
            L1 += ((Ts * (Li1 + Le1)) * A.step_size) * kInv4Pi;
            L2 += ((Ts * (Li2 + Le2)) * A.step_size) * kInv4Pi;
        }
        T *= expf(-A.step_size * (sa + ss));
        if (T <= A.t_eps) break;
    }
    R0 = L0 + T * A.env[0];
    R1 = L1 + T * A.env[1];
    R2 = L2 + T * A.env[2];
}

__global__ __launch_bounds__(256) void rm_spheres_kernel(RenderArgs A) {
    const uint32_t tile_local = xcd_tile(blockIdx.x, gridDim.x);
    int lx, ly, x, y;
    tile_pixel(A, tile_local, threadIdx.x, lx, ly, x, y);
    float r = 0.0f, g = 0.0f, b = 0.0f;
    if (x < (int)A.width && y < (int)A.height) march_spheres(A, x, y, r, g, b);
    store_px(A, tile_local, lx, ly, x, y, r, g, b);
}

// TestIntegrator: magenta where the primary ray has any event, env colour elsewhere.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void hitmask_kernel(RenderArgs A, int spheres) {
    __shared__ int s_stack[kStackSize * BLOCK];
    const uint32_t tile_local = xcd_tile(blockIdx.x, gridDim.x);
    int lx, ly, x, y;
    tile_pixel(A, tile_local, threadIdx.x, lx, ly, x, y);
    float r = 0.0f, g = 0.0f, b = 0.0f;
    if (x < (int)A.width && y < (int)A.height) {
        const Ray ray = primary_ray(A, x, y);
        bool any = false;
        if (spheres) {
            for (int i = 0; i < A.num_prims && !any; ++i) {
                float te, tx;
                any = sphere_hit(A.spheres[i], ray, te, tx);
            }
        } else if (A.num_prims > 0) {
            traverse(A.nodes, ray, s_stack + threadIdx.x, BLOCK, [&](float, float) { return !any; },
                     [&](uint32_t first, uint32_t count) {
                         for (uint32_t j = first; j < first + count; ++j) {
                             GRec gg = load_rec(A.gauss, j);
                             float a, bb;
                             if (intersect(quad(gg, ray), a, bb)) any = true;
                         }
                     });
        }
        if (any) { r = 1.0f; g = 0.0f; b = 1.0f; }
        else { r = A.env[0]; g = A.env[1]; b = A.env[2]; }
    }
    store_px(A, tile_local, lx, ly, x, y, r, g, b);
}

// Slabs (rank r holds tiles r, r + nslabs, ...) -> row-major frame.
__global__ void unshuffle_kernel(const float* __restrict__ slabs, uint32_t nslabs, uint32_t tiles_per_slab,
                                 uint32_t tiles_x, uint32_t W, uint32_t H, float* __restrict__ img) {
    uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t total = (uint64_t)nslabs * tiles_per_slab * 256u;
    if (gid >= total) return;
    uint32_t p = (uint32_t)(gid % 256u);
    uint64_t tl = gid / 256u;
    uint32_t slab = (uint32_t)(tl / tiles_per_slab);
    uint32_t i = (uint32_t)(tl % tiles_per_slab);
    uint64_t tile = (uint64_t)slab + (uint64_t)i * nslabs;
    uint32_t x = (uint32_t)((tile % tiles_x) * kTile) + p % kTile;
    uint32_t y = (uint32_t)((tile / tiles_x) * kTile) + p / kTile;
    if (x >= W || y >= H) return;
    const float* s = slabs + gid * 3u;
    float* d = img + ((size_t)y * W + x) * 3u;
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
}

}  // namespace dev

// ---- launchers (host) ----
constexpr int kActFast = 16, kBlockFast = 256;
constexpr int kActFallback = 64, kBlockFallback = 64;

hipError_t launch_render(const RenderArgs& A, hipStream_t stream, int volume_type, int integrator) {
    dim3 grid(A.num_tiles);
    if (integrator == VR_TEST_HITMASK) {
        hipLaunchKernelGGL((dev::hitmask_kernel<256>), grid, dim3(256), 0, stream, A, volume_type == VR_VOLUME_SPHERES ? 1 : 0);
        return hipGetLastError();
    }
    if (volume_type == VR_VOLUME_SPHERES) {
        hipLaunchKernelGGL(dev::rm_spheres_kernel, grid, dim3(256), 0, stream, A);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((dev::rm_gaussians_kernel<kActFast, kBlockFast>), grid, dim3(kBlockFast), 0, stream, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((dev::rm_gaussians_fallback_kernel<kActFallback, kBlockFallback>), dim3(1024), dim3(kBlockFallback), 0,
                       stream, A);
    return hipGetLastError();
}

hipError_t launch_unshuffle(const float* slabs, uint32_t nslabs, uint32_t tiles_per_slab, uint32_t tiles_x, uint32_t W,
                            uint32_t H, float* img, hipStream_t stream) {
    uint64_t total = (uint64_t)nslabs * tiles_per_slab * 256u;
    if (total == 0) return hipSuccess;
    dim3 grid((unsigned)((total + 255) / 256));
    hipLaunchKernelGGL(dev::unshuffle_kernel, grid, dim3(256), 0, stream, slabs, nslabs, tiles_per_slab, tiles_x, W, H, img);
    return hipGetLastError();
}

}  // namespace vr
