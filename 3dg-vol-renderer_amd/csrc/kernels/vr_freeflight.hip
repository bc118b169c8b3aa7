// Free-flight integrators on the device:
//   FreeFlightGaussians    include/integrator.h:300-408  (single scattering, float optical-depth sum)
//   MultiScatterGaussians  include/integrator.h:532-717  (free-flight bounces, NEE, Russian roulette)
// with the ANALYTIC_PLUS_NEWTON distance solver (distance_solvers.h:25-187, gaussian.h:10-25,
// 235-297) and the unsorted shadow transmittance transmittance_up_to_BVH (gmm.h:517-578).
//
// One thread = one path (pixel, sample index si). A 256-thread workgroup is one 16x16 tile at one
// sample index, so a wave's 64 paths start from an 8x8 pixel block with the same stratum.
//
// Sortless event sweep. The reference builds every ray's full sorted event list (gmm.h:457-515)
// and walks it segment by segment. Here a ray collects, in one BVH walk, the hits overlapping the
// window [W0, inf) into a bounded per-thread buffer (ff_hit_cap entries, keyed by entry distance
// max(t0, W0)); when the buffer is full the largest key is evicted and the window is cut at the
// smallest evicted key t_cut, so the buffer holds EVERY hit that enters before t_cut. The buffer
// is sorted by key, and the sweep merges those entries with the exits of the active list
// (swap-remove order, integrator.h:470-492), producing exactly the reference's segments up to
// t_cut (t_cut itself is an event of the reference: the evicted entry). The next window starts
// at t_cut. Usual scenes need a single window.
//
// Floating point: ray generation, intersection distances and every discrete decision use the
// exact (correctly rounded, uncontracted) forms of vr_march.h. libm functions (log, erf, acos,
// sin, cos) come from the device library, so individual paths can diverge from the oracle when a
// comparison lands within an ulp; parity is per pixel on most pixels and on the image mean.
#include <algorithm>
#include <type_traits>

#include "vr_dev_common.h"

namespace vr {
namespace dev {

constexpr int kFFBlock = 256;
// The loops over the active list stay rolled (unrolled by 4, independent row loads in flight: within +-2 %, round
// 3); the event sweep recomputes F at each segment start instead of keeping it in the rows (C2 147.3 -> 141.1 ms).

// Per-thread scratch rows (global memory, [slot][thread] so a wave's lanes touch consecutive 16-B
// cells): every slot is one float4, so an insert shift, an entry or a cache read is ONE 16-B access
// instead of three or seven 4-B ones (fewer memory instructions and dependent round trips).
//   hit[slot]  = { entry key max(t0, W0), exit t1, record id (leaf order, as bits), - }
//   a0[entry]  = { P, B, 2A, den }   per active entry, cached for the bounce's ray when it enters
//   a1[entry]  = { F0, F1, t1, record id (bits) }
// (optical_depth's factors, gaussian.h:208-231: od(t_prev, t) = P * (erf((B + 2A t) / den) - F) with
// F = erf(.. t_prev ..), the same float operations as optical_depth(), so the values are bit-identical).
// F at the current segment start is F0 or F1 as `ph` says: an event writes the new F into the other
// component and flips ph, so the sweep touches every active entry once per event (one 16-B read
// and one 4-B write) and the solver still sees F at t_prev when the target is crossed.
// Work counters of the instrumented build (vr_count_work): CNT = false compiles them away.
enum { kFFPaths = 0, kFFBounces, kFFNode4, kFFNode2, kFFPrims, kFFErf, kFFNeeInline, kFFNeeQueued, kFFNumCtr };
enum { kNeeRays = 0, kNeeNode4, kNeePrims, kNeeOD };
template <bool CNT>
struct FFCount {
    __device__ __forceinline__ void add(int, uint32_t = 1) {}
};
template <>
struct FFCount<true> {
    uint32_t v[kFFNumCtr] = {};
    __device__ __forceinline__ void add(int k, uint32_t n = 1) {
#ifdef VR_DIAG_FF_CYCLES  // these slots hold phase cycles in the diagnostic build (FFScratch::lap)
        if (k == kFFErf || k == kFFNode2 || k == kFFNeeInline || k == kFFNeeQueued) return;
#endif
#ifdef VR_DIAG_FFSM  // every slot holds ff_path_sm_kernel's per-phase wave statistics in this diagnostic build
        return;
#endif
        v[k] += n;
    }
};

template <bool CNT>
struct FFScratch {
    float4* hit;
    float4* a0;
    float4* a1;
    uint32_t stride;
    int ph;  // which of a1.x / a1.y holds F at the current segment start
    [[no_unique_address]] mutable FFCount<CNT> C;
#ifdef VR_DIAG_FF_CYCLES  // diagnostic builds only (CNT = true): wave cycles per phase of a bounce, lane 0
    mutable uint64_t dt = 0;
    // (lane 0's bounces only; a lap starts at the bounce's start, so waiting for a refill is not counted)
    __device__ __forceinline__ void lap(int k) const {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        if constexpr (CNT) C.v[k] += (__lane_id() == 0u) ? (uint32_t)((now - dt) >> 4) : 0u;  // (16-cycle units)
        dt = now;
    }
    __device__ __forceinline__ void lap_start() const { dt = __builtin_amdgcn_s_memtime(); }
#else
    __device__ __forceinline__ void lap(int) const {}
    __device__ __forceinline__ void lap_start() const {}
#endif
    __device__ __forceinline__ float4& H(int i) const { return hit[(size_t)i * stride]; }
    __device__ __forceinline__ float4& A0(int i) const { return a0[(size_t)i * stride]; }
    __device__ __forceinline__ float4& A1(int i) const { return a1[(size_t)i * stride]; }
    __device__ __forceinline__ float K(int i) const { return H(i).x; }
    __device__ __forceinline__ int Rec(int i) const { return __float_as_int(A1(i).w); }  // record of active entry i
    // entry i (hit slot `slot`) becomes active at t: cache its factors (optical_depth's own ops);
    // returns its exit t1
    __device__ __forceinline__ float enter(const RenderArgs& A, int i, int slot, const Ray& r, float t) const {
        return enter_row(A, i, H(slot), r, t);
    }
    __device__ __forceinline__ float T1(int i) const { return reinterpret_cast<const float*>(a1 + (size_t)i * stride)[2]; }
    template <bool F = true>
    __device__ __forceinline__ float enter_row(const RenderArgs& A, int i, const float4 h, const Ray& r, float t) const {
        GRec g = load_rec(A.gauss, __float_as_int(h.z));
        Quad q = quad(g, r);
        float twoA = 2.0f * q.A;
        float pref = (g.density * g.norm) * sqrtf(__fdiv_rn(3.14159265358979323846f, twoA));
        float den = 2.0f * sqrtf(twoA);
        float e = expf(-0.5f * (q.Cq - __fdiv_rn(q.B * q.B, 4.0f * q.A)));
        A0(i) = make_float4(pref * e, q.B, twoA, den);
        if constexpr (F) {
            C.add(kFFErf);
            const float Fv = erff(__fdiv_rn(q.B + twoA * t, den));
            A1(i) = make_float4(Fv, Fv, h.y, h.z);
        } else {  // (the sweep recomputes F at each segment start)
            A1(i) = make_float4(0.0f, 0.0f, h.y, h.z);
        }
        return h.y;
    }
    __device__ __forceinline__ void move(int dst, int src) const {
        A0(dst) = A0(src);
        A1(dst) = A1(src);
    }
    // optical depth of active entry i on [t_prev, t]
    __device__ __forceinline__ float od_to(int i, float t) const {
        const float4 c = A0(i);
        const float4 e = A1(i);
        C.add(kFFErf);
        return c.x * (erff(__fdiv_rn(c.y + c.z * t, c.w)) - (ph ? e.y : e.x));
    }
};

// The persistent path kernels' rows of thread gt ([slot][thread]; a wave-major [wave][slot][lane] layout measured
// the same, round 5).
template <bool CNT>
__device__ __forceinline__ FFScratch<CNT> ff_thread_scratch(const RenderArgs& A, uint32_t gt) {
    return FFScratch<CNT>{A.ff_hit + gt, A.ff_act0 + gt, A.ff_act1 + gt, A.ff_threads, 0, {}};
}

// camera.h:45-53 / :64-73 for a float (u, v) (the stratified sample of integrator.h:564-568).
__device__ __forceinline__ Ray camera_ray(const RenderArgs& A, float uvx, float uvy) {
    float u, v;
    if (A.cam_type == 0) {
        u = 1.0f - uvx * 2.0f;
        v = uvy * 2.0f - 1.0f;
    } else {
        u = uvx * 2.0f - 1.0f;
        v = 1.0f - uvy * 2.0f;
    }
    float o0 = (A.cam_pos[0] + u * A.cam_right[0]) + v * A.cam_up[0];
    float o1 = (A.cam_pos[1] + u * A.cam_right[1]) + v * A.cam_up[1];
    float o2 = (A.cam_pos[2] + u * A.cam_right[2]) + v * A.cam_up[2];
    float d0, d1, d2;
    if (A.cam_type == 0) {
        d0 = A.cam_pinhole[0] - o0;
        d1 = A.cam_pinhole[1] - o1;
        d2 = A.cam_pinhole[2] - o2;
    } else {
        d0 = A.cam_view[0];
        d1 = A.cam_view[1];
        d2 = A.cam_view[2];
    }
    normalize3(d0, d1, d2);
    return make_ray(o0, o1, o2, d0, d1, d2);
}

// integrator.h:32-44: theta = 2.0f * pi (double) * xi1 rounded to float; phi = acos(1 - 2 xi2).
__device__ __forceinline__ void sample_uniform_direction(PCG32& rng, float& x, float& y, float& z) {
    float xi1 = rng.uniform();
    float xi2 = rng.uniform();
    float theta = (float)(6.283185307179586 * (double)xi1);
    float phi = acosf(1.0f - 2.0f * xi2);
    float sp = sinf(phi);
    x = sp * cosf(theta);
    y = sp * sinf(theta);
    z = cosf(phi);
}

// BVH walk over the 4-wide half-precision tree when the scene has one (half as many dependent node
// fetches per ray as the child-pair tree), else the 32-B half-precision child-pair nodes, else the
// f32 nodes. Boxes are rounded outward, so every tree yields the same hit set (every candidate gets
// the exact ellipsoid test); only the walk order among equal keys differs. A 4-wide walk that could
// overflow its LDS stack stops; `reset` then clears what the walk collected and the pair tree
// (at most one push per level) redoes it.
template <typename Prune, typename Leaf, typename Reset, typename Cnt = FFCount<false>>
__device__ __forceinline__ void walk(const RenderArgs& A, const Ray& r, int* stack, int stride, Prune prune, Leaf leaf,
                                     Reset reset, Cnt* cnt = nullptr) {
    auto on4 = [&]() {
        if (cnt) cnt->add(kFFNode4);
    };
    auto on2 = [&]() {
        if (cnt) cnt->add(kFFNode2);
    };
    if (A.hnodes4) {
        if (traverse_wide<kStackSize>(A, r, stack, stride, prune, leaf, on4)) return;
        reset();
    }
    if (A.hnodes)
        traverse<true>(A, r, stack, stride, prune, leaf, on2);
    else
        traverse<false>(A, r, stack, stride, prune, leaf, on2);
}

// gaussian.h:10-25
__device__ __forceinline__ double erfinv_approx(double x) {
    if (isnan(x)) return __builtin_nan("");
    if (x <= -1.0) return -__builtin_inf();
    if (x >= 1.0) return __builtin_inf();
    const double a = 0.14;
    double sign = (x < 0.0) ? -1.0 : 1.0;
    double ln_term = log(1.0 - x * x);
    double first = 2.0 / (3.14159265358979323846 * a) + ln_term / 2.0;
    double inside = first * first - ln_term / a;
    if (inside < 0.0) inside = 0.0;
    return sign * sqrt(sqrt(inside) - first);
}

// gaussian.h:235-297 (double)
__device__ bool solve_for_t_given_tau(const GRec& g, const Ray& r, float t0, float tb, float target_tau, float& t_out) {
    Quad q = quad(g, r);
    double Ad = (double)q.A;
    if (!(Ad > 0.0) || !isfinite(Ad)) return false;
    double B = 2.0 * (double)(q.B * 0.5f);  // q.B = 2 p.Md exactly (power-of-two scaling)
    double C = (double)q.Cq;
    double sqrtA = sqrt(Ad);
    double pref = (double)g.density * (double)g.norm * sqrt(3.14159265358979323846 / (2.0 * Ad));
    double exp_factor = exp(-0.5 * (C - (B * B) / (4.0 * Ad)));
    double denom = pref * exp_factor;
    if (!(denom > 0.0) || !isfinite(denom)) return false;
    double two_sqrt2_sqrtA = 2.0 * sqrt(2.0) * sqrtA;
    double erf_t0 = erf((B + 2.0 * Ad * (double)t0) / two_sqrt2_sqrtA);
    double target_erf = (double)target_tau / denom + erf_t0;
    const double one_eps = 1.0 - 1e-14;
    if (target_erf >= one_eps) {
        t_out = tb;
        return true;
    }
    if (target_erf <= -one_eps) {
        t_out = t0;
        return true;
    }
    if (!isfinite(target_erf)) return false;
    if (target_erf <= -1.0 || target_erf >= 1.0) return false;
    double arg_t = erfinv_approx(target_erf);
    double t_candidate = (two_sqrt2_sqrtA * arg_t - B) / (2.0 * Ad);
    if (!isfinite(t_candidate)) return false;
    if (t_candidate < (double)t0 - 1e-6) t_candidate = t0;
    if (t_candidate > (double)tb + 1e-6) t_candidate = tb;
    t_out = (float)t_candidate;
    return true;
}

// sum_i tau_i(ta, t) over the active list, in list order (distance_solvers.h:38-40, 72-78)
template <class SC>
__device__ __forceinline__ float act_tau(const RenderArgs& A, const SC& S, int m, const Ray& r, float ta, float t) {
    float s = 0.0f;  // ta is the segment start t_prev, where the cached F values were taken
#pragma unroll 1
    for (int i = 0; i < m; ++i) s += S.od_to(i, t);
    return s;
}

// distance_solvers.h:25-57
template <class SC>
__device__ float solve_bisection(const RenderArgs& A, const SC& S, int m, const Ray& r, float ta, float tb, float target) {
    float a = ta, b = tb;
    for (int i = 0; i < 15; ++i) {
        float mid = 0.5f * (a + b);
        float f = act_tau(A, S, m, r, ta, mid) - target;
        if (fabsf(f) <= 1e-6f) return mid;
        if (f < 0.0f) a = mid;
        else b = mid;
    }
    return 0.5f * (a + b);
}

// distance_solvers.h:62-127
template <class SC>
__device__ float solve_newton(const RenderArgs& A, const SC& S, int m, const Ray& r, float ta, float tb, float target) {
    const float a = ta, b = tb, tol = 1e-6f;
    float t = 0.5f * (a + b);
    for (int iter = 0; iter < 8; ++iter) {
        float f = act_tau(A, S, m, r, ta, fminf(t, b)) - target;
        if (fabsf(f) <= tol) return fminf(fmaxf(t, a), b);
        float h = fmaxf(1e-5f, (b - a) * 1e-6f);
        float tp = fminf(b, t + h);
        float fp = act_tau(A, S, m, r, ta, fminf(tp, b)) - target;
        float deriv = __fdiv_rn(fp - f, tp - t);
        if (!(deriv > 0.0f) || !isfinite(deriv) || fabsf(deriv) < 1e-12f) return solve_bisection(A, S, m, r, ta, tb, target);
        float t_next = t - __fdiv_rn(f, deriv);
        if (!isfinite(t_next) || t_next < a || t_next > b) return solve_bisection(A, S, m, r, ta, tb, target);
        if (fabsf(t_next - t) <= tol * fmaxf(1.0f, fabsf(t))) return fminf(fmaxf(t_next, a), b);
        t = t_next;
    }
    return solve_bisection(A, S, m, r, ta, tb, target);
}

// distance_solvers.h:143-187. The reference picks its solver at compile time (ANALYTIC_PLUS_NEWTON,
// :146); here A.ff_solver (VR_OPT_FF_SOLVER, wave-uniform) selects it per frame. UNIFORM (:132-137)
// draws rand01() from a non-reproducible mt19937(random_device); the device draws the textbook-PCG32
// uniform of stream 2 + bounce of the path's seed instead (the oracle does the same; documented
// deviation), leaving the path's own stream untouched as rand01() does.
enum { kSolverAnalyticNewton = 0, kSolverBisection = 1, kSolverNewton = 2, kSolverAnalyticBisection = 3, kSolverUniform = 4 };
template <class SC>
__device__ float solve_distance(const RenderArgs& A, const SC& S, int m, const Ray& r, float ta, float tb, float rem,
                                uint64_t path_seed, int bounce) {
    const int mode = A.ff_solver;
    if (mode == kSolverUniform) {
        PCG32 u(path_seed, 2u + (uint64_t)bounce);
        return ta + u.uniform_env() * (tb - ta);
    }
    if (mode == kSolverBisection) return solve_bisection(A, S, m, r, ta, tb, rem);
    if (mode == kSolverNewton) return solve_newton(A, S, m, r, ta, tb, rem);
    if (m == 1) {
        float t_an = 0.0f;
        if (solve_for_t_given_tau(load_rec(A.gauss, S.Rec(0)), r, ta, tb, rem, t_an)) return fminf(fmaxf(t_an, ta), tb);
    }
    if (mode == kSolverAnalyticBisection) return solve_bisection(A, S, m, r, ta, tb, rem);
    return solve_newton(A, S, m, r, ta, tb, rem);
}

// gmm.h:128-143
template <class SC>
__device__ float evaluate_albedo(const RenderArgs& A, const SC& S, int m, float x, float y, float z) {
    float sum = 0.0f, sum_alb = 0.0f;
#pragma unroll 1
    for (int i = 0; i < m; ++i) {
        GRec g = load_rec(A.gauss, S.Rec(i));
        float mt = mu_t(g, x, y, z);
        sum += mt;
        sum_alb += mt * g.albedo;
    }
    float a = __fdiv_rn(sum_alb, sum);
    return a < 0.0f ? 0.0f : (1.0f < a ? 1.0f : a);  // std::clamp: a NaN (0/0) passes through
}

// gmm.h:517-578: exp(-sum tau_i(max(0,t0_i), min(tmax,t1_i))), unsorted, double accumulation.
// The shadow ray only feeds a continuous quantity (Tr), so it uses the FMA-contracted quadratic and
// hardware rcp/rsq forms (vr_march.h *_fast, as the ray-march's secondary rays do); the path's own
// discrete decisions keep the exact forms.
template <class Cnt = FFCount<false>>
__device__ __forceinline__ void shadow_leaf(const RenderArgs& A, const Ray& r, float tmax, uint32_t first, uint32_t count,
                                            double& sum, Cnt* cnt = nullptr) {
    for (uint32_t j = first; j < first + count; ++j) {
        if (cnt) cnt->add(kNeePrims);
        GRec g = load_rec(A.gauss, (int)j);
        Quad q = quad_fast(g, r);
        float t0, t1;
        if (!intersect_fast(q, t0, t1)) continue;
        float a = fmaxf(0.0f, t0);
        float b = fminf(tmax, t1);
        if (b > a) {
            if (cnt) cnt->add(kNeeOD);
            sum += (double)optical_depth_fast(g, q, a, b);
        }
    }
}
__device__ __forceinline__ float shadow_prune_lim(float tmax) { return tmax + kTPad * (1.0f + fminf(tmax, 1e30f)); }

__device__ __forceinline__ float transmittance_up_to(const RenderArgs& A, const Ray& r, float tmax, int* stack, int stride) {
    if (!(tmax > 0.0f)) return 1.0f;
#ifdef VR_DIAG_FF_NO_NEE  // diagnostic builds only (cost attribution): the shadow walk is skipped
    return 0.5f;
#endif
    double sum = 0.0;
    const float lim = shadow_prune_lim(tmax);
    walk(
        A, r, stack, stride, [&](float tmin, float) { return tmin <= lim; },
        [&](uint32_t first, uint32_t count) {
            shadow_leaf(A, r, tmax, first, count, sum);
            return sum < 104.0;  // expf(-x) == 0 in f32 for x >= 104: later terms cannot change Tr
        },
        [&]() { sum = 0.0; });
    return expf(-(float)sum);
}

// While-while form of the 4-wide walk for the hit collection (the shadow-ray kernel's scheme): each
// wave iteration is a NODE iteration (up to kCollectSteps node steps per lane, leaf children into an
// 8-entry LDS FIFO near-first) or a PRIM iteration (up to kCollectSteps Gaussians per lane), whichever
// more of the wave's walking lanes can use. Leaves come out of the FIFO in the order the walk reaches
// them, so ties among equal keys keep the walk order; `prune` reads the buffer's current bounds, which
// may lag the node steps by a few primitives (it then prunes less, never more). Returns false if the
// stack could overflow (the caller redoes the walk on the pair tree).
#ifndef VR_COLLECT_STEPS
#define VR_COLLECT_STEPS 6  // node steps / primitives per lane per wave iteration of the collection walk (round 6 A/B,
                            // 4 / 6 / 8: C4 multi-scatter 81.8 / 82.9 / 81.9, C5 260.8 / 263.0 / - Mpaths/s)
#endif
#ifndef VR_FFSM_COLLECT_STEPS
#define VR_FFSM_COLLECT_STEPS 8  // the same in the phase-scheduled kernel's COLLECT phase (C2: 4 / 6 / 8 -> 33.5 / 33.6 / 34.1)
#endif
constexpr int kCollectQueue = 8, kCollectSteps = VR_COLLECT_STEPS, kSmCollectSteps = VR_FFSM_COLLECT_STEPS;
template <typename Prune, typename Prim, typename Cnt>
__device__ __forceinline__ bool collect_walk(const RenderArgs& A, const Ray& r0, int* stack, int* ring, Prune prune,
                                             Prim prim, Cnt* cnt) {
    float ox = r0.ox, oy = r0.oy, oz = r0.oz;
    node_space<true>(A, ox, oy, oz);
    auto inv = [&](float d) {
        d *= A.hn_scale;
        return __frcp_rn(fabsf(d) > 1e-30f ? d : copysignf(1e-30f, d));
    };
    const float ix = inv(r0.dx), iy = inv(r0.dy), iz = inv(r0.dz);
    const float oxi = ox * ix, oyi = oy * iy, ozi = oz * iz;
    int sp = 0, node = 0, qh = 0, qn = 0;
    uint32_t j = 0, end = 0;
    bool ovf = false;
    for (;;) {
        const bool has_prim = j < end || qn > 0;
        const bool can_node = node >= 0 && qn <= kCollectQueue - 4;
        const uint64_t bp = __ballot(has_prim), bn = __ballot(can_node);
        if ((bp | bn) == 0ull) break;
        const int np = __popcll(bp), nn = __popcll(bn);
        if (nn == 0 || (np > 0 && np >= nn)) {  // PRIM iteration
            bool go = has_prim;
            for (int k = 0; k < kCollectSteps; ++k) {
                if (go) {
                    if (j == end) {
                        const int32_t ref = ring[qh * kFFBlock];
                        qh = (qh + 1) & (kCollectQueue - 1);
                        --qn;
                        j = leaf_first(ref);
                        end = j + leaf_count(ref);
                    }
                    prim(j);
                    ++j;
                }
                go = go && (j < end || qn > 0);
            }
        } else {  // NODE iteration
            bool go = can_node;
            for (int k = 0; k < kCollectSteps; ++k) {
                if (go) {
                    if (cnt) cnt->add(kFFNode4);
                    float key[4];
                    int32_t kr[4];
                    wide_children(A, node, ix, iy, iz, oxi, oyi, ozi, prune, key, kr);
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (kr[i] < 0) {
                            ring[((qh + qn) & (kCollectQueue - 1)) * kFFBlock] = kr[i];
                            ++qn;
                        }
                    int first = -1;
                    int32_t next = 0;
#pragma unroll
                    for (int i = 3; i >= 0; --i) {
                        first = kr[i] > 0 ? i : first;
                        next = kr[i] > 0 ? kr[i] : next;
                    }
                    if (sp + 3 > kStackSize) {
                        ovf = true;
                        node = -1;
                        qn = 0;
                        j = end;
                    } else {
#pragma unroll
                        for (int i = 3; i >= 0; --i)
                            if (kr[i] > 0 && i != first) stack[(sp++) * kFFBlock] = kr[i];
                        if (first >= 0) node = next;
                        else if (sp > 0) node = stack[(--sp) * kFFBlock];
                        else node = -1;
                    }
                }
                go = go && node >= 0 && qn <= kCollectQueue - 4;
            }
        }
    }
    return !ovf;
}

// RECORD_PIXEL_GAUSSIANS (integrator.h:616-644): mark, for pixel p, every Gaussian whose events on
// this ray lie at or before t_scatter + 1e-6 (entries t0 <= lim), or every Gaussian the ray hits
// when it did not scatter. Bits are per original scene index: word (g >> 5) of pixel p.
__device__ void record_hits(const RenderArgs& A, const Ray& r, float lim, uint32_t p, int* stack, int stride) {
    auto prune = [&](float tmin, float) { return tmin <= lim + kTPad * (1.0f + fminf(lim, 1e30f)); };
    auto prim = [&](uint32_t j) {
        GRec g = load_rec(A.gauss, (int)j);
        float t0, t1;
        if (!intersect(quad(g, r), t0, t1)) return;
        if (!(t0 <= lim)) return;
        const uint32_t o = A.gauss_order[j];
        atomicOr(A.rec_bits + (size_t)(o >> 5) * A.rec_npix + p, 1u << (o & 31u));
    };
    auto leaf = [&](uint32_t first, uint32_t count) {
        for (uint32_t j = first; j < first + count; ++j) prim(j);
        return true;
    };
    // while-while walk (the collection's); the pair tree redoes a walk whose stack could overflow
    // (marking again is idempotent)
    if (A.hnodes4 == nullptr || !collect_walk(A, r, stack, stack + kStackSize * stride, prune, prim, (FFCount<false>*)nullptr)) {
        if (A.hnodes) traverse<true>(A, r, stack, stride, prune, leaf);
        else traverse<false>(A, r, stack, stride, prune, leaf);
    }
}

// derive_path_seed(x, y, si) of path `out` of the launch (the numbering of ff_start).
__device__ __forceinline__ uint64_t ff_path_seed(const RenderArgs& A, uint32_t out) {
    const uint32_t b = out / kFFBlock, lane_id = out % kFFBlock;
    int lx, ly, x, y;
    tile_pixel(A, A.ff_tile_base + b / A.ff_nsb, (int)lane_id, lx, ly, x, y);
    return derive_path_seed(x, y, (int)(A.ff_si0 + b % A.ff_nsb));
}

// Free-flight distance along r for target optical depth `target` (integrator.h:330-360 for
// MULTI = false with a float sum, :422-498 for MULTI = true with a double sum). Returns t >= 0,
// -1 (no scatter before the last event) or -2 (a per-thread capacity was exceeded). On return
// with t >= 0 the active list holds the critical segment's Gaussians (count in m).
template <bool MULTI, class SC>
__device__ float free_flight_distance(const RenderArgs& A, SC& S, const Ray& r, float target, int& m, int* stack,
                                      int stride, uint32_t path, int bounce) {
    using Acc = typename std::conditional<MULTI, double, float>::type;
    Acc acc = 0;
    float t_prev = 0.0f;
    float W0 = 0.0f;
    // Window capacity starts small (most scatters happen within the first few events) and doubles
    // after every window without a scatter, or when the overlap at W0 does not fit, up to ff_hit_cap.
    int cap = A.ff_hit_cap0;
    for (;;) {
        // ---- collect the hits overlapping [W0, inf): the cap smallest entry keys, kept sorted ----
        // The walk is near-first; once the buffer is full, subtrees starting beyond its largest key
        // are skipped (their hits could only be evicted), and the window is then cut at that key.
        int n = 0;
        float t_cut = INFINITY;
        float kfull = INFINITY;  // largest kept key while the buffer is full
        auto prune = [&](float tmin, float tmax) {
            if (tmax < W0 - kTPad * (1.0f + W0)) return false;
            const float lim = fminf(t_cut, kfull);
            return !(tmin > lim + kTPad * (1.0f + fminf(lim, 1e30f)));
        };
        auto prim = [&](uint32_t j) {
            S.C.add(kFFPrims);
            GRec g = load_rec(A.gauss, (int)j);
            float t0, t1;
            if (!intersect(quad(g, r), t0, t1)) return;
            if (!(t0 <= t1)) return;  // NaN distances (degenerate covariance): no event
            if (W0 > 0.0f && !(t1 > W0)) return;
            const float key = fmaxf(t0, W0);
            if (key >= t_cut) return;
            if (n == cap) {
                if (key >= kfull) {  // would be the largest: not kept
                    t_cut = fminf(t_cut, key);
                    return;
                }
                t_cut = fminf(t_cut, kfull);  // evict the largest
                --n;
            }
            int p = n;  // sorted insert after equal keys (walk order among ties)
            while (p > 0) {
                const float4 prev = S.H(p - 1);
                if (!(prev.x > key)) break;
                S.H(p) = prev;
                --p;
            }
            S.H(p) = make_float4(key, t1, __int_as_float((int)j), 0.0f);
            ++n;
            if (n == cap) kfull = S.K(n - 1);
        };
        auto leaf = [&](uint32_t first, uint32_t count) {
            for (uint32_t j = first; j < first + count; ++j) prim(j);
            return true;
        };
        auto reset = [&]() {
            n = 0;
            t_cut = kfull = INFINITY;
        };
        S.lap(kFFErf);  // (diagnostic builds: bounce setup / window bookkeeping, with the rest of the bounce)
        if (A.hnodes4 == nullptr || !collect_walk(A, r, stack, stack + kStackSize * kFFBlock, prune, prim, &S.C)) {
            reset();  // pair tree (at most one push per level; no 4-wide tree, or its stack could overflow)
            auto on2 = [&]() { S.C.add(kFFNode2); };
            if (A.hnodes) traverse<true>(A, r, stack, stride, prune, leaf, on2);
            else traverse<false>(A, r, stack, stride, prune, leaf, on2);
        }
        // a buffer that filled ends the window at its largest kept key (subtrees skipped while full hold
        // only larger keys; whether one was skipped depends on the wave's NODE/PRIM schedule, so the cut must not)
        S.lap(kFFNode2);  // (diagnostic builds: hit collection)
        if (n == cap) t_cut = fminf(t_cut, S.K(n - 1));
        while (n > 0 && S.K(n - 1) >= t_cut) --n;  // entries past the window (t_cut fell after they were kept)
        if (t_cut <= W0) {  // more than cap Gaussians overlap at W0: no progress possible at this cap
            if (cap >= A.ff_hit_cap) return -2.0f;
            cap = min(2 * cap, A.ff_hit_cap);
            continue;
        }
        if (n == 0 && t_cut == INFINITY) return -1.0f;
        // ---- sweep the window's events (integrator.h:438-495) ----
        // The active list's next exit (the first entry with the smallest t1, as the reference's
        // scan finds it) is carried from event to event: the pass that integrates the segment also
        // finds the smallest t1 of the list as it will be after this event (entry appended, or the
        // exiting entry swap-removed), so each event reads every active entry once.
        int i = 0;
        m = 0;
        float next_exit = INFINITY;
        int exit_pos = -1;
        for (;;) {
            const float4 hn = i < n ? S.H(i) : make_float4(INFINITY, 0.0f, 0.0f, 0.0f);  // (the entry's row, once)
            const float next_entry = hn.x;
            float t_evt = fminf(next_entry, next_exit);
            const bool window_end = t_cut <= t_evt;
            if (window_end) t_evt = t_cut;
            if (t_evt == INFINITY) {  // past the last event: no scatter (integrator.h:362-366)
                S.lap(kFFNeeInline);
                return -1.0f;
            }
            const bool is_entry = next_entry <= next_exit;
            float nx = INFINITY;  // smallest t1 after the event, and its position in the list then
            int npos = -1;
            Acc seg = 0;
            // F at the segment start recomputed (the same float operations as the cached value), so the
            // sweep reads 20 B per active entry (factors and exit) and writes nothing; the next entry's
            // read is in flight while this one is evaluated
            float4 cn = m > 0 ? S.A0(0) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            float tn = m > 0 ? S.T1(0) : 0.0f;
#pragma unroll 1
            for (int a = 0; a < m; ++a) {
                const float4 c = cn;
                const float t1a = tn;
                if (a + 1 < m) {
                    cn = S.A0(a + 1);
                    tn = S.T1(a + 1);
                }
                S.C.add(kFFErf);
                const float f1 = erff(__fdiv_rn(c.y + c.z * t_evt, c.w));
                const float f0 = erff(__fdiv_rn(c.y + c.z * t_prev, c.w));
                seg += (Acc)(c.x * (f1 - f0));
                int pp = a;  // position after a swap-remove of exit_pos
                if (!is_entry && a == m - 1) pp = exit_pos;
                const bool gone = !is_entry && a == exit_pos;
                if (!gone && (t1a < nx || (t1a == nx && pp < npos))) {
                    nx = t1a;
                    npos = pp;
                }
            }
            if (acc + seg > (Acc)target) {
                S.ph = 0;  // the solver reads F at the segment start from .x
                for (int a = 0; a < m; ++a) {
                    const float4 c = S.A0(a);
                    S.A1(a).x = erff(__fdiv_rn(c.y + c.z * t_prev, c.w));
                }
                float rem = (float)((Acc)target - acc);
                S.lap(kFFNeeInline);  // (diagnostic builds: event sweep)
                const uint64_t useed = A.ff_solver == kSolverUniform ? ff_path_seed(A, path) : 0ull;
                const float ts = solve_distance(A, S, m, r, t_prev, t_evt, rem, useed, bounce);
                S.lap(kFFNeeQueued);  // (diagnostic builds: distance solver)
                return ts;
            }
            acc += seg;
            t_prev = t_evt;
            if (window_end) break;
            if (is_entry) {
                if (m >= A.ff_act_cap) return -2.0f;
                const float t1n = S.template enter_row<false>(A, m, hn, r, t_evt);
                ++i;
                if (t1n < nx) {  // ties: the earlier position stays first
                    nx = t1n;
                    npos = m;
                }
                ++m;
            } else {
                S.move(exit_pos, m - 1);
                --m;
            }
            next_exit = nx;
            exit_pos = npos;
        }
        S.lap(kFFNeeInline);
        W0 = t_cut;
        cap = min(2 * cap, A.ff_hit_cap);
    }
}

// Deferred NEE: queue the shadow ray r (tmax: the light distance, +inf for the environment; li: the
// light, -1 the environment) with its weight m, linked after the path's previous queued ray. The
// claim is wave-aggregated (one atomic per wave). Returns false if the ray must be traced inline
// (deferral off, or the queue is full); from then on the path stays inline, so its deferred
// contributions all come before its inline ones (bounce order).
__device__ __forceinline__ bool nee_queue(const RenderArgs& A, const Ray& r, float tmax, int li, float m0, float m1,
                                          float m2, uint32_t& first, uint32_t& last, bool& defer) {
    const uint64_t mask = __ballot(defer);
    if (!defer) return false;
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
    uint32_t base = 0;
    if (rank == 0) base = atomicAdd(A.ff_nee_n, (uint32_t)__popcll(mask));
    base = __shfl(base, __ffsll((unsigned long long)mask) - 1, 64);
    const uint32_t q = base + rank;
    if (q >= A.ff_nee_cap) {
        defer = false;
        return false;
    }
    float4* e = A.ff_nee + 3 * (size_t)q;
    e[0] = make_float4(r.ox, r.oy, r.oz, tmax);
    e[1] = make_float4(r.dx, r.dy, r.dz, __uint_as_float(kFFNone));
    e[2] = make_float4(m0, m1, m2, __int_as_float(li));
    if (last != kFFNone) A.ff_nee[3 * (size_t)last + 1].w = __uint_as_float(q);
    else first = q;
    last = q;
    return true;
}

// Incident radiance of a shadow ray with transmittance Tr: I_l Tr / d^2 (integrator.h:385-388) or
// env Tr 4 pi (:390-394), in the reference's operation order.
__device__ __forceinline__ void nee_radiance(const RenderArgs& A, float Tr, int li, float dist, float& Li0, float& Li1,
                                             float& Li2) {
    if (li >= 0) {
        const LightRecord& Lt = A.lights[li];
        const float d2 = dist * dist;
        Li0 = __fdiv_rn(Tr * Lt.ix, d2);
        Li1 = __fdiv_rn(Tr * Lt.iy, d2);
        Li2 = __fdiv_rn(Tr * Lt.iz, d2);
    } else {
        Li0 = (Tr * A.env[0]) * k4Pi;
        Li1 = (Tr * A.env[1]) * k4Pi;
        Li2 = (Tr * A.env[2]) * k4Pi;
    }
}

// One path: path group b = (tile b / nsb, sample si0 + b % nsb), lane_id = pixel of the tile.
// A path between bounces: everything the bounce loop of integrator.h:560-700 carries.
struct FFPath {
    PCG32 rng;
    Ray ray;
    float tp0, tp1, tp2, L0, L1, L2;
    uint32_t first, last;  // the path's queued shadow rays
    uint32_t out;          // path index of the launch (its ff_tail slot)
    uint32_t px;           // y * W + x (recording)
    int bounce;
    bool defer, after;
};

// Path `out` = (tile b / nsb, sample si0 + b % nsb, pixel lane_id of the tile): its camera ray
// (integrator.h:560-570). Returns false (tail written) for a pixel outside the frame.
__device__ __forceinline__ bool ff_start(const RenderArgs& A, uint32_t out, FFPath& P) {
    const uint32_t b = out / kFFBlock, lane_id = out % kFFBlock;
    const uint32_t tile_local = A.ff_tile_base + b / A.ff_nsb;
    const int si = (int)(A.ff_si0 + b % A.ff_nsb);
    int lx, ly, x, y;
    tile_pixel(A, tile_local, (int)lane_id, lx, ly, x, y);
    if (!(x < (int)A.width && y < (int)A.height)) {
        A.ff_tail[out] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(kFFNone));
        return false;
    }
    P.rng = PCG32(derive_path_seed(x, y, si), 1);
    const int n = A.ff_n;
    const int sx = si % n, sy = si / n;
    float xi = P.rng.uniform();
    float u = __fdiv_rn((float)x + __fdiv_rn((float)sx + xi, (float)n), (float)A.width);
    xi = P.rng.uniform();
    float v = __fdiv_rn((float)y + __fdiv_rn((float)sy + xi, (float)n), (float)A.height);
    P.ray = camera_ray(A, u, v);
    P.tp0 = P.tp1 = P.tp2 = 1.0f;
    P.L0 = P.L1 = P.L2 = 0.0f;
    P.first = P.last = kFFNone;
    P.out = out;
    P.px = (uint32_t)y * A.width + (uint32_t)x;
    P.bounce = 0;
    P.defer = A.ff_nee_cap > 0;
    P.after = false;
    return true;
}

// One bounce of path P (integrator.h:572-700). Returns false once the path is complete (its
// radiance written to ff_tail: the queued contributions in bounce order, then L if `after`).
template <bool MULTI, class SC>
__device__ __forceinline__ bool ff_bounce(const RenderArgs& A, SC& S, int* stack, FFPath& P) {
    bool done = false;
    int m = 0;
    S.lap_start();
    const float target = -logf(1.0f - P.rng.uniform());
    S.C.add(kFFBounces);
    const float ts = free_flight_distance<MULTI>(A, S, P.ray, target, m, stack, kFFBlock, P.out, P.bounce);
    if (MULTI && A.rec_bits && ts != -2.0f) record_hits(A, P.ray, ts >= 0.0f ? ts + 1e-6f : INFINITY, P.px, stack, kFFBlock);
    if (ts == -2.0f && A.ff_fbq != nullptr) {  // over the hit-buffer capacity: the whole path re-runs
        const uint32_t q = atomicAdd(A.ff_fbq, 1u);        // in ff_fallback_kernel with larger rows
        atomicAdd(A.counters + 2, 1u);                      // vr_render_stats.fallback_pixels (whole frame)
        if (q < A.ff_fbq_cap) {
            A.ff_fbq[1 + q] = P.out;
            A.ff_tail[P.out] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(kFFNone));  // overwritten there
            return false;
        }
    }
    if (ts == -2.0f || P.bounce >= A.ff_max_bounces) {
        P.L0 = P.L1 = P.L2 = __builtin_nanf("");
        P.after = true;
        atomicAdd(A.counters, 1u);
        done = true;
    } else if (ts < 0.0f) {  // no event, or no scatter before the last event: environment
        P.L0 += P.tp0 * A.env[0];
        P.L1 += P.tp1 * A.env[1];
        P.L2 += P.tp2 * A.env[2];
        P.after |= P.first != kFFNone;
        done = true;
    } else {
        const float px = P.ray.ox + ts * P.ray.dx, py = P.ray.oy + ts * P.ray.dy, pz = P.ray.oz + ts * P.ray.dz;
        const float albedo = evaluate_albedo(A, S, m, px, py, pz);
        // NEE (integrator.h:380-399 / 650-687): a light (distance-bounded) or environment shadow ray
        const int nl = A.num_lights;
        const bool is_env = P.rng.uniform() < __fdiv_rn(1.0f, (float)(nl + 1));
        int li = -1;
        float dist = INFINITY;
        Ray sr;
        if (!is_env) {
            li = (int)(P.rng.uniform() * (float)nl);
            const LightRecord& Lt = A.lights[li];
            float wx = Lt.px - px, wy = Lt.py - py, wz = Lt.pz - pz;
            dist = sqrtf(dot3(wx, wy, wz, wx, wy, wz));
            normalize3(wx, wy, wz);
            sr = make_ray(px, py, pz, wx, wy, wz);
        } else {
            float wx, wy, wz;
            sample_uniform_direction(P.rng, wx, wy, wz);
            sr = make_ray(px, py, pz, wx, wy, wz);
        }
        const float w = (albedo * kInv4Pi) * (float)(nl + 1);
        // the contribution is m * Li: L += (tp * w) * Li (integrator.h:681-687), L = w * Li (:396-399)
        const float m0 = MULTI ? P.tp0 * w : w, m1 = MULTI ? P.tp1 * w : w, m2 = MULTI ? P.tp2 * w : w;
        const bool queued = nee_queue(A, sr, dist, li, m0, m1, m2, P.first, P.last, P.defer);
        S.C.add(queued ? kFFNeeQueued : kFFNeeInline);
        if (!queued) {
            float Li0, Li1, Li2;
            nee_radiance(A, transmittance_up_to(A, sr, dist, stack, kFFBlock), li, dist, Li0, Li1, Li2);
            P.after |= P.first != kFFNone;
            if constexpr (!MULTI) {
                P.L0 = m0 * Li0;
                P.L1 = m1 * Li1;
                P.L2 = m2 * Li2;
            } else {
                P.L0 += m0 * Li0;
                P.L1 += m1 * Li1;
                P.L2 += m2 * Li2;
            }
        }
        if constexpr (!MULTI) {
            done = true;
        } else {
            P.tp0 *= albedo;
            P.tp1 *= albedo;
            P.tp2 *= albedo;
            if (P.bounce >= A.ff_min_bounces) {  // integrator.h:691-695
                float rr = fminf(fmaxf(P.tp0, fmaxf(P.tp1, P.tp2)), 0.9f);
                if (P.rng.uniform() > rr) {
                    done = true;
                } else {
                    P.tp0 = __fdiv_rn(P.tp0, rr);
                    P.tp1 = __fdiv_rn(P.tp1, rr);
                    P.tp2 = __fdiv_rn(P.tp2, rr);
                }
            }
            if (!done) {
                float nx, ny, nz;
                sample_uniform_direction(P.rng, nx, ny, nz);
                P.ray = make_ray(px, py, pz, nx, ny, nz);
                ++P.bounce;
            }
        }
    }
    if (done) A.ff_tail[P.out] = make_float4(P.L0, P.L1, P.L2, __uint_as_float(P.first | (P.after ? kFFTailAfter : 0u)));
    S.lap(kFFErf);  // (diagnostic builds: the rest of the bounce — albedo, next-event ray, roulette, direction)
    return !done;
}

// Persistent: a grid of resident waves; every lane follows one path a bounce per wave iteration and,
// once its path is complete, starts the next unclaimed path of the launch (claimed per wave when
// kFFRefill lanes are idle), so a wave never waits for its longest path. Launch bounds: 4 waves/SIMD
// (128 VGPRs, some spills) measured faster than 2, 3 and 5.
#ifndef VR_FF_WAVES
#define VR_FF_WAVES 4  // waves per SIMD of the path kernel (launch bounds; the grid fills them)
#endif
// CNT: the instrumented build (vr_count_work) counts its work into A.work[0..7].
#ifndef VR_FF_REFILL
#define VR_FF_REFILL 16  // idle lanes of a wave that trigger its path refill
#endif
template <bool MULTI, bool CNT = false>
__global__ void __launch_bounds__(kFFBlock, VR_FF_WAVES) ff_path_kernel(RenderArgs A) {
    __shared__ int s_stack[(kStackSize + kCollectQueue) * kFFBlock];  // walk stack + the walks' leaf FIFO
    int* stack = s_stack + threadIdx.x;
    const uint32_t gt = blockIdx.x * kFFBlock + threadIdx.x;
    FFScratch<CNT> S = ff_thread_scratch<CNT>(A, gt);
    const uint32_t lane = threadIdx.x & 63u;
    FFPath P{PCG32(0, 1)};
    bool live = false, exhausted = false;
    for (;;) {
        const uint64_t idle = __ballot(!live);
        if (!exhausted && (idle == ~0ull || __popcll(idle) >= VR_FF_REFILL)) {
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(A.ff_next, (unsigned long long)__popcll(idle));
            base = __shfl(base, 0, 64);
            exhausted = base + (unsigned long long)__popcll(idle) >= A.ff_total;
            if (!live) {
                const unsigned long long pid =
                    base + __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                if (pid < A.ff_total) {
                    S.C.add(kFFPaths);
                    live = ff_start(A, (uint32_t)pid, P);
                }
            }
        }
        if (!__any(live)) {
            if (exhausted) break;
            continue;
        }
        if (live) live = ff_bounce<MULTI>(A, S, stack, P);
    }
    if constexpr (CNT) {
        Ctr c{};
        for (int i = 0; i < kFFNumCtr; ++i) c.v[i] = S.C.v[i];
        flush_counters(A.work, c);
    }
}

// Phase-scheduled persistent path kernel. ff_path_kernel runs a whole bounce per wave iteration, so a
// wave waits at every phase for its slowest lane (the hit collection of one lane's second window, the
// event sweep of the lane with the most events, the shading of the lanes that scattered). Here every
// lane carries its path's bounce as a state (COLLECT: the resumable while-while walk of the window's hit
// collection; SWEEP: the window's events, one (or a budget of) per iteration; SHADE: the distance solver,
// the albedo and the rest of the bounce), and each wave iteration runs the ONE phase most of the wave's
// lanes are in, with those lanes only. Every path runs ff_bounce's operations in ff_bounce's order (the
// same RNG draws, sums and decisions), so frames are the persistent kernel's, bit for bit.
#ifndef VR_FFSM_EVENT_BUDGET
#define VR_FFSM_EVENT_BUDGET 24  // active-entry evaluations a lane may spend on events per SWEEP iteration (0: one event)
#endif
// The sweep reads an entry's row once and the next active entry's rows one ahead, and recomputes F at each segment
// start instead of keeping it in the rows. (Measured and not kept: the PRIM iterations reading the next Gaussian one
// step ahead, 134.8 vs 134.3 ms at C2.)
#ifndef VR_FFSM_SHADE_MIN
#define VR_FFSM_SHADE_MIN 20  // SHADE runs when it has the most lanes and at least this many (or nothing else is left)
#endif
#ifndef VR_FFSM_WAVES
#define VR_FFSM_WAVES 4  // waves per SIMD of the phase-scheduled path kernel (launch bounds)
#endif
enum : int { kSmIdle = 0, kSmCollect = 1, kSmSweep = 2, kSmShade = 3 };
template <bool MULTI, bool CNT = false>
__global__ void __launch_bounds__(kFFBlock, VR_FFSM_WAVES) ff_path_sm_kernel(RenderArgs A) {
    using Acc = typename std::conditional<MULTI, double, float>::type;
    __shared__ int s_stack[(kStackSize + kCollectQueue) * kFFBlock];  // walk stack + the walks' leaf FIFO
    int* stack = s_stack + threadIdx.x;
    int* ring = stack + kStackSize * kFFBlock;
    const uint32_t gt = blockIdx.x * kFFBlock + threadIdx.x;
    FFScratch<CNT> S = ff_thread_scratch<CNT>(A, gt);
    const uint32_t lane = threadIdx.x & 63u;
    FFPath P{PCG32(0, 1)};
    int phase = kSmIdle;
    bool exhausted = false;
    // the bounce (free_flight_distance's state across windows)
    float target = 0.0f, t_prev = 0.0f, W0 = 0.0f;
    Acc acc = 0;
    int cap = 0;
    // the window's hit collection (ffs_collect_kernel's walk state); in SHADE, t_cut holds ts (m < 0) or
    // the scatter segment's end t_evt, and kfull the target left on that segment
    int n = 0, sp = 0, node = -1, qh = 0, qn = 0;
    float t_cut = INFINITY, kfull = INFINITY, klast = 0.0f;
    bool redo = false;
    uint32_t j = 0, end = 0;
    // the window's event sweep
    int i = 0, m = 0, exit_pos = -1;
    float next_exit = INFINITY;
    auto begin_window = [&]() {
        n = 0;
        t_cut = kfull = INFINITY;
        sp = 0;
        node = 0;
        qh = qn = 0;
        j = end = 0;
        redo = A.hnodes4 == nullptr;  // no 4-wide tree: the pair-tree walk at once
        phase = kSmCollect;
    };
    auto begin_bounce = [&]() {  // ff_bounce's start: the target draw, window 0 from t = 0
        target = -logf(1.0f - P.rng.uniform());
        S.C.add(kFFBounces);
        acc = 0;
        t_prev = W0 = 0.0f;
        cap = A.ff_hit_cap0;
        begin_window();
    };
    auto to_shade = [&](float ts) {
        m = -1;
        t_cut = ts;
        phase = kSmShade;
    };
    auto prune = [&](float tmin, float tmax) {
        if (tmax < W0 - kTPad * (1.0f + W0)) return false;
        const float lim = fminf(t_cut, kfull);
        return !(tmin > lim + kTPad * (1.0f + fminf(lim, 1e30f)));
    };
    auto prim_g = [&](uint32_t jj, const GRec& g) {  // free_flight_distance's insertion, term for term
        S.C.add(kFFPrims);
        float t0, t1;
        if (!intersect(quad(g, P.ray), t0, t1)) return;
        if (!(t0 <= t1)) return;
        if (W0 > 0.0f && !(t1 > W0)) return;
        const float key = fmaxf(t0, W0);
        if (key >= t_cut) return;
        if (n == cap) {
            if (key >= kfull) {
                t_cut = fminf(t_cut, key);
                return;
            }
            t_cut = fminf(t_cut, kfull);
            --n;
            if (n > 0) klast = S.K(n - 1);  // (the evicted entry was the largest)
        }
        // klast = the largest kept key (the last row): an entry in walk order past it is appended without
        // reading the rows back (the rows live in global memory: a read there is a dependent round trip)
        int p = n;
        if (n > 0 && klast > key) {
            while (p > 0) {
                const float4 prev = S.H(p - 1);
                if (!(prev.x > key)) break;
                S.H(p) = prev;
                --p;
            }
        } else {
            klast = key;
        }
        S.H(p) = make_float4(key, t1, __int_as_float((int)jj), 0.0f);
        ++n;
        if (n == cap) kfull = klast;
    };
    auto prim = [&](uint32_t jj) { prim_g(jj, load_rec(A.gauss, (int)jj)); };
    for (;;) {
        const uint64_t idle = __ballot(phase == kSmIdle);
        if (!exhausted && (idle == ~0ull || __popcll(idle) >= VR_FF_REFILL)) {
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(A.ff_next, (unsigned long long)__popcll(idle));
            base = __shfl(base, 0, 64);
            exhausted = base + (unsigned long long)__popcll(idle) >= A.ff_total;
            if (phase == kSmIdle) {
                const unsigned long long pid =
                    base + __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                if (pid < A.ff_total) {
                    S.C.add(kFFPaths);
                    if (ff_start(A, (uint32_t)pid, P)) begin_bounce();
                }
            }
        }
        const int nc = __popcll(__ballot(phase == kSmCollect)), ns = __popcll(__ballot(phase == kSmSweep)),
                  nh = __popcll(__ballot(phase == kSmShade));
        if (nc + ns + nh == 0) {
            if (exhausted) break;
            continue;
        }
        const bool shade_now = nh >= VR_FFSM_SHADE_MIN ? (nh >= ns && nh >= nc) : (ns + nc == 0);
#ifdef VR_DIAG_FFSM  // (CNT builds) lane 0 of each wave: cycles/16 of each phase [0..2], its iterations [3..5], and the
        // lanes it ran with, COLLECT [6] and SWEEP [7] (SHADE's are the bounces)
        // (VR_DIAG_FFSM=2: cycles/16 of NODE, PRIM, SWEEP, SHADE iterations [0..3] and their counts [4..7])
        const int dphase = shade_now ? 2 : (ns >= nc ? 1 : 0);
        const uint64_t dt0 = __builtin_amdgcn_s_memtime();
        bool dnode = false;
#endif
        if (shade_now) {
            // ---- SHADE: ff_bounce after free_flight_distance, term for term ----
            if (phase == kSmShade) {
                float ts = t_cut;
                const int ma = m;
                if (ma >= 0) {  // the scatter lies in [t_prev, t_cut] with kfull of the target left
                    S.ph = 0;  // the solver reads F at the segment start from .x
                    for (int a = 0; a < ma; ++a) {
                        const float4 c = S.A0(a);
                        reinterpret_cast<float*>(&S.A1(a))[0] = erff(__fdiv_rn(c.y + c.z * t_prev, c.w));
                    }
                    const uint64_t useed = A.ff_solver == kSolverUniform ? ff_path_seed(A, P.out) : 0ull;
                    ts = solve_distance(A, S, ma, P.ray, t_prev, t_cut, kfull, useed, P.bounce);
                }
                bool done = false, requeued = false;
                if (MULTI && A.rec_bits && ts != -2.0f)
                    record_hits(A, P.ray, ts >= 0.0f ? ts + 1e-6f : INFINITY, P.px, stack, kFFBlock);
                if (ts == -2.0f && A.ff_fbq != nullptr) {  // over the hit-buffer capacity: the whole path re-runs
                    const uint32_t q = atomicAdd(A.ff_fbq, 1u);  // in ff_fallback_kernel with larger rows
                    atomicAdd(A.counters + 2, 1u);
                    if (q < A.ff_fbq_cap) {
                        A.ff_fbq[1 + q] = P.out;
                        A.ff_tail[P.out] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(kFFNone));
                        requeued = true;
                    }
                }
                if (requeued) {
                    done = true;
                } else if (ts == -2.0f || P.bounce >= A.ff_max_bounces) {
                    P.L0 = P.L1 = P.L2 = __builtin_nanf("");
                    P.after = true;
                    atomicAdd(A.counters, 1u);
                    done = true;
                } else if (ts < 0.0f) {  // no event, or no scatter before the last event: environment
                    P.L0 += P.tp0 * A.env[0];
                    P.L1 += P.tp1 * A.env[1];
                    P.L2 += P.tp2 * A.env[2];
                    P.after |= P.first != kFFNone;
                    done = true;
                } else {
                    const float px = P.ray.ox + ts * P.ray.dx, py = P.ray.oy + ts * P.ray.dy, pz = P.ray.oz + ts * P.ray.dz;
                    const float albedo = evaluate_albedo(A, S, ma, px, py, pz);
                    const int nl = A.num_lights;
                    const bool is_env = P.rng.uniform() < __fdiv_rn(1.0f, (float)(nl + 1));
                    int li = -1;
                    float dist = INFINITY;
                    Ray sr;
                    if (!is_env) {
                        li = (int)(P.rng.uniform() * (float)nl);
                        const LightRecord& Lt = A.lights[li];
                        float wx = Lt.px - px, wy = Lt.py - py, wz = Lt.pz - pz;
                        dist = sqrtf(dot3(wx, wy, wz, wx, wy, wz));
                        normalize3(wx, wy, wz);
                        sr = make_ray(px, py, pz, wx, wy, wz);
                    } else {
                        float wx, wy, wz;
                        sample_uniform_direction(P.rng, wx, wy, wz);
                        sr = make_ray(px, py, pz, wx, wy, wz);
                    }
                    const float w = (albedo * kInv4Pi) * (float)(nl + 1);
                    const float m0 = MULTI ? P.tp0 * w : w, m1 = MULTI ? P.tp1 * w : w, m2 = MULTI ? P.tp2 * w : w;
                    const bool queued = nee_queue(A, sr, dist, li, m0, m1, m2, P.first, P.last, P.defer);
                    S.C.add(queued ? kFFNeeQueued : kFFNeeInline);
                    if (!queued) {
                        float Li0, Li1, Li2;
                        nee_radiance(A, transmittance_up_to(A, sr, dist, stack, kFFBlock), li, dist, Li0, Li1, Li2);
                        P.after |= P.first != kFFNone;
                        if constexpr (!MULTI) {
                            P.L0 = m0 * Li0;
                            P.L1 = m1 * Li1;
                            P.L2 = m2 * Li2;
                        } else {
                            P.L0 += m0 * Li0;
                            P.L1 += m1 * Li1;
                            P.L2 += m2 * Li2;
                        }
                    }
                    if constexpr (!MULTI) {
                        done = true;
                    } else {
                        P.tp0 *= albedo;
                        P.tp1 *= albedo;
                        P.tp2 *= albedo;
                        if (P.bounce >= A.ff_min_bounces) {  // integrator.h:691-695
                            const float rr = fminf(fmaxf(P.tp0, fmaxf(P.tp1, P.tp2)), 0.9f);
                            if (P.rng.uniform() > rr) {
                                done = true;
                            } else {
                                P.tp0 = __fdiv_rn(P.tp0, rr);
                                P.tp1 = __fdiv_rn(P.tp1, rr);
                                P.tp2 = __fdiv_rn(P.tp2, rr);
                            }
                        }
                        if (!done) {
                            float nx, ny, nz;
                            sample_uniform_direction(P.rng, nx, ny, nz);
                            P.ray = make_ray(px, py, pz, nx, ny, nz);
                            ++P.bounce;
                        }
                    }
                }
                if (done) {
                    if (!requeued)
                        A.ff_tail[P.out] = make_float4(P.L0, P.L1, P.L2, __uint_as_float(P.first | (P.after ? kFFTailAfter : 0u)));
                    phase = kSmIdle;
                } else {
                    begin_bounce();
                }
            }
        } else if (ns >= nc) {
            // ---- SWEEP: free_flight_distance's event sweep, term for term ----
            int budget = VR_FFSM_EVENT_BUDGET;
            bool go = phase == kSmSweep;
            while (go) {
                budget -= max(m, 1);
                const float4 hn = i < n ? S.H(i) : make_float4(INFINITY, 0.0f, 0.0f, 0.0f);  // (the entry's row, once)
                const float next_entry = hn.x;
                float t_evt = fminf(next_entry, next_exit);
                const bool window_end = t_cut <= t_evt;
                if (window_end) t_evt = t_cut;
                if (t_evt == INFINITY) {  // past the last event: no scatter (integrator.h:362-366)
                    to_shade(-1.0f);
                    break;
                }
                const bool is_entry = next_entry <= next_exit;
                float nx = INFINITY;
                int npos = -1;
                Acc seg = 0;
                // F at the segment start recomputed (the cached value's own float operations: bit-identical),
                // so the sweep reads 20 B per active entry and writes nothing; the next entry's read in flight
                float4 cn = m > 0 ? S.A0(0) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                float tn = m > 0 ? S.T1(0) : 0.0f;
#pragma unroll 1
                for (int a = 0; a < m; ++a) {
                    const float4 c = cn;
                    const float t1a = tn;
                    if (a + 1 < m) {
                        cn = S.A0(a + 1);
                        tn = S.T1(a + 1);
                    }
                    S.C.add(kFFErf);
                    const float f1 = erff(__fdiv_rn(c.y + c.z * t_evt, c.w));
                    const float f0 = erff(__fdiv_rn(c.y + c.z * t_prev, c.w));
                    seg += (Acc)(c.x * (f1 - f0));
                    int pp = a;
                    if (!is_entry && a == m - 1) pp = exit_pos;
                    const bool gone = !is_entry && a == exit_pos;
                    if (!gone && (t1a < nx || (t1a == nx && pp < npos))) {
                        nx = t1a;
                        npos = pp;
                    }
                }
                if (acc + seg > (Acc)target) {  // the scatter lies in [t_prev, t_evt]: SHADE solves for it
                    kfull = (float)((Acc)target - acc);
                    t_cut = t_evt;
                    phase = kSmShade;
                    break;
                }
                acc += seg;
                t_prev = t_evt;
                S.ph ^= 1;
                if (window_end) {  // the next window starts at t_cut
                    W0 = t_cut;
                    cap = min(2 * cap, A.ff_hit_cap);
                    begin_window();
                    break;
                }
                if (is_entry) {
                    if (m >= A.ff_act_cap) {
                        to_shade(-2.0f);
                        break;
                    }
                    const float t1n = S.template enter_row<false>(A, m, hn, P.ray, t_evt);
                    ++i;
                    if (t1n < nx) {
                        nx = t1n;
                        npos = m;
                    }
                    ++m;
                } else {
                    S.move(exit_pos, m - 1);
                    --m;
                }
                next_exit = nx;
                exit_pos = npos;
                go = budget > 0;
            }
        } else {
            // ---- COLLECT: one NODE or PRIM iteration of the window's while-while walk ----
            const bool col = phase == kSmCollect;
            const bool walking = col && !redo;
            const bool has_prim = walking && (j < end || qn > 0);
            const bool can_node = walking && node >= 0 && qn <= kCollectQueue - 4;
            const int np = __popcll(__ballot(has_prim)), nn = __popcll(__ballot(can_node));
            if (nn == 0 || (np > 0 && np >= nn)) {  // PRIM iteration
                bool go = has_prim;
                for (int k = 0; k < kSmCollectSteps; ++k) {
                    if (go) {
                        if (j == end) {
                            const int32_t ref = ring[qh * kFFBlock];
                            qh = (qh + 1) & (kCollectQueue - 1);
                            --qn;
                            j = leaf_first(ref);
                            end = j + leaf_count(ref);
                        }
                        prim(j);
                        ++j;
                    }
                    go = go && (j < end || qn > 0);
                }
            } else {  // NODE iteration (the ray's node-space slab constants, recomputed per iteration)
#ifdef VR_DIAG_FFSM
                dnode = true;
#endif
                float ox = P.ray.ox, oy = P.ray.oy, oz = P.ray.oz;
                node_space<true>(A, ox, oy, oz);
                auto inv = [&](float d) {
                    d *= A.hn_scale;
                    return __frcp_rn(fabsf(d) > 1e-30f ? d : copysignf(1e-30f, d));
                };
                const float ix = inv(P.ray.dx), iy = inv(P.ray.dy), iz = inv(P.ray.dz);
                const float oxi = ox * ix, oyi = oy * iy, ozi = oz * iz;
                bool go = can_node;
                for (int k = 0; k < kSmCollectSteps; ++k) {
                    if (go) {
                        S.C.add(kFFNode4);
                        float key[4];
                        int32_t kr[4];
                        wide_children(A, node, ix, iy, iz, oxi, oyi, ozi, prune, key, kr);
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            if (kr[c] < 0) {
                                ring[((qh + qn) & (kCollectQueue - 1)) * kFFBlock] = kr[c];
                                ++qn;
                            }
                        int first = -1;
                        int32_t next = 0;
#pragma unroll
                        for (int c = 3; c >= 0; --c) {
                            first = kr[c] > 0 ? c : first;
                            next = kr[c] > 0 ? kr[c] : next;
                        }
                        if (sp + 3 > kStackSize) {
                            redo = true;
                            node = -1;
                        } else {
#pragma unroll
                            for (int c = 3; c >= 0; --c)
                                if (kr[c] > 0 && c != first) stack[(sp++) * kFFBlock] = kr[c];
                            if (first >= 0) node = next;
                            else if (sp > 0) node = stack[(--sp) * kFFBlock];
                            else node = -1;
                        }
                    }
                    go = go && node >= 0 && qn <= kCollectQueue - 4 && !redo;
                }
            }
            if (col && (redo || (node < 0 && j == end && qn == 0))) {  // the window's collection is complete
                if (redo) {  // the pair tree (at most one push per level) redoes the whole collection
                    n = 0;
                    t_cut = kfull = INFINITY;
                    auto leaf = [&](uint32_t first, uint32_t count) {
                        for (uint32_t jj = first; jj < first + count; ++jj) prim(jj);
                        return true;
                    };
                    auto on2 = [&]() { S.C.add(kFFNode2); };
                    if (A.hnodes) traverse<true>(A, P.ray, stack, kFFBlock, prune, leaf, on2);
                    else traverse<false>(A, P.ray, stack, kFFBlock, prune, leaf, on2);
                }
                // a buffer that filled ends the window at its largest kept key (subtrees skipped while full hold
                // only larger keys; whether one was skipped depends on the wave's NODE/PRIM schedule, so the cut must not)
                if (n == cap) t_cut = fminf(t_cut, S.K(n - 1));
                while (n > 0 && S.K(n - 1) >= t_cut) --n;
                if (t_cut <= W0) {  // more than cap Gaussians overlap at W0: no progress at this cap
                    if (cap >= A.ff_hit_cap) {
                        to_shade(-2.0f);
                    } else {
                        cap = min(2 * cap, A.ff_hit_cap);
                        begin_window();
                    }
                } else if (n == 0 && t_cut == INFINITY) {
                    to_shade(-1.0f);
                } else {
                    i = m = 0;
                    next_exit = INFINITY;
                    exit_pos = -1;
                    S.ph = 0;  // (entries write both F slots: the phase at a window's start is free)
                    phase = kSmSweep;
                }
            }
        }
#ifdef VR_DIAG_FFSM
        if constexpr (CNT) {
            if (lane == 0u) {
                const uint32_t dc = (uint32_t)((__builtin_amdgcn_s_memtime() - dt0) >> 4);
#if VR_DIAG_FFSM == 2
                const int k = dphase == 0 ? (dnode ? 0 : 1) : dphase + 1;
                S.C.v[k] += dc;
                S.C.v[4 + k] += 1u;
#else
                S.C.v[dphase] += dc;
                S.C.v[3 + dphase] += 1u;
                if (dphase == 0) S.C.v[6] += (uint32_t)nc;
                if (dphase == 1) S.C.v[7] += (uint32_t)ns;
#endif
            }
        }
#endif
    }
    if constexpr (CNT) {
        Ctr c{};
        for (int k = 0; k < kFFNumCtr; ++k) c.v[k] = S.C.v[k];
        flush_counters(A.work, c);
    }
}

// Paths the path kernel queued because more Gaussians overlapped one point than its rows hold: each
// re-runs from its first bounce (same seed, so the same path) with kFFBigCap-entry rows and inline
// shadow rays, and writes its radiance as one inline sum (its earlier queued shadow rays are dropped).
// Only a path over kFFBigCap fails (NaN, VR_ERR_OVERFLOW).
template <bool MULTI>
__global__ void __launch_bounds__(kFFBlock) ff_fallback_kernel(RenderArgs A) {
    __shared__ int s_stack[(kStackSize + kCollectQueue) * kFFBlock];
    int* stack = s_stack + threadIdx.x;
    const uint32_t gt = blockIdx.x * kFFBlock + threadIdx.x, nt = gridDim.x * kFFBlock;
    const uint32_t n = min(A.ff_fbq[0], A.ff_fbq_cap);
    RenderArgs B = A;
    B.ff_threads = nt;
    B.ff_hit_cap = B.ff_act_cap = kFFBigCap;
    B.ff_hit = A.ff_big;
    B.ff_act0 = A.ff_big + (size_t)kFFBigCap * nt;
    B.ff_act1 = A.ff_big + (size_t)2 * kFFBigCap * nt;
    B.ff_nee_cap = 0;  // shadow rays inline
    B.ff_fbq = nullptr;
    FFScratch<false> S{B.ff_hit + gt, B.ff_act0 + gt, B.ff_act1 + gt, nt, 0, {}};
    for (uint32_t q = gt; q < n; q += nt) {
        FFPath P{PCG32(0, 1)};
        if (!ff_start(B, A.ff_fbq[1 + q], P)) continue;
        while (ff_bounce<MULTI>(B, S, stack, P)) {
        }
    }
}

// Traces the launch's queued shadow rays (the walk of transmittance_up_to on the 4-wide tree, the
// same double sum and early stop) as a persistent while-while kernel: a lane whose ray is done takes
// the next queued ray, claimed per wave once ff_nee_refill lanes are idle, so a wave never waits for
// its longest ray. Each ray's contribution m * Li replaces its weight m in place.
__device__ __forceinline__ void nee_finish(const RenderArgs& A, uint32_t id, float tmax, float Tr) {
    float4& c = A.ff_nee[3 * (size_t)id + 2];
    const float4 m = c;
    float Li0, Li1, Li2;
    nee_radiance(A, Tr, __float_as_int(m.w), tmax, Li0, Li1, Li2);
    c = make_float4(m.x * Li0, m.y * Li1, m.z * Li2, m.w);
}

#ifndef VR_NEE_BLOCKS
#define VR_NEE_BLOCKS 4  // resident 256-lane blocks per CU
#endif
// A wave iteration is either a NODE iteration (lanes with room in their leaf FIFO take up to
// kNeeSteps 4-wide node steps, leaf children queued near-first) or a PRIM iteration (lanes with queued leaves test up to kNeeSteps
// Gaussians), whichever more lanes can use, so node and primitive work no longer split a wave. The
// FIFO hands leaves out in the order the walk reaches them, so the double sum adds the same terms in
// the same order as transmittance_up_to (bit-identical Tr; a sum stopped mid-leaf is >= 104 either way).
#ifndef VR_NEE_STEPS
#define VR_NEE_STEPS 4  // node steps / primitives per lane per wave iteration of the shadow-ray kernel
#endif
constexpr int kNeeQueue = 8, kNeeSteps = VR_NEE_STEPS;
template <bool CNT = false>
__global__ void __launch_bounds__(kFFBlock) ff_nee_kernel(RenderArgs A) {
    FFCount<CNT> C;
    __shared__ int s_stack[(kStackSize + kNeeQueue) * kFFBlock];
    int* stack = s_stack + threadIdx.x;
    int* ring = stack + kStackSize * kFFBlock;
    const uint32_t n = min(A.ff_nee_n[0], A.ff_nee_cap);
    const uint32_t lane = threadIdx.x & 63u;
    bool live = false, exhausted = false;
    uint32_t id = 0;
    Ray r{};
    float tmax = 0.0f, lim = 0.0f, ix = 0.0f, iy = 0.0f, iz = 0.0f, oxi = 0.0f, oyi = 0.0f, ozi = 0.0f;
    double sum = 0.0;
    int sp = 0, node = -1, qh = 0, qn = 0;
    uint32_t j = 0, end = 0;  // primitives of the leaf being tested
    bool redo = false;        // the 4-wide stack could overflow: whole walk at the end (pair-tree fallback)
    for (;;) {
        const uint64_t idle = __ballot(!live);
        if (!exhausted && (idle == ~0ull || __popcll(idle) >= A.ff_nee_refill)) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(A.ff_nee_n + 1, (uint32_t)__popcll(idle));
            base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
            exhausted = base + (uint32_t)__popcll(idle) >= n;
            if (!live) {
                id = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                if (id < n) {
                    const float4 a = A.ff_nee[3 * (size_t)id], b = A.ff_nee[3 * (size_t)id + 1];
                    r = Ray{a.x, a.y, a.z, b.x, b.y, b.z};
                    tmax = a.w;
                    if (!(tmax > 0.0f)) {
                        nee_finish(A, id, tmax, 1.0f);
                    } else {
                        float ox = r.ox, oy = r.oy, oz = r.oz;
                        node_space<true>(A, ox, oy, oz);
                        auto inv = [&](float d) {
                            d *= A.hn_scale;
                            return __frcp_rn(fabsf(d) > 1e-30f ? d : copysignf(1e-30f, d));
                        };
                        ix = inv(r.dx), iy = inv(r.dy), iz = inv(r.dz);
                        oxi = ox * ix, oyi = oy * iy, ozi = oz * iz;
                        lim = shadow_prune_lim(tmax);
                        sum = 0.0;
                        sp = 0;
                        qh = qn = 0;
                        j = end = 0;
                        // no 4-wide tree (VR_OPT_HALF_NODES = 0 or f32 boxes): the ray goes straight to the
                        // pair-tree walk of transmittance_up_to at its completion
                        redo = A.hnodes4 == nullptr;
                        node = redo ? -1 : 0;
                        live = true;
                        C.add(kNeeRays);
                    }
                }
            }
        }
        if (!__any(live)) {
            if (exhausted) break;
            continue;
        }
        const bool has_prim = live && (j < end || qn > 0);
        const bool can_node = live && node >= 0 && qn <= kNeeQueue - 4;
        const int np = __popcll(__ballot(has_prim)), nn = __popcll(__ballot(can_node));
        if (nn == 0 || (np > 0 && np >= nn)) {  // PRIM iteration
            bool go = has_prim;
            for (int k = 0; k < kNeeSteps; ++k) {
                if (go) {
                    if (j == end) {
                        const int32_t ref = ring[qh * kFFBlock];
                        qh = (qh + 1) & (kNeeQueue - 1);
                        --qn;
                        j = leaf_first(ref);
                        end = j + leaf_count(ref);
                    }
                    shadow_leaf(A, r, tmax, j, 1u, sum, &C);
                    ++j;
                }
                go = go && (j < end || qn > 0) && sum < 104.0;
            }
        } else {  // NODE iteration
            bool go = can_node;
            for (int k = 0; k < kNeeSteps; ++k) {
                if (go) {
                    C.add(kNeeNode4);
                    float key[4];
                    int32_t kr[4];
                    wide_children(A, node, ix, iy, iz, oxi, oyi, ozi, [&](float tmin, float) { return tmin <= lim; }, key, kr);
#pragma unroll
                    for (int i = 0; i < 4; ++i)  // leaves, near first
                        if (kr[i] < 0) {
                            ring[((qh + qn) & (kNeeQueue - 1)) * kFFBlock] = kr[i];
                            ++qn;
                        }
                    int first = -1;
                    int32_t next = 0;
#pragma unroll
                    for (int i = 3; i >= 0; --i) {
                        first = kr[i] > 0 ? i : first;
                        next = kr[i] > 0 ? kr[i] : next;
                    }
                    if (sp + 3 > kStackSize) {
                        redo = true;
                        node = -1;
                    } else {
#pragma unroll
                        for (int i = 3; i >= 0; --i)
                            if (kr[i] > 0 && i != first) stack[(sp++) * kFFBlock] = kr[i];
                        if (first >= 0) node = next;
                        else if (sp > 0) node = stack[(--sp) * kFFBlock];
                        else node = -1;
                    }
                }
                go = go && node >= 0 && qn <= kNeeQueue - 4;
            }
        }
        if (live && (redo || !(sum < 104.0) || (node < 0 && j == end && qn == 0))) {
            const float Tr = redo ? transmittance_up_to(A, r, tmax, stack, kFFBlock) : expf(-(float)sum);
            nee_finish(A, id, tmax, Tr);
            live = false;
        }
    }
    if constexpr (CNT) {
        Ctr c{};
        for (int i = 0; i < kFFNumCtr; ++i) c.v[i] = C.v[i];
        flush_counters(A.work + 8, c);
    }
}

// Each path's radiance from its queued contributions (bounce order) and its inline part, one thread
// per path of the launch (the chains are walked in parallel, not by the pixel's thread sample after
// sample); written back into the path's ff_tail entry with no chain left.
__global__ void __launch_bounds__(kFFBlock) ff_path_radiance_kernel(RenderArgs A) {
    const size_t q = (size_t)blockIdx.x * kFFBlock + threadIdx.x;
    if (q == 0) atomicMax(A.counters + 3, A.ff_nee_n[0]);  // the frame's largest launch queue need (host sizing)
    if (q >= A.ff_total) return;
    const float4 t = A.ff_tail[q];
    const uint32_t f = __float_as_uint(t.w);
    if ((f & ~kFFTailAfter) == kFFNone) return;
    float p0 = 0.0f, p1 = 0.0f, p2 = 0.0f;
    for (uint32_t e = f & ~kFFTailAfter; e != kFFNone; e = __float_as_uint(A.ff_nee[3 * (size_t)e + 1].w)) {
        const float4 c = A.ff_nee[3 * (size_t)e + 2];
        p0 += c.x;
        p1 += c.y;
        p2 += c.z;
    }
    if (f & kFFTailAfter) {
        p0 += t.x;
        p1 += t.y;
        p2 += t.z;
    }
    A.ff_tail[q] = make_float4(p0, p1, p2, __uint_as_float(kFFNone));
}

// pixel_L += L_accum in sample order (integrator.h:706), then pixel_L / num_samples on the last batch.
__global__ void __launch_bounds__(kFFBlock) ff_accumulate_kernel(RenderArgs A, uint32_t chunk_tiles) {
    const uint32_t tl = blockIdx.x;  // tile within the chunk
    if (tl >= chunk_tiles) return;
    const uint32_t tile_local = A.ff_tile_base + tl;
    const size_t p = (size_t)tile_local * kFFBlock + threadIdx.x;
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
    if (A.ff_si0 != 0) {
        s0 = A.ff_sum[p * 3 + 0];
        s1 = A.ff_sum[p * 3 + 1];
        s2 = A.ff_sum[p * 3 + 2];
    }
    for (uint32_t s = 0; s < A.ff_nsb; ++s) {
        const size_t q = (size_t)(tl * A.ff_nsb + s) * kFFBlock + threadIdx.x;
        const float4 t = A.ff_tail[q];  // the path's radiance: its queued contributions in order, then t.xyz
        const uint32_t f = __float_as_uint(t.w);
        float p0 = t.x, p1 = t.y, p2 = t.z;
        if ((f & ~kFFTailAfter) != kFFNone) {
            p0 = p1 = p2 = 0.0f;
            for (uint32_t e = f & ~kFFTailAfter; e != kFFNone; e = __float_as_uint(A.ff_nee[3 * (size_t)e + 1].w)) {
                const float4 c = A.ff_nee[3 * (size_t)e + 2];
                p0 += c.x;
                p1 += c.y;
                p2 += c.z;
            }
            if (f & kFFTailAfter) {
                p0 += t.x;
                p1 += t.y;
                p2 += t.z;
            }
        }
        s0 += p0;
        s1 += p1;
        s2 += p2;
    }
    if (A.ff_si0 + A.ff_nsb < (uint32_t)A.ff_samples) {
        A.ff_sum[p * 3 + 0] = s0;
        A.ff_sum[p * 3 + 1] = s1;
        A.ff_sum[p * 3 + 2] = s2;
        return;
    }
    int lx, ly, x, y;
    tile_pixel(A, tile_local, threadIdx.x, lx, ly, x, y);
    const float fs = (float)A.ff_samples;
    store_px(A, tile_local, lx, ly, x, y, __fdiv_rn(s0, fs), __fdiv_rn(s1, fs), __fdiv_rn(s2, fs));
}

// inverse_integrator.h:166-182: out[g] += sum over pixels p whose bit g is set in bits0 or bits1 of
// (loss_plus[p] - loss_base[p]) (double). Grid: (words, pixel chunks); each thread keeps the 32
// Gaussians of its word in registers, a wave reduces them, lane 0 adds them atomically.
__global__ void __launch_bounds__(256) sfd_loss_diff_kernel(const uint32_t* __restrict__ bits0, const uint32_t* __restrict__ bits1,
                                                            const float* __restrict__ loss_base, const float* __restrict__ loss_plus,
                                                            uint32_t npix, uint32_t chunk, uint32_t n, double* out) {
    const uint32_t w = blockIdx.x;
    const uint32_t p0 = blockIdx.y * chunk, p1 = min(npix, p0 + chunk);
    double acc[32];
#pragma unroll
    for (int b = 0; b < 32; ++b) acc[b] = 0.0;
    for (uint32_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const uint32_t word = bits0[(size_t)w * npix + p] | bits1[(size_t)w * npix + p];
        if (!word) continue;
        const double d = (double)loss_plus[p] - (double)loss_base[p];
#pragma unroll
        for (int b = 0; b < 32; ++b)
            if ((word >> b) & 1u) acc[b] += d;
    }
#pragma unroll
    for (int b = 0; b < 32; ++b) {
        double v = acc[b];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        const uint32_t g = w * 32u + (uint32_t)b;
        if ((threadIdx.x & 63) == 0 && v != 0.0 && g < n) atomicAdd(out + g, v);
    }
}

// compute_pixel_losses (inverse_integrator.h:21-30): per-pixel L1 over RGB, d.cwiseAbs().sum()
// (Eigen's 3-term reduction: |d0| + (|d1| + |d2|)).
__global__ void __launch_bounds__(256) pixel_loss_kernel(const float* __restrict__ img, const float* __restrict__ ref,
                                                         uint32_t npix, float* __restrict__ out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    const float d0 = img[3 * (size_t)p] - ref[3 * (size_t)p];
    const float d1 = img[3 * (size_t)p + 1] - ref[3 * (size_t)p + 1];
    const float d2 = img[3 * (size_t)p + 2] - ref[3 * (size_t)p + 2];
    out[p] = fabsf(d0) + (fabsf(d1) + fabsf(d2));
}

}  // namespace dev

hipError_t launch_pixel_losses(const float* img, const float* ref, uint32_t npix, float* out, hipStream_t stream) {
    hipLaunchKernelGGL(dev::pixel_loss_kernel, dim3((npix + 255) / 256), dim3(256), 0, stream, img, ref, npix, out);
    return hipGetLastError();
}

hipError_t launch_sfd_loss_diff(const uint32_t* bits0, const uint32_t* bits1, const float* lb, const float* lp, uint32_t npix,
                                uint32_t n, double* out, hipStream_t stream) {
    const uint32_t words = (n + 31) / 32, chunk = 4096;
    dim3 grid(words, (npix + chunk - 1) / chunk);
    hipLaunchKernelGGL(dev::sfd_loss_diff_kernel, grid, dim3(256), 0, stream, bits0, bits1, lb, lp, npix, chunk, n, out);
    return hipGetLastError();
}

// Threads of the resident path-kernel grid on a device with `cus` CUs (the scratch row stride).
uint32_t free_flight_threads(int cus) {
    int per_cu = 0;
    int per_sm = 0;  // (both path kernels run a resident grid over the same rows: the smaller occupancy)
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)dev::ff_path_kernel<true, false>, dev::kFFBlock, 0) !=
            hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_sm, (const void*)dev::ff_path_sm_kernel<true, false>, dev::kFFBlock, 0) !=
            hipSuccess)
        per_cu = per_sm = 1;
    per_cu = std::max(1, std::min(per_cu, per_sm));
    return (uint32_t)std::max(1, cus) * (uint32_t)per_cu * (uint32_t)dev::kFFBlock;
}

// Host launcher: one (tile chunk, sample batch) step. A.ff_* describe the step.
hipError_t launch_free_flight(const RenderArgs& A, uint32_t chunk_tiles, hipStream_t stream, hipEvent_t* ev) {
    hipError_t e0 = hipMemsetAsync(A.ff_next, 0, sizeof(unsigned long long), stream);
    if (e0 != hipSuccess) return e0;
    if (A.ff_nee_cap > 0 && (e0 = hipMemsetAsync(A.ff_nee_n, 0, 2 * sizeof(uint32_t), stream)) != hipSuccess) return e0;
    if (A.ff_fbq != nullptr && (e0 = hipMemsetAsync(A.ff_fbq, 0, sizeof(uint32_t), stream)) != hipSuccess) return e0;
    dim3 grid(A.ff_threads / dev::kFFBlock);
    const bool cnt = A.work != nullptr;  // vr_count_work: the instrumented kernels
    if ((e0 = hipEventRecord(ev[0], stream)) != hipSuccess) return e0;
    if (A.ff_sm) {  // the phase-scheduled path kernel (VR_OPT_FF_KERNEL)
        if (A.ff_multi) {
            if (cnt) hipLaunchKernelGGL((dev::ff_path_sm_kernel<true, true>), grid, dim3(dev::kFFBlock), 0, stream, A);
            else hipLaunchKernelGGL((dev::ff_path_sm_kernel<true>), grid, dim3(dev::kFFBlock), 0, stream, A);
        } else {
            if (cnt) hipLaunchKernelGGL((dev::ff_path_sm_kernel<false, true>), grid, dim3(dev::kFFBlock), 0, stream, A);
            else hipLaunchKernelGGL((dev::ff_path_sm_kernel<false>), grid, dim3(dev::kFFBlock), 0, stream, A);
        }
    } else if (A.ff_multi) {
        if (cnt) hipLaunchKernelGGL((dev::ff_path_kernel<true, true>), grid, dim3(dev::kFFBlock), 0, stream, A);
        else hipLaunchKernelGGL((dev::ff_path_kernel<true>), grid, dim3(dev::kFFBlock), 0, stream, A);
    } else {
        if (cnt) hipLaunchKernelGGL((dev::ff_path_kernel<false, true>), grid, dim3(dev::kFFBlock), 0, stream, A);
        else hipLaunchKernelGGL((dev::ff_path_kernel<false>), grid, dim3(dev::kFFBlock), 0, stream, A);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (A.ff_fbq != nullptr) {  // paths over the hit-buffer capacity (usually none: the kernel exits at once)
        if (A.ff_multi) hipLaunchKernelGGL((dev::ff_fallback_kernel<true>), dim3(kFFBigThreads / dev::kFFBlock), dim3(dev::kFFBlock), 0, stream, A);
        else hipLaunchKernelGGL((dev::ff_fallback_kernel<false>), dim3(kFFBigThreads / dev::kFFBlock), dim3(dev::kFFBlock), 0, stream, A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if ((e = hipEventRecord(ev[1], stream)) != hipSuccess) return e;
    if (A.ff_nee_cap > 0) {
        int dv = 0, cus = 1;
        if (hipGetDevice(&dv) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dv);
        const dim3 ng((unsigned)std::max(1, cus) * VR_NEE_BLOCKS);
        if (cnt) hipLaunchKernelGGL(dev::ff_nee_kernel<true>, ng, dim3(dev::kFFBlock), 0, stream, A);
        else hipLaunchKernelGGL(dev::ff_nee_kernel<false>, ng, dim3(dev::kFFBlock), 0, stream, A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if ((e = hipEventRecord(ev[2], stream)) != hipSuccess) return e;
    if (A.ff_nee_cap > 0) {
        hipLaunchKernelGGL(dev::ff_path_radiance_kernel, dim3((unsigned)((A.ff_total + dev::kFFBlock - 1) / dev::kFFBlock)),
                           dim3(dev::kFFBlock), 0, stream, A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(dev::ff_accumulate_kernel, dim3(chunk_tiles), dim3(dev::kFFBlock), 0, stream, A, chunk_tiles);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return hipEventRecord(ev[3], stream);
}

}  // namespace vr
