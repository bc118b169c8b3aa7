// RayMarchingGaussians (test_integrators.h:160-296) as a three-stage wavefront pipeline for gfx950.
//
// The reference marches every pixel on one CPU thread and, at each step that scatters, traces
// nlights + env_samples secondary rays one after another. The transmittance T of the primary ray
// never depends on those secondary rays (they only add to L), so the device path splits the loop:
//
//   1. march_kernel (one thread per pixel, 256-thread workgroup per 16x16 tile): walks the primary
//      ray's steps and emits one *scatter record* per step with sigma_s > 0 (position, T*sigma_s,
//      step index k, the active Gaussian set). Run twice: MODE 0 counts records per pixel, an
//      exclusive scan places them, MODE 1 writes them — so the record order is a pure function of
//      the frame, and the final image is bitwise reproducible.
//   2. secondary_persistent_kernel (every light / environment ray of every record; ray ids in
//      sample-major order so that neighbouring lanes trace rays from neighbouring pixels towards the
//      same light): transmittance of each secondary ray, see Stage 2 below.
//   3. accumulate_kernel (one thread per pixel): L += T*sigma_s*(Li + Le)*dt/(4 pi) over the
//      pixel's records in step order, then L += T*env — the reference's operation order.
//
// No per-ray event list is ever built or sorted:
//   * the step sequence t_k is the reference's own iterated float sum (host table), so empty
//     stretches are skipped by index;
//   * the active set at step k is {i : a_i <= t_k < b_i}; it is kept as a short sorted list of
//     Gaussian ids in LDS, extended by BVH queries restricted to the window (t_{k-1}, t_k] or by a
//     closest-entry query when it runs empty;
//   * a secondary ray's transmittance telescopes the reference's segment loop into one sum of
//     per-Gaussian optical depths over each Gaussian's active interval on that ray, reproducing the
//     quirks: primary-active Gaussians are pre-activated at t = 0 (test_integrators.h:209-211), a
//     light ray's last segment runs to the first event at or past the light (:220-235), an
//     environment ray runs to its last event (:258-271);
//   * a ray stops marching when T <= t_eps (exactly 0 by default: bit-neutral).
// Pixels whose active set outgrows the fast path's LDS list (32) are queued and re-run by the
// fallback kernels (64), so results never depend on capacity.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include <type_traits>

#include <hipcub/hipcub.hpp>

#include "vr_dev_common.h"

namespace vr {
namespace dev {

// Optical-depth cut-off of a secondary ray: expf(-104) rounds to 0 in f32 and every optical depth
// is >= 0, so once the running sum reaches kTauCut the ray's transmittance is exactly 0 whatever
// else it crosses — the traversal stops there. (The reference's product of per-segment
// exponentials reaches 0 or a denormal <= 1.4e-45 at the same point.)
constexpr float kTauCut = 104.0f;

// Band around a list member's 3-sigma surface (in p.M.p and in the chord's 9 - e2) inside which a secondary
// ray's decision for that member is left to the exact slow path: ~10x the f32 difference between the
// whitened and the reference's M forms for an origin near the Gaussian (~1e-7 relative, times the
// covariance's condition number). The march marks a record whose members include one with p.M.p above
// 9 - 2 kMemberAmb (kRecBoundary in the active count), so only the rays of such records (~1 %) test it.
#ifndef VR_MEMBER_AMB
#define VR_MEMBER_AMB 5e-5f  // (A/B: 0 removes the test)
#endif
constexpr float kMemberAmb = VR_MEMBER_AMB;

// Band around a secondary ray's grazing chords inside which the reference's f32 quadratic (gaussian.h:137-151:
// B*B - 4*A*C with A = d.M.d, B = 2 p.M.d, C = p.M.p - 9) may decide otherwise than the whitened chord test: its
// discriminant, in units of D = 9 - e2 (the chord's half length squared in whitened units), carries an absolute
// error of up to ~5 eps c (eps = 2^-23, c = p.M.p; measured maximum 5.1 eps c over 2.3e5 grazing rays of the
// make_random distribution, tools/chord_band.py). Inside it the reference can collapse a chord to a point or miss it
// (C4 at t_eps 0, pixel (598, 3212): D = 3.3e-4 at c = 2735, [0.32260, 0.32282] became [0.3227114, 0.3227114] and its
// 0.078 of optical depth was lost) or keep a tiny phantom chord the whitened test misses. A ray with a test inside
// |D| < kChordBand c goes to the exact slow path, which runs the reference's M forms on the exactly normalised ray.
#ifndef VR_CHORD_BAND
#define VR_CHORD_BAND 8.0f  // in eps c (A/B: 0 removes the test)
#endif
constexpr float kChordBand = VR_CHORD_BAND * 1.1920928955078125e-7f;
constexpr uint32_t kRecBoundary = 0x80000000u;  // rec_meta.w: active count | this flag
// An environment ray with one non-member chord in the f32 error band (kChordBand) keeps that Gaussian's id in its
// `lim` (the last event so far, only needed for a missed member: such a ray goes to the exact slow path anyway) as
// a NaN payload, which `t1 > lim` never overwrites: no register and no store on the traversal's path.
__device__ __forceinline__ float band_lim(uint32_t j) { return __uint_as_float(0x7f800000u | (j + 1u)); }
__device__ __forceinline__ uint32_t band_id(float lim) { return (__float_as_uint(lim) & 0x007fffffu) - 1u; }
#ifndef VR_MARCH_DEEP
// Private-memory (scratch) stack entries of the primary march's 4-wide walks past its LDS stack; a walk past both goes
// to the fallback pass. Round 6, C4 (same frame hash): LDS 24 + 0 -> 14 + 10 moved the quarter-tile workgroup from
// 10 to 7.5 KB of LDS, 4 -> 5 waves/SIMD, march 13.95 -> 12.92 ms (12 + 12: 13.02, 10 + 14: 13.2, 16 + 8: 13.7).
#define VR_MARCH_DEEP 10
#endif

#ifdef VR_DIAG_UNION  // diagnostic builds only: the march's counter slots report the union-walk census
constexpr bool kDiagUnion = true;
#else
constexpr bool kDiagUnion = false;
#endif

// Bit of active-list slot `slot` in a ray's 64-bit hit mask. Records with more than 64 active
// Gaussians (march_deep_kernel) find their missed members by re-intersecting the whole list instead.
__device__ __forceinline__ uint64_t slot_bit(int slot) { return slot < 64 ? 1ull << slot : 0ull; }

// Scatter records of the frame, read on the device: the host never waits for the march (the
// buffers are sized from the previous frame; a frame that outgrew them is reported and re-run).
// Clamped to the capacity, so an overflowing frame stays in bounds.
__device__ __forceinline__ uint32_t dev_nrec(const RenderArgs& A) { return min(A.rec_alloc[0], A.rec_cap); }

// ---------------------------------------------------------------------------------------------
// Exact light-ray transmittance (the slow path of Stage 2)
// ---------------------------------------------------------------------------------------------

// Towards a point light at distance `dist` (test_integrators.h:202-237).
template <bool S>
__device__ float light_transmittance(const RenderArgs& A, const Ray& sr, float dist, const ActList& act, int* stack,
                                     int stride, Ctr& c) {
    if (!(dist > 0.0f)) return 1.0f;  // `while (t_prev < dist)` never runs
    const GaussianRecord* __restrict__ G = A.gauss;
    float tau = 0.0f;
    bool needs_stop = false;
    uint64_t hitmask = 0;
    // the 4-wide half-precision tree when the scene has one (half the dependent node fetches of the
    // f32 pair tree; boxes only propose candidates, every decision is the exact quadratic), the pair
    // tree when it has not or when a 4-wide walk could overflow its stack (`reset` undoes the partial walk)
    auto walk = [&](auto prune, auto leaf, auto reset) {
        if (A.hnodes4 != nullptr) {
            if (traverse_wide<kStackSize>(A, sr, stack, stride, prune, leaf, NodeCount<S>{&c})) return;
            reset();
        }
        traverse<false>(A, sr, stack, stride, prune, leaf, NodeCount<S>{&c});
    };
    walk(
        [&](float tmin, float) { return tmin <= dist + kTPad * (1.0f + dist); },
        [&](uint32_t first, uint32_t count) {
            for (uint32_t j = first; j < first + count; ++j) {
                if constexpr (S) c.v[kCtrPrims]++;
                GRec g = load_rec(G, j);
                Quad q = quad(g, sr);
                float a, b;
                if (!intersect(q, a, b)) continue;
                int slot = act.find((int)j);
                float lo = a;
                if (slot >= 0) {
                    lo = 0.0f;
                    hitmask |= slot_bit(slot);
                }
                if (b < dist) {
                    if constexpr (S) c.v[kCtrOD]++;
                    tau += optical_depth(g, q, lo, b);
                } else if (lo < dist) {
                    needs_stop = true;  // straddles the light: needs the stopping event
                }
            }
            return tau < kTauCut;
        },
        [&]() {
            tau = 0.0f;
            needs_stop = false;
            hitmask = 0;
        });
    uint64_t all = act.n >= 64 ? ~0ull : ((1ull << act.n) - 1ull);
    uint64_t missed = all & ~hitmask;  // pre-activated but not intersected (rounding at the surface)
    if (tau >= kTauCut) return 0.0f;   // exp(-tau) == 0 exactly; later terms are >= 0
    // more than 64 active Gaussians: a member is missed iff the ray does not intersect it
    auto deep_missed = [&](int s, GRec& g, Quad& q) {
        float a, b;
        g = load_rec(G, act.get(s));
        q = quad(g, sr);
        return !intersect(q, a, b);
    };
    bool deep_any = false;
    if (act.n > 64) {
        missed = 0;
        for (int s = 0; s < act.n && !deep_any; ++s) {
            GRec g;
            Quad q;
            deep_any = deep_missed(s, g, q);
        }
    }
    if (needs_stop || missed || deep_any) {
        float tstop = INFINITY;  // first event at or beyond the light
        walk(
            [&](float tmin, float tmax) {
                return tmax >= dist - kTPad * (1.0f + dist) && tmin <= tstop + kTPad * (1.0f + tstop);
            },
            [&](uint32_t first, uint32_t count) {
                for (uint32_t j = first; j < first + count; ++j) {
                    if constexpr (S) c.v[kCtrPrims]++;
                    GRec g = load_rec(G, j);
                    Quad q = quad(g, sr);
                    float a, b;
                    if (!intersect(q, a, b)) continue;
                    if (b >= dist) tstop = fminf(tstop, (a >= dist) ? a : b);
                }
                return true;
            },
            [&]() { tstop = INFINITY; });
        if (tstop == INFINITY) tstop = dist;
        if (needs_stop) {
            const float tau0 = tau;
            walk(
                [&](float tmin, float tmax) {
                    return tmin <= dist + kTPad * (1.0f + dist) && tmax >= dist - kTPad * (1.0f + dist);
                },
                [&](uint32_t first, uint32_t count) {
                    for (uint32_t j = first; j < first + count; ++j) {
                        if constexpr (S) c.v[kCtrPrims]++;
                        GRec g = load_rec(G, j);
                        Quad q = quad(g, sr);
                        float a, b;
                        if (!intersect(q, a, b)) continue;
                        float lo = act.find((int)j) >= 0 ? 0.0f : a;
                        if (lo < dist && b >= dist) {
                            if constexpr (S) c.v[kCtrOD]++;
                            tau += optical_depth(g, q, lo, tstop);
                        }
                    }
                    return tau < kTauCut;
                },
                [&]() { tau = tau0; });
        }
        while (missed) {
            int s = __ffsll((unsigned long long)missed) - 1;
            missed &= missed - 1;
            GRec g = load_rec(G, act.get(s));
            Quad q = quad(g, sr);
            if constexpr (S) c.v[kCtrOD]++;
            tau += optical_depth(g, q, 0.0f, tstop);
        }
        if (deep_any)
            for (int s = 0; s < act.n; ++s) {
                GRec g;
                Quad q;
                if (deep_missed(s, g, q)) tau += optical_depth(g, q, 0.0f, tstop);
            }
    }
    return expf(-tau);
}

// Exact environment-ray transmittance (test_integrators.h:242-271): the record's active Gaussians are
// pre-activated at t = 0, every event comes from the exact intersect on the exactly normalised ray, so a
// member's decision matches the reference bit for bit: a member the ray crosses is active on [0, t1], a member
// it misses (t1 < 0 through rounding) stays active to the ray's last event, any other Gaussian on [t0, t1].
// For the rare environment rays whose whitened member test sits at the decision boundary (sec_finish).
template <bool S>
__device__ float env_transmittance(const RenderArgs& A, const Ray& er, const ActList& act, int* stack, int stride, Ctr& c) {
    const GaussianRecord* __restrict__ G = A.gauss;
    float tau = 0.0f, t_last = 0.0f;
    uint64_t hitmask = 0;
    auto walk = [&](auto prune, auto leaf, auto reset) {
        if (A.hnodes4 != nullptr) {
            if (traverse_wide<kStackSize>(A, er, stack, stride, prune, leaf, NodeCount<S>{&c})) return;
            reset();
        }
        traverse<false>(A, er, stack, stride, prune, leaf, NodeCount<S>{&c});
    };
    walk([&](float, float) { return true; },
         [&](uint32_t first, uint32_t count) {
             for (uint32_t j = first; j < first + count; ++j) {
                 if constexpr (S) c.v[kCtrPrims]++;
                 const GRec g = load_rec(G, j);
                 const Quad q = quad(g, er);
                 float a, b;
                 if (!intersect(q, a, b)) continue;
                 t_last = fmaxf(t_last, b);  // (entries come before their exits)
                 const int slot = act.find((int)j);
                 if (slot >= 0) hitmask |= slot_bit(slot);
                 if constexpr (S) c.v[kCtrOD]++;
                 tau += optical_depth(g, q, slot >= 0 ? 0.0f : a, b);
             }
             // the whole walk (a missed member needs the last event) unless Tr is already 0: expf(-tau) == 0
             // in f32 from tau >= 104, and later terms (the missed members' too) only add to tau
             return tau < 104.0f;
         },
         [&]() {
             tau = t_last = 0.0f;
             hitmask = 0;
         });
    for (int s = 0; s < act.n; ++s) {  // members the ray misses: active to the last event
        if (s < 64 && ((hitmask >> s) & 1ull)) continue;
        const GRec g = load_rec(G, act.get(s));
        const Quad q = quad(g, er);
        float a, b;
        if (s >= 64 && intersect(q, a, b)) continue;
        if constexpr (S) c.v[kCtrOD]++;
        tau += optical_depth(g, q, 0.0f, t_last);
    }
    return expf(-tau);
}

// ---------------------------------------------------------------------------------------------
// The same exact transmittances with the whole wave on one ray (the slow path, round 6). A serial walk of one
// long ray is a chain of ~100 dependent node and record loads (~250-400 us); here the wave expands the walk one
// tree level at a time — each lane one frontier node (its four child boxes), the hit inner children appended to
// the next level and the hit leaves to a list in lane order (ballots: a deterministic order), then each lane
// one listed leaf's primitives — so the chain is the tree's depth. Every Gaussian the serial walk tests is
// tested (no prune is tighter), with the same exact M forms; only the order of the optical-depth sum differs
// (per-lane partial sums, then a fixed butterfly). kCoopCap nodes or leaves per level at most: a wider level
// (never seen at C4) falls back to the serial walk on lane 0.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kCoopCap = 256;
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
    return x;
}
__device__ __forceinline__ float wave_min(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fminf(x, __shfl_xor(x, o, 64));
    return x;
}
__device__ __forceinline__ uint64_t wave_or(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)x, o, 64), hi = __shfl_xor((uint32_t)(x >> 32), o, 64);
        x |= ((uint64_t)hi << 32) | lo;
    }
    return x;
}
// Level-by-level walk of the 4-wide tree by the whole wave (every lane calls it with the same ray); leaf(j) runs
// for every primitive of every hit leaf, on the lane the leaf fell to. False: a level outgrew kCoopCap.
template <typename Prune, typename Leaf>
__device__ bool coop_walk(const RenderArgs& A, const Ray& r0, int* buf, Prune prune, Leaf leaf) {
    float ox = r0.ox, oy = r0.oy, oz = r0.oz;
    node_space<true>(A, ox, oy, oz);
    auto inv = [&](float d) {
        d *= A.hn_scale;
        return __frcp_rn(fabsf(d) > 1e-30f ? d : copysignf(1e-30f, d));
    };
    const float ix = inv(r0.dx), iy = inv(r0.dy), iz = inv(r0.dz);
    const float oxi = ox * ix, oyi = oy * iy, ozi = oz * iz;
    const uint32_t lane = __lane_id();
    int* cur = buf;
    int* nxt = buf + kCoopCap;
    int* lv = buf + 2 * kCoopCap;
    if (lane == 0) cur[0] = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t n = 1;
    while (n > 0) {
        uint32_t nn = 0, nl = 0;
        for (uint32_t base = 0; base < n; base += 64u) {
            const bool valid = base + lane < n;
            float key[4];
            int32_t kr[4] = {0, 0, 0, 0};
            if (valid) wide_children<Prune, false>(A, cur[base + lane], ix, iy, iz, oxi, oyi, ozi, prune, key, kr);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t bi = __ballot(kr[k] > 0), bl = __ballot(kr[k] < 0);
                const uint32_t ci = (uint32_t)__popcll(bi), cl = (uint32_t)__popcll(bl);
                if (nn + ci > kCoopCap || nl + cl > kCoopCap) return false;
                const uint64_t below = (1ull << lane) - 1ull;
                if (kr[k] > 0) nxt[nn + (uint32_t)__popcll(bi & below)] = kr[k];
                if (kr[k] < 0) lv[nl + (uint32_t)__popcll(bl & below)] = kr[k];
                nn += ci;
                nl += cl;
            }
        }
        __builtin_amdgcn_wave_barrier();
        for (uint32_t base = 0; base < nl; base += 64u)
            if (base + lane < nl) {
                const int32_t ref = lv[base + lane];
                for (uint32_t j = leaf_first(ref); j < leaf_first(ref) + leaf_count(ref); ++j) leaf(j);
            }
        __builtin_amdgcn_wave_barrier();
        int* t = cur;
        cur = nxt;
        nxt = t;
        n = nn;
    }
    return true;
}

// light_transmittance with the wave on one ray (test_integrators.h:202-237): the three passes as there.
template <bool S>
__device__ float light_transmittance_coop(const RenderArgs& A, const Ray& sr, float dist, const ActList& act, int* buf,
                                          Ctr& c, bool& ok) {
    ok = true;
    if (!(dist > 0.0f)) return 1.0f;
    const GaussianRecord* __restrict__ G = A.gauss;
    const float pad = kTPad * (1.0f + dist);
    float tau = 0.0f;
    bool needs_stop = false;
    uint64_t hitmask = 0;
    ok = coop_walk(
        A, sr, buf, [&](float tmin, float) { return tmin <= dist + pad; },
        [&](uint32_t j) {
            if constexpr (S) c.v[kCtrPrims]++;
            const GRec g = load_rec(G, (int)j);
            const Quad q = quad(g, sr);
            float a, b;
            if (!intersect(q, a, b)) return;
            const int slot = act.find((int)j);
            float lo = a;
            if (slot >= 0) {
                lo = 0.0f;
                hitmask |= slot_bit(slot);
            }
            if (b < dist) {
                if constexpr (S) c.v[kCtrOD]++;
                tau += optical_depth(g, q, lo, b);
            } else if (lo < dist) {
                needs_stop = true;
            }
        });
    if (!ok) return 0.0f;
    tau = wave_sum(tau);
    hitmask = wave_or(hitmask);
    needs_stop = __any(needs_stop);
    if (tau >= kTauCut) return 0.0f;  // exp(-tau) == 0 exactly; later terms are >= 0
    const uint64_t all = act.n >= 64 ? ~0ull : ((1ull << act.n) - 1ull);
    uint64_t missed = all & ~hitmask;
    bool deep_any = false;
    if (act.n > 64) {  // a member is missed iff the ray does not intersect it
        missed = 0;
        for (int s = 0; s < act.n && !deep_any; ++s) {
            float a, b;
            deep_any = !intersect(quad(load_rec(G, act.get(s)), sr), a, b);
        }
    }
    if (needs_stop || missed || deep_any) {
        float tstop = INFINITY;  // first event at or beyond the light
        ok = coop_walk(
            A, sr, buf, [&](float, float tmax) { return tmax >= dist - pad; },
            [&](uint32_t j) {
                if constexpr (S) c.v[kCtrPrims]++;
                const GRec g = load_rec(G, (int)j);
                float a, b;
                if (!intersect(quad(g, sr), a, b)) return;
                if (b >= dist) tstop = fminf(tstop, (a >= dist) ? a : b);
            });
        if (!ok) return 0.0f;
        tstop = wave_min(tstop);
        if (tstop == INFINITY) tstop = dist;
        if (needs_stop) {
            float t3 = 0.0f;
            ok = coop_walk(
                A, sr, buf, [&](float tmin, float tmax) { return tmin <= dist + pad && tmax >= dist - pad; },
                [&](uint32_t j) {
                    if constexpr (S) c.v[kCtrPrims]++;
                    const GRec g = load_rec(G, (int)j);
                    const Quad q = quad(g, sr);
                    float a, b;
                    if (!intersect(q, a, b)) return;
                    const float lo = act.find((int)j) >= 0 ? 0.0f : a;
                    if (lo < dist && b >= dist) {
                        if constexpr (S) c.v[kCtrOD]++;
                        t3 += optical_depth(g, q, lo, tstop);
                    }
                });
            if (!ok) return 0.0f;
            tau += wave_sum(t3);
        }
        while (missed) {
            const int s = __ffsll((unsigned long long)missed) - 1;
            missed &= missed - 1;
            const GRec g = load_rec(G, act.get(s));
            tau += optical_depth(g, quad(g, sr), 0.0f, tstop);
        }
        if (deep_any)
            for (int s = 0; s < act.n; ++s) {
                const GRec g = load_rec(G, act.get(s));
                const Quad q = quad(g, sr);
                float a, b;
                if (!intersect(q, a, b)) tau += optical_depth(g, q, 0.0f, tstop);
            }
    }
    return expf(-tau);
}

// env_transmittance with the wave on one ray (test_integrators.h:242-271).
template <bool S>
__device__ float env_transmittance_coop(const RenderArgs& A, const Ray& er, const ActList& act, int* buf, Ctr& c, bool& ok) {
    const GaussianRecord* __restrict__ G = A.gauss;
    float tau = 0.0f, t_last = 0.0f;
    uint64_t hitmask = 0;
    ok = coop_walk(
        A, er, buf, [&](float, float) { return true; },
        [&](uint32_t j) {
            if constexpr (S) c.v[kCtrPrims]++;
            const GRec g = load_rec(G, (int)j);
            const Quad q = quad(g, er);
            float a, b;
            if (!intersect(q, a, b)) return;
            t_last = fmaxf(t_last, b);
            const int slot = act.find((int)j);
            if (slot >= 0) hitmask |= slot_bit(slot);
            if constexpr (S) c.v[kCtrOD]++;
            tau += optical_depth(g, q, slot >= 0 ? 0.0f : a, b);
        });
    if (!ok) return 0.0f;
    tau = wave_sum(tau);
    t_last = wave_max(t_last);
    hitmask = wave_or(hitmask);
    for (int s = 0; s < act.n; ++s) {  // members the ray misses: active to the last event
        if (s < 64 && ((hitmask >> s) & 1ull)) continue;
        const GRec g = load_rec(G, act.get(s));
        const Quad q = quad(g, er);
        float a, b;
        if (s >= 64 && intersect(q, a, b)) continue;
        tau += optical_depth(g, q, 0.0f, t_last);
    }
    return expf(-tau);
}

// ---------------------------------------------------------------------------------------------
// Stage 1: primary march
// ---------------------------------------------------------------------------------------------
// Early-out weight (t_eps > 0). Stopping after step k drops
//   sum_{j>k} T_j sigma_s,j dt (Li_j + Le_j) / (4 pi) + T_end env
// and T_j sigma_s,j dt is not bounded by T alone: the reference's point-sampled estimator can
// weigh a step by sigma_t dt >> 1 inside an opaque blob (C4's blobs carry tau ~ 400 per chord).
// With every Tr <= 1 a record adds at most T sigma_s dt W per channel, W = max_c (sum_l I_lc /
// (4 pi d_l^2) + env_c), and for exponentially falling T the tail sums to <= T_{k+1} W (1 +
// sigma_t,k+1 dt). The ray therefore stops once T (1 + sigma_t,k dt) W <= t_eps: this step's
// point density stands in for the next one's (one step of look-ahead), so a ray inside a dense
// blob takes the extra step that drives T to 0 instead of dropping it.
__device__ __forceinline__ float tail_weight(const RenderArgs& A, float x, float y, float z, float sigma_t) {
    float w0 = fabsf(A.env[0]), w1 = fabsf(A.env[1]), w2 = fabsf(A.env[2]);
    for (int l = 0; l < A.num_lights; ++l) {
        const LightRecord& lr = A.lights[l];
        const float dx = lr.px - x, dy = lr.py - y, dz = lr.pz - z;
        const float s = kInv4Pi / (dx * dx + dy * dy + dz * dz);
        w0 += fabsf(lr.ix) * s;
        w1 += fabsf(lr.iy) * s;
        w2 += fabsf(lr.iz) * s;
    }
    return fmaxf(fmaxf(w0, w1), w2) * (1.0f + sigma_t * A.step_size);
}

// One step k of a pixel's march once its entrants are in `act` (test_integrators.h:202-289): retire
// the Gaussians that exited (b <= t_k), sigma at the position (gmm.h:98-126), the step's optical depth
// (:146-157), a scatter record if sigma_s > 0, T. Returns false once the march ends (T == 0 or the
// early-out). COOP: one pixel per wave (see march).
template <bool S, bool COOP>
__device__ __forceinline__ bool march_step(const RenderArgs& A, const Ray& ray, uint32_t p, int px, int py, int k, float t_k,
                                           ActList& act, float& T, uint32_t& prev, Ctr& c, bool writer) {
    const GaussianRecord* __restrict__ G = A.gauss;
    const float step = A.step_size;
    // retire (b <= t_k); sigma at pos (gmm.h:98-126); the step's optical depth (:146-157)
    const float px_ = ray.ox + t_k * ray.dx;
    const float py_ = ray.oy + t_k * ray.dy;
    const float pz_ = ray.oz + t_k * ray.dz;
    const float t_k1 = t_k + step;  // `t + step_size` (test_integrators.h:286)
    float smu = 0.0f, smua = 0.0f, tau_seg = 0.0f;
    int w = 0;
    bool bnd = false;  // a member's 3-sigma surface passes within the band of the position (kRecBoundary)
    if constexpr (COOP) {
        const int lane = (int)__lane_id();
        for (int i0 = 0; i0 < act.n; i0 += 64) {  // (compaction writes stay below i0 + 64)
            const int i = i0 + lane;
            int j = 0;
            bool surv = false;
            float m = 0.0f, ma = 0.0f, od = 0.0f;
            if (i < act.n) {
                j = act.get(i);
                GRec g = load_rec(G, j);
                Quad q = quad(g, ray);
                float a, b;
                if (intersect(q, a, b) && b > t_k) {
                    surv = true;
                    float ex;
                    m = mu_t(g, px_, py_, pz_, &ex);
                    bnd = bnd || -2.0f * ex > 9.0f - 2.0f * kMemberAmb;
                    ma = m * g.albedo;
                    if (!A.pure) od = optical_depth(g, q, t_k, t_k1);
                }
            }
            bnd = __ballot(bnd) != 0ull;
            for (uint64_t sm = __ballot(surv); sm; sm &= sm - 1) {  // survivors in list order
                const int sl = __ffsll((unsigned long long)sm) - 1;
                act.set(w++, __shfl(j, sl, 64));
                smu += __shfl(m, sl, 64);
                smua += __shfl(ma, sl, 64);
                if (!A.pure) tau_seg += __shfl(od, sl, 64);
                if constexpr (S && !kDiagUnion) {
                    c.v[kCtrMu]++;
                    c.v[kCtrOD]++;
                    c.v[kCtrPrims]++;
                }
            }
        }
    } else {
        for (int i = 0; i < act.n; ++i) {
            int j = act.get(i);
            GRec g = load_rec(G, j);
            Quad q = quad(g, ray);
            float a, b;
            if (!intersect(q, a, b) || b <= t_k) continue;
            act.set(w++, j);
            float ex;
            float m = mu_t(g, px_, py_, pz_, &ex);
            bnd = bnd || -2.0f * ex > 9.0f - 2.0f * kMemberAmb;
            smu += m;
            smua += m * g.albedo;
            if (!A.pure) tau_seg += optical_depth(g, q, t_k, t_k1);
            if constexpr (S && !kDiagUnion) {
                c.v[kCtrMu]++;
                c.v[kCtrOD]++;
                c.v[kCtrPrims]++;
            }
        }
    }
    act.n = w;
    if (w == 0) return true;
    if constexpr (S && !kDiagUnion) c.v[kCtrSteps]++;
    float sigma_s = 0.0f;
    if (smu > 0.0f) {
        float a_mix = smua / smu;
        sigma_s = a_mix * smu;
    }
    if (sigma_s > 0.0f) {  // scattering step -> one record
        uint32_t r, o = 0;
        if constexpr (COOP) {  // one pixel per wave: lane 0 allocates
            uint32_t base = 0;
            if (writer) {
                base = atomicAdd(&A.rec_alloc[0], 1u);
                if (w > kActInline) o = atomicAdd(&A.rec_alloc[1], (uint32_t)w);
            }
            r = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
            o = (uint32_t)__builtin_amdgcn_readfirstlane((int)o);
        } else {
            // lanes emitting now share one atomic (this branch is divergent: ballot = them)
            const uint64_t m = __ballot(true);
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
            uint32_t base = 0;
            if (__lane_id() == leader) base = atomicAdd(&A.rec_alloc[0], (uint32_t)__popcll(m));
            base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);
            r = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (w > kActInline) o = atomicAdd(&A.rec_alloc[1], (uint32_t)w);  // rare: the overflow pool
        }
        uint32_t aoff = r * (uint32_t)kActInline;
        bool fits = r < A.rec_cap;
        if (w > kActInline) {  // long active lists go to the overflow pool
            aoff = A.rec_cap * (uint32_t)kActInline + o;
            fits = fits && o + (uint32_t)w <= A.act_ovf_cap;
        }
        if (fits) {
            uint64_t bl = 0;
            for (int i = 0; i < w; ++i) {
                const int j = act.get(i);
                if (COOP ? (i & 63) == (int)__lane_id() : true) A.rec_act[aoff + i] = j;
                bl |= 1ull << (j & 63);
            }
            if (writer) {
                A.rec_pos[r] = make_float4(px_, py_, pz_, T * sigma_s);
                A.rec_meta[r] = make_uint4((uint32_t)px | ((uint32_t)py << 16), (uint32_t)k, aoff,
                                           (uint32_t)w | (bnd && kMemberAmb > 0.0f ? kRecBoundary : 0u));
                A.rec_bloom[r] = bl;
                A.rec_next[r] = kNoRecord;
                if (prev == kNoRecord) A.px_first[p] = r;
                else A.rec_next[prev] = r;
            }
            prev = r;
        } else if (writer) {
            A.rec_alloc[2] = 1u;  // capacity exceeded: the frame is reported and rendered again
            if (r < A.rec_cap) {  // a slot inside [0, nrec) whose active list did not fit the pool:
                // the later stages still read it (the host does not wait for the march), so
                // it must be a valid record, not the previous frame's: an empty one
                A.rec_pos[r] = make_float4(px_, py_, pz_, 0.0f);
                A.rec_meta[r] = make_uint4((uint32_t)px | ((uint32_t)py << 16), (uint32_t)k, 0u, 0u);
                A.rec_bloom[r] = 0ull;
                A.rec_next[r] = kNoRecord;
            }
        }
    }
    if (A.pure) {  // integrator.h:196-198, 259: T *= exp(-sigma_t * step), sigma_t = sigma_a + sigma_s
        float sa = 0.0f, ss = 0.0f;
        if (smu > 0.0f) {
            const float a_mix = smua / smu;
            ss = a_mix * smu;
            sa = (1.0f - a_mix) * smu;
        }
        T *= expf(-(sa + ss) * step);
    } else {
        T *= expf(-tau_seg);
    }
    if (T <= 0.0f) return false;  // exact: nothing after this step can add to L or to T * env
    return !(A.t_eps > 0.0f && T * tail_weight(A, px_, py_, pz_, smu) <= A.t_eps);
}

// One pass: each scattering step allocates its record with a wave-aggregated atomic and links it
// to the pixel's previous record (px_first / rec_next), so a pixel's records are visited in step
// order by accumulate_kernel wherever they landed in memory. Records that do not fit the
// capacity raise rec_alloc[2]; the host then grows the buffers and re-runs the march.
// W: BVH window queries on the 4-wide half-precision tree (CAP-entry stack; a query that could
// overflow it sends the pixel to the fallback kernel, which walks the pair tree).
// COOP: the whole wave marches the same pixel (the fallback passes: a pixel whose active set
// outgrew the fast kernel's slots marches serially for a long time). Every lane runs the same
// queries and keeps its own identical copy of the active list; only the per-step evaluation of the
// active list is split over the lanes (one Gaussian each), its sums and compaction then taken in
// list order through lane broadcasts — the serial loop's operations in its order, so the result is
// bit-identical — and lane 0 writes the records.
#ifdef VR_DIAG_UNION
// Diagnostic builds only (with vr_count_work): what a wave-coherent walk of the march's window queries would cost.
// At every query call, the lanes running the query this iteration walk the 4-wide tree as one wave: a node is
// fetched once for the wave (wave-uniform stack in LDS) and descended into if any lane's box test and prune keep
// it (ballot). Counted per call, in the march counters' slots: kCtrSecRays += union node visits, kCtrMu += union
// leaf visits, kCtrOD += the per-lane walk's node-fetch passes (the largest per-lane node-step count among the
// calling lanes: what the SIMT walk's loop runs), kCtrSteps += calls; kCtrNodes keeps the per-lane node steps.
template <typename Prune>
__device__ void union_walk_count(const RenderArgs& A, const Ray& r0, Prune prune, Ctr& c) {
    __shared__ int ustack[256];  // (march workgroups are one wave)
    float ox = r0.ox, oy = r0.oy, oz = r0.oz;
    node_space<true>(A, ox, oy, oz);
    auto inv = [&](float d) {
        d *= A.hn_scale;
        return __frcp_rn(fabsf(d) > 1e-30f ? d : copysignf(1e-30f, d));
    };
    const float ix = inv(r0.dx), iy = inv(r0.dy), iz = inv(r0.dz);
    const float oxi = ox * ix, oyi = oy * iy, ozi = oz * iz;
    const uint64_t act = __ballot(1);
    const bool first_lane = __lane_id() == (uint32_t)(__ffsll((unsigned long long)act) - 1);
    uint32_t visits = 0, leaves = 0;
    int sp = 0, node = 0;
    for (;;) {
        ++visits;
        float key[4];
        int32_t kr[4];
        wide_children<Prune, false>(A, node, ix, iy, iz, oxi, oyi, ozi, prune, key, kr);
        const int4 rf = reinterpret_cast<const int4*>(A.hnodes4 + node)[3];
        const int32_t ref[4] = {rf.x, rf.y, rf.z, rf.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool any = __ballot(kr[i] != 0) != 0ull;
            if (!any) continue;
            if (ref[i] < 0) {
                ++leaves;
            } else if (sp < 256) {
                if (first_lane) ustack[sp] = ref[i];
                ++sp;
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (sp == 0) break;
        --sp;
        node = __builtin_amdgcn_readfirstlane(ustack[sp]);
    }
    if (first_lane) {
        c.v[kCtrSecRays] += visits;
        c.v[kCtrMu] += leaves;
        c.v[kCtrSteps] += 1u;
    }
}
// Largest per-lane value among the calling lanes (bit-sliced ballots), added once.
__device__ __forceinline__ void union_walk_simt(uint32_t steps, Ctr& c) {
    const uint64_t act = __ballot(1);
    uint32_t m = 0;
    for (int b = 15; b >= 0; --b)
        if (__ballot(steps >= (m | (1u << b))) != 0ull) m |= 1u << b;
    if (__lane_id() == (uint32_t)(__ffsll((unsigned long long)act) - 1)) c.v[kCtrOD] += m;
}
#endif

// (Measured and not kept, DESIGN.md §3: window queries starting in the subtree holding the window and climbing,
// a fast-form pre-test of the candidates, look-ahead windows over 2-4 steps, a closest-entry query merged with
// the following entrant query, a sorting network in the entrant walk; all bit-identical, all slower at C4.)
template <int ACT, bool S, bool H, bool W = false, int CAP = kStackSize, bool COOP = false, int DEEP = 0>
__device__ int march(const RenderArgs& A, uint32_t p, int px, int py, int* act_base, int* stack, int stride, Ctr& c,
                     int act_stride = -1) {
    const bool writer = !COOP || __lane_id() == 0u;  // COOP: lane 0 writes the pixel's records
    const Ray ray = primary_ray(A, px, py);
    const GaussianRecord* __restrict__ G = A.gauss;
    const float* __restrict__ ts = A.tsteps;
    const int nts = A.num_tsteps;
    const float step = A.step_size;
    float T = 1.0f;
    uint32_t prev = kNoRecord;  // this pixel's last record
    if (writer) A.px_first[p] = kNoRecord;
    ActList act{act_base, act_stride < 0 ? stride : act_stride, 0, 0};
    auto walk = [&](auto prune, auto leaf) -> bool {
        if constexpr (W) {
            return traverse_wide<CAP, decltype(prune), decltype(leaf), NodeCount<S>, true, DEEP>(A, ray, stack, stride, prune, leaf,
                                                                                                NodeCount<S>{&c});
        } else {
            traverse<H>(A, ray, stack, stride, prune, leaf, NodeCount<S>{&c});
            return true;
        }
    };
    // the entrants query collects every entry of (t_lo, t_k] whatever the visit order: no sorting network
    auto walk_any = [&](auto prune, auto leaf) -> bool {
        if constexpr (W) {
            return traverse_wide<CAP, decltype(prune), decltype(leaf), NodeCount<S>, false, DEEP>(A, ray, stack, stride, prune, leaf,
                                                                                                    NodeCount<S>{&c});
        } else {
            return walk(prune, leaf);
        }
    };
    int kq = 0;
    if (A.num_prims > 0) {
        for (;;) {
            float t_lo = (kq == 0) ? -1.0f : ts[kq - 1];
            int k;
            if (act.n == 0) {  // closest entry strictly after t_lo
                if constexpr (S) c.v[kCtrPrimQueries]++;
                float best = INFINITY;
                auto prune_c = [&](float tmin, float tmax) {
                    return tmax >= t_lo - kTPad * (1.0f + fabsf(t_lo)) && tmin <= best + kTPad * (1.0f + best);
                };
                auto leaf_c = [&](uint32_t first, uint32_t count) {
                    for (uint32_t j = first; j < first + count; ++j) {
                        if constexpr (S) c.v[kCtrPrims]++;
                        GRec g = load_rec(G, j);
                        Quad q = quad(g, ray);
                        float a, b;
                        if (!intersect(q, a, b) || !(a > t_lo)) continue;
                        if (a < best) best = a;
                    }
                    return true;
                };
#ifdef VR_DIAG_UNION
                if constexpr (S && W && !COOP) union_walk_count(A, ray, prune_c, c);
                const uint32_t n0 = c.v[kCtrNodes];
#endif
                if (!walk(prune_c, leaf_c)) return kOverflow;
#ifdef VR_DIAG_UNION
                if constexpr (S && W && !COOP) union_walk_simt(c.v[kCtrNodes] - n0, c);
#endif
                if (best == INFINITY) break;
                k = kfirst(ts, nts, step, best);
                // No entry lies in (t_lo, best) and ts[k - 1] < best: the step's entrant window (t_lo, t_k] holds
                // exactly the entries of (ts[k - 1], t_k]. The short window keeps the query local to the step
                // (from t_lo = -1 the first query of every pixel walked every box along [0, t_k]). Same set.
                if (k > kq) t_lo = ts[k - 1];
            } else {
                k = kq;
            }
            if (k >= nts - 1) return kError;  // step table too short (host sizes it from scene bounds)
            const float t_k = ts[k];
            bool ovf = false;
            // entrants: t_lo < a <= t_k and still inside at t_k (b > t_k)
            if constexpr (S) c.v[kCtrPrimQueries]++;
            auto prune_w = [&](float tmin, float tmax) {
                return tmax >= t_lo - kTPad * (1.0f + fabsf(t_lo)) && tmin <= t_k + kTPad * (1.0f + t_k);
            };
#ifdef VR_DIAG_UNION
            if constexpr (S && W && !COOP) union_walk_count(A, ray, prune_w, c);
            const uint32_t n1 = c.v[kCtrNodes];
#endif
            const bool ok = walk_any(
                prune_w,
                [&](uint32_t first, uint32_t count) {
                    for (uint32_t j = first; j < first + count; ++j) {
                        if constexpr (S) c.v[kCtrPrims]++;
                        GRec g = load_rec(G, j);
                        Quad q = quad(g, ray);
                        float a, b;
                        if (!intersect(q, a, b) || !(a > t_lo) || !(a <= t_k)) continue;
                        if (!(b > t_k)) continue;
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
                    return true;
                });
#ifdef VR_DIAG_UNION
            if constexpr (S && W && !COOP) union_walk_simt(c.v[kCtrNodes] - n1, c);
#endif
            if (ovf || !ok) return kOverflow;
            kq = k + 1;
            if (!march_step<S, COOP>(A, ray, p, px, py, k, t_k, act, T, prev, c, writer)) break;
        }
    }
    if (writer) A.px_T[p] = T;
    if constexpr (S) c.v[kCtrPixels]++;
    return kOK;
}

__device__ __forceinline__ void mark_error(const RenderArgs& A, uint32_t p) {
    atomicAdd(A.counters, 1u);
    A.px_T[p] = __builtin_nanf("");
}

// A pixel that overflowed a pass is marched again from its start by the next pass, which relinks it;
// the records this pass already wrote for it are unreachable. Their weight T sigma_s (rec_pos.w, >= 0 for
// every live record) is set to the sentinel -1 so the secondary stage starts none of their rays (sec_init).
constexpr float kOrphanWeight = -1.0f;  // rec_pos.w of an orphaned record (a live record's T sigma_s is >= 0)
__device__ __forceinline__ void orphan_records(const RenderArgs& A, uint32_t p) {
    for (uint32_t r = A.px_first[p]; r != kNoRecord && r < A.rec_cap; r = A.rec_next[r])
        reinterpret_cast<float*>(A.rec_pos + r)[3] = kOrphanWeight;
}

template <int ACT, int BLOCK, bool S, int STACK, bool H, bool W = false>
__global__ __launch_bounds__(BLOCK) void march_kernel(RenderArgs A) {
    __shared__ int s_act[ACT * BLOCK];
    __shared__ int s_stack[STACK * BLOCK];
    // A workgroup is one 16x16 tile (BLOCK 256) or one of its 8x8 quarters (BLOCK 64: four times as
    // many, shorter workgroups, so the frame's last ones leave a shorter tail). Lanes never share LDS.
    constexpr uint32_t kParts = 256u / BLOCK;
    const uint32_t q = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t tile_local = q / kParts;
    const int tid = (int)((q % kParts) * BLOCK + threadIdx.x);  // lane within the tile
    const uint32_t p = tile_local * 256u + (uint32_t)tid;
    int lx, ly, x, y;
    tile_pixel(A, tile_local, tid, lx, ly, x, y);
    Ctr c{};
    int st = kOK;
    if (x < (int)A.width && y < (int)A.height) {
        st = march<ACT, S, H, W, STACK, false, W ? VR_MARCH_DEEP : 0>(A, p, x, y, s_act + threadIdx.x, s_stack + threadIdx.x, BLOCK, c);
    } else {
        A.px_first[p] = kNoRecord;
        A.px_T[p] = 0.0f;
    }
    if constexpr (S) flush_counters(A.work, c);
    if (st == kOverflow) {
        orphan_records(A, p);
        uint32_t slot = atomicAdd(A.queue, 1u);
        if (slot < A.queue_cap) A.queue[1 + slot] = p;
        else mark_error(A, p);
    } else if (st == kError) {
        mark_error(A, p);
    }
}

// The fallback passes march one pixel per wave (march<COOP>): a pixel lands here because its active
// set is large, and its serial march was the tail of the whole march stage (~1 ms at C4, also for a
// 1/8 multi-GPU share). BLOCK = one wave.
template <int ACT, int BLOCK, bool S, bool H, bool W = false>
__global__ __launch_bounds__(BLOCK) void march_fallback_kernel(RenderArgs A) {
    static_assert(BLOCK == 64, "one pixel per wave");
    __shared__ int s_act[ACT * BLOCK];
    __shared__ int s_stack[kStackSize * BLOCK];
    const int tid = threadIdx.x;
    const uint32_t n = min(A.queue[0], A.queue_cap);
    if (n >= A.wide_min) return;  // a long queue: march_wide_kernel takes it (one pixel per lane)
    for (uint32_t q = blockIdx.x; q < n; q += gridDim.x) {
        const uint32_t p = A.queue[1 + q];
        int lx, ly, x, y;
        tile_pixel(A, p >> 8, (int)(p & 255u), lx, ly, x, y);
        Ctr c{};
        // (W: the 4-wide walks — half the dependent node fetches of the pair tree on a single pixel's
        // serial queries; a walk past the kStackSize stack goes to the deep pass)
        int st = march<ACT, S, H, W, kStackSize, true>(A, p, x, y, s_act + tid, s_stack + tid, BLOCK, c);  // re-links px_first
        if (tid != 0) continue;
        if constexpr (S)
            for (int i = 0; i < kNumCtr; ++i) atomicAdd(A.work + i, (unsigned long long)c.v[i]);
        if (st == kOverflow) {  // more than ACT Gaussians active at one step: the deep pass
            orphan_records(A, p);
            const uint32_t slot = atomicAdd(A.deepq, 1u);
            if (slot < A.deepq_cap) A.deepq[1 + slot] = p;
            else mark_error(A, p);
        } else if (st != kOK) {
            mark_error(A, p);
        }
    }
}

// A long fallback queue (translucent scenes with many overlapping Gaussians: C2 sends most pixels here)
// one pixel per lane: the main kernel's march with kActWide active-list slots per lane in global memory
// ([slot][thread] rows, coalesced over a wave's lanes) instead of 16 in LDS. One wave per pixel
// (march_fallback_kernel) shortens a single pixel's march but runs the queue 64x narrower; it keeps
// queues shorter than A.wide_min (C4: 833 pixels). Same march<> operations as every other pass, so
// a pixel's records do not depend on which pass marched it. Overflow (more than kActWide active, or a
// 4-wide walk past its stack): the deep pass.
template <bool S, bool H, bool W>
__global__ __launch_bounds__(kWideBlock) void march_wide_kernel(RenderArgs A) {
    __shared__ int s_stack[kStackSize * kWideBlock];
    const int tid = threadIdx.x;
    const uint32_t gt = blockIdx.x * kWideBlock + tid, nthreads = gridDim.x * kWideBlock;
    const uint32_t n = min(A.queue[0], A.queue_cap);
    if (n < A.wide_min) return;
    Ctr c{};
    for (uint32_t q = gt; q < n; q += nthreads) {
        const uint32_t p = A.queue[1 + q];
        int lx, ly, x, y;
        tile_pixel(A, p >> 8, (int)(p & 255u), lx, ly, x, y);
        const int st = march<kActWide, S, H, W, kStackSize>(A, p, x, y, A.wide_act + gt, s_stack + tid, kWideBlock, c, (int)nthreads);
        if (st == kOverflow) {
            orphan_records(A, p);
            const uint32_t slot = atomicAdd(A.deepq, 1u);
            if (slot < A.deepq_cap) A.deepq[1 + slot] = p;
            else mark_error(A, p);
        } else if (st != kOK) {
            mark_error(A, p);
        }
    }
    if constexpr (S) flush_counters(A.work, c);
}

// Pixels whose active set outgrew the fallback's 64 LDS slots: the same march with the active list in
// global memory (kActDeep slots per lane, [slot][thread] rows, one pixel per wave).
// Only an active set past kActDeep, Gaussians overlapping one point, fails (NaN, VR_ERR_OVERFLOW).
template <bool S, bool H>
__global__ __launch_bounds__(kDeepBlock) void march_deep_kernel(RenderArgs A) {
    static_assert(kDeepBlock == 64, "one pixel per wave");
    __shared__ int s_stack[kStackSize * kDeepBlock];
    const int tid = threadIdx.x;
    const uint32_t gt = blockIdx.x * kDeepBlock + tid, nthreads = gridDim.x * kDeepBlock;
    const uint32_t n = min(A.deepq[0], A.deepq_cap);
    for (uint32_t q = blockIdx.x; q < n; q += gridDim.x) {
        const uint32_t p = A.deepq[1 + q];
        int lx, ly, x, y;
        tile_pixel(A, p >> 8, (int)(p & 255u), lx, ly, x, y);
        Ctr c{};
        const int st =
            march<kActDeep, S, H, false, kStackSize, true>(A, p, x, y, A.deep_act + gt, s_stack + tid, kDeepBlock, c, (int)nthreads);
        if (tid != 0) continue;
        if constexpr (S)
            for (int i = 0; i < kNumCtr; ++i) atomicAdd(A.work + i, (unsigned long long)c.v[i]);
        if (st != kOK) mark_error(A, p);
    }
}

// ---------------------------------------------------------------------------------------------
// Stage 1, binned variant (VR_OPT_MARCH_BINNED; A/B against the BVH window queries):
// every record is binned to the 16x16 tiles its 3.15-sigma box can project onto, by a depth bucket of
// a lower bound of the entry distance of the tile's pixel rays; a quarter-tile wave then streams its
// tile's entries bucket by bucket (wave-uniform: scalar loads of index and record), tests each against
// every lane's ray with the exact intersect, keeps the hits that have not entered yet in a per-lane
// pending list sorted by entry distance, and marches every step that lies before the next bucket's
// lower bound (no later entry can enter at or before it). The active lists, steps and records are
// those of march(): the same intersect decides every entry, the same march_step evaluates.
// ---------------------------------------------------------------------------------------------
#ifndef VR_BIN_PEND
#define VR_BIN_PEND 48
#endif
constexpr int kPendCap = VR_BIN_PEND;  // pending entries per lane (more: the pixel re-runs in march_fallback_kernel)
constexpr int kBinAct = 16;      // active Gaussians per lane (as march_kernel's)

// The pixel rectangle (inclusive, clamped to the frame) that the box [lo, hi] can project onto, and
// false if it projects onto nothing; all = true when the box reaches the pinhole's side of the image
// plane (then every tile).
__device__ __forceinline__ bool bin_rect(const RenderArgs& A, const float* lo, const float* hi, int& x0, int& x1, int& y0,
                                         int& y1) {
    const float* R = A.cam_right;
    const float* U = A.cam_up;
    const float n0 = R[1] * U[2] - R[2] * U[1], n1 = R[2] * U[0] - R[0] * U[2], n2 = R[0] * U[1] - R[1] * U[0];
    const float rr = R[0] * R[0] + R[1] * R[1] + R[2] * R[2], uu = U[0] * U[0] + U[1] * U[1] + U[2] * U[2];
    float umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY;
    bool all = false;
    for (int c = 0; c < 8; ++c) {
        const float X[3] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]};
        float o[3];
        if (A.cam_type == 0) {  // the ray from o passes through the pinhole P: o = P + s (X - P) on the plane
            const float* P = A.cam_pinhole;
            const float pn = (P[0] - A.cam_pos[0]) * n0 + (P[1] - A.cam_pos[1]) * n1 + (P[2] - A.cam_pos[2]) * n2;
            const float xn = (X[0] - P[0]) * n0 + (X[1] - P[1]) * n1 + (X[2] - P[2]) * n2;
            if (!(xn * pn > 1e-6f * fabsf(pn) * (fabsf(pn) + fabsf(xn)))) {  // not strictly beyond the pinhole
                all = true;
                break;
            }
            const float sc = -pn / xn;
            for (int k = 0; k < 3; ++k) o[k] = P[k] + sc * (X[k] - P[k]);
        } else {  // orthographic: along the view direction onto the plane
            const float* V = A.cam_view;
            const float vn = V[0] * n0 + V[1] * n1 + V[2] * n2;
            if (!(fabsf(vn) > 0.0f)) {
                all = true;
                break;
            }
            const float lam = ((X[0] - A.cam_pos[0]) * n0 + (X[1] - A.cam_pos[1]) * n1 + (X[2] - A.cam_pos[2]) * n2) / vn;
            for (int k = 0; k < 3; ++k) o[k] = X[k] - lam * V[k];
        }
        const float d0 = o[0] - A.cam_pos[0], d1 = o[1] - A.cam_pos[1], d2 = o[2] - A.cam_pos[2];
        const float u = (d0 * R[0] + d1 * R[1] + d2 * R[2]) / rr, v = (d0 * U[0] + d1 * U[1] + d2 * U[2]) / uu;
        umin = fminf(umin, u);
        umax = fmaxf(umax, u);
        vmin = fminf(vmin, v);
        vmax = fmaxf(vmax, v);
    }
    const float W = (float)A.width, H = (float)A.height;
    float fx0, fx1, fy0, fy1;
    if (all) {
        fx0 = fy0 = 0.0f;
        fx1 = W;
        fy1 = H;
    } else if (A.cam_type == 0) {  // u = 1 - 2 (x + .5) / W, v = 2 (y + .5) / H - 1
        fx0 = (1.0f - umax) * 0.5f * W - 0.5f;
        fx1 = (1.0f - umin) * 0.5f * W - 0.5f;
        fy0 = (vmin + 1.0f) * 0.5f * H - 0.5f;
        fy1 = (vmax + 1.0f) * 0.5f * H - 0.5f;
    } else {  // u = 2 (x + .5) / W - 1, v = 1 - 2 (y + .5) / H
        fx0 = (umin + 1.0f) * 0.5f * W - 0.5f;
        fx1 = (umax + 1.0f) * 0.5f * W - 0.5f;
        fy0 = (1.0f - vmax) * 0.5f * H - 0.5f;
        fy1 = (1.0f - vmin) * 0.5f * H - 0.5f;
    }
    // two pixels of slack for rounding (directions, the box's own projection)
    x0 = (int)fmaxf(floorf(fx0) - 2.0f, 0.0f);
    y0 = (int)fmaxf(floorf(fy0) - 2.0f, 0.0f);
    x1 = (int)fminf(ceilf(fx1) + 2.0f, W - 1.0f);
    y1 = (int)fminf(ceilf(fy1) + 2.0f, H - 1.0f);
    return fx1 + 2.0f >= 0.0f && fy1 + 2.0f >= 0.0f && fx0 - 2.0f <= W && fy0 - 2.0f <= H;
}

// 3.15-sigma box of record j (Sigma = M^-1 in double; the intersect's 3-sigma ellipsoid of the f32 M
// lies inside with a 5 % margin, as the BVH boxes).
__device__ __forceinline__ void bin_box(const GaussianRecord& g, float* lo, float* hi) {
    const double m00 = g.m00, m01 = g.m01, m02 = g.m02, m11 = g.m11, m12 = g.m12, m22 = g.m22;
    const double c00 = m11 * m22 - m12 * m12, c11 = m00 * m22 - m02 * m02, c22 = m00 * m11 - m01 * m01;
    const double det = m00 * c00 - m01 * (m01 * m22 - m12 * m02) + m02 * (m01 * m12 - m11 * m02);
    const double s[3] = {c00 / det, c11 / det, c22 / det};
    const float m[3] = {g.mx, g.my, g.mz};
    for (int k = 0; k < 3; ++k) {
        const float e = (float)(3.15 * sqrt(fmax(s[k], 0.0)));
        const bool ok = det > 0.0 && e == e;
        lo[k] = ok ? m[k] - e : -INFINITY;
        hi[k] = ok ? m[k] + e : INFINITY;
    }
}

// Tile tile_local (of this call's strided tile set) if global tile (tx, ty) belongs to it, else -1.
__device__ __forceinline__ int local_tile(const RenderArgs& A, uint32_t tx, uint32_t ty) {
    const uint32_t g = ty * A.tiles_x + tx;
    if (g < A.first_tile) return -1;
    const uint32_t d = g - A.first_tile;
    if (d % A.tile_stride) return -1;
    const uint32_t t = d / A.tile_stride;
    return t < A.num_tiles ? (int)t : -1;
}

// Lower bound of the entry distance into box [lo, hi] of every pixel ray of global tile (tx, ty): the
// distance from the tile's central ray origin less the half diagonal of its origins (|d| = 1, so a
// ray's t is the distance from its origin), less a relative margin for rounding.
__device__ __forceinline__ float bin_key(const RenderArgs& A, uint32_t tx, uint32_t ty, const float* lo, const float* hi,
                                         float hd) {
    const float cx = (float)(tx * kTile) + 0.5f * kTile, cy = (float)(ty * kTile) + 0.5f * kTile;
    const float uvx = cx / (float)A.width, uvy = cy / (float)A.height;
    const float u = A.cam_type == 0 ? 1.0f - 2.0f * uvx : 2.0f * uvx - 1.0f;
    const float v = A.cam_type == 0 ? 2.0f * uvy - 1.0f : 1.0f - 2.0f * uvy;
    float d2 = 0.0f;
    for (int k = 0; k < 3; ++k) {
        const float o = A.cam_pos[k] + u * A.cam_right[k] + v * A.cam_up[k];
        const float e = fmaxf(fmaxf(lo[k] - o, o - hi[k]), 0.0f);
        d2 += e * e;
    }
    return fmaxf((sqrtf(d2) - hd) * (1.0f - 1e-4f) - 1e-4f, 0.0f);
}

__device__ __forceinline__ float bin_half_diag(const RenderArgs& A) {
    const float* R = A.cam_right;
    const float* U = A.cam_up;
    const float du = 2.0f * kTile / (float)A.width * sqrtf(R[0] * R[0] + R[1] * R[1] + R[2] * R[2]);
    const float dv = 2.0f * kTile / (float)A.height * sqrtf(U[0] * U[0] + U[1] * U[1] + U[2] * U[2]);
    return 0.5f * sqrtf(du * du + dv * dv);
}

// EMIT = false: count the entries of every bin; true: write them at bin_off + a cursor per bin.
template <bool EMIT>
__global__ __launch_bounds__(256) void bin_kernel(RenderArgs A) {
    const float hd = bin_half_diag(A);
    const uint32_t nb = A.bin_nb;
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < (uint32_t)A.num_prims; j += gridDim.x * 256u) {
        const GaussianRecord g = A.gauss[j];
        float lo[3], hi[3];
        bin_box(g, lo, hi);
        int x0, x1, y0, y1;
        if (!bin_rect(A, lo, hi, x0, x1, y0, y1)) continue;
        for (uint32_t ty = (uint32_t)y0 / kTile; ty <= (uint32_t)y1 / kTile; ++ty)
            for (uint32_t tx = (uint32_t)x0 / kTile; tx <= (uint32_t)x1 / kTile; ++tx) {
                const int t = local_tile(A, tx, ty);
                if (t < 0) continue;
                const uint32_t b = min(nb - 1u, (uint32_t)(bin_key(A, tx, ty, lo, hi, hd) / A.bin_dz));
                const uint32_t bin = (uint32_t)t * nb + b;
                if constexpr (EMIT) {
                    const uint32_t pos = A.bin_off[bin] + atomicAdd(&A.bin_cnt[bin], 1u);
                    A.bin_out[pos] = j;
                } else {
                    atomicAdd(&A.bin_cnt[bin], 1u);
                }
            }
    }
}

// The binned march of one quarter tile (a wave, one lane per pixel). Returns the per-lane status.
template <bool S>
__global__ __launch_bounds__(64) void march_binned_kernel(RenderArgs A) {
    __shared__ float s_pa[kPendCap * 64];  // pending entries, sorted by entry distance, largest first
    __shared__ int s_pj[kPendCap * 64];
    __shared__ int s_act[kBinAct * 64];
    const uint32_t q = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t tile_local = q >> 2;
    const int lane = (int)threadIdx.x;
    const int tid = (int)((q & 3u) * 64u) + lane;
    const uint32_t p = tile_local * 256u + (uint32_t)tid;
    int lx, ly, x, y;
    tile_pixel(A, tile_local, tid, lx, ly, x, y);
    Ctr c{};
    const bool valid = x < (int)A.width && y < (int)A.height;
    const Ray ray = primary_ray(A, x, y);
    float* pa = s_pa + lane;
    int* pj = s_pj + lane;
    ActList act{s_act + lane, 64, 0, 0};
    float T = 1.0f;
    uint32_t prev = kNoRecord;
    int np = 0, kq = 0, st = kOK;
    float t_lo = -1.0f;
    bool done = !valid;
    if (valid) A.px_first[p] = kNoRecord;
    const float* __restrict__ ts = A.tsteps;
    const int nts = A.num_tsteps;
    // every step before `bound` (no entry of a later bucket can enter at or before it)
    auto march_to = [&](float bound) {
        for (;;) {
            int k;
            if (act.n == 0) {
                if (np == 0) return;
                k = kfirst(ts, nts, A.step_size, pa[(np - 1) * 64]);  // the closest entry after t_lo
            } else {
                k = kq;
            }
            if (k >= nts - 1) {
                st = kError;
                done = true;
                return;
            }
            const float t_k = ts[k];
            if (!(t_k < bound)) return;
            while (np > 0 && pa[(np - 1) * 64] <= t_k) {  // entrants: entered at or before t_k, still inside
                const int j = pj[--np * 64];
                if constexpr (S) c.v[kCtrPrims]++;
                float a, b;
                if (!intersect(quad(load_rec(A.gauss, j), ray), a, b) || !(b > t_k)) continue;
                if (act.n >= kBinAct) {
                    if constexpr (S) c.v[kCtrSecRays]++;  // (instrumented build: overflow causes)
                    st = kOverflow;
                    done = true;
                    return;
                }
                int i = act.n;  // sorted insert (index order, gmm.h:98-126)
                while (i > 0 && act.get(i - 1) > j) {
                    act.set(i, act.get(i - 1));
                    --i;
                }
                act.set(i, j);
                act.n++;
            }
            kq = k + 1;
            t_lo = t_k;
            if (!march_step<S, false>(A, ray, p, x, y, k, t_k, act, T, prev, c, true)) {
                done = true;
                return;
            }
        }
    };
    if (A.num_prims > 0) {
        const uint32_t nb = A.bin_nb;
        const uint32_t* __restrict__ off = A.bin_off + tile_local * nb;
        for (uint32_t b = 0;; ++b) {  // wave-uniform: bucket by bucket
            while (b < nb && off[b] == off[b + 1]) ++b;  // (empty buckets)
            // every entry of bucket b on enters at or after b * dz: march the steps before it first
            if (!done) march_to(b < nb ? (float)b * A.bin_dz : INFINITY);
            if (b >= nb || __ballot(!done) == 0ull) break;
            for (uint32_t pos = off[b]; pos < off[b + 1]; ++pos) {
                const int j = (int)A.bin_ent[pos];
                if (!done) {
                    if constexpr (S) c.v[kCtrPrims]++;
                    float ta, tb;
                    if (intersect(quad(load_rec(A.gauss, j), ray), ta, tb)) {
                        if (!(ta > t_lo)) {  // (a key below its bound: the exact BVH march re-runs the pixel)
                            if constexpr (S) c.v[kCtrPrimQueries]++;
                            st = kOverflow;
                            done = true;
                        } else if (np >= kPendCap) {
                            if constexpr (S) c.v[kCtrNodes]++;
                            st = kOverflow;
                            done = true;
                        } else {
                            int i = np++;  // sorted insert, largest entry distance first
                            while (i > 0 && pa[(i - 1) * 64] < ta) {
                                pa[i * 64] = pa[(i - 1) * 64];
                                pj[i * 64] = pj[(i - 1) * 64];
                                --i;
                            }
                            pa[i * 64] = ta;
                            pj[i * 64] = j;
                        }
                    }
                }
            }
        }
    }
    if (valid && st == kOK) A.px_T[p] = T;
    if constexpr (S) {
        c.v[kCtrPixels] += valid ? 1u : 0u;
        flush_counters(A.work, c);
    }
    if (!valid) {
        A.px_first[p] = kNoRecord;
        A.px_T[p] = 0.0f;
    } else if (st == kOverflow) {
        orphan_records(A, p);
        uint32_t slot = atomicAdd(A.queue, 1u);
        if (slot < A.queue_cap) A.queue[1 + slot] = p;
        else mark_error(A, p);
    } else if (st == kError) {
        mark_error(A, p);
    }
}

// ---------------------------------------------------------------------------------------------
// Stage 2: persistent "while-while" tracing of all secondary rays, per-lane ray refill.
//
// Secondary rays have very uneven lengths (the optical-depth cut-off ends a ray after a few
// dense hits, a ray through empty space walks many nodes), so one ray per lane per round leaves
// most of a wave idle behind its slowest lane. Here every wave owns a contiguous chunk of ray
// ids (sample-major: neighbouring pixels, same light / same env sample index) and each lane
// pulls the next id from it the moment its ray completes; one loop iteration = one BVH node
// pair (+ the primitives of a leaf child). Light rays whose result depends on the first event
// past the light (a Gaussian straddling the light, or a pre-activated Gaussian the ray misses
// through rounding) are rare; they go to a queue served by secondary_slow_kernel's exact
// three-pass light_transmittance.
// ---------------------------------------------------------------------------------------------
// A 4-wide node index (< 2^27 nodes) in the walk's `node`; bits 28-30 may carry a child slot to skip.
constexpr int32_t kNodeIndexMask = 0x0fffffff;
#ifdef VR_DIAG_LEVELS
// Diagnostic builds only: VR_DIAG_LEVELS = 1 counts the node steps of the rays that end uncut, 2 those of
// the rays that reach their cut-off, by tree depth (secondary counters [8 + b]: depths 2b, 2b + 1; b = 7:
// deeper). Depths of the 4-wide nodes from their parents (depth_kernel, before the secondary stage).
__device__ uint8_t g_diag_depth[1u << 23];
#endif

struct SecRay {
    Ray ray;
    float ix, iy, iz, oxi, oyi, ozi;  // 1/d and o/d for the slab test
    float tau, lim;                   // optical depth so far; light: dist, env: +inf
    // `lim`: a light ray's distance to the light; an environment ray's last event so far (the
    // reference's t_env_end, test_integrators.h:258-271), which bounds nothing during traversal
    float cut;         // optical depth at which the ray's transmittance counts as 0 (error budget)
    float plim;        // node boxes entered beyond this distance hold nothing for the ray (light: past the light)
    uint64_t hitmask;  // which of the record's active Gaussians the ray has met
    uint64_t bloom;    // membership mask of the record's active list (act_find; PureRayMarching)
    float cmax;        // largest p.M.p (p = origin - mean) over the record's active list
    float credit;      // RayMarchingGaussians: list members' optical depth not yet met again by the tree walk
    uint32_t act_off, act_n;  // the record's active list
    bool light, needs_stop;
    bool bnd;          // the record has a member at its 3-sigma surface (kRecBoundary): the list phase tests the band
    uint32_t nsteps;  // instrumented build only: node steps taken by this ray
    int32_t from;     // 4-wide walk: root of the subtree the ray walks / has finished (climbs from the record's start subtree)
#ifdef VR_DIAG_LEVELS  // diagnostic builds only: this ray's node steps per tree depth (2 levels per bucket)
    uint32_t lv[8];
#endif
    uint32_t rec;     // record index
    uint32_t slot;    // result slot s * rec_cap + rec in tr
};

// The ray's optical depth is known to have reached its cut-off. RayMarchingGaussians: tau holds what
// the tree walk met (list members included), credit the list members' depth it has not met yet, so
// tau + credit is a lower bound of the final depth (see wtest in secondary_ww_kernel; a credit that a
// non-member candidate drove below 0 only makes the bound lower).
template <bool PURE>
__device__ __forceinline__ bool cut_reached(const SecRay& R) {
    if constexpr (PURE) return R.tau >= R.cut;
    else return R.tau + R.credit >= R.cut;
}

// Slot of Gaussian j in the record's active list, or -1. The list is scanned four entries per
// round trip (independent loads), since a scan sits on the dependent chain of a primitive test.
__device__ __forceinline__ int act_find(const RenderArgs& A, const SecRay& R, int j) {
    if (!((R.bloom >> (j & 63)) & 1ull)) return -1;
    const int* __restrict__ p = A.rec_act + R.act_off;
    const int n = (int)R.act_n;
    for (int i = 0; i < n; i += 4) {
        const int v0 = p[i];
        const int v1 = i + 1 < n ? p[i + 1] : -1;
        const int v2 = i + 2 < n ? p[i + 2] : -1;
        const int v3 = i + 3 < n ? p[i + 3] : -1;
        if (v0 == j) return i;
        if (v1 == j) return i + 1;
        if (v2 == j) return i + 2;
        if (v3 == j) return i + 3;
    }
    return -1;
}

// Direction of environment sample e of a record: PCG32 keyed by (pixel, step) as the oracle does;
// the 2e draws of the earlier samples are skipped by LCG jump-ahead s -> M s + C (host table).
// A record's environment samples all jump from one state: its path's seeded stream-1 generator.
__device__ __forceinline__ uint64_t env_base_state(const uint4& meta) {
    const int px = (int)(meta.x & 0xffffu), py = (int)(meta.x >> 16);
    return PCG32(derive_path_seed(px, py, (int)meta.y), 1).state;
}
__device__ __forceinline__ void env_xi_at(const RenderArgs& A, uint64_t base, uint32_t e, float& xi1, float& xi2) {
    PCG32 rng(PCG32::FromState{}, A.pcg_jump[4 * e] * base + A.pcg_jump[4 * e + 1], 1);
    xi1 = rng.uniform_env();
    xi2 = rng.uniform_env();
}
__device__ __forceinline__ void env_sample_xi(const RenderArgs& A, const uint4& meta, uint32_t e, float& xi1, float& xi2) {
    env_xi_at(A, env_base_state(meta), e, xi1, xi2);
}
__device__ __forceinline__ void env_sample_dir(const RenderArgs& A, const uint4& meta, uint32_t e, float& wx, float& wy,
                                               float& wz) {
    float xi1, xi2;
    env_sample_xi(A, meta, e, xi1, xi2);
    env_dir(xi1, xi2, wx, wy, wz);
}

// Direction cells of the environment rays: the 16 x 16 cells of the sample's (xi1, xi2) = (azimuth, cos polar)
// grid, Morton-numbered (equal-area direction cells without evaluating the direction; measured against the
// octahedral map of the evaluated direction, round 3: 3.3 ms slower at C4).
constexpr int kEnvBits = 4, kEnvSide = 1 << kEnvBits, kEnvCells = kEnvSide * kEnvSide;

// One sorting group per record chunk: counting sort of the chunk's environment rays by direction key
// (order inside a key is arbitrary: every ray's result is independent of when it is traced). A group
// is one wave: BLOCK/64 chunks in flight per workgroup, wave-local LDS and no workgroup barriers; the
// chunk's chain of dependent loads is the cost, not its arithmetic (C4: 1.56 ms; a workgroup per chunk 1.91).
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void env_order_kernel(RenderArgs A) {
    constexpr int G = 64, kGroups = BLOCK / G;
    constexpr uint32_t kKeyCap = 8192 / kGroups;  // keys kept in LDS per group; larger chunks recompute them
    using KeyT = typename std::conditional<(kEnvCells <= 256), uint8_t, uint16_t>::type;
    constexpr int kPer = kEnvCells / 64;  // counts per lane of the scan
    __shared__ uint32_t hist_s[kGroups][kEnvCells];
    __shared__ KeyT keys_s[kGroups][kKeyCap];
    __shared__ uint64_t base_s[kGroups][256];  // the chunk's generator states (record-in-chunk fits 8 bits)
    const uint32_t grp = threadIdx.x / G, tid = threadIdx.x % G;
    uint32_t* hist = hist_s[grp];
    KeyT* keys = keys_s[grp];
    uint64_t* base = base_s[grp];
    auto group_sync = [] {
        if constexpr (G == 64) {  // the wave's own LDS traffic: wait for it, keep the compiler from moving it
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
        } else {
            __syncthreads();
        }
    };
    const uint32_t nrec = dev_nrec(A);
    const uint32_t cr = A.chunk_rec, ne = (uint32_t)A.env_samples;
    const uint32_t n = cr * ne, nch = (nrec + cr - 1) / cr;
    const bool cached = n <= kKeyCap;
    for (uint32_t chunk = blockIdx.x * kGroups + grp; chunk < nch; chunk += gridDim.x * kGroups) {  // group-uniform loop
        const uint32_t r0 = chunk * cr;
        for (uint32_t i = tid; i < kEnvCells; i += G) hist[i] = 0;
        for (uint32_t rl = tid; rl < cr; rl += G)  // seeded once per record, not per sample
            if (r0 + rl < nrec) {
                base[rl] = env_base_state(A.rec_meta[r0 + rl]);
                A.env_base[r0 + rl] = base[rl];  // for sec_init: one 8-B load instead of the seeding per ray
            }
        group_sync();
        auto key = [&](uint32_t i) -> uint32_t {
            const uint32_t rl = i / ne, r = r0 + rl;
            if (r >= nrec) return kEnvCells - 1;  // padding records
            // the cell of the sample's (xi1, xi2) = (azimuth, cos polar) grid: equal-area direction
            // cells without evaluating the direction
            float xi1, xi2;
            env_xi_at(A, base[rl], i - rl * ne, xi1, xi2);
            const uint32_t cu = min((uint32_t)(xi1 * kEnvSide), (uint32_t)kEnvSide - 1u);
            const uint32_t cv = min((uint32_t)(xi2 * kEnvSide), (uint32_t)kEnvSide - 1u);
            uint32_t k = 0;
#pragma unroll
            for (int b = 0; b < kEnvBits; ++b) k |= (((cu >> b) & 1u) << (2 * b)) | (((cv >> b) & 1u) << (2 * b + 1));
            return k;
        };
        for (uint32_t i = tid; i < n; i += G) {
            const uint32_t k = key(i);
            if (cached) keys[i] = (KeyT)k;
            atomicAdd(&hist[k], 1u);
        }
        group_sync();
        if (tid < 64) {  // exclusive scan of the counts by one wave (kPer consecutive per lane)
            const uint32_t l = tid;
            uint32_t v[kPer], sum = 0;
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
                v[j] = hist[kPer * l + j];
                sum += v[j];
            }
            uint32_t incl = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (l >= (uint32_t)o) incl += y;
            }
            uint32_t ex = incl - sum;
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
                hist[kPer * l + j] = ex;
                ex += v[j];
            }
        }
        group_sync();
        uint16_t* out = A.env_order + (size_t)chunk * n;
        for (uint32_t i = tid; i < n; i += G) {
            const uint32_t rl = i / ne;
            out[atomicAdd(&hist[cached ? (uint32_t)keys[i] : key(i)], 1u)] = (uint16_t)((rl << 8) | (i - rl * ne));
        }
        group_sync();  // hist / keys / base are reused by the group's next chunk (staging the order in LDS
                       // for coalesced stores measured slower: 1.64 vs 1.56 ms at C4)
    }
}

// Ray ids are scheduled record-chunk-major: a chunk is A.chunk_rec consecutive records x all
// their samples (light rays first, then environment rays), so a wave that takes consecutive ids
// reads each record's data (position, active list, neighbour list) from its cache instead of
// once per sample. Light rays of a chunk go sample-major (neighbouring records towards the same
// light: coherent). Environment rays are random directions; with A.env_order they are handed
// out in the direction order env_order_kernel computed for the chunk, so a wave traces similar
// directions from nearby records. The result slot stays sample-major: tr[s * rec_cap + r].
__device__ __forceinline__ bool ray_slot(const RenderArgs& A, uint32_t chunk, uint32_t rem, uint32_t nrec, uint32_t& s,
                                         uint32_t& r) {
    const uint32_t cr = A.chunk_rec, lights = cr * (uint32_t)A.num_lights;
    if (A.env_order == nullptr || rem < lights) {
        s = rem >> A.chunk_shift;
        r = chunk * cr + (rem & (cr - 1u));
    } else {  // entry = record-in-chunk << 8 | environment sample
        const uint32_t v = A.env_order[(size_t)chunk * (cr * (uint32_t)A.env_samples) + (rem - lights)];
        s = (uint32_t)A.num_lights + (v & 0xffu);
        r = chunk * cr + (v >> 8);
    }
    return r < nrec;
}

// Result slot of a secondary ray: its position in the hand-out order (chunk-major, then the order
// ray_slot hands the chunk's rays out). A wave takes a chunk's rays in that order and writes each Tr
// when its ray completes, so one chunk's results fill a contiguous run of lines within a short time
// (a [sample][record] layout scattered every chunk's 4-B stores over S rows: lines left L2 partially
// written and were re-read — 7x write amplification). record_radiance_kernel reads a chunk back
// whole.
__device__ __forceinline__ uint32_t rays_per_chunk(const RenderArgs& A) {
    return A.chunk_rec * (uint32_t)(A.num_lights + A.env_samples);
}
// Start ray `rem` of record chunk `chunk`. Returns false if the ray is already complete (Tr
// written) or a padding id. norm: slab-test terms in the half nodes' scene-normalised
// coordinates (HNode).
__device__ __forceinline__ bool sec_init(const RenderArgs& A, uint32_t nrec, uint32_t chunk, uint32_t rem, SecRay& R,
                                         bool norm = false) {
    uint32_t s, r;
    if (!ray_slot(A, chunk, rem, nrec, s, r)) return false;  // padding id
    R.slot = chunk * rays_per_chunk(A) + rem;
    const float4 pos = A.rec_pos[r];
    if (!(pos.w > 0.0f)) {  // no ray to trace
        // a live record whose weight T sigma_s is 0 (an f32 underflow, or an over-capacity frame's empty
        // record): its radiance is weighed by 0, but record_radiance reads every slot, so a finite Tr;
        // an orphaned record (orphan_records, weight -1): no pixel reads its rays
        if (!(pos.w < 0.0f)) A.tr[R.slot] = 0.0f;
        return false;
    }
    const uint4 meta = A.rec_meta[r];
    R.rec = r;
    R.cut = A.tau_cut;  // (a select of the two addresses would make this one flat load)
    if (A.rec_cut != nullptr) R.cut = __builtin_nontemporal_load(A.rec_cut + r);
    R.act_off = meta.z;
    R.act_n = meta.w & ~kRecBoundary;
    R.bnd = (meta.w & kRecBoundary) != 0u;
    R.bloom = A.rec_bloom[r];
    R.cmax = -INFINITY;
    R.credit = 0.0f;
    R.hitmask = 0;
    R.nsteps = 0;
    R.from = 0;
#ifdef VR_DIAG_LEVELS
    for (int b = 0; b < 8; ++b) R.lv[b] = 0;
#endif
    R.tau = 0.0f;
    R.needs_stop = false;
    if (s < (uint32_t)A.num_lights) {
        const LightRecord& lr = A.lights[s];
        float dx = lr.px - pos.x, dy = lr.py - pos.y, dz = lr.pz - pos.z;
        // a secondary ray feeds only its Tr (continuous): one hardware-rsqrt normalisation instead of
        // the reference's two correctly rounded ones (direction within ~1 ulp)
        const float d2 = dot3(dx, dy, dz, dx, dy, dz);
        const float dist = sqrtf(d2);
        const float inv = __builtin_amdgcn_rsqf(d2);
        R.ray = Ray{pos.x, pos.y, pos.z, dx * inv, dy * inv, dz * inv};
        R.light = true;
        R.lim = dist;
        if (!(dist > 0.0f)) {  // `while (t_prev < dist)` never runs
            A.tr[R.slot] = 1.0f;
            return false;
        }
    } else {
        float wx, wy, wz;
        float xi1, xi2;  // (env_order_kernel left the record's generator state when it ran)
        env_xi_at(A, A.env_order != nullptr ? A.env_base[r] : env_base_state(meta), s - (uint32_t)A.num_lights, xi1, xi2);
        env_dir(xi1, xi2, wx, wy, wz);
        R.ray = Ray{pos.x, pos.y, pos.z, wx, wy, wz};  // env_dir's direction is unit up to rounding
        R.light = false;
        R.lim = 0.0f;  // last event so far
    }
    R.plim = R.light ? R.lim + kTPad * (1.0f + R.lim) : INFINITY;
    // |d| clamped away from 0: the fma slab form b/d - o/d must never see inf - inf
    const float sc = norm ? A.hn_scale : 1.0f;
    const float dx = R.ray.dx * sc, dy = R.ray.dy * sc, dz = R.ray.dz * sc;
    R.ix = __builtin_amdgcn_rcpf(fabsf(dx) > 1e-30f ? dx : copysignf(1e-30f, dx));
    R.iy = __builtin_amdgcn_rcpf(fabsf(dy) > 1e-30f ? dy : copysignf(1e-30f, dy));
    R.iz = __builtin_amdgcn_rcpf(fabsf(dz) > 1e-30f ? dz : copysignf(1e-30f, dz));
    if (norm) {
        R.oxi = (R.ray.ox - A.hn_center[0]) * sc * R.ix;
        R.oyi = (R.ray.oy - A.hn_center[1]) * sc * R.iy;
        R.ozi = (R.ray.oz - A.hn_center[2]) * sc * R.iz;
    } else {
        R.oxi = R.ray.ox * R.ix;
        R.oyi = R.ray.oy * R.iy;
        R.ozi = R.ray.oz * R.iz;
    }
    return true;
}

// PureRayMarching (integrator.h:105-135): the marched transmittance multiplies exp(-sigma_t dt)
// over the iterated steps t_k = 0, dt, 2dt, ... of the secondary ray; grouped per Gaussian that is
// dt * sum of its mu_t at the steps t_k in [lo, hi) where it is active.
__device__ __forceinline__ float marched_depth(const RenderArgs& A, const GRec& g, const Ray& r, float lo, float hi) {
    const float* __restrict__ ts = A.tsteps;
    float s = 0.0f;
    for (int k = kfirst(ts, A.num_tsteps, A.step_size, lo); k < A.num_tsteps; ++k) {
        const float t = ts[k];
        if (!(t < hi)) break;
        s += mu_t(g, r.ox + t * r.dx, r.oy + t * r.dy, r.oz + t * r.dz);
    }
    return s * A.step_size;
}

// Adds Gaussian g (active on the secondary ray over [lo, b)) to the ray's optical depth.
//   RayMarchingGaussians: analytic segment depth; a light ray's Gaussian straddling the light
//   needs the first event past the light (test_integrators.h:220-235) -> exact slow path.
//   PureRayMarching: marched to t < dist (light) / t < last event (environment, b <= tlast).
template <bool S, bool FAST, bool PURE>
__device__ __forceinline__ void sec_add(const RenderArgs& A, SecRay& R, const GRec& g, const Quad& q, float lo, float b,
                                        Ctr& c) {
    if constexpr (S) c.v[kCtrOD]++;
    if constexpr (PURE) {
        if (!R.light) {
            R.tau += marched_depth(A, g, R.ray, lo, b);
            R.lim = fmaxf(R.lim, b);
        } else if (lo < R.lim) {
            R.tau += marched_depth(A, g, R.ray, lo, fminf(b, R.lim));
        }
        return;
    }
    if constexpr (FAST) {  // one optical-depth evaluation for light and environment lanes alike
        const bool add = !R.light || b < R.lim;
        R.needs_stop = R.needs_stop || (!add && lo < R.lim);
        if (!R.light) R.lim = fmaxf(R.lim, b);
        if (add) R.tau += optical_depth_chord(g, q, lo, b);  // [lo, b] lies on the 3-sigma chord
    } else if (!R.light) {
        R.tau += optical_depth(g, q, lo, b);
        R.lim = fmaxf(R.lim, b);
    } else if (b < R.lim) {
        R.tau += optical_depth(g, q, lo, b);
    } else if (lo < R.lim) {
        R.needs_stop = true;
    }
}

// VR_DIAG_SKIP_TR_STORES: diagnostic builds only (tools_dbg, never the product library): the
// secondary rays' Tr stores are dropped so that rocprofv3 WRITE_SIZE attributes the kernel's write
// traffic (Tr stores vs traversal-stack spills). The traversal itself is unchanged.
#ifdef VR_DIAG_SKIP_TR_STORES
#define VR_TR_STORE(A, slot, v) ((void)(slot), (void)(v))
#else
#define VR_TR_STORE(A, slot, v) ((A).tr[slot] = (v))
#endif

// Hands a ray to the exact slow path (secondary_slow_kernel). A full queue raises the frame's capacity flag
// (rec_alloc[2], as a full record buffer does): the frame is reported and rendered again with the queue grown to
// what this one queued (the host's slow_hint), so no ray is ever lost to the queue's size.
__device__ __forceinline__ void to_slow(const RenderArgs& A, uint32_t slot) {
    const uint32_t q = atomicAdd(A.slowq, 1u);
    if (q < A.slowq_cap) {
        A.slowq[1 + q] = slot;
    } else {
        A.rec_alloc[2] = 1u;
        A.tr[slot] = __builtin_nanf("");
    }
}

// Hands an environment ray with one chord in the f32 error band to secondary_fix_kernel: its slot, the optical
// depth of everything else it crossed and the band Gaussian. A full queue: as to_slow.
__device__ __forceinline__ void to_fix(const RenderArgs& A, uint32_t slot, float tau, uint32_t j) {
    const uint32_t q = atomicAdd(A.fixq, 1u);
    if (q < A.fixq_cap) {
        A.fixq[1 + 3 * q] = slot;
        A.fixq[2 + 3 * q] = __float_as_uint(tau);
        A.fixq[3 + 3 * q] = j;
    } else {
        A.rec_alloc[2] = 1u;
        A.tr[slot] = __builtin_nanf("");
    }
}

// One queued ray of the exact slow path (result slot t, hand-out order: see tr_slot).
template <bool S>
__device__ void slow_ray(const RenderArgs& A, uint64_t t, int* stack, int stride, Ctr& c) {
    const uint32_t per = rays_per_chunk(A), chunk = (uint32_t)(t / per), rem = (uint32_t)(t - (uint64_t)chunk * per);
    uint32_t s, r;
    ray_slot(A, chunk, rem, dev_nrec(A), s, r);
    const float4 pos = A.rec_pos[r];
    const uint4 meta = A.rec_meta[r];
    ActList act{A.rec_act + meta.z, 1, (int)(meta.w & ~kRecBoundary), A.rec_bloom[r]};
    if (s < (uint32_t)A.num_lights) {  // test_integrators.h:202-237
        const LightRecord& lr = A.lights[s];
        float dx = lr.px - pos.x, dy = lr.py - pos.y, dz = lr.pz - pos.z;
        float dist = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
        normalize3(dx, dy, dz);
        Ray sr = make_ray(pos.x, pos.y, pos.z, dx, dy, dz);
        A.tr[t] = light_transmittance<S>(A, sr, dist, act, stack, stride, c);
    } else {  // :242-271, Ray env_ray(pos, wi) normalises the sampled direction
        float xi1, xi2, wx, wy, wz;
        env_xi_at(A, A.env_order != nullptr ? A.env_base[r] : env_base_state(meta), s - (uint32_t)A.num_lights, xi1, xi2);
        env_dir(xi1, xi2, wx, wy, wz);
        A.tr[t] = env_transmittance<S>(A, make_ray(pos.x, pos.y, pos.z, wx, wy, wz), act, stack, stride, c);
    }
}

// Ray complete: write its transmittance (or hand it to the exact slow path). WH: the scene's whitened
// records (A.wrec); false: the M forms of the records (a scene with a non-positive-definite M).
template <bool S, bool FAST, bool PURE, bool WH = !PURE>
__device__ __forceinline__ void sec_finish(const RenderArgs& A, SecRay& R, Ctr& c) {
#ifdef VR_DIAG_LEVELS
    if constexpr (S)
        if ((VR_DIAG_LEVELS == 2) == cut_reached<PURE>(R))
            for (int b = 0; b < 8; ++b)
                if (R.lv[b]) atomicAdd(A.work + kNumCtr + b, (unsigned long long)R.lv[b]);
#elif !defined(VR_DIAG_WAVE_UTIL) && !defined(VR_DIAG_CYCLES)
    if constexpr (S) {  // secondary-stage diagnostics in otherwise unused counter slots
#ifdef VR_DIAG_LIGHT  // diagnostic builds only: the light rays and their node steps instead of the cut rays'
        if (R.light) {
#else
        if (cut_reached<PURE>(R)) {
#endif
            c.v[kCtrSteps]++;                 // rays ended by the optical-depth cut-off
            c.v[kCtrPrimQueries] += R.nsteps;  // ... and their node steps
        }
    }
#endif
    if (cut_reached<PURE>(R)) {
        VR_TR_STORE(A, R.slot, 0.0f);
        return;
    }
    if (!PURE && R.needs_stop) {  // the exact slow path: a light ray's stopping event, a member at the boundary,
        to_slow(A, R.slot);       // a chord in the f32 error band
        return;
    }
    const bool band = !PURE && !R.light && isnan(R.lim);
    if (band && (R.act_n >= 64 || (R.hitmask & ((1ull << R.act_n) - 1ull)) != ((1ull << R.act_n) - 1ull))) {
        to_slow(A, R.slot);  // a band ray with a missed member (active to the last event): the whole ray exactly
        return;
    }
    if (R.act_n > 64) {  // (march_deep_kernel records) missed members: re-intersect the whole list
        bool any = false;
        for (uint32_t s = 0; s < R.act_n; ++s) {
            const int j = A.rec_act[R.act_off + s];
            if constexpr (!PURE && WH) {  // the list phase's whitened test
                const WRec g = load_wrec(A.wrec, j);
                const WQuad q = wquad(g, R.ray);
                float t0, t1, sd;
                if (wintersect(q, t0, t1, sd)) continue;
                any = true;
                if (!R.light) R.tau += wod_range(g, q, 0.0f, R.lim);
                else break;
                continue;
            }
            const GRec g = load_rec(A.gauss, j);
            const Quad q = FAST ? quad_fast(g, R.ray) : quad(g, R.ray);
            float a, b;
            if (FAST ? intersect_fast(q, a, b) : intersect(q, a, b)) continue;
            any = true;
            if constexpr (PURE) R.tau += marched_depth(A, g, R.ray, 0.0f, R.lim);
            else if (!R.light) R.tau += FAST ? optical_depth_fast(g, q, 0.0f, R.lim) : optical_depth(g, q, 0.0f, R.lim);
            else break;
        }
        if (!PURE && R.light && (R.needs_stop || any)) {
            to_slow(A, R.slot);
            return;
        }
        VR_TR_STORE(A, R.slot, expf(-R.tau));
        return;
    }
    const uint64_t all = R.act_n >= 64 ? ~0ull : ((1ull << R.act_n) - 1ull);
    uint64_t missed = all & ~R.hitmask;
    if constexpr (PURE) {  // pre-activated, missed through rounding: active to the end of the march
        while (missed) {
            int s = __ffsll((unsigned long long)missed) - 1;
            missed &= missed - 1;
            GRec g = load_rec(A.gauss, A.rec_act[R.act_off + s]);
            R.tau += marched_depth(A, g, R.ray, 0.0f, R.lim);  // dist (light) / last event (environment)
        }
    } else if (R.light) {
        if (R.needs_stop || missed) {
            to_slow(A, R.slot);
            return;
        }
    } else if (band) {  // (no missed member: see above)
    } else {
        while (missed) {  // pre-activated, missed through rounding: active up to the last event
            int s = __ffsll((unsigned long long)missed) - 1;
            missed &= missed - 1;
            if constexpr (S) c.v[kCtrOD]++;
            if constexpr (WH) {
                const WRec g = load_wrec(A.wrec, A.rec_act[R.act_off + s]);
                R.tau += wod_range(g, wquad(g, R.ray), 0.0f, R.lim);
            } else {
                const GRec g = load_rec(A.gauss, A.rec_act[R.act_off + s]);
                R.tau += optical_depth_fast(g, quad_fast(g, R.ray), 0.0f, R.lim);
            }
        }
    }
    if (band) {  // the band Gaussian's contribution: secondary_fix_kernel
        to_fix(A, R.slot, R.tau, band_id(R.lim));
        return;
    }
    VR_TR_STORE(A, R.slot, expf(-R.tau));
}

// ---------------------------------------------------------------------------------------------
// Stage 2 (default): persistent while-while tracing with postponed leaves.
//
// One ray per lane, but a wave never runs the node code and the primitive code in the same
// iteration: every iteration is either a NODE iteration (lanes with room in their leaf queue take
// one child-pair step; leaf children are queued, not tested) or a PRIM iteration (lanes with a
// queued leaf test ONE primitive), whichever more lanes can use. A lane whose ray completes is
// refilled from the wave's pool of ray ids (64 consecutive ids per atomic fetch: neighbouring
// records, same light / env-sample index, so a wave's rays stay spatially coherent). This removes
// the two divergence costs of one-ray-per-lane traversal: a wave no longer waits for its longest
// ray, and a leaf visit no longer stalls the lanes that are still walking inner nodes.
// ---------------------------------------------------------------------------------------------
// FIFO of up to QCAP leaf refs + the leaf being tested. QCAP = 2 or 4: the first two entries live
// in registers (q0, q1), entries 2 and 3 in the two LDS words per lane just above the traversal
// stack (ext[0], ext[BLOCK]). QCAP = 1 + 2^k (k >= 2): the head entry in q0, the others in an
// LDS ring of QCAP - 1 words above the stack, ring head in q1. A lane may take a NODE step while
// the queue has room for the 2 leaves a step can add, so a lane holding queued leaves keeps
// walking the tree.
template <int QCAP>
constexpr bool kQueueRing = QCAP > 4;
template <int QCAP>
constexpr int kQueueLds = kQueueRing<QCAP> ? QCAP - 1 : QCAP - 2;  // LDS words per lane of the queue

// An int in LDS (address space 3). The traversal stack and leaf queue are reached through this type
// so that a pop that may come from the LDS stack or the global overflow stays two typed loads (a
// ds_read and a global_load) instead of one flat load whose wait covers every outstanding access.
using LdsInt = __attribute__((address_space(3))) int;

struct LeafQueue {
    int32_t q0, q1;
    int n;
    uint32_t j, end;  // current primitive range [j, end)
    // branch-free for the register entries: writes r at slot `idx` (no slot matches idx < 0)
    template <int QCAP, int BLOCK>
    __device__ __forceinline__ void put(int idx, int32_t r, LdsInt* ext) {
        if constexpr (kQueueRing<QCAP>) {
            q0 = idx == 0 ? r : q0;
            if (idx >= 1) ext[((q1 + idx - 1) & (QCAP - 2)) * BLOCK] = r;
        } else {
            q0 = idx == 0 ? r : q0;
            q1 = idx == 1 ? r : q1;
            if constexpr (QCAP > 2)
                if (idx >= 2) ext[(idx - 2) * BLOCK] = r;
        }
    }
    __device__ __forceinline__ bool has_prim() const { return j < end || n > 0; }
    template <int QCAP, int BLOCK>
    __device__ __forceinline__ uint32_t next(LdsInt* ext) {  // requires has_prim()
        if (j == end) {
            j = leaf_first(q0);
            end = j + leaf_count(q0);
            if constexpr (kQueueRing<QCAP>) {
                if (n > 1) {
                    q0 = ext[(q1 & (QCAP - 2)) * BLOCK];
                    q1 = (q1 + 1) & (QCAP - 2);
                }
            } else {
                q0 = q1;
                if constexpr (QCAP > 2) {
                    if (n > 2) {
                        q1 = ext[0];
                        if (n > 3) ext[0] = ext[BLOCK];
                    }
                }
            }
            --n;
        }
        return j++;
    }
};

// Traversal-stack entries past the STACK held in LDS spill to the global overflow buffer, laid
// out [depth - STACK][lane of the resident grid]: the lanes of a wave that are at the same depth
// share cache lines, and the shallow overflow levels every deep walk touches stay a small, dense,
// L2-resident region (a per-lane [lane][depth] layout gives every lane its own line per level).
template <int BLOCK, int STACK>
__device__ __forceinline__ uint32_t ovf_slot(const RenderArgs& A, int sp) {
    return (uint32_t)(sp - STACK) * A.stack_ovf_lanes + blockIdx.x * BLOCK + threadIdx.x;
}

// One step of the 4-wide traversal without a sorting network (measured against one with a near-to-far sorting
// network of the children, round 3: 102.4 -> 99.2 ms at C4): the nearest inner child is walked next
// (a min-reduction over the inner children's entry distances), the other inner children are pushed
// and the leaf children queued in the node's child order. Empty slots carry NaN boxes, so the slab
// test alone rejects them. Ring queues only (QCAP = 1 + 2^k).
template <int BLOCK, bool S, int QCAP, int STACK, bool SOA = false>
__device__ __forceinline__ void sec_node4v(const RenderArgs& A, SecRay& R, LdsInt* stack, int& sp, int& node, LeafQueue& Q,
                                           Ctr& c) {
    static_assert(kQueueRing<QCAP>, "sec_node4v: ring leaf queue");
    if constexpr (S) {
        c.v[kCtrNodes]++;
        ++R.nsteps;
    }
    const int skip = node >> 28;  // a climb's node: the finished child's slot + 1 (0: none)
#ifdef VR_DIAG_LEVELS
    R.lv[min((int)g_diag_depth[node & kNodeIndexMask] >> 1, 7)]++;
#endif
    const uint4* np = reinterpret_cast<const uint4*>((SOA ? A.hnodes4t : A.hnodes4s) + (node & kNodeIndexMask));
    const uint4 q0 = np[0], q1 = np[1], q2 = np[2], rf = np[3];
    const uint32_t w[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
    const int32_t ref[4] = {(int32_t)rf.x, (int32_t)rf.y, (int32_t)rf.z, (int32_t)rf.w};
    // SOA (soa_nodes_kernel's layout): per axis, the ray's near bound word pair and far bound word pair, picked once
    // for the four children by the sign of its direction: for 1/d > 0 the near slab is the min (fma is monotone in
    // the bound), so the slab distances are the min/max of the AoS test bit for bit, without the per-child min/max
    float smin[4], smax[4];  // SOA: the children's slab entry / exit (a child pair at a time, in the child loop)
    LdsInt* ext = stack + STACK * BLOCK;
    float best = INFINITY;
    int32_t next = 0;  // the nearest inner child
    bool inner[4];
    // ring cursor: the next leaf goes to ring slot cur & (QCAP - 2); cur == head while the queue is
    // empty (the next leaf is the register head q0). Q.n follows from cur after the four children.
    const int head = Q.q1 - 1;
    int cur = head + Q.n;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float tmin, tmax;
        if constexpr (SOA) {
            // children i, i + 1 from one word pair per axis, just before child i: computing all four children's slabs
            // up front kept 8 more values live across the step (12 spilled VGPRs at the 72-VGPR limit, twice the
            // write traffic, 77.5 vs 76.0 ms at C4)
            if (i == 0 || i == 2) {
                const int pr = i >> 1;
                const float inv[3] = {R.ix, R.iy, R.iz}, oi[3] = {R.oxi, R.oyi, R.ozi};
#pragma unroll
                for (int ax = 0; ax < 3; ++ax) {
                    const bool neg = inv[ax] < 0.0f;
                    const uint32_t nwd = neg ? w[4 * ax + 2 + pr] : w[4 * ax + pr], fwd = neg ? w[4 * ax + pr] : w[4 * ax + 2 + pr];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const float nb = (float)__builtin_bit_cast(_Float16, (uint16_t)(h ? (nwd >> 16) : (nwd & 0xffffu)));
                        const float fb = (float)__builtin_bit_cast(_Float16, (uint16_t)(h ? (fwd >> 16) : (fwd & 0xffffu)));
                        const float tn = fmaf(nb, inv[ax], -oi[ax]), tf = fmaf(fb, inv[ax], -oi[ax]);
                        smin[i + h] = ax == 0 ? tn : fmaxf(smin[i + h], tn);
                        smax[i + h] = ax == 0 ? tf : fminf(smax[i + h], tf);
                    }
                }
            }
            tmin = smin[i];
            tmax = smax[i];
        } else {
            float f[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const uint32_t word = w[(6 * i + k) >> 1];
                f[k] = (float)__builtin_bit_cast(_Float16, (uint16_t)(((6 * i + k) & 1) ? (word >> 16) : (word & 0xffffu)));
            }
            const float tx1 = fmaf(f[0], R.ix, -R.oxi), tx2 = fmaf(f[3], R.ix, -R.oxi);
            const float ty1 = fmaf(f[1], R.iy, -R.oyi), ty2 = fmaf(f[4], R.iy, -R.oyi);
            const float tz1 = fmaf(f[2], R.iz, -R.ozi), tz2 = fmaf(f[5], R.iz, -R.ozi);
            tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
            tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
        }
        // [max(tmin, 0), min(tmax, plim)] not empty; a NaN box (empty slot) fails the first compare; the
        // subtree the ray has just finished (child slot skip - 1, right after a climb) is skipped
        const bool hit = (tmin <= fminf(tmax, R.plim)) & (tmax >= 0.0f) & (skip != i + 1);
        const bool leaf = hit & (ref[i] < 0);
        inner[i] = hit & !leaf;  // an empty slot (ref 0) never hits
        // leaf -> the queue's end: branch-free, a non-leaf store lands past the last entry (never
        // read). A NODE step starts with at most QCAP - 4 entries, so that slot is a free ring word.
        Q.q0 = (leaf & (cur == head)) ? ref[i] : Q.q0;
        ext[(cur & (QCAP - 2)) * BLOCK] = ref[i];
        cur += (int)leaf;
        const bool nearer = inner[i] & (tmin < best);
        best = nearer ? tmin : best;
        next = nearer ? ref[i] : next;
    }
    Q.n = cur - head;
    // the other inner children -> stack (branch-free while every stepping lane has room for 3)
    if (__builtin_expect(__ballot(sp > STACK - 3) == 0ull, 1)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            stack[sp * BLOCK] = ref[i];
            sp += (int)(inner[i] & (ref[i] != next));
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (inner[i] & (ref[i] != next)) {
                if (sp < STACK) stack[sp * BLOCK] = ref[i];
                else A.stack_ovf[ovf_slot<BLOCK, STACK>(A, sp)] = ref[i];
                ++sp;
            }
        }
    }
    if (next != 0) {
        node = next;
    } else if (sp > 0) {
        --sp;
        node = sp < STACK ? stack[sp * BLOCK] : A.stack_ovf[ovf_slot<BLOCK, STACK>(A, sp)];
    } else if (R.from > 0) {
        // the subtree rooted at R.from is done: its parent next, without that child (every node is still
        // visited at most once: the walk from the record's start subtree up to the root covers the tree).
        // The parent entry carries the child's slot in bits 28-30 (slot + 1), which the next step skips.
        const int32_t up = A.hn4_parent[R.from];
        R.from = up & kNodeIndexMask;
        node = up;  // (-1: the root's subtree is done)
    } else {
        node = -1;
    }
}

// One child-pair step of the postponed-leaf traversal: leaf children go to the queue (nearer
// first); node < 0 afterwards means the traversal is finished. Written branch-free (bitwise
// predicates, selects) so a wave does not split inside the step.
template <int BLOCK, bool S, int QCAP, int STACK, bool H>
__device__ __forceinline__ void sec_node(const RenderArgs& A, SecRay& R, LdsInt* stack, int& sp, int& node, LeafQueue& Q,
                                         Ctr& c) {
    if constexpr (S) {
        c.v[kCtrNodes]++;
        ++R.nsteps;
    }
    float f[12];  // left min xyz, left max xyz, right min xyz, right max xyz
    int2 nc;
    load_pair<H>(A, node, f, nc);  // H: scene-normalised coordinates (R.ix.. are normalised too)
    const float tx1 = fmaf(f[0], R.ix, -R.oxi), tx2 = fmaf(f[3], R.ix, -R.oxi);
    const float ty1 = fmaf(f[1], R.iy, -R.oyi), ty2 = fmaf(f[4], R.iy, -R.oyi);
    const float tz1 = fmaf(f[2], R.iz, -R.ozi), tz2 = fmaf(f[5], R.iz, -R.ozi);
    const float lmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float lmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    const float ux1 = fmaf(f[6], R.ix, -R.oxi), ux2 = fmaf(f[9], R.ix, -R.oxi);
    const float uy1 = fmaf(f[7], R.iy, -R.oyi), uy2 = fmaf(f[10], R.iy, -R.oyi);
    const float uz1 = fmaf(f[8], R.iz, -R.ozi), uz2 = fmaf(f[11], R.iz, -R.ozi);
    const float rmin = fmaxf(fmaxf(fminf(ux1, ux2), fminf(uy1, uy2)), fminf(uz1, uz2));
    const float rmax = fminf(fminf(fmaxf(ux1, ux2), fmaxf(uy1, uy2)), fmaxf(uz1, uz2));
    const float lim = R.plim;
    const bool hl = (nc.x != 0) & (lmax >= fmaxf(lmin, 0.0f)) & (lmin <= lim);
    const bool hr = (nc.y != 0) & (rmax >= fmaxf(rmin, 0.0f)) & (rmin <= lim);
    const bool r_near = rmin < lmin;
    const bool ll = hl & (nc.x < 0), lr = hr & (nc.y < 0);  // leaf refs are negative
    const int32_t near_ref = r_near ? nc.y : nc.x, far_ref = r_near ? nc.x : nc.y;
    // leaves -> queue, nearer first
    const int32_t first_leaf = (ll & lr) ? near_ref : (ll ? nc.x : nc.y);
    Q.put<QCAP, BLOCK>((ll | lr) ? Q.n : -1, first_leaf, stack + STACK * BLOCK);
    Q.put<QCAP, BLOCK>((ll & lr) ? Q.n + 1 : -1, far_ref, stack + STACK * BLOCK);
    Q.n += (int)ll + (int)lr;
    // inner children -> continue / stack
    const bool il = hl & !ll, ir = hr & !lr;
    if (il & ir) {
        if (sp < STACK) stack[sp * BLOCK] = far_ref;
        else A.stack_ovf[ovf_slot<BLOCK, STACK>(A, sp)] = far_ref;
        ++sp;
    }
    if (il | ir) {
        node = (il & ir) ? near_ref : (il ? nc.x : nc.y);
    } else if (sp > 0) {
        --sp;
        node = sp < STACK ? stack[sp * BLOCK] : A.stack_ovf[ovf_slot<BLOCK, STACK>(A, sp)];
    } else {
        node = -1;
    }
}

// The list phase: every secondary ray of a record first tests the record's active list (the
// Gaussians active at the record's step: they contain the record position, so they carry the
// largest optical depths from it and most rays become opaque right there, without touching the
// tree); the tree walk that follows skips exactly these members (act_find). The phase lives in
// `node`: kNodeList (-2) walks the active list [Q.j, Q.end), node >= 0 is the tree walk, -1 the end.
// (Until round 3 the phase walked a per-record neighbour list {j : q_j(pos) <= 9.5} built by a BVH
// point query per record; the active list is a subset the march already holds: no list stage
// (-6.1 ms at C4) and a 2.4 % faster secondary stage)
constexpr int kNodeList = -2;


// Start ray R's list phase (or go straight to the tree).
__device__ __forceinline__ void list_begin(SecRay& R, LeafQueue& Q, int& node) {
    Q.n = 0;
    Q.q1 = 0;  // ring head (ring queues): valid whenever the tree walk starts here
    Q.j = R.act_off;
    Q.end = R.act_off + R.act_n;
    node = R.act_n > 0u ? kNodeList : R.from;
}

// After a list slot was consumed: move to the tree (its start subtree) once the list is done.
__device__ __forceinline__ void list_advance(LeafQueue& Q, int& node, int start) {
    if (node != kNodeList || Q.j < Q.end) return;
    Q.j = Q.end = 0;
    node = start;
}

// Scheduling constants of the persistent kernel (tuned on C4): refill once this many
// lanes are idle (amortises sec_init), and up to this many NODE / PRIM steps per lane per iteration
// (amortises the per-iteration ballots and decisions).
#ifndef VR_WW_REFILL
#define VR_WW_REFILL 24
#endif
#ifndef VR_WW_NODE_STEPS
#define VR_WW_NODE_STEPS 6
#endif
#ifndef VR_WW_PRIM_STEPS
#define VR_WW_PRIM_STEPS 3  // A/B round 4 (tight tree, C4 secondary): 3: 77.1, 4: 77.1-77.3, 5: 77.6-78.0, 7: 85.7 ms;
                            // round 6 (with PRIM bias 85, tools/gpu_r6n.sh): 3 + 85 %: 78.0 vs 4 + 70 %: 78.4-78.5 ms
#endif
#ifndef VR_WW_PRIM_UNROLL
#define VR_WW_PRIM_UNROLL 5  // unroll of the PRIM iteration's step loop (A/B: code size vs. scheduling)
#endif
#ifndef VR_WW_NODE_UNROLL
#define VR_WW_NODE_UNROLL 1
#endif
constexpr int kRefillMin = VR_WW_REFILL, kNodeSteps = VR_WW_NODE_STEPS, kPrimSteps = VR_WW_PRIM_STEPS;
#ifndef VR_WW_PRIM_BIAS
#define VR_WW_PRIM_BIAS 85  // a PRIM iteration needs this many % of the lanes a NODE iteration could use (A/B, round 6:
                            // 60 / 70 / 85 / 100 % -> 79.1 / 78.5 / 78.0-78.3 / 78.7 ms at 4 PRIM steps)
#endif
constexpr int kPrimBias = VR_WW_PRIM_BIAS;
constexpr int kPrimUnroll = VR_WW_PRIM_UNROLL, kNodeUnroll = VR_WW_NODE_UNROLL;

// 6 waves/SIMD = 80 VGPRs: the ray state is kept small enough for that without scratch spills (a
// spilling 6-wave build measured 9 % slower than 5 waves; this one is 5 % faster than 5 waves).
// S = true is the instrumented build (vr_count_work): the same schedule, counting its own work.
// WH: the whitened records (A.wrec); false (PureRayMarching, or a scene with a non-positive-definite M):
// the records' M forms with the membership lookup of the record's active list.
#ifdef VR_DIAG_DRAIN  // diagnostic builds only: the persistent kernel's tail (100 MHz clock ticks, printed by the last wave)
// [0] ray latencies, [1] latencies of the rays handed out once the claim counter was exhausted (log2 us buckets);
// wave exits after the exhaustion in 50-us buckets
__device__ unsigned long long g_dr_t0, g_dr_done, g_dr_end;
__device__ uint32_t g_dr_hist[2][20], g_dr_max[2], g_dr_exit[64], g_dr_waves;
#endif
template <int BLOCK, int STACK, bool S, bool PURE, int WAVES, int QCAP, bool H, bool W, bool WH = !PURE, bool SOA = false>
__global__ __launch_bounds__(BLOCK, WAVES) void secondary_ww_kernel(RenderArgs A) {
    __shared__ int s_stack[(STACK + kQueueLds<QCAP>) * BLOCK];
    LdsInt* stack = (LdsInt*)(s_stack + threadIdx.x);  // LDS-typed: stack/queue accesses are ds_* ops, never flat
    const uint32_t lane = threadIdx.x & 63u;
    Ctr c{};
    SecRay R;
    LeafQueue Q{0, 0, 0, 0u, 0u};
    uint32_t t = 0;
    int sp = 0, node = -1;
    bool live = false;
    // wave-uniform: the record chunk being handed out and its rays [pool, pool_end) not yet handed out
    uint32_t chunk = 0, pool = 0, pool_end = 0;
    bool counter_done = false;  // wave-uniform: the global chunk counter has passed nchunks
    bool fin = false;           // the lane's ray is complete and its Tr not yet written (batched completions)
    const uint32_t per = A.chunk_rec * (uint32_t)(A.num_lights + A.env_samples);
    const uint32_t nrec = dev_nrec(A), nchunks = (nrec + A.chunk_rec - 1u) >> A.chunk_shift;
    // Claim units: a chunk's rays in hand-out order, cut into 2^split equal parts when the launch has
    // few chunks per resident wave (a frame share of a multi-GPU split): shorter last units, a shorter
    // tail of the persistent launch (8-way C4 share: 22.7 -> 21.7 ms). Whole chunks otherwise (record
    // locality). (Measured and not kept, round 6: a guided tail — the launch's last 1/2/4 units per wave handed
    // out in 1/8 or 1/16 chunks — 8-way share prediction 7.12 -> 7.19/7.15/7.13, 1/16: 6.93; the tail after
    // the counter runs out is the in-flight rays' latency, not the unstarted rays left in a wave's pool. Nor is
    // that latency a few long walks: handing rays past 150/300/600/1200 node steps to the wave-per-ray slow path
    // re-routed 17 k/15/0/0 rays per C4 frame and cost 1.8 ms in spills. A ray waits on its wave's NODE/PRIM
    // schedule: ~100-250 us typical, up to ~2 ms, over ~30 node steps; VR_DIAG_DRAIN.)
    const uint32_t waves = gridDim.x * (BLOCK / 64u), cpw = nchunks / max(waves, 1u);
#ifndef VR_WW_SPLIT_CPW
#define VR_WW_SPLIT_CPW 32  // chunks per resident wave below which claim units get shorter (A/B)
#endif
    constexpr uint32_t kSplitCpw = VR_WW_SPLIT_CPW;
    const uint32_t split = cpw >= kSplitCpw ? 0u : cpw >= kSplitCpw / 2u ? 1u : cpw >= kSplitCpw / 4u ? 2u : 3u;
    const uint32_t nunits = nchunks << split;
    counter_done = nunits == 0u;
#ifdef VR_DIAG_CYCLES  // diagnostic builds only (S = true): wave cycles per phase, lane 0's counters
    // kCtrSteps: NODE iterations, kCtrPrimQueries: PRIM iterations, kCtrPixels: refill + completion
    uint64_t diag_t = __builtin_amdgcn_s_memtime();
    auto diag_lap = [&](int slot) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        if constexpr (S) c.v[slot] += lane == 0u ? (uint32_t)(now - diag_t) : 0u;
        diag_t = now;
    };
#else
    auto diag_lap = [](int) {};
#endif
#ifdef VR_DIAG_REFILL  // diagnostic builds only (with VR_DIAG_CYCLES): the refill split into its parts (lane 0's
    // cycles, written over the work counters kCtrNodes (batch completion), kCtrPrims (chunk claim), kCtrOD
    // (sec_init, the start node and list_begin, with their loads waited for), kCtrMu (hand-out bookkeeping))
    uint32_t rf_cyc[4] = {0u, 0u, 0u, 0u};
    uint64_t rf_t = 0;
    auto rf_lap = [&](int k, bool wait) {
        if (wait) __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const uint64_t now = __builtin_amdgcn_s_memtime();
        rf_cyc[k] += lane == 0u ? (uint32_t)(now - rf_t) : 0u;
        rf_t = now;
    };
#else
    auto rf_lap = [](int, bool) {};
#endif
#ifdef VR_DIAG_DRAIN
    uint64_t dr_ray0 = 0;
    bool dr_late = false, dr_seen = false;
    __shared__ uint32_t s_dr_hist[2][20], s_dr_max[2];  // (workgroup-local: global atomics per ray slow the frame ~90x)
    if (threadIdx.x < 40u) (&s_dr_hist[0][0])[threadIdx.x] = 0u;
    if (threadIdx.x < 2u) s_dr_max[threadIdx.x] = 0u;
    __syncthreads();
    if (lane == 0u) atomicCAS(&g_dr_t0, 0ull, (unsigned long long)wall_clock64());
#endif
    for (;;) {
        const uint64_t idle = __ballot(!live);
        if (__popcll(idle) >= kRefillMin) {  // refill once enough lanes are idle (amortises sec_init)
#ifdef VR_DIAG_REFILL
            rf_t = __builtin_amdgcn_s_memtime();
#endif
            if (fin) {  // the completions since the last refill, in one pass
                sec_finish<S, true, PURE, WH>(A, R, c);
                fin = false;
            }
            rf_lap(0, true);
            if (pool == pool_end && !counter_done) {  // next unit of a record chunk
                uint32_t cnext = 0;
                if (lane == 0) cnext = (uint32_t)atomicAdd(A.ray_next, 1ull);
                cnext = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnext);  // wave-uniform: scalar register
                if (cnext < nunits) {
                    chunk = cnext >> split;
                    const uint32_t part = cnext & ((1u << split) - 1u);
                    pool = (part * per) >> split;
                    pool_end = ((part + 1u) * per) >> split;
                }
                counter_done = cnext + 1u >= nunits;
#ifdef VR_DIAG_DRAIN
                if (cnext + 1u >= nunits && !dr_seen && lane == 0u) atomicCAS(&g_dr_done, 0ull, (unsigned long long)wall_clock64());
                dr_seen = dr_seen || cnext + 1u >= nunits;
#endif
            }
            rf_lap(1, true);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            if (!live && pool + rank < pool_end) {
                t = pool + rank;
                if constexpr (S) c.v[kCtrSecRays]++;
                live = sec_init(A, nrec, chunk, t, R, H);  // false: padding id, or complete already (Tr written)
#ifdef VR_DIAG_DRAIN
                dr_ray0 = wall_clock64();
                dr_late = counter_done;
#endif
                sp = 0;
                node = -1;
                Q.n = 0;
                Q.j = Q.end = 0;
                if (live) {
                    if constexpr (W)  // the tree walk starts in the record's start subtree
                        if (A.rec_start != nullptr) R.from = A.rec_start[R.rec];
                    list_begin(R, Q, node);
                }
            }
            rf_lap(2, true);
            const uint32_t handed = (uint32_t)__popcll(idle);
            pool = pool_end - pool > handed ? pool + handed : pool_end;
            rf_lap(3, true);
        }
        if (!__any(live)) {
            if (fin) {  // (only if the refill threshold exceeded the wave: every lane idle refills above)
                sec_finish<S, true, PURE, WH>(A, R, c);
                fin = false;
            }
            if (counter_done && pool == pool_end) break;
            continue;
        }
#ifdef VR_DIAG_WAVE_UTIL  // diagnostic builds only: wave iterations with a live lane, and live lanes in them
        if constexpr (S) c.v[kCtrPixels] += (lane == 0u ? 1u : 0u);
#endif
        diag_lap(kCtrPixels);
        const bool has_prim = live && Q.has_prim();
        constexpr int kRoom = W ? 4 : 2;  // leaves one NODE step can queue
        const bool can_node = live && node >= 0 && (QCAP == 2 ? Q.n == 0 : Q.n <= QCAP - kRoom);
        const int np = __popcll(__ballot(has_prim)), nn = __popcll(__ballot(can_node));
        // whichever kind more lanes can use; never a kind no lane can use (that would not progress)
        const bool prim_iter = nn == 0 || (np > 0 && np * 100 >= nn * kPrimBias);
        if (prim_iter) {  // PRIM iteration: up to kPrimSteps primitive tests per lane
            LdsInt* ext = stack + STACK * BLOCK;
            // next primitive of the lane: a list member (ls = its slot) or a queued leaf's (ls = -1)
            auto fetch = [&](uint32_t& j, int& ls) {
                if (node == kNodeList) {
                    ls = (int)(Q.j - R.act_off);
                    j = (uint32_t)A.rec_act[Q.j++];
                    list_advance(Q, node, R.from);
                } else {
                    ls = -1;
                    j = Q.next<QCAP, BLOCK>(ext);
                }
            };
            // one primitive test; ls >= 0: list member ls (pre-activated: optical depth from 0).
            // RayMarchingGaussians: the whitened record (WRecord); PureRayMarching: the record itself
            // (its marched depth evaluates mu_t)
            // The whitened primitive test (RayMarchingGaussians). The list phase sums the members' depths into
            // `credit` (the cut-off sees them at once); the tree walk then sums every Gaussian it meets into
            // tau, members included, so no membership lookup is needed. A member's p.M.p is <= cmax (the same
            // bits the list phase took), so it is a candidate when the walk meets it again; a candidate's
            // depth comes off the credit, which stays a lower bound of what the walk has still to meet. The
            // walk sums every Gaussian from its entry max(t0, 0): for a member that holds the origin (and for
            // any Gaussian that does) that is 0, the reference's pre-activation. A member whose chord starts
            // ahead of the origin (t0 > 0: the march's camera-ray test can activate a Gaussian a few percent
            // outside its ellipsoid) is pre-activated all the same: the list phase adds its stretch [0, t0]
            // to tau at once and only [t0, t1] to the credit. (Until round 5 every candidate was summed from
            // 0, so a non-member the origin lies just outside of, heading in, had [0, t0] too — with cmax > 9
            // such Gaussians pass the c test, and for a dense one that stretch is worth ~0.1 of optical depth:
            // C4 at t_eps 0, pixel (2224, 3653) 2.3e-3 dark.) Selects rather than fmaxf where an operand is
            // not known canonical: fmaxf would canonicalise it first, one more VALU op each.
            auto wtest = [&](const WRec& g, uint32_t j, int ls) {
                if constexpr (S) c.v[ls >= 0 ? kCtrMu : kCtrPrims]++;  // list members counted apart
                const WQuad q = wquad(g, R.ray);
                // A chord within the reference's f32 error band (kChordBand): on an environment ray, that one
                // Gaussian's contribution is left to the reference's M form (secondary_fix_kernel; the ray's tau
                // leaves it out, its id rides in R.lim); a member, a light ray or a second such chord sends the
                // whole ray to the exact slow path
                if constexpr (kChordBand > 0.0f) {
                    if (__builtin_expect(fmaf(-kChordBand, q.c, fabsf(9.0f - q.e2)) < 0.0f, false)) {
                        if (ls >= 0 || R.light || isnan(R.lim) || j >= 0x007fffffu) {
                            R.needs_stop = true;  // a member, a light ray or a second band chord: the whole ray exactly
                        } else {
                            R.lim = band_lim(j);
                            return;
                        }
                    }
                }
                R.cmax = (ls >= 0 && q.c > R.cmax) ? q.c : R.cmax;
                const bool cand = ls < 0 && q.c <= R.cmax;
                // A member whose 3-sigma surface passes within rounding of the record position (or that the ray
                // grazes): whether the reference's f32 test finds it crossed (active on [0, t1]) or missed
                // (active to the ray's last event — for a dense Gaussian ~1 of optical depth) is a rounding
                // decision the whitened form cannot reproduce: the exact slow path decides the ray (C4 at
                // t_eps 0, pixel (470, 3144): c = 9.00000, t1 = -0.00000 in the reference, 2.6e-2 bright).
                if (__builtin_expect(R.bnd, false))  // (~1 % of the records: rarely taken by a wave)
                    if (ls >= 0 && (fabsf(q.c - 9.0f) < kMemberAmb || fabsf(9.0f - q.e2) < kMemberAmb)) R.needs_stop = true;
                float t0, t1, sd;
                if (!wintersect(q, t0, t1, sd)) return;
                const bool inside = q.hr > -sd;  // t0 < 0: the origin lies in the 3-sigma sphere
                const bool pre = ls >= 0 || inside;
                const float lo = pre ? 0.0f : t0;
                const float u0 = pre ? q.hr : -sd;  // erf argument x sqrt 2 at lo
                if (ls >= 0) R.hitmask |= slot_bit(ls);
                if constexpr (S) {
                    c.v[kCtrOD]++;
#if !defined(VR_DIAG_WAVE_UTIL) && !defined(VR_DIAG_CYCLES)
                    c.v[kCtrPixels] += cand ? 1u : 0u;  // a list member's depth again (the credit scheme)
#endif
                }
                // sec_add's FAST rule: one optical-depth evaluation for light and environment lanes
                const bool add = !R.light || t1 < R.lim;
                R.needs_stop = R.needs_stop | (!add & (lo < R.lim));
                R.lim = (!R.light && t1 > R.lim) ? t1 : R.lim;
                if (add) {  // wod_chord over [lo, t1] (the 3-sigma chord, but for a member's stretch [0, t0])
                    constexpr float kRs2 = 0.70710678118654752f;
                    const float F1 = erf_chord(sd * kRs2), F0 = erf_chord(u0 * kRs2);
                    const float pf = (g.dn * q.r) * __expf(-0.5f * q.e2);
                    const float od = pf * fmaxf(F1 - F0, 0.0f);  // (f32 noise can invert a tiny interval)
                    if (ls >= 0) {  // the credit takes the chord [max(t0, 0), t1] (erf_chord is odd), tau the rest
                        const float chord = inside ? od : pf * (F1 + F1);
                        R.credit += chord;
                        R.tau += od - chord;  // + 0 when the origin lies inside
                    } else {
                        R.tau += od;
                        if (cand) R.credit -= od;
                    }
                }
            };
            auto test = [&](const GRec& g, uint32_t j, int ls) {
                if constexpr (S) c.v[ls >= 0 ? kCtrMu : kCtrPrims]++;  // list members counted apart
                const Quad q = quad_fast(g, R.ray);
                int slot = ls;
                if (ls >= 0) {
                    R.cmax = fmaxf(R.cmax, q.Cq);
                } else if (q.Cq <= R.cmax) {
                    // a tree leaf skips the record's active Gaussians (already summed by the list phase).
                    // Only a Gaussian that holds the origin as far as the members' own p.M.p values go
                    // (the same cq_fast bits, taken by the list phase) can be one: no scan otherwise
                    slot = act_find(A, R, (int)j);
                    if (slot >= 0) return;
                }
                float a, b;
                if (intersect_fast(q, a, b)) {
                    float lo = a;
                    if (slot >= 0) {
                        lo = 0.0f;
                        R.hitmask |= slot_bit(slot);
                    }
                    sec_add<S, true, PURE>(A, R, g, q, lo, b, c);
                }
            };
            bool go = has_prim;
#pragma unroll kPrimUnroll
            for (int k = 0; k < kPrimSteps; ++k) {
#ifdef VR_DIAG_WAVE_UTIL  // diagnostic builds only: wave-level PRIM steps (lane utilisation)
                if constexpr (S) c.v[kCtrPrimQueries] += (__ballot(go) != 0ull && lane == 0u) ? 1u : 0u;
#endif
                if (go) {
                    uint32_t j;
                    int ls;
                    fetch(j, ls);
                    if constexpr (!WH) test(load_rec(A.gauss, (int)j), j, ls);
                    else wtest(load_wrec(A.wrec, (int)j), j, ls);
                }
                go = go && Q.has_prim() && !cut_reached<PURE>(R);
            }
            diag_lap(kCtrPrimQueries);
        } else {  // NODE iteration: up to kNodeSteps node steps per lane
            bool go = can_node;
#pragma unroll kNodeUnroll
            for (int k = 0; k < kNodeSteps; ++k) {
#ifdef VR_DIAG_WAVE_UTIL  // diagnostic builds only: wave-level NODE steps (lane utilisation)
                if constexpr (S) c.v[kCtrSteps] += (__ballot(go) != 0ull && lane == 0u) ? 1u : 0u;
#endif
                if (go) {
                    if constexpr (W) sec_node4v<BLOCK, S, QCAP, STACK, SOA>(A, R, stack, sp, node, Q, c);
                    else sec_node<BLOCK, S, QCAP, STACK, H>(A, R, stack, sp, node, Q, c);
                }
                go = go && node >= 0 && Q.n <= QCAP - kRoom;
            }
            diag_lap(kCtrSteps);
        }
        if (live && (cut_reached<PURE>(R) || (node == -1 && !Q.has_prim()))) {
            fin = true;  // written at the next refill (the lane idles until then anyway)
            live = false;
#ifdef VR_DIAG_DRAIN
            const uint32_t us = (uint32_t)((wall_clock64() - dr_ray0) / 100u);
            atomicAdd(&s_dr_hist[0][min(31 - __clz(us | 1), 19)], 1u);
            atomicMax(&s_dr_max[0], us);
            if (dr_late) {
                atomicAdd(&s_dr_hist[1][min(31 - __clz(us | 1), 19)], 1u);
                atomicMax(&s_dr_max[1], us);
            }
#endif
        }
    }
#ifdef VR_DIAG_DRAIN
    {
        const unsigned long long now = wall_clock64(), done = atomicAdd(&g_dr_done, 0ull);
        if (lane == 0u && done != 0ull && now > done) atomicAdd(&g_dr_exit[min((uint32_t)((now - done) / 5000u), 63u)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 40u) {
        const uint32_t v = (&s_dr_hist[0][0])[threadIdx.x];
        if (v) atomicAdd(&g_dr_hist[0][0] + threadIdx.x, v);
    }
    if (threadIdx.x < 2u) atomicMax(&g_dr_max[threadIdx.x], s_dr_max[threadIdx.x]);
    if (lane == 0u) {
        const unsigned long long now = wall_clock64();
        atomicMax(&g_dr_end, now);
        __threadfence();
        if (atomicAdd(&g_dr_waves, 1u) == waves - 1u) {
            const unsigned long long t0 = atomicExch(&g_dr_t0, 0ull), end = atomicExch(&g_dr_end, 0ull);
            const unsigned long long dn = atomicExch(&g_dr_done, 0ull);
            printf("drain: waves %u units %u kernel %.1f us, claims exhausted at %.1f us, drain %.1f us; max ray %u us, max late ray %u us\n",
                   waves, nunits, (end - t0) / 100.0, (dn - t0) / 100.0, (end - dn) / 100.0, atomicExch(&g_dr_max[0], 0u),
                   atomicExch(&g_dr_max[1], 0u));
            for (int k = 0; k < 2; ++k)
                for (int b = 0; b < 20; ++b) {
                    const uint32_t v = atomicExch(&g_dr_hist[k][b], 0u);
                    if (v) printf("  %s rays us<%u: %u\n", k ? "late" : "all", 2u << b, v);
                }
            for (int b = 0; b < 64; ++b) {
                const uint32_t v = atomicExch(&g_dr_exit[b], 0u);
                if (v) printf("  wave exits %u-%u us after exhaustion: %u\n", 50u * b, 50u * b + 50u, v);
            }
            atomicExch(&g_dr_waves, 0u);
        }
    }
#endif
#ifdef VR_DIAG_REFILL
    c.v[kCtrNodes] = rf_cyc[0];
    c.v[kCtrPrims] = rf_cyc[1];
    c.v[kCtrOD] = rf_cyc[2];
    c.v[kCtrMu] = rf_cyc[3];
#endif
#ifndef VR_DIAG_LEVELS
    if constexpr (S) flush_counters(A.work + kNumCtr, c);
#endif
}

// Environment rays with one chord in the reference f32 quadratic's error band (to_fix): the band Gaussian's
// contribution as the reference computes it — its M-form crossing on the exactly normalised ray (a collapsed chord
// contributes nothing, a phantom one its tiny depth), active from max(t0, 0) to t1 (test_integrators.h:242-271 with
// stable tie order) — added to the optical depth of everything else the ray crossed.
__global__ __launch_bounds__(64) void secondary_fix_kernel(RenderArgs A) {
    const uint32_t n = min(A.fixq[0], A.fixq_cap);
    for (uint32_t q = blockIdx.x * 64u + threadIdx.x; q < n; q += gridDim.x * 64u) {
        const uint32_t t = A.fixq[1 + 3 * q];
        const float tau = __uint_as_float(A.fixq[2 + 3 * q]);
        const GRec g = load_rec(A.gauss, (int)A.fixq[3 + 3 * q]);
        const uint32_t per = rays_per_chunk(A), chunk = t / per, rem = t - chunk * per;
        uint32_t s, r;
        ray_slot(A, chunk, rem, dev_nrec(A), s, r);
        const float4 pos = A.rec_pos[r];
        float xi1, xi2, wx, wy, wz;
        env_xi_at(A, A.env_order != nullptr ? A.env_base[r] : env_base_state(A.rec_meta[r]), s - (uint32_t)A.num_lights, xi1, xi2);
        env_dir(xi1, xi2, wx, wy, wz);
        const Ray er = make_ray(pos.x, pos.y, pos.z, wx, wy, wz);
        const Quad qd = quad(g, er);
        float a, b;
        const float od = intersect(qd, a, b) ? optical_depth(g, qd, a, b) : 0.0f;
        A.tr[t] = expf(-(tau + od));
    }
}

#ifndef VR_SLOW_RPW
#define VR_SLOW_RPW 8  // rays per wave of the exact slow path: each ray is a long dependent chain (~250 us), so a wave
                        // of 64 lasts as long as its slowest; 64 / 16 / 12 / 8 / 6 / 4 / 2 / 1 -> 377 / 309 / 273 / 254-270 /
                        // 262 / 276-290 / 306 / 342 us per C4 frame (round 5). (Measured and not kept, round 6: the
                        // persistent kernel's idle waves tracing queued rays in its drain — slow kernel 412 -> 130 us,
                        // but the persistent kernel 76.8 -> 78.9 ms with the slow path's registers in it.)
#endif
#ifdef VR_DIAG_SLOW
__device__ uint32_t g_slow_hist[2][16], g_slow_max[2], g_slow_done;
#endif
// Exact three-pass light transmittance for the queued rays (see light_transmittance).
template <int BLOCK, bool S>
__global__ __launch_bounds__(BLOCK) void secondary_slow_kernel(RenderArgs A) {
    __shared__ int s_stack[kStackSize * BLOCK];
    int* stack = s_stack + threadIdx.x;
    const uint32_t n = min(A.slowq[0], A.slowq_cap);
    Ctr c{};
#ifdef VR_DIAG_SLOW  // diagnostic builds only: a histogram of the rays' latencies, printed by the last block
    uint32_t my_max = 0;
#endif
    // VR_SLOW_RPW rays per wave (the rest of its lanes idle): a wave lasts as long as its slowest ray. A queue
    // longer than one pass at that rate (many chord-band rays) takes as many lanes per wave as one pass needs
    // (a power of two up to 64): a second pass would cost a whole ray chain again.
    const uint32_t lane = threadIdx.x % 64u, wave = (blockIdx.x * BLOCK + threadIdx.x) / 64u;
    const uint32_t waves = gridDim.x * (BLOCK / 64u);
    uint32_t rpw = VR_SLOW_RPW;
    while (rpw < 64u && (uint64_t)waves * rpw < n) rpw *= 2u;
    const uint32_t q0 = lane < rpw ? wave * rpw + lane : n;
    for (uint32_t q = q0; q < n; q += waves * rpw) {
#ifdef VR_DIAG_SLOW
        const uint64_t t_beg = wall_clock64();
#endif
        slow_ray<S>(A, A.slowq[1 + q], stack, BLOCK, c);
#ifdef VR_DIAG_SLOW
        const uint32_t us = (uint32_t)((wall_clock64() - t_beg) / 100);  // 100 MHz constant clock
        const int kind = s < (uint32_t)A.num_lights;
        atomicAdd(&g_slow_hist[kind][min(31 - __clz(us | 1), 15)], 1u);
        atomicMax(&g_slow_max[kind], us);
        my_max = max(my_max, us);
#endif
    }
#ifdef VR_DIAG_SLOW
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&g_slow_done, 1u) == gridDim.x - 1) {
            printf("slowq n=%u grid=%u max_us env %u light %u\n", n, gridDim.x, atomicAdd(&g_slow_max[0], 0u), atomicAdd(&g_slow_max[1], 0u));
            for (int k = 0; k < 2; ++k)
                for (int b = 0; b < 16; ++b) {
                    const uint32_t v = atomicExch(&g_slow_hist[k][b], 0u);
                    if (v) printf("  %s us<%u: %u\n", k ? "light" : "env", 2u << b, v);
                }
            atomicExch(&g_slow_max[0], 0u);
            atomicExch(&g_slow_max[1], 0u);
            atomicExch(&g_slow_done, 0u);
        }
    }
#endif
    if constexpr (S)
        for (int i = 0; i < kNumCtr; ++i)
            if (c.v[i]) atomicAdd(A.work + kNumCtr + i, (unsigned long long)c.v[i]);
}

// The exact slow path with the wave on one ray at a time (coop_walk; scenes with the 4-wide tree): the queue's
// rays one per wave, so a ray's latency is the tree's depth in node and record loads instead of its whole walk.
template <bool S>
__global__ __launch_bounds__(64) void secondary_slow_coop_kernel(RenderArgs A) {
    __shared__ int s_buf[3 * kCoopCap];
    const uint32_t n = min(A.slowq[0], A.slowq_cap);
    const uint32_t lane = __lane_id();
    Ctr c{};
    for (uint32_t q = blockIdx.x; q < n; q += gridDim.x) {
        const uint64_t t = A.slowq[1 + q];
        const uint32_t per = rays_per_chunk(A), chunk = (uint32_t)(t / per), rem = (uint32_t)(t - (uint64_t)chunk * per);
        uint32_t s, r;
        ray_slot(A, chunk, rem, dev_nrec(A), s, r);
        const float4 pos = A.rec_pos[r];
        const uint4 meta = A.rec_meta[r];
        ActList act{A.rec_act + meta.z, 1, (int)(meta.w & ~kRecBoundary), A.rec_bloom[r]};
        bool ok = true;
        float tr;
        if (s < (uint32_t)A.num_lights) {  // test_integrators.h:202-237
            const LightRecord& lr = A.lights[s];
            float dx = lr.px - pos.x, dy = lr.py - pos.y, dz = lr.pz - pos.z;
            const float dist = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
            normalize3(dx, dy, dz);
            const Ray sr = make_ray(pos.x, pos.y, pos.z, dx, dy, dz);
            tr = light_transmittance_coop<S>(A, sr, dist, act, s_buf, c, ok);
            __builtin_amdgcn_wave_barrier();
            if (!ok && lane == 0) tr = light_transmittance<S>(A, sr, dist, act, s_buf, 1, c);  // a level over kCoopCap
        } else {  // :242-271
            float xi1, xi2, wx, wy, wz;
            env_xi_at(A, A.env_order != nullptr ? A.env_base[r] : env_base_state(meta), s - (uint32_t)A.num_lights, xi1, xi2);
            env_dir(xi1, xi2, wx, wy, wz);
            const Ray er = make_ray(pos.x, pos.y, pos.z, wx, wy, wz);
            tr = env_transmittance_coop<S>(A, er, act, s_buf, c, ok);
            __builtin_amdgcn_wave_barrier();
            if (!ok && lane == 0) tr = env_transmittance<S>(A, er, act, s_buf, 1, c);
        }
        if (lane == 0) A.tr[t] = tr;
        __builtin_amdgcn_wave_barrier();
    }
    if constexpr (S)
        for (int i = 0; i < kNumCtr; ++i)
            if (c.v[i]) atomicAdd(A.work + kNumCtr + i, (unsigned long long)c.v[i]);
}

#ifdef VR_DIAG_LEVELS
__global__ __launch_bounds__(256) void depth_kernel(const int32_t* __restrict__ parent, uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n || i >= (1u << 23)) return;
    uint32_t d = 0;
    for (int32_t x = (int32_t)i; x > 0; x = parent[x] & kNodeIndexMask) ++d;
    g_diag_depth[i] = (uint8_t)min(d, 255u);
}
#endif

// Parent of every 4-wide node with the node's slot in it: parent | (slot + 1) << 28 (root: -1).
__global__ __launch_bounds__(256) void parents_kernel(const HNode4* __restrict__ nodes, uint32_t n, int32_t* __restrict__ parent) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    if (i == 0) parent[0] = -1;
    const int4 c = reinterpret_cast<const int4*>(nodes + i)[3];
    if (c.x > 0) parent[c.x] = (int32_t)(i | (1u << 28));
    if (c.y > 0) parent[c.y] = (int32_t)(i | (2u << 28));
    if (c.z > 0) parent[c.z] = (int32_t)(i | (3u << 28));
    if (c.w > 0) parent[c.w] = (int32_t)(i | (4u << 28));
}

// ---- the secondary rays' own 4-wide tree: the same nodes with tight boxes (round 4) -------------------
// The shared tree's boxes are the primitives' 3-sigma boxes padded by 5 % (gaussian_bounds): the exact
// M-form quadratic of the primary and free-flight rays, evaluated from a camera several units away,
// accepts points a few percent outside the ellipsoid, and their boxes must hold those. The secondary
// rays' whitened test takes the distance from the chord to the centre directly (wquad: |Lp - (h/a) Ld|^2,
// error linear in the origin's whitened distance instead of quadratic), so what it accepts lies within
// ~1e-5 of the ellipsoid, and their tree gets the exact box of {x : x^T M x <= 9}: half extent
// 3 sqrt((M^-1)_kk) from the record's M in double, outward rounding, and a relative pad of
// 2e-4 + 3.2e-7 rw, rw = diag sqrt(trace M) >= the whitened distance of any origin in the scene box
// (diagonal diag): the chord distance's f32 error is ~1.4e-6 rw in e2, i.e. ~8e-8 rw of the radius, so
// the pad keeps a factor >= 4 at any scene scale (C4: 2e-4 .. 6e-4). C4: 9.5 % fewer node steps and 19 %
// fewer primitive tests.
__device__ __forceinline__ uint16_t f16_out(double v, bool up) {  // smallest half >= v (up) / largest <= v
    uint16_t h = __builtin_bit_cast(uint16_t, (_Float16)(float)v);
    for (int it = 0; it < 4; ++it) {
        const double hv = (double)__builtin_bit_cast(_Float16, h);
        if (up ? hv >= v : hv <= v) break;
        const bool neg = (h & 0x8000u) != 0;
        if ((h & 0x7fffu) == 0) h = up ? 0x0001u : 0x8001u;
        else h = (uint16_t)((neg != up) ? h + 1 : h - 1);
    }
    return h;
}
// Tight box of record j (f32, rounded outward); a record whose M is not positive definite keeps an
// infinite box (the secondary kernel then runs the M forms on the shared tree anyway).
__device__ __forceinline__ void tight_box(const GaussianRecord& g, float diag, float lo[3], float hi[3]) {
    const double m0 = g.m00, m1 = g.m01, m2 = g.m02, m3 = g.m11, m4 = g.m12, m5 = g.m22;
    const double c00 = m3 * m5 - m4 * m4, c11 = m0 * m5 - m2 * m2, c22 = m0 * m3 - m1 * m1;
    const double c01 = m2 * m4 - m1 * m5, c02 = m1 * m4 - m2 * m3;
    const double det = m0 * c00 + m1 * c01 + m2 * c02;
    const double s[3] = {c00 / det, c11 / det, c22 / det};
    const double mean[3] = {g.mx, g.my, g.mz};
    const bool pd = m0 > 0.0 && c22 > 0.0 && det > 0.0 && s[0] > 0.0 && s[1] > 0.0 && s[2] > 0.0;
    const double pad = 1.0 + 2e-4 + 3.2e-7 * (double)diag * sqrt(m0 + m3 + m5);
    for (int k = 0; k < 3; ++k) {
        const double h = pd ? 3.0 * sqrt(s[k]) * pad + 1e-6 : INFINITY;
        lo[k] = __double2float_rd(mean[k] - h);
        hi[k] = __double2float_ru(mean[k] + h);
    }
}
// Depth of every 4-wide node (from the parents) and the deepest.
__global__ __launch_bounds__(256) void node_depth_kernel(const int32_t* __restrict__ parent, uint32_t n, uint8_t* __restrict__ depth,
                                                         uint32_t* __restrict__ maxd) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    uint32_t d = 0;
    for (int32_t x = (int32_t)i; x > 0 && d < 255u; x = parent[x] & kNodeIndexMask) ++d;
    depth[i] = (uint8_t)d;
    atomicMax(maxd, d);
}
// One level of the refit, deepest first: every node at `level` gets its children's tight boxes (a leaf:
// the union of its records' boxes; an inner child: the union its own refit left in nbox) as outward
// rounded f16 in the shared tree's normalisation, and leaves the union of them in nbox for its parent.
__global__ __launch_bounds__(256) void refit_kernel(const HNode4* __restrict__ src, HNode4* __restrict__ dst,
                                                    const GaussianRecord* __restrict__ rec, const uint8_t* __restrict__ depth,
                                                    uint32_t level, uint32_t n, float* __restrict__ nbox, float3 hc, float hs,
                                                    float diag) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n || depth[i] != level) return;
    HNode4 h = src[i];
    float ul[3] = {INFINITY, INFINITY, INFINITY}, uh[3] = {-INFINITY, -INFINITY, -INFINITY};
    const double c[3] = {hc.x, hc.y, hc.z};
    for (int s = 0; s < 4; ++s) {
        const int32_t r = h.c[s];
        if (r == 0) continue;  // empty slot: its NaN box stays
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        if (r < 0) {
            const uint32_t first = leaf_first(r), cnt = leaf_count(r);
            for (uint32_t j = first; j < first + cnt; ++j) {
                float a[3], b[3];
                tight_box(rec[j], diag, a, b);
                for (int k = 0; k < 3; ++k) {
                    lo[k] = fminf(lo[k], a[k]);
                    hi[k] = fmaxf(hi[k], b[k]);
                }
            }
        } else {
            for (int k = 0; k < 3; ++k) {
                lo[k] = nbox[6 * (size_t)r + k];
                hi[k] = nbox[6 * (size_t)r + 3 + k];
            }
        }
        for (int k = 0; k < 3; ++k) {
            ul[k] = fminf(ul[k], lo[k]);
            uh[k] = fmaxf(uh[k], hi[k]);
            // never wider than the shared tree's box (both hold the child; the tighter one is kept)
            const uint16_t a = f16_out(((double)lo[k] - c[k]) * (double)hs, false);
            const uint16_t b = f16_out(((double)hi[k] - c[k]) * (double)hs, true);
            const float sa = (float)__builtin_bit_cast(_Float16, h.h[s][k]), sb = (float)__builtin_bit_cast(_Float16, h.h[s][3 + k]);
            if ((float)__builtin_bit_cast(_Float16, a) > sa) h.h[s][k] = a;
            if ((float)__builtin_bit_cast(_Float16, b) < sb) h.h[s][3 + k] = b;
        }
    }
    dst[i] = h;
    for (int k = 0; k < 3; ++k) {
        nbox[6 * (size_t)i + k] = ul[k];
        nbox[6 * (size_t)i + 3 + k] = uh[k];
    }
}

// Start subtree of a record's secondary rays: the deepest 4-wide node whose box holds the record position,
// taking at every level the inner child with the most room. The rays walk that subtree first and then climb to its parents (sec_node4v), so every node is
// still visited at most once, and a ray whose optical-depth cut-off is reached near its origin — most of
// them: the record sits inside an opaque blob's neighbours — skips the descent from the root.
// Every record has an active Gaussian (a step scatters only with sigma_s > 0): the 4-wide node whose
// child is that Gaussian's leaf is a leaf-level node near the record (the Gaussian holds the position),
// found with two loads instead of a descent from the root (record_start_kernel 0.63 -> ~0.1 ms at C4); the
// descent remains for a record without one.
// The secondary rays' per-axis node copy (VR_SEC_SOA): node i's words 4a..4a+3 hold axis a's box bounds as f16
// pairs {min of children 0, 1}, {min of 2, 3}, {max of 0, 1}, {max of 2, 3}; words 12-15 the child refs. A ray
// picks its near and far bound of an axis once per node (the sign of its direction), for all four children at
// once, instead of a min and a max per child and axis (sec_node4v<SOA>).
__global__ __launch_bounds__(256) void soa_nodes_kernel(const HNode4* __restrict__ src, HNode4* __restrict__ dst, uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const HNode4 a = src[i];
    uint32_t w[16];
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
        w[4 * ax + 0] = (uint32_t)a.h[0][ax] | ((uint32_t)a.h[1][ax] << 16);
        w[4 * ax + 1] = (uint32_t)a.h[2][ax] | ((uint32_t)a.h[3][ax] << 16);
        w[4 * ax + 2] = (uint32_t)a.h[0][3 + ax] | ((uint32_t)a.h[1][3 + ax] << 16);
        w[4 * ax + 3] = (uint32_t)a.h[2][3 + ax] | ((uint32_t)a.h[3][3 + ax] << 16);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) w[12 + k] = (uint32_t)a.c[k];
    uint4* o = reinterpret_cast<uint4*>(dst + i);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    o[2] = make_uint4(w[8], w[9], w[10], w[11]);
    o[3] = make_uint4(w[12], w[13], w[14], w[15]);
}

__global__ __launch_bounds__(256) void prim_node_kernel(const HNode4* __restrict__ nodes, uint32_t n, int32_t* __restrict__ map) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const int4 c = reinterpret_cast<const int4*>(nodes + i)[3];
    const int32_t ref[4] = {c.x, c.y, c.z, c.w};
    for (int s = 0; s < 4; ++s)
        if (ref[s] < 0)
            for (uint32_t j = leaf_first(ref[s]); j < leaf_first(ref[s]) + leaf_count(ref[s]); ++j) map[j] = (int32_t)i;
}
__global__ __launch_bounds__(256) void record_start_kernel(RenderArgs A) {
    const uint32_t nrec = dev_nrec(A);
    for (uint32_t r = blockIdx.x * 256u + threadIdx.x; r < nrec; r += gridDim.x * 256u) {
        if (A.prim_node4 != nullptr) {
            const uint4 meta = A.rec_meta[r];
            if ((meta.w & ~kRecBoundary) > 0u) {
                A.rec_start[r] = A.prim_node4[A.rec_act[meta.z]];
                continue;
            }
        }
        const float4 pos = A.rec_pos[r];
        float p[3] = {pos.x, pos.y, pos.z};
        node_space<true>(A, p[0], p[1], p[2]);
        int32_t node = 0;
        for (int depth = 0; depth < kWideStackMax; ++depth) {
            const uint4* np = reinterpret_cast<const uint4*>(A.hnodes4s + node);
            const uint4 q0 = np[0], q1 = np[1], q2 = np[2], rf = np[3];
            const uint32_t w[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
            const int32_t ref[4] = {(int32_t)rf.x, (int32_t)rf.y, (int32_t)rf.z, (int32_t)rf.w};
            float best = 0.0f;
            int32_t next = -1;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float room = INFINITY;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const uint32_t wl = w[(6 * i + k) >> 1], wh = w[(6 * i + 3 + k) >> 1];
                    const float lo = (float)__builtin_bit_cast(_Float16, (uint16_t)(((6 * i + k) & 1) ? (wl >> 16) : (wl & 0xffffu)));
                    const float hi =
                        (float)__builtin_bit_cast(_Float16, (uint16_t)(((6 * i + 3 + k) & 1) ? (wh >> 16) : (wh & 0xffffu)));
                    room = fminf(room, fminf(p[k] - lo, hi - p[k]));
                }
                const bool take = (ref[i] > 0) & (room >= best);  // (a NaN box never has room)
                best = take ? room : best;
                next = take ? ref[i] : next;
            }
            if (next < 0) break;
            node = next;
        }
        A.rec_start[r] = node;
    }
}

// WRecord of every record (vr_internal.h): Cholesky factor of M = Sigma^-1 in double. A record whose M
// is not positive definite gets NaN factors (wintersect never reports a crossing for it).
__global__ __launch_bounds__(256) void whiten_kernel(const GaussianRecord* __restrict__ rec, WRecord* __restrict__ out,
                                                     uint32_t n, uint32_t* bad) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const GaussianRecord g = rec[i];
    const double m00 = g.m00, m01 = g.m01, m02 = g.m02, m11 = g.m11, m12 = g.m12, m22 = g.m22;
    const double l00 = sqrt(m00), l01 = m01 / l00, l02 = m02 / l00;
    const double l11 = sqrt(m11 - l01 * l01), l12 = (m12 - l01 * l02) / l11;
    const double l22 = sqrt(m22 - l02 * l02 - l12 * l12);
    const bool pd = l00 > 0.0 && l11 > 0.0 && l22 > 0.0;  // (sqrt of a negative pivot: NaN, fails too)
    if (!pd) atomicAdd(bad, 1u);  // the host then traces the scene's secondary rays with the M forms
    const float nan = __builtin_nanf("");
    const float dn = (float)((double)g.density * (double)g.norm * 1.2533141373155002512);  // sqrt(pi / 2)
    out[i] = WRecord{g.mx, g.my, g.mz, dn, pd ? (float)l00 : nan, (float)l01, (float)l02, (float)l11,
                     (float)l12, (float)l22, 0.0f, 0.0f};
}

// ---------------------------------------------------------------------------------------------
// Stage 3: per-pixel accumulation in step order (test_integrators.h:237, 272-277, 292).
// ---------------------------------------------------------------------------------------------
// Per-pixel error budget of the secondary optical-depth cut-off. accumulate_kernel weighs a light
// ray's Tr by C = Ts dt I_l / (4 pi d_l^2) and an environment ray's by Ts dt env / NE (per
// channel), so a ray stopped at optical depth >= cut (its true Tr <= e^-cut, output 0) moves the
// pixel by at most C e^-cut. Every ray of the pixel gets an equal share budget / N_p of the
// budget (N_p: the pixel's secondary rays): a record's rays stop at
//   cut_r = ln(Cmax_r * N_p / budget),   Cmax_r = the largest C of the record's rays,
// so the pixel moves by at most sum C e^-cut <= N_p * budget / N_p = budget in every channel.
// (Equal shares minimise the work: dim records deep in a pixel get small cut-offs.)
__device__ __forceinline__ float record_weight(const RenderArgs& A, const float4& pos) {
    float w = fmaxf(fmaxf(fabsf(A.env[0]), fabsf(A.env[1])), fabsf(A.env[2])) / (float)max(A.env_samples, 1);
    for (int l = 0; l < A.num_lights; ++l) {
        const LightRecord& lr = A.lights[l];
        const float dx = lr.px - pos.x, dy = lr.py - pos.y, dz = lr.pz - pos.z;
        const float s = kInv4Pi / (dx * dx + dy * dy + dz * dz);
        w = fmaxf(w, fmaxf(fmaxf(fabsf(lr.ix), fabsf(lr.iy)), fabsf(lr.iz)) * s);
    }
    return pos.w * A.step_size * w;
}

__global__ __launch_bounds__(256) void record_cut_kernel(RenderArgs A, float budget) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= A.num_tiles * 256u) return;
    uint32_t n = 0;
    for (uint32_t r = A.px_first[p]; r != kNoRecord; r = A.rec_next[r]) ++n;
    const float rays = (float)n * (float)(A.num_lights + A.env_samples);
    // 1.001: headroom for the f32 rounding of the weights and of the optical depths themselves
    for (uint32_t r = A.px_first[p]; r != kNoRecord; r = A.rec_next[r])
        A.rec_cut[r] = fminf(kTauCut, fmaxf(0.0f, logf(1.001f * record_weight(A, A.rec_pos[r]) * rays / budget)));
}

// Per-record incident radiance Li + Le (test_integrators.h:212-275), one wave per record chunk: the
// chunk's Tr values are one contiguous run in hand-out order; they are read once, coalesced, into
// LDS as [record][sample] (env_order tells where each environment ray went), then each lane sums its
// record's lights and environment samples in the reference's order. Without env_order a chunk's
// rays are sample-major ([sample][record-in-chunk]) and are read in place (coalesced).
constexpr int kRadBlock = 64;
template <bool ORDERED>
__global__ __launch_bounds__(kRadBlock) void record_radiance_kernel(RenderArgs A) {
    extern __shared__ float s_tr[];  // ORDERED: [record-in-chunk][sample]
    const uint32_t nrec = dev_nrec(A), cr = A.chunk_rec, nl = (uint32_t)A.num_lights, ne = (uint32_t)A.env_samples;
    const uint32_t S = nl + ne, per = rays_per_chunk(A), nch = (nrec + cr - 1u) >> A.chunk_shift;
    for (uint32_t chunk = blockIdx.x; chunk < nch; chunk += gridDim.x) {
        const float* tr = A.tr + (size_t)chunk * per;
        if constexpr (ORDERED) {
          // the chunk gather in 16-B Tr / 8-B order loads (C4: 0.96 ms; 4-B loads 1.59, unrolled 4-B loads 1.85-2.48)
          if ((cr & 3u) == 0u) {  // four rays per load: the light rows and the env entries stay 4-aligned
            const uint32_t nlc = nl * cr;
            const uint16_t* ord = A.env_order + (size_t)chunk * (cr * ne);
            for (uint32_t q = threadIdx.x; q < per / 4u; q += kRadBlock) {
                const uint32_t i = 4u * q;
                const float4 v = *reinterpret_cast<const float4*>(tr + i);
                const float vv[4] = {v.x, v.y, v.z, v.w};
                if (i < nlc) {
                    const uint32_t s = i >> A.chunk_shift, rl = i & (cr - 1u);
#pragma unroll
                    for (int j = 0; j < 4; ++j) s_tr[(rl + j) * S + s] = vv[j];
                } else {
                    const uint2 o = *reinterpret_cast<const uint2*>(ord + (i - nlc));
                    const uint32_t e4[4] = {o.x & 0xffffu, o.x >> 16, o.y & 0xffffu, o.y >> 16};
#pragma unroll
                    for (int j = 0; j < 4; ++j) s_tr[(e4[j] >> 8) * S + nl + (e4[j] & 0xffu)] = vv[j];
                }
            }
          } else
            for (uint32_t i = threadIdx.x; i < per; i += kRadBlock) {
                uint32_t s, rl;
                if (i < nl * cr) {
                    s = i >> A.chunk_shift;
                    rl = i & (cr - 1u);
                } else {
                    const uint32_t v = A.env_order[(size_t)chunk * (cr * ne) + (i - nl * cr)];
                    s = nl + (v & 0xffu);
                    rl = v >> 8;
                }
                s_tr[rl * S + s] = tr[i];
            }
            __syncthreads();
        }
        const uint32_t r = chunk * cr + threadIdx.x;
        if (threadIdx.x < cr && r < nrec) {
            auto t = [&](uint32_t s) { return ORDERED ? s_tr[threadIdx.x * S + s] : tr[s * cr + threadIdx.x]; };
            const float4 pos = A.rec_pos[r];
            float Li0 = 0.0f, Li1 = 0.0f, Li2 = 0.0f;
            for (int l = 0; l < A.num_lights; ++l) {
                const LightRecord& lr = A.lights[l];
                float dx = lr.px - pos.x, dy = lr.py - pos.y, dz = lr.pz - pos.z;
                float dist = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
                float Tr = t((uint32_t)l);
                float d2 = dist * dist;
                Li0 += __fdiv_rn(Tr * lr.ix, d2);
                Li1 += __fdiv_rn(Tr * lr.iy, d2);
                Li2 += __fdiv_rn(Tr * lr.iz, d2);
            }
            float Le0 = 0.0f, Le1 = 0.0f, Le2 = 0.0f;
            for (uint32_t e = 0; e < ne; ++e) {
                float Tr = t(nl + e);
                Le0 += Tr * A.env[0];
                Le1 += Tr * A.env[1];
                Le2 += Tr * A.env[2];
            }
            const float fs = (float)A.env_samples;
            Le0 = __fdiv_rn(Le0, fs) * k4Pi;
            Le1 = __fdiv_rn(Le1, fs) * k4Pi;
            Le2 = __fdiv_rn(Le2, fs) * k4Pi;
            A.rec_rad[r] = make_float4(Li0 + Le0, Li1 + Le1, Li2 + Le2, 0.0f);
        }
        if constexpr (ORDERED) __syncthreads();  // s_tr is reused by the next chunk
    }
}

__global__ __launch_bounds__(256) void accumulate_kernel(RenderArgs A) {
    const uint32_t tile_local = blockIdx.x;
    const int tid = threadIdx.x;
    const uint32_t p = tile_local * 256u + (uint32_t)tid;
    int lx, ly, x, y;
    tile_pixel(A, tile_local, tid, lx, ly, x, y);
    if (!(x < (int)A.width && y < (int)A.height)) {
        store_px(A, tile_local, lx, ly, x, y, 0.0f, 0.0f, 0.0f);
        return;
    }
    const float step = A.step_size;
    float L0 = 0.0f, L1 = 0.0f, L2 = 0.0f;
    for (uint32_t r = A.px_first[p]; r != kNoRecord; r = A.rec_next[r]) {  // step order
        const float Ts = A.rec_pos[r].w;
        const float4 rad = A.rec_rad[r];  // Li + Le
        L0 += ((Ts * rad.x) * step) * kInv4Pi;
        L1 += ((Ts * rad.y) * step) * kInv4Pi;
        L2 += ((Ts * rad.z) * step) * kInv4Pi;
    }
    const float T = A.px_T[p];
    store_px(A, tile_local, lx, ly, x, y, L0 + T * A.env[0], L1 + T * A.env[1], L2 + T * A.env[2]);
}

}  // namespace dev

// ---------------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------------
#ifndef VR_MARCH_BLOCK
#define VR_MARCH_BLOCK 64  // lanes per march workgroup: 256 (a tile) or 64 (a quarter tile; -6 % march time)
#endif
#ifndef VR_MARCH_ACT
#define VR_MARCH_ACT 16  // active-list LDS slots per lane of the primary march (A/B)
#endif
#ifndef VR_MARCH_STACK4
#define VR_MARCH_STACK4 14  // LDS stack entries per lane of the primary march's 4-wide walks (A/B; then VR_MARCH_DEEP)
#endif
#ifndef VR_MARCH_ACT_BIG
#define VR_MARCH_ACT_BIG 32  // the primary march's slots once a scene's frames overflow 16 on >= 5 % of their pixels
#endif
constexpr int kActFast = VR_MARCH_ACT, kActBig = VR_MARCH_ACT_BIG, kBlockFast = VR_MARCH_BLOCK;
constexpr int kActFallback = 64, kBlockFallback = 64;
constexpr int kBlockSecondary = 256;

hipError_t gauss_bin(const RenderArgs& A, bool emit, hipStream_t stream) {
    const unsigned grid = (unsigned)std::min<uint64_t>(((uint64_t)A.num_prims + 255) / 256, 16384);
    if (emit) hipLaunchKernelGGL(dev::bin_kernel<true>, dim3(std::max(grid, 1u)), dim3(256), 0, stream, A);
    else hipLaunchKernelGGL(dev::bin_kernel<false>, dim3(std::max(grid, 1u)), dim3(256), 0, stream, A);
    return hipGetLastError();
}

hipError_t gauss_bin_scan(const uint32_t* cnt, uint32_t* off, uint32_t n, void* tmp, size_t& tmp_bytes, hipStream_t stream) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, off, (int)n, stream);
}

template <bool S, bool H>
static hipError_t march_pass(const RenderArgs& A, hipStream_t stream) {
    // LDS per 256-lane workgroup = (active-list slots + stack entries) * 1 KiB. Shallow trees use a
    // 24-entry stack; the 16-slot active list overflows to the 64-slot fallback kernel. H: the
    // half-precision node copy (boxes only propose candidates; every decision is the exact quadratic).
    const bool shallow = A.bvh_depth <= kShallowStack + 1;
    if (A.bin_ent != nullptr)  // binned march (its overflowing pixels re-run in the BVH fallback below)
        hipLaunchKernelGGL((dev::march_binned_kernel<S>), dim3(A.num_tiles * 4), dim3(64), 0, stream, A);
    else if (H && A.hnodes4 != nullptr && A.march_big)  // translucent, densely overlapping scenes (C2): fewer
        // pixels overflow, and their records come from coherent quarter tiles instead of the fallback queue
        hipLaunchKernelGGL((dev::march_kernel<kActBig, kBlockFast, S, VR_MARCH_STACK4, true, true>), dim3(A.num_tiles * (256 / kBlockFast)),
                           dim3(kBlockFast), 0, stream, A);
    else if (H && A.hnodes4 != nullptr)  // 4-wide tree; a query that could overflow the stack goes to the fallback
        hipLaunchKernelGGL((dev::march_kernel<kActFast, kBlockFast, S, VR_MARCH_STACK4, true, true>), dim3(A.num_tiles * (256 / kBlockFast)),
                           dim3(kBlockFast), 0, stream, A);
    else if (shallow)
        hipLaunchKernelGGL((dev::march_kernel<kActFast, kBlockFast, S, kShallowStack, H>), dim3(A.num_tiles * (256 / kBlockFast)),
                           dim3(kBlockFast), 0, stream, A);
    else
        hipLaunchKernelGGL((dev::march_kernel<kActFast, kBlockFast, S, kStackSize, H>), dim3(A.num_tiles * (256 / kBlockFast)),
                           dim3(kBlockFast), 0, stream, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (H && A.hnodes4 != nullptr)  // the one-pixel-per-wave fallback march walks the 4-wide tree
        hipLaunchKernelGGL((dev::march_fallback_kernel<kActFallback, kBlockFallback, S, H, true>), dim3(1024), dim3(kBlockFallback), 0,
                           stream, A);
    else
        hipLaunchKernelGGL((dev::march_fallback_kernel<kActFallback, kBlockFallback, S, H>), dim3(1024), dim3(kBlockFallback), 0,
                           stream, A);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (H && A.hnodes4 != nullptr)  // (exactly one of the two passes takes the queue, by its length)
        hipLaunchKernelGGL((dev::march_wide_kernel<S, H, true>), dim3(kWideThreads / kWideBlock), dim3(kWideBlock), 0, stream, A);
    else
        hipLaunchKernelGGL((dev::march_wide_kernel<S, H, false>), dim3(kWideThreads / kWideBlock), dim3(kWideBlock), 0, stream, A);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL((dev::march_deep_kernel<S, H>), dim3(kDeepThreads / kDeepBlock), dim3(kDeepBlock), 0, stream, A);
    return hipGetLastError();
}

hipError_t gauss_march(const RenderArgs& A, hipStream_t stream, bool stats) {
    if (A.hnodes != nullptr) return stats ? march_pass<true, true>(A, stream) : march_pass<false, true>(A, stream);
    return stats ? march_pass<true, false>(A, stream) : march_pass<false, false>(A, stream);
}

// One launch of the persistent kernel: one resident grid (every CU filled to the kernel's occupancy).
// LDS words per lane: 14 traversal-stack entries (deeper ones overflow to global memory) + the
// 8-entry LDS ring of the 9-entry leaf queue = 22 (7 blocks of 256 lanes per CU).
template <bool S, bool PURE, bool H, bool W, bool WH = !PURE, bool SOA = false>
static hipError_t ww_launch(const RenderArgs& A, hipStream_t stream) {
#ifndef VR_WW_STACK
#define VR_WW_STACK 14  // LDS traversal-stack entries per lane (deeper ones spill to the global overflow)
#endif
#ifndef VR_WW_WAVES
#define VR_WW_WAVES 7  // waves per SIMD (launch bounds: 72 VGPRs at 7; A/B at C4: 7 + 14-entry stack 95.6 ms, 6 + 18 99.2 ms)
#endif
#ifndef VR_WW_QCAP
#define VR_WW_QCAP 9  // leaf queue of the persistent kernel: the head entry + an LDS ring of QCAP - 1 (1 + 2^k)
#endif
    constexpr int kStack = VR_WW_STACK, kQueue = VR_WW_QCAP;
    constexpr int kWaves = PURE ? 5 : WH ? VR_WW_WAVES : 6;  // PureRayMarching's marched depth does not fit 80 VGPRs without spills
    const void* fn = (const void*)dev::secondary_ww_kernel<kBlockSecondary, kStack, S, PURE, kWaves, kQueue, H, W, WH, SOA>;
    int dv = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dv) != hipSuccess) return hipErrorUnknown;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dv) != hipSuccess) return hipErrorUnknown;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlockSecondary, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    uint64_t grid = (uint64_t)cus * (uint64_t)per_cu;
    if (grid * kBlockSecondary > A.stack_ovf_lanes) grid = A.stack_ovf_lanes / kBlockSecondary;  // overflow slots
    if (grid == 0) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(A.ray_next, 0, sizeof(unsigned long long), stream);
    if (e != hipSuccess) return e;
    RenderArgs B = A;  // the tight tree only under the whitened test (the M forms: the shared tree's padded boxes)
    if (PURE || !WH) B.hnodes4s = A.hnodes4;
    if (SOA && B.hnodes4s == A.hnodes4) B.hnodes4t = A.hnodes4w;  // the per-axis copy of the tree walked
    hipLaunchKernelGGL((dev::secondary_ww_kernel<kBlockSecondary, kStack, S, PURE, kWaves, kQueue, H, W, WH, SOA>), dim3((unsigned)grid),
                       dim3(kBlockSecondary), 0, stream, B);
    return hipGetLastError();
}

template <bool S, bool PURE>
static hipError_t secondary_launch(const RenderArgs& A, hipStream_t stream) {
    hipError_t e;
    // (4-wide trees: the node step reads the per-axis copy of the tree the variant walks, VR_SEC_SOA)
    if (!PURE && A.wrec == nullptr) {  // a record without a Cholesky factor: the M forms (rare scenes)
        if (A.hnodes != nullptr && A.hnodes4 != nullptr) e = ww_launch<S, PURE, true, true, false, VR_SEC_SOA != 0>(A, stream);
        else if (A.hnodes != nullptr) e = ww_launch<S, PURE, true, false, false>(A, stream);
        else e = ww_launch<S, PURE, false, false, false>(A, stream);
    } else if (A.hnodes != nullptr && A.hnodes4 != nullptr)  // 4-wide half-precision tree
        e = ww_launch<S, PURE, true, true, !PURE, VR_SEC_SOA != 0>(A, stream);
    else if (A.hnodes != nullptr)
        e = ww_launch<S, PURE, true, false>(A, stream);
    else  // f32 child-pair tree (scenes whose leaf boxes are too small for f16 boxes)
        e = ww_launch<S, PURE, false, false>(A, stream);
    if (e != hipSuccess) return e;
    if (!PURE) {  // PureRayMarching has no first-event-past-the-light quirk, hence no slow path
#ifndef VR_SLOW_GRID
#define VR_SLOW_GRID 4096  // workgroups of the exact slow path (grid-stride over its queue; 32 k rays a pass at 8 per wave)
#endif
        hipLaunchKernelGGL(dev::secondary_fix_kernel, dim3(1024), dim3(64), 0, stream, A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
#ifndef VR_SLOW_COOP
#define VR_SLOW_COOP 1  // 1: the wave-cooperative exact slow path on scenes with the 4-wide tree (A/B)
#endif
#ifndef VR_SLOW_COOP_GRID
#define VR_SLOW_COOP_GRID 8192  // one-wave workgroups of the cooperative slow path (one queued ray at a time each)
#endif
        if (VR_SLOW_COOP && A.hnodes4 != nullptr)
            hipLaunchKernelGGL(dev::secondary_slow_coop_kernel<S>, dim3(VR_SLOW_COOP_GRID), dim3(64), 0, stream, A);
        else
            hipLaunchKernelGGL((dev::secondary_slow_kernel<64, S>), dim3(VR_SLOW_GRID), dim3(64), 0, stream, A);
        e = hipGetLastError();
    }
    return e;
}

// Grid for a per-record kernel over at most rec_cap records (the live count is read on the device).
static unsigned record_grid(const RenderArgs& A, uint32_t per_block, unsigned max_blocks) {
    const uint64_t b = ((uint64_t)A.rec_cap + per_block - 1) / per_block;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, max_blocks));
}

hipError_t gauss_secondary(const RenderArgs& A, hipStream_t stream, bool stats) {
    if (A.num_lights + A.env_samples == 0) return hipSuccess;
#ifdef VR_DIAG_LEVELS
    if (A.hn4_parent != nullptr && A.num_nodes4 > 0)
        hipLaunchKernelGGL(dev::depth_kernel, dim3((A.num_nodes4 + 255) / 256), dim3(256), 0, stream, A.hn4_parent, A.num_nodes4);
#endif
    if (A.rec_start != nullptr) {  // every record's start subtree (the 4-wide walk with parents only)
        hipLaunchKernelGGL(dev::record_start_kernel, dim3(record_grid(A, 256, 16384)), dim3(256), 0, stream, A);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (A.env_order != nullptr) {
        hipLaunchKernelGGL(dev::env_order_kernel<256>, dim3(record_grid(A, A.chunk_rec * 4, 4096)), dim3(256), 0,
                           stream, A);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    // stats: the instrumented build of the same persistent kernel (vr_count_work), which counts
    // the work this schedule really does (node steps, list and leaf primitive tests, optical depths)
    if (A.pure) return stats ? secondary_launch<true, true>(A, stream) : secondary_launch<false, true>(A, stream);
    return stats ? secondary_launch<true, false>(A, stream) : secondary_launch<false, false>(A, stream);
}

hipError_t gauss_parents(const HNode4* nodes, uint32_t n, int32_t* parent, int32_t* prim_node, hipStream_t stream) {
    hipLaunchKernelGGL(dev::parents_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, nodes, n, parent);
    if (prim_node != nullptr) hipLaunchKernelGGL(dev::prim_node_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, nodes, n, prim_node);
    return hipGetLastError();
}

// The secondary rays' tree (refit_kernel): nodes 0..n-1 of `src` with tight boxes into `dst`. Scratch:
// depth (n B), nbox (24 n B), maxd (one word, device) and host_maxd (pinned or pageable host word).
hipError_t gauss_refit_secondary(const HNode4* src, HNode4* dst, HNode4* dst_t, uint32_t n, const GaussianRecord* rec,
                                 const int32_t* parent, uint8_t* depth, float* nbox, uint32_t* maxd, const float hc[3], float hs,
                                 float diag, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(maxd, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(dev::node_depth_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, parent, n, depth, maxd);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    uint32_t md = 0;
    if ((e = hipMemcpyAsync(&md, maxd, sizeof(uint32_t), hipMemcpyDeviceToHost, stream)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return e;
    if (md >= 255u) return hipErrorNotSupported;
    const float3 c = make_float3(hc[0], hc[1], hc[2]);
    for (int level = (int)md; level >= 0; --level) {
        hipLaunchKernelGGL(dev::refit_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, src, dst, rec, depth, (uint32_t)level, n,
                           nbox, c, hs, diag);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (dst_t != nullptr) {
        hipLaunchKernelGGL(dev::soa_nodes_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, dst, dst_t, n);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t gauss_soa_nodes(const HNode4* src, HNode4* dst, uint32_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::soa_nodes_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, src, dst, n);
    return hipGetLastError();
}

hipError_t gauss_whiten(const GaussianRecord* rec, WRecord* out, uint32_t n, uint32_t* bad, hipStream_t stream) {
    hipLaunchKernelGGL(dev::whiten_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, rec, out, n, bad);
    return hipGetLastError();
}

hipError_t gauss_record_cut(const RenderArgs& A, float budget, hipStream_t stream) {
    if (A.rec_cut == nullptr) return hipSuccess;
    hipLaunchKernelGGL(dev::record_cut_kernel, dim3(A.num_tiles), dim3(256), 0, stream, A, budget);
    return hipGetLastError();
}

hipError_t gauss_accumulate(const RenderArgs& A, hipStream_t stream) {
    {  // (also with no secondary rays: Le = 0 / 0 reproduces the reference's NaN for env_samples = 0)
        const dim3 grid(record_grid(A, A.chunk_rec, 65536));
        if (A.env_order != nullptr)  // <= 64 KB of LDS: env_samples <= kEnvOrderMax, lights <= kMaxLights
            hipLaunchKernelGGL(dev::record_radiance_kernel<true>, grid, dim3(dev::kRadBlock),
                               (size_t)A.chunk_rec * (size_t)(A.num_lights + A.env_samples) * sizeof(float), stream, A);
        else
            hipLaunchKernelGGL(dev::record_radiance_kernel<false>, grid, dim3(dev::kRadBlock), 0, stream, A);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(dev::accumulate_kernel, dim3(A.num_tiles), dim3(256), 0, stream, A);
    return hipGetLastError();
}

}  // namespace vr
