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
//   2. secondary_kernel (one thread per secondary ray, sample-major order so that consecutive
//      lanes trace rays towards the same light from neighbouring pixels): transmittance of every
//      light / environment ray of every record.
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
#include <hipcub/hipcub.hpp>

#include "vr_dev_common.h"

namespace vr {
namespace dev {

// Optical-depth cut-off of a secondary ray: expf(-104) rounds to 0 in f32 and every optical depth
// is >= 0, so once the running sum reaches kTauCut the ray's transmittance is exactly 0 whatever
// else it crosses — the traversal stops there. (The reference's product of per-segment
// exponentials reaches 0 or a denormal <= 1.4e-45 at the same point.)
constexpr float kTauCut = 104.0f;

// ---------------------------------------------------------------------------------------------
// Secondary-ray transmittance (shared by the secondary kernel)
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
    traverse(
        A.nodes, sr, stack, stride, [&](float tmin, float) { return tmin <= dist + kTPad * (1.0f + dist); },
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
                    hitmask |= 1ull << slot;
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
        NodeCount<S>{&c});
    uint64_t all = act.n >= 64 ? ~0ull : ((1ull << act.n) - 1ull);
    uint64_t missed = all & ~hitmask;  // pre-activated but not intersected (rounding at the surface)
    if (tau >= kTauCut) return 0.0f;   // exp(-tau) == 0 exactly; later terms are >= 0
    if (needs_stop || missed) {
        float tstop = INFINITY;  // first event at or beyond the light
        traverse(
            A.nodes, sr, stack, stride,
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
            NodeCount<S>{&c});
        if (tstop == INFINITY) tstop = dist;
        if (needs_stop) {
            traverse(
                A.nodes, sr, stack, stride,
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
                NodeCount<S>{&c});
        }
        while (missed) {
            int s = __ffsll((unsigned long long)missed) - 1;
            missed &= missed - 1;
            GRec g = load_rec(G, act.get(s));
            Quad q = quad(g, sr);
            if constexpr (S) c.v[kCtrOD]++;
            tau += optical_depth(g, q, 0.0f, tstop);
        }
    }
    return expf(-tau);
}

// Environment ray, to its last event (test_integrators.h:241-273).
template <bool S>
__device__ float env_transmittance(const RenderArgs& A, const Ray& er, const ActList& act, int* stack, int stride,
                                   Ctr& c) {
    const GaussianRecord* __restrict__ G = A.gauss;
    float tau = 0.0f, tlast = 0.0f;
    uint64_t hitmask = 0;
    traverse(
        A.nodes, er, stack, stride, [&](float, float) { return true; },
        [&](uint32_t first, uint32_t count) {
            for (uint32_t j = first; j < first + count; ++j) {
                if constexpr (S) c.v[kCtrPrims]++;
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
                if constexpr (S) c.v[kCtrOD]++;
                tau += optical_depth(g, q, lo, b);
                tlast = fmaxf(tlast, b);
            }
            return tau < kTauCut;
        },
        NodeCount<S>{&c});
    if (tau >= kTauCut) return 0.0f;
    uint64_t all = act.n >= 64 ? ~0ull : ((1ull << act.n) - 1ull);
    uint64_t missed = all & ~hitmask;
    while (missed) {
        int s = __ffsll((unsigned long long)missed) - 1;
        missed &= missed - 1;
        GRec g = load_rec(G, act.get(s));
        Quad q = quad(g, er);
        if constexpr (S) c.v[kCtrOD]++;
        tau += optical_depth(g, q, 0.0f, tlast);
    }
    return expf(-tau);
}

// ---------------------------------------------------------------------------------------------
// Stage 1: primary march
// ---------------------------------------------------------------------------------------------
// MODE 0: count scatter records / active entries of pixel p. MODE 1: write them (offsets from the
// scan of MODE 0's counts). Both modes run the identical march, so they agree record for record.
template <int ACT, int MODE, bool S>
__device__ int march(const RenderArgs& A, uint32_t p, int px, int py, int* act_base, int* stack, int stride, Ctr& c) {
    const Ray ray = primary_ray(A, px, py);
    const GaussianRecord* __restrict__ G = A.gauss;
    const float* __restrict__ ts = A.tsteps;
    const int nts = A.num_tsteps;
    const float step = A.step_size;
    float T = 1.0f;
    uint32_t nrec = 0, nact = 0;
    uint32_t rbase = 0, abase = 0;
    if constexpr (MODE == 1) {
        rbase = A.px_off[p];
        abase = A.px_aoff[p];
    }
    ActList act{act_base, stride, 0, 0};
    int kq = 0;
    if (A.num_prims > 0) {
        for (;;) {
            const float t_lo = (kq == 0) ? -1.0f : ts[kq - 1];
            int k;
            if (act.n == 0) {  // closest entry strictly after t_lo
                if constexpr (S) c.v[kCtrPrimQueries]++;
                float best = INFINITY;
                traverse(
                    A.nodes, ray, stack, stride,
                    [&](float tmin, float tmax) {
                        return tmax >= t_lo - kTPad * (1.0f + fabsf(t_lo)) && tmin <= best + kTPad * (1.0f + best);
                    },
                    [&](uint32_t first, uint32_t count) {
                        for (uint32_t j = first; j < first + count; ++j) {
                            if constexpr (S) c.v[kCtrPrims]++;
                            GRec g = load_rec(G, j);
                            Quad q = quad(g, ray);
                            float a, b;
                            if (intersect(q, a, b) && a > t_lo && a < best) best = a;
                        }
                        return true;
                    },
                    NodeCount<S>{&c});
                if (best == INFINITY) break;
                k = kfirst(ts, nts, step, best);
            } else {
                k = kq;
            }
            if (k >= nts - 1) return kError;  // step table too short (host sizes it from scene bounds)
            const float t_k = ts[k];
            // entrants: t_lo < a <= t_k and still inside at t_k (b > t_k)
            if constexpr (S) c.v[kCtrPrimQueries]++;
            bool ovf = false;
            traverse(
                A.nodes, ray, stack, stride,
                [&](float tmin, float tmax) {
                    return tmax >= t_lo - kTPad * (1.0f + fabsf(t_lo)) && tmin <= t_k + kTPad * (1.0f + t_k);
                },
                [&](uint32_t first, uint32_t count) {
                    for (uint32_t j = first; j < first + count; ++j) {
                        if constexpr (S) c.v[kCtrPrims]++;
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
                    return true;
                },
                NodeCount<S>{&c});
            if (ovf) return kOverflow;
            kq = k + 1;
            // retire (b <= t_k); sigma at pos (gmm.h:98-126); the step's optical depth (:146-157)
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
                if (!intersect(q, a, b) || b <= t_k) continue;
                act.set(w++, j);
                float m = mu_t(g, px_, py_, pz_);
                smu += m;
                smua += m * g.albedo;
                tau_seg += optical_depth(g, q, t_k, t_k1);
                if constexpr (S) {
                    c.v[kCtrMu]++;
                    c.v[kCtrOD]++;
                    c.v[kCtrPrims]++;
                }
            }
            act.n = w;
            if (w == 0) continue;
            if constexpr (S) c.v[kCtrSteps]++;
            float sigma_s = 0.0f;
            if (smu > 0.0f) {
                float a_mix = smua / smu;
                sigma_s = a_mix * smu;
            }
            if (sigma_s > 0.0f) {  // scattering step -> one record
                if constexpr (MODE == 1) {
                    // never write past the slots MODE 0 reserved for this pixel
                    if (nrec >= A.px_cnt[p] || nact + (uint32_t)w > A.px_acnt[p]) return kError;
                    uint32_t r = rbase + nrec;
                    A.rec_pos[r] = make_float4(px_, py_, pz_, T * sigma_s);
                    A.rec_meta[r] = make_uint4((uint32_t)px | ((uint32_t)py << 16), (uint32_t)k, abase + nact, (uint32_t)w);
                    for (int i = 0; i < w; ++i) A.rec_act[abase + nact + i] = act.get(i);
                }
                nrec++;
                nact += (uint32_t)w;
            }
            T *= expf(-tau_seg);
            if (T <= A.t_eps) break;
        }
    }
    if constexpr (MODE == 0) {
        A.px_cnt[p] = nrec;
        A.px_acnt[p] = nact;
    } else {
        A.px_T[p] = T;
        if constexpr (S) c.v[kCtrPixels]++;
    }
    return kOK;
}

__device__ __forceinline__ void mark_error(const RenderArgs& A, uint32_t p, int mode) {
    atomicAdd(A.counters, 1u);
    if (mode == 0) {
        A.px_cnt[p] = 0;
        A.px_acnt[p] = 0;
    } else {
        A.px_T[p] = __builtin_nanf("");
    }
}

template <int ACT, int BLOCK, int MODE, bool S>
__global__ __launch_bounds__(BLOCK) void march_kernel(RenderArgs A) {
    __shared__ int s_act[ACT * BLOCK];
    __shared__ int s_stack[kStackSize * BLOCK];
    const int tid = threadIdx.x;
    const uint32_t tile_local = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t p = tile_local * 256u + (uint32_t)tid;
    int lx, ly, x, y;
    tile_pixel(A, tile_local, tid, lx, ly, x, y);
    Ctr c{};
    int st = kOK;
    if (x < (int)A.width && y < (int)A.height) {
        st = march<ACT, MODE, S>(A, p, x, y, s_act + tid, s_stack + tid, BLOCK, c);
    } else if constexpr (MODE == 0) {
        A.px_cnt[p] = 0;
        A.px_acnt[p] = 0;
    } else {
        A.px_T[p] = 0.0f;
    }
    if constexpr (S) flush_counters(A.work, c);
    if (st == kOverflow) {
        uint32_t slot = atomicAdd(A.queue, 1u);
        if (slot < A.queue_cap) A.queue[1 + slot] = p;
        else mark_error(A, p, MODE);
    } else if (st == kError) {
        mark_error(A, p, MODE);
    }
}

template <int ACT, int BLOCK, int MODE, bool S>
__global__ __launch_bounds__(BLOCK) void march_fallback_kernel(RenderArgs A) {
    __shared__ int s_act[ACT * BLOCK];
    __shared__ int s_stack[kStackSize * BLOCK];
    const int tid = threadIdx.x;
    const uint32_t n = min(A.queue[0], A.queue_cap);
    for (uint32_t q = blockIdx.x * BLOCK + tid; q < n; q += gridDim.x * BLOCK) {
        const uint32_t p = A.queue[1 + q];
        int lx, ly, x, y;
        tile_pixel(A, p >> 8, (int)(p & 255u), lx, ly, x, y);
        Ctr c{};
        int st = march<ACT, MODE, S>(A, p, x, y, s_act + tid, s_stack + tid, BLOCK, c);
        if constexpr (S)
            for (int i = 0; i < kNumCtr; ++i) atomicAdd(A.work + i, (unsigned long long)c.v[i]);
        if (st != kOK) mark_error(A, p, MODE);
    }
}

__global__ void totals_kernel(const uint32_t* cnt, const uint32_t* off, const uint32_t* acnt, const uint32_t* aoff,
                              uint32_t n, uint32_t* totals) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        totals[0] = n ? off[n - 1] + cnt[n - 1] : 0u;
        totals[1] = n ? aoff[n - 1] + acnt[n - 1] : 0u;
    }
}

// ---------------------------------------------------------------------------------------------
// Stage 2: one thread per secondary ray. Ray id t = s * nrec + r (sample-major).
// ---------------------------------------------------------------------------------------------
template <int BLOCK, bool S>
__global__ __launch_bounds__(BLOCK) void secondary_kernel(RenderArgs A, uint32_t nrec) {
    __shared__ int s_stack[kStackSize * BLOCK];
    int* stack = s_stack + threadIdx.x;
    const uint32_t nsamp = (uint32_t)(A.num_lights + A.env_samples);
    const uint64_t total = (uint64_t)nrec * nsamp;
    Ctr c{};
    const uint64_t stride_t = (uint64_t)gridDim.x * BLOCK;
    const uint64_t t0 = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t rounds = (total + stride_t - 1) / stride_t;  // uniform trip count (all lanes flush)
    for (uint64_t it = 0; it < rounds; ++it) {
        const uint64_t t = t0 + it * stride_t;
        if (t >= total) continue;
        const uint32_t s = (uint32_t)(t / nrec);
        const uint32_t r = (uint32_t)(t - (uint64_t)s * nrec);
        const float4 pos = A.rec_pos[r];
        const uint4 meta = A.rec_meta[r];
        ActList act{A.rec_act + meta.z, 1, (int)meta.w, 0};
        act.rebuild_bloom();
        if constexpr (S) c.v[kCtrSecRays]++;
        float Tr;
        if (s < (uint32_t)A.num_lights) {
            const LightRecord& lr = A.lights[s];
            float dx = lr.px - pos.x, dy = lr.py - pos.y, dz = lr.pz - pos.z;
            float dist = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
            normalize3(dx, dy, dz);
            Ray sr = make_ray(pos.x, pos.y, pos.z, dx, dy, dz);
            Tr = light_transmittance<S>(A, sr, dist, act, stack, BLOCK, c);
        } else {
            const uint32_t e = s - (uint32_t)A.num_lights;
            const int px = (int)(meta.x & 0xffffu), py = (int)(meta.x >> 16);
            PCG32 rng(derive_path_seed(px, py, (int)meta.y), 1);
            for (uint32_t i = 0; i < 2 * e; ++i) rng.next_u32();
            float xi1 = rng.uniform();
            float xi2 = rng.uniform();
            float wx, wy, wz;
            env_dir(xi1, xi2, wx, wy, wz);
            Ray er = make_ray(pos.x, pos.y, pos.z, wx, wy, wz);
            Tr = env_transmittance<S>(A, er, act, stack, BLOCK, c);
        }
        A.tr[t] = Tr;
    }
    if constexpr (S) flush_counters(A.work, c);
}

// ---------------------------------------------------------------------------------------------
// Stage 3: per-pixel accumulation in step order (test_integrators.h:237, 272-277, 292).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void accumulate_kernel(RenderArgs A, uint32_t nrec) {
    const uint32_t tile_local = blockIdx.x;
    const int tid = threadIdx.x;
    const uint32_t p = tile_local * 256u + (uint32_t)tid;
    int lx, ly, x, y;
    tile_pixel(A, tile_local, tid, lx, ly, x, y);
    if (!(x < (int)A.width && y < (int)A.height)) {
        store_px(A, tile_local, lx, ly, x, y, 0.0f, 0.0f, 0.0f);
        return;
    }
    const uint32_t n = A.px_cnt[p], o = A.px_off[p];
    const float fs = (float)A.env_samples;
    const float step = A.step_size;
    float L0 = 0.0f, L1 = 0.0f, L2 = 0.0f;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t r = o + i;
        const float4 pos = A.rec_pos[r];
        float Li0 = 0.0f, Li1 = 0.0f, Li2 = 0.0f;
        for (int l = 0; l < A.num_lights; ++l) {
            const LightRecord& lr = A.lights[l];
            float dx = lr.px - pos.x, dy = lr.py - pos.y, dz = lr.pz - pos.z;
            float dist = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
            float Tr = A.tr[(size_t)l * nrec + r];
            float d2 = dist * dist;
            Li0 += __fdiv_rn(Tr * lr.ix, d2);
            Li1 += __fdiv_rn(Tr * lr.iy, d2);
            Li2 += __fdiv_rn(Tr * lr.iz, d2);
        }
        float Le0 = 0.0f, Le1 = 0.0f, Le2 = 0.0f;
        for (int e = 0; e < A.env_samples; ++e) {
            float Tr = A.tr[(size_t)(A.num_lights + e) * nrec + r];
            Le0 += Tr * A.env[0];
            Le1 += Tr * A.env[1];
            Le2 += Tr * A.env[2];
        }
        Le0 = __fdiv_rn(Le0, fs) * k4Pi;
        Le1 = __fdiv_rn(Le1, fs) * k4Pi;
        Le2 = __fdiv_rn(Le2, fs) * k4Pi;
        const float Ts = pos.w;
        L0 += ((Ts * (Li0 + Le0)) * step) * kInv4Pi;
        L1 += ((Ts * (Li1 + Le1)) * step) * kInv4Pi;
        L2 += ((Ts * (Li2 + Le2)) * step) * kInv4Pi;
    }
    const float T = A.px_T[p];
    store_px(A, tile_local, lx, ly, x, y, L0 + T * A.env[0], L1 + T * A.env[1], L2 + T * A.env[2]);
}

}  // namespace dev

// ---------------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------------
constexpr int kActFast = 32, kBlockFast = 256;
constexpr int kActFallback = 64, kBlockFallback = 64;
constexpr int kBlockSecondary = 256;

template <int MODE, bool S>
static hipError_t march_pass(const RenderArgs& A, hipStream_t stream) {
    hipLaunchKernelGGL((dev::march_kernel<kActFast, kBlockFast, MODE, S>), dim3(A.num_tiles), dim3(kBlockFast), 0, stream, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((dev::march_fallback_kernel<kActFallback, kBlockFallback, MODE, S>), dim3(1024), dim3(kBlockFallback),
                       0, stream, A);
    return hipGetLastError();
}

hipError_t gauss_march(const RenderArgs& A, hipStream_t stream, int mode, bool stats) {
    if (mode == 0) return stats ? march_pass<0, true>(A, stream) : march_pass<0, false>(A, stream);
    return stats ? march_pass<1, true>(A, stream) : march_pass<1, false>(A, stream);
}

// Exclusive scans of the per-pixel counts + totals. temp == nullptr queries temp_bytes.
hipError_t gauss_scan(const RenderArgs& A, uint32_t npix, void* temp, size_t& temp_bytes, uint32_t* totals,
                      hipStream_t stream) {
    if (!temp) {
        size_t b = 0;
        hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, b, A.px_cnt, A.px_off, (int)npix, stream);
        temp_bytes = b;
        return e;
    }
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, A.px_cnt, A.px_off, (int)npix, stream);
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, A.px_acnt, A.px_aoff, (int)npix, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(dev::totals_kernel, dim3(1), dim3(64), 0, stream, A.px_cnt, A.px_off, A.px_acnt, A.px_aoff, npix,
                       totals);
    return hipGetLastError();
}

hipError_t gauss_secondary(const RenderArgs& A, uint32_t nrec, hipStream_t stream, bool stats) {
    uint64_t total = (uint64_t)nrec * (uint64_t)(A.num_lights + A.env_samples);
    if (total == 0) return hipSuccess;
    uint64_t blocks = (total + kBlockSecondary - 1) / kBlockSecondary;
    if (blocks > 65536ull * 16ull) blocks = 65536ull * 16ull;
    if (stats)
        hipLaunchKernelGGL((dev::secondary_kernel<kBlockSecondary, true>), dim3((unsigned)blocks), dim3(kBlockSecondary), 0,
                           stream, A, nrec);
    else
        hipLaunchKernelGGL((dev::secondary_kernel<kBlockSecondary, false>), dim3((unsigned)blocks), dim3(kBlockSecondary), 0,
                           stream, A, nrec);
    return hipGetLastError();
}

hipError_t gauss_accumulate(const RenderArgs& A, uint32_t nrec, hipStream_t stream) {
    hipLaunchKernelGGL(dev::accumulate_kernel, dim3(A.num_tiles), dim3(256), 0, stream, A, nrec);
    return hipGetLastError();
}

}  // namespace vr
