// RayMarchingSpheres (test_integrators.h:23-135), TestIntegrator (integrator.h:65-94) and the
// multi-GPU tile unshuffle, for gfx950.
#include <hip/hip_runtime.h>

#include "vr_dev_common.h"

namespace vr {
namespace dev {

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
                float xi1 = rng.uniform_env();
                float xi2 = rng.uniform_env();
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
            traverse<false>(A, ray, s_stack + threadIdx.x, BLOCK, [&](float, float) { return !any; },
                     [&](uint32_t first, uint32_t count) {
                         for (uint32_t j = first; j < first + count; ++j) {
                             GRec gg = load_rec(A.gauss, j);
                             float a, bb;
                             if (intersect(quad(gg, ray), a, bb)) any = true;
                         }
                         return !any;
                     });
        }
        if (any) { r = 1.0f; g = 0.0f; b = 1.0f; }
        else { r = A.env[0]; g = A.env[1]; b = A.env[2]; }
    }
    store_px(A, tile_local, lx, ly, x, y, r, g, b);
}

// Slabs (rank r holds tiles r, r + nslabs, ...) -> row-major frame.
// Slab k of `slabs` holds the tiles first + k, first + k + stride, ... (rank first + k of a stride-way
// split); nslabs of them are scattered into the row-major frame.
__global__ void unshuffle_kernel(const float* __restrict__ slabs, uint32_t first, uint32_t nslabs, uint32_t stride,
                                 uint32_t tiles_per_slab, uint32_t tiles_x, uint32_t W, uint32_t H, float* __restrict__ img) {
    uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t total = (uint64_t)nslabs * tiles_per_slab * 256u;
    if (gid >= total) return;
    uint32_t p = (uint32_t)(gid % 256u);
    uint64_t tl = gid / 256u;
    uint32_t slab = (uint32_t)(tl / tiles_per_slab);
    uint32_t i = (uint32_t)(tl % tiles_per_slab);
    uint64_t tile = (uint64_t)(first + slab) + (uint64_t)i * stride;
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

hipError_t launch_render(const RenderArgs& A, hipStream_t stream, int volume_type, int integrator) {
    dim3 grid(A.num_tiles);
    if (integrator == VR_TEST_HITMASK) {
        hipLaunchKernelGGL((dev::hitmask_kernel<256>), grid, dim3(256), 0, stream, A, volume_type == VR_VOLUME_SPHERES ? 1 : 0);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(dev::rm_spheres_kernel, grid, dim3(256), 0, stream, A);
    return hipGetLastError();
}

hipError_t launch_unshuffle_part(const float* slabs, uint32_t first, uint32_t nslabs, uint32_t stride, uint32_t tiles_per_slab,
                                 uint32_t tiles_x, uint32_t W, uint32_t H, float* img, hipStream_t stream) {
    uint64_t total = (uint64_t)nslabs * tiles_per_slab * 256u;
    if (total == 0) return hipSuccess;
    dim3 grid((unsigned)((total + 255) / 256));
    hipLaunchKernelGGL(dev::unshuffle_kernel, grid, dim3(256), 0, stream, slabs, first, nslabs, stride, tiles_per_slab, tiles_x,
                       W, H, img);
    return hipGetLastError();
}

hipError_t launch_unshuffle(const float* slabs, uint32_t nslabs, uint32_t tiles_per_slab, uint32_t tiles_x, uint32_t W,
                            uint32_t H, float* img, hipStream_t stream) {
    return launch_unshuffle_part(slabs, 0, nslabs, nslabs, tiles_per_slab, tiles_x, W, H, img, stream);
}

}  // namespace vr
