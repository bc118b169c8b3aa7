// Device-side building blocks of the ray-march kernels (gfx950, wave64).
//
// Floating point: the whole library is compiled with -ffp-contract=off and HIP's default
// correctly rounded f32 division and square root, and every geometric expression below keeps
// the reference's (Eigen 3.4) evaluation order. Ray origins/directions, ellipsoid entry/exit
// distances t0/t1 and the march positions are therefore bit-identical to the CPU restatement,
// which is what makes the discrete decisions (which Gaussian is active at which step, which
// secondary event is the first one past a light) agree exactly. exp/erf come from the device
// math library and differ from glibc by a few ulp; those only feed continuous quantities.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../vr_internal.h"

namespace vr {
namespace dev {

struct Ray {
    float ox, oy, oz, dx, dy, dz;
};

__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    return a0 * b0 + (a1 * b1 + a2 * b2);
}

// Eigen normalized(): v / sqrt(squaredNorm) when squaredNorm > 0.
__device__ __forceinline__ void normalize3(float& x, float& y, float& z) {
    float s = dot3(x, y, z, x, y, z);
    if (s > 0.0f) {
        float r = sqrtf(s);
        x = __fdiv_rn(x, r);
        y = __fdiv_rn(y, r);
        z = __fdiv_rn(z, r);
    }
}

__device__ __forceinline__ Ray make_ray(float ox, float oy, float oz, float dx, float dy, float dz) {
    normalize3(dx, dy, dz);  // ray.h:11-12
    return Ray{ox, oy, oz, dx, dy, dz};
}

// camera.h:45-53 (pinhole) / :64-73 (orthographic); u,v = (x + 0.5f) / W, (y + 0.5f) / H.
__device__ __forceinline__ Ray primary_ray(const RenderArgs& A, int x, int y) {
    float uvx = __fdiv_rn((float)x + 0.5f, (float)A.width);
    float uvy = __fdiv_rn((float)y + 0.5f, (float)A.height);
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
    normalize3(d0, d1, d2);  // sample_ray's .normalized()
    return make_ray(o0, o1, o2, d0, d1, d2);
}

// ---- Gaussian record access (3 x 16-B loads) ----
struct GRec {
    float mx, my, mz, density, m00, m01, m02, m11, m12, m22, norm, albedo;
};
__device__ __forceinline__ GRec load_rec(const GaussianRecord* __restrict__ g, int i) {
    const float4* p = reinterpret_cast<const float4*>(g + i);
    float4 a = p[0], b = p[1], c = p[2];
    return GRec{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
}

// Quadratic coefficients shared by intersect_direct and optical_depth (gaussian.h:126-136,
// 208-218): A = d.Md, B = 2 p.Md, Cq = p.Mp with p = o - mean.
struct Quad {
    float A, B, Cq;
};
__device__ __forceinline__ Quad quad(const GRec& g, const Ray& r) {
    float px = r.ox - g.mx, py = r.oy - g.my, pz = r.oz - g.mz;
    // inv_cov * d, rows (M00 M01 M02), (M10 M11 M12), (M20 M21 M22); M symmetric
    float mdx = g.m00 * r.dx + (g.m01 * r.dy + g.m02 * r.dz);
    float mdy = g.m01 * r.dx + (g.m11 * r.dy + g.m12 * r.dz);
    float mdz = g.m02 * r.dx + (g.m12 * r.dy + g.m22 * r.dz);
    float mpx = g.m00 * px + (g.m01 * py + g.m02 * pz);
    float mpy = g.m01 * px + (g.m11 * py + g.m12 * pz);
    float mpz = g.m02 * px + (g.m12 * py + g.m22 * pz);
    Quad q;
    q.A = dot3(r.dx, r.dy, r.dz, mdx, mdy, mdz);
    q.B = 2.0f * dot3(px, py, pz, mdx, mdy, mdz);
    q.Cq = dot3(px, py, pz, mpx, mpy, mpz);
    return q;
}

// Gaussian::intersect_direct (gaussian.h:126-164), R = 3.
__device__ __forceinline__ bool intersect(const Quad& q, float& t_enter, float& t_exit) {
    float C = q.Cq - 9.0f;
    float disc = q.B * q.B - 4.0f * q.A * C;
    if (disc < 0.0f) return false;
    float sqrtD = sqrtf(disc);
    float twoA = 2.0f * q.A;
    float t0 = __fdiv_rn(-q.B - sqrtD, twoA);
    float t1 = __fdiv_rn(-q.B + sqrtD, twoA);
    if (t0 > t1) {
        float tmp = t0;
        t0 = t1;
        t1 = tmp;
    }
    if (t1 < 0.0f) return false;
    t_enter = (t0 >= 0.0f) ? t0 : 0.0f;
    t_exit = t1;
    return true;
}

// Gaussian::optical_depth (gaussian.h:208-231) for the same ray. The reference evaluates
// sqrt(pi / (2A)) in double; f32 here (relative difference ~1 ulp).
__device__ __forceinline__ float optical_depth(const GRec& g, const Quad& q, float t0, float t1) {
    float twoA = 2.0f * q.A;
    float pref = (g.density * g.norm) * sqrtf(__fdiv_rn(3.14159265358979323846f, twoA));
    float den = 2.0f * sqrtf(twoA);
    float F1 = erff(__fdiv_rn(q.B + twoA * t1, den));
    float F0 = erff(__fdiv_rn(q.B + twoA * t0, den));
    float e = expf(-0.5f * (q.Cq - __fdiv_rn(q.B * q.B, 4.0f * q.A)));
    return pref * e * (F1 - F0);
}

// ---- secondary-ray variants ------------------------------------------------------------------
// Light / environment rays only feed transmittances (continuous) and decisions at the 3-sigma
// boundary whose optical-depth weight is ~0, so they may round differently from the reference:
// FMA-contracted products and hardware reciprocal / square root (1 ulp) instead of correctly
// rounded division and sqrt — about half the VALU instructions of the exact forms. The primary
// march keeps the exact forms (its activation decisions must match the oracle bit for bit).
// p^T M p with p = origin - mean, in exactly the arithmetic quad_fast uses for Cq (the record
// neighbour lists compare it bit for bit against the value a secondary ray computes).
__device__ __forceinline__ float cq_fast(const GRec& g, float px, float py, float pz) {
    const float mpx = fmaf(g.m00, px, fmaf(g.m01, py, g.m02 * pz));
    const float mpy = fmaf(g.m01, px, fmaf(g.m11, py, g.m12 * pz));
    const float mpz = fmaf(g.m02, px, fmaf(g.m12, py, g.m22 * pz));
    return fmaf(px, mpx, fmaf(py, mpy, pz * mpz));
}

__device__ __forceinline__ Quad quad_fast(const GRec& g, const Ray& r) {
    const float px = r.ox - g.mx, py = r.oy - g.my, pz = r.oz - g.mz;
    const float mdx = fmaf(g.m00, r.dx, fmaf(g.m01, r.dy, g.m02 * r.dz));
    const float mdy = fmaf(g.m01, r.dx, fmaf(g.m11, r.dy, g.m12 * r.dz));
    const float mdz = fmaf(g.m02, r.dx, fmaf(g.m12, r.dy, g.m22 * r.dz));
    Quad q;
    q.A = fmaf(r.dx, mdx, fmaf(r.dy, mdy, r.dz * mdz));
    q.B = 2.0f * fmaf(px, mdx, fmaf(py, mdy, pz * mdz));
    q.Cq = cq_fast(g, px, py, pz);
    return q;
}

__device__ __forceinline__ bool intersect_fast(const Quad& q, float& t_enter, float& t_exit) {
    const float disc = fmaf(q.B, q.B, -4.0f * q.A * (q.Cq - 9.0f));
    if (disc < 0.0f) return false;
    const float s = __builtin_amdgcn_sqrtf(disc);
    const float inv2A = __builtin_amdgcn_rcpf(2.0f * q.A);  // A = d.Md > 0 (M positive definite)
    const float u0 = (-q.B - s) * inv2A, u1 = (-q.B + s) * inv2A;
    const float t1 = fmaxf(u0, u1);  // (ordered already whenever A > 0)
    if (t1 < 0.0f) return false;
    t_enter = fmaxf(fminf(u0, u1), 0.0f);
    t_exit = t1;
    return true;
}

__device__ __forceinline__ float optical_depth_fast(const GRec& g, const Quad& q, float t0, float t1) {
    const float twoA = 2.0f * q.A;
    const float r2A = __builtin_amdgcn_rcpf(twoA);
    const float pref = (g.density * g.norm) * __builtin_amdgcn_sqrtf(3.14159265358979323846f * r2A);
    const float inv_den = 0.5f * __builtin_amdgcn_rsqf(twoA);  // 1 / (2 sqrt(2A))
    const float F1 = erff(fmaf(twoA, t1, q.B) * inv_den);
    const float F0 = erff(fmaf(twoA, t0, q.B) * inv_den);
    const float e = __expf(-0.5f * fmaf(-q.B * q.B, 0.5f * r2A, q.Cq));  // C - B^2 / (4A)
    return pref * e * (F1 - F0);
}

// erf on a 3-sigma chord. Every optical depth a secondary ray adds over an interval inside the
// Gaussian's 3-sigma ellipsoid has erf arguments x = (B + 2A t) / (2 sqrt(2A)) with |x| <= sqrt(9/2)
// = 2.121 (t0 and t1 are the chord's ends; x^2 = (9 - (Cq - B^2/4A)) / 2 there), so one
// branch-free polynomial covers it: erf(x) = x P(2x^2/6.25 - 1), P of degree 10 fitted in the
// Chebyshev variable on |x| <= 2.5 (least squares weighted by x), |error| <= 2e-7 including the f32
// evaluation (ocml's erff: ~1e-7, but two branches on |x| < 1 that a wave runs both of). Arguments
// are clamped to the fitted range; intervals reaching past a chord (a ray's last event) keep erff.
__device__ __forceinline__ float erf_chord(float x) {
    x = __builtin_amdgcn_fmed3f(x, -2.5f, 2.5f);
    const float t = fmaf(x * x, 0.32f, -1.0f);
    float p = 8.204215555e-05f;
    p = fmaf(p, t, -3.410060599e-04f);
    p = fmaf(p, t, 9.705630946e-04f);
    p = fmaf(p, t, -2.884618938e-03f);
    p = fmaf(p, t, 8.081957698e-03f);
    p = fmaf(p, t, -2.004199103e-02f);
    p = fmaf(p, t, 4.414051399e-02f);
    p = fmaf(p, t, -8.646185696e-02f);
    p = fmaf(p, t, 1.521729976e-01f);
    p = fmaf(p, t, -2.545413673e-01f);
    p = fmaf(p, t, 5.586599708e-01f);
    return x * p;
}

// optical_depth_fast for an interval [t0, t1] inside the 3-sigma chord (erf_chord).
__device__ __forceinline__ float optical_depth_chord(const GRec& g, const Quad& q, float t0, float t1) {
    const float twoA = 2.0f * q.A;
    const float r2A = __builtin_amdgcn_rcpf(twoA);
    const float pref = (g.density * g.norm) * __builtin_amdgcn_sqrtf(3.14159265358979323846f * r2A);
    const float inv_den = 0.5f * __builtin_amdgcn_rsqf(twoA);  // 1 / (2 sqrt(2A))
    const float F1 = erf_chord(fmaf(twoA, t1, q.B) * inv_den);
    const float F0 = erf_chord(fmaf(twoA, t0, q.B) * inv_den);
    const float e = __expf(-0.5f * fmaf(-q.B * q.B, 0.5f * r2A, q.Cq));  // C - B^2 / (4A)
    return pref * e * fmaxf(F1 - F0, 0.0f);  // (f32 noise can invert a tiny interval)
}

// ---- whitened secondary-ray forms (WRecord) ---------------------------------------------------
// In the coordinates u = L (x - mean) (M = L^T L) a Gaussian's 3-sigma ellipsoid is the sphere |u| = 3
// and a ray o + t d is u = Lp + t Ld. With a = |Ld|^2, h = Lp.Ld, c = |Lp|^2, r = a^-1/2, hr = h r:
//   intersect_direct (gaussian.h:126-164): D = hr^2 - (c - 9) = 9 - e2 >= 0, t = r (-hr -+ sqrt(D))
//   optical_depth (gaussian.h:208-231): dn r exp((hr^2 - c) / 2) (erf(x1) - erf(x0)) = dn r exp(-e2 / 2) (..),
//     x(t) = (hr + t / r) / sqrt(2); at the exit t1, x1 = sqrt(D / 2); at the entry t0, x0 = -x1
// (the same quantities as quad_fast / intersect_fast / optical_depth_fast in about half the VALU
// operations and three transcendentals — rsq, sqrt, exp — instead of six).
struct WRec {
    float mx, my, mz, dn, l00, l01, l02, l11, l12, l22;
};
__device__ __forceinline__ WRec load_wrec(const WRecord* __restrict__ g, int i) {
    const float4* p = reinterpret_cast<const float4*>(g + i);
    const float4 a = p[0], b = p[1];
    const float2 c = *reinterpret_cast<const float2*>(p + 2);
    return WRec{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y};
}
struct WQuad {
    float c;   // |Lp|^2 = p.M.p (origin - mean): depends on the ray origin only
    float r;   // |Ld|^-1
    float hr;  // Lp.Ld / |Ld|
    float sa;  // |Ld|
    float e2;  // |Lp - (h / a) Ld|^2: the chord's squared distance from the centre (c - hr^2, without the
               // cancellation: its error grows with the origin's whitened distance, not with its square)
};
__device__ __forceinline__ WQuad wquad(const WRec& g, const Ray& ray) {
    const float px = ray.ox - g.mx, py = ray.oy - g.my, pz = ray.oz - g.mz;
    const float p0 = fmaf(g.l00, px, fmaf(g.l01, py, g.l02 * pz)), p1 = fmaf(g.l11, py, g.l12 * pz), p2 = g.l22 * pz;
    const float d0 = fmaf(g.l00, ray.dx, fmaf(g.l01, ray.dy, g.l02 * ray.dz));
    const float d1 = fmaf(g.l11, ray.dy, g.l12 * ray.dz), d2 = g.l22 * ray.dz;
    const float a = fmaf(d0, d0, fmaf(d1, d1, d2 * d2));
    const float h = fmaf(p0, d0, fmaf(p1, d1, p2 * d2));
    WQuad q;
    q.c = fmaf(p0, p0, fmaf(p1, p1, p2 * p2));
    q.r = __builtin_amdgcn_rsqf(a);
    q.hr = h * q.r;
    q.sa = a * q.r;
    const float k = -q.hr * q.r;  // -h / a
    const float e0 = fmaf(k, d0, p0), e1 = fmaf(k, d1, p1), e2 = fmaf(k, d2, p2);
    q.e2 = fmaf(e0, e0, fmaf(e1, e1, e2 * e2));
    return q;
}
// Entry / exit of the 3-sigma sphere (t0 <= t1, not clamped); s = sqrt(D). False: no crossing, or it
// lies behind the origin (t1 < 0), as intersect_fast.
__device__ __forceinline__ bool wintersect(const WQuad& q, float& t0, float& t1, float& s) {
    const float D = 9.0f - q.e2;
    if (!(D >= 0.0f)) return false;  // (NaN: a degenerate covariance never intersects)
    s = __builtin_amdgcn_sqrtf(D);
    t1 = q.r * (s - q.hr);
    if (t1 < 0.0f) return false;
    t0 = q.r * (-q.hr - s);
    return true;
}
// Optical depth between erf arguments x0 <= x1 (times sqrt 2) on the 3-sigma chord: erf_chord.
__device__ __forceinline__ float wod_chord(const WRec& g, const WQuad& q, float u0, float u1) {
    constexpr float kRs2 = 0.70710678118654752f;
    const float F1 = erf_chord(u1 * kRs2), F0 = erf_chord(u0 * kRs2);
    const float e = __expf(-0.5f * q.e2);
    return (g.dn * q.r) * e * fmaxf(F1 - F0, 0.0f);  // (f32 noise can invert a tiny interval)
}
// Optical depth over [t0, t1] anywhere on the ray (device erff: arguments past the chord).
__device__ __forceinline__ float wod_range(const WRec& g, const WQuad& q, float t0, float t1) {
    constexpr float kRs2 = 0.70710678118654752f;
    const float F1 = erff(fmaf(q.sa, t1, q.hr) * kRs2), F0 = erff(fmaf(q.sa, t0, q.hr) * kRs2);
    const float e = __expf(-0.5f * q.e2);
    return (g.dn * q.r) * e * (F1 - F0);
}

// Gaussian::mu_t = density * evaluate(x) (gaussian.h:111-117), exponent -0.5 d^T M d with
// Eigen's lazy-product order.
// ex_out: the exponent -0.5 d^T M d (the march's record flag reads p.M.p = -2 ex off it).
__device__ __forceinline__ float mu_t(const GRec& g, float x, float y, float z, float* ex_out = nullptr) {
    float d0 = x - g.mx, d1 = y - g.my, d2 = z - g.mz;
    float l0 = -0.5f * d0, l1 = -0.5f * d1, l2 = -0.5f * d2;
    float w0 = l0 * g.m00 + (l1 * g.m01 + l2 * g.m02);
    float w1 = l0 * g.m01 + (l1 * g.m11 + l2 * g.m12);
    float w2 = l0 * g.m02 + (l1 * g.m12 + l2 * g.m22);
    float ex = w0 * d0 + (w1 * d1 + w2 * d2);
    if (ex_out) *ex_out = ex;
    return g.density * (g.norm * expf(ex));
}

// ---- rng.h:13-57 ----
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
struct PCG32 {
    uint64_t state, inc;
    __device__ __forceinline__ PCG32(uint64_t seed_state, uint64_t seed_seq) {
        state = 0;
        inc = (seed_seq << 1) | 1;
        next_u32();
        state += seed_state;
        next_u32();
    }
    struct FromState {};
    // a generator already seeded: `s` is the state a seeding constructor left (stream seed_seq)
    __device__ __forceinline__ PCG32(FromState, uint64_t s, uint64_t seed_seq) : state(s), inc((seed_seq << 1) | 1) {}
    __device__ __forceinline__ uint32_t next_u32() {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t shifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (shifted >> rot) | (shifted << ((-rot + 1u) & 31));
    }
    __device__ __forceinline__ float uniform() { return (float)(next_u32() >> 8) * (1.0f / 16777216.0f); }
    // Textbook PCG32 output ((-rot) & 31) of the same state sequence: the deterministic stand-in
    // for the reference's unbiased mt19937 environment sampler (integrator.h:13-28). rng.h:43's
    // (-rot + 1) & 31 ORs overlapping halves whenever rot <= 1, biasing uniform() upwards; the
    // free-flight integrators keep it (that is the reference's own PCG32), the env sampler does not.
    __device__ __forceinline__ float uniform_env() {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t shifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (float)(((shifted >> rot) | (shifted << ((0u - rot) & 31))) >> 8) * (1.0f / 16777216.0f);
    }
};
__device__ __forceinline__ uint64_t derive_path_seed(int x, int y, int si) {
    uint64_t seed = ((uint64_t)(uint32_t)si << 32) | ((uint64_t)(uint32_t)y << 16) | (uint64_t)(uint32_t)x;
    return splitmix64(seed);
}

// Deterministic environment direction (replaces the non-reproducible
// sample_uniform_direction_old, integrator.h:13-28; same distribution). Identical float
// operations to oracle/vr_oracle.cpp env_dir.
__device__ __forceinline__ void env_dir(float xi1, float xi2, float& x, float& y, float& z) {
    z = 1.0f - 2.0f * xi2;
    float s2 = (1.0f - z) * (1.0f + z);
    float s = sqrtf(s2 > 0.0f ? s2 : 0.0f);
    float t = xi1 * 4.0f;
    float q = floorf(t + 0.5f);
    float f = t - q;
    float a = f * 1.57079632679489662f;
    float a2 = a * a;
    float sp = a * (1.0f + a2 * (-1.66666672e-1f + a2 * (8.33333377e-3f + a2 * (-1.98412701e-4f + a2 * 2.75573188e-6f))));
    float cp = 1.0f + a2 * (-0.5f + a2 * (4.16666679e-2f + a2 * (-1.38888892e-3f + a2 * (2.48015876e-5f + a2 * -2.75573188e-7f))));
    int qi = ((int)q) & 3;
    float ct, st;
    if (qi == 0) { ct = cp; st = sp; }
    else if (qi == 1) { ct = -sp; st = cp; }
    else if (qi == 2) { ct = -cp; st = -sp; }
    else { ct = sp; st = -cp; }
    x = s * ct;
    y = s * st;
}

// Slab test against a child box; returns [tmin, tmax] (NaN-robust: fminf/fmaxf drop NaNs).
__device__ __forceinline__ void slab(const float* b, const Ray& r, float ix, float iy, float iz, float& tmin, float& tmax) {
    float tx1 = (b[0] - r.ox) * ix, tx2 = (b[3] - r.ox) * ix;
    float ty1 = (b[1] - r.oy) * iy, ty2 = (b[4] - r.oy) * iy;
    float tz1 = (b[2] - r.oz) * iz, tz2 = (b[5] - r.oz) * iz;
    tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
}

// Generic stack traversal of the child-pair BVH. `prune(tmin, tmax)` says whether a child box
// whose ray interval is [tmin, tmax] (already known to satisfy tmax >= max(tmin, 0)) must be
// visited; `leaf(first, count)` handles a leaf's primitive range and returns false to stop the
// whole traversal. The stack lives in LDS with a
// per-thread stride (bank-conflict-free: lane i uses word i of every row).
struct NoCount {
    __device__ __forceinline__ void operator()() const {}
};

// Child-pair node `node` as 12 box floats (left min xyz, left max xyz, right min xyz, right max
// xyz) + the two child refs. H: the 32-B half node (HNode, scene-normalised coordinates).
template <bool H>
__device__ __forceinline__ void load_pair(const RenderArgs& A, int node, float* f, int2& nc) {
    if constexpr (H) {
        const uint4* np = reinterpret_cast<const uint4*>(A.hnodes + node);
        const uint4 a = np[0], b = np[1];
        const uint32_t w[6] = {a.x, a.y, a.z, a.w, b.x, b.y};
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            f[2 * i] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[i] & 0xffffu));
            f[2 * i + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[i] >> 16));
        }
        nc = make_int2((int)b.z, (int)b.w);
    } else {
        const float4* np = reinterpret_cast<const float4*>(A.nodes + node);
        const float4 n0 = np[0], n1 = np[1], n2 = np[2];
        const int4 c4 = reinterpret_cast<const int4*>(A.nodes + node)[3];
        f[0] = n0.x, f[1] = n0.y, f[2] = n0.z, f[3] = n0.w, f[4] = n1.x, f[5] = n1.y;
        f[6] = n1.z, f[7] = n1.w, f[8] = n2.x, f[9] = n2.y, f[10] = n2.z, f[11] = n2.w;
        nc = make_int2(c4.x, c4.y);
    }
}

// A point in the coordinates of the H = true / false node boxes.
template <bool H>
__device__ __forceinline__ void node_space(const RenderArgs& A, float& x, float& y, float& z) {
    if constexpr (H) {
        x = (x - A.hn_center[0]) * A.hn_scale;
        y = (y - A.hn_center[1]) * A.hn_scale;
        z = (z - A.hn_center[2]) * A.hn_scale;
    }
}

template <bool H, typename Prune, typename Leaf, typename OnNode = NoCount>
__device__ __forceinline__ void traverse(const RenderArgs& A, const Ray& r0, int* stack, int stride, Prune prune, Leaf leaf,
                                         OnNode on_node = OnNode()) {
    // H: the ray in the half nodes' normalised coordinates (same parameter t along it)
    Ray r = r0;
    if constexpr (H) {
        node_space<true>(A, r.ox, r.oy, r.oz);
        r.dx *= A.hn_scale;
        r.dy *= A.hn_scale;
        r.dz *= A.hn_scale;
    }
    const float ix = __frcp_rn(r.dx), iy = __frcp_rn(r.dy), iz = __frcp_rn(r.dz);
    int sp = 0;
    int node = 0;
    for (;;) {
        float f[12];
        int2 nc;
        load_pair<H>(A, node, f, nc);
        on_node();
        float lmin, lmax, rmin, rmax;
        slab(f, r, ix, iy, iz, lmin, lmax);
        slab(f + 6, r, ix, iy, iz, rmin, rmax);
        bool hl = nc.x != 0 && lmax >= fmaxf(lmin, 0.0f) && prune(lmin, lmax);
        bool hr = nc.y != 0 && rmax >= fmaxf(rmin, 0.0f) && prune(rmin, rmax);
        // leaf children are handled at once, nearer first; a leaf callback returning false ends
        // the traversal (used by the optical-depth cut-off of the secondary rays)
        const bool ll = hl && ref_is_leaf(nc.x), lr = hr && ref_is_leaf(nc.y);
        if (ll || lr) {
            const bool r_first = lr && (!ll || rmin < lmin);
            const int32_t first_ref = r_first ? nc.y : nc.x;
            if (!leaf(leaf_first(first_ref), leaf_count(first_ref))) return;
            if (ll && lr) {
                const int32_t second_ref = r_first ? nc.x : nc.y;
                if (!leaf(leaf_first(second_ref), leaf_count(second_ref))) return;
            }
            if (ll) hl = false;
            if (lr) hr = false;
        }
        if (hl && hr) {
            int nearer = nc.x, farther = nc.y;
            if (rmin < lmin) {
                nearer = nc.y;
                farther = nc.x;
            }
            stack[sp * stride] = farther;
            ++sp;
            node = nearer;
        } else if (hl) {
            node = nc.x;
        } else if (hr) {
            node = nc.y;
        } else {
            if (sp == 0) break;
            --sp;
            node = stack[sp * stride];
        }
    }
}

// Compare-exchange of (key, ref) pairs: afterwards ka <= kb.
__device__ __forceinline__ void cswap(float& ka, int32_t& ra, float& kb, int32_t& rb) {
    const bool sw = kb < ka;
    const float k = sw ? kb : ka;
    kb = sw ? ka : kb;
    ka = k;
    const int32_t r = sw ? rb : ra;
    rb = sw ? ra : rb;
    ra = r;
}

// Slab tests of the four children of 4-wide half node `node` (HNode4) for a ray already in the
// nodes' normalised coordinates, sorted near to far; misses (and empty slots) get key +inf, ref 0.
// The node comes from the per-axis copy (A.hnodes4w, soa_nodes_kernel: per axis the f16 word pairs {min of children
// 0, 1}, {min 2, 3}, {max 0, 1}, {max 2, 3}; then the refs): the ray takes its near and far word pair of each axis
// once for the four children by the sign of 1/d — for 1/d > 0 the fma is monotone in the bound, so the near
// bound's slab distance is the min of the two — the same tmin / tmax bit for bit as a min and a max per child.
template <typename Hit, bool SORT = true>
__device__ __forceinline__ void wide_children(const RenderArgs& A, int node, float ix, float iy, float iz, float oxi,
                                              float oyi, float ozi, Hit hit, float* key, int32_t* kr) {
    const uint4* np = reinterpret_cast<const uint4*>(A.hnodes4w + node);
    const uint4 q0 = np[0], q1 = np[1], q2 = np[2], rf = np[3];
    const uint32_t w[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
    const int32_t ref[4] = {(int32_t)rf.x, (int32_t)rf.y, (int32_t)rf.z, (int32_t)rf.w};
    float smin[4], smax[4];
    {
        const float inv[3] = {ix, iy, iz}, oi[3] = {oxi, oyi, ozi};
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
            const bool neg = inv[ax] < 0.0f;
            const uint32_t n01 = neg ? w[4 * ax + 2] : w[4 * ax], n23 = neg ? w[4 * ax + 3] : w[4 * ax + 1];
            const uint32_t f01 = neg ? w[4 * ax] : w[4 * ax + 2], f23 = neg ? w[4 * ax + 1] : w[4 * ax + 3];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t nwd = i < 2 ? n01 : n23, fwd = i < 2 ? f01 : f23;
                const float nb = (float)__builtin_bit_cast(_Float16, (uint16_t)((i & 1) ? (nwd >> 16) : (nwd & 0xffffu)));
                const float fb = (float)__builtin_bit_cast(_Float16, (uint16_t)((i & 1) ? (fwd >> 16) : (fwd & 0xffffu)));
                const float tn = fmaf(nb, inv[ax], -oi[ax]), tf = fmaf(fb, inv[ax], -oi[ax]);
                smin[i] = ax == 0 ? tn : fmaxf(smin[i], tn);
                smax[i] = ax == 0 ? tf : fminf(smax[i], tf);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float tmin = smin[i], tmax = smax[i];
        const bool h = (ref[i] != 0) && (tmax >= fmaxf(tmin, 0.0f)) && hit(tmin, tmax);
        key[i] = h ? tmin : INFINITY;
        kr[i] = h ? ref[i] : 0;
    }
    if constexpr (SORT) {
        cswap(key[0], kr[0], key[1], kr[1]);  // 4-input sorting network
        cswap(key[2], kr[2], key[3], kr[3]);
        cswap(key[0], kr[0], key[2], kr[2]);
        cswap(key[1], kr[1], key[3], kr[3]);
        cswap(key[1], kr[1], key[2], kr[2]);
    }
}

// Stack traversal of the 4-wide half-precision tree (HNode4) with the generic traverse's
// contract (prune / leaf / on_node); leaves are handled near-first as a node's children are
// reached, the nearest inner child is walked next and the others pushed far-first. Returns false
// if the LDS stack (cap entries) could overflow — the caller then re-runs the work on the pair tree.
// SORT = false: children in the node's order (a query whose result does not depend on the visit order,
// e.g. a window query that collects every entry of an interval).
// DEEP > 0: entries past the CAP LDS entries go to DEEP more in the lane's private (scratch) memory before the walk
// gives up (the LDS stack then sizes the kernel's occupancy, not the deepest walk).
template <int CAP, typename Prune, typename Leaf, typename OnNode = NoCount, bool SORT = true, int DEEP = 0>
__device__ __forceinline__ bool traverse_wide(const RenderArgs& A, const Ray& r0, int* stack, int stride, Prune prune,
                                              Leaf leaf, OnNode on_node = OnNode()) {
    [[maybe_unused]] volatile int deep[DEEP > 0 ? DEEP : 1];
    float ox = r0.ox, oy = r0.oy, oz = r0.oz;
    node_space<true>(A, ox, oy, oz);
    // |d| clamped away from 0 (axis-parallel rays, e.g. an orthographic camera looking along an
    // axis): the fma slab form b/d - o/d must never see inf - inf
    auto inv = [&](float d) {
        d *= A.hn_scale;
        return __frcp_rn(fabsf(d) > 1e-30f ? d : copysignf(1e-30f, d));
    };
    const float ix = inv(r0.dx), iy = inv(r0.dy), iz = inv(r0.dz);
    const float oxi = ox * ix, oyi = oy * iy, ozi = oz * iz;
    int sp = 0;
    int node = 0;
    for (;;) {
        on_node();
        float key[4];
        int32_t kr[4];
        wide_children<Prune, SORT>(A, node, ix, iy, iz, oxi, oyi, ozi, prune, key, kr);
#pragma unroll
        for (int i = 0; i < 4; ++i)  // leaves, near first (SORT)
            if (kr[i] < 0 && !leaf(leaf_first(kr[i]), leaf_count(kr[i]))) return true;
        int first = -1;
        int32_t next = 0;  // the nearest inner child (selects only: no dynamic register indexing)
#pragma unroll
        for (int i = 3; i >= 0; --i) {
            first = kr[i] > 0 ? i : first;
            next = kr[i] > 0 ? kr[i] : next;
        }
        if (sp + 3 > CAP + DEEP) return false;
        // (DEEP: the LDS-only form while no lane of the wave can reach past CAP)
        if (DEEP == 0 || __builtin_expect(__ballot(sp > CAP - 3) == 0ull, 1)) {
#pragma unroll
            for (int i = 3; i >= 0; --i)
                if (kr[i] > 0 && i != first) stack[(sp++) * stride] = kr[i];
        } else {
#pragma unroll
            for (int i = 3; i >= 0; --i)
                if (kr[i] > 0 && i != first) {
                    if (sp < CAP) stack[sp * stride] = kr[i];
                    else deep[sp - CAP] = kr[i];
                    ++sp;
                }
        }
        if (first >= 0) {
            node = next;
        } else {
            if (sp == 0) return true;
            --sp;
            if (DEEP == 0 || __builtin_expect(__ballot(sp >= CAP) == 0ull, 1)) node = stack[sp * stride];
            else node = sp < CAP ? stack[sp * stride] : deep[sp - CAP];
        }
    }
}

// First index k with t_k >= a in the iterated step table (returns n if beyond the table).
__device__ __forceinline__ int kfirst(const float* __restrict__ ts, int n, float step, float a) {
    int k = (int)(a / step);
    if (k < 0) k = 0;
    if (k > n - 1) k = n - 1;
    while (k > 0 && ts[k - 1] >= a) --k;
    while (k < n && ts[k] < a) ++k;
    return k;
}

}  // namespace dev
}  // namespace vr

// NOTE on rounding: HIP's __fsqrt_rn maps to __ocml_native_sqrt_f32 (approximate) unless
// OCML_BASIC_ROUNDED_OPERATIONS is defined; plain sqrtf / '/' are correctly rounded under hipcc's
// default -fhip-fp32-correctly-rounded-divide-sqrt, which is what the bit-exactness relies on
// (host side: tests/test_host_abi.py::test_camera_and_primary_rays_bit_identical; device side: the
// L-inf parity tests of tests/test_gpu_parity.py, which a flipped activation decision would break).
