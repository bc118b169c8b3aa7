// =================================================================================================
//  vr_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
//  A line-faithful CPU restatement of wantonsushi/3DG-vol-renderer's forward ray-march path, used
//  ONLY as the checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. It is
//  never linked into, loaded by, or called from the product (libvr_hip.so / vr_amd). The product
//  path fails loudly when its HIP extension is missing; it never falls back to this file.
//
//  Parity status:
//    * The reference cannot be built here (Eigen 3.4.0 / gif-h are empty submodules, no network).
//      This file restates the algorithm from the reference sources, citing file:line, and
//      restates the Eigen 3.4.0 operations it relies on (evaluation order of 3-term reductions,
//      3x3 inverse/determinant) from Eigen's published algorithm. Bits at the Eigen boundary are
//      therefore "parity unpinned"; the restatement is pinned against the reference's own golden
//      renders (tests/golden/renders/*.ppm, produced by the reference) statistically and by the
//      exact miss-mask known-answer test (tests/test_oracle_golden.py).
//    * Documented deviation: the reference samples environment directions from a thread-local
//      std::mt19937 seeded by std::random_device (integrator.h:13-28) and is therefore not
//      reproducible. Here env directions come from the reference's own PCG32 (rng.h:20-57) keyed
//      by (pixel x, pixel y, march-step index) and a trig-free mapping of the same uniform-sphere
//      distribution (env_dir below). The GPU path implements the identical sampler so that GPU and
//      oracle agree per pixel.
//
//  Build: oracle/Makefile  (g++ -O3 -ffp-contract=off -fopenmp, shared library, C ABI for ctypes).
// =================================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <numbers>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>
#include <map>
#include <omp.h>

namespace orc {

// ---------------------------------------------------------------------------------------------
// Minimal fixed-size float vector/matrix with Eigen 3.4 evaluation order.
//   dot / squaredNorm / sum of 3 terms: Eigen redux_novec_unroller splits 3 as 1 + 2, i.e.
//   e0 + (e1 + e2). Matrix3f * Vector3f (lazy coeff product) rows use the same reduction.
//   normalized(): v / sqrt(squaredNorm()) when squaredNorm() > 0 (Eigen Dot.h).
// ---------------------------------------------------------------------------------------------
struct V3 {
    float x, y, z;
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
static inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
static inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
static inline float dot(V3 a, V3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
static inline float sqnorm(V3 a) { return dot(a, a); }
static inline float norm(V3 a) { return std::sqrt(sqnorm(a)); }
static inline V3 normalized(V3 a) {
    float z = sqnorm(a);
    if (z > 0.0f) return a / std::sqrt(z);
    return a;
}
static inline V3 cross(V3 l, V3 r) {  // Eigen OrthoMethods.h cross()
    return {l.y * r.z - l.z * r.y, l.z * r.x - l.x * r.z, l.x * r.y - l.y * r.x};
}
struct M3 {  // row-major
    float m[3][3];
    float operator()(int i, int j) const { return m[i][j]; }
};
static inline V3 mul(const M3& M, V3 v) {
    return {M.m[0][0] * v.x + (M.m[0][1] * v.y + M.m[0][2] * v.z),
            M.m[1][0] * v.x + (M.m[1][1] * v.y + M.m[1][2] * v.z),
            M.m[2][0] * v.x + (M.m[2][1] * v.y + M.m[2][2] * v.z)};
}
// Eigen InverseImpl.h cofactor_3x3<M,i,j>
static inline float cofactor(const M3& m, int i, int j) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m(i1, j1) * m(i2, j2) - m(i1, j2) * m(i2, j1);
}
// Eigen InverseImpl.h compute_inverse<..., 3>::run + compute_inverse_size3_helper
static inline M3 inverse3(const M3& m) {
    float c00 = cofactor(m, 0, 0), c10 = cofactor(m, 1, 0), c20 = cofactor(m, 2, 0);
    float det = c00 * m(0, 0) + (c10 * m(1, 0) + c20 * m(2, 0));
    float invdet = 1.0f / det;
    M3 r;
    float c01 = cofactor(m, 0, 1) * invdet;
    float c11 = cofactor(m, 1, 1) * invdet;
    float c02 = cofactor(m, 0, 2) * invdet;
    r.m[1][2] = cofactor(m, 2, 1) * invdet;
    r.m[2][1] = cofactor(m, 1, 2) * invdet;
    r.m[2][2] = cofactor(m, 2, 2) * invdet;
    r.m[1][0] = c01;
    r.m[1][1] = c11;
    r.m[2][0] = c02;
    r.m[0][0] = c00 * invdet;
    r.m[0][1] = c10 * invdet;
    r.m[0][2] = c20 * invdet;
    return r;
}
// Eigen Determinant.h determinant_impl<Derived,3> / bruteforce_det3_helper
static inline float det3_helper(const M3& m, int a, int b, int c) {
    return m(0, a) * (m(1, b) * m(2, c) - m(1, c) * m(2, b));
}
static inline float determinant3(const M3& m) {
    return det3_helper(m, 0, 1, 2) - det3_helper(m, 1, 0, 2) + det3_helper(m, 2, 0, 1);
}

// ---------------------------------------------------------------------------------------------
// Eigen 3.4.0 SelfAdjointEigenSolver<Matrix3f>(cov) (gaussian.h:57-59), restated from Eigen's
// published algorithm (third-party, absent here: extern/eigen-3.4.0 is an empty submodule) in f32,
// statement for statement: SelfAdjointEigenSolver::compute (the lower triangle scaled by its largest
// magnitude), tridiagonalization_inplace_selector<MatrixType, 3, false> (closed-form 3x3
// Householder), computeFromTridiagonal_impl (deflation test scaled by 1/epsilon, at most 30 * n
// implicit QR steps), tridiagonal_qr_step (Wilkinson shift through numext::hypot, Givens rotations
// from JacobiRotation::makeGivens, Q = Q * G through applyOnTheRight), then the selection sort of the
// eigenvalues (ascending, first minimum) with their vectors and the eigenvalues scaled back.
// Only get_aabb (gaussian.h:304-319) reads the result here: the reference's BVH boxes.
// ---------------------------------------------------------------------------------------------
static inline float eig_hypot(float x, float y) {  // Eigen MathFunctions.h positive_real_hypot(|x|, |y|)
    x = std::fabs(x);
    y = std::fabs(y);
    if (std::isinf(x) || std::isinf(y)) return INFINITY;
    if (std::isnan(x) || std::isnan(y)) return NAN;
    const float p = std::max(x, y);
    if (p == 0.0f) return 0.0f;
    const float qp = std::min(y, x) / p;
    return p * std::sqrt(1.0f + qp * qp);
}
static inline void eig_givens(float p, float q, float& c, float& s) {  // Jacobi.h makeGivens (real)
    if (q == 0.0f) {
        c = p < 0.0f ? -1.0f : 1.0f;
        s = 0.0f;
    } else if (p == 0.0f) {
        c = 0.0f;
        s = q < 0.0f ? 1.0f : -1.0f;
    } else if (std::fabs(p) > std::fabs(q)) {
        const float t = q / p;
        float u = std::sqrt(1.0f + t * t);
        if (p < 0.0f) u = -u;
        c = 1.0f / u;
        s = -t * c;
    } else {
        const float t = p / q;
        float u = std::sqrt(1.0f + t * t);
        if (q < 0.0f) u = -u;
        s = -1.0f / u;
        c = -t * s;
    }
}
// eigvals ascending; eigvecs column j (Q[.][j]) belongs to eigvals[j]
static void eigen_selfadjoint3(const M3& A, float eigvals[3], float Q[3][3]) {
    // compute(): mat = lower triangle of A, scaled
    float L[3][3] = {{A(0, 0), 0.0f, 0.0f}, {A(1, 0), A(1, 1), 0.0f}, {A(2, 0), A(2, 1), A(2, 2)}};
    float scale = 0.0f;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) scale = std::max(scale, std::fabs(L[i][j]));
    if (scale == 0.0f) scale = 1.0f;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j <= i; ++j) L[i][j] /= scale;
    // tridiagonalization_inplace_selector<MatrixType, 3, false>::run(..., extractQ = true)
    float diag[3], sub[2];
    const float tol = std::numeric_limits<float>::min();
    diag[0] = L[0][0];
    const float v1norm2 = L[2][0] * L[2][0];
    if (v1norm2 <= tol) {
        diag[1] = L[1][1];
        diag[2] = L[2][2];
        sub[0] = L[1][0];
        sub[1] = L[2][1];
        const float I[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
        std::memcpy(Q, I, sizeof(I));
    } else {
        const float beta = std::sqrt(L[1][0] * L[1][0] + v1norm2);
        const float invBeta = 1.0f / beta;
        const float m01 = L[1][0] * invBeta;
        const float m02 = L[2][0] * invBeta;
        const float q = 2.0f * m01 * L[2][1] + m02 * (L[2][2] - L[1][1]);
        diag[1] = L[1][1] + m02 * q;
        diag[2] = L[2][2] - m02 * q;
        sub[0] = beta;
        sub[1] = L[2][1] - m01 * q;
        const float M[3][3] = {{1, 0, 0}, {0, m01, m02}, {0, m02, -m01}};
        std::memcpy(Q, M, sizeof(M));
    }
    // computeFromTridiagonal_impl (maxIterations = 30)
    const int n = 3;
    int end = n - 1, start = 0, iter = 0;
    const float considerAsZero = std::numeric_limits<float>::min();
    const float precision_inv = 1.0f / std::numeric_limits<float>::epsilon();
    bool ok = true;
    while (end > 0) {
        for (int i = start; i < end; ++i) {
            if (std::fabs(sub[i]) < considerAsZero) {
                sub[i] = 0.0f;
            } else {
                const float scaled = precision_inv * sub[i];
                if (scaled * scaled <= (std::fabs(diag[i]) + std::fabs(diag[i + 1]))) sub[i] = 0.0f;
            }
        }
        while (end > 0 && sub[end - 1] == 0.0f) end--;
        if (end <= 0) break;
        iter++;
        if (iter > 30 * n) {
            ok = false;
            break;
        }
        start = end - 1;
        while (start > 0 && sub[start - 1] != 0.0f) start--;
        // tridiagonal_qr_step: Wilkinson shift
        const float td = (diag[end - 1] - diag[end]) * 0.5f;
        const float e = sub[end - 1];
        float mu = diag[end];
        if (td == 0.0f) {
            mu -= std::fabs(e);
        } else if (e != 0.0f) {
            const float e2 = e * e;
            const float h = eig_hypot(td, e);
            if (e2 == 0.0f) mu -= e / ((td + (td > 0.0f ? h : -h)) / e);
            else mu -= e2 / (td + (td > 0.0f ? h : -h));
        }
        float x = diag[start] - mu;
        float z = sub[start];
        for (int k = start; k < end && z != 0.0f; ++k) {
            float c, s;
            eig_givens(x, z, c, s);
            const float sdk = s * diag[k] + c * sub[k];
            const float dkp1 = s * sub[k] + c * diag[k + 1];
            diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1]);
            diag[k + 1] = s * sdk + c * dkp1;
            sub[k] = c * sdk - s * dkp1;
            if (k > start) sub[k - 1] = c * sub[k - 1] - s * z;
            x = sub[k];
            if (k < end - 1) {
                z = -s * sub[k + 1];
                sub[k + 1] = c * sub[k + 1];
            }
            // Q.applyOnTheRight(k, k + 1, G): apply_rotation_in_the_plane(col k, col k+1, G^T), G^T = (c, -s)
            if (!(c == 1.0f && s == 0.0f)) {
                for (int i = 0; i < 3; ++i) {
                    const float xi = Q[i][k], yi = Q[i][k + 1];
                    Q[i][k] = c * xi + (-s) * yi;
                    Q[i][k + 1] = -(-s) * xi + c * yi;
                }
            }
        }
    }
    if (ok) {  // sort ascending (minCoeff keeps the first minimum), vectors with their values
        for (int i = 0; i < n - 1; ++i) {
            int k = 0;
            float best = diag[i];
            for (int j = 1; j < n - i; ++j)
                if (diag[i + j] < best) {
                    best = diag[i + j];
                    k = j;
                }
            if (k > 0) {
                std::swap(diag[i], diag[k + i]);
                for (int r = 0; r < 3; ++r) std::swap(Q[r][i], Q[r][k + i]);
            }
        }
    }
    for (int i = 0; i < 3; ++i) eigvals[i] = diag[i] * scale;
}

// ---------------------------------------------------------------------------------------------
// rng.h:13-57 — splitmix64, non-standard PCG32 (rotation (-rot+1u)&31 at rng.h:43), path seed.
// ---------------------------------------------------------------------------------------------
static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
// rng.h:43 rotates with (-rot + 1u) & 31, not PCG's (-rot) & 31: whenever rot is 0 or 1 the two
// shifted halves overlap and are OR-ed, so outputs are biased upwards (mean of uniform() ~0.503,
// E[-log(1 - u)] ~1.08 instead of 1). The oracle keeps that (it is the reference's behaviour);
// g_pcg_textbook = true (test switch, orc_set_pcg_textbook) selects textbook PCG32 instead, which is
// how the free-flight goldens in tests/renders were evidently rendered (tests/test_oracle_freeflight.py).
static bool g_pcg_textbook = false;
// Event-sort tie order. The reference sorts a ray's events with std::sort on t alone (gmm.h:508-511),
// which is not stable: when a ray grazes a 3-sigma ellipsoid so closely that both roots round to the
// same float (t0 == t1), libstdc++'s introsort may put that Gaussian's exit before its entry, and the
// event loop then leaves it active for the rest of the ray. Which way it falls depends on the whole
// event array (BVH traversal order, partition pivots), not on the scene geometry. g_stable_ties = true
// (test switch, orc_set_stable_ties) resolves ties in emission order (entry before exit: the Gaussian
// is never active), which is the device path's rule; the default is the reference's std::sort.
static bool g_stable_ties = false;
// Secondary-ray chords in double (test switch, orc_set_accurate_chords; sparse-list restatement only). The
// reference's f32 quadratic loses a chord that grazes a Gaussian seen from far away: from an origin at
// whitened distance sqrt(c) the discriminant carries an absolute error ~c * 1e-7, so with c ~ 2700 a chord
// of 9 - e2 = 3e-4 collapses to a point (C4 pixel (598, 3212): [0.32260, 0.32282] becomes
// [0.3227114, 0.3227114], 0.078 of optical depth lost). The device computes the chord in whitened
// coordinates (error linear in sqrt(c)); with this switch the restatement does so too, in double, so a
// pixel that differs from the reference only through such a chord can be told apart (tests/helpers.py).
static bool g_accurate_chords = false;
// BVH boxes (test switch, orc_set_padded_boxes; read when a scene is built). The default is the reference's own
// boxes, get_aabb (gaussian.h:304-319) from the eigen-decomposition, so the midpoint BVH (gmm.h:231-446), its
// near-first traversal order (gmm.h:457-506) and with them std::sort's tie outcome (gmm.h:510-514) are the
// reference's, up to the bits of Eigen's f32 eigensolver (restated below from Eigen 3.4.0's algorithm: parity
// unpinned at that boundary). A box only culls: it also decides which fringe hits the f32 quadratic accepts
// outside the ellipsoid the reference keeps. g_padded_boxes = true builds the tree on the padded tight 3-sigma
// boxes instead (every such hit kept, the event set tree-independent), the oracle's rule before round 6.
static bool g_padded_boxes = false;
struct PCG32 {
    uint64_t state, inc;
    PCG32(uint64_t seed_state, uint64_t seed_seq) {
        state = 0;
        inc = (seed_seq << 1) | 1;
        next_u32();
        state += seed_state;
        next_u32();
    }
    uint32_t next_u32() {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t shifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (shifted >> rot) | (shifted << ((-rot + (g_pcg_textbook ? 0u : 1u)) & 31));
    }
    float uniform() { return (next_u32() >> 8) * (1.0f / 16777216.0f); }
    // Textbook PCG32 output of the same state sequence: the deterministic stand-in for the
    // reference's mt19937 environment sampler (integrator.h:13-28), which draws unbiased uniforms.
    float uniform_env() {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t shifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (((shifted >> rot) | (shifted << ((-rot) & 31))) >> 8) * (1.0f / 16777216.0f);
    }
};
static inline uint64_t derive_path_seed(int x, int y, int sample_index) {
    uint64_t seed = (uint64_t(sample_index) << 32) | (uint64_t(y) << 16) | (uint64_t(x));
    return splitmix64(seed);
}

// Deterministic replacement for sample_uniform_direction_old (integrator.h:13-28): same
// distribution (theta = 2 pi xi1, cos(phi) = 1 - 2 xi2), evaluated trig-free for phi and with a
// fixed polynomial for theta so that the GPU implementation is bit-identical.
static inline void sincos_2pi(float u, float* c, float* s) {
    float t = u * 4.0f;
    float q = std::floor(t + 0.5f);
    float f = t - q;                          // [-0.5, 0.5]
    float a = f * 1.57079632679489662f;       // [-pi/4, pi/4]
    float a2 = a * a;
    float sp = a * (1.0f + a2 * (-1.66666672e-1f + a2 * (8.33333377e-3f + a2 * (-1.98412701e-4f + a2 * 2.75573188e-6f))));
    float cp = 1.0f + a2 * (-0.5f + a2 * (4.16666679e-2f + a2 * (-1.38888892e-3f + a2 * (2.48015876e-5f + a2 * -2.75573188e-7f))));
    int qi = ((int)q) & 3;
    if (qi == 0) { *c = cp; *s = sp; }
    else if (qi == 1) { *c = -sp; *s = cp; }
    else if (qi == 2) { *c = -cp; *s = -sp; }
    else { *c = sp; *s = -cp; }
}
static inline V3 env_dir(float xi1, float xi2) {
    float z = 1.0f - 2.0f * xi2;
    float s2 = (1.0f - z) * (1.0f + z);
    float s = std::sqrt(s2 > 0.0f ? s2 : 0.0f);
    float ct, st;
    sincos_2pi(xi1, &ct, &st);
    return {s * ct, s * st, z};
}

// ---------------------------------------------------------------------------------------------
// ray.h:7-16 — direction normalised in the constructor.
// ---------------------------------------------------------------------------------------------
struct Ray {
    V3 origin, direction;
    Ray() {}
    Ray(V3 o, V3 d) : origin(o), direction(normalized(d)) {}
};

// ---------------------------------------------------------------------------------------------
// camera.h:7-74. NB the base ctor body uses the *parameter* view_dir (unnormalised) for right/up
// (camera.h:20-21); Pinhole uses the parameter for the pinhole point (camera.h:42).
// ---------------------------------------------------------------------------------------------
struct Camera {
    int type = 0;  // 0 pinhole, 1 orthographic
    V3 position, view_dir, right, up, pinhole;
    float focal_length = 0.0f;
    void base(V3 pos, V3 vd) {
        position = pos;
        view_dir = normalized(vd);
        const V3 world_up{0.0f, 1.0f, 0.0f};
        right = normalized(cross(vd, world_up));
        up = normalized(cross(right, vd));
    }
    static Camera make_pinhole(V3 pos, V3 vd, float fov) {
        Camera c;
        c.base(pos, vd);
        c.type = 0;
        c.focal_length = 1.0f / std::tan(0.5f * fov);
        c.pinhole = pos + c.focal_length * vd;
        return c;
    }
    static Camera make_ortho(V3 pos, V3 fwd) {
        Camera c;
        c.base(pos, fwd);
        c.type = 1;
        return c;
    }
    Ray sample_ray(double uvx, double uvy) const {
        if (type == 0) {  // camera.h:45-53
            float u = 1.0f - static_cast<float>(uvx) * 2.0f;
            float v = static_cast<float>(uvy) * 2.0f - 1.0f;
            V3 o = position + u * right + v * up;
            V3 d = pinhole - o;
            return Ray(o, normalized(d));
        } else {  // camera.h:64-73
            float u = static_cast<float>(uvx) * 2.0f - 1.0f;
            float v = 1.0f - static_cast<float>(uvy) * 2.0f;
            V3 o = position + u * right + v * up;
            V3 d = view_dir;
            return Ray(o, normalized(d));
        }
    }
};

// ---------------------------------------------------------------------------------------------
// gaussian.h:28-321 — only the members used by the forward integrators.
// ---------------------------------------------------------------------------------------------
static constexpr float R = 3.0f;  // gaussian.h:36
struct Gaussian {
    V3 mean;
    M3 cov;
    float density, albedo;
    M3 inv_cov;
    float norm;
    V3 bmin, bmax;    // BVH box: the reference's get_aabb (gaussian.h:304-319), or the padded box (g_padded_boxes)
    V3 tbmin, tbmax;  // padded tight 3-sigma box (B_frame binning, orc_tile_bins)

    Gaussian(V3 mean_, const M3& cov_, float density_, float albedo_)
        : mean(mean_), cov(cov_), density(density_), albedo(albedo_) {
        // gaussian.h:52-55
        inv_cov = inverse3(cov);
        float det_cov = determinant3(cov);
        norm = std::pow(2.0f * std::numbers::pi, -1.5f) * std::pow(det_cov, -0.5f);
        // Tight 3-sigma box of the ellipsoid, +-R*sqrt(Sigma_kk), padded by 5 % (it holds every point the f32
        // M-form quadratic accepts from a camera several units away).
        for (int k = 0; k < 3; ++k) {
            float h = R * std::sqrt(std::max(cov(k, k), 0.0f));
            h = h * 1.05f + 1e-6f;
            tbmin[k] = mean[k] - h;
            tbmax[k] = mean[k] + h;
        }
        if (g_padded_boxes) {
            bmin = tbmin;
            bmax = tbmax;
            return;
        }
        // gaussian.h:57-59 (SelfAdjointEigenSolver) + get_aabb gaussian.h:304-319: extents_j = R sqrt(max(l_j, 0)),
        // h = sum_j |u_j| extents_j (u_j = column j of eigvecs, accumulated j = 0, 1, 2 from zero)
        float ev[3], U[3][3];
        eigen_selfadjoint3(cov, ev, U);
        float ext[3];
        for (int j = 0; j < 3; ++j) ext[j] = R * std::sqrt(std::max(ev[j], 0.0f));
        V3 h{0.0f, 0.0f, 0.0f};
        for (int j = 0; j < 3; ++j) {
            const V3 u{std::fabs(U[0][j]), std::fabs(U[1][j]), std::fabs(U[2][j])};
            h = h + ext[j] * u;
        }
        bmin = mean - h;
        bmax = mean + h;
    }
    // gaussian.h:111-117
    float evaluate(V3 x) const {
        V3 d = x - mean;
        // (-0.5f * d^T) * inv_cov * d, coefficient-wise lazy products (1+2 reductions)
        V3 l{-0.5f * d.x, -0.5f * d.y, -0.5f * d.z};
        V3 w{l.x * inv_cov(0, 0) + (l.y * inv_cov(1, 0) + l.z * inv_cov(2, 0)),
             l.x * inv_cov(0, 1) + (l.y * inv_cov(1, 1) + l.z * inv_cov(2, 1)),
             l.x * inv_cov(0, 2) + (l.y * inv_cov(1, 2) + l.z * inv_cov(2, 2))};
        float exponent = w.x * d.x + (w.y * d.y + w.z * d.z);
        return norm * std::exp(exponent);
    }
    float mu_t(V3 x) const { return density * evaluate(x); }
    // gaussian.h:126-164
    bool intersect_direct(const Ray& ray, float& t_enter, float& t_exit) const {
        V3 p = ray.origin - mean;
        V3 Md = mul(inv_cov, ray.direction);
        V3 Mp = mul(inv_cov, p);
        float A = dot(ray.direction, Md);
        float B = 2.0f * dot(p, Md);
        float C = dot(p, Mp) - (R * R);
        float discriminant = B * B - 4.0f * A * C;
        if (discriminant < 0.0f) return false;
        float sqrtD = std::sqrt(discriminant);
        float t0 = (-B - sqrtD) / (2.0f * A);
        float t1 = (-B + sqrtD) / (2.0f * A);
        if (t0 > t1) std::swap(t0, t1);
        if (t1 < 0.0f) return false;
        t_enter = (t0 >= 0.0f) ? t0 : 0.0f;
        t_exit = t1;
        return true;
    }
    // intersect_direct / optical_depth in double (g_accurate_chords: secondary rays of the sparse-list restatement)
    void quad_acc(const Ray& ray, double& A, double& B, double& C) const {
        const double p[3] = {(double)ray.origin.x - mean.x, (double)ray.origin.y - mean.y, (double)ray.origin.z - mean.z};
        const double d[3] = {ray.direction.x, ray.direction.y, ray.direction.z};
        A = B = C = 0.0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                A += d[i] * inv_cov(i, j) * d[j];
                B += 2.0 * p[i] * inv_cov(i, j) * d[j];
                C += p[i] * inv_cov(i, j) * p[j];
            }
    }
    bool intersect_direct_acc(const Ray& ray, float& t_enter, float& t_exit) const {
        double A, B, C;
        quad_acc(ray, A, B, C);
        const double disc = B * B - 4.0 * A * (C - 9.0);
        if (disc < 0.0) return false;
        const double t0 = (-B - std::sqrt(disc)) / (2.0 * A), t1 = (-B + std::sqrt(disc)) / (2.0 * A);
        if (t1 < 0.0) return false;
        t_enter = (float)std::max(t0, 0.0);
        t_exit = (float)t1;
        return true;
    }
    float optical_depth_acc(const Ray& ray, float t0, float t1) const {
        double A, B, C;
        quad_acc(ray, A, B, C);
        const double pref = (double)density * (double)norm * std::sqrt(std::numbers::pi / (2.0 * A));
        auto F = [&](double t) { return std::erf((B + 2.0 * A * t) / (2.0 * std::sqrt(2.0 * A))); };
        return (float)(pref * std::exp(-0.5 * (C - B * B / (4.0 * A))) * (F(t1) - F(t0)));
    }
    // gaussian.h:208-231
    float optical_depth(const Ray& ray, float t0, float t1) const {
        V3 p = ray.origin - mean;
        V3 Md = mul(inv_cov, ray.direction);
        V3 Mp = mul(inv_cov, p);
        float A = dot(ray.direction, Md);
        float B = 2.0f * dot(p, Md);
        float C = dot(p, Mp);
        float pref = density * norm * std::sqrt(std::numbers::pi / (2.0f * A));
        auto F = [&](float t) {
            float arg = (B + 2.0f * A * t) / (2.0f * std::sqrt(2.0f * A));
            return std::erf(arg);
        };
        return pref * std::exp(-0.5f * (C - B * B / (4.0f * A))) * (F(t1) - F(t0));
    }
};

// Tangent-hit ties met by the calling thread (intersect_events: a Gaussian whose entry and exit keys are equal);
// orc_render reports them per pixel into g_tie_out when set (orc_tie_flags).
static thread_local int64_t g_ties = 0;
static int32_t* g_tie_out = nullptr;

// smm.h:7-15
struct PrimitiveHitEvent {
    float t;
    bool entering;
    size_t index;
    bool operator<(const PrimitiveHitEvent& o) const { return t < o.t; }
};

// ---------------------------------------------------------------------------------------------
// gmm.h:35-578 — mixture + midpoint-split BVH (leaf <= 4; SAH compiled out, gmm.h:162).
// ---------------------------------------------------------------------------------------------
struct GMM {
    struct Node {
        V3 bmin{INFINITY, INFINITY, INFINITY}, bmax{-INFINITY, -INFINITY, -INFINITY};
        V3 tbmin{INFINITY, INFINITY, INFINITY}, tbmax{-INFINITY, -INFINITY, -INFINITY};  // union of the padded boxes
        uint32_t leftFirst = 0, count = 0;
        bool isLeaf() const { return count > 0; }
    };
    std::vector<Gaussian> gaussians;
    std::vector<uint32_t> indices;
    std::vector<Node> nodes;

    static float IntersectAABB(const Ray& ray, V3 bmin, V3 bmax) {  // gmm.h:48-63
        V3 rD{1.0f / ray.direction.x, 1.0f / ray.direction.y, 1.0f / ray.direction.z};
        float tx1 = (bmin.x - ray.origin.x) * rD.x;
        float tx2 = (bmax.x - ray.origin.x) * rD.x;
        float tmin = std::min(tx1, tx2), tmax = std::max(tx1, tx2);
        float ty1 = (bmin.y - ray.origin.y) * rD.y;
        float ty2 = (bmax.y - ray.origin.y) * rD.y;
        tmin = std::max(tmin, std::min(ty1, ty2));
        tmax = std::min(tmax, std::max(ty1, ty2));
        float tz1 = (bmin.z - ray.origin.z) * rD.z;
        float tz2 = (bmax.z - ray.origin.z) * rD.z;
        tmin = std::max(tmin, std::min(tz1, tz2));
        tmax = std::min(tmax, std::max(tz1, tz2));
        if (tmax >= tmin && tmin < std::numeric_limits<float>::infinity() && tmax > 0.0f) return tmin;
        return std::numeric_limits<float>::infinity();
    }
    void UpdateNodeBounds(uint32_t ni) {
        Node& n = nodes[ni];
        n.bmin = n.tbmin = {INFINITY, INFINITY, INFINITY};
        n.bmax = n.tbmax = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = 0; i < n.count; ++i) {
            const Gaussian& g = gaussians[indices[n.leftFirst + i]];
            for (int k = 0; k < 3; ++k) {
                n.bmin[k] = std::min(n.bmin[k], g.bmin[k]);
                n.bmax[k] = std::max(n.bmax[k], g.bmax[k]);
                n.tbmin[k] = std::min(n.tbmin[k], g.tbmin[k]);
                n.tbmax[k] = std::max(n.tbmax[k], g.tbmax[k]);
            }
        }
    }
    void BuildBVH() {  // gmm.h:231-260
        uint32_t N = (uint32_t)gaussians.size();
        indices.resize(N);
        for (uint32_t i = 0; i < N; ++i) indices[i] = i;
        nodes.clear();
        nodes.reserve(std::max<size_t>(1, 2 * N));
        nodes.emplace_back();
        nodes[0].leftFirst = 0;
        nodes[0].count = N;
        UpdateNodeBounds(0);
        // iterative version of SubdivideNode (gmm.h:318-446, midpoint branch) — same splits
        std::vector<uint32_t> todo{0};
        while (!todo.empty()) {
            uint32_t ni = todo.back();
            todo.pop_back();
            Node node = nodes[ni];
            if (node.count <= 4) continue;
            V3 e = node.bmax - node.bmin;
            int axis = (e.y > e.x) ? 1 : 0;
            if (e.z > e[axis]) axis = 2;
            float splitPos = 0.5f * (node.bmin[axis] + node.bmax[axis]);
            int64_t i = node.leftFirst;
            int64_t j = i + node.count - 1;
            while (i <= j) {
                if (gaussians[indices[i]].mean[axis] < splitPos) ++i;
                else { std::swap(indices[i], indices[j]); --j; }
            }
            uint32_t leftCount = (uint32_t)(i - node.leftFirst);
            if (leftCount == 0 || leftCount == node.count) continue;
            uint32_t l = (uint32_t)nodes.size();
            nodes.emplace_back();
            uint32_t r = (uint32_t)nodes.size();
            nodes.emplace_back();
            nodes[l].leftFirst = node.leftFirst;
            nodes[l].count = leftCount;
            nodes[r].leftFirst = node.leftFirst + leftCount;
            nodes[r].count = node.count - leftCount;
            nodes[ni].leftFirst = l;
            nodes[ni].count = 0;
            UpdateNodeBounds(l);
            UpdateNodeBounds(r);
            todo.push_back(r);
            todo.push_back(l);
        }
    }
    // gmm.h:457-515
    void intersect_events(const Ray& ray, std::vector<PrimitiveHitEvent>& out, bool acc = false) const {
        out.clear();
        if (gaussians.empty() || nodes.empty()) return;
        std::vector<int> stack;
        stack.reserve(64);
        stack.push_back(0);
        const float inf = std::numeric_limits<float>::infinity();
        while (!stack.empty()) {
            int ni = stack.back();
            stack.pop_back();
            const Node& node = nodes[ni];
            float tmin = IntersectAABB(ray, node.bmin, node.bmax);
            if (tmin == inf) continue;
            if (node.isLeaf()) {
                for (int ii = 0; ii < (int)node.count; ++ii) {
                    uint32_t gidx = indices[node.leftFirst + ii];
                    float t0, t1;
                    if (acc ? gaussians[gidx].intersect_direct_acc(ray, t0, t1) : gaussians[gidx].intersect_direct(ray, t0, t1)) {
                        if (t0 >= 0.0f) out.push_back({t0, true, gidx});
                        if (t1 >= 0.0f) out.push_back({t1, false, gidx});
                        if (t0 == t1) ++g_ties;  // entry and exit with equal keys: std::sort decides their order
                    }
                }
            } else {
                int li = (int)node.leftFirst, ri = li + 1;
                float dl = IntersectAABB(ray, nodes[li].bmin, nodes[li].bmax);
                float dr = IntersectAABB(ray, nodes[ri].bmin, nodes[ri].bmax);
                if (dl > dr) {
                    if (dl != inf) stack.push_back(li);
                    if (dr != inf) stack.push_back(ri);
                } else {
                    if (dr != inf) stack.push_back(ri);
                    if (dl != inf) stack.push_back(li);
                }
            }
        }
        if (!out.empty()) {
            auto by_t = [](const PrimitiveHitEvent& a, const PrimitiveHitEvent& b) { return a.t < b.t; };
            if (g_stable_ties) std::stable_sort(out.begin(), out.end(), by_t);
            else std::sort(out.begin(), out.end(), by_t);
        }
    }
    // gmm.h:98-126
    void evaluate_sigma(const std::vector<bool>& active, V3 pos, float& sigma_a, float& sigma_s) const {
        float sum_mu_t = 0.0f, sum_mu_t_alb = 0.0f;
        for (size_t i = 0; i < gaussians.size(); ++i) {
            if (!active[i]) continue;
            float mu_t_i = gaussians[i].mu_t(pos);
            sum_mu_t += mu_t_i;
            sum_mu_t_alb += mu_t_i * gaussians[i].albedo;
        }
        if (sum_mu_t <= 0.0f) { sigma_s = sigma_a = 0.0f; return; }
        float a_mix = sum_mu_t_alb / sum_mu_t;
        sigma_s = a_mix * sum_mu_t;
        sigma_a = (1.0f - a_mix) * sum_mu_t;
    }
    // gmm.h:146-157
    float transmittance_over_segment(const Ray& ray, float t0, float t1, const std::vector<size_t>& act, bool acc = false) const {
        float s = 0.0f;
        for (size_t i : act) s += acc ? gaussians[i].optical_depth_acc(ray, t0, t1) : gaussians[i].optical_depth(ray, t0, t1);
        return std::exp(-s);
    }
};

// smm.h:17-103
struct Sphere {
    V3 center;
    float radius, sigma_a, sigma_s;
    bool intersect(const Ray& ray, float& t_enter, float& t_exit) const {  // smm.h:29-39
        V3 L = center - ray.origin;
        float tca = dot(L, ray.direction);
        float d2 = sqnorm(L) - tca * tca;
        float r2 = radius * radius;
        if (d2 > r2) return false;
        float thc = std::sqrt(r2 - d2);
        t_enter = tca - thc;
        t_exit = tca + thc;
        return t_exit >= 0.0f;
    }
};
struct SMM {
    std::vector<Sphere> spheres;
    void intersect_events(const Ray& ray, std::vector<PrimitiveHitEvent>& out) const {  // smm.h:54-63
        for (size_t i = 0; i < spheres.size(); ++i) {
            float a, b;
            if (spheres[i].intersect(ray, a, b)) {
                if (a >= 0.0f) out.push_back({a, true, i});
                if (b >= 0.0f) out.push_back({b, false, i});
            }
        }
        std::sort(out.begin(), out.end());
    }
    void evaluate_sigma(const std::vector<bool>& active, float& sa, float& ss) const {  // :66-76
        sa = 0.0f; ss = 0.0f;
        for (size_t i = 0; i < spheres.size(); ++i)
            if (active[i]) { sa += spheres[i].sigma_a; ss += spheres[i].sigma_s; }
    }
    float transmittance_from_events(const Ray&, const std::vector<PrimitiveHitEvent>& events, float tmax) const {  // :79-103
        float T = 1.0f;
        std::vector<bool> active(spheres.size(), false);
        float t_prev = 0.0f;
        for (const auto& e : events) {
            if (e.t > tmax) break;
            float dt = e.t - t_prev;
            float sigma_t = 0.0f;
            for (size_t i = 0; i < spheres.size(); ++i)
                if (active[i]) sigma_t += spheres[i].sigma_a + spheres[i].sigma_s;
            T *= std::exp(-sigma_t * dt);
            active[e.index] = e.entering;
            t_prev = e.t;
        }
        return T;
    }
};

struct Light { V3 position, intensity; };

struct Scene {
    int volume_type = 0;  // 0 gaussians, 1 spheres
    GMM gmm;
    SMM smm;
    std::vector<Light> lights;
    V3 env_color{0.53f, 0.81f, 0.92f};  // scene.h:29
    size_t num() const { return volume_type == 0 ? gmm.gaussians.size() : smm.spheres.size(); }
};

// scene.h:38-68 (CRLF-tolerant through operator>>, any other tag skipped)
static Scene load_SMM(const std::string& fn) {
    Scene s;
    s.volume_type = 1;
    std::ifstream file(fn);
    if (!file) throw std::runtime_error("Failed to open scene file: " + fn);
    std::string tag;
    while (file >> tag) {
        if (tag == "l") {
            float x, y, z, r, g, b;
            file >> x >> y >> z >> r >> g >> b;
            s.lights.push_back({{x, y, z}, {r, g, b}});
        } else if (tag == "s") {
            float x, y, z, rad, sa, ss;
            file >> x >> y >> z >> rad >> sa >> ss;
            s.smm.spheres.push_back({{x, y, z}, rad, sa, ss});
        }
    }
    return s;
}
// scene.h:72-120 — including the emission peek quirk (scene.h:99-106).
static Scene load_GMM(const std::string& fn) {
    Scene s;
    s.volume_type = 0;
    std::ifstream file(fn);
    if (!file) throw std::runtime_error("Failed to open scene file: " + fn);
    std::string tag;
    while (file >> tag) {
        if (tag == "l") {
            float x, y, z, r, g, b;
            file >> x >> y >> z >> r >> g >> b;
            s.lights.push_back({{x, y, z}, {r, g, b}});
        } else if (tag == "g") {
            float mx, my, mz, cxx, cxy, cxz, cyy, cyz, czz, density, albedo;
            file >> mx >> my >> mz >> cxx >> cxy >> cxz >> cyy >> cyz >> czz >> density >> albedo;
            int next = file.peek();
            if (next != '\n' && next != EOF) {
                float er, eg, eb;
                if (file >> er >> eg >> eb) { (void)er; }
            }
            M3 cov{{{cxx, cxy, cxz}, {cxy, cyy, cyz}, {cxz, cyz, czz}}};
            s.gmm.gaussians.emplace_back(V3{mx, my, mz}, cov, density, albedo);
        }
    }
    s.gmm.BuildBVH();
    return s;
}

// =============================================================================================
// Integrators
// =============================================================================================
static const float kInv4Pi = (float)(1.0f / (4.0f * std::numbers::pi));  // Vector3f * double → float
static const float k4Pi = (float)(4.0f * std::numbers::pi);

// test_integrators.h:160-296 — RayMarchingGaussians per pixel.
// DEBUG trace of one rm_gaussians_pixel call (orc_debug_march): per step (t, #active, sigma_s, T after)
static thread_local std::vector<float>* g_rm_trace = nullptr;
static V3 rm_gaussians_pixel(const Scene& scene, const Camera& cam, int x, int y, int W, int H,
                             float step_size, int env_samples) {
    const GMM& gmm = scene.gmm;
    float u = (x + 0.5f) / W, v = (y + 0.5f) / H;
    Ray ray = cam.sample_ray(u, v);
    std::vector<PrimitiveHitEvent> events;
    gmm.intersect_events(ray, events);
    if (events.empty()) return scene.env_color;
    float t_end = events.back().t;
    std::vector<bool> active(gmm.gaussians.size(), false);
    size_t evt_i = 0;
    float t = 0.0f, T = 1.0f;
    V3 L{0, 0, 0};
    int k = 0;  // step counter (keys the deterministic env RNG)
    while (t < t_end) {
        while (evt_i < events.size() && events[evt_i].t <= t) {
            active[events[evt_i].index] = events[evt_i].entering;
            ++evt_i;
        }
        V3 pos = ray.origin + t * ray.direction;
        float sigma_a, sigma_s;
        gmm.evaluate_sigma(active, pos, sigma_a, sigma_s);
        if (sigma_s > 0.0f) {
            V3 Li{0, 0, 0};
            for (const auto& light : scene.lights) {
                V3 wi = normalized(light.position - pos);
                float dist = norm(light.position - pos);
                Ray shadow_ray(pos, wi);
                std::vector<PrimitiveHitEvent> shadow_ev;
                gmm.intersect_events(shadow_ray, shadow_ev);
                for (size_t i = 0; i < active.size(); ++i)
                    if (active[i]) shadow_ev.insert(shadow_ev.begin(), {0.0f, true, i});
                std::vector<size_t> active_idxs;
                std::vector<bool> mask = active;
                float t_prev = 0;
                size_t se_i = 0;
                float Tr = 1.0f;
                while (t_prev < dist) {
                    float t_next = (se_i < shadow_ev.size() ? shadow_ev[se_i].t : dist);
                    active_idxs.clear();
                    for (size_t i = 0; i < mask.size(); ++i)
                        if (mask[i]) active_idxs.push_back(i);
                    Tr *= gmm.transmittance_over_segment(shadow_ray, t_prev, t_next, active_idxs);
                    if (se_i < shadow_ev.size()) {
                        mask[shadow_ev[se_i].index] = shadow_ev[se_i].entering;
                        ++se_i;
                    }
                    t_prev = t_next;
                }
                float d2 = dist * dist;
                Li = Li + V3{(Tr * light.intensity.x) / d2, (Tr * light.intensity.y) / d2, (Tr * light.intensity.z) / d2};
            }
            V3 Le{0, 0, 0};
            PCG32 rng(derive_path_seed(x, y, k), 1);
            for (int si = 0; si < env_samples; ++si) {
                float xi1 = rng.uniform_env();
                float xi2 = rng.uniform_env();
                V3 wi = env_dir(xi1, xi2);
                Ray env_ray(pos, wi);
                std::vector<PrimitiveHitEvent> env_ev;
                gmm.intersect_events(env_ray, env_ev);
                for (size_t i = 0; i < active.size(); ++i)
                    if (active[i]) env_ev.insert(env_ev.begin(), {0.0f, true, i});
                std::vector<size_t> active_idxs;
                std::vector<bool> mask = active;
                float t_prev = 0, Tr_env = 1.0f;
                size_t ei = 0;
                while (ei < env_ev.size()) {
                    float t_next = env_ev[ei].t;
                    active_idxs.clear();
                    for (size_t i = 0; i < mask.size(); ++i)
                        if (mask[i]) active_idxs.push_back(i);
                    Tr_env *= gmm.transmittance_over_segment(env_ray, t_prev, t_next, active_idxs);
                    mask[env_ev[ei].index] = env_ev[ei].entering;
                    t_prev = t_next;
                    ++ei;
                }
                Le = Le + Tr_env * scene.env_color;
            }
            float fs = float(env_samples);
            Le = V3{(Le.x / fs) * k4Pi, (Le.y / fs) * k4Pi, (Le.z / fs) * k4Pi};
            float Ts = T * sigma_s;
            V3 S = Li + Le;
            L = L + V3{((Ts * S.x) * step_size) * kInv4Pi, ((Ts * S.y) * step_size) * kInv4Pi, ((Ts * S.z) * step_size) * kInv4Pi};
        }
        std::vector<size_t> active_idxs;
        for (size_t i = 0; i < active.size(); ++i)
            if (active[i]) active_idxs.push_back(i);
        float segmentTr = gmm.transmittance_over_segment(ray, t, t + step_size, active_idxs);
        T *= segmentTr;
        if (g_rm_trace && !active_idxs.empty()) {
            g_rm_trace->insert(g_rm_trace->end(), {t, (float)active_idxs.size(), sigma_s, T});
            for (size_t i : active_idxs) g_rm_trace->push_back((float)i);
        }
        t += step_size;
        ++k;
    }
    L = L + T * scene.env_color;
    return L;
}

// integrator.h:105-135 — PureRayMarching::march_transmittance: marched transmittance on [0, t_max).
static float march_transmittance(const Scene& scene, const Ray& ray, float t_max, const std::vector<PrimitiveHitEvent>& events,
                                 const std::vector<bool>& active0, float step_size) {
    const GMM& gmm = scene.gmm;
    std::vector<bool> active = active0;
    float T = 1.0f;
    size_t evt_idx = 0, n_evt = events.size();
    for (float t = 0.0f; t < t_max; t += step_size) {
        while (evt_idx < n_evt && events[evt_idx].t <= t) {
            active[events[evt_idx].index] = events[evt_idx].entering;
            ++evt_idx;
        }
        V3 pos = ray.origin + t * ray.direction;
        float sigma_a, sigma_s;
        gmm.evaluate_sigma(active, pos, sigma_a, sigma_s);
        float sigma_t = sigma_a + sigma_s;
        T *= std::exp(-sigma_t * step_size);
    }
    return T;
}

// integrator.h:150-265 — PureRayMarching::render per pixel (environment directions from the same
// deterministic PCG32 sampler as rm_gaussians_pixel, keyed by the step index).
static V3 rm_pure_pixel(const Scene& scene, const Camera& cam, int x, int y, int W, int H, float step_size,
                        int env_samples) {
    const GMM& gmm = scene.gmm;
    float u = (x + 0.5f) / W, v = (y + 0.5f) / H;
    Ray ray = cam.sample_ray(u, v);
    std::vector<PrimitiveHitEvent> primary_events;
    gmm.intersect_events(ray, primary_events);
    if (primary_events.empty()) return scene.env_color;
    float t_end = primary_events.back().t;
    std::vector<bool> primary_active(gmm.gaussians.size(), false);
    for (auto& e : primary_events)
        if (e.t == 0.0f && e.entering) primary_active[e.index] = true;
    float T = 1.0f;
    V3 L{0, 0, 0};
    size_t idx_evt = 0, n_evt = primary_events.size();
    int k = 0;
    for (float t = 0.0f; t < t_end; t += step_size, ++k) {
        while (idx_evt < n_evt && primary_events[idx_evt].t <= t) {
            primary_active[primary_events[idx_evt].index] = primary_events[idx_evt].entering;
            ++idx_evt;
        }
        V3 pos = ray.origin + t * ray.direction;
        float sigma_a, sigma_s;
        gmm.evaluate_sigma(primary_active, pos, sigma_a, sigma_s);
        float sigma_t = sigma_a + sigma_s;
        if (sigma_s > 0.0f) {
            V3 Li{0, 0, 0};
            for (const auto& light : scene.lights) {
                V3 wi = normalized(light.position - pos);
                float dist = norm(light.position - pos);
                Ray shadow_ray(pos, wi);
                std::vector<PrimitiveHitEvent> shadow_events;
                gmm.intersect_events(shadow_ray, shadow_events);
                std::vector<bool> shadow_active = primary_active;
                for (size_t i = 0; i < shadow_active.size(); ++i)
                    if (primary_active[i]) shadow_events.insert(shadow_events.begin(), {0.0f, true, i});
                float Tr = march_transmittance(scene, shadow_ray, dist, shadow_events, shadow_active, step_size);
                float d2 = dist * dist;
                Li = Li + V3{(Tr * light.intensity.x) / d2, (Tr * light.intensity.y) / d2, (Tr * light.intensity.z) / d2};
            }
            V3 Le{0, 0, 0};
            PCG32 rng(derive_path_seed(x, y, k), 1);
            for (int s = 0; s < env_samples; ++s) {
                float xi1 = rng.uniform_env();
                float xi2 = rng.uniform_env();
                Ray env_ray(pos, env_dir(xi1, xi2));
                std::vector<PrimitiveHitEvent> env_events;
                gmm.intersect_events(env_ray, env_events);
                std::vector<bool> env_active = primary_active;
                for (size_t i = 0; i < env_active.size(); ++i)
                    if (primary_active[i]) env_events.insert(env_events.begin(), {0.0f, true, i});
                float t_env_end = env_events.empty() ? 0.0f : env_events.back().t;
                float Tr_env = march_transmittance(scene, env_ray, t_env_end, env_events, env_active, step_size);
                Le = Le + Tr_env * scene.env_color;
            }
            float fs = float(env_samples);
            Le = V3{(Le.x / fs) * k4Pi, (Le.y / fs) * k4Pi, (Le.z / fs) * k4Pi};
            float Ts = T * sigma_s;
            V3 S = Li + Le;
            L = L + V3{((Ts * S.x) * step_size) * kInv4Pi, ((Ts * S.y) * step_size) * kInv4Pi, ((Ts * S.z) * step_size) * kInv4Pi};
        }
        T *= std::exp(-sigma_t * step_size);
    }
    L = L + T * scene.env_color;
    return L;
}

// ---------------------------------------------------------------------------------------------
// Same per-pixel algorithm as rm_gaussians_pixel, for the CPU *baseline* of bench.py only.
// Two changes, both bit-neutral (tests/test_oracle_golden.py checks bitwise equality with the
// faithful function above):
//   * the reference's O(N) std::vector<bool> active masks (test_integrators.h:181, 224, 262,
//     281-283; gmm.h:108-113) are kept as an index-sorted list plus a byte mask, so every sum runs
//     over exactly the same indices in exactly the same (ascending) order;
//   * the march stops once T == 0: every later term is T*sigma_s*(...) = +0 and the final T*env is
//     +0, so L is unchanged (the device path stops at the same point).
// Without them one 1M-Gaussian pixel costs minutes of mask scans (DESIGN.md §CPU baseline).
// ---------------------------------------------------------------------------------------------
struct SparseSet {
    std::vector<uint8_t>* mask;  // shared scratch of size N, all zero outside `list`
    std::vector<size_t> list;    // ascending indices i with mask[i] == 1
    void set(size_t i, bool v) {
        uint8_t& m = (*mask)[i];
        if ((m != 0) == v) return;
        m = v ? 1 : 0;
        auto it = std::lower_bound(list.begin(), list.end(), i);
        if (v) list.insert(it, i);
        else list.erase(it);
    }
    void clear() {
        for (size_t i : list) (*mask)[i] = 0;
        list.clear();
    }
};

// DEBUG trace of one rm_gaussians_pixel_lists call (orc_debug_pixel_records): per scattering step a row
// (k, pos xyz, T sigma_s, Li + Le rgb, #active, then every secondary ray's Tr: lights, then env samples)
static thread_local std::vector<float>* g_rec_trace = nullptr;
static thread_local std::vector<float>* g_rec_active = nullptr;  // with it: per row, #active then the active ids
static V3 rm_gaussians_pixel_lists(const Scene& scene, const Camera& cam, int x, int y, int W, int H,
                                   float step_size, int env_samples) {
    const GMM& gmm = scene.gmm;
    static thread_local std::vector<uint8_t> mask_a, mask_b;
    if (mask_a.size() != gmm.gaussians.size()) mask_a.assign(gmm.gaussians.size(), 0);
    if (mask_b.size() != gmm.gaussians.size()) mask_b.assign(gmm.gaussians.size(), 0);
    float u = (x + 0.5f) / W, v = (y + 0.5f) / H;
    Ray ray = cam.sample_ray(u, v);
    std::vector<PrimitiveHitEvent> events;
    gmm.intersect_events(ray, events);
    if (events.empty()) return scene.env_color;
    float t_end = events.back().t;
    SparseSet active{&mask_a, {}};
    size_t evt_i = 0;
    float t = 0.0f, T = 1.0f;
    V3 L{0, 0, 0};
    int k = 0;
    // secondary-ray segment loop on a copy of the primary active set (test_integrators.h:208-235, 255-271)
    auto secondary = [&](const Ray& r, std::vector<PrimitiveHitEvent>& ev, bool to_light, float dist) {
        for (size_t i : active.list) ev.insert(ev.begin(), {0.0f, true, i});
        SparseSet mask{&mask_b, active.list};
        for (size_t i : mask.list) mask_b[i] = 1;
        float t_prev = 0, Tr = 1.0f;
        size_t ei = 0;
        if (to_light) {
            while (t_prev < dist) {
                float t_next = (ei < ev.size() ? ev[ei].t : dist);
                Tr *= gmm.transmittance_over_segment(r, t_prev, t_next, mask.list, g_accurate_chords);
                if (ei < ev.size()) {
                    mask.set(ev[ei].index, ev[ei].entering);
                    ++ei;
                }
                t_prev = t_next;
            }
        } else {
            while (ei < ev.size()) {
                float t_next = ev[ei].t;
                Tr *= gmm.transmittance_over_segment(r, t_prev, t_next, mask.list, g_accurate_chords);
                mask.set(ev[ei].index, ev[ei].entering);
                t_prev = t_next;
                ++ei;
            }
        }
        mask.clear();
        return Tr;
    };
    while (t < t_end) {
        while (evt_i < events.size() && events[evt_i].t <= t) {
            active.set(events[evt_i].index, events[evt_i].entering);
            ++evt_i;
        }
        V3 pos = ray.origin + t * ray.direction;
        float sum_mu_t = 0.0f, sum_mu_t_alb = 0.0f, sigma_s = 0.0f;  // gmm.h:98-126 over the list
        for (size_t i : active.list) {
            float mu_t_i = gmm.gaussians[i].mu_t(pos);
            sum_mu_t += mu_t_i;
            sum_mu_t_alb += mu_t_i * gmm.gaussians[i].albedo;
        }
        if (!(sum_mu_t <= 0.0f)) {
            float a_mix = sum_mu_t_alb / sum_mu_t;
            sigma_s = a_mix * sum_mu_t;
        }
        if (sigma_s > 0.0f) {
            V3 Li{0, 0, 0};
            std::vector<float> trs;
            for (const auto& light : scene.lights) {
                V3 wi = normalized(light.position - pos);
                float dist = norm(light.position - pos);
                Ray shadow_ray(pos, wi);
                std::vector<PrimitiveHitEvent> shadow_ev;
                gmm.intersect_events(shadow_ray, shadow_ev, g_accurate_chords);
                float Tr = secondary(shadow_ray, shadow_ev, true, dist);
                if (g_rec_trace) trs.push_back(Tr);
                float d2 = dist * dist;
                Li = Li + V3{(Tr * light.intensity.x) / d2, (Tr * light.intensity.y) / d2, (Tr * light.intensity.z) / d2};
            }
            V3 Le{0, 0, 0};
            PCG32 rng(derive_path_seed(x, y, k), 1);
            for (int si = 0; si < env_samples; ++si) {
                float xi1 = rng.uniform_env();
                float xi2 = rng.uniform_env();
                Ray env_ray(pos, env_dir(xi1, xi2));
                std::vector<PrimitiveHitEvent> env_ev;
                gmm.intersect_events(env_ray, env_ev, g_accurate_chords);
                float Tr_env = secondary(env_ray, env_ev, false, 0.0f);
                if (g_rec_trace) trs.push_back(Tr_env);
                Le = Le + Tr_env * scene.env_color;
            }
            float fs = float(env_samples);
            Le = V3{(Le.x / fs) * k4Pi, (Le.y / fs) * k4Pi, (Le.z / fs) * k4Pi};
            float Ts = T * sigma_s;
            V3 S = Li + Le;
            if (g_rec_trace) {
                g_rec_trace->insert(g_rec_trace->end(), {(float)k, pos.x, pos.y, pos.z, Ts, S.x, S.y, S.z, (float)active.list.size()});
                g_rec_trace->insert(g_rec_trace->end(), trs.begin(), trs.end());
                if (g_rec_active) {
                    g_rec_active->push_back((float)active.list.size());
                    for (size_t i : active.list) g_rec_active->push_back((float)i);
                }
            }
            L = L + V3{((Ts * S.x) * step_size) * kInv4Pi, ((Ts * S.y) * step_size) * kInv4Pi, ((Ts * S.z) * step_size) * kInv4Pi};
        }
        T *= gmm.transmittance_over_segment(ray, t, t + step_size, active.list);
        t += step_size;
        ++k;
        if (T == 0.0f) break;
    }
    active.clear();
    L = L + T * scene.env_color;
    return L;
}

// test_integrators.h:23-135 — RayMarchingSpheres per pixel.
static V3 rm_spheres_pixel(const Scene& scene, const Camera& cam, int i, int j, int W, int H,
                           float step_size, int env_samples) {
    const SMM& smm = scene.smm;
    float u = (i + 0.5f) / W;
    float v = (j + 0.5f) / H;
    Ray ray = cam.sample_ray(u, v);
    V3 radiance{0, 0, 0};
    std::vector<PrimitiveHitEvent> events;
    smm.intersect_events(ray, events);
    if (events.empty()) return scene.env_color;
    std::vector<bool> active(smm.spheres.size(), false);
    size_t current_event = 0;
    float t = 0.0f, T = 1.0f;
    float t_end = events.back().t;
    int k = 0;
    while (t < t_end) {
        while (current_event < events.size() && events[current_event].t <= t) {
            active[events[current_event].index] = events[current_event].entering;
            current_event++;
        }
        V3 pos = ray.origin + t * ray.direction;
        float sigma_a, sigma_s;
        smm.evaluate_sigma(active, sigma_a, sigma_s);
        if (sigma_s > 0.0f) {
            V3 Li{0, 0, 0};
            for (const auto& light : scene.lights) {
                V3 wi = normalized(light.position - pos);
                float dist = norm(light.position - pos);
                Ray shadow_ray(pos, wi);
                std::vector<PrimitiveHitEvent> shadow_events;
                smm.intersect_events(shadow_ray, shadow_events);
                for (size_t ii = 0; ii < active.size(); ++ii)
                    if (active[ii]) shadow_events.insert(shadow_events.begin(), {0.0f, true, ii});
                float Tr = smm.transmittance_from_events(shadow_ray, shadow_events, dist);
                float d2 = dist * dist;
                Li = Li + V3{(Tr * light.intensity.x) / d2, (Tr * light.intensity.y) / d2, (Tr * light.intensity.z) / d2};
            }
            V3 Le_env{0, 0, 0};
            PCG32 rng(derive_path_seed(i, j, k), 1);
            for (int s = 0; s < env_samples; ++s) {
                float xi1 = rng.uniform_env();
                float xi2 = rng.uniform_env();
                V3 wi = env_dir(xi1, xi2);
                Ray shadow(pos, wi);
                std::vector<PrimitiveHitEvent> shadow_ev;
                smm.intersect_events(shadow, shadow_ev);
                for (size_t ii = 0; ii < active.size(); ++ii)
                    if (active[ii]) shadow_ev.insert(shadow_ev.begin(), {0.0f, true, ii});
                float Tr_env = smm.transmittance_from_events(shadow, shadow_ev, std::numeric_limits<float>::infinity());
                Le_env = Le_env + Tr_env * scene.env_color;
            }
            float fs = float(env_samples);
            Le_env = V3{Le_env.x / fs, Le_env.y / fs, Le_env.z / fs};
            Le_env = V3{Le_env.x * k4Pi, Le_env.y * k4Pi, Le_env.z * k4Pi};
            float Ts = T * sigma_s;
            V3 S = Li + Le_env;
            radiance = radiance + V3{((Ts * S.x) * step_size) * kInv4Pi, ((Ts * S.y) * step_size) * kInv4Pi, ((Ts * S.z) * step_size) * kInv4Pi};
        }
        T *= std::exp(-step_size * (sigma_a + sigma_s));
        t += step_size;
        ++k;
    }
    radiance = radiance + T * scene.env_color;
    return radiance;
}

// =============================================================================================
// Free-flight integrators. The reference's paths are deterministic per
// (x, y, sample) through PCG32(derive_path_seed(x, y, si), 1) (rng.h:20-57), so these are
// restated as written, incl. sample_uniform_direction's libm trigonometry (integrator.h:32-44).
// =============================================================================================

// integrator.h:32-44. theta: 2.0f * pi (double) * xi1 -> double product rounded to float.
static V3 sample_uniform_direction(PCG32& rng) {
    float xi1 = rng.uniform();
    float xi2 = rng.uniform();
    float theta = 2.0f * std::numbers::pi * xi1;
    float phi = std::acos(1.0f - 2.0f * xi2);
    float x = std::sin(phi) * std::cos(theta);
    float y = std::sin(phi) * std::sin(theta);
    float z = std::cos(phi);
    return {x, y, z};
}

// gaussian.h:10-25 (Winitzki, a = 0.14, double).
static double erfinv_approx(double x) {
    if (std::isnan(x)) return std::numeric_limits<double>::quiet_NaN();
    if (x <= -1.0) return -std::numeric_limits<double>::infinity();
    if (x >= 1.0) return std::numeric_limits<double>::infinity();
    const double a = 0.14;
    double sign = (x < 0.0) ? -1.0 : 1.0;
    double ln_term = std::log(1.0 - x * x);
    double first = 2.0 / (std::numbers::pi * a) + ln_term / 2.0;
    double inside = first * first - ln_term / a;
    if (inside < 0.0) inside = 0.0;
    return sign * std::sqrt(std::sqrt(inside) - first);
}

// gaussian.h:235-297 — analytic inverse of one Gaussian's optical depth (double).
static bool solve_for_t_given_tau(const Gaussian& g, const Ray& ray, float t0, float tb, float target_tau, float& t_out) {
    V3 p = ray.origin - g.mean;
    V3 Md = mul(g.inv_cov, ray.direction);
    V3 Mp = mul(g.inv_cov, p);
    double A = double(dot(ray.direction, Md));
    if (!(A > 0.0) || !std::isfinite(A)) return false;
    double B = 2.0 * double(dot(p, Md));
    double C = double(dot(p, Mp));
    double sqrtA = std::sqrt(A);
    double pref = double(g.density) * double(g.norm) * std::sqrt(std::numbers::pi / (2.0 * A));
    double exp_factor = std::exp(-0.5 * (C - (B * B) / (4.0 * A)));
    double denom = pref * exp_factor;
    if (!(denom > 0.0) || !std::isfinite(denom)) return false;
    double two_sqrt2_sqrtA = 2.0 * std::sqrt(2.0) * sqrtA;
    double erf_t0 = std::erf((B + 2.0 * A * double(t0)) / two_sqrt2_sqrtA);
    double target_erf = double(target_tau) / denom + erf_t0;
    constexpr double one_eps = 1.0 - 1e-14;
    if (target_erf >= one_eps) { t_out = tb; return true; }
    if (target_erf <= -one_eps) { t_out = t0; return true; }
    if (!std::isfinite(target_erf)) return false;
    if (target_erf <= -1.0 || target_erf >= 1.0) return false;
    double arg_t = erfinv_approx(target_erf);
    double t_candidate = (two_sqrt2_sqrtA * arg_t - B) / (2.0 * A);
    if (!std::isfinite(t_candidate)) return false;
    if (t_candidate < double(t0) - 1e-6) t_candidate = t0;
    if (t_candidate > double(tb) + 1e-6) t_candidate = tb;
    t_out = float(t_candidate);
    return true;
}

// distance_solvers.h:25-57
static float solve_distance_bisection(const Ray& ray, float ta, float tb, const std::vector<size_t>& act, float target,
                                      const GMM& gmm, int max_iters = 15, float tol = 1e-6f) {
    float a = ta, b = tb;
    for (int i = 0; i < max_iters; ++i) {
        float m = 0.5f * (a + b);
        float tau = 0.0f;
        for (auto idx : act) tau += gmm.gaussians[idx].optical_depth(ray, ta, m);
        float f = tau - target;
        if (std::fabs(f) <= tol) return m;
        if (f < 0.0f) a = m;
        else b = m;
    }
    return 0.5f * (a + b);
}

// distance_solvers.h:62-127
static float solve_distance_newton_raphson(const Ray& ray, float ta, float tb, const std::vector<size_t>& act,
                                           float target_tau, const GMM& gmm, int max_iters = 8, float tol = 1e-6f) {
    float a = ta, b = tb;
    float t = 0.5f * (a + b);
    auto compute_f = [&](float tt) -> float {
        float sum_tau = 0.0f;
        float tt_clamped = std::min(tt, b);
        for (auto idx : act) sum_tau += gmm.gaussians[idx].optical_depth(ray, ta, tt_clamped);
        return sum_tau - target_tau;
    };
    for (int iter = 0; iter < max_iters; ++iter) {
        float f = compute_f(t);
        if (std::fabs(f) <= tol) return std::clamp(t, a, b);
        float h = std::max(1e-5f, (b - a) * 1e-6f);
        float tp = std::min(b, t + h);
        float fp = compute_f(tp);
        float deriv = (fp - f) / (tp - t);
        if (!(deriv > 0.0f) || !std::isfinite(deriv) || std::fabs(deriv) < 1e-12f)
            return solve_distance_bisection(ray, ta, tb, act, target_tau, gmm);
        float t_next = t - f / deriv;
        if (!std::isfinite(t_next) || t_next < a || t_next > b)
            return solve_distance_bisection(ray, ta, tb, act, target_tau, gmm);
        if (std::fabs(t_next - t) <= tol * std::max(1.0f, std::fabs(t))) {
            t = t_next;
            return std::clamp(t, a, b);
        }
        t = t_next;
    }
    return solve_distance_bisection(ray, ta, tb, act, target_tau, gmm);
}

// distance_solvers.h:150-187. The reference selects the solver at compile time (:143-147);
// ANALYTIC_PLUS_NEWTON is the compiled-in mode (:146) and the default here. g_solver picks the
// others for the goldens rendered with them (tests/renders/250_rand_{bisection,newton,uniform}_big).
enum { kSolverAnalyticNewton = 0, kSolverBisection = 1, kSolverNewton = 2, kSolverAnalyticBisection = 3, kSolverUniform = 4 };
static int g_solver = kSolverAnalyticNewton;
// The path being solved (free_flight_pixel): UNIFORM's draw comes from its own PCG32 stream.
static thread_local uint64_t g_uniform_seed = 0;
static thread_local int g_uniform_bounce = 0;
static float solve_distance(const Ray& ray, float ta, float tb, const std::vector<size_t>& act, float remaining_tau,
                            const GMM& gmm) {
    if (g_solver == kSolverUniform) {
        // :132-137 draws rand01() from mt19937(random_device) (rng.h:6-10): not reproducible. Documented
        // deviation (the device does the same): the textbook-PCG32 uniform of stream 2 + bounce of the
        // path's seed derive_path_seed(x, y, si) — unbiased like mt19937, and it leaves the path's own
        // PCG32 stream (stream 1) untouched, as rand01() does.
        PCG32 u(g_uniform_seed, 2u + (uint64_t)g_uniform_bounce);
        return ta + u.uniform_env() * (tb - ta);
    }
    if (g_solver == kSolverBisection) return solve_distance_bisection(ray, ta, tb, act, remaining_tau, gmm);
    if (g_solver == kSolverNewton) return solve_distance_newton_raphson(ray, ta, tb, act, remaining_tau, gmm);
    if (act.size() == 1) {
        float t_analytic = 0.0f;
        if (solve_for_t_given_tau(gmm.gaussians[act[0]], ray, ta, tb, remaining_tau, t_analytic))
            return std::clamp(t_analytic, ta, tb);
    }
    if (g_solver == kSolverAnalyticBisection) return solve_distance_bisection(ray, ta, tb, act, remaining_tau, gmm);
    return solve_distance_newton_raphson(ray, ta, tb, act, remaining_tau, gmm);
}

// gmm.h:128-143
static float evaluate_albedo(const GMM& gmm, const std::vector<size_t>& act, V3 pos) {
    float sum_mu_t = 0.0f, sum_mu_t_alb = 0.0f;
    for (size_t idx : act) {
        float mu_t_i = gmm.gaussians[idx].mu_t(pos);
        sum_mu_t += mu_t_i;
        sum_mu_t_alb += mu_t_i * gmm.gaussians[idx].albedo;
    }
    float a = sum_mu_t_alb / sum_mu_t;
    return std::clamp(a, 0.0f, 1.0f);
}

// gmm.h:517-578 — unsorted, clipped, double-accumulated shadow optical depth on [0, tmax].
static float transmittance_up_to(const GMM& gmm, const Ray& ray, float tmax) {
    if (tmax <= 0.0f) return 1.0f;
    if (gmm.gaussians.empty() || gmm.nodes.empty()) return 1.0f;
    const float inf = std::numeric_limits<float>::infinity();
    double sum = 0.0;
    std::vector<int> stack{0};
    while (!stack.empty()) {
        int ni = stack.back();
        stack.pop_back();
        const GMM::Node& node = gmm.nodes[ni];
        float tmin = GMM::IntersectAABB(ray, node.bmin, node.bmax);
        if (tmin == inf || tmin > tmax) continue;
        if (node.isLeaf()) {
            for (int ii = 0; ii < (int)node.count; ++ii) {
                uint32_t gidx = gmm.indices[node.leftFirst + ii];
                float g_t0, g_t1;
                if (!gmm.gaussians[gidx].intersect_direct(ray, g_t0, g_t1)) continue;
                float a = std::max(0.0f, g_t0);
                float b = std::min(tmax, g_t1);
                if (b > a) sum += gmm.gaussians[gidx].optical_depth(ray, a, b);
            }
        } else {
            int li = (int)node.leftFirst, ri = li + 1;
            float dl = GMM::IntersectAABB(ray, gmm.nodes[li].bmin, gmm.nodes[li].bmax);
            float dr = GMM::IntersectAABB(ray, gmm.nodes[ri].bmin, gmm.nodes[ri].bmax);
            if (dl == inf || dl > tmax) dl = inf;
            if (dr == inf || dr > tmax) dr = inf;
            if (dl > dr) {
                if (dl != inf) stack.push_back(li);
                if (dr != inf) stack.push_back(ri);
            } else {
                if (dr != inf) stack.push_back(ri);
                if (dl != inf) stack.push_back(li);
            }
        }
    }
    return std::exp(-float(sum));
}

// integrator.h:422-498 — MultiScatterGaussians::get_free_flight_distance (double accumulation,
// swap-remove active list). `pos_of` is the index -> list-position map (-1 = absent).
static float free_flight_distance_ms(const Ray& ray, const std::vector<PrimitiveHitEvent>& events, float target_tau,
                                     const GMM& gmm, std::vector<size_t>& act, std::vector<int>& pos_of) {
    double acc_tau = 0.0;
    float t_prev = 0.0f;
    float result = -1.0f;
    for (size_t ev = 0; ev < events.size(); ++ev) {
        float t_evt = events[ev].t;
        double seg_tau = 0.0;
        for (size_t idx : act) seg_tau += gmm.gaussians[idx].optical_depth(ray, t_prev, t_evt);
        if (acc_tau + seg_tau > double(target_tau)) {
            float remaining_tau = float(double(target_tau) - acc_tau);
            result = solve_distance(ray, t_prev, t_evt, act, remaining_tau, gmm);
            break;
        }
        acc_tau += seg_tau;
        size_t g = events[ev].index;
        if (events[ev].entering) {
            if (pos_of[g] < 0) {
                pos_of[g] = (int)act.size();
                act.push_back(g);
            }
        } else if (pos_of[g] >= 0) {
            int p = pos_of[g];
            size_t last = act.back();
            act[p] = last;
            pos_of[last] = p;
            act.pop_back();
            pos_of[g] = -1;
        }
        t_prev = t_evt;
    }
    for (size_t idx : act) pos_of[idx] = -1;  // leave the map clean for the next call
    return result;
}

static float* g_ff_dbg = nullptr;  // debug: first-bounce values of sample 0 per pixel (8 floats)

// integrator.h:300-408 (single scatter, float accumulation, index-ordered active list) when
// multi == false; integrator.h:532-717 (multi-scatter, min_bounces, Russian roulette) otherwise.
static V3 free_flight_pixel(const Scene& scene, const Camera& cam, int x, int y, int W, int H, int num_samples,
                            int min_scatter, bool multi, std::vector<uint32_t>* pixel_list = nullptr) {
    const GMM& gmm = scene.gmm;
    const size_t N = gmm.gaussians.size();
    const float phase_pdf = kInv4Pi;
    const float w_light = float(scene.lights.size() + 1);
    std::vector<PrimitiveHitEvent> events;
    std::vector<size_t> act;
    std::vector<int> pos_of(N, -1);
    std::vector<bool> active(N, false);
    V3 pixel_L{0, 0, 0};
    const int n = int(std::sqrt(num_samples));
    for (int si = 0; si < num_samples; ++si) {
        PCG32 rng(derive_path_seed(x, y, si), 1);
        g_uniform_seed = derive_path_seed(x, y, si);
        int sx = si % n, sy = si / n;
        float u = (x + (sx + rng.uniform()) / n) / W;
        float v = (y + (sy + rng.uniform()) / n) / H;
        Ray ray = cam.sample_ray(u, v);
        V3 throughput{1, 1, 1}, L_accum{0, 0, 0};
        for (int bounce = 0;; ++bounce) {
            g_uniform_bounce = bounce;
            gmm.intersect_events(ray, events);
            if (events.empty()) {
                L_accum = L_accum + V3{throughput.x * scene.env_color.x, throughput.y * scene.env_color.y,
                                       throughput.z * scene.env_color.z};
                break;
            }
            float target_tau = -std::log(1.0f - rng.uniform());
            float t_scatter = -1.0f;
            act.clear();
            if (multi) {
                t_scatter = free_flight_distance_ms(ray, events, target_tau, gmm, act, pos_of);
            } else {  // integrator.h:330-360
                std::fill(active.begin(), active.end(), false);
                float acc_tau = 0.0f, t_prev = 0.0f;
                for (size_t ev = 0; ev < events.size(); ++ev) {
                    float t_evt = events[ev].t;
                    act.clear();
                    for (size_t i = 0; i < N; ++i)
                        if (active[i]) act.push_back(i);
                    float seg_tau = 0.0f;
                    for (auto idx : act) seg_tau += gmm.gaussians[idx].optical_depth(ray, t_prev, t_evt);
                    if (acc_tau + seg_tau > target_tau) {
                        t_scatter = solve_distance(ray, t_prev, t_evt, act, target_tau - acc_tau, gmm);
                        break;
                    }
                    acc_tau += seg_tau;
                    active[events[ev].index] = events[ev].entering;
                    t_prev = t_evt;
                }
            }
            if (pixel_list && multi) {  // RECORD_PIXEL_GAUSSIANS, integrator.h:616-644
                auto add = [&](uint32_t g) {
                    if (std::find(pixel_list->begin(), pixel_list->end(), g) == pixel_list->end()) pixel_list->push_back(g);
                };
                const float tol = 1e-6f;
                if (t_scatter >= 0.0f) {
                    for (const auto& ev : events) {
                        if (ev.t <= t_scatter + tol) add((uint32_t)ev.index);
                        else break;
                    }
                } else {
                    for (const auto& ev : events)
                        if (!(ev.t < 0.0f)) add((uint32_t)ev.index);
                }
            }
            if (t_scatter < 0.0f) {
                L_accum = L_accum + V3{throughput.x * scene.env_color.x, throughput.y * scene.env_color.y,
                                       throughput.z * scene.env_color.z};
                break;
            }
            V3 pos = ray.origin + t_scatter * ray.direction;
            float albedo = evaluate_albedo(gmm, act, pos);
            bool is_env = (rng.uniform() < 1.0f / (scene.lights.size() + 1));
            V3 Li{0, 0, 0};
            if (!is_env) {
                int li = int(rng.uniform() * scene.lights.size());
                const Light& Lt = scene.lights[li];
                V3 wi = normalized(Lt.position - pos);
                float dist = norm(Lt.position - pos);
                Ray shadow(pos, wi);
                float Tr = transmittance_up_to(gmm, shadow, dist);
                float d2 = dist * dist;
                Li = V3{(Tr * Lt.intensity.x) / d2, (Tr * Lt.intensity.y) / d2, (Tr * Lt.intensity.z) / d2};
            } else {
                V3 wi = sample_uniform_direction(rng);
                Ray eray(pos, wi);
                float Tr = transmittance_up_to(gmm, eray, std::numeric_limits<float>::infinity());
                Li = V3{(Tr * scene.env_color.x) * k4Pi, (Tr * scene.env_color.y) * k4Pi, (Tr * scene.env_color.z) * k4Pi};
            }
            if (g_ff_dbg && si == 0 && bounce == 0) {
                float* d = g_ff_dbg + ((size_t)y * W + x) * 8;
                d[0] = target_tau, d[1] = t_scatter, d[2] = albedo, d[3] = is_env ? 0.0f : Li.x, d[4] = pos.x, d[5] = pos.y,
                d[6] = pos.z, d[7] = is_env ? 1.0f : 0.0f;
            }
            if (!multi) {  // integrator.h:396-399
                float w = (albedo * phase_pdf) * w_light;
                L_accum = V3{w * Li.x, w * Li.y, w * Li.z};
                break;
            }
            float w = (albedo * phase_pdf) * w_light;  // integrator.h:682-687
            L_accum = L_accum + V3{(throughput.x * w) * Li.x, (throughput.y * w) * Li.y, (throughput.z * w) * Li.z};
            throughput = V3{throughput.x * albedo, throughput.y * albedo, throughput.z * albedo};
            if (bounce >= min_scatter) {  // integrator.h:691-695
                float rr = std::min(std::max(throughput.x, std::max(throughput.y, throughput.z)), 0.9f);
                if (rng.uniform() > rr) break;
                throughput = V3{throughput.x / rr, throughput.y / rr, throughput.z / rr};
            }
            V3 new_dir = sample_uniform_direction(rng);
            ray = Ray(pos, new_dir);
        }
        pixel_L = pixel_L + L_accum;
    }
    float fs = float(num_samples);
    return V3{pixel_L.x / fs, pixel_L.y / fs, pixel_L.z / fs};
}

}  // namespace orc

// =============================================================================================
// C ABI for ctypes (tests / bench cpu_baseline only)
// =============================================================================================
using namespace orc;
static thread_local std::string g_err;

extern "C" {

const char* orc_last_error() { return g_err.c_str(); }

void* orc_load_gmm(const char* path) {
    try { return new Scene(load_GMM(path)); } catch (const std::exception& e) { g_err = e.what(); return nullptr; }
}
void* orc_load_smm(const char* path) {
    try { return new Scene(load_SMM(path)); } catch (const std::exception& e) { g_err = e.what(); return nullptr; }
}
// n Gaussians: mean[3n], cov6[6n] (xx xy xz yy yz zz), density[n], albedo[n]; lights pos[3nl], int[3nl]
void* orc_scene_from_gaussians(int64_t n, const float* mean, const float* cov6, const float* density,
                               const float* albedo, int64_t nl, const float* lpos, const float* lint) {
    Scene* s = new Scene();
    s->volume_type = 0;
    s->gmm.gaussians.reserve(n);
    for (int64_t i = 0; i < n; ++i) {
        const float* c = cov6 + 6 * i;
        M3 cov{{{c[0], c[1], c[2]}, {c[1], c[3], c[4]}, {c[2], c[4], c[5]}}};
        s->gmm.gaussians.emplace_back(V3{mean[3 * i], mean[3 * i + 1], mean[3 * i + 2]}, cov, density[i], albedo[i]);
    }
    for (int64_t i = 0; i < nl; ++i)
        s->lights.push_back({{lpos[3 * i], lpos[3 * i + 1], lpos[3 * i + 2]}, {lint[3 * i], lint[3 * i + 1], lint[3 * i + 2]}});
    s->gmm.BuildBVH();
    return s;
}
void orc_scene_free(void* s) { delete (Scene*)s; }
void orc_scene_set_env(void* s, float r, float g, float b) { ((Scene*)s)->env_color = {r, g, b}; }
int64_t orc_scene_num(void* s) { return (int64_t)((Scene*)s)->num(); }
int64_t orc_scene_num_lights(void* s) { return (int64_t)((Scene*)s)->lights.size(); }
int orc_scene_type(void* s) { return ((Scene*)s)->volume_type; }
// per Gaussian 12 floats: mean3, density, inv_cov(00 01 02 11 12 22), norm, albedo
void orc_scene_records(void* sp, float* out) {
    Scene* s = (Scene*)sp;
    for (size_t i = 0; i < s->gmm.gaussians.size(); ++i) {
        const Gaussian& g = s->gmm.gaussians[i];
        float* o = out + 12 * i;
        o[0] = g.mean.x; o[1] = g.mean.y; o[2] = g.mean.z; o[3] = g.density;
        o[4] = g.inv_cov(0, 0); o[5] = g.inv_cov(0, 1); o[6] = g.inv_cov(0, 2);
        o[7] = g.inv_cov(1, 1); o[8] = g.inv_cov(1, 2); o[9] = g.inv_cov(2, 2);
        o[10] = g.norm; o[11] = g.albedo;
    }
}
// camera: type 0 pinhole (pos, view_dir, fov), 1 ortho (pos, forward). out[17]:
// type, position3, view_dir3, right3, up3, pinhole3, focal
void orc_camera(int type, const float* pos, const float* vd, float fov, float* out) {
    Camera c = type == 0 ? Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov)
                         : Camera::make_ortho({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]});
    float v[17] = {(float)c.type, c.position.x, c.position.y, c.position.z, c.view_dir.x, c.view_dir.y, c.view_dir.z,
                   c.right.x, c.right.y, c.right.z, c.up.x, c.up.y, c.up.z, c.pinhole.x, c.pinhole.y, c.pinhole.z, c.focal_length};
    std::memcpy(out, v, sizeof(v));
}
// primary ray for pixel (x,y): out[6] origin, direction
void orc_primary_ray(int type, const float* pos, const float* vd, float fov, int x, int y, int W, int H, float* out) {
    Camera c = type == 0 ? Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov)
                         : Camera::make_ortho({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]});
    float u = (x + 0.5f) / W, v = (y + 0.5f) / H;
    Ray r = c.sample_ray(u, v);
    out[0] = r.origin.x; out[1] = r.origin.y; out[2] = r.origin.z;
    out[3] = r.direction.x; out[4] = r.direction.y; out[5] = r.direction.z;
}
// Gaussian i vs a ray: out[4] = hit, t_enter, t_exit, optical_depth(t_enter, t_exit)
void orc_gaussian_probe(void* sp, int64_t i, const float* o, const float* d, float* out) {
    Scene* s = (Scene*)sp;
    Ray r{{o[0], o[1], o[2]}, {d[0], d[1], d[2]}};
    const Gaussian& g = s->gmm.gaussians[i];
    float a = 0, b = 0;
    bool hit = g.intersect_direct(r, a, b);
    out[0] = hit ? 1.0f : 0.0f; out[1] = a; out[2] = b;
    out[3] = hit ? g.optical_depth(r, a, b) : 0.0f;
}

// DEBUG: for pixel (x,y) of RayMarchingGaussians, compare every secondary-ray transmittance of the
// faithful segment loop with the telescoped per-Gaussian-interval model used by the device code.
// out[0] = max |Tr_ref - Tr_model| (light rays), out[1] = same (env rays), out[2] = #rays checked,
// out[3..6] = (step k, ray kind 0/1, Tr_ref, Tr_model) of the worst ray.
void orc_debug_secondary(void* sp, const float* pos, const float* vd, float fov, int x, int y, int W, int H,
                         float step_size, int env_samples, float* out) {
    Scene& s = *(Scene*)sp;
    const GMM& gmm = s.gmm;
    Camera c = Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov);
    float u = (x + 0.5f) / W, v = (y + 0.5f) / H;
    Ray ray = c.sample_ray(u, v);
    std::vector<PrimitiveHitEvent> events;
    gmm.intersect_events(ray, events);
    for (int i = 0; i < 7; ++i) out[i] = 0;
    if (events.empty()) return;
    float t_end = events.back().t;
    std::vector<bool> active(gmm.gaussians.size(), false);
    size_t evt_i = 0;
    float t = 0.0f;
    int k = 0;
    auto model = [&](const Ray& r, bool is_light, float dist) {
        // telescoped model
        std::vector<PrimitiveHitEvent> ev;
        gmm.intersect_events(r, ev);
        std::vector<float> lo(gmm.gaussians.size(), NAN), hi(gmm.gaussians.size(), NAN);
        std::vector<bool> hit(gmm.gaussians.size(), false);
        for (size_t i = 0; i < gmm.gaussians.size(); ++i) {
            float a, b;
            if (gmm.gaussians[i].intersect_direct(r, a, b)) { hit[i] = true; lo[i] = a; hi[i] = b; }
        }
        float tstop;
        if (is_light) {
            tstop = INFINITY;
            for (auto& e : ev) if (e.t >= dist) tstop = std::min(tstop, e.t);
            if (tstop == INFINITY) tstop = dist;
        } else {
            tstop = 0.0f;
            for (auto& e : ev) tstop = std::max(tstop, e.t);
        }
        double tau = 0;
        for (size_t i = 0; i < gmm.gaussians.size(); ++i) {
            float l, h;
            if (active[i]) { l = 0.0f; h = hit[i] ? hi[i] : tstop; }
            else if (hit[i]) { l = lo[i]; h = hi[i]; }
            else continue;
            h = std::min(h, tstop);
            if (l < h) tau += gmm.gaussians[i].optical_depth(r, l, h);
        }
        return (float)std::exp(-tau);
    };
    int nrays = 0;
    while (t < t_end) {
        while (evt_i < events.size() && events[evt_i].t <= t) {
            active[events[evt_i].index] = events[evt_i].entering;
            ++evt_i;
        }
        V3 p = ray.origin + t * ray.direction;
        float sa, ss;
        gmm.evaluate_sigma(active, p, sa, ss);
        if (ss > 0.0f) {
            for (const auto& light : s.lights) {
                V3 wi = normalized(light.position - p);
                float dist = norm(light.position - p);
                Ray sr(p, wi);
                std::vector<PrimitiveHitEvent> sev;
                gmm.intersect_events(sr, sev);
                for (size_t i = 0; i < active.size(); ++i) if (active[i]) sev.insert(sev.begin(), {0.0f, true, i});
                std::vector<size_t> ai;
                std::vector<bool> mask = active;
                float tp = 0, Tr = 1.0f;
                size_t se = 0;
                while (tp < dist) {
                    float tn = se < sev.size() ? sev[se].t : dist;
                    ai.clear();
                    for (size_t i = 0; i < mask.size(); ++i) if (mask[i]) ai.push_back(i);
                    Tr *= gmm.transmittance_over_segment(sr, tp, tn, ai);
                    if (se < sev.size()) { mask[sev[se].index] = sev[se].entering; ++se; }
                    tp = tn;
                }
                float Tm = model(sr, true, dist);
                float d = std::fabs(Tr - Tm);
                ++nrays;
                if (d > out[0]) out[0] = d;
                if (d >= out[0] && d > 0 && d >= out[1]) { out[3] = k; out[4] = 0; out[5] = Tr; out[6] = Tm; }
            }
            PCG32 rng(derive_path_seed(x, y, k), 1);
            for (int si = 0; si < env_samples; ++si) {
                float xi1 = rng.uniform_env(), xi2 = rng.uniform_env();
                Ray er(p, env_dir(xi1, xi2));
                std::vector<PrimitiveHitEvent> eev;
                gmm.intersect_events(er, eev);
                for (size_t i = 0; i < active.size(); ++i) if (active[i]) eev.insert(eev.begin(), {0.0f, true, i});
                std::vector<size_t> ai;
                std::vector<bool> mask = active;
                float tp = 0, Tr = 1.0f;
                for (size_t ei = 0; ei < eev.size(); ++ei) {
                    float tn = eev[ei].t;
                    ai.clear();
                    for (size_t i = 0; i < mask.size(); ++i) if (mask[i]) ai.push_back(i);
                    Tr *= gmm.transmittance_over_segment(er, tp, tn, ai);
                    mask[eev[ei].index] = eev[ei].entering;
                    tp = tn;
                }
                float Tm = model(er, false, 0.0f);
                float d = std::fabs(Tr - Tm);
                ++nrays;
                if (d > out[1]) { out[1] = d; if (d >= out[0]) { out[3] = k; out[4] = 1; out[5] = Tr; out[6] = Tm; } }
            }
        }
        t += step_size;
        ++k;
    }
    out[2] = nrays;
}

uint64_t orc_derive_path_seed(int x, int y, int si) { return derive_path_seed(x, y, si); }
void orc_pcg32(uint64_t seed, uint64_t seq, int n, uint32_t* out) {
    PCG32 r(seed, seq);
    for (int i = 0; i < n; ++i) out[i] = r.next_u32();
}
void orc_env_dir(float xi1, float xi2, float* out) {
    V3 d = env_dir(xi1, xi2);
    out[0] = d.x; out[1] = d.y; out[2] = d.z;
}

// integrator: 0 RayMarchingGaussians, 1 RayMarchingSpheres, 2 RayMarchingGaussians with sorted
// active lists + stop at T == 0 (bit-identical to 0; bench.py's CPU baseline), 3 PureRayMarching.
// If pix != nullptr, render only the npix pixels pix[2k]=x, pix[2k+1]=y into out[3*npix];
// otherwise the whole W*H frame into out[3*W*H] (row-major, image.h:13-17).
int orc_render(void* sp, int cam_type, const float* pos, const float* vd, float fov, int integrator,
               float step_size, int env_samples, int W, int H, const int* pix, int64_t npix, float* out,
               int nthreads) {
    try {
        Scene* s = (Scene*)sp;
        Camera c = cam_type == 0 ? Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov)
                                 : Camera::make_ortho({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]});
        if (integrator < 0 || integrator > 3) { g_err = "unknown integrator"; return 1; }
        if ((integrator != 1) != (s->volume_type == 0)) { g_err = "integrator/scene type mismatch"; return 1; }
        int64_t total = pix ? npix : (int64_t)W * H;
        if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t q = 0; q < total; ++q) {
            int x = pix ? pix[2 * q] : (int)(q % W);
            int y = pix ? pix[2 * q + 1] : (int)(q / W);
            g_ties = 0;
            V3 L = integrator == 0   ? rm_gaussians_pixel(*s, c, x, y, W, H, step_size, env_samples)
                   : integrator == 2 ? rm_gaussians_pixel_lists(*s, c, x, y, W, H, step_size, env_samples)
                   : integrator == 3 ? rm_pure_pixel(*s, c, x, y, W, H, step_size, env_samples)
                                     : rm_spheres_pixel(*s, c, x, y, W, H, step_size, env_samples);
            out[3 * q] = L.x; out[3 * q + 1] = L.y; out[3 * q + 2] = L.z;
            if (g_tie_out) g_tie_out[q] = (int32_t)std::min<int64_t>(g_ties, INT32_MAX);
        }
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return 2;
    }
}

void orc_ff_debug(float* buf) { g_ff_dbg = buf; }
// SURVEY.md §8(d) algorithmic bytes, step 1: each pixel's primary-ray termination distance under
// the RayMarchingGaussians march (test_integrators.h:178-290, the list variant's active sets, no
// secondary rays): the end of the first step after which T <= t_eps, or t_end (the last event) if T
// never falls that far; -1 for a ray without events. depth[y * W + x].
int orc_primary_depths(void* sp, int cam_type, const float* pos, const float* vd, float fov, int W, int H,
                       float step_size, float t_eps, float* depth, int nthreads) {
    const Scene& s = *(const Scene*)sp;
    const GMM& gmm = s.gmm;
    Camera c = cam_type == 0 ? Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov)
                             : Camera::make_ortho({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]});
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t q = 0; q < (int64_t)W * H; ++q) {
        static thread_local std::vector<uint8_t> mask;
        if (mask.size() != gmm.gaussians.size()) mask.assign(gmm.gaussians.size(), 0);
        const int x = (int)(q % W), y = (int)(q / W);
        Ray ray = c.sample_ray((x + 0.5f) / W, (y + 0.5f) / H);
        std::vector<PrimitiveHitEvent> events;
        gmm.intersect_events(ray, events);
        if (events.empty()) { depth[q] = -1.0f; continue; }
        const float t_end = events.back().t;
        SparseSet active{&mask, {}};
        size_t evt_i = 0;
        float t = 0.0f, T = 1.0f, d = t_end;
        while (t < t_end) {
            while (evt_i < events.size() && events[evt_i].t <= t) {
                active.set(events[evt_i].index, events[evt_i].entering);
                ++evt_i;
            }
            T *= gmm.transmittance_over_segment(ray, t, t + step_size, active.list);
            t += step_size;
            if (T <= t_eps) { d = t; break; }
        }
        active.clear();
        depth[q] = d;
    }
    return 0;
}

// SURVEY.md §8(d) algorithmic bytes, step 2: per 16x16 tile, n_t = the Gaussians whose conservative
// 3-sigma box (gaussian.h:304-319) overlaps the tile's frustum and whose conservative near depth is
// <= D_t (the largest termination distance of the tile's rays, orc_primary_depths). Pinhole camera:
// every ray of the tile passes through the pinhole, so the frustum is the pyramid from the pinhole
// through the tile's four outer pixel-corner rays; a ray reaches the pinhole at t >= focal length
// (the sensor plane's distance), so a box's near depth is >= f + |box - pinhole|. The query walks
// the oracle's BVH. n_tiles[t] for row-major tiles; returns the sum of n_t.
int64_t orc_tile_bins(void* sp, const float* pos, const float* vd, float fov, int W, int H, const float* depth,
                      uint32_t* n_tiles, int nthreads) {
    const Scene& s = *(const Scene*)sp;
    const GMM& gmm = s.gmm;
    Camera c = Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov);
    const int tx = (W + 15) / 16, ty = (H + 15) / 16;
    const V3 apex = c.pinhole;
    int64_t total = 0;
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : total)
    for (int64_t t = 0; t < (int64_t)tx * ty; ++t) {
        const int x0 = (int)(t % tx) * 16, y0 = (int)(t / tx) * 16;
        const int x1 = std::min(x0 + 16, W), y1 = std::min(y0 + 16, H);
        float D = -1.0f;
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) D = std::max(D, depth[(int64_t)y * W + x]);
        n_tiles[t] = 0;
        if (D < 0.0f || gmm.nodes.empty()) continue;
        V3 dir[4];  // outer corner rays, counter-clockwise
        const double cu[4] = {(double)x0 / W, (double)x1 / W, (double)x1 / W, (double)x0 / W};
        const double cv[4] = {(double)y0 / H, (double)y0 / H, (double)y1 / H, (double)y1 / H};
        V3 centre{0, 0, 0};
        for (int k = 0; k < 4; ++k) {
            dir[k] = c.sample_ray(cu[k], cv[k]).direction;
            centre = centre + dir[k];
        }
        V3 nrm[4];  // side planes through the apex, normals pointing into the pyramid
        for (int k = 0; k < 4; ++k) {
            V3 n = cross(dir[k], dir[(k + 1) % 4]);
            if (dot(n, centre) < 0.0f) n = V3{-n.x, -n.y, -n.z};
            nrm[k] = n;
        }
        const float limit = D - c.focal_length;  // |box - apex| must not exceed this
        auto overlaps = [&](const V3& bmin, const V3& bmax) {
            double d2 = 0.0;  // squared distance apex -> box
            for (int k = 0; k < 3; ++k) {
                const double v = std::max({(double)bmin[k] - apex[k], 0.0, (double)apex[k] - bmax[k]});
                d2 += v * v;
            }
            if (d2 > (double)limit * limit * (1.0 + 1e-6) + 1e-12 && limit >= 0.0f) return false;
            if (limit < 0.0f) return false;
            for (int k = 0; k < 4; ++k) {  // box entirely outside one side plane -> no overlap
                const V3& n = nrm[k];
                const V3 p{n.x >= 0 ? bmax.x : bmin.x, n.y >= 0 ? bmax.y : bmin.y, n.z >= 0 ? bmax.z : bmin.z};
                if (dot(n, p - apex) < 0.0f) return false;
            }
            return true;
        };
        uint32_t cnt = 0;
        std::vector<uint32_t> stack{0};
        while (!stack.empty()) {
            const GMM::Node& nd = gmm.nodes[stack.back()];
            stack.pop_back();
            if (!overlaps(nd.tbmin, nd.tbmax)) continue;
            if (nd.isLeaf()) {
                for (uint32_t i = 0; i < nd.count; ++i) {
                    const Gaussian& g = gmm.gaussians[gmm.indices[nd.leftFirst + i]];
                    if (overlaps(g.tbmin, g.tbmax)) ++cnt;
                }
            } else {
                stack.push_back(nd.leftFirst);
                stack.push_back(nd.leftFirst + 1);
            }
        }
        n_tiles[t] = cnt;
        total += cnt;
    }
    return total;
}

// DEBUG: the faithful RayMarchingGaussians march of one pixel; out gets, per step with a non-empty
// active set, (t, n_active, sigma_s, T after the step, active ids...). Returns the floats written.
// DEBUG: the scattering steps of pixel (x, y) of RayMarchingGaussians (sparse-list restatement, pinhole), one
// row of 9 + nlights + env_samples floats each (see g_rec_trace); the device side is vr_debug_pixel_records.
// Returns the number of rows (writes at most cap).
int64_t orc_debug_pixel_records(void* sp, const float* pos, const float* vd, float fov, int x, int y, int W, int H,
                                float step_size, int env_samples, float* out, int64_t cap) {
    Scene& s = *(Scene*)sp;
    Camera c = Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov);
    std::vector<float> tr;
    g_rec_trace = &tr;
    rm_gaussians_pixel_lists(s, c, x, y, W, H, step_size, env_samples);
    g_rec_trace = nullptr;
    const size_t row = 9 + s.lights.size() + (size_t)env_samples;
    const int64_t n = (int64_t)(tr.size() / row);
    std::copy(tr.begin(), tr.begin() + (size_t)std::min(n, cap) * row, out);
    return n;
}

// DEBUG: the active list (scene indices) of the scattering step k of pixel (x, y) (see orc_debug_pixel_records);
// returns its length (-1: no such step).
int64_t orc_debug_record_active(void* sp, const float* pos, const float* vd, float fov, int x, int y, int W, int H,
                                float step_size, int env_samples, int k, int64_t* out, int64_t cap) {
    Scene& s = *(Scene*)sp;
    Camera c = Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov);
    std::vector<float> tr, act;
    g_rec_trace = &tr;
    g_rec_active = &act;
    rm_gaussians_pixel_lists(s, c, x, y, W, H, step_size, env_samples);
    g_rec_trace = nullptr;
    g_rec_active = nullptr;
    const size_t row = 9 + s.lights.size() + (size_t)env_samples;
    size_t a = 0;
    for (size_t r = 0; r * row < tr.size(); ++r) {
        const int64_t n = (int64_t)act[a];
        if ((int)tr[r * row] == k) {
            for (int64_t i = 0; i < n && i < cap; ++i) out[i] = (int64_t)act[a + 1 + i];
            return n;
        }
        a += 1 + (size_t)n;
    }
    return -1;
}

// DEBUG: one secondary ray of RayMarchingGaussians (test_integrators.h:202-271, the restatement's segment loop)
// from origin o along d (normalised by the Ray constructor) with the primary active set `pre` pre-activated;
// is_light: a light at distance dist. Per Gaussian ever active on the ray, a row (index, pre-activated,
// M-form hit, t0, t1, optical depth it contributed over the ray's segments (double)); out_tr[0] = the ray's Tr.
// Returns the row count (writes at most cap).
int64_t orc_debug_secondary_ray(void* sp, const float* o, const float* d, int is_light, float dist, const int64_t* pre,
                                int64_t npre, float* out, int64_t cap, float* out_tr) {
    Scene& s = *(Scene*)sp;
    const GMM& gmm = s.gmm;
    Ray r({o[0], o[1], o[2]}, {d[0], d[1], d[2]});
    std::vector<PrimitiveHitEvent> ev;
    gmm.intersect_events(r, ev);
    std::map<size_t, double> contrib;
    std::vector<size_t> act;  // ascending
    for (int64_t i = 0; i < npre; ++i) act.push_back((size_t)pre[i]);
    std::sort(act.begin(), act.end());
    for (size_t i : act) ev.insert(ev.begin(), {0.0f, true, i});
    auto set = [&](size_t i, bool on) {
        auto it = std::lower_bound(act.begin(), act.end(), i);
        const bool has = it != act.end() && *it == i;
        if (on && !has) act.insert(it, i);
        if (!on && has) act.erase(it);
    };
    float t_prev = 0.0f, Tr = 1.0f;
    size_t ei = 0;
    auto segment = [&](float t_next) {
        float sum = 0.0f;
        for (size_t i : act) {
            const float od = gmm.gaussians[i].optical_depth(r, t_prev, t_next);
            contrib[i] += (double)od;
            sum += od;
        }
        Tr *= std::exp(-sum);
    };
    if (is_light) {
        while (t_prev < dist) {
            const float t_next = ei < ev.size() ? ev[ei].t : dist;
            segment(t_next);
            if (ei < ev.size()) { set(ev[ei].index, ev[ei].entering); ++ei; }
            t_prev = t_next;
        }
    } else {
        while (ei < ev.size()) {
            const float t_next = ev[ei].t;
            segment(t_next);
            set(ev[ei].index, ev[ei].entering);
            t_prev = t_next;
            ++ei;
        }
    }
    out_tr[0] = Tr;
    int64_t n = 0;
    for (auto& [i, od] : contrib) {
        if (n < cap) {
            float a = NAN, b = NAN;
            const bool hit = gmm.gaussians[i].intersect_direct(r, a, b);
            const bool is_pre = std::binary_search(pre, pre + npre, (int64_t)i) || std::find(pre, pre + npre, (int64_t)i) != pre + npre;
            float* row = out + 6 * n;
            row[0] = (float)i; row[1] = is_pre ? 1.0f : 0.0f; row[2] = hit ? 1.0f : 0.0f; row[3] = a; row[4] = b; row[5] = (float)od;
        }
        ++n;
    }
    return n;
}

int64_t orc_debug_march(void* sp, const float* pos, const float* vd, float fov, int x, int y, int W, int H,
                        float step_size, int env_samples, float* L_out, float* out, int64_t cap) {
    Scene& s = *(Scene*)sp;
    Camera c = Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov);
    std::vector<float> tr;
    g_rm_trace = &tr;
    V3 L = rm_gaussians_pixel(s, c, x, y, W, H, step_size, env_samples);
    g_rm_trace = nullptr;
    L_out[0] = L.x; L_out[1] = L.y; L_out[2] = L.z;
    for (int64_t i = 0; i < (int64_t)tr.size() && i < cap; ++i) out[i] = tr[i];
    return (int64_t)tr.size();
}
// distance solver of the free-flight integrators (see solve_distance); returns the previous one
int orc_set_solver(int mode) { int o = g_solver; g_solver = mode; return o; }
// event-sort tie order: 0 = the reference's std::sort (default), 1 = stable (see g_stable_ties)
int orc_set_stable_ties(int on) { int o = g_stable_ties; g_stable_ties = on != 0; return o; }
// secondary-ray chords: 0 = the reference's f32 forms (default), 1 = double (see g_accurate_chords)
// DEBUG: orc_render writes each pixel's count of tangent-hit ties (over all its rays) into buf (NULL: off).
void orc_tie_flags(int32_t* buf) { g_tie_out = buf; }
int orc_set_padded_boxes(int on) { int o = g_padded_boxes; g_padded_boxes = on != 0; return o; }
int orc_set_accurate_chords(int on) { int o = g_accurate_chords; g_accurate_chords = on != 0; return o; }
// PCG32 output rotation: 0 = the reference's rng.h:43 (default), 1 = textbook PCG32 (see PCG32)
int orc_set_pcg_textbook(int on) { int o = g_pcg_textbook; g_pcg_textbook = on != 0; return o; }

// MultiScatterGaussians::render with RECORD_PIXEL_GAUSSIANS (integrator.h:532-536, 616-644): the
// frame into out[3*W*H] and the per-pixel Gaussian sets into bits[(g >> 5) * W*H + p] (bit g & 31).
int orc_render_ms_record(void* sp, int cam_type, const float* pos, const float* vd, float fov, int num_samples,
                         int min_bounces, int W, int H, float* out, uint32_t* bits, int nthreads) {
    try {
        Scene* s = (Scene*)sp;
        if (s->volume_type != 0) { g_err = "free-flight integrators need a Gaussian scene"; return 1; }
        Camera c = cam_type == 0 ? Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov)
                                 : Camera::make_ortho({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]});
        const int64_t total = (int64_t)W * H;
        if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t q = 0; q < total; ++q) {
            int x = (int)(q % W), y = (int)(q / W);
            std::vector<uint32_t> list;
            V3 L = free_flight_pixel(*s, c, x, y, W, H, num_samples, min_bounces, true, &list);
            out[3 * q] = L.x; out[3 * q + 1] = L.y; out[3 * q + 2] = L.z;
            for (uint32_t g : list) bits[(size_t)(g >> 5) * total + q] |= 1u << (g & 31u);
        }
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return 2;
    }
}

// orc_render_ms_record on the pixels pix[2 q], pix[2 q + 1] only (q < npix): out (npix x 3) and bits
// ((N + 31) / 32 rows of npix words). bench.py's CPU baseline of an SFD iteration times these on a pixel sample.
int orc_render_ms_record_px(void* sp, int cam_type, const float* pos, const float* vd, float fov, int num_samples,
                            int min_bounces, int W, int H, const int* pix, int64_t npix, float* out, uint32_t* bits,
                            int nthreads) {
    try {
        Scene* s = (Scene*)sp;
        if (s->volume_type != 0) { g_err = "free-flight integrators need a Gaussian scene"; return 1; }
        Camera c = cam_type == 0 ? Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov)
                                 : Camera::make_ortho({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]});
        if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t q = 0; q < npix; ++q) {
            std::vector<uint32_t> list;
            V3 L = free_flight_pixel(*s, c, pix[2 * q], pix[2 * q + 1], W, H, num_samples, min_bounces, true, &list);
            out[3 * q] = L.x; out[3 * q + 1] = L.y; out[3 * q + 2] = L.z;
            for (uint32_t g : list) bits[(size_t)(g >> 5) * npix + q] |= 1u << (g & 31u);
        }
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return 2;
    }
}

// FreeFlightGaussians (multi = 0, integrator.h:300-408) / MultiScatterGaussians (multi = 1,
// integrator.h:532-717). Same pixel selection and output convention as orc_render.
int orc_render_ff(void* sp, int cam_type, const float* pos, const float* vd, float fov, int multi, int num_samples,
                  int min_bounces, int W, int H, const int* pix, int64_t npix, float* out, int nthreads) {
    try {
        Scene* s = (Scene*)sp;
        if (s->volume_type != 0) { g_err = "free-flight integrators need a Gaussian scene"; return 1; }
        if (num_samples <= 0) { g_err = "num_samples must be > 0"; return 1; }
        Camera c = cam_type == 0 ? Camera::make_pinhole({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]}, fov)
                                 : Camera::make_ortho({pos[0], pos[1], pos[2]}, {vd[0], vd[1], vd[2]});
        int64_t total = pix ? npix : (int64_t)W * H;
        if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t q = 0; q < total; ++q) {
            int x = pix ? pix[2 * q] : (int)(q % W);
            int y = pix ? pix[2 * q + 1] : (int)(q / W);
            V3 L = free_flight_pixel(*s, c, x, y, W, H, num_samples, min_bounces, multi != 0);
            out[3 * q] = L.x; out[3 * q + 1] = L.y; out[3 * q + 2] = L.z;
        }
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return 2;
    }
}

}  // extern "C"
