// Synthetic Gaussian scenes with the distribution of the reference's scene generators
// (tests/make_random.py:21-45, tests/make_nonuniform_random.py:19-30). Used for the C3/C4
// benchmark configurations (100k / 1M Gaussians), which have no scene file in the reference.
#include <cmath>

#include "vr_common.h"

using namespace vr;

namespace {

struct Pcg {  // rng.h:20-50 PCG32 (same non-standard output rotation)
    uint64_t state, inc;
    Pcg(uint64_t seed_state, uint64_t seed_seq) {
        state = 0;
        inc = (seed_seq << 1) | 1;
        next();
        state += seed_state;
        next();
    }
    uint32_t next() {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t shifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (shifted >> rot) | (shifted << ((-rot + 1u) & 31));
    }
    double uniform() {  // [0, 1), 53 bits
        uint64_t hi = next() >> 5, lo = next() >> 6;
        return (double)(hi * 67108864ull + lo) * (1.0 / 9007199254740992.0);
    }
    double uniform(double a, double b) { return a + (b - a) * uniform(); }
    double normal() {  // Box-Muller
        double u1 = uniform(), u2 = uniform();
        if (u1 < 1e-300) u1 = 1e-300;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
    }
};

inline float printed(double v, double scale) { return (float)(std::nearbyint(v * scale) / scale); }

}  // namespace

extern "C" vr_status vr_scene_add_random_gaussians(vr_scene* s, uint64_t n, uint64_t seed, int32_t variant) {
    if (!s) return fail(VR_ERR_INVALID, "vr_scene_add_random_gaussians: NULL scene");
    if (s->s.type != VR_VOLUME_GAUSSIANS) return fail(VR_ERR_INVALID, "vr_scene_add_random_gaussians: not a Gaussian scene");
    if (variant != 0 && variant != 1) return fail(VR_ERR_INVALID, "vr_scene_add_random_gaussians: variant must be 0 or 1");
    if (n > (1ull << 27)) return fail(VR_ERR_UNSUPPORTED, "vr_scene_add_random_gaussians: too many Gaussians");
    Pcg rng(seed, 0x5eed5eedull);
    s->s.gaussians.reserve(s->s.gaussians.size() + n);
    s->s.pre.reserve(s->s.pre.size() + n);
    for (uint64_t i = 0; i < n; ++i) {
        double x = rng.uniform(-1.0, 1.0);
        double y;
        if (variant == 0) y = rng.uniform(0.0, 2.0);
        else {
            double u = rng.uniform();
            y = 0.0 + 2.0 * (u * u);  // biased_y(0, 2, power=2)
        }
        double z = rng.uniform(-1.0, 1.0);
        double d[3] = {rng.uniform(0.01, 0.035), rng.uniform(0.01, 0.035), rng.uniform(0.01, 0.035)};
        // Q from QR of a standard-normal 3x3 (Gram-Schmidt on columns), det fixed to +1
        double A[3][3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) A[r][c] = rng.normal();
        double Q[3][3];
        for (int c = 0; c < 3; ++c) {
            double v[3] = {A[0][c], A[1][c], A[2][c]};
            for (int p = 0; p < c; ++p) {
                double dp = Q[0][p] * A[0][c] + Q[1][p] * A[1][c] + Q[2][p] * A[2][c];
                for (int r = 0; r < 3; ++r) v[r] -= dp * Q[r][p];
            }
            double nv = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            for (int r = 0; r < 3; ++r) Q[r][c] = v[r] / nv;
        }
        double det = Q[0][0] * (Q[1][1] * Q[2][2] - Q[1][2] * Q[2][1]) - Q[0][1] * (Q[1][0] * Q[2][2] - Q[1][2] * Q[2][0]) +
                     Q[0][2] * (Q[1][0] * Q[2][1] - Q[1][1] * Q[2][0]);
        if (det < 0)
            for (int r = 0; r < 3; ++r) Q[r][0] = -Q[r][0];
        double var[3] = {(d[0] / 2) * (d[0] / 2), (d[1] / 2) * (d[1] / 2), (d[2] / 2) * (d[2] / 2)};
        double C[3][3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) C[r][c] = Q[r][0] * var[0] * Q[c][0] + Q[r][1] * var[1] * Q[c][1] + Q[r][2] * var[2] * Q[c][2];
        vr_gaussian g{};
        g.mean[0] = printed(x, 1e4);
        g.mean[1] = printed(y, 1e4);
        g.mean[2] = printed(z, 1e4);
        g.cov[0] = printed(C[0][0], 1e6);
        g.cov[1] = printed(C[0][1], 1e6);
        g.cov[2] = printed(C[0][2], 1e6);
        g.cov[3] = printed(C[1][1], 1e6);
        g.cov[4] = printed(C[1][2], 1e6);
        g.cov[5] = printed(C[2][2], 1e6);
        g.density = printed(rng.uniform(0.2, 0.5), 1e4);
        g.albedo = printed(rng.uniform(0.25, 0.95), 1e4);
        for (int k = 0; k < 3; ++k) g.emission[k] = printed(rng.uniform(0.0, 1.0), 1e4);
        s->s.gaussians.push_back(g);
        s->s.pre.push_back(precompute_gaussian(g));
    }
    return VR_OK;
}
