// Host scene: loaders (scene.h), Gaussian precompute (gaussian.h), camera (camera.h), PPM I/O
// (image.h) and the Mitsuba-subset XML loader. Plain C++; compiled into libvr_hip.so.
//
// Floating-point policy: this file is compiled with -ffp-contract=off and evaluates every
// expression in the order the reference (through Eigen 3.4.0) does, so that the HBM records and
// camera bases are bit-identical to what the reference's host code would produce:
//   * 3-term reductions (dot, squaredNorm, Matrix3f*Vector3f rows) are e0 + (e1 + e2)
//     (Eigen redux_novec_unroller splits a length-3 reduction as 1 + 2);
//   * normalized() is v / sqrt(squaredNorm()) guarded by squaredNorm() > 0;
//   * the 3x3 inverse is the cofactor/adjugate form of Eigen's compute_inverse<..., 3> and the
//     determinant is Eigen's bruteforce_det3 expansion.
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <numbers>
#include <sstream>

#include "vr_common.h"

namespace vr {

static thread_local std::string g_last_error;

vr_status fail(vr_status st, const std::string& msg) {
    g_last_error = msg;
    return st;
}
void clear_error() { g_last_error.clear(); }

namespace {

struct F3 {
    float v[3];
};
inline float dot3(const float* a, const float* b) { return a[0] * b[0] + (a[1] * b[1] + a[2] * b[2]); }
inline F3 normalized3(const float* a) {
    float z = dot3(a, a);
    if (z > 0.0f) {
        float s = std::sqrt(z);
        return {{a[0] / s, a[1] / s, a[2] / s}};
    }
    return {{a[0], a[1], a[2]}};
}
inline F3 cross3(const float* l, const float* r) {
    return {{l[1] * r[2] - l[2] * r[1], l[2] * r[0] - l[0] * r[2], l[0] * r[1] - l[1] * r[0]}};
}

// 3x3 helpers on a full row-major matrix m[i][j]
inline float cof(const float m[3][3], int i, int j) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1];
}

}  // namespace

GaussianPre precompute_gaussian(const vr_gaussian& g) {
    GaussianPre p{};
    const float* c = g.cov;
    const float m[3][3] = {{c[0], c[1], c[2]}, {c[1], c[3], c[4]}, {c[2], c[4], c[5]}};
    // inverse (Eigen compute_inverse<...,3>): det from column-0 cofactors, adjugate * invdet
    float c00 = cof(m, 0, 0), c10 = cof(m, 1, 0), c20 = cof(m, 2, 0);
    float det_inv = c00 * m[0][0] + (c10 * m[1][0] + c20 * m[2][0]);
    float invdet = 1.0f / det_inv;
    float inv[3][3];
    inv[0][0] = c00 * invdet;
    inv[0][1] = c10 * invdet;
    inv[0][2] = c20 * invdet;
    inv[1][0] = cof(m, 0, 1) * invdet;
    inv[1][1] = cof(m, 1, 1) * invdet;
    inv[1][2] = cof(m, 2, 1) * invdet;
    inv[2][0] = cof(m, 0, 2) * invdet;
    inv[2][1] = cof(m, 1, 2) * invdet;
    inv[2][2] = cof(m, 2, 2) * invdet;
    // determinant (Eigen bruteforce_det3_helper expansion along row 0)
    auto d3 = [&](int a, int b, int cc) { return m[0][a] * (m[1][b] * m[2][cc] - m[1][cc] * m[2][b]); };
    float det_cov = d3(0, 1, 2) - d3(1, 0, 2) + d3(2, 0, 1);
    // gaussian.h:55 — first factor evaluated in double (float * std::numbers::pi is double)
    p.norm = (float)(std::pow(2.0f * std::numbers::pi, -1.5f) * std::pow(det_cov, -0.5f));
    p.mean[0] = g.mean[0];
    p.mean[1] = g.mean[1];
    p.mean[2] = g.mean[2];
    p.density = g.density;
    p.albedo = g.albedo;
    p.inv_cov[0] = inv[0][0];
    p.inv_cov[1] = inv[0][1];
    p.inv_cov[2] = inv[0][2];
    p.inv_cov[3] = inv[1][1];
    p.inv_cov[4] = inv[1][2];
    p.inv_cov[5] = inv[2][2];
    std::memcpy(p.cov, g.cov, sizeof(p.cov));
    return p;
}

// Conservative box of the 3-sigma ellipsoid: half extent R*sqrt(Sigma_kk) (exact for an
// ellipsoid), padded by 5% so that near-tangent intersections the float quadratic still reports
// are never culled. The reference's eigen-derived box (gaussian.h:304-319) is also conservative;
// the event SET seen by the integrators does not depend on the box.
void gaussian_bounds(const GaussianPre& g, float bmin[3], float bmax[3]) {
    const float d[3] = {g.cov[0], g.cov[3], g.cov[5]};
    for (int k = 0; k < 3; ++k) {
        float h = 3.0f * std::sqrt(std::max(d[k], 0.0f));
        h = h * 1.05f + 1e-6f;
        bmin[k] = g.mean[k] - h;
        bmax[k] = g.mean[k] + h;
    }
}
void sphere_bounds(const vr_sphere& s, float bmin[3], float bmax[3]) {
    for (int k = 0; k < 3; ++k) {
        float h = std::fabs(s.radius) * 1.001f + 1e-6f;
        bmin[k] = s.center[k] - h;
        bmax[k] = s.center[k] + h;
    }
}

std::vector<float> step_table(float step, float t_max) {
    std::vector<float> t;
    float x = 0.0f;
    t.push_back(x);
    while (x <= t_max) {
        float nx = x + step;
        if (!(nx > x)) break;  // step below ulp: sequence stalls (reference would loop forever)
        x = nx;
        t.push_back(x);
        if (t.size() > (1u << 24)) break;
    }
    return t;
}

}  // namespace vr

using namespace vr;

// =============================================================================================
// C ABI: library / scene
// =============================================================================================
extern "C" {

const char* vr_version(void) { return "vr_hip 0.1 (gfx950)"; }
const char* vr_last_error(void) { return vr::g_last_error.c_str(); }

vr_status vr_scene_create(int32_t volume_type, vr_scene** out) {
    if (!out) return fail(VR_ERR_INVALID, "vr_scene_create: out is NULL");
    if (volume_type != VR_VOLUME_GAUSSIANS && volume_type != VR_VOLUME_SPHERES)
        return fail(VR_ERR_INVALID, "vr_scene_create: unknown volume type");
    *out = new vr_scene();
    (*out)->s.type = volume_type;
    return VR_OK;
}

void vr_scene_destroy(vr_scene* s) { delete s; }

vr_status vr_scene_add_gaussians(vr_scene* s, const vr_gaussian* g, size_t n) {
    if (!s || (n && !g)) return fail(VR_ERR_INVALID, "vr_scene_add_gaussians: NULL argument");
    if (s->s.type != VR_VOLUME_GAUSSIANS) return fail(VR_ERR_INVALID, "vr_scene_add_gaussians: not a Gaussian scene");
    s->s.gaussians.reserve(s->s.gaussians.size() + n);
    s->s.pre.reserve(s->s.pre.size() + n);
    for (size_t i = 0; i < n; ++i) {
        s->s.gaussians.push_back(g[i]);
        s->s.pre.push_back(precompute_gaussian(g[i]));
    }
    return VR_OK;
}

vr_status vr_scene_add_spheres(vr_scene* s, const vr_sphere* sp, size_t n) {
    if (!s || (n && !sp)) return fail(VR_ERR_INVALID, "vr_scene_add_spheres: NULL argument");
    if (s->s.type != VR_VOLUME_SPHERES) return fail(VR_ERR_INVALID, "vr_scene_add_spheres: not a sphere scene");
    s->s.spheres.insert(s->s.spheres.end(), sp, sp + n);
    return VR_OK;
}

vr_status vr_scene_add_lights(vr_scene* s, const vr_light* l, size_t n) {
    if (!s || (n && !l)) return fail(VR_ERR_INVALID, "vr_scene_add_lights: NULL argument");
    s->s.lights.insert(s->s.lights.end(), l, l + n);
    return VR_OK;
}

vr_status vr_scene_set_env_color(vr_scene* s, const float rgb[3]) {
    if (!s || !rgb) return fail(VR_ERR_INVALID, "vr_scene_set_env_color: NULL argument");
    std::memcpy(s->s.env, rgb, sizeof(float) * 3);
    return VR_OK;
}

vr_status vr_scene_get_info(const vr_scene* s, vr_scene_info* o) {
    if (!s || !o) return fail(VR_ERR_INVALID, "vr_scene_get_info: NULL argument");
    const HostScene& h = s->s;
    o->volume_type = h.type;
    o->num_primitives = (int64_t)(h.type == VR_VOLUME_GAUSSIANS ? h.gaussians.size() : h.spheres.size());
    o->num_lights = (int64_t)h.lights.size();
    std::memcpy(o->env_color, h.env, sizeof(h.env));
    for (int k = 0; k < 3; ++k) {
        o->bounds_min[k] = INFINITY;
        o->bounds_max[k] = -INFINITY;
    }
    float bmin[3], bmax[3];
    for (size_t i = 0; i < (size_t)o->num_primitives; ++i) {
        if (h.type == VR_VOLUME_GAUSSIANS) gaussian_bounds(h.pre[i], bmin, bmax);
        else sphere_bounds(h.spheres[i], bmin, bmax);
        for (int k = 0; k < 3; ++k) {
            o->bounds_min[k] = std::min(o->bounds_min[k], bmin[k]);
            o->bounds_max[k] = std::max(o->bounds_max[k], bmax[k]);
        }
    }
    return VR_OK;
}

vr_status vr_scene_get_records(const vr_scene* s, float* out, size_t n) {
    if (!s || (n && !out)) return fail(VR_ERR_INVALID, "vr_scene_get_records: NULL argument");
    if (n > s->s.pre.size()) return fail(VR_ERR_INVALID, "vr_scene_get_records: n exceeds scene size");
    for (size_t i = 0; i < n; ++i) {
        const GaussianPre& p = s->s.pre[i];
        float* o = out + 12 * i;
        o[0] = p.mean[0]; o[1] = p.mean[1]; o[2] = p.mean[2]; o[3] = p.density;
        for (int k = 0; k < 6; ++k) o[4 + k] = p.inv_cov[k];
        o[10] = p.norm; o[11] = p.albedo;
    }
    return VR_OK;
}

vr_status vr_scene_get_lights(const vr_scene* s, vr_light* out, size_t n) {
    if (!s || (n && !out) || n > s->s.lights.size()) return fail(VR_ERR_INVALID, "vr_scene_get_lights: bad argument");
    std::copy(s->s.lights.begin(), s->s.lights.begin() + n, out);
    return VR_OK;
}
vr_status vr_scene_get_gaussians(const vr_scene* s, vr_gaussian* out, size_t n) {
    if (!s || (n && !out) || n > s->s.gaussians.size()) return fail(VR_ERR_INVALID, "vr_scene_get_gaussians: bad argument");
    std::copy(s->s.gaussians.begin(), s->s.gaussians.begin() + n, out);
    return VR_OK;
}
vr_status vr_scene_get_spheres(const vr_scene* s, vr_sphere* out, size_t n) {
    if (!s || (n && !out) || n > s->s.spheres.size()) return fail(VR_ERR_INVALID, "vr_scene_get_spheres: bad argument");
    std::copy(s->s.spheres.begin(), s->s.spheres.begin() + n, out);
    return VR_OK;
}

// scene.h:72-120. Same std::ifstream >> token loop: unknown tokens (e.g. "//", words of a
// comment line) are skipped one at a time; emission is read only when the character right after
// the albedo is neither '\n' nor EOF (scene.h:99-106) — a 'g' line with trailing blanks and no
// emission therefore swallows the next line's tag exactly as the reference does.
vr_status vr_scene_load_gmm(const char* path, vr_scene** out) {
    if (!path || !out) return fail(VR_ERR_INVALID, "vr_scene_load_gmm: NULL argument");
    std::ifstream file(path);
    if (!file) return fail(VR_ERR_IO, std::string("Failed to open scene file: ") + path);
    vr_scene* sc = new vr_scene();
    sc->s.type = VR_VOLUME_GAUSSIANS;
    std::string tag;
    while (file >> tag) {
        if (tag == "l") {
            vr_light l{};
            file >> l.position[0] >> l.position[1] >> l.position[2] >> l.intensity[0] >> l.intensity[1] >> l.intensity[2];
            sc->s.lights.push_back(l);
        } else if (tag == "g") {
            vr_gaussian g{};
            file >> g.mean[0] >> g.mean[1] >> g.mean[2] >> g.cov[0] >> g.cov[1] >> g.cov[2] >> g.cov[3] >> g.cov[4] >>
                g.cov[5] >> g.density >> g.albedo;
            int next = file.peek();
            if (next != '\n' && next != EOF) {
                float er, eg, eb;
                if (file >> er >> eg >> eb) {
                    g.emission[0] = er;
                    g.emission[1] = eg;
                    g.emission[2] = eb;
                }
            }
            sc->s.gaussians.push_back(g);
            sc->s.pre.push_back(precompute_gaussian(g));
        }
    }
    *out = sc;
    return VR_OK;
}

// scene.h:38-68
vr_status vr_scene_load_smm(const char* path, vr_scene** out) {
    if (!path || !out) return fail(VR_ERR_INVALID, "vr_scene_load_smm: NULL argument");
    std::ifstream file(path);
    if (!file) return fail(VR_ERR_IO, std::string("Failed to open scene file: ") + path);
    vr_scene* sc = new vr_scene();
    sc->s.type = VR_VOLUME_SPHERES;
    std::string tag;
    while (file >> tag) {
        if (tag == "l") {
            vr_light l{};
            file >> l.position[0] >> l.position[1] >> l.position[2] >> l.intensity[0] >> l.intensity[1] >> l.intensity[2];
            sc->s.lights.push_back(l);
        } else if (tag == "s") {
            vr_sphere sp{};
            file >> sp.center[0] >> sp.center[1] >> sp.center[2] >> sp.radius >> sp.sigma_a >> sp.sigma_s;
            sc->s.spheres.push_back(sp);
        }
    }
    *out = sc;
    return VR_OK;
}

// =============================================================================================
// Camera (camera.h). The base constructor body uses the *parameter* view_dir (shadowing the
// normalised member) for right/up (camera.h:20-21); Pinhole uses the parameter for the pinhole
// point (camera.h:42).
// =============================================================================================
static void camera_base(const float pos[3], const float vd[3], vr_camera* c) {
    std::memset(c, 0, sizeof(*c));
    std::memcpy(c->position, pos, sizeof(float) * 3);
    F3 n = normalized3(vd);
    std::memcpy(c->view_dir, n.v, sizeof(float) * 3);
    const float world_up[3] = {0.0f, 1.0f, 0.0f};
    F3 cr = cross3(vd, world_up);
    F3 r = normalized3(cr.v);
    std::memcpy(c->right, r.v, sizeof(float) * 3);
    F3 cu = cross3(r.v, vd);
    F3 u = normalized3(cu.v);
    std::memcpy(c->up, u.v, sizeof(float) * 3);
}

vr_status vr_camera_pinhole(const float position[3], const float view_dir[3], float fov, vr_camera* out) {
    if (!position || !view_dir || !out) return fail(VR_ERR_INVALID, "vr_camera_pinhole: NULL argument");
    camera_base(position, view_dir, out);
    out->type = VR_CAMERA_PINHOLE;
    out->fov = fov;
    out->focal_length = 1.0f / std::tan(0.5f * fov);
    for (int k = 0; k < 3; ++k) out->pinhole[k] = position[k] + out->focal_length * view_dir[k];
    return VR_OK;
}

vr_status vr_camera_orthographic(const float position[3], const float forward[3], vr_camera* out) {
    if (!position || !forward || !out) return fail(VR_ERR_INVALID, "vr_camera_orthographic: NULL argument");
    camera_base(position, forward, out);
    out->type = VR_CAMERA_ORTHOGRAPHIC;
    return VR_OK;
}

vr_status vr_camera_sample_ray(const vr_camera* c, double uvx, double uvy, float origin[3], float direction[3]) {
    if (!c || !origin || !direction) return fail(VR_ERR_INVALID, "vr_camera_sample_ray: NULL argument");
    float u, v, d[3];
    if (c->type == VR_CAMERA_PINHOLE) {
        u = 1.0f - static_cast<float>(uvx) * 2.0f;
        v = static_cast<float>(uvy) * 2.0f - 1.0f;
    } else {
        u = static_cast<float>(uvx) * 2.0f - 1.0f;
        v = 1.0f - static_cast<float>(uvy) * 2.0f;
    }
    for (int k = 0; k < 3; ++k) origin[k] = (c->position[k] + u * c->right[k]) + v * c->up[k];
    if (c->type == VR_CAMERA_PINHOLE)
        for (int k = 0; k < 3; ++k) d[k] = c->pinhole[k] - origin[k];
    else
        std::memcpy(d, c->view_dir, sizeof(d));
    F3 n1 = normalized3(d);      // camera.h:52 / :72
    F3 n2 = normalized3(n1.v);   // ray.h:11-12
    std::memcpy(direction, n2.v, sizeof(float) * 3);
    return VR_OK;
}

// =============================================================================================
// Image (image.h)
// =============================================================================================
vr_status vr_image_write_ppm(const char* path, const float* rgb, uint32_t W, uint32_t H) {
    if (!path || (!rgb && W && H)) return fail(VR_ERR_INVALID, "vr_image_write_ppm: NULL argument");
    std::ofstream f(path, std::ios::binary);
    if (!f) return fail(VR_ERR_IO, std::string("cannot open ") + path);
    f << "P6\n" << W << " " << H << "\n255\n";
    std::vector<unsigned char> row(3 * (size_t)W);
    for (uint32_t j = 0; j < H; ++j) {
        for (uint32_t i = 0; i < 3 * W; ++i)  // image.h:66 clamp then truncate
            row[i] = static_cast<unsigned char>(std::clamp(rgb[(size_t)3 * W * j + i] * 255.0f, 0.0f, 255.0f));
        f.write(reinterpret_cast<const char*>(row.data()), (std::streamsize)row.size());
    }
    if (!f) return fail(VR_ERR_IO, std::string("write failed: ") + path);
    return VR_OK;
}

vr_status vr_image_read_ppm(const char* path, float* rgb, uint32_t* W, uint32_t* H) {
    if (!path || !W || !H) return fail(VR_ERR_INVALID, "vr_image_read_ppm: NULL argument");
    std::ifstream in(path, std::ios::binary);
    if (!in) return fail(VR_ERR_IO, std::string("Failed to open PPM file: ") + path);
    std::string magic;
    in >> magic;
    if (magic != "P6") return fail(VR_ERR_PARSE, "Not a P6 PPM file.");
    unsigned w = 0, h = 0;
    int maxval = 0;
    in >> w >> h >> maxval;
    in.get();
    if (!in || w == 0 || h == 0) return fail(VR_ERR_PARSE, "bad PPM header");
    *W = w;
    *H = h;
    if (!rgb) return VR_OK;
    std::vector<unsigned char> buf(3 * (size_t)w * h);
    in.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)buf.size());
    if ((size_t)in.gcount() != buf.size()) return fail(VR_ERR_PARSE, "truncated PPM data");
    for (size_t i = 0; i < buf.size(); ++i) rgb[i] = buf[i] / 255.f;
    return VR_OK;
}

}  // extern "C"
