// Mitsuba-3 XML subset loader.
//
// The reference has no XML parser: tests/env_one_sphere_test_ortho.xml was rendered in Mitsuba
// and compared visually (slides p.42). This loader maps the subset that file uses onto the
// reference's own scene model, so the XML scene renders through RayMarchingSpheres /
// RayMarchingGaussians exactly like the equivalent text scene (scenes/spheres/1_spheres.txt):
//
//   <integrator type="volpath|...">            -> params: RayMarchingSpheres (sphere scenes) or
//                                                  RayMarchingGaussians; step 0.01; env samples
//                                                  5 / 20 (test_integrators.h:17,152)
//   <sensor type="orthographic|perspective">    -> Orthographic_Camera(origin, normalize(target-origin))
//       <transform><lookat origin target up/>      or Pinhole_Camera(..., fov[deg] -> radians).
//       <film> width/height                         `up` is ignored: camera.h:18 hard-codes +y.
//   <emitter type="constant"> rgb radiance     -> Scene::env_color
//   <emitter type="point"> point position, rgb intensity -> Light{position, intensity}
//   <medium type="homogeneous" id> rgb albedo, rgb sigma_t, float scale
//   <shape type="sphere"> point center, float radius, ref interior -> Sphere(c, r,
//                          sigma_a = sigma_t (1 - albedo) scale, sigma_s = sigma_t albedo scale)
//   <shape type="gaussian"> (extension) point mean, cov "xx xy xz yy yz zz", float density,
//                          float albedo -> Gaussian
// Anything else is ignored.
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>

#include "vr_common.h"

using namespace vr;

namespace {

struct XNode {
    std::string tag;
    std::map<std::string, std::string> attr;
    std::vector<std::unique_ptr<XNode>> kids;
    const XNode* child(const std::string& t, const std::string& name = "") const {
        for (auto& k : kids)
            if (k->tag == t && (name.empty() || k->get("name") == name)) return k.get();
        return nullptr;
    }
    std::string get(const std::string& k, const std::string& def = "") const {
        auto it = attr.find(k);
        return it == attr.end() ? def : it->second;
    }
};

struct XParser {
    const std::string& s;
    size_t i = 0;
    std::string err;
    explicit XParser(const std::string& str) : s(str) {}
    void ws() { while (i < s.size() && std::isspace((unsigned char)s[i])) ++i; }
    bool starts(const char* p) const { return s.compare(i, std::strlen(p), p) == 0; }
    bool skip_misc() {  // comments, <? ?>, <! >
        for (;;) {
            ws();
            if (starts("<!--")) {
                size_t e = s.find("-->", i);
                if (e == std::string::npos) { err = "unterminated comment"; return false; }
                i = e + 3;
            } else if (starts("<?")) {
                size_t e = s.find("?>", i);
                if (e == std::string::npos) { err = "unterminated <?"; return false; }
                i = e + 2;
            } else if (starts("<!")) {
                size_t e = s.find('>', i);
                if (e == std::string::npos) { err = "unterminated <!"; return false; }
                i = e + 1;
            } else return true;
        }
    }
    std::string name() {
        size_t b = i;
        while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '-' || s[i] == ':' || s[i] == '.')) ++i;
        return s.substr(b, i - b);
    }
    std::unique_ptr<XNode> element() {
        if (!skip_misc()) return nullptr;
        if (i >= s.size() || s[i] != '<') { err = "expected '<'"; return nullptr; }
        ++i;
        auto n = std::make_unique<XNode>();
        n->tag = name();
        if (n->tag.empty()) { err = "empty tag name"; return nullptr; }
        for (;;) {
            ws();
            if (i >= s.size()) { err = "unexpected end in tag"; return nullptr; }
            if (s[i] == '/') {
                if (i + 1 < s.size() && s[i + 1] == '>') { i += 2; return n; }
                err = "bad '/'"; return nullptr;
            }
            if (s[i] == '>') { ++i; break; }
            std::string k = name();
            ws();
            if (k.empty() || i >= s.size() || s[i] != '=') { err = "bad attribute"; return nullptr; }
            ++i;
            ws();
            if (i >= s.size() || (s[i] != '"' && s[i] != '\'')) { err = "unquoted attribute"; return nullptr; }
            char q = s[i++];
            size_t e = s.find(q, i);
            if (e == std::string::npos) { err = "unterminated attribute"; return nullptr; }
            n->attr[k] = s.substr(i, e - i);
            i = e + 1;
        }
        for (;;) {  // children until </tag>
            if (!skip_misc()) return nullptr;
            if (starts("</")) {
                i += 2;
                std::string t = name();
                ws();
                if (t != n->tag || i >= s.size() || s[i] != '>') { err = "mismatched </" + t + ">"; return nullptr; }
                ++i;
                return n;
            }
            if (i < s.size() && s[i] == '<') {
                auto c = element();
                if (!c) return nullptr;
                n->kids.push_back(std::move(c));
            } else {  // text content: skip
                size_t e = s.find('<', i);
                if (e == std::string::npos) { err = "unexpected end"; return nullptr; }
                i = e;
            }
        }
    }
};

bool parse_floats(const std::string& str, float* out, int n) {
    std::string t = str;
    for (char& c : t)
        if (c == ',') c = ' ';
    std::istringstream is(t);
    int k = 0;
    float v;
    while (k < n && (is >> v)) out[k++] = v;
    if (k == 1 && n == 3) { out[1] = out[0]; out[2] = out[0]; k = 3; }  // Mitsuba scalar rgb
    return k == n;
}
bool rgb_of(const XNode* parent, const std::string& name, float out[3]) {
    for (auto& k : parent->kids)
        if ((k->tag == "rgb" || k->tag == "spectrum" || k->tag == "color") && k->get("name") == name)
            return parse_floats(k->get("value"), out, 3);
    return false;
}
bool float_of(const XNode* parent, const std::string& name, float& out) {
    for (auto& k : parent->kids)
        if ((k->tag == "float" || k->tag == "integer") && k->get("name") == name) {
            float v[1];
            if (!parse_floats(k->get("value"), v, 1)) return false;
            out = v[0];
            return true;
        }
    return false;
}
bool point_of(const XNode* parent, const std::string& name, float out[3]) {
    for (auto& k : parent->kids)
        if ((k->tag == "point" || k->tag == "vector") && k->get("name") == name) {
            if (k->attr.count("value")) return parse_floats(k->get("value"), out, 3);
            out[0] = std::stof(k->get("x", "0"));
            out[1] = std::stof(k->get("y", "0"));
            out[2] = std::stof(k->get("z", "0"));
            return true;
        }
    return false;
}

}  // namespace

extern "C" vr_status vr_scene_load_xml(const char* path, vr_scene** out, vr_camera* camera, uint32_t* width,
                                       uint32_t* height, vr_render_params* params) {
    if (!path || !out) return fail(VR_ERR_INVALID, "vr_scene_load_xml: NULL argument");
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail(VR_ERR_IO, std::string("Failed to open scene file: ") + path);
    std::stringstream ss;
    ss << f.rdbuf();
    std::string text = ss.str();
    XParser P(text);
    std::unique_ptr<XNode> root;
    try {
        root = P.element();
    } catch (const std::exception& e) {
        return fail(VR_ERR_PARSE, std::string("XML: ") + e.what());
    }
    if (!root) return fail(VR_ERR_PARSE, "XML: " + P.err);
    if (root->tag != "scene") return fail(VR_ERR_PARSE, "XML: root element is not <scene>");

    std::map<std::string, const XNode*> media;
    bool has_gauss = false;
    for (auto& k : root->kids) {
        if (k->tag == "medium" && k->attr.count("id")) media[k->get("id")] = k.get();
        if (k->tag == "shape" && k->get("type") == "gaussian") has_gauss = true;
    }
    auto sc = std::make_unique<vr_scene>();
    sc->s.type = has_gauss ? VR_VOLUME_GAUSSIANS : VR_VOLUME_SPHERES;

    vr_camera cam{};
    bool have_cam = false;
    uint32_t W = 512, H = 512;
    try {
        for (auto& k : root->kids) {
            const std::string type = k->get("type");
            if (k->tag == "sensor") {
                float o[3] = {0, 0, 0}, t[3] = {0, 0, -1};
                if (const XNode* tr = k->child("transform"))
                    if (const XNode* la = tr->child("lookat")) {
                        if (!parse_floats(la->get("origin"), o, 3) || !parse_floats(la->get("target"), t, 3))
                            return fail(VR_ERR_PARSE, "XML: bad <lookat>");
                    }
                float d[3] = {t[0] - o[0], t[1] - o[1], t[2] - o[2]};
                // normalize(target - origin) as main.cpp:33 does for its camera
                float z = d[0] * d[0] + (d[1] * d[1] + d[2] * d[2]);
                if (z > 0.0f) {
                    float sq = std::sqrt(z);
                    d[0] /= sq; d[1] /= sq; d[2] /= sq;
                }
                vr_status st;
                if (type == "orthographic") st = vr_camera_orthographic(o, d, &cam);
                else {
                    float fov_deg = 45.0f;
                    float_of(k.get(), "fov", fov_deg);
                    st = vr_camera_pinhole(o, d, fov_deg * (float)(M_PI / 180.0), &cam);
                }
                if (st != VR_OK) return st;
                have_cam = true;
                if (const XNode* film = k->child("film")) {
                    float w = 0, h = 0;
                    if (float_of(film, "width", w)) W = (uint32_t)w;
                    if (float_of(film, "height", h)) H = (uint32_t)h;
                }
            } else if (k->tag == "emitter" && type == "constant") {
                float c[3];
                if (!rgb_of(k.get(), "radiance", c)) return fail(VR_ERR_PARSE, "XML: constant emitter without radiance");
                std::memcpy(sc->s.env, c, sizeof(c));
            } else if (k->tag == "emitter" && type == "point") {
                vr_light l{};
                if (!point_of(k.get(), "position", l.position)) return fail(VR_ERR_PARSE, "XML: point emitter without position");
                if (!rgb_of(k.get(), "intensity", l.intensity)) return fail(VR_ERR_PARSE, "XML: point emitter without intensity");
                sc->s.lights.push_back(l);
            } else if (k->tag == "shape" && type == "sphere") {
                vr_sphere sp{};
                if (!point_of(k.get(), "center", sp.center)) return fail(VR_ERR_PARSE, "XML: sphere without center");
                sp.radius = 1.0f;
                float_of(k.get(), "radius", sp.radius);
                const XNode* med = nullptr;
                for (auto& c : k->kids)
                    if (c->tag == "ref" && c->get("name") == "interior") {
                        auto it = media.find(c->get("id"));
                        if (it != media.end()) med = it->second;
                    }
                if (!med) return fail(VR_ERR_PARSE, "XML: sphere without an interior homogeneous medium");
                float alb[3] = {1, 1, 1}, st[3] = {1, 1, 1}, scale = 1.0f;
                rgb_of(med, "albedo", alb);
                rgb_of(med, "sigma_t", st);
                float_of(med, "scale", scale);
                // grey media only (the reference's spheres carry scalar coefficients)
                sp.sigma_s = (float)((double)st[0] * (double)alb[0] * (double)scale);
                sp.sigma_a = (float)((double)st[0] * (1.0 - (double)alb[0]) * (double)scale);
                if (sc->s.type != VR_VOLUME_SPHERES) return fail(VR_ERR_UNSUPPORTED, "XML: mixing spheres and Gaussians");
                sc->s.spheres.push_back(sp);
            } else if (k->tag == "shape" && type == "gaussian") {
                vr_gaussian g{};
                if (!point_of(k.get(), "mean", g.mean)) return fail(VR_ERR_PARSE, "XML: gaussian without mean");
                bool okc = false;
                for (auto& c : k->kids)
                    if (c->get("name") == "cov") okc = parse_floats(c->get("value"), g.cov, 6);
                if (!okc) return fail(VR_ERR_PARSE, "XML: gaussian without cov");
                float_of(k.get(), "density", g.density);
                float_of(k.get(), "albedo", g.albedo);
                sc->s.gaussians.push_back(g);
                sc->s.pre.push_back(precompute_gaussian(g));
            }
        }
    } catch (const std::exception& e) {
        return fail(VR_ERR_PARSE, std::string("XML: ") + e.what());
    }
    if (camera) {
        if (!have_cam) return fail(VR_ERR_PARSE, "XML: no <sensor>");
        *camera = cam;
    }
    if (width) *width = W;
    if (height) *height = H;
    if (params) {
        params->integrator = sc->s.type == VR_VOLUME_SPHERES ? VR_RAYMARCH_SPHERES : VR_RAYMARCH_GAUSSIANS;
        params->step_size = 0.01f;
        params->env_samples = sc->s.type == VR_VOLUME_SPHERES ? 5 : 20;
        params->t_eps = 0.0f;
        params->flags = 0;
        params->num_samples = 1;  // sample_count (the ray-march integrators take one sample per pixel)
        params->min_bounces = 5;
    }
    *out = sc.release();
    return VR_OK;
}
