// Host C++ API of the MI355X volume renderer: a header-only mirror of the reference's classes
// (wantonsushi/3DG-vol-renderer include/*.h) on top of the C ABI in include/vr_hip.h.
//
//   Scene scene = Scene::load_GMM("scenes/gaussians/many_gaussians.txt");     // scene.h:72-120
//   auto camera = std::make_shared<Pinhole_Camera>(pos, view_dir, fov);        // camera.h:31-54
//   Image image(512, 512);                                                     // image.h:9-20
//   auto integrator = std::make_unique<RayMarchingGaussians>(camera);          // test_integrators.h:143
//   integrator->render(scene, image);                                          // integrator.h:56
//   image.make_PPM("output.ppm");                                              // image.h:62-84
//
// Same class names, constructor arguments, public members and error behaviour
// (std::runtime_error). Rendering runs on the GPU through libvr_hip.so; there is no CPU renderer
// here. Link with -lvr_hip.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <filesystem>
#include <iostream>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/vr_hip.h"
#include "linalg.h"

namespace vr_cpp {

inline void check(vr_status st) {
    if (st != VR_OK) throw std::runtime_error(vr_last_error());
}

// One device context per GPU, created on first use (vr_init), destroyed at exit.
inline vr_ctx* device(int dev = 0) {
    static std::mutex mu;
    static std::vector<std::unique_ptr<vr_ctx, void (*)(vr_ctx*)>> ctxs;
    std::lock_guard<std::mutex> lock(mu);
    while ((int)ctxs.size() <= dev) ctxs.emplace_back(nullptr, &vr_destroy);
    if (!ctxs[dev]) {
        vr_ctx* c = nullptr;
        check(vr_init(dev, &c));
        ctxs[dev].reset(c);
    }
    return ctxs[dev].get();
}

// Number of visible GPUs.
inline int device_count() {
    int32_t n = 0;
    check(vr_device_count(&n));
    return n;
}

// One multi-GPU context per device list (vr_init_multi), created on first use.
inline vr_ctx* device_group(const std::vector<int>& devs) {
    static std::mutex mu;
    static std::map<std::vector<int>, std::unique_ptr<vr_ctx, void (*)(vr_ctx*)>> groups;
    std::lock_guard<std::mutex> lock(mu);
    auto it = groups.find(devs);
    if (it == groups.end()) {
        std::vector<int32_t> d(devs.begin(), devs.end());
        vr_ctx* c = nullptr;
        check(vr_init_multi((int32_t)d.size(), d.data(), &c));
        it = groups.emplace(devs, std::unique_ptr<vr_ctx, void (*)(vr_ctx*)>(c, &vr_destroy)).first;
    }
    return it->second.get();
}

inline uint64_t next_serial() {
    static std::atomic<uint64_t> serial{0};
    return ++serial;
}

inline uint64_t fnv1a(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

}  // namespace vr_cpp

// ---------------------------------------------------------------------------------------------
// ray.h:7-16
// ---------------------------------------------------------------------------------------------
struct Ray {
    Eigen::Vector3f origin;
    Eigen::Vector3f direction;
    Eigen::Vector3f throughput;
    Ray() {}
    Ray(const Eigen::Vector3f& o, const Eigen::Vector3f& d) : origin(o), direction(d.normalized()) {}
    Eigen::Vector3f operator()(float t) const { return origin + t * direction; }
};

// ---------------------------------------------------------------------------------------------
// camera.h:7-74 — state computed by vr_camera_pinhole / vr_camera_orthographic
// ---------------------------------------------------------------------------------------------
class Camera {
protected:
    vr_camera state_{};

public:
    virtual ~Camera() = default;
    const vr_camera& state() const { return state_; }
    virtual Ray sample_ray(const Eigen::Vector2d& uv) const {
        float o[3], d[3];
        vr_cpp::check(vr_camera_sample_ray(&state_, uv.x(), uv.y(), o, d));
        Ray r;
        r.origin = Eigen::Vector3f(o[0], o[1], o[2]);
        r.direction = Eigen::Vector3f(d[0], d[1], d[2]);
        return r;
    }
};

// A camera whose state came from elsewhere (e.g. the sensor of Scene::load_XML).
class State_Camera : public Camera {
public:
    explicit State_Camera(const vr_camera& s) { state_ = s; }
};

class Pinhole_Camera : public Camera {
public:
    Pinhole_Camera(const Eigen::Vector3f& position, const Eigen::Vector3f& view_dir, float fov) {
        const float p[3] = {position.x(), position.y(), position.z()};
        const float v[3] = {view_dir.x(), view_dir.y(), view_dir.z()};
        vr_cpp::check(vr_camera_pinhole(p, v, fov, &state_));
    }
};

class Orthographic_Camera : public Camera {
public:
    Orthographic_Camera(const Eigen::Vector3f& position, const Eigen::Vector3f& forward) {
        const float p[3] = {position.x(), position.y(), position.z()};
        const float v[3] = {forward.x(), forward.y(), forward.z()};
        vr_cpp::check(vr_camera_orthographic(p, v, &state_));
    }
};

// ---------------------------------------------------------------------------------------------
// gaussian.h / gmm.h / smm.h / scene.h data model
// ---------------------------------------------------------------------------------------------
class Gaussian {
    Eigen::Vector3f mean;
    Eigen::Matrix3f covariance;
    float density;
    float albedo;
    Eigen::Vector3f emission;

public:
    Gaussian(const Eigen::Vector3f& mean, const Eigen::Matrix3f& covariance, float density, float albedo,
             const Eigen::Vector3f& emission = Eigen::Vector3f::Zero())
        : mean(mean), covariance(covariance), density(density), albedo(albedo), emission(emission) {}
    Eigen::Vector3f centroid() const { return mean; }
    const Eigen::Matrix3f& get_covariance() const { return covariance; }
    float get_density() const { return density; }
    float get_albedo() const { return albedo; }
    const Eigen::Vector3f& get_emission() const { return emission; }
    vr_gaussian to_record() const {
        vr_gaussian g{};
        for (int k = 0; k < 3; ++k) g.mean[k] = mean[k];
        g.cov[0] = covariance(0, 0);
        g.cov[1] = covariance(0, 1);
        g.cov[2] = covariance(0, 2);
        g.cov[3] = covariance(1, 1);
        g.cov[4] = covariance(1, 2);
        g.cov[5] = covariance(2, 2);
        g.density = density;
        g.albedo = albedo;
        for (int k = 0; k < 3; ++k) g.emission[k] = emission[k];
        return g;
    }
    static Gaussian from_record(const vr_gaussian& g) {
        Eigen::Matrix3f c;
        c << g.cov[0], g.cov[1], g.cov[2], g.cov[1], g.cov[3], g.cov[4], g.cov[2], g.cov[4], g.cov[5];
        return Gaussian(Eigen::Vector3f(g.mean[0], g.mean[1], g.mean[2]), c, g.density, g.albedo,
                        Eigen::Vector3f(g.emission[0], g.emission[1], g.emission[2]));
    }
};

class GaussianMixtureModel {
public:
    std::vector<Gaussian> gaussians;
    GaussianMixtureModel() = default;
    explicit GaussianMixtureModel(const std::vector<Gaussian>& gs) : gaussians(gs) {}
    size_t get_num_gaussians() const { return gaussians.size(); }
    bool empty() const { return gaussians.empty(); }
    // gmm.h:583-628 (native vr_gmm_pack_parameters)
    void pack_parameters(std::vector<float>& out) const;
};

struct Sphere {
    Eigen::Vector3f center;
    float radius;
    float sigma_a;
    float sigma_s;
    Sphere(const Eigen::Vector3f& c, float r, float sa = 0.0f, float ss = 1.0f)
        : center(c), radius(r), sigma_a(sa), sigma_s(ss) {}
};

class SphereMixtureModel {
public:
    std::vector<Sphere> spheres;
    SphereMixtureModel() = default;
    explicit SphereMixtureModel(const std::vector<Sphere>& s) : spheres(s) {}
    size_t get_num_spheres() const { return spheres.size(); }
};

struct Light {
    Eigen::Vector3f position;
    Eigen::Vector3f intensity;
};

struct Scene {
    enum class VolumeType { GAUSSIANS, SPHERES, VOXELS } volume_type = VolumeType::GAUSSIANS;
    std::optional<std::vector<GaussianMixtureModel>> gmm;
    std::optional<std::vector<SphereMixtureModel>> smm;
    std::vector<Light> lights;
    Eigen::Vector3f env_color = {0.53f, 0.81f, 0.92f};  // scene.h:29

    static Scene load_GMM(const std::string& filename) {
        vr_scene* h = nullptr;
        vr_cpp::check(vr_scene_load_gmm(filename.c_str(), &h));
        return from_native(h);
    }
    static Scene load_SMM(const std::string& filename) {
        vr_scene* h = nullptr;
        vr_cpp::check(vr_scene_load_smm(filename.c_str(), &h));
        return from_native(h);
    }
    // Mitsuba-subset XML: the scene plus the sensor it describes.
    static Scene load_XML(const std::string& filename, vr_camera* camera = nullptr, uint32_t* width = nullptr,
                          uint32_t* height = nullptr, vr_render_params* params = nullptr) {
        vr_scene* h = nullptr;
        vr_cpp::check(vr_scene_load_xml(filename.c_str(), &h, camera, width, height, params));
        return from_native(h);
    }
    size_t get_num_primitives() const {
        if (volume_type == VolumeType::SPHERES) return (smm && !smm->empty()) ? (*smm)[0].get_num_spheres() : 0;
        return (gmm && !gmm->empty()) ? (*gmm)[0].get_num_gaussians() : 0;
    }

    // Native (C ABI) copy of this scene, rebuilt when the public members changed.
    vr_scene* native() const {
        uint64_t fp = fingerprint();
        if (!native_ || fp != native_fp_) {
            vr_scene* h = nullptr;
            int32_t type = volume_type == VolumeType::SPHERES ? VR_VOLUME_SPHERES : VR_VOLUME_GAUSSIANS;
            vr_cpp::check(vr_scene_create(type, &h));
            native_.reset(h, &vr_scene_destroy);
            if (type == VR_VOLUME_GAUSSIANS && gmm && !gmm->empty()) {
                std::vector<vr_gaussian> g;
                g.reserve((*gmm)[0].gaussians.size());
                for (const Gaussian& x : (*gmm)[0].gaussians) g.push_back(x.to_record());
                vr_cpp::check(vr_scene_add_gaussians(h, g.data(), g.size()));
            }
            if (type == VR_VOLUME_SPHERES && smm && !smm->empty()) {
                std::vector<vr_sphere> sp;
                for (const Sphere& s : (*smm)[0].spheres)
                    sp.push_back(vr_sphere{{s.center[0], s.center[1], s.center[2]}, s.radius, s.sigma_a, s.sigma_s});
                vr_cpp::check(vr_scene_add_spheres(h, sp.data(), sp.size()));
            }
            std::vector<vr_light> ls;
            for (const Light& l : lights)
                ls.push_back(vr_light{{l.position[0], l.position[1], l.position[2]},
                                      {l.intensity[0], l.intensity[1], l.intensity[2]}});
            vr_cpp::check(vr_scene_add_lights(h, ls.data(), ls.size()));
            const float env[3] = {env_color[0], env_color[1], env_color[2]};
            vr_cpp::check(vr_scene_set_env_color(h, env));
            native_fp_ = fp;
            native_version_ = vr_cpp::next_serial();
        }
        return native_.get();
    }
    // process-unique id of the current native copy (a freed handle's address may be reused)
    uint64_t native_version() const { return native_version_; }
    // A Scene owning a native scene handle (e.g. vr_gmm_apply_parameters' result).
    static Scene adopt_native(vr_scene* h) { return from_native(h); }

private:
    mutable std::shared_ptr<vr_scene> native_;
    mutable uint64_t native_fp_ = 0;
    mutable uint64_t native_version_ = 0;

    uint64_t fingerprint() const {
        uint64_t h = vr_cpp::fnv1a(&volume_type, sizeof(volume_type));
        if (gmm && !gmm->empty())
            for (const Gaussian& g : (*gmm)[0].gaussians) {
                vr_gaussian r = g.to_record();
                h = vr_cpp::fnv1a(&r, sizeof(r), h);
            }
        if (smm && !smm->empty())
            for (const Sphere& s : (*smm)[0].spheres) {
                float v[6] = {s.center[0], s.center[1], s.center[2], s.radius, s.sigma_a, s.sigma_s};
                h = vr_cpp::fnv1a(v, sizeof(v), h);
            }
        for (const Light& l : lights) {
            float v[6] = {l.position[0], l.position[1], l.position[2], l.intensity[0], l.intensity[1], l.intensity[2]};
            h = vr_cpp::fnv1a(v, sizeof(v), h);
        }
        float e[3] = {env_color[0], env_color[1], env_color[2]};
        return vr_cpp::fnv1a(e, sizeof(e), h);
    }

    static Scene from_native(vr_scene* h) {
        std::shared_ptr<vr_scene> owner(h, &vr_scene_destroy);
        vr_scene_info info{};
        vr_cpp::check(vr_scene_get_info(h, &info));
        Scene s;
        std::vector<vr_light> ls((size_t)info.num_lights);
        vr_cpp::check(vr_scene_get_lights(h, ls.data(), ls.size()));
        for (const vr_light& l : ls)
            s.lights.push_back({Eigen::Vector3f(l.position[0], l.position[1], l.position[2]),
                                Eigen::Vector3f(l.intensity[0], l.intensity[1], l.intensity[2])});
        s.env_color = Eigen::Vector3f(info.env_color[0], info.env_color[1], info.env_color[2]);
        if (info.volume_type == VR_VOLUME_GAUSSIANS) {
            s.volume_type = VolumeType::GAUSSIANS;
            std::vector<vr_gaussian> g((size_t)info.num_primitives);
            vr_cpp::check(vr_scene_get_gaussians(h, g.data(), g.size()));
            std::vector<Gaussian> gs;
            gs.reserve(g.size());
            for (const vr_gaussian& x : g) gs.push_back(Gaussian::from_record(x));
            s.gmm = std::vector<GaussianMixtureModel>{GaussianMixtureModel(gs)};
        } else {
            s.volume_type = VolumeType::SPHERES;
            std::vector<vr_sphere> sp((size_t)info.num_primitives);
            vr_cpp::check(vr_scene_get_spheres(h, sp.data(), sp.size()));
            std::vector<Sphere> ss;
            for (const vr_sphere& x : sp)
                ss.emplace_back(Eigen::Vector3f(x.center[0], x.center[1], x.center[2]), x.radius, x.sigma_a, x.sigma_s);
            s.smm = std::vector<SphereMixtureModel>{SphereMixtureModel(ss)};
        }
        s.native_ = owner;  // the loaded native scene is already up to date
        s.native_fp_ = s.fingerprint();
        s.native_version_ = vr_cpp::next_serial();
        return s;
    }
};

// ---------------------------------------------------------------------------------------------
// image.h:9-106
// ---------------------------------------------------------------------------------------------
class Image {
    unsigned int width = 0, height = 0;
    std::vector<float> pixels;

public:
    Image(unsigned int w, unsigned int h) : width(w), height(h), pixels(3 * (size_t)w * h, 0.0f) {}
    explicit Image(const std::string& filename) {
        vr_cpp::check(vr_image_read_ppm(filename.c_str(), nullptr, &width, &height));
        pixels.resize(3 * (size_t)width * height);
        vr_cpp::check(vr_image_read_ppm(filename.c_str(), pixels.data(), &width, &height));
    }
    unsigned int get_width() const { return width; }
    unsigned int get_height() const { return height; }
    Eigen::Vector3f get_pixel(unsigned i, unsigned j) const {
        size_t k = 3 * ((size_t)j * width + i);
        return Eigen::Vector3f(pixels[k], pixels[k + 1], pixels[k + 2]);
    }
    void set_pixel(unsigned i, unsigned j, const Eigen::Vector3f& rgb) {
        size_t k = 3 * ((size_t)j * width + i);
        pixels[k] = rgb[0];
        pixels[k + 1] = rgb[1];
        pixels[k + 2] = rgb[2];
    }
    void make_PPM(const std::string& filename) const {
        vr_cpp::check(vr_image_write_ppm(filename.c_str(), pixels.data(), width, height));
    }
    std::vector<uint8_t> get_rgba_buffer() const {
        std::vector<uint8_t> buf(4 * (size_t)width * height);
        for (size_t p = 0; p < (size_t)width * height; ++p) {
            for (int c = 0; c < 3; ++c)
                buf[4 * p + c] = static_cast<uint8_t>(std::clamp(pixels[3 * p + c] * 255.0f, 0.0f, 255.0f));
            buf[4 * p + 3] = 255;
        }
        return buf;
    }
    float* data() { return pixels.data(); }
    const float* data() const { return pixels.data(); }
};

// ---------------------------------------------------------------------------------------------
// gmm.h:583-706: GMM <-> feature vector (11 floats per Gaussian), native (host/vr_inverse.cpp)
// ---------------------------------------------------------------------------------------------
namespace vr_cpp {
inline vr_scene* gaussians_native(const GaussianMixtureModel& g) {
    vr_scene* h = nullptr;
    check(vr_scene_create(VR_VOLUME_GAUSSIANS, &h));
    std::vector<vr_gaussian> r;
    r.reserve(g.gaussians.size());
    for (const Gaussian& x : g.gaussians) r.push_back(x.to_record());
    vr_status st = vr_scene_add_gaussians(h, r.data(), r.size());
    if (st != VR_OK) {
        vr_scene_destroy(h);
        check(st);
    }
    return h;
}
}  // namespace vr_cpp

inline void GaussianMixtureModel::pack_parameters(std::vector<float>& out) const {
    std::unique_ptr<vr_scene, void (*)(vr_scene*)> h(vr_cpp::gaussians_native(*this), &vr_scene_destroy);
    out.assign(gaussians.size() * 11, 0.0f);
    vr_cpp::check(vr_gmm_pack_parameters(h.get(), out.data(), out.size()));
}

// gmm.h:634-674: rebuild every Gaussian of gmm from params (throws on a size mismatch, :637)
inline void apply_params_to_gmm_local(const std::vector<float>& params, GaussianMixtureModel& gmm) {
    std::unique_ptr<vr_scene, void (*)(vr_scene*)> base(vr_cpp::gaussians_native(gmm), &vr_scene_destroy);
    vr_scene* out = nullptr;
    vr_cpp::check(vr_gmm_apply_parameters(base.get(), params.data(), params.size(), &out));
    Scene s = Scene::adopt_native(out);
    gmm = (*s.gmm)[0];
}

// gmm.h:678-706
inline std::vector<float> make_default_eps_for_params(const std::vector<float>& base_params) {
    std::vector<float> eps(base_params.size());
    vr_cpp::check(vr_gmm_default_eps(eps.data(), eps.size()));
    return eps;
}

// optimizer.h:13-55 — AdamOptimizer (the step is vr_adam_step)
class AdamOptimizer {
public:
    AdamOptimizer(size_t ndim, float lr = 1e-3f, float beta1 = 0.9f, float beta2 = 0.999f, float eps = 1e-8f)
        : m(ndim, 0.0f), v(ndim, 0.0f), lr(lr), beta1(beta1), beta2(beta2), eps(eps), t(0) {}
    bool step(std::vector<float>& params, const std::vector<float>& grads) {
        if (params.size() != grads.size() || params.size() != m.size() || params.size() != v.size()) return false;
        ++t;
        vr_cpp::check(vr_adam_step(params.data(), grads.data(), m.data(), v.data(), params.size(), t, lr, beta1, beta2, eps));
        return true;
    }
    void reset_state() {
        std::fill(m.begin(), m.end(), 0.0f);
        std::fill(v.begin(), v.end(), 0.0f);
        t = 0;
    }
    size_t dim() const { return m.size(); }

private:
    std::vector<float> m, v;
    float lr, beta1, beta2, eps;
    int t;
};

// ---------------------------------------------------------------------------------------------
// integrator.h:49-57 and the device integrators
// ---------------------------------------------------------------------------------------------
class Integrator {
protected:
    const std::shared_ptr<Camera> camera;

public:
    Integrator(const std::shared_ptr<Camera>& camera) : camera(camera) {}
    virtual ~Integrator() = default;
    virtual void render(const Scene& scene, Image& image) = 0;
};

// The device integrators render on every visible GPU by default, as the reference's render uses
// every CPU core (OpenMP): one GPU renders on its own; several split the frame's tiles and gather
// over RCCL (vr_init_multi). set_devices() picks the GPUs explicitly (a device
// listed more than once rehearses the split on one GPU); the `dev` constructor argument pins one GPU.
class HipIntegrator : public Integrator {
protected:
    vr_render_params params_{};
    int device_ = -1;            // >= 0: this one GPU
    std::vector<int> devices_;   // explicit device list (multi-GPU context, even for one device)

public:
    HipIntegrator(const std::shared_ptr<Camera>& camera, int integrator, float step_size, int env_samples, int dev)
        : Integrator(camera), device_(dev) {
        params_.integrator = integrator;
        params_.step_size = step_size;
        params_.env_samples = env_samples;
        params_.t_eps = 0.0f;
        params_.flags = 0;
    }
    void set_t_eps(float t) { params_.t_eps = t; }
    void set_devices(const std::vector<int>& devs) { devices_ = devs; }
    const vr_render_params& params() const { return params_; }
    vr_ctx* context() const {
        if (!devices_.empty()) return vr_cpp::device_group(devices_);
        if (device_ >= 0) return vr_cpp::device(device_);
        const int n = vr_cpp::device_count();
        if (n <= 1) return vr_cpp::device(0);
        std::vector<int> all(n);
        for (int i = 0; i < n; ++i) all[i] = i;
        return vr_cpp::device_group(all);
    }
    void render(const Scene& scene, Image& image) override {
        vr_ctx* ctx = context();
        upload(ctx, scene);
        vr_cpp::check(vr_render(ctx, &camera->state(), &params_, image.get_width(), image.get_height(), image.data()));
    }
    // re-upload when the scene (or the scene object) changed since the last upload to this context
    static void upload(vr_ctx* ctx, const Scene& scene) {
        vr_scene* ns = scene.native();
        std::lock_guard<std::mutex> lock(upload_mutex());
        auto& uploaded = upload_cache();
        auto it = uploaded.find(ctx);
        if (it == uploaded.end() || it->second.first != (const void*)ns || it->second.second != scene.native_version()) {
            vr_cpp::check(vr_upload_scene(ctx, ns));
            uploaded[ctx] = {ns, scene.native_version()};
        }
    }
    // a context's scene was replaced behind upload()'s back (vr_sfd_optimize re-uploads): forget it
    static void forget(vr_ctx* ctx) {
        std::lock_guard<std::mutex> lock(upload_mutex());
        upload_cache().erase(ctx);
    }

private:
    static std::mutex& upload_mutex() {
        static std::mutex mu;
        return mu;
    }
    static std::map<vr_ctx*, std::pair<const void*, uint64_t>>& upload_cache() {  // per device context
        static std::map<vr_ctx*, std::pair<const void*, uint64_t>> uploaded;
        return uploaded;
    }

public:
    vr_render_stats stats() const {
        vr_render_stats s{};
        vr_cpp::check(vr_get_stats(context(), &s));
        return s;
    }
};

// test_integrators.h:143-158 — RayMarchingGaussians(camera, step_size = 0.01, env_samples = 20)
class RayMarchingGaussians : public HipIntegrator {
public:
    RayMarchingGaussians(const std::shared_ptr<Camera>& camera, float step_size = 0.01f, int env_samples = 20,
                         int dev = -1)
        : HipIntegrator(camera, VR_RAYMARCH_GAUSSIANS, step_size, env_samples, dev) {}
};

// integrator.h:100-142 — PureRayMarching(camera, step_size = 0.01, env_samples = 20)
class PureRayMarching : public HipIntegrator {
public:
    PureRayMarching(const std::shared_ptr<Camera>& camera, float step_size = 0.01f, int env_samples = 20, int dev = -1)
        : HipIntegrator(camera, VR_PURE_RAYMARCH, step_size, env_samples, dev) {}
};

// test_integrators.h:11-21 — RayMarchingSpheres(camera, step_size = 0.01, env_samples = 5)
class RayMarchingSpheres : public HipIntegrator {
public:
    RayMarchingSpheres(const std::shared_ptr<Camera>& camera, float step_size = 0.01f, int env_samples = 5, int dev = -1)
        : HipIntegrator(camera, VR_RAYMARCH_SPHERES, step_size, env_samples, dev) {}
};

// integrator.h:273-408 — FreeFlightGaussians(camera, num_samples = 256)
class FreeFlightGaussians : public HipIntegrator {
public:
    FreeFlightGaussians(const std::shared_ptr<Camera>& camera, int num_samples = 256, int dev = -1)
        : HipIntegrator(camera, VR_FREE_FLIGHT, 0.01f, 0, dev) {
        params_.num_samples = num_samples;
    }
};

// integrator.h:416-720 — MultiScatterGaussians(camera, samples = 16, min_bounces = 5)
class MultiScatterGaussians : public HipIntegrator {
public:
    MultiScatterGaussians(const std::shared_ptr<Camera>& camera, int samples = 16, int min_bounces = 5, int dev = -1)
        : HipIntegrator(camera, VR_MULTI_SCATTER, 0.01f, 0, dev) {
        params_.num_samples = samples;
        params_.min_bounces = min_bounces;
    }
    void set_num_samples(int n) { params_.num_samples = n; }  // integrator.h:719
    using HipIntegrator::render;
    // integrator.h:532-536 with RECORD_PIXEL_GAUSSIANS: per_pixel_gaussians[y * W + x] receives the
    // sorted indices of the Gaussians recorded at that pixel (integrator.h:616-644, 700-705).
    void render(const Scene& scene, Image& image, std::vector<std::vector<uint32_t>>* per_pixel_gaussians) {
        if (!per_pixel_gaussians) return render(scene, image);
        vr_ctx* ctx = context();
        upload(ctx, scene);
        vr_cpp::check(vr_render_record(ctx, &camera->state(), &params_, image.get_width(), image.get_height(), image.data(), 0));
        const size_t npix = (size_t)image.get_width() * image.get_height(), n = scene.get_num_primitives();
        const size_t words = (n + 31) / 32;
        std::vector<uint32_t> bits(words * npix);
        vr_cpp::check(vr_get_pixel_gaussians(ctx, 0, bits.data(), bits.size()));
        per_pixel_gaussians->assign(npix, {});
        for (size_t w = 0; w < words; ++w)
            for (size_t p = 0; p < npix; ++p)
                for (uint32_t b = bits[w * npix + p]; b; b &= b - 1)
                    (*per_pixel_gaussians)[p].push_back((uint32_t)(32 * w + __builtin_ctz(b)));
    }
    int num_samples() const { return params_.num_samples; }
};

// ---------------------------------------------------------------------------------------------
// inverse_integrator.h:34-246 — the stochastic finite-difference inverse loop (vr_sfd_optimize)
// ---------------------------------------------------------------------------------------------
class InverseIntegrator {
protected:
    const std::shared_ptr<Camera> camera;

public:
    InverseIntegrator(const std::shared_ptr<Camera>& camera) : camera(camera) {}
    virtual ~InverseIntegrator() = default;
    virtual bool optimize(Scene scene_initial, const Image& I_ref) = 0;
};

// inverse_integrator.h:52-57, plus the run's sign-vector seed, final-render samples (:230) and image
// directory (the reference writes ./sfd_output; "" writes nothing)
struct SFDDConfig {
    int max_iters = 1000;
    int save_every = 25;
    int num_stoch_samples = 4;
    float lr = 1e-2f;
    uint64_t seed = 0;
    int final_samples = 16384;
    std::string out_dir = "./sfd_output";
};

class StochasticFiniteDiffInverseIntegrator : public InverseIntegrator {
public:
    StochasticFiniteDiffInverseIntegrator(const std::shared_ptr<Camera>& cam,
                                          const std::shared_ptr<MultiScatterGaussians>& forward_integrator,
                                          const SFDDConfig& cfg = SFDDConfig())
        : InverseIntegrator(cam), forward_integrator(forward_integrator), cfg(cfg) {}

    bool optimize(Scene scene_initial, const Image& I_ref) override {
        const size_t n = scene_initial.get_num_primitives();
        if (n == 0) return false;  // "Scene has no GMM." (:71-74)
        params_.assign(11 * n, 0.0f);
        history_.assign(std::max(cfg.max_iters, 0), 0.0);
        grads_.assign(11 * n, 0.0);
        final_image_ = Image(I_ref.get_width(), I_ref.get_height());
        vr_sfd_config c{cfg.max_iters, cfg.save_every, cfg.num_stoch_samples, cfg.lr, cfg.seed, cfg.final_samples,
                        cfg.out_dir.c_str()};
        vr_sfd_result r{params_.data(), history_.data(), grads_.data(), final_image_.data(), 0.0};
        if (!cfg.out_dir.empty()) std::filesystem::create_directories(cfg.out_dir);
        vr_ctx* ctx = forward_integrator->context();
        vr_status st = vr_sfd_optimize(ctx, &camera->state(), &forward_integrator->params(), scene_initial.native(),
                                       I_ref.data(), I_ref.get_width(), I_ref.get_height(), &c, &r);
        HipIntegrator::forget(ctx);  // the context now holds the last parameter set
        if (st != VR_OK) {
            std::cerr << "[SFD] " << vr_last_error() << std::endl;
            return false;
        }
        final_loss_ = r.final_loss;
        if (cfg.final_samples > 0) forward_integrator->set_num_samples(cfg.final_samples);  // as the reference leaves it
        return true;
    }
    const std::vector<float>& parameters() const { return params_; }
    const std::vector<double>& loss_history() const { return history_; }
    const std::vector<double>& last_gradients() const { return grads_; }
    double final_loss() const { return final_loss_; }
    const Image& final_image() const { return final_image_; }

private:
    std::shared_ptr<MultiScatterGaussians> forward_integrator;
    SFDDConfig cfg;
    std::vector<float> params_;
    std::vector<double> history_, grads_;
    double final_loss_ = -1.0;
    Image final_image_{1, 1};
};

// integrator.h:65-94 — TestIntegrator(camera)
class TestIntegrator : public HipIntegrator {
public:
    TestIntegrator(const std::shared_ptr<Camera>& camera, int dev = -1)
        : HipIntegrator(camera, VR_TEST_HITMASK, 0.01f, 0, dev) {}
};
