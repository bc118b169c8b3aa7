// integrator.h — C++ mirror of the reference's include/integrator.h over the C ABI (include/vr_hip.h).
#pragma once
#include "camera.h"
#include "image.h"
#include "scene.h"
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
    int solver_ = -1;            // free-flight integrators: VR_OPT_FF_SOLVER set before each render

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
        apply_solver(ctx);
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
    void apply_solver(vr_ctx* ctx) const {
        if (solver_ >= 0) vr_cpp::check(vr_set_option(ctx, VR_OPT_FF_SOLVER, solver_));
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

// integrator.h:100-142 — PureRayMarching(camera, step_size = 0.01, env_samples = 20)
class PureRayMarching : public HipIntegrator {
public:
    PureRayMarching(const std::shared_ptr<Camera>& camera, float step_size = 0.01f, int env_samples = 20, int dev = -1)
        : HipIntegrator(camera, VR_PURE_RAYMARCH, step_size, env_samples, dev) {}
};

// distance_solvers.h:143-147: the reference picks one of these with a #define (ANALYTIC_PLUS_NEWTON
// compiled in); here a run-time choice per free-flight integrator (VR_OPT_FF_SOLVER). UNIFORM draws
// from a seeded PCG32 stream instead of rand01()'s random_device (include/vr_hip.h).
enum DistanceSolver { ANALYTIC_PLUS_NEWTON = 0, BISECTION = 1, NEWTON = 2, ANALYTIC_PLUS_BISECTION = 3, UNIFORM = 4 };

// integrator.h:273-408 — FreeFlightGaussians(camera, num_samples = 256)
class FreeFlightGaussians : public HipIntegrator {
public:
    FreeFlightGaussians(const std::shared_ptr<Camera>& camera, int num_samples = 256, int dev = -1)
        : HipIntegrator(camera, VR_FREE_FLIGHT, 0.01f, 0, dev) {
        params_.num_samples = num_samples;
        solver_ = ANALYTIC_PLUS_NEWTON;
    }
    void set_distance_solver(DistanceSolver s) { solver_ = (int)s; }
};

// integrator.h:416-720 — MultiScatterGaussians(camera, samples = 16, min_bounces = 5)
class MultiScatterGaussians : public HipIntegrator {
public:
    MultiScatterGaussians(const std::shared_ptr<Camera>& camera, int samples = 16, int min_bounces = 5, int dev = -1)
        : HipIntegrator(camera, VR_MULTI_SCATTER, 0.01f, 0, dev) {
        params_.num_samples = samples;
        params_.min_bounces = min_bounces;
        solver_ = ANALYTIC_PLUS_NEWTON;
    }
    void set_num_samples(int n) { params_.num_samples = n; }  // integrator.h:719
    void set_distance_solver(DistanceSolver s) { solver_ = (int)s; }
    using HipIntegrator::render;
    // integrator.h:532-536 with RECORD_PIXEL_GAUSSIANS: per_pixel_gaussians[y * W + x] receives the
    // sorted indices of the Gaussians recorded at that pixel (integrator.h:616-644, 700-705).
    void render(const Scene& scene, Image& image, std::vector<std::vector<uint32_t>>* per_pixel_gaussians) {
        if (!per_pixel_gaussians) return render(scene, image);
        vr_ctx* ctx = context();
        upload(ctx, scene);
        apply_solver(ctx);
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

// integrator.h:65-94 — TestIntegrator(camera)
class TestIntegrator : public HipIntegrator {
public:
    TestIntegrator(const std::shared_ptr<Camera>& camera, int dev = -1)
        : HipIntegrator(camera, VR_TEST_HITMASK, 0.01f, 0, dev) {}
};

