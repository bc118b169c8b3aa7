// inverse_integrator.h — C++ mirror of the reference's include/inverse_integrator.h over the C ABI (include/vr_hip.h).
#pragma once
#include <filesystem>
#include <iostream>

#include "integrator.h"
#include "optimizer.h"
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

