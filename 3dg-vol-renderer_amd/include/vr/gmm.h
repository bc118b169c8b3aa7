// gmm.h — C++ mirror of the reference's include/gmm.h over the C ABI (include/vr_hip.h).
#pragma once
#include <memory>
#include <vector>

#include "gaussian.h"
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
    std::unique_ptr<vr_scene, void (*)(vr_scene*)> built(out, &vr_scene_destroy);
    std::vector<vr_gaussian> g(gmm.gaussians.size());
    vr_cpp::check(vr_scene_get_gaussians(out, g.data(), g.size()));
    for (size_t i = 0; i < g.size(); ++i) gmm.gaussians[i] = Gaussian::from_record(g[i]);
}

// gmm.h:678-706
inline std::vector<float> make_default_eps_for_params(const std::vector<float>& base_params) {
    std::vector<float> eps(base_params.size());
    vr_cpp::check(vr_gmm_default_eps(eps.data(), eps.size()));
    return eps;
}

