// scene.h — C++ mirror of the reference's include/scene.h over the C ABI (include/vr_hip.h).
#pragma once
#include <optional>

#include "gmm.h"
#include "smm.h"
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

