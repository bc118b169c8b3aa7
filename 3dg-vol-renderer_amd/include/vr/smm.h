// smm.h — C++ mirror of the reference's include/smm.h over the C ABI (include/vr_hip.h).
#pragma once
#include "runtime.h"
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

