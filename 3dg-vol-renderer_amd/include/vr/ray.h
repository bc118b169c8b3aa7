// ray.h — C++ mirror of the reference's include/ray.h over the C ABI (include/vr_hip.h).
#pragma once
#include "runtime.h"
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

