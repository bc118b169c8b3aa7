// camera.h — C++ mirror of the reference's include/camera.h over the C ABI (include/vr_hip.h).
#pragma once
#include <memory>

#include "ray.h"
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

