// test_integrators.h — C++ mirror of the reference's include/test_integrators.h over the C ABI (include/vr_hip.h).
#pragma once
#include "integrator.h"
// test_integrators.h:143-158 — RayMarchingGaussians(camera, step_size = 0.01, env_samples = 20)
class RayMarchingGaussians : public HipIntegrator {
public:
    RayMarchingGaussians(const std::shared_ptr<Camera>& camera, float step_size = 0.01f, int env_samples = 20,
                         int dev = -1)
        : HipIntegrator(camera, VR_RAYMARCH_GAUSSIANS, step_size, env_samples, dev) {}
};

// test_integrators.h:11-21 — RayMarchingSpheres(camera, step_size = 0.01, env_samples = 5)
class RayMarchingSpheres : public HipIntegrator {
public:
    RayMarchingSpheres(const std::shared_ptr<Camera>& camera, float step_size = 0.01f, int env_samples = 5, int dev = -1)
        : HipIntegrator(camera, VR_RAYMARCH_SPHERES, step_size, env_samples, dev) {}
};

