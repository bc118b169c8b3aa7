// gaussian.h — C++ mirror of the reference's include/gaussian.h over the C ABI (include/vr_hip.h).
#pragma once
#include "runtime.h"
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

