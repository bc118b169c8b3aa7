// Linear-algebra types of the host API.
//
// The reference's public API is written in Eigen types (Eigen::Vector3f, Eigen::Vector2d,
// Eigen::Matrix3f). When Eigen is available these headers use it unchanged, so reference code
// such as tests/main.cpp compiles against them. This image has no Eigen (the reference's
// extern/eigen-3.4.0 submodule is empty), so a minimal subset with the same names, operations and
// 3-term evaluation order (e0 + (e1 + e2)) is provided instead. Rendering never depends on these
// types: geometry is computed inside libvr_hip.so.
#pragma once

#if __has_include(<Eigen/Core>) && !defined(VR_NO_EIGEN)
#include <Eigen/Core>
#include <Eigen/Geometry>
#define VR_HAVE_EIGEN 1
#else
#include <algorithm>
#include <cmath>
#include <initializer_list>

namespace Eigen {

struct Vector3f {
    float v[3] = {0.0f, 0.0f, 0.0f};
    Vector3f() = default;
    Vector3f(float x, float y, float z) : v{x, y, z} {}
    static Vector3f Zero() { return {0.0f, 0.0f, 0.0f}; }
    static Vector3f Ones() { return {1.0f, 1.0f, 1.0f}; }
    static Vector3f Constant(float c) { return {c, c, c}; }
    float& x() { return v[0]; }
    float& y() { return v[1]; }
    float& z() { return v[2]; }
    float x() const { return v[0]; }
    float y() const { return v[1]; }
    float z() const { return v[2]; }
    float& operator[](int i) { return v[i]; }
    float operator[](int i) const { return v[i]; }
    float& operator()(int i) { return v[i]; }
    float operator()(int i) const { return v[i]; }
    float* data() { return v; }
    const float* data() const { return v; }
    Vector3f operator+(const Vector3f& o) const { return {v[0] + o.v[0], v[1] + o.v[1], v[2] + o.v[2]}; }
    Vector3f operator-(const Vector3f& o) const { return {v[0] - o.v[0], v[1] - o.v[1], v[2] - o.v[2]}; }
    Vector3f operator-() const { return {-v[0], -v[1], -v[2]}; }
    Vector3f operator*(float s) const { return {v[0] * s, v[1] * s, v[2] * s}; }
    Vector3f operator/(float s) const { return {v[0] / s, v[1] / s, v[2] / s}; }
    Vector3f& operator+=(const Vector3f& o) { return *this = *this + o; }
    Vector3f& operator-=(const Vector3f& o) { return *this = *this - o; }
    Vector3f& operator*=(float s) { return *this = *this * s; }
    Vector3f& operator/=(float s) { return *this = *this / s; }
    float dot(const Vector3f& o) const { return v[0] * o.v[0] + (v[1] * o.v[1] + v[2] * o.v[2]); }
    float squaredNorm() const { return dot(*this); }
    float norm() const { return std::sqrt(squaredNorm()); }
    Vector3f normalized() const {
        float z = squaredNorm();
        return z > 0.0f ? *this / std::sqrt(z) : *this;
    }
    Vector3f cross(const Vector3f& r) const {
        return {v[1] * r.v[2] - v[2] * r.v[1], v[2] * r.v[0] - v[0] * r.v[2], v[0] * r.v[1] - v[1] * r.v[0]};
    }
    Vector3f cwiseProduct(const Vector3f& o) const { return {v[0] * o.v[0], v[1] * o.v[1], v[2] * o.v[2]}; }
    Vector3f cwiseMin(const Vector3f& o) const {
        return {std::min(v[0], o.v[0]), std::min(v[1], o.v[1]), std::min(v[2], o.v[2])};
    }
    Vector3f cwiseMax(const Vector3f& o) const {
        return {std::max(v[0], o.v[0]), std::max(v[1], o.v[1]), std::max(v[2], o.v[2])};
    }
    Vector3f cwiseAbs() const { return {std::fabs(v[0]), std::fabs(v[1]), std::fabs(v[2])}; }
    float maxCoeff() const { return std::max(v[0], std::max(v[1], v[2])); }
    float minCoeff() const { return std::min(v[0], std::min(v[1], v[2])); }
    bool operator==(const Vector3f& o) const { return v[0] == o.v[0] && v[1] == o.v[1] && v[2] == o.v[2]; }
};
inline Vector3f operator*(float s, const Vector3f& a) { return {s * a.v[0], s * a.v[1], s * a.v[2]}; }

struct Vector2d {
    double v[2] = {0.0, 0.0};
    Vector2d() = default;
    Vector2d(double x, double y) : v{x, y} {}
    double& x() { return v[0]; }
    double& y() { return v[1]; }
    double x() const { return v[0]; }
    double y() const { return v[1]; }
};

struct Matrix3f {
    float m[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    static Matrix3f Zero() { return Matrix3f(); }
    static Matrix3f Identity() {
        Matrix3f r;
        r.m[0][0] = r.m[1][1] = r.m[2][2] = 1.0f;
        return r;
    }
    float& operator()(int i, int j) { return m[i][j]; }
    float operator()(int i, int j) const { return m[i][j]; }
    Matrix3f transpose() const {
        Matrix3f r;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) r.m[i][j] = m[j][i];
        return r;
    }
    Vector3f operator*(const Vector3f& x) const {
        return {m[0][0] * x[0] + (m[0][1] * x[1] + m[0][2] * x[2]), m[1][0] * x[0] + (m[1][1] * x[1] + m[1][2] * x[2]),
                m[2][0] * x[0] + (m[2][1] * x[1] + m[2][2] * x[2])};
    }
    // comma initializer: cov << a, b, c, d, e, f, g, h, i;
    struct Comma {
        Matrix3f& M;
        int k;
        Comma& operator,(float x) {
            M.m[k / 3][k % 3] = x;
            ++k;
            return *this;
        }
    };
    Comma operator<<(float x) {
        m[0][0] = x;
        return Comma{*this, 1};
    }
};

}  // namespace Eigen
#endif
