// Host-side internals of libvr_hip.so (not part of the public ABI).
#pragma once
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

#include "../../../include/vr_hip.h"
#include "../vr_internal.h"

namespace vr {

// Error channel: every C entry point funnels failures through fail(), which records a
// thread-local message for vr_last_error() and returns the status.
vr_status fail(vr_status st, const std::string& msg);
void clear_error();

// Precomputed per-Gaussian quantities (gaussian.h:52-55), in scene order.
struct GaussianPre {
    float mean[3];
    float density;
    float inv_cov[6];  // 00 01 02 11 12 22
    float norm;
    float albedo;
    float cov[6];      // input covariance (for bounds)
};

// Host scene.
struct HostScene {
    int32_t type = VR_VOLUME_GAUSSIANS;
    std::vector<vr_gaussian> gaussians;
    std::vector<GaussianPre> pre;
    std::vector<vr_sphere> spheres;
    std::vector<vr_light> lights;
    float env[3] = {0.53f, 0.81f, 0.92f};  // scene.h:29
};

GaussianPre precompute_gaussian(const vr_gaussian& g);
void gaussian_bounds(const GaussianPre& g, float bmin[3], float bmax[3]);
void sphere_bounds(const vr_sphere& s, float bmin[3], float bmax[3]);

// BVH over primitive boxes. Output: child-pair nodes + primitive order (leaf-contiguous).
struct BVHBuild {
    std::vector<BVHNode> nodes;
    std::vector<uint32_t> order;  // order[j] = scene index of the j-th primitive in leaf order
    int max_depth = 0;
};
BVHBuild build_bvh(const std::vector<float>& boxes /* 6 per prim: min xyz, max xyz */);

// Iterated float step sequence t_0 = 0, t_{k+1} = t_k + step (test_integrators.h:184,289).
std::vector<float> step_table(float step, float t_max);

}  // namespace vr

struct vr_scene {
    vr::HostScene s;
};

// Multi-GPU group behind a vr_init_multi context (host/vr_multi.cpp).
struct vr_group;
namespace vr {
// Runs fn(i) for every i in [0, n) on a host thread of its own (n == 1: on the calling thread); the
// first failure's status wins, its message prefixed by label(i).
template <class F, class L>
vr_status run_parallel(int n, F fn, L label) {
    if (n == 1) return fn(0);
    std::vector<vr_status> st(n, VR_OK);
    std::vector<std::string> msg(n);
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            st[i] = fn(i);
            if (st[i] != VR_OK) msg[i] = vr_last_error();
        });
    for (auto& t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (st[i] != VR_OK) return fail(st[i], label(i) + ": " + msg[i]);
    return VR_OK;
}
// The device contexts behind a context: its group's ranks (vr_init_multi), or the context itself.
int ctx_ranks(vr_ctx* c);
vr_ctx* ctx_rank(vr_ctx* c, int r);
vr_status group_create(int ndev, const int* devices, vr_group** out);
void group_destroy(vr_group* g);
int group_size(const vr_group* g);
vr_ctx* group_rank(vr_group* g, int rank);
bool group_uses_rccl(const vr_group* g);
vr_status group_upload(vr_group* g, const vr_scene* s);
vr_status group_render(vr_group* g, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H, float* rgb);
vr_status group_set_option(vr_group* g, int32_t option, int64_t value);
vr_status group_synchronize(vr_group* g);
vr_status group_stats(vr_group* g, vr_render_stats* out);
// device side of the inverse loop (host/vr_device.cpp)
vr_status sfd_set_reference(vr_ctx* c, const float* I_ref, uint32_t W, uint32_t H);
vr_status sfd_render(vr_ctx* c, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H, int32_t slot,
                     int which, float* loss_host, float* rgb);
vr_status sfd_loss_diff_device(vr_ctx* c, uint32_t npix, double* out, size_t n);
}  // namespace vr
