// Device context: scene upload (BVH build + HBM layout), step tables, launch and statistics.
// Host C++ over the HIP runtime; the kernels live in kernels/vr_gauss.hip (RayMarchingGaussians
// wavefront pipeline) and kernels/vr_spheres.hip (RayMarchingSpheres, TestIntegrator, unshuffle).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <map>
#include <mutex>

#include "vr_common.h"
#include "../vr_lbvh.h"

namespace vr {
hipError_t launch_render(const RenderArgs& A, hipStream_t stream, int volume_type, int integrator);
hipError_t gauss_march(const RenderArgs& A, hipStream_t stream, bool stats);
hipError_t gauss_secondary(const RenderArgs& A, hipStream_t stream, bool stats);
hipError_t gauss_accumulate(const RenderArgs& A, hipStream_t stream);
hipError_t launch_free_flight(const RenderArgs& A, uint32_t chunk_tiles, hipStream_t stream, hipEvent_t* ev);
uint32_t free_flight_threads(int cus);
hipError_t launch_sfd_loss_diff(const uint32_t* bits0, const uint32_t* bits1, const float* lb, const float* lp, uint32_t npix,
                                uint32_t n, double* out, hipStream_t stream);
hipError_t gauss_record_cut(const RenderArgs& A, float budget, hipStream_t stream);
hipError_t gauss_whiten(const GaussianRecord* rec, WRecord* out, uint32_t n, uint32_t* bad, hipStream_t stream);
hipError_t gauss_bin(const RenderArgs& A, bool emit, hipStream_t stream);
hipError_t gauss_parents(const HNode4* nodes, uint32_t n, int32_t* parent, int32_t* prim_node, hipStream_t stream);
hipError_t gauss_soa_nodes(const HNode4* src, HNode4* dst, uint32_t n, hipStream_t stream);
hipError_t gauss_refit_secondary(const HNode4* src, HNode4* dst, HNode4* dst_t, uint32_t n, const GaussianRecord* rec, const int32_t* parent,
                                 uint8_t* depth, float* nbox, uint32_t* maxd, const float hc[3], float hs, float diag,
                                 hipStream_t stream);
hipError_t gauss_bin_scan(const uint32_t* cnt, uint32_t* off, uint32_t n, void* tmp, size_t& tmp_bytes, hipStream_t stream);
hipError_t launch_pixel_losses(const float* img, const float* ref, uint32_t npix, float* out, hipStream_t stream);

hipError_t launch_unshuffle(const float* slabs, uint32_t nslabs, uint32_t tiles_per_slab, uint32_t tiles_x, uint32_t W,
                            uint32_t H, float* img, hipStream_t stream);
hipError_t launch_unshuffle_part(const float* slabs, uint32_t first, uint32_t nslabs, uint32_t stride, uint32_t tiles_per_slab,
                                 uint32_t tiles_x, uint32_t W, uint32_t H, float* img, hipStream_t stream);
}  // namespace vr

using namespace vr;

// Pinned report of a frame's counts (launch): [0] fallback queue, [1] error pixels, [2..4] rec_alloc (records,
// overflow-pool words, capacity exceeded), [5] deep queue, [6..7] counters 2..3 (free-flight fallback paths,
// shadow-ray queue need), [8] exact slow-path queue, [9] band fix-up queue.
constexpr int kReportWords = 10;
struct vr_ctx {
    int device = 0;
    hipStream_t stream = nullptr;  // used by the synchronous vr_render
    // scene
    bool has_scene = false;
    int32_t type = VR_VOLUME_GAUSSIANS;
    int32_t num_prims = 0;
    GaussianRecord* d_gauss = nullptr;
    WRecord* d_wrec = nullptr;  // whitened copy (secondary rays)
    bool wrec_pd = true;        // every record's M is positive definite (else the secondary rays use the M forms)
    BVHNode* d_nodes = nullptr;
    HNode* d_hnodes = nullptr;
    HNode4* d_hnodes4 = nullptr;
    HNode4* d_hnodes4s = nullptr;  // the secondary rays' copy with tight boxes (VR_OPT_SEC_TIGHT)
    HNode4* d_hnodes4w = nullptr;  // d_hnodes4 laid out per axis (the 4-wide walks' node tests, wide_children)
    int32_t* d_parent4 = nullptr;  // parent of every HNode4 (the secondary rays' climb out of their start subtree)
    int32_t* d_prim_node4 = nullptr;  // the HNode4 whose child is each record's leaf (record starts)
    size_t num_nodes4 = 0;
    float hn_center[3] = {0, 0, 0}, hn_scale = 1.0f;
    float sig_max[3] = {0, 0, 0};  // largest per-axis standard deviation of any Gaussian
    SphereRecord* d_spheres = nullptr;
    std::vector<LightRecord> lights;
    float env[3] = {0, 0, 0};
    float bmin[3] = {0, 0, 0}, bmax[3] = {0, 0, 0};
    int bvh_depth = 0;
    size_t num_nodes = 0;
    // step tables keyed by step size
    struct Table {
        float* d = nullptr;
        int n = 0;
        float tmax = 0;
    };
    std::map<uint32_t, Table> tables;
    // workspaces
    uint32_t* d_queue = nullptr;
    uint32_t queue_cap = 0;
    uint32_t* d_counters = nullptr;  // [0] error pixels / paths of the frame
    // Pinned report of the last frame, copied on the render stream after its last kernel:
    // [0] fallback-queue length, [1] error pixels, [2] scatter records, [3] overflow-pool entries,
    // [4] record capacity exceeded (the frame is invalid and must be rendered again), [5] deep-pass
    // pixels, [6] free-flight paths re-run in ff_fallback_kernel, [7] free-flight: the most shadow rays
    // one launch tried to queue
    uint32_t* h_report = nullptr;  // kReportWords words: see launch()
    bool report_gauss = false;  // the last frame ran the RayMarchingGaussians pipeline (fields [2..4])
    uint64_t report_pixels = 0; // pixels of that frame (its march)
    bool march_big = false;     // this scene's frames overflow the primary march's 16 slots often: kActBig (reset at upload)
    float* d_frame = nullptr;
    size_t frame_cap = 0;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    hipEvent_t ev_report = nullptr;  // after the frame report's copies (collect() waits for it)
    hipEvent_t ev_stage[3] = {nullptr, nullptr, nullptr};  // stage boundaries of gauss_pipeline
    bool staged = false;                                   // last launch recorded ev_stage
    // free-flight frames: per launch, events before the path kernel, after it, after the shadow-ray
    // kernel and after the accumulation (stage_ms of vr_get_stats sums them over the frame's launches)
    std::vector<hipEvent_t> ff_ev;
    uint32_t ff_launches = 0;
    bool stats_pending = false;  // h_report of the last frame has not been collected yet
    bool sync_pending = false;   // the last frame's outcome (retry / overflow) is collected but not yet reported by
                                 // vr_synchronize: sticky, whoever collected it (vr_get_stats, an upload, ...)
    int64_t last_pixels = 0;
    uint32_t last_first_tile = 0, last_tile_stride = 1, last_tiles_x = 1, last_w = 0, last_h = 0;  // tile map of the last frame
    uint32_t last_secondary_per_record = 0;
    // wavefront pipeline buffers (grown on demand, never shrunk)
    struct Buf {
        void* p = nullptr;
        size_t bytes = 0;
    };
    Buf px_first, px_T, rec_pos, rec_meta, rec_next, rec_act, tr, rec_rad, rec_alloc, rec_bloom, slowq, fixq;
    Buf pcg_jump, ray_next, stack_ovf, env_order, env_base, rec_cut, rec_start;
    Buf deep;  // march_deep_kernel: pixel queue + global active lists (vr_gauss.hip)
    Buf bin_cnt, bin_off, bin_ent;  // tile bins of the binned march (VR_OPT_MARCH_BINNED)
    Buf ff_scratch, ff_tail, ff_sum, ff_nee;  // free-flight integrators (vr_freeflight.hip)
    Buf ff_fb;                                // ff_fallback_kernel: path queue + kFFBigCap rows
    uint32_t* d_order = nullptr;      // record (leaf order) -> scene index
    Buf rec_bits[2];                  // RECORD_PIXEL_GAUSSIANS bitsets (vr_render_record slots)
    uint32_t rec_npix[2] = {0, 0}, rec_n[2] = {0, 0};
    Buf sfd_tmp;                      // vr_sfd_loss_diff: losses + output
    Buf sfd_ref, sfd_loss[2], sfd_out;  // device inverse loop (vr_sfd_optimize): I_ref, base / perturbed losses
    int pcg_jump_n = -1;
    uint32_t* h_sizing = nullptr;  // pinned copy of rec_alloc for the sizing march of a context's first frame
    uint64_t rec_hint = 0, ovf_hint = 0;  // record / overflow-pool capacities (0: not known yet)
    uint64_t slow_hint = 0;               // exact slow-path queue: the most rays an earlier frame queued (+ 1/8)
    uint64_t fix_hint = 0;                // band fix-up queue (secondary_fix_kernel): the same
    uint64_t nee_hint = 0;                // deferred-NEE queue capacity from earlier free-flight frames (0: not known)
    uint32_t last_nee_cap = 0, last_nee_bound = 0;  // the last free-flight frame's queue capacity and its bound
    // A launch found the shadow-ray queue full at its VR_OPT_FF_NEE_QUEUE bound: the frame is reported
    // (VR_ERR_RETRY) and this context's later frames trace every shadow ray inline — the queue's own walk and
    // sums, so the same frame bit for bit as a queue with room — until the next upload or option change.
    bool nee_inline = false;
    bool report_ff = false;               // the last frame ran the free-flight pipeline (h_report[7])
    // vr_set_option values (explicit per-context tuning; no environment variables are read)
    int64_t opt_half_nodes = 1;        // VR_OPT_HALF_NODES
    int64_t opt_secondary_budget = 1;  // VR_OPT_SECONDARY_BUDGET
    int64_t opt_ff_window0 = 0;        // VR_OPT_FF_WINDOW0 (0: auto_window0)
    int32_t auto_window0 = 8;          // first hit-window capacity derived from the uploaded scene
    int32_t auto_nee_refill = 40;      // shadow-ray kernel refill threshold derived from the uploaded scene
    int64_t opt_ff_kernel = 0;         // VR_OPT_FF_KERNEL (0: auto_ff_sm)
    bool auto_ff_sm = false;           // the uploaded scene's free-flight paths take the phase-scheduled kernel
    int64_t opt_ff_nee_queue = 6;      // VR_OPT_FF_NEE_QUEUE
    int64_t opt_device_bvh = 0;        // VR_OPT_DEVICE_BVH
    int64_t opt_march_binned = 0;      // VR_OPT_MARCH_BINNED
    int64_t opt_ff_solver = 0;         // VR_OPT_FF_SOLVER
    int64_t opt_start_subtree = 1;     // VR_OPT_START_SUBTREE
    int64_t opt_sec_tight = 1;         // VR_OPT_SEC_TIGHT (next upload)
    int64_t opt_march_wide_min = 2048;  // VR_OPT_MARCH_WIDE_MIN
    bool last_upload_device_bvh = false;  // the current scene's tree came from the device builder
    vr_group* group = nullptr;         // vr_init_multi: the devices this context drives (host/vr_multi.cpp)
};

// Single-device entry points called on a multi-GPU context act on its first device.
static inline vr_ctx* first_device(vr_ctx* c) { return (c && c->group) ? vr::group_rank(c->group, 0) : c; }
namespace vr {
int ctx_ranks(vr_ctx* c) { return (c && c->group) ? group_size(c->group) : 1; }
vr_ctx* ctx_rank(vr_ctx* c, int r) { return (c && c->group) ? group_rank(c->group, r) : (r == 0 ? c : nullptr); }
}  // namespace vr

namespace {

vr_status hip_fail(hipError_t e, const char* what) {
    return fail(VR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(expr, what)                          \
    do {                                             \
        hipError_t e_ = (expr);                      \
        if (e_ != hipSuccess) return hip_fail(e_, what); \
    } while (0)

void free_scene(vr_ctx* c) {
    if (c->d_order) (void)hipFree(c->d_order);
    c->d_order = nullptr;
    if (c->d_gauss) (void)hipFree(c->d_gauss);
    if (c->d_wrec) (void)hipFree(c->d_wrec);
    c->d_wrec = nullptr;
    if (c->d_nodes) (void)hipFree(c->d_nodes);
    if (c->d_hnodes) (void)hipFree(c->d_hnodes);
    c->d_hnodes = nullptr;
    if (c->d_hnodes4) (void)hipFree(c->d_hnodes4);
    c->d_hnodes4 = nullptr;
    if (c->d_hnodes4s) (void)hipFree(c->d_hnodes4s);
    c->d_hnodes4s = nullptr;
    if (c->d_hnodes4w) (void)hipFree(c->d_hnodes4w);
    c->d_hnodes4w = nullptr;
    if (c->d_parent4) (void)hipFree(c->d_parent4);
    c->d_parent4 = nullptr;
    if (c->d_prim_node4) (void)hipFree(c->d_prim_node4);
    c->d_prim_node4 = nullptr;
    c->num_nodes4 = 0;
    if (c->d_spheres) (void)hipFree(c->d_spheres);
    c->d_gauss = nullptr;
    c->d_nodes = nullptr;
    c->d_spheres = nullptr;
    c->has_scene = false;
}

// ---- half-precision node copy for the secondary rays ----
uint16_t f16_bits(_Float16 h) {
    uint16_t b;
    std::memcpy(&b, &h, 2);
    return b;
}
double f16_to_double(uint16_t b) {
    _Float16 h;
    std::memcpy(&h, &b, 2);
    return (double)h;
}
uint16_t f16_step(uint16_t h, bool up) {  // next representable half toward +inf (up) or -inf
    const bool neg = h & 0x8000u;
    if ((h & 0x7fffu) == 0) return up ? 0x0001u : 0x8001u;
    return (uint16_t)((neg != up) ? h + 1 : h - 1);
}
uint16_t f16_directed(double v, bool up) {  // smallest half >= v (up) / largest half <= v
    if (std::isinf(v)) return v > 0 ? 0x7c00u : 0xfc00u;
    uint16_t h = f16_bits((_Float16)v);  // nearest, then stepped outward
    if (up) {
        while (f16_to_double(h) < v) h = f16_step(h, true);
    } else {
        while (f16_to_double(h) > v) h = f16_step(h, false);
    }
    return h;
}

// Builds the 32-B half-precision node copy (HNode) when the scene suits it: f16 keeps ~11 bits,
// so boxes widen by up to ~1e-3 of the scene's half extent; scenes whose leaf boxes are small
// against that (median leaf box under 3 % of the half extent) keep the f32 nodes only.
vr_status upload_half_nodes(vr_ctx* c, const std::vector<BVHNode>& nodes) {
    if (c->d_hnodes) (void)hipFree(c->d_hnodes);
    c->d_hnodes = nullptr;
    if (c->d_hnodes4) (void)hipFree(c->d_hnodes4);
    c->d_hnodes4 = nullptr;
    if (c->d_hnodes4s) (void)hipFree(c->d_hnodes4s);
    c->d_hnodes4s = nullptr;
    if (c->d_hnodes4w) (void)hipFree(c->d_hnodes4w);
    c->d_hnodes4w = nullptr;
    if (!c->opt_half_nodes) return VR_OK;
    double half = 0.0;
    for (int k = 0; k < 3; ++k) {
        c->hn_center[k] = 0.5f * (c->bmin[k] + c->bmax[k]);
        half = std::max(half, 0.5 * ((double)c->bmax[k] - (double)c->bmin[k]));
    }
    if (!(half > 0.0) || !std::isfinite(half)) return VR_OK;
    c->hn_scale = (float)(1.0 / half);
    std::vector<float> leaf_ext;
    for (const BVHNode& n : nodes)
        for (int side = 0; side < 2; ++side)
            if (n.c[side] < 0) {
                float e = 0.0f;
                for (int k = 0; k < 3; ++k) e = std::max(e, n.f[6 * side + 3 + k] - n.f[6 * side + k]);
                leaf_ext.push_back(e);
            }
    if (!leaf_ext.empty()) {
        std::nth_element(leaf_ext.begin(), leaf_ext.begin() + leaf_ext.size() / 2, leaf_ext.end());
        if (!(leaf_ext[leaf_ext.size() / 2] >= 0.03 * half)) return VR_OK;
    }
    std::vector<HNode> hn(nodes.size());
    for (size_t i = 0; i < nodes.size(); ++i) {
        for (int side = 0; side < 2; ++side) {
            for (int k = 0; k < 3; ++k) {
                const float lo = nodes[i].f[6 * side + k], hi = nodes[i].f[6 * side + 3 + k];
                const double ulo = std::isinf(lo) ? (double)lo : ((double)lo - c->hn_center[k]) * (double)c->hn_scale;
                const double uhi = std::isinf(hi) ? (double)hi : ((double)hi - c->hn_center[k]) * (double)c->hn_scale;
                hn[i].h[6 * side + k] = f16_directed(ulo, false);
                hn[i].h[6 * side + 3 + k] = f16_directed(uhi, true);
            }
            hn[i].c[side] = nodes[i].c[side];
        }
    }
    HIP_TRY(hipMalloc(&c->d_hnodes, hn.size() * sizeof(HNode)), "hipMalloc(half nodes)");
    HIP_TRY(hipMemcpy(c->d_hnodes, hn.data(), hn.size() * sizeof(HNode), hipMemcpyHostToDevice), "hipMemcpy(half nodes)");

    // 4-wide collapse for the secondary rays: a pair node's two children, then repeatedly the
    // inner child with the largest box surface replaced by its own two children, up to 4.
    struct Kid {
        int side;      // box source: nodes[pair].f[6 side ..]
        int32_t pair;  // pair node holding this child's box
        int32_t ref;   // the child's ref in the pair tree
    };
    auto area = [&](const Kid& k) {
        const float* f = &nodes[k.pair].f[6 * k.side];
        const float d0 = f[3] - f[0], d1 = f[4] - f[1], d2 = f[5] - f[2];
        return d0 * d1 + d0 * d2 + d1 * d2;
    };
    std::vector<HNode4> w4;
    std::vector<std::pair<int32_t, int32_t>> todo{{0, 0}};  // (pair node, HNode4 slot)
    w4.emplace_back();
    while (!todo.empty()) {
        const auto [pn, slot] = todo.back();
        todo.pop_back();
        Kid kids[4];
        int nk = 0;
        for (int side = 0; side < 2; ++side)
            if (nodes[pn].c[side] != 0) kids[nk++] = Kid{side, pn, nodes[pn].c[side]};
        for (;;) {
            int best = -1;
            float best_a = -1.0f;
            for (int i = 0; i < nk; ++i)
                if (kids[i].ref > 0) {
                    const int extra = (nodes[kids[i].ref].c[0] != 0) + (nodes[kids[i].ref].c[1] != 0) - 1;
                    if (nk + extra <= 4 && area(kids[i]) > best_a) {
                        best_a = area(kids[i]);
                        best = i;
                    }
                }
            if (best < 0) break;
            const int32_t inner = kids[best].ref;
            Kid repl[2];
            int nr = 0;
            for (int side = 0; side < 2; ++side)
                if (nodes[inner].c[side] != 0) repl[nr++] = Kid{side, inner, nodes[inner].c[side]};
            kids[best] = repl[0];
            if (nr == 2) kids[nk++] = repl[1];
        }
        HNode4 h{};
        for (int i = 0; i < 4; ++i) {
            if (i >= nk) {
                for (int k = 0; k < 6; ++k) h.h[i][k] = 0x7e00u;  // NaN box: no slab test reports a hit
                h.c[i] = 0;
                continue;
            }
            for (int k = 0; k < 6; ++k) h.h[i][k] = hn[kids[i].pair].h[6 * kids[i].side + k];
            if (kids[i].ref < 0) {
                h.c[i] = kids[i].ref;
            } else {
                h.c[i] = (int32_t)w4.size();
                w4.emplace_back();
                todo.push_back({kids[i].ref, h.c[i]});
            }
        }
        w4[slot] = h;
    }
    HIP_TRY(hipMalloc(&c->d_hnodes4, w4.size() * sizeof(HNode4)), "hipMalloc(wide nodes)");
    HIP_TRY(hipMemcpy(c->d_hnodes4, w4.data(), w4.size() * sizeof(HNode4), hipMemcpyHostToDevice), "hipMemcpy(wide nodes)");
    c->num_nodes4 = w4.size();
    return VR_OK;
}

// Scenes at least this large may use the device builder (VR_OPT_DEVICE_BVH); smaller ones build on
// the host in well under a millisecond.
constexpr size_t kDeviceBvhMin = 256;

// Device BVH build (kernels/vr_lbvh.hip): records and boxes go up in scene order, the device sorts
// them by Morton code and emits the child-pair, half-precision and 4-wide trees. VR_ERR_UNSUPPORTED:
// the tree is deeper than the traversal stacks allow (the caller builds on the host instead).

// Whitened record copy for the secondary rays (WRecord), converted on the device from d_gauss.
// A record whose f32 inverse covariance is not positive definite (a nearly singular covariance) has no
// Cholesky factor: such a scene's secondary rays use the records' M forms instead (wrec_pd = false,
// secondary_ww_kernel's M-form variant), as the reference's intersect_direct / optical_depth take any M.
static vr_status upload_whitened(vr_ctx* c, size_t N) {
    c->wrec_pd = true;
    HIP_TRY(hipMalloc(&c->d_wrec, std::max<size_t>(N, 1) * sizeof(WRecord)), "hipMalloc(whitened records)");
    if (N == 0) return VR_OK;
    HIP_TRY(hipMemsetAsync(c->d_counters, 0, sizeof(uint32_t), c->stream), "hipMemsetAsync(whitened records)");
    HIP_TRY(gauss_whiten(c->d_gauss, c->d_wrec, (uint32_t)N, c->d_counters, c->stream), "whitened records");
    uint32_t bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, c->d_counters, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream), "whitened records D2H");
    HIP_TRY(hipStreamSynchronize(c->stream), "hipStreamSynchronize(whitened records)");
    c->wrec_pd = bad == 0;
    return VR_OK;
}

vr_status upload_device_bvh(vr_ctx* c, const HostScene& s, const std::vector<float>& boxes) {
    const size_t N = s.pre.size();
    std::vector<GaussianRecord> rec(N);
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    std::vector<float> ext(N);
    for (size_t i = 0; i < N; ++i) {
        const GaussianPre& p = s.pre[i];
        rec[i] = GaussianRecord{p.mean[0], p.mean[1], p.mean[2], p.density, p.inv_cov[0], p.inv_cov[1], p.inv_cov[2],
                                p.inv_cov[3], p.inv_cov[4], p.inv_cov[5], p.norm, p.albedo};
        float e = 0.0f;
        for (int k = 0; k < 3; ++k) {
            const float ce = 0.5f * (boxes[6 * i + k] + boxes[6 * i + 3 + k]);
            cmin[k] = std::min(cmin[k], ce);
            cmax[k] = std::max(cmax[k], ce);
            e = std::max(e, boxes[6 * i + 3 + k] - boxes[6 * i + k]);
        }
        ext[i] = e;
    }
    // half-precision trees: the host rule (median leaf box >= 3 % of the half extent) with the
    // primitive boxes (leaves hold up to kLeafMax of them) standing in for the leaf boxes
    double half = 0.0;
    for (int k = 0; k < 3; ++k) {
        c->hn_center[k] = 0.5f * (c->bmin[k] + c->bmax[k]);
        half = std::max(half, 0.5 * ((double)c->bmax[k] - (double)c->bmin[k]));
    }
    bool use_half = c->opt_half_nodes && half > 0.0 && std::isfinite(half);
    if (use_half) {
        c->hn_scale = (float)(1.0 / half);
        std::nth_element(ext.begin(), ext.begin() + N / 2, ext.end());
        use_half = ext[N / 2] >= 0.03 * half;
    }
    GaussianRecord* d_rec = nullptr;
    float* d_boxes = nullptr;
    HIP_TRY(hipMalloc(&d_rec, N * sizeof(GaussianRecord)), "hipMalloc(records)");
    HIP_TRY(hipMalloc(&d_boxes, N * 24), "hipMalloc(boxes)");
    HIP_TRY(hipMemcpyAsync(d_rec, rec.data(), N * sizeof(GaussianRecord), hipMemcpyHostToDevice, c->stream), "hipMemcpy(records)");
    HIP_TRY(hipMemcpyAsync(d_boxes, boxes.data(), N * 24, hipMemcpyHostToDevice, c->stream), "hipMemcpy(boxes)");
    LbvhResult R;
    hipError_t e = lbvh_build(d_rec, d_boxes, (uint32_t)N, cmin, cmax, use_half, c->hn_center, c->hn_scale, c->stream, R);
    (void)hipFree(d_rec);
    (void)hipFree(d_boxes);
    if (e == hipErrorNotSupported) return fail(VR_ERR_UNSUPPORTED, "device BVH deeper than the traversal stacks");
    if (e != hipSuccess) return hip_fail(e, "device BVH build");
    c->d_gauss = R.gauss;  // every buffer of the build belongs to the context first (free_scene frees them on error)
    c->d_order = R.order;
    c->d_nodes = R.nodes;
    c->d_hnodes = R.hnodes;
    c->d_hnodes4 = R.hnodes4;
    c->num_nodes4 = R.hnodes4 ? R.num_nodes4 : 0;
    c->num_nodes = R.num_nodes;
    c->bvh_depth = R.max_depth;
    c->num_prims = (int32_t)N;
    c->last_upload_device_bvh = true;
    return upload_whitened(c, N);
}

// The secondary rays' 4-wide tree: the shared tree's nodes refit with the records' tight boxes on the
// device (vr_gauss.hip, refit_kernel; whitened scenes only: the M forms keep the padded boxes).
vr_status upload_secondary_tree(vr_ctx* c) {
    if (c->d_hnodes4s) (void)hipFree(c->d_hnodes4s);
    c->d_hnodes4s = nullptr;
    if (!c->opt_sec_tight || !c->wrec_pd || !c->d_wrec || !c->d_hnodes4 || !c->d_parent4 || !c->d_gauss || c->num_nodes4 == 0)
        return VR_OK;
    const size_t n = c->num_nodes4;
    double d2 = 0.0;  // the scene box's diagonal: no ray origin is farther than that from a record
    for (int k = 0; k < 3; ++k) d2 += ((double)c->bmax[k] - c->bmin[k]) * ((double)c->bmax[k] - c->bmin[k]);
    uint8_t* depth = nullptr;
    float* nbox = nullptr;
    uint32_t* maxd = nullptr;
    // n nodes as refit (HNode4), then (VR_SEC_SOA) the same n nodes with their boxes laid out per axis for the
    // secondary kernel's node step (soa_nodes_kernel)
    hipError_t e = hipMalloc(&c->d_hnodes4s, (VR_SEC_SOA ? 2 : 1) * n * sizeof(HNode4));
    if (e == hipSuccess) e = hipMalloc(&depth, n);
    if (e == hipSuccess) e = hipMalloc(&nbox, n * 6 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&maxd, sizeof(uint32_t));
    if (e == hipSuccess)
        e = gauss_refit_secondary(c->d_hnodes4, c->d_hnodes4s, VR_SEC_SOA ? c->d_hnodes4s + n : nullptr, (uint32_t)n, c->d_gauss,
                                  c->d_parent4, depth, nbox, maxd, c->hn_center, c->hn_scale, (float)std::sqrt(d2), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    for (void* p : {(void*)depth, (void*)nbox, (void*)maxd})
        if (p) (void)hipFree(p);
    if (e == hipErrorNotSupported) {  // a tree deeper than 255 levels: the shared boxes
        (void)hipFree(c->d_hnodes4s);
        c->d_hnodes4s = nullptr;
        return VR_OK;
    }
    if (e != hipSuccess) return hip_fail(e, "secondary-ray tree");
    return VR_OK;
}

// Parent of every 4-wide node (built on the device from the children refs): a secondary ray starts its
// tree walk in the subtree holding its origin and climbs to the parents once that subtree is done
// (vr_gauss.hip, record_start_kernel / sec_node4v).
vr_status upload_parents(vr_ctx* c) {
    if (c->d_parent4) (void)hipFree(c->d_parent4);
    c->d_parent4 = nullptr;
    if (c->d_prim_node4) (void)hipFree(c->d_prim_node4);
    c->d_prim_node4 = nullptr;
    if (c->d_hnodes4w) (void)hipFree(c->d_hnodes4w);
    c->d_hnodes4w = nullptr;
    if (!c->d_hnodes4 || c->num_nodes4 == 0) return VR_OK;
    // every 4-wide walk's node test reads the per-axis copy (wide_children): it exists whenever d_hnodes4 does
    HIP_TRY(hipMalloc(&c->d_hnodes4w, c->num_nodes4 * sizeof(HNode4)), "hipMalloc(per-axis wide nodes)");
    HIP_TRY(gauss_soa_nodes(c->d_hnodes4, c->d_hnodes4w, (uint32_t)c->num_nodes4, c->stream), "per-axis wide nodes");
    HIP_TRY(hipMalloc(&c->d_parent4, c->num_nodes4 * sizeof(int32_t)), "hipMalloc(wide-node parents)");
    if (c->num_prims > 0)
        HIP_TRY(hipMalloc(&c->d_prim_node4, (size_t)c->num_prims * sizeof(int32_t)), "hipMalloc(record leaf nodes)");
    HIP_TRY(gauss_parents(c->d_hnodes4, (uint32_t)c->num_nodes4, c->d_parent4, c->d_prim_node4, c->stream),
            "wide-node parents");
    HIP_TRY(hipStreamSynchronize(c->stream), "wide-node parents");
    return upload_secondary_tree(c);
}

// Farthest distance any ray can travel before leaving the scene box: the rays of both camera
// models start on the 2x2 sensor square position +- right +- up (camera.h:50,69).
float scene_tmax(const vr_ctx* c, const vr_camera* cam) {
    float best = 0.0f;
    for (int su = -1; su <= 1; su += 2)
        for (int sv = -1; sv <= 1; sv += 2) {
            float o[3];
            for (int k = 0; k < 3; ++k) o[k] = cam->position[k] + su * cam->right[k] + sv * cam->up[k];
            for (int cx = 0; cx < 2; ++cx)
                for (int cy = 0; cy < 2; ++cy)
                    for (int cz = 0; cz < 2; ++cz) {
                        float p[3] = {cx ? c->bmax[0] : c->bmin[0], cy ? c->bmax[1] : c->bmin[1], cz ? c->bmax[2] : c->bmin[2]};
                        double d = 0;
                        for (int k = 0; k < 3; ++k) d += (double)(p[k] - o[k]) * (p[k] - o[k]);
                        best = std::max(best, (float)std::sqrt(d));
                    }
        }
    // secondary rays start inside the scene box: a Gaussian interval on them ends within one
    // box diagonal (PureRayMarching marches them over the same step table)
    double diag = 0.0;
    for (int k = 0; k < 3; ++k) diag += (double)(c->bmax[k] - c->bmin[k]) * (c->bmax[k] - c->bmin[k]);
    best = std::max(best, (float)std::sqrt(diag));
    return best * 1.01f + 1.0f;
}

vr_status get_table(vr_ctx* c, float step, float tmax, const float** d, int* n) {
    if (!(step > 0.0f) || !std::isfinite(step)) return fail(VR_ERR_INVALID, "step_size must be a positive finite float");
    uint32_t key;
    std::memcpy(&key, &step, 4);
    auto it = c->tables.find(key);
    if (it == c->tables.end() || it->second.tmax < tmax) {
        float want = it == c->tables.end() ? tmax : std::max(tmax, 2.0f * it->second.tmax);
        std::vector<float> t = step_table(step, want);
        if (t.back() <= tmax) return fail(VR_ERR_OVERFLOW, "step_size too small for the scene extent (float step sequence stalls)");
        vr_ctx::Table tb;
        tb.n = (int)t.size();
        tb.tmax = want;
        HIP_TRY(hipMalloc(&tb.d, t.size() * sizeof(float)), "hipMalloc(step table)");
        HIP_TRY(hipMemcpy(tb.d, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy(step table)");
        if (it != c->tables.end()) (void)hipFree(it->second.d);
        c->tables[key] = tb;
        it = c->tables.find(key);
    }
    *d = it->second.d;
    *n = it->second.n;
    return VR_OK;
}

vr_status ensure_queue(vr_ctx* c, uint64_t pixels) {
    if (pixels + 1 > (uint64_t)c->queue_cap + 1 || !c->d_queue) {
        if (c->d_queue) (void)hipFree(c->d_queue);
        c->d_queue = nullptr;
        uint64_t cap = std::max<uint64_t>(pixels, 4096);
        if (cap > 0xffffffffull) return fail(VR_ERR_INVALID, "frame too large");
        HIP_TRY(hipMalloc(&c->d_queue, (cap + 1) * sizeof(uint32_t)), "hipMalloc(queue)");
        c->queue_cap = (uint32_t)cap;
    }
    return VR_OK;
}

vr_status fill_args(vr_ctx* c, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H, RenderArgs& A) {
    if (!c->has_scene) return fail(VR_ERR_NOSCENE, "no scene uploaded (call vr_upload_scene first)");
    if (!cam || !p) return fail(VR_ERR_INVALID, "NULL camera or params");
    if (W == 0 || H == 0 || W > 65535 || H > 65535) return fail(VR_ERR_INVALID, "width/height must be in [1, 65535]");
    if (cam->type != VR_CAMERA_PINHOLE && cam->type != VR_CAMERA_ORTHOGRAPHIC) return fail(VR_ERR_INVALID, "unknown camera type");
    if (p->flags != 0) return fail(VR_ERR_INVALID, "vr_render_params.flags must be 0");
    if ((p->integrator == VR_RAYMARCH_GAUSSIANS || p->integrator == VR_PURE_RAYMARCH) && c->type != VR_VOLUME_GAUSSIANS)
        return fail(VR_ERR_INVALID, "RayMarchingGaussians needs a Gaussian scene");
    if (p->integrator == VR_RAYMARCH_SPHERES && c->type != VR_VOLUME_SPHERES)
        return fail(VR_ERR_INVALID, "RayMarchingSpheres needs a sphere scene");
    const bool ff = p->integrator == VR_FREE_FLIGHT || p->integrator == VR_MULTI_SCATTER;
    if (p->integrator != VR_RAYMARCH_GAUSSIANS && p->integrator != VR_RAYMARCH_SPHERES && p->integrator != VR_TEST_HITMASK &&
        p->integrator != VR_PURE_RAYMARCH && !ff)
        return fail(VR_ERR_UNSUPPORTED, "integrator has no device implementation");
    if (ff && c->type != VR_VOLUME_GAUSSIANS)
        return fail(VR_ERR_INVALID, "free-flight integrators need a Gaussian scene (integrator.h:327 reads scene.gmm)");
    if (ff && p->num_samples <= 0) return fail(VR_ERR_INVALID, "num_samples must be > 0");
    if (ff && p->min_bounces < 0) return fail(VR_ERR_INVALID, "min_bounces must be >= 0");
    if (!ff && p->integrator != VR_TEST_HITMASK && p->env_samples < 0) return fail(VR_ERR_INVALID, "env_samples must be >= 0");
    if (!(p->t_eps >= 0.0f) || p->t_eps >= 1.0f) return fail(VR_ERR_INVALID, "t_eps must be in [0, 1)");
    std::memset(&A, 0, sizeof(A));
    A.cam_type = cam->type;
    for (int k = 0; k < 3; ++k) {
        A.cam_pos[k] = cam->position[k];
        A.cam_view[k] = cam->view_dir[k];
        A.cam_right[k] = cam->right[k];
        A.cam_up[k] = cam->up[k];
        A.cam_pinhole[k] = cam->pinhole[k];
    }
    A.width = W;
    A.height = H;
    A.tiles_x = (W + kTile - 1) / kTile;
    A.gauss = c->d_gauss;
    A.wrec = c->wrec_pd ? c->d_wrec : nullptr;
    A.nodes = c->d_nodes;
    A.hnodes = c->d_hnodes;
    A.hnodes4 = c->d_hnodes4;
    A.hnodes4s = c->d_hnodes4s ? c->d_hnodes4s : c->d_hnodes4;
    A.hnodes4t = (VR_SEC_SOA && c->d_hnodes4s) ? c->d_hnodes4s + c->num_nodes4 : nullptr;
    A.hnodes4w = c->d_hnodes4w;
    A.hn4_parent = c->d_parent4;
    A.prim_node4 = c->d_prim_node4;
    A.num_nodes4 = (uint32_t)c->num_nodes4;
    for (int k = 0; k < 3; ++k) A.hn_center[k] = c->hn_center[k];
    A.hn_scale = c->hn_scale;
    A.spheres = c->d_spheres;
    A.num_prims = c->num_prims;
    A.bvh_depth = c->bvh_depth;
    A.num_lights = (int32_t)c->lights.size();
    for (size_t l = 0; l < c->lights.size(); ++l) A.lights[l] = c->lights[l];
    for (int k = 0; k < 3; ++k) A.env[k] = c->env[k];
    A.step_size = p->step_size;
    A.env_samples = p->env_samples;
    A.t_eps = p->t_eps;
    A.pure = p->integrator == VR_PURE_RAYMARCH ? 1 : 0;
    A.env_order = nullptr;  // set per frame by gauss_pipeline
    A.env_base = nullptr;
    A.rec_cut = nullptr;
    A.chunk_rec = 64u;
    A.chunk_shift = 6u;
    // Secondary-ray optical-depth cut-off. Exact mode (t_eps = 0): 104, where expf(-tau) is already
    // 0 in f32, so stopping is bit-neutral. With an early-out budget t_eps > 0 the cut-off is
    // ln(1/t_eps) + ln(1000): a dropped transmittance is <= 1e-3 * t_eps, a thousandth of the error
    // the primary early-out itself is allowed (DESIGN.md §Error budget).
    A.tau_cut = p->t_eps > 0.0f ? std::min(104.0f, (float)(std::log(1.0 / p->t_eps) + std::log(1000.0))) : 104.0f;
    if (ff) {
        A.ff_multi = p->integrator == VR_MULTI_SCATTER ? 1 : 0;
        A.ff_samples = p->num_samples;
        A.ff_n = (int32_t)std::sqrt((double)p->num_samples);  // int(std::sqrt(num_samples)), integrator.h:564
        A.ff_min_bounces = p->min_bounces;
        A.ff_max_bounces = 1 << 16;
        A.ff_solver = (int32_t)c->opt_ff_solver;
        A.ff_sm = c->opt_ff_kernel == 2 || (c->opt_ff_kernel == 0 && c->auto_ff_sm) ? 1 : 0;
    } else if (p->integrator != VR_TEST_HITMASK) {
        const float* d;
        int n;
        vr_status st = get_table(c, p->step_size, scene_tmax(c, cam), &d, &n);
        if (st != VR_OK) return st;
        A.tsteps = d;
        A.num_tsteps = n;
    }
    A.counters = c->d_counters;
    A.gauss_order = c->d_order;
    return VR_OK;
}

vr_status grow(vr_ctx::Buf& b, size_t bytes, const char* what) {
    if (bytes <= b.bytes && b.p) return VR_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    size_t want = std::max<size_t>(bytes + bytes / 4, 256);
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) return hip_fail(e, what);
    b.bytes = want;
    return VR_OK;
}

// RayMarchingGaussians: march (records) -> sizing / cut-offs -> secondary rays -> accumulate.
vr_status gauss_pipeline(vr_ctx* c, RenderArgs& A, hipStream_t s, bool stats) {
    const uint32_t npix = A.num_tiles * 256u;
    vr_status st;
    if ((st = grow(c->px_first, npix * 4ull, "hipMalloc(px_first)")) != VR_OK) return st;
    if ((st = grow(c->px_T, npix * 4ull, "hipMalloc(px_T)")) != VR_OK) return st;
    if ((st = grow(c->rec_alloc, 16, "hipMalloc(rec_alloc)")) != VR_OK) return st;
    A.px_first = (uint32_t*)c->px_first.p;
    A.px_T = (float*)c->px_T.p;
    A.rec_alloc = (uint32_t*)c->rec_alloc.p;
    // PCG32 (rng.h:20-50, seq 1 -> inc 3) jump-ahead table for the environment samples
    if (c->pcg_jump_n < 2 * A.env_samples + 2) {
        const int n = 2 * A.env_samples + 2;
        std::vector<unsigned long long> tab(2 * (size_t)n);
        unsigned long long m = 1ull, a = 0ull;
        for (int k = 0; k < n; ++k) {
            tab[2 * k] = m;
            tab[2 * k + 1] = a;
            m *= 6364136223846793005ull;
            a = a * 6364136223846793005ull + 3ull;
        }
        if ((st = grow(c->pcg_jump, tab.size() * 8, "hipMalloc(pcg)")) != VR_OK) return st;
        HIP_TRY(hipMemcpy(c->pcg_jump.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice), "hipMemcpy(pcg)");
        c->pcg_jump_n = n;
    }
    A.pcg_jump = (const unsigned long long*)c->pcg_jump.p;
    if ((st = grow(c->deep, (kDeepQueue + 1) * 4ull + (uint64_t)kActDeep * kDeepThreads * 4ull + (uint64_t)kActWide * kWideThreads * 4ull,
                   "hipMalloc(deep march)")) != VR_OK)
        return st;
    A.deepq = (uint32_t*)c->deep.p;
    A.deepq_cap = kDeepQueue;
    A.deep_act = (int32_t*)(A.deepq + kDeepQueue + 1);
    A.wide_act = A.deep_act + (size_t)kActDeep * kDeepThreads;
    A.wide_min = (uint32_t)c->opt_march_wide_min;
    A.march_big = c->march_big ? 1 : 0;

    // Tile bins of the binned march: count, scan, then (with one host sync for the entry count) emit.
    A.bin_off = A.bin_ent = nullptr;
    A.bin_cnt = A.bin_out = nullptr;
    if (c->opt_march_binned && A.num_prims > 0) {
#ifndef VR_BIN_BUCKETS
#define VR_BIN_BUCKETS 256  // depth buckets per tile (a bucket's hits wait in a 16-entry per-lane list)
#endif
        const uint32_t nb = VR_BIN_BUCKETS, nbins = A.num_tiles * nb;
        if ((st = grow(c->bin_cnt, (nbins + 1) * 4ull, "hipMalloc(bins)")) != VR_OK) return st;
        if ((st = grow(c->bin_off, (nbins + 1) * 4ull, "hipMalloc(bins)")) != VR_OK) return st;
        A.bin_nb = nb;
        {  // depth buckets over [0, the farthest scene-box corner from any ray origin]
            float r = 0.0f, far = 0.0f;
            for (int k = 0; k < 3; ++k) r += std::fabs(A.cam_right[k]) + std::fabs(A.cam_up[k]);
            for (int cn = 0; cn < 8; ++cn) {
                float d2 = 0.0f;
                for (int k = 0; k < 3; ++k) {
                    const float v = ((cn >> k) & 1) ? c->bmax[k] : c->bmin[k];
                    d2 += (v - A.cam_pos[k]) * (v - A.cam_pos[k]);
                }
                far = std::max(far, std::sqrt(d2));
            }
            A.bin_dz = std::max((far + r) / (float)nb, 1e-6f);
        }
        A.bin_cnt = (uint32_t*)c->bin_cnt.p;
        HIP_TRY(hipMemsetAsync(A.bin_cnt, 0, (nbins + 1) * 4ull, s), "hipMemsetAsync(bins)");
        HIP_TRY(gauss_bin(A, false, s), "bin count");
        size_t tmp = 0;
        HIP_TRY(gauss_bin_scan(A.bin_cnt, (uint32_t*)c->bin_off.p, nbins + 1, nullptr, tmp, s), "bin scan");
        if ((st = grow(c->bin_ent, std::max<size_t>(tmp, 64), "hipMalloc(bin scan)")) != VR_OK) return st;
        HIP_TRY(gauss_bin_scan(A.bin_cnt, (uint32_t*)c->bin_off.p, nbins + 1, c->bin_ent.p, tmp, s), "bin scan");
        uint32_t total = 0;
        HIP_TRY(hipMemcpyAsync(&total, (uint32_t*)c->bin_off.p + nbins, 4, hipMemcpyDeviceToHost, s), "bin total D2H");
        HIP_TRY(hipStreamSynchronize(s), "bin count");
        if ((st = grow(c->bin_ent, std::max<uint64_t>(total, 1) * 4ull, "hipMalloc(bin entries)")) != VR_OK) return st;
        A.bin_off = (const uint32_t*)c->bin_off.p;
        A.bin_out = (uint32_t*)c->bin_ent.p;
        HIP_TRY(hipMemsetAsync(A.bin_cnt, 0, (nbins + 1) * 4ull, s), "hipMemsetAsync(bins)");
        HIP_TRY(gauss_bin(A, true, s), "bin emit");
        A.bin_ent = A.bin_out;
    }

    // Record capacity: from earlier frames of this context (hints), so the host never waits for
    // the march. A context's first frame sizes it: one host sync after the march, re-run with the
    // exact need if it did not fit. A later frame that outgrows the buffers is reported
    // (h_report[4]) and the synchronous entry points render it again with grown buffers.
    const bool sized = c->rec_hint != 0;
    const uint32_t S = (uint32_t)(A.num_lights + A.env_samples);
    uint64_t cap = std::max<uint64_t>({c->rec_hint, 2ull * npix, 4096ull});
    // secondary-ray slots are 32-bit: a hint carried over from an earlier, larger frame (or one with
    // fewer samples per record) is clamped to what this frame's samples allow
    cap = std::min<uint64_t>(cap, std::max<uint64_t>(4096ull, (0xfffffffeull / std::max(S, 1u)) / 64 * 64 - 64));
    uint64_t ovf = std::max<uint64_t>({c->ovf_hint, cap, 4096ull});
    for (int attempt = 0;; ++attempt) {
        if (cap > 0xffffffffull / kActInline || ovf > 0xffffffffull - cap * kActInline || (cap + 63) / 64 * 64 * std::max(S, 1u) >= 0xffffffffull)
            return fail(VR_ERR_UNSUPPORTED, "too many scatter records in one call (split the frame)");
        if ((st = grow(c->rec_pos, cap * 16ull, "hipMalloc(records)")) != VR_OK) return st;
        if ((st = grow(c->rec_meta, cap * 16ull, "hipMalloc(records)")) != VR_OK) return st;
        if ((st = grow(c->rec_next, cap * 4ull, "hipMalloc(records)")) != VR_OK) return st;
        if ((st = grow(c->rec_bloom, cap * 8ull, "hipMalloc(record blooms)")) != VR_OK) return st;
        if ((st = grow(c->rec_act, (cap * kActInline + ovf) * 4ull, "hipMalloc(active lists)")) != VR_OK) return st;
        A.rec_pos = (float4*)c->rec_pos.p;
        A.rec_meta = (uint4*)c->rec_meta.p;
        A.rec_next = (uint32_t*)c->rec_next.p;
        A.rec_bloom = (unsigned long long*)c->rec_bloom.p;
        A.rec_act = (int32_t*)c->rec_act.p;
        A.rec_cap = (uint32_t)cap;
        A.act_ovf_cap = (uint32_t)ovf;
        HIP_TRY(hipMemsetAsync(A.rec_alloc, 0, 16, s), "hipMemsetAsync(rec_alloc)");
        HIP_TRY(hipMemsetAsync(c->d_queue, 0, sizeof(uint32_t), s), "hipMemsetAsync(queue)");
        HIP_TRY(hipMemsetAsync(A.deepq, 0, sizeof(uint32_t), s), "hipMemsetAsync(deep queue)");
        HIP_TRY(gauss_march(A, s, stats), "march");
        if (attempt == 0) HIP_TRY(hipEventRecord(c->ev_stage[0], s), "hipEventRecord");
        if (sized) break;
        HIP_TRY(hipMemcpyAsync(c->h_sizing, A.rec_alloc, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, s), "rec_alloc D2H");
        HIP_TRY(hipStreamSynchronize(s), "march");
        if (c->h_sizing[2] == 0) {
            c->rec_hint = std::max<uint64_t>(4096, (uint64_t)c->h_sizing[0] + c->h_sizing[0] / 8);
            c->ovf_hint = std::max<uint64_t>(c->ovf_hint, (uint64_t)c->h_sizing[1] + c->h_sizing[1] / 8);
            break;
        }
        if (attempt >= 3) return fail(VR_ERR_OVERFLOW, "scatter-record capacity could not be sized");
        cap = std::max<uint64_t>(2 * cap, (uint64_t)c->h_sizing[0] + c->h_sizing[0] / 4 + 1024);
        ovf = std::max<uint64_t>(2 * ovf, (uint64_t)c->h_sizing[1] + c->h_sizing[1] / 4 + 1024);
    }

    // Everything below is sized by the capacity; the kernels read the live record count on the device.
    // Tr slots: whole record chunks (<= 64 records; hand-out order, vr_gauss.hip)
    if ((st = grow(c->tr, std::max<uint64_t>((cap + 63) / 64 * 64 * S, 1) * 4ull, "hipMalloc(secondary)")) != VR_OK) return st;
    A.tr = (float*)c->tr.p;
    if ((st = grow(c->rec_rad, std::max<uint64_t>(cap, 1) * 16ull, "hipMalloc(record radiance)")) != VR_OK) return st;
    A.rec_rad = (float4*)c->rec_rad.p;
    // exact slow path: light rays (stopping event / missed member), the rare rays with a member at its 3-sigma
    // boundary and those with a chord in the f32 error band (light or environment). Sized for every light ray plus
    // one more ray per record, or what earlier frames queued (+ 1/8); a frame that queues more (a boundary record's
    // environment rays can all go there) raises rec_alloc[2] and is rendered again with the grown queue
    const uint64_t nslow = std::min<uint64_t>(std::max<uint64_t>(cap * (uint64_t)A.num_lights + cap, c->slow_hint), 0xfffffffeull);
    if ((st = grow(c->slowq, (nslow + 1) * 4ull, "hipMalloc(slow queue)")) != VR_OK) return st;
    A.slowq = (uint32_t*)c->slowq.p;
    A.slowq_cap = (uint32_t)nslow;
    HIP_TRY(hipMemsetAsync(A.slowq, 0, sizeof(uint32_t), s), "hipMemsetAsync(slow queue)");
    {  // rays with one chord in the f32 error band (secondary_fix_kernel): one per record, or what earlier frames queued
        const uint64_t nfix = std::min<uint64_t>(std::max<uint64_t>(cap, c->fix_hint), 0x7ffffffeull / 3);
        if ((st = grow(c->fixq, (3 * nfix + 1) * 4ull, "hipMalloc(band queue)")) != VR_OK) return st;
        A.fixq = (uint32_t*)c->fixq.p;
        A.fixq_cap = (uint32_t)nfix;
        HIP_TRY(hipMemsetAsync(A.fixq, 0, sizeof(uint32_t), s), "hipMemsetAsync(band queue)");
    }
    if ((st = grow(c->ray_next, 8, "hipMalloc(ray counter)")) != VR_OK) return st;
    A.ray_next = (unsigned long long*)c->ray_next.p;
    {  // traversal-stack overflow of the persistent kernel: kWideStackMax entries for every lane it can keep resident
        int cus = 0;
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device), "hipDeviceGetAttribute");
        const uint64_t lanes = (uint64_t)std::max(cus, 1) * 2048ull;  // 32 waves of 64 lanes per CU at most
        if ((st = grow(c->stack_ovf, lanes * kWideStackMax * 4ull, "hipMalloc(stack overflow)")) != VR_OK) return st;
        A.stack_ovf = (int32_t*)c->stack_ovf.p;
        A.stack_ovf_lanes = (uint32_t)lanes;
    }
    {  // per-pixel error budget of the secondary cut-off (record_cut_kernel): budget = t_eps, so the
       // secondary rays' truncation moves a pixel by at most t_eps, the same bound as the primary
       // early-out (error budget). t_eps = 0 (exact mode) keeps the bit-neutral 104.
        A.rec_cut = nullptr;
        if (c->opt_secondary_budget && A.t_eps > 0.0f) {
            if ((st = grow(c->rec_cut, cap * 4ull, "hipMalloc(record cut-offs)")) != VR_OK) return st;
            A.rec_cut = (float*)c->rec_cut.p;
            HIP_TRY(gauss_record_cut(A, A.t_eps, s), "record cut-offs");
        }
    }
    HIP_TRY(hipEventRecord(c->ev_stage[1], s), "hipEventRecord");
    A.rec_start = nullptr;  // per record: the 4-wide subtree its secondary rays walk first (record_start_kernel)
    if (A.hnodes4 != nullptr && A.hn4_parent != nullptr && c->opt_start_subtree) {
        if ((st = grow(c->rec_start, cap * 4ull, "hipMalloc(record start nodes)")) != VR_OK) return st;
        A.rec_start = (int32_t*)c->rec_start.p;
    }
    {  // environment rays traced in direction order within chunks of 32 records (see ray_slot; larger
       // chunks measured 2-20 % slower: record locality is lost)
#ifndef VR_CHUNK_SHIFT
#define VR_CHUNK_SHIFT 5  // 32-record chunks (A/B at C4: 8/16/32/64/128 -> 156.1/150.4/149.1/152.9/161.9 ms)
#endif
        constexpr uint32_t shift = VR_CHUNK_SHIFT, cr = 1u << shift;  // entries hold record-in-chunk in 8 bits
        static_assert(VR_CHUNK_SHIFT <= 8, "environment-order entries and env_order_kernel hold record-in-chunk in 8 bits");
        A.env_order = nullptr;
        A.chunk_rec = cr;
        A.chunk_shift = shift;
        if (A.env_samples > 0 && A.env_samples <= kEnvOrderMax) {
            const uint64_t nch = (cap + cr - 1) / cr;
            if ((st = grow(c->env_order, nch * cr * (uint64_t)A.env_samples * 2ull, "hipMalloc(environment-ray order)")) != VR_OK)
                return st;
            A.env_order = (uint16_t*)c->env_order.p;
            if ((st = grow(c->env_base, nch * cr * 8ull, "hipMalloc(environment generator states)")) != VR_OK) return st;
            A.env_base = (uint64_t*)c->env_base.p;
        }
    }
    HIP_TRY(gauss_secondary(A, s, stats), "secondary rays");
    HIP_TRY(hipEventRecord(c->ev_stage[2], s), "hipEventRecord");
    HIP_TRY(gauss_accumulate(A, s), "accumulate");
    c->staged = true;
    c->report_gauss = true;
    c->report_pixels = (uint64_t)A.num_tiles * 256u;
    c->last_secondary_per_record = S;
    return VR_OK;
}

// Free-flight integrators: one persistent launch per chunk of tiles x batch of samples (at most
// kFFMaxPaths paths) on a grid of resident waves that claim 64-path groups from a counter, the
// launch's queued shadow rays (deferred NEE), then the paths' radiance is added to the pixels in
// sample order (vr_freeflight.hip).
constexpr uint64_t kFFMaxPaths = 1ull << 23;
// The active list indexes the hit buffer, so it never holds more than kFFHitCap entries: the only
// capacity a path can exceed is kFFHitCap Gaussians overlapping one point; such a path re-runs in
// ff_fallback_kernel with kFFBigCap-entry rows (only beyond that: error path, NaN).
constexpr int32_t kFFHitCap = 128, kFFActCap = kFFHitCap;
vr_status free_flight_pipeline(vr_ctx* c, RenderArgs& A, hipStream_t s) {
    const uint32_t spp = (uint32_t)A.ff_samples;
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device), "hipDeviceGetAttribute");
    const uint32_t nsb = (uint32_t)std::min<uint64_t>(spp, kFFMaxPaths / 256u);  // samples per launch
    const uint32_t chunk = (uint32_t)std::min<uint64_t>(A.num_tiles, kFFMaxPaths / ((uint64_t)nsb * 256u));
    const uint64_t paths = (uint64_t)chunk * nsb * 256u;  // most paths of one launch
    // the persistent path kernel's resident grid (scratch rows per thread)
    const uint32_t threads = free_flight_threads(cus);
    vr_status st = grow(c->ff_scratch, (size_t)threads * (kFFHitCap + 2 * kFFActCap) * 16 + 64, "free-flight scratch");
    if (st != VR_OK) return st;
    if ((st = grow(c->ff_tail, paths * sizeof(float4), "free-flight paths")) != VR_OK) return st;
    if ((st = grow(c->ff_sum, (size_t)A.num_tiles * 256 * 3 * sizeof(float), "free-flight sums")) != VR_OK) return st;
    {  // Deferred-NEE queue: VR_OPT_FF_NEE_QUEUE rays per path of a launch bound it; within that bound it is
       // sized from the need of this context's earlier frames (the most rays any launch queued, + 1/8;
       // never shrunk, like the record buffers, so a frame that fitted before fits again),
       // a first frame from the integrator (one shadow ray per bounce, min_bounces + 1 bounces before
       // Russian roulette). A launch that outgrows it is reported and the frame rendered again with a
       // grown queue (as the ray-march's record buffers), so frames never depend on the capacity.
        const uint64_t bound = std::min<uint64_t>(paths * (uint64_t)c->opt_ff_nee_queue, kFFNone);
        const uint64_t first = paths * (A.ff_multi ? (uint64_t)A.ff_min_bounces + 1ull : 1ull) + 4096ull;
        const uint64_t cap = c->nee_inline ? 0ull : std::min<uint64_t>(bound, c->nee_hint ? std::max<uint64_t>(c->nee_hint, 4096ull) : first);
        const size_t bytes = (size_t)cap * 3 * sizeof(float4);
        A.ff_nee_cap = (uint32_t)cap;
        c->last_nee_cap = (uint32_t)cap;
        c->last_nee_bound = (uint32_t)bound;
        if (cap > 0) {
            if ((st = grow(c->ff_nee, bytes, "free-flight shadow-ray queue")) != VR_OK) return st;
            A.ff_nee = (float4*)c->ff_nee.p;
        }
    }
    A.ff_nee_refill = c->auto_nee_refill;
    {  // paths over the hit-buffer capacity re-run in ff_fallback_kernel (queue + its own rows)
        const uint64_t qcap = paths;
        const uint64_t rows = (uint64_t)kFFBigThreads * 3ull * (uint64_t)kFFBigCap * 16ull;
        if ((st = grow(c->ff_fb, rows + (qcap + 1) * 4ull + 64, "free-flight fallback")) != VR_OK) return st;
        A.ff_big = (float4*)c->ff_fb.p;
        A.ff_fbq = (uint32_t*)((char*)c->ff_fb.p + rows);
        A.ff_fbq_cap = (uint32_t)qcap;
    }
    float4* base = (float4*)c->ff_scratch.p;
    A.ff_threads = threads;
    A.ff_hit_cap = kFFHitCap;
    A.ff_act_cap = kFFActCap;
    const int64_t w0 = c->opt_ff_window0 > 0 ? c->opt_ff_window0 : (int64_t)c->auto_window0;
    A.ff_hit_cap0 = (int32_t)std::max<int64_t>(1, std::min<int64_t>(kFFHitCap, w0));
    A.ff_hit = base;
    A.ff_act0 = base + (size_t)kFFHitCap * threads;
    A.ff_act1 = base + (size_t)(kFFHitCap + kFFActCap) * threads;
    A.ff_next = (unsigned long long*)(base + (size_t)(kFFHitCap + 2 * kFFActCap) * threads);
    A.ff_nee_n = (uint32_t*)(A.ff_next + 1);
    A.ff_tail = (float4*)c->ff_tail.p;
    A.ff_sum = (float*)c->ff_sum.p;
    c->ff_launches = 0;
    for (uint32_t t0 = 0; t0 < A.num_tiles; t0 += chunk) {
        const uint32_t nt = std::min(chunk, A.num_tiles - t0);
        for (uint32_t si = 0; si < spp; si += nsb) {
            A.ff_tile_base = t0;
            A.ff_si0 = si;
            A.ff_nsb = std::min(nsb, spp - si);
            A.ff_total = (unsigned long long)nt * A.ff_nsb * 256ull;
            const size_t e0 = 4 * (size_t)c->ff_launches;
            while (c->ff_ev.size() < e0 + 4) {
                hipEvent_t e = nullptr;
                HIP_TRY(hipEventCreate(&e), "hipEventCreate");
                c->ff_ev.push_back(e);
            }
            HIP_TRY(launch_free_flight(A, nt, s, &c->ff_ev[e0]),
                    "free-flight launch");
            ++c->ff_launches;
        }
    }
    return VR_OK;
}

// Collect the report of the last frame (waits for it). Grows the record capacity hints from its
// counts, so a frame that outgrew them renders correctly the next time.
vr_status collect(vr_ctx* c) {
    if (!c->stats_pending) return VR_OK;
    HIP_TRY(hipEventSynchronize(c->ev_report), "hipEventSynchronize");
    c->stats_pending = false;
    c->sync_pending = true;
    if (c->report_gauss) {
        const uint64_t nrec = c->h_report[2], nact = c->h_report[3], nslow = c->h_report[8];
        c->rec_hint = std::max<uint64_t>(c->rec_hint, nrec + nrec / 8);
        c->ovf_hint = std::max<uint64_t>(c->ovf_hint, nact + nact / 8);
        c->slow_hint = std::max<uint64_t>(c->slow_hint, nslow + nslow / 8);
        const uint64_t nfix = c->h_report[9];
        c->fix_hint = std::max<uint64_t>(c->fix_hint, nfix + nfix / 8);
        // >= 5 % of the pixels re-marched: the scene's active sets outgrow 16 slots; later frames march with
        // kActBig (same operations, so the frames are identical; kept until the next upload)
        if ((uint64_t)c->h_report[0] * 20ull >= c->report_pixels && c->report_pixels > 0) c->march_big = true;
    }
    if (c->report_ff && c->last_nee_bound > 0) {
        // a launch that found the queue full counted its paths' first refused claim only (they then
        // trace inline): grow at least twice over
        const uint64_t need = c->h_report[7];
        const bool over = need > c->last_nee_cap;
        c->nee_hint = std::max<uint64_t>({c->nee_hint, need + need / 8, over ? 2ull * c->last_nee_cap : 0ull});
        // full at the bound: a path that met it traced the rest inline and added them as one partial sum (float
        // association); the frame is rendered again with every shadow ray inline, which is the queued frame
        if (over && c->last_nee_cap >= c->last_nee_bound) c->nee_inline = true;
    }
    return VR_OK;
}

bool frame_exceeded(const vr_ctx* c) {
    if (c->report_gauss && c->h_report[4] != 0) return true;
    // the shadow-ray queue overflowed below its VR_OPT_FF_NEE_QUEUE bound: render again with a larger one
    // (or at it: the next frame traces inline, see nee_inline). A frame traced inline queues nothing.
    return c->report_ff && c->h_report[7] > c->last_nee_cap;
}

vr_status launch(vr_ctx* c, RenderArgs& A, const vr_render_params* p, hipStream_t s, bool stats = false) {
    vr_status st = ensure_queue(c, (uint64_t)A.num_tiles * 256u);
    if (st != VR_OK) return st;
    A.queue = c->d_queue;
    A.queue_cap = c->queue_cap;
    if ((st = collect(c)) != VR_OK) return st;  // the previous report must land before the pinned buffer is reused
    c->sync_pending = false;  // vr_synchronize reports the last frame's outcome: this one's from here on
    HIP_TRY(hipMemsetAsync(c->d_queue, 0, sizeof(uint32_t), s), "hipMemsetAsync(queue)");
    HIP_TRY(hipMemsetAsync(c->d_counters, 0, 4 * sizeof(uint32_t), s), "hipMemsetAsync(counters)");
    HIP_TRY(hipEventRecord(c->ev_start, s), "hipEventRecord");
    c->staged = false;
    c->report_gauss = false;
    c->report_ff = false;
    c->ff_launches = 0;
    if (c->type == VR_VOLUME_GAUSSIANS && (p->integrator == VR_RAYMARCH_GAUSSIANS || p->integrator == VR_PURE_RAYMARCH)) {
        st = gauss_pipeline(c, A, s, stats);
        if (st != VR_OK) return st;
    } else if (p->integrator == VR_FREE_FLIGHT || p->integrator == VR_MULTI_SCATTER) {
        st = free_flight_pipeline(c, A, s);
        if (st != VR_OK) return st;
        c->report_ff = true;
    } else {
        HIP_TRY(launch_render(A, s, c->type, p->integrator), "kernel launch");
    }
    HIP_TRY(hipEventRecord(c->ev_stop, s), "hipEventRecord");
    HIP_TRY(hipMemcpyAsync(&c->h_report[0], c->d_queue, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "hipMemcpyAsync(report)");
    HIP_TRY(hipMemcpyAsync(&c->h_report[1], c->d_counters, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "hipMemcpyAsync(report)");
    if (c->report_gauss) {
        HIP_TRY(hipMemcpyAsync(&c->h_report[2], A.rec_alloc, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, s),
                "hipMemcpyAsync(report)");
        HIP_TRY(hipMemcpyAsync(&c->h_report[5], A.deepq, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "hipMemcpyAsync(report)");
        HIP_TRY(hipMemcpyAsync(&c->h_report[8], A.slowq, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "hipMemcpyAsync(report)");
        HIP_TRY(hipMemcpyAsync(&c->h_report[9], A.fixq, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "hipMemcpyAsync(report)");
    }
    HIP_TRY(hipMemcpyAsync(&c->h_report[6], c->d_counters + 2, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s),
            "hipMemcpyAsync(report)");
    HIP_TRY(hipEventRecord(c->ev_report, s), "hipEventRecord");
    c->stats_pending = true;
    c->last_pixels = (int64_t)A.num_tiles * 256;
    c->last_first_tile = A.first_tile;
    c->last_tile_stride = A.tile_stride;
    c->last_tiles_x = A.tiles_x;
    c->last_w = A.width;
    c->last_h = A.height;
    return VR_OK;
}

// Synchronous frame into the context's device frame buffer (vr_render, vr_render_record,
// vr_count_work): a frame that outgrew the record buffers sized from earlier frames is rendered
// again with grown ones; pixels / paths over every per-ray capacity fail the call.
vr_status render_sync(vr_ctx* c, RenderArgs& A, const vr_render_params* p, bool stats, const char* what) {
    struct Reported {  // every exit reports this frame's outcome itself: vr_synchronize must not report it again
        vr_ctx* c;
        ~Reported() { c->sync_pending = false; }
    } reported{c};
    for (int attempt = 1;; ++attempt) {
        vr_status st = launch(c, A, p, c->stream, stats);
        if (st != VR_OK) return st;
        if ((st = collect(c)) != VR_OK) return st;
        if (!frame_exceeded(c)) break;
        if (attempt >= kFrameAttempts)
            return fail(VR_ERR_OVERFLOW, "scatter-record / shadow-ray queue capacity could not be sized");
    }
    if (c->h_report[1] != 0)
        return fail(VR_ERR_OVERFLOW, std::to_string(c->h_report[1]) + std::string(" ") + what);
    return VR_OK;
}

}  // namespace

extern "C" {

vr_status vr_init(int device, vr_ctx** out) {
    if (!out) return fail(VR_ERR_INVALID, "vr_init: out is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return fail(VR_ERR_HIP, "vr_init: no HIP device available");
    if (device < 0 || device >= n) return fail(VR_ERR_INVALID, "vr_init: device index out of range");
    HIP_TRY(hipSetDevice(device), "hipSetDevice");
    vr_ctx* c = new vr_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_counters, 4 * sizeof(uint32_t)) != hipSuccess ||
        hipHostMalloc(&c->h_report, kReportWords * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&c->h_sizing, 4 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
        hipEventCreate(&c->ev_start) != hipSuccess || hipEventCreate(&c->ev_stop) != hipSuccess ||
        hipEventCreate(&c->ev_report) != hipSuccess ||
        hipEventCreate(&c->ev_stage[0]) != hipSuccess || hipEventCreate(&c->ev_stage[1]) != hipSuccess ||
        hipEventCreate(&c->ev_stage[2]) != hipSuccess) {
        vr_destroy(c);
        return fail(VR_ERR_HIP, "vr_init: failed to create stream/workspace");
    }
    std::memset(c->h_report, 0, kReportWords * sizeof(uint32_t));
    *out = c;
    return VR_OK;
}

vr_status vr_device_count(int32_t* n) {
    if (!n) return fail(VR_ERR_INVALID, "vr_device_count: NULL argument");
    int k = 0;
    if (hipGetDeviceCount(&k) != hipSuccess) k = 0;
    *n = k;
    return VR_OK;
}

vr_status vr_init_multi(int32_t ndev, const int32_t* devices, vr_ctx** out) {
    if (!out) return fail(VR_ERR_INVALID, "vr_init_multi: out is NULL");
    vr_group* g = nullptr;
    vr_status st = vr::group_create(ndev, devices, &g);
    if (st != VR_OK) return st;
    vr_ctx* c = nullptr;
    if ((st = vr_init(devices ? devices[0] : 0, &c)) != VR_OK) {
        std::string m = vr_last_error();
        vr::group_destroy(g);
        return fail(st, m);
    }
    c->group = g;
    *out = c;
    return VR_OK;
}

int32_t vr_ctx_num_devices(const vr_ctx* c) { return !c ? 0 : c->group ? vr::group_size(c->group) : 1; }

int32_t vr_ctx_uses_rccl(const vr_ctx* c) { return c && c->group && vr::group_uses_rccl(c->group) ? 1 : 0; }

vr_status vr_get_rank_stats(vr_ctx* c, int32_t rank, vr_render_stats* out) {
    if (!c || !out) return fail(VR_ERR_INVALID, "vr_get_rank_stats: NULL argument");
    if (!c->group) {
        if (rank != 0) return fail(VR_ERR_INVALID, "vr_get_rank_stats: rank out of range");
        return vr_get_stats(c, out);
    }
    vr_ctx* r = vr::group_rank(c->group, rank);
    if (!r) return fail(VR_ERR_INVALID, "vr_get_rank_stats: rank out of range");
    return vr_get_stats(r, out);
}

void vr_destroy(vr_ctx* c) {
    if (!c) return;
    if (c->group) {
        vr::group_destroy(c->group);
        c->group = nullptr;
    }
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    free_scene(c);
    for (auto& kv : c->tables) (void)hipFree(kv.second.d);
    if (c->d_queue) (void)hipFree(c->d_queue);
    if (c->d_counters) (void)hipFree(c->d_counters);
    if (c->h_report) (void)hipHostFree(c->h_report);
    if (c->h_sizing) (void)hipHostFree(c->h_sizing);
    for (vr_ctx::Buf* b : {&c->px_first, &c->px_T, &c->rec_pos, &c->rec_meta, &c->rec_next, &c->rec_act, &c->tr, &c->rec_rad,
                           &c->rec_alloc, &c->rec_bloom, &c->slowq, &c->fixq, &c->pcg_jump, &c->ray_next,
                           &c->stack_ovf, &c->env_order, &c->env_base, &c->rec_cut, &c->rec_start, &c->deep, &c->bin_cnt, &c->bin_off, &c->bin_ent,
                           &c->ff_scratch, &c->ff_tail, &c->ff_sum, &c->ff_nee, &c->ff_fb, &c->rec_bits[0], &c->rec_bits[1],
                           &c->sfd_tmp, &c->sfd_ref, &c->sfd_loss[0], &c->sfd_loss[1], &c->sfd_out})
        if (b->p) (void)hipFree(b->p);
    if (c->d_frame) (void)hipFree(c->d_frame);
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->ev_stop) (void)hipEventDestroy(c->ev_stop);
    if (c->ev_report) (void)hipEventDestroy(c->ev_report);
    for (hipEvent_t e : c->ff_ev) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_stage)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

// Median central-chord optical depth of the scene's Gaussians and what it sets. First hit-window
// capacity of the free-flight sweep: a path scatters once the optical
// depth of the hits it crossed passes an Exp(1) target, so the hits a bounce needs scale like
// 1 / (optical depth per hit). Median over (up to 4096 sampled) Gaussians of the central-chord depth
// density * norm * sqrt(2 pi / d^T M d) along a fixed direction per Gaussian; window0 = the power of
// two >= 64 / median, in [4, 32] (measured optima: 1000_random, median 4.5 -> 16; make_random and
// 10k_random, median ~450 -> 4). Results do not depend on it (every window yields the same events).
double scene_median_chord_depth(const HostScene& s) {
    const size_t N = s.pre.size();
    if (N == 0) return 0.0;
    const size_t step = std::max<size_t>(1, N / 4096);
    static const float dirs[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0.57735027f, 0.57735027f, 0.57735027f}};
    std::vector<double> tau;
    for (size_t i = 0, k = 0; i < N; i += step, ++k) {
        const GaussianPre& p = s.pre[i];
        const float* d = dirs[k & 3];
        const float* m = p.inv_cov;  // 00 01 02 11 12 22
        const double a = (double)m[0] * d[0] * d[0] + (double)m[3] * d[1] * d[1] + (double)m[5] * d[2] * d[2] +
                         2.0 * ((double)m[1] * d[0] * d[1] + (double)m[2] * d[0] * d[2] + (double)m[4] * d[1] * d[2]);
        if (a > 0.0 && std::isfinite(a)) tau.push_back((double)p.density * (double)p.norm * std::sqrt(2.0 * M_PI / a));
    }
    if (tau.empty()) return 0.0;
    std::nth_element(tau.begin(), tau.begin() + tau.size() / 2, tau.end());
    return tau[tau.size() / 2];
}
// Mean number of 3-sigma ellipsoids covering a point of the scene's bounding box.
double scene_overlap(const HostScene& s) {
    double vol = 0.0, lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const GaussianPre& p : s.pre) {
        const double a = p.cov[0], b = p.cov[1], cc = p.cov[2], d = p.cov[3], e = p.cov[4], f = p.cov[5];
        const double det = a * (d * f - e * e) - b * (b * f - e * cc) + cc * (b * e - d * cc);
        if (det > 0.0) vol += 4.0 / 3.0 * M_PI * 27.0 * std::sqrt(det);
        const double ext[3] = {3.0 * std::sqrt(std::max(a, 0.0)), 3.0 * std::sqrt(std::max(d, 0.0)), 3.0 * std::sqrt(std::max(f, 0.0))};
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], (double)p.mean[k] - ext[k]);
            hi[k] = std::max(hi[k], (double)p.mean[k] + ext[k]);
        }
    }
    const double box = (hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]);
    return box > 0.0 && std::isfinite(box) ? vol / box : 0.0;
}
// ... and a path starting inside a dense region first meets every Gaussian covering its start point
// (all with entry key 0): scenes whose ellipsoids overlap >= 8-fold on average start at 8
// (1M make_random, overlap 17: 190 vs 205 ms at 4; 100k, overlap 1.8, and 10k_random, 0.2: 4 best).
int32_t scene_window0(double med, double overlap) {
    if (!(med > 0.0)) return 8;
    int32_t w = overlap >= 8.0 ? 8 : 4;
    while (w < 32 && (double)w * med < 64.0) w *= 2;
    return w;
}
// Refill threshold of the shadow-ray kernel: a refill (queue claim + ray setup) costs about a node
// step; opaque scenes end most shadow rays after a few steps (optical depth 104 reached), so waves
// refill in larger batches there (while-while kernel, measured: 56 for make_random and 10k_random,
// 16-32 alike for 1000_random).
#ifndef VR_NEE_REFILL_OPAQUE
#define VR_NEE_REFILL_OPAQUE 56
#endif
#ifndef VR_NEE_REFILL_TRANSLUCENT
#define VR_NEE_REFILL_TRANSLUCENT 24
#endif
int32_t scene_nee_refill(double med) { return med >= 50.0 ? VR_NEE_REFILL_OPAQUE : VR_NEE_REFILL_TRANSLUCENT; }

vr_status vr_upload_scene(vr_ctx* c, const vr_scene* sc) {
    if (!c || !sc) return fail(VR_ERR_INVALID, "vr_upload_scene: NULL argument");
    if (c->group) return vr::group_upload(c->group, sc);
    const HostScene& s = sc->s;
    if (s.lights.size() > (size_t)kMaxLights) return fail(VR_ERR_UNSUPPORTED, "more than 16 lights");
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    if (vr_status cs = collect(c); cs != VR_OK) return cs;  // the previous scene's last report, before the reset
    free_scene(c);
    c->march_big = false;
    c->nee_inline = false;  // (nee_hint is kept: the inverse loop re-uploads every iteration and renders alike)
    c->type = s.type;
    c->lights.clear();
    for (const vr_light& l : s.lights)
        c->lights.push_back(LightRecord{l.position[0], l.position[1], l.position[2], l.intensity[0], l.intensity[1], l.intensity[2]});
    std::memcpy(c->env, s.env, sizeof(c->env));
    for (int k = 0; k < 3; ++k) {
        c->bmin[k] = INFINITY;
        c->bmax[k] = -INFINITY;
    }
    if (s.type == VR_VOLUME_GAUSSIANS) {
        const size_t N = s.pre.size();
        if (N >= (1u << 27)) return fail(VR_ERR_UNSUPPORTED, "more than 2^27 Gaussians");
        const double med = scene_median_chord_depth(s);
        c->auto_window0 = scene_window0(med, scene_overlap(s));
        c->auto_nee_refill = scene_nee_refill(med);
        // long per-bounce collections and sweeps (many translucent Gaussians per bounce: C2's 1000_random, median
        // 4.5) favour the phase-scheduled kernel; short ones its per-iteration scheduling cost (C3/C4/C5, main)
        c->auto_ff_sm = N >= 256 && med > 0.0 && med < 16.0;
        std::vector<float> boxes(6 * N);
        for (int k = 0; k < 3; ++k) c->sig_max[k] = 0.0f;
        for (size_t i = 0; i < N; ++i) {
            const float dg[3] = {s.pre[i].cov[0], s.pre[i].cov[3], s.pre[i].cov[5]};
            for (int k = 0; k < 3; ++k) c->sig_max[k] = std::max(c->sig_max[k], std::sqrt(std::max(dg[k], 0.0f)));
            gaussian_bounds(s.pre[i], &boxes[6 * i], &boxes[6 * i + 3]);
            for (int k = 0; k < 3; ++k) {
                c->bmin[k] = std::min(c->bmin[k], boxes[6 * i + k]);
                c->bmax[k] = std::max(c->bmax[k], boxes[6 * i + 3 + k]);
            }
        }
        c->last_upload_device_bvh = false;
        if (c->opt_device_bvh && N >= kDeviceBvhMin) {
            vr_status ds = upload_device_bvh(c, s, boxes);
            if (ds == VR_OK) {
                if ((ds = upload_parents(c)) != VR_OK) return ds;
                c->has_scene = true;
                return VR_OK;
            }
            if (ds != VR_ERR_UNSUPPORTED) return ds;  // UNSUPPORTED: too deep for the stacks -> host build
            free_scene(c);
        }
        BVHBuild b = build_bvh(boxes);
        if (b.max_depth > kMaxDepth + 1) return fail(VR_ERR_OVERFLOW, "BVH deeper than the traversal stack");
        std::vector<GaussianRecord> rec(std::max<size_t>(N, 1));
        for (size_t j = 0; j < N; ++j) {
            const GaussianPre& p = s.pre[b.order[j]];
            rec[j] = GaussianRecord{p.mean[0], p.mean[1], p.mean[2], p.density, p.inv_cov[0], p.inv_cov[1],
                                    p.inv_cov[2], p.inv_cov[3], p.inv_cov[4], p.inv_cov[5], p.norm, p.albedo};
        }
        HIP_TRY(hipMalloc(&c->d_gauss, rec.size() * sizeof(GaussianRecord)), "hipMalloc(records)");
        HIP_TRY(hipMemcpy(c->d_gauss, rec.data(), rec.size() * sizeof(GaussianRecord), hipMemcpyHostToDevice), "hipMemcpy(records)");
        if (vr_status ws = upload_whitened(c, N); ws != VR_OK) return ws;
        {
            std::vector<uint32_t> order(std::max<size_t>(N, 1), 0u);
            for (size_t j = 0; j < N; ++j) order[j] = (uint32_t)b.order[j];
            HIP_TRY(hipMalloc(&c->d_order, order.size() * sizeof(uint32_t)), "hipMalloc(order)");
            HIP_TRY(hipMemcpy(c->d_order, order.data(), order.size() * sizeof(uint32_t), hipMemcpyHostToDevice), "hipMemcpy(order)");
        }
        HIP_TRY(hipMalloc(&c->d_nodes, b.nodes.size() * sizeof(BVHNode)), "hipMalloc(nodes)");
        HIP_TRY(hipMemcpy(c->d_nodes, b.nodes.data(), b.nodes.size() * sizeof(BVHNode), hipMemcpyHostToDevice), "hipMemcpy(nodes)");
        c->num_prims = (int32_t)N;
        c->bvh_depth = b.max_depth;
        if (vr_status hs = upload_half_nodes(c, b.nodes); hs != VR_OK) return hs;
        c->num_nodes = b.nodes.size();
    } else {
        const size_t N = s.spheres.size();
        if (N > 16) return fail(VR_ERR_UNSUPPORTED, "the device sphere path supports at most 16 spheres");
        std::vector<SphereRecord> rec(std::max<size_t>(N, 1));
        for (size_t i = 0; i < N; ++i) {
            const vr_sphere& sp = s.spheres[i];
            rec[i] = SphereRecord{sp.center[0], sp.center[1], sp.center[2], sp.radius, sp.sigma_a, sp.sigma_s, 0, 0};
            float lo[3], hi[3];
            sphere_bounds(sp, lo, hi);
            for (int k = 0; k < 3; ++k) {
                c->bmin[k] = std::min(c->bmin[k], lo[k]);
                c->bmax[k] = std::max(c->bmax[k], hi[k]);
            }
        }
        HIP_TRY(hipMalloc(&c->d_spheres, rec.size() * sizeof(SphereRecord)), "hipMalloc(spheres)");
        HIP_TRY(hipMemcpy(c->d_spheres, rec.data(), rec.size() * sizeof(SphereRecord), hipMemcpyHostToDevice), "hipMemcpy(spheres)");
        c->num_prims = (int32_t)N;
    }
    if (c->num_prims == 0)
        for (int k = 0; k < 3; ++k) c->bmin[k] = c->bmax[k] = 0.0f;
    if (vr_status ps = upload_parents(c); ps != VR_OK) return ps;
    c->has_scene = true;
    return VR_OK;
}

uint32_t vr_num_tiles(uint32_t W, uint32_t H) { return ((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile); }

vr_status vr_render(vr_ctx* c, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H, float* rgb) {
    if (!c || !rgb) return fail(VR_ERR_INVALID, "vr_render: NULL argument");
    if (c->group) return vr::group_render(c->group, cam, p, W, H, rgb);
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    RenderArgs A;
    vr_status st = fill_args(c, cam, p, W, H, A);
    if (st != VR_OK) return st;
    size_t bytes = (size_t)W * H * 3 * sizeof(float);
    if (bytes > c->frame_cap) {
        if (c->d_frame) (void)hipFree(c->d_frame);
        c->d_frame = nullptr;
        HIP_TRY(hipMalloc(&c->d_frame, bytes), "hipMalloc(frame)");
        c->frame_cap = bytes;
    }
    A.first_tile = 0;
    A.tile_stride = 1;
    A.num_tiles = vr_num_tiles(W, H);
    A.packed = 0;
    A.out = c->d_frame;
    st = render_sync(c, A, p, false, "pixels / paths exceeded a per-ray capacity (NaN)");
    if (st != VR_OK) return st;
    HIP_TRY(hipMemcpy(rgb, c->d_frame, bytes, hipMemcpyDeviceToHost), "hipMemcpy(frame)");
    return VR_OK;
}

vr_status vr_render_tiles_device(vr_ctx* c, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H,
                                 uint32_t first_tile, uint32_t tile_stride, uint32_t num_tiles, int32_t packed,
                                 float* d_out, void* stream) {
    c = first_device(c);
    if (!c || !d_out) return fail(VR_ERR_INVALID, "vr_render_tiles_device: NULL argument");
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    RenderArgs A;
    vr_status st = fill_args(c, cam, p, W, H, A);
    if (st != VR_OK) return st;
    uint32_t total = vr_num_tiles(W, H);
    if (tile_stride == 0) return fail(VR_ERR_INVALID, "tile_stride must be >= 1");
    if (num_tiles == 0) return VR_OK;
    if ((uint64_t)first_tile + (uint64_t)(num_tiles - 1) * tile_stride >= total)
        return fail(VR_ERR_INVALID, "tile range exceeds the frame");
    if (num_tiles >= (1u << 24)) return fail(VR_ERR_INVALID, "too many tiles in one call");
    A.first_tile = first_tile;
    A.tile_stride = tile_stride;
    A.num_tiles = num_tiles;
    A.packed = packed ? 1 : 0;
    A.out = d_out;
    return launch(c, A, p, (hipStream_t)stream);  // outcome: vr_synchronize / vr_get_stats
}

vr_status vr_count_work(vr_ctx* c, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H,
                        uint32_t first_tile, uint32_t tile_stride, uint32_t num_tiles, uint64_t counts[16]) {
    c = first_device(c);
    if (!c || !counts) return fail(VR_ERR_INVALID, "vr_count_work: NULL argument");
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    RenderArgs A;
    vr_status st = fill_args(c, cam, p, W, H, A);
    if (st != VR_OK) return st;
    if (p->integrator != VR_RAYMARCH_GAUSSIANS && p->integrator != VR_PURE_RAYMARCH && p->integrator != VR_FREE_FLIGHT &&
        p->integrator != VR_MULTI_SCATTER)
        return fail(VR_ERR_UNSUPPORTED, "vr_count_work: Gaussian ray-march and free-flight integrators only");
    uint32_t total = vr_num_tiles(W, H);
    if (tile_stride == 0 || num_tiles == 0 || (uint64_t)first_tile + (uint64_t)(num_tiles - 1) * tile_stride >= total)
        return fail(VR_ERR_INVALID, "vr_count_work: bad tile range");
    float* d_out = nullptr;
    unsigned long long* d_work = nullptr;
    HIP_TRY(hipMalloc(&d_out, (size_t)num_tiles * 256 * 3 * sizeof(float)), "hipMalloc(count_work out)");
    HIP_TRY(hipMalloc(&d_work, 16 * sizeof(unsigned long long)), "hipMalloc(count_work)");
    HIP_TRY(hipMemsetAsync(d_work, 0, 16 * sizeof(unsigned long long), c->stream), "hipMemsetAsync");
    A.first_tile = first_tile;
    A.tile_stride = tile_stride;
    A.num_tiles = num_tiles;
    A.packed = 1;
    A.out = d_out;
    A.work = d_work;
    unsigned long long h[16] = {0};
    for (int attempt = 0;; ++attempt) {  // a frame over the record capacity is counted again (grown)
        if (hipMemsetAsync(d_work, 0, 16 * sizeof(unsigned long long), c->stream) != hipSuccess) break;
        st = launch(c, A, p, c->stream, true);
        if (st == VR_OK) st = collect(c);
        if (st != VR_OK || !frame_exceeded(c) || attempt + 1 >= kFrameAttempts) break;
    }
    if (st == VR_OK) {
        hipError_t e = hipMemcpy(h, d_work, sizeof(h), hipMemcpyDeviceToHost);
        if (e != hipSuccess) st = hip_fail(e, "vr_count_work");
    }
    (void)hipFree(d_out);
    (void)hipFree(d_work);
    for (int i = 0; i < 16; ++i) counts[i] = h[i];
    return st;
}

vr_status vr_unshuffle_tiles_device(vr_ctx* c, const float* d_slabs, uint32_t nslabs, uint32_t tiles_per_slab, uint32_t W,
                                    uint32_t H, float* d_image, void* stream) {
    c = first_device(c);
    if (!c || !d_slabs || !d_image || nslabs == 0) return fail(VR_ERR_INVALID, "vr_unshuffle_tiles_device: bad argument");
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    HIP_TRY(launch_unshuffle(d_slabs, nslabs, tiles_per_slab, (W + kTile - 1) / kTile, W, H, d_image, (hipStream_t)stream),
            "unshuffle launch");
    return VR_OK;
}

vr_status vr_unshuffle_tiles_part_device(vr_ctx* c, const float* d_slabs, uint32_t first, uint32_t nslabs, uint32_t stride,
                                         uint32_t tiles_per_slab, uint32_t W, uint32_t H, float* d_image, void* stream) {
    c = first_device(c);
    if (!c || !d_slabs || !d_image || nslabs == 0 || stride == 0 || (uint64_t)first + nslabs > stride)
        return fail(VR_ERR_INVALID, "vr_unshuffle_tiles_part_device: bad argument");
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    HIP_TRY(launch_unshuffle_part(d_slabs, first, nslabs, stride, tiles_per_slab, (W + kTile - 1) / kTile, W, H, d_image,
                                  (hipStream_t)stream),
            "unshuffle launch");
    return VR_OK;
}

// A full frame into the context's device frame buffer; slot 0/1 records RECORD_PIXEL_GAUSSIANS
// bitsets (MultiScatterGaussians only), slot -1 renders without recording.
static vr_status render_frame_device(vr_ctx* c, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H,
                                     int32_t slot) {
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    RenderArgs A;
    vr_status st = fill_args(c, cam, p, W, H, A);
    if (st != VR_OK) return st;
    const uint64_t npix = (uint64_t)W * H;
    if (slot >= 0) {
        const uint64_t words = ((uint64_t)c->num_prims + 31) / 32;
        const size_t bytes = std::max<size_t>((size_t)(words * npix * 4), 4);
        if ((st = grow(c->rec_bits[slot], bytes, "hipMalloc(pixel Gaussian bits)")) != VR_OK) return st;
        HIP_TRY(hipMemsetAsync(c->rec_bits[slot].p, 0, bytes, c->stream), "hipMemsetAsync(bits)");
        c->rec_npix[slot] = (uint32_t)npix;
        c->rec_n[slot] = (uint32_t)c->num_prims;
        A.rec_bits = (uint32_t*)c->rec_bits[slot].p;
        A.rec_npix = (uint32_t)npix;
    }
    size_t fb = npix * 3 * sizeof(float);
    if (fb > c->frame_cap) {
        if (c->d_frame) (void)hipFree(c->d_frame);
        c->d_frame = nullptr;
        HIP_TRY(hipMalloc(&c->d_frame, fb), "hipMalloc(frame)");
        c->frame_cap = fb;
    }
    A.first_tile = 0;
    A.tile_stride = 1;
    A.num_tiles = vr_num_tiles(W, H);
    A.packed = 0;
    A.out = c->d_frame;
    return render_sync(c, A, p, false, "pixels / paths exceeded a per-ray capacity (NaN)");
}

vr_status vr_render_record(vr_ctx* c, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H, float* rgb,
                           int32_t slot) {
    c = first_device(c);
    if (!c || !rgb || !p) return fail(VR_ERR_INVALID, "vr_render_record: NULL argument");
    if (slot != 0 && slot != 1) return fail(VR_ERR_INVALID, "vr_render_record: slot must be 0 or 1");
    if (p->integrator != VR_MULTI_SCATTER)
        return fail(VR_ERR_INVALID, "vr_render_record: MultiScatterGaussians only (integrator.h:532-536)");
    vr_status st = render_frame_device(c, cam, p, W, H, slot);
    if (st != VR_OK) return st;
    HIP_TRY(hipMemcpy(rgb, c->d_frame, (size_t)W * H * 3 * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy(frame)");
    return VR_OK;
}

vr_status vr_get_pixel_gaussians(vr_ctx* c, int32_t slot, uint32_t* bits, size_t n_words) {
    c = first_device(c);
    if (!c || !bits || (slot != 0 && slot != 1)) return fail(VR_ERR_INVALID, "vr_get_pixel_gaussians: bad argument");
    const size_t need = (size_t)((c->rec_n[slot] + 31) / 32) * c->rec_npix[slot];
    if (!c->rec_bits[slot].p || c->rec_npix[slot] == 0) return fail(VR_ERR_INVALID, "slot holds no recording");
    if (n_words != need) return fail(VR_ERR_INVALID, "n_words must be ceil(N/32) * W * H = " + std::to_string(need));
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    HIP_TRY(hipMemcpy(bits, c->rec_bits[slot].p, need * 4, hipMemcpyDeviceToHost), "hipMemcpy(bits)");
    return VR_OK;
}

vr_status vr_sfd_loss_diff(vr_ctx* c, const float* loss_base, const float* loss_plus, uint32_t W, uint32_t H, double* out,
                           size_t n) {
    c = first_device(c);
    if (!c || !loss_base || !loss_plus || !out) return fail(VR_ERR_INVALID, "vr_sfd_loss_diff: NULL argument");
    const uint32_t npix = W * H;
    if (c->rec_npix[0] != npix || c->rec_npix[1] != npix || c->rec_n[0] != c->rec_n[1] || n != c->rec_n[0])
        return fail(VR_ERR_INVALID, "vr_sfd_loss_diff: slots 0 and 1 must hold recordings of this frame size and n Gaussians");
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    vr_status st = grow(c->sfd_tmp, (size_t)npix * 8 + n * 8 + 16, "hipMalloc(sfd)");
    if (st != VR_OK) return st;
    float* lb = (float*)c->sfd_tmp.p;
    float* lp = lb + npix;
    double* d_out = (double*)((char*)c->sfd_tmp.p + (((size_t)npix * 8 + 15) & ~(size_t)15));
    HIP_TRY(hipMemcpyAsync(lb, loss_base, (size_t)npix * 4, hipMemcpyHostToDevice, c->stream), "hipMemcpyAsync");
    HIP_TRY(hipMemcpyAsync(lp, loss_plus, (size_t)npix * 4, hipMemcpyHostToDevice, c->stream), "hipMemcpyAsync");
    HIP_TRY(hipMemsetAsync(d_out, 0, n * 8, c->stream), "hipMemsetAsync");
    if (n > 0)
        HIP_TRY(launch_sfd_loss_diff((const uint32_t*)c->rec_bits[0].p, (const uint32_t*)c->rec_bits[1].p, lb, lp, npix,
                                     (uint32_t)n, d_out, c->stream), "sfd launch");
    HIP_TRY(hipMemcpyAsync(out, d_out, n * 8, hipMemcpyDeviceToHost, c->stream), "hipMemcpyAsync");
    HIP_TRY(hipStreamSynchronize(c->stream), "sfd");
    return VR_OK;
}

}  // extern "C"

namespace vr {

// ---- device side of the inverse loop (host/vr_inverse.cpp) ----
vr_status sfd_set_reference(vr_ctx* c, const float* I_ref, uint32_t W, uint32_t H) {
    c = first_device(c);
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    const size_t npix = (size_t)W * H;
    vr_status st;
    if ((st = grow(c->sfd_ref, npix * 12, "hipMalloc(I_ref)")) != VR_OK) return st;
    for (auto& b : c->sfd_loss)
        if ((st = grow(b, npix * 4, "hipMalloc(pixel losses)")) != VR_OK) return st;
    HIP_TRY(hipMemcpy(c->sfd_ref.p, I_ref, npix * 12, hipMemcpyHostToDevice), "hipMemcpy(I_ref)");
    return VR_OK;
}

// One forward render of the loop (slot 0/1: recorded, -1: plain) and its per-pixel L1 losses against
// the reference image into device loss buffer `which`; loss_host (W*H floats) receives a copy, and
// rgb (3*W*H floats, may be NULL) the frame.
vr_status sfd_render(vr_ctx* c, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H, int32_t slot,
                     int which, float* loss_host, float* rgb) {
    c = first_device(c);
    vr_status st = render_frame_device(c, cam, p, W, H, slot);
    if (st != VR_OK) return st;
    const uint32_t npix = W * H;
    HIP_TRY(launch_pixel_losses(c->d_frame, (const float*)c->sfd_ref.p, npix, (float*)c->sfd_loss[which].p, c->stream),
            "pixel losses");
    HIP_TRY(hipMemcpyAsync(loss_host, c->sfd_loss[which].p, (size_t)npix * 4, hipMemcpyDeviceToHost, c->stream),
            "hipMemcpyAsync(losses)");
    if (rgb)
        HIP_TRY(hipMemcpyAsync(rgb, c->d_frame, (size_t)npix * 12, hipMemcpyDeviceToHost, c->stream), "hipMemcpyAsync(frame)");
    HIP_TRY(hipStreamSynchronize(c->stream), "sfd render");
    return VR_OK;
}

// out[g] = sum over the union of the pixels recorded for g in slots 0 and 1 of loss[1] - loss[0].
vr_status sfd_loss_diff_device(vr_ctx* c, uint32_t npix, double* out, size_t n) {
    c = first_device(c);
    vr_status st = grow(c->sfd_out, std::max<size_t>(n, 1) * 8, "hipMalloc(sfd)");
    if (st != VR_OK) return st;
    HIP_TRY(hipMemsetAsync(c->sfd_out.p, 0, n * 8, c->stream), "hipMemsetAsync");
    if (n > 0)
        HIP_TRY(launch_sfd_loss_diff((const uint32_t*)c->rec_bits[0].p, (const uint32_t*)c->rec_bits[1].p,
                                     (const float*)c->sfd_loss[0].p, (const float*)c->sfd_loss[1].p, npix, (uint32_t)n,
                                     (double*)c->sfd_out.p, c->stream),
                "sfd launch");
    HIP_TRY(hipMemcpyAsync(out, c->sfd_out.p, n * 8, hipMemcpyDeviceToHost, c->stream), "hipMemcpyAsync");
    HIP_TRY(hipStreamSynchronize(c->stream), "sfd");
    return VR_OK;
}

}  // namespace vr

extern "C" {

vr_status vr_set_option(vr_ctx* c, int32_t option, int64_t value) {
    if (!c) return fail(VR_ERR_INVALID, "vr_set_option: NULL ctx");
    if (c->group) return vr::group_set_option(c->group, option, value);
    switch (option) {
        case VR_OPT_HALF_NODES:
            if (value != 0 && value != 1) return fail(VR_ERR_INVALID, "VR_OPT_HALF_NODES must be 0 or 1");
            c->opt_half_nodes = value;
            return VR_OK;
        case VR_OPT_SECONDARY_BUDGET:
            if (value != 0 && value != 1) return fail(VR_ERR_INVALID, "VR_OPT_SECONDARY_BUDGET must be 0 or 1");
            c->opt_secondary_budget = value;
            return VR_OK;
        case VR_OPT_FF_WINDOW0:
            if (value < 0 || value > kFFHitCap) return fail(VR_ERR_INVALID, "VR_OPT_FF_WINDOW0 must be in [0, 128]");
            c->opt_ff_window0 = value;
            return VR_OK;
        case VR_OPT_FF_NEE_QUEUE:
            if (value < 0 || value > (int64_t)kFFNeeMaxPerPath) return fail(VR_ERR_INVALID, "VR_OPT_FF_NEE_QUEUE must be in [0, 16]");
            c->opt_ff_nee_queue = value;
            c->nee_inline = false;
            return VR_OK;
        case VR_OPT_DEVICE_BVH:
            if (value != 0 && value != 1) return fail(VR_ERR_INVALID, "VR_OPT_DEVICE_BVH must be 0 or 1");
            c->opt_device_bvh = value;
            return VR_OK;
        case VR_OPT_MARCH_BINNED:
            if (value != 0 && value != 1) return fail(VR_ERR_INVALID, "VR_OPT_MARCH_BINNED must be 0 or 1");
            c->opt_march_binned = value;
            return VR_OK;
        case VR_OPT_FF_SOLVER:
            if (value < 0 || value > 4) return fail(VR_ERR_INVALID, "VR_OPT_FF_SOLVER must be in [0, 4]");
            c->opt_ff_solver = value;
            return VR_OK;
        case VR_OPT_START_SUBTREE:
            if (value != 0 && value != 1) return fail(VR_ERR_INVALID, "VR_OPT_START_SUBTREE must be 0 or 1");
            c->opt_start_subtree = value;
            return VR_OK;
        case VR_OPT_FF_KERNEL:
            if (value < 0 || value > 2) return fail(VR_ERR_INVALID, "VR_OPT_FF_KERNEL must be in [0, 2]");
            c->opt_ff_kernel = value;
            return VR_OK;
        case VR_OPT_SEC_TIGHT:
            if (value != 0 && value != 1) return fail(VR_ERR_INVALID, "VR_OPT_SEC_TIGHT must be 0 or 1");
            c->opt_sec_tight = value;
            return VR_OK;
        case VR_OPT_MARCH_WIDE_MIN:
            if (value < 0 || value > 0xffffffffll) return fail(VR_ERR_INVALID, "VR_OPT_MARCH_WIDE_MIN must be in [0, 2^32)");
            c->opt_march_wide_min = value;
            return VR_OK;
        case VR_OPT_RECORD_CAPACITY:
            if ((value != 0 && value < 4096) || value > 0x3fffffff)
                return fail(VR_ERR_INVALID, "VR_OPT_RECORD_CAPACITY must be 0 or in [4096, 2^30)");
            c->rec_hint = c->ovf_hint = (uint64_t)value;
            return VR_OK;
        default:
            return fail(VR_ERR_INVALID, "vr_set_option: unknown option " + std::to_string(option));
    }
}

vr_status vr_get_option(vr_ctx* c, int32_t option, int64_t* value) {
    c = first_device(c);
    if (!c || !value) return fail(VR_ERR_INVALID, "vr_get_option: NULL argument");
    switch (option) {
        case VR_OPT_HALF_NODES: *value = c->opt_half_nodes; return VR_OK;
        case VR_OPT_SECONDARY_BUDGET: *value = c->opt_secondary_budget; return VR_OK;
        case VR_OPT_FF_WINDOW0: *value = c->opt_ff_window0; return VR_OK;
        case VR_OPT_RECORD_CAPACITY: *value = (int64_t)c->rec_hint; return VR_OK;
        case VR_OPT_DEVICE_BVH: *value = c->opt_device_bvh; return VR_OK;
        case VR_OPT_FF_NEE_QUEUE: *value = c->opt_ff_nee_queue; return VR_OK;
        case VR_OPT_MARCH_BINNED: *value = c->opt_march_binned; return VR_OK;
        case VR_OPT_FF_SOLVER: *value = c->opt_ff_solver; return VR_OK;
        case VR_OPT_START_SUBTREE: *value = c->opt_start_subtree; return VR_OK;
        case VR_OPT_SEC_TIGHT: *value = c->opt_sec_tight; return VR_OK;
        case VR_OPT_MARCH_WIDE_MIN: *value = c->opt_march_wide_min; return VR_OK;
        case VR_OPT_FF_KERNEL: *value = c->opt_ff_kernel; return VR_OK;
        default: return fail(VR_ERR_INVALID, "vr_get_option: unknown option " + std::to_string(option));
    }
}

vr_status vr_synchronize(vr_ctx* c) {
    if (!c) return fail(VR_ERR_INVALID, "vr_synchronize: NULL ctx");
    if (c->group) return vr::group_synchronize(c->group);
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    vr_status st = collect(c);
    if (st != VR_OK || !c->sync_pending) return st;
    c->sync_pending = false;  // (a frame that vr_get_stats or an upload collected first is still reported here)
    if (frame_exceeded(c))
        return fail(VR_ERR_RETRY, "the last frame outgrew the scatter-record buffers / shadow-ray queue sized from earlier frames; "
                                  "they have been grown: render it again");
    if (c->h_report[1] != 0)
        return fail(VR_ERR_OVERFLOW, std::to_string(c->h_report[1]) + " pixels / paths of the last frame exceeded a "
                                     "per-ray capacity (NaN)");
    return VR_OK;
}

vr_status vr_get_fallback_pixels(vr_ctx* c, uint32_t* xy, size_t cap, size_t* n) {
    c = first_device(c);
    if (!c || !n || (cap > 0 && !xy)) return fail(VR_ERR_INVALID, "vr_get_fallback_pixels: bad argument");
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    vr_status st = collect(c);
    if (st != VR_OK) return st;
    const size_t count = std::min<size_t>(c->h_report[0], c->queue_cap);
    *n = count;
    if (count == 0 || cap == 0) return VR_OK;
    std::vector<uint32_t> q(std::min(count, cap));
    HIP_TRY(hipMemcpy(q.data(), c->d_queue + 1, q.size() * sizeof(uint32_t), hipMemcpyDeviceToHost), "hipMemcpy(queue)");
    for (size_t i = 0; i < q.size(); ++i) {  // tile_pixel (kernels/vr_dev_common.h): tile-local id << 8 | lane
        const uint32_t lane = q[i] & 255u, wv = lane >> 6, ln = lane & 63u;
        const uint32_t tile = c->last_first_tile + (q[i] >> 8) * c->last_tile_stride;
        xy[2 * i] = (tile % c->last_tiles_x) * kTile + (wv & 1u) * 8u + (ln & 7u);
        xy[2 * i + 1] = (tile / c->last_tiles_x) * kTile + (wv >> 1) * 8u + (ln >> 3);
    }
    return VR_OK;
}

vr_status vr_debug_pixel_records(vr_ctx* c, uint32_t x, uint32_t y, float* out, size_t cap, size_t row_in, size_t* n,
                                 size_t* row_out) {
    c = first_device(c);
    if (!c || !n || (cap > 0 && !out)) return fail(VR_ERR_INVALID, "vr_debug_pixel_records: bad argument");
    if (!c->report_gauss) return fail(VR_ERR_INVALID, "vr_debug_pixel_records: the last frame was not a ray-march frame");
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    vr_status st = collect(c);
    if (st != VR_OK) return st;
    // the pixel's tile-local index (vr_dev_common.h tile_pixel: wave = 8x8 quadrant, lane row-major)
    const uint32_t tx = x / kTile, ty = y / kTile, g = ty * c->last_tiles_x + tx;
    if (x >= c->last_w || y >= c->last_h || g < c->last_first_tile || (g - c->last_first_tile) % c->last_tile_stride)
        return fail(VR_ERR_INVALID, "vr_debug_pixel_records: pixel not rendered by the last frame");
    const uint32_t lx = x % kTile, ly = y % kTile;
    const uint32_t lane = ((lx >> 3) + 2u * (ly >> 3)) * 64u + (ly & 7u) * 8u + (lx & 7u);
    const uint32_t p = ((g - c->last_first_tile) / c->last_tile_stride) * 256u + lane;
    const uint32_t nl = (uint32_t)c->lights.size(), S = c->last_secondary_per_record, ne = S - nl, cr = 1u << VR_CHUNK_SHIFT;
    const size_t row = 9 + S;
    if (row_out) *row_out = row;
    if (cap > 0 && row_in != row)
        return fail(VR_ERR_INVALID, "vr_debug_pixel_records: rows of " + std::to_string(row_in) + " floats, the frame's are " +
                                        std::to_string(row) + " (9 + lights + env_samples)");
    uint32_t r = 0;
    HIP_TRY(hipMemcpy(&r, (uint32_t*)c->px_first.p + p, 4, hipMemcpyDeviceToHost), "hipMemcpy");
    size_t k = 0;
    std::vector<uint16_t> ord(cr * ne);
    for (; r != kNoRecord; ++k) {
        float4 pos, rad;
        uint4 meta;
        uint32_t next = kNoRecord;
        HIP_TRY(hipMemcpy(&pos, (float4*)c->rec_pos.p + r, 16, hipMemcpyDeviceToHost), "hipMemcpy");
        HIP_TRY(hipMemcpy(&meta, (uint4*)c->rec_meta.p + r, 16, hipMemcpyDeviceToHost), "hipMemcpy");
        HIP_TRY(hipMemcpy(&rad, (float4*)c->rec_rad.p + r, 16, hipMemcpyDeviceToHost), "hipMemcpy");
        HIP_TRY(hipMemcpy(&next, (uint32_t*)c->rec_next.p + r, 4, hipMemcpyDeviceToHost), "hipMemcpy");
        if (k < cap) {
            float* o = out + k * row;
            const float v[9] = {(float)meta.y, pos.x, pos.y, pos.z, pos.w, rad.x, rad.y, rad.z, (float)(meta.w & 0x7fffffffu)};
            std::copy(v, v + 9, o);
            // Tr slots: hand-out order within the record's chunk (vr_gauss.hip ray_slot / tr_slot)
            const uint32_t chunk = r / cr, rl = r % cr;
            const size_t base = (size_t)chunk * cr * S;
            if (ne > 0 && c->env_order.p)
                HIP_TRY(hipMemcpy(ord.data(), (uint16_t*)c->env_order.p + (size_t)chunk * cr * ne, ord.size() * 2,
                                  hipMemcpyDeviceToHost), "hipMemcpy");
            for (uint32_t s = 0; s < S; ++s) {
                size_t rem = 0;
                if (s < nl) rem = (size_t)s * cr + rl;
                else if (c->env_order.p) {
                    const uint16_t want = (uint16_t)((rl << 8) | (s - nl));
                    rem = (size_t)nl * cr + (size_t)(std::find(ord.begin(), ord.end(), want) - ord.begin());
                } else rem = (size_t)s * cr + rl;
                HIP_TRY(hipMemcpy(o + 9 + s, (float*)c->tr.p + base + rem, 4, hipMemcpyDeviceToHost), "hipMemcpy");
            }
        }
        r = next;
    }
    *n = k;
    return VR_OK;
}

vr_status vr_get_stats(vr_ctx* c, vr_render_stats* o) {
    if (!c || !o) return fail(VR_ERR_INVALID, "vr_get_stats: NULL argument");
    if (c->group) return vr::group_stats(c->group, o);
    HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
    vr_status st = collect(c);
    if (st != VR_OK) return st;
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev_start, c->ev_stop), "hipEventElapsedTime");
    o->kernel_ms = ms;
    o->pixels = c->last_pixels;
    o->fallback_pixels = !c->report_gauss && c->ff_launches > 0 ? c->h_report[6] : c->h_report[0];
    o->error_pixels = c->h_report[1];
    for (double& v : o->stage_ms) v = 0.0;
    if (c->staged) {
        hipEvent_t b[5] = {c->ev_start, c->ev_stage[0], c->ev_stage[1], c->ev_stage[2], c->ev_stop};
        for (int i = 0; i < 4; ++i) {
            float m = 0.0f;
            HIP_TRY(hipEventElapsedTime(&m, b[i], b[i + 1]), "hipEventElapsedTime");
            o->stage_ms[i] = m;
        }
    }
    if (!c->report_gauss && c->ff_launches > 0) {  // free-flight: [0] path kernel, [2] shadow rays, [3] accumulation
        for (uint32_t l = 0; l < c->ff_launches; ++l) {
            const hipEvent_t* e = &c->ff_ev[4 * (size_t)l];
            float m[3] = {0.0f, 0.0f, 0.0f};
            for (int i = 0; i < 3; ++i) HIP_TRY(hipEventElapsedTime(&m[i], e[i], e[i + 1]), "hipEventElapsedTime");
            o->stage_ms[0] += m[0];
            o->stage_ms[2] += m[1];
            o->stage_ms[3] += m[2];
        }
    }
    o->scatter_records = c->report_gauss ? (int64_t)c->h_report[2] : 0;
    o->secondary_rays = o->scatter_records * (int64_t)c->last_secondary_per_record;
    o->record_overflow = frame_exceeded(c) ? 1 : 0;
    o->deep_pixels = c->report_gauss ? (int64_t)std::min(c->h_report[5], kDeepQueue) : 0;
    o->slow_rays = c->report_gauss ? (int64_t)c->h_report[8] : 0;
    o->band_rays = c->report_gauss ? (int64_t)c->h_report[9] : 0;
    return VR_OK;
}

}  // extern "C"
