// Multi-GPU context (vr_init_multi): the GPUs of one node, each rank's launches issued from a host
// thread of its own.
//
// The reference parallelises its pixel loop over CPU threads (test_integrators.h:164,
// integrator.h:547); pixels are independent, so the frame is the data-parallel axis here too
// (SURVEY.md §8(e)). Every device holds a full scene replica; rank r renders the 16x16 tiles
// r, r + n, r + 2n, ... of the frame (interleaving balances dense and empty regions); the root renders
// its tiles straight into the row-major frame, every other rank into a packed slab on its own device;
// those slabs are gathered to the root device with RCCL — one ncclGroupStart/End holding ranks 1..n-1's
// ncclSend and the root's ncclRecv, over xGMI — and the root's unshuffle kernel writes them into the
// frame, which is copied to the host once.
//
// RCCL is loaded with dlopen at vr_init_multi, so libvr_hip.so itself needs no RCCL and a process
// that already carries another copy (PyTorch's) does not see symbol clashes. A device listed more
// than once shares its GPU between ranks (a rehearsal of the split on a one-GPU box): RCCL cannot
// hold two ranks on one device, so such a group moves the slabs with device copies instead.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "vr_common.h"

using namespace vr;

namespace vr {
hipError_t launch_unshuffle_part(const float* slabs, uint32_t first, uint32_t nslabs, uint32_t stride, uint32_t tiles_per_slab,
                                 uint32_t tiles_x, uint32_t W, uint32_t H, float* img, hipStream_t stream);
}

namespace {

struct Rccl {  // the RCCL entry points the group uses (rccl.h)
    void* so = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;

    std::string load() {
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (so) break;
        }
        if (!so) return std::string("cannot load librccl: ") + dlerror();
        init_all = (decltype(init_all))dlsym(so, "ncclCommInitAll");
        destroy = (decltype(destroy))dlsym(so, "ncclCommDestroy");
        group_start = (decltype(group_start))dlsym(so, "ncclGroupStart");
        group_end = (decltype(group_end))dlsym(so, "ncclGroupEnd");
        send = (decltype(send))dlsym(so, "ncclSend");
        recv = (decltype(recv))dlsym(so, "ncclRecv");
        error_string = (decltype(error_string))dlsym(so, "ncclGetErrorString");
        if (!init_all || !destroy || !group_start || !group_end || !send || !recv || !error_string)
            return "librccl lacks ncclCommInitAll / ncclSend / ncclRecv / ncclGroupStart";
        return "";
    }
};

}  // namespace

struct vr_group {
    std::vector<int> devices;
    std::vector<vr_ctx*> ranks;         // one full device context per rank
    std::vector<hipStream_t> streams;   // per rank, on its device
    std::vector<float*> slab;           // per rank, on its device: its packed tiles
    size_t slab_floats = 0;
    float* d_recv = nullptr;            // root device: the n gathered slabs
    float* d_frame = nullptr;           // root device: the row-major frame
    size_t recv_floats = 0, frame_floats = 0;
    bool use_rccl = false;
    Rccl rccl;
    std::vector<ncclComm_t> comms;
    double last_wall_ms = 0.0;
};

namespace {

vr_status hipf(hipError_t e, const char* what) { return fail(VR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e)); }
#define GHIP(expr, what)                          \
    do {                                          \
        hipError_t e_ = (expr);                   \
        if (e_ != hipSuccess) return hipf(e_, what); \
    } while (0)

vr_status ncclf(vr_group* g, ncclResult_t r, const char* what) {
    return fail(VR_ERR_HIP, std::string(what) + ": " + (g->rccl.error_string ? g->rccl.error_string(r) : "RCCL error"));
}

// Runs fn(rank) on one host thread per rank; the first failure's status and message win.
template <class F>
vr_status each_rank_parallel(vr_group* g, F fn) {
    return run_parallel((int)g->ranks.size(), fn, [&](int r) {
        return "rank " + std::to_string(r) + " (device " + std::to_string(g->devices[r]) + ")";
    });
}

vr_status grow_dev(int dev, float** p, size_t* cap, size_t floats, const char* what) {
    if (*p && *cap >= floats) return VR_OK;
    GHIP(hipSetDevice(dev), "hipSetDevice");
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    GHIP(hipMalloc(p, std::max<size_t>(floats, 1) * sizeof(float)), what);
    *cap = floats;
    return VR_OK;
}

// One frame: the root renders its own tiles straight into the row-major frame; every other rank renders
// its tiles into a packed slab, the slabs are gathered to the root and unshuffled into the frame there,
// which is then copied to the host once. Sets *again if a rank reported that the frame outgrew its
// buffers (they have been grown: render it again).
vr_status group_frame(vr_group* g, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H, float* rgb,
                      bool* again) {
    const int n = (int)g->ranks.size();
    const uint32_t nt = vr_num_tiles(W, H);
    const uint32_t per = (nt + n - 1) / n;
    const size_t slab_floats = (size_t)per * 256 * 3;
    vr_status st;
    for (int r = 1; r < n; ++r) {  // every other rank's slab: sized for the largest share
        size_t cap = g->slab_floats;
        if ((st = grow_dev(g->devices[r], &g->slab[r], &cap, slab_floats, "hipMalloc(slab)")) != VR_OK) return st;
    }
    g->slab_floats = std::max(g->slab_floats, slab_floats);
    if (n > 1 && (st = grow_dev(g->devices[0], &g->d_recv, &g->recv_floats, slab_floats * (n - 1), "hipMalloc(gathered slabs)")) != VR_OK)
        return st;
    if ((st = grow_dev(g->devices[0], &g->d_frame, &g->frame_floats, (size_t)W * H * 3, "hipMalloc(frame)")) != VR_OK) return st;
    // 1) every rank renders its interleaved share (asynchronous on its own stream), each rank's ~15
    // launches issued from a host thread of its own so the ranks start together; the root's tiles land
    // in the frame itself (no copy of the root's share, no self-send)
    st = each_rank_parallel(g, [&](int r) -> vr_status {
        const uint32_t count = (uint32_t)r < nt ? (nt - 1 - (uint32_t)r) / (uint32_t)n + 1 : 0;
        if (count == 0) return VR_OK;
        return vr_render_tiles_device(g->ranks[r], cam, p, W, H, (uint32_t)r, (uint32_t)n, count, r == 0 ? 0 : 1,
                                      r == 0 ? g->d_frame : g->slab[r], g->streams[r]);
    });
    if (st != VR_OK) return st;
    // 2) gather the other ranks' slabs to the root: one group of sends / receives (the links run
    // concurrently; each rank's send starts as soon as its own render is done)
    if (n > 1 && g->use_rccl) {
        ncclResult_t e = g->rccl.group_start();
        if (e != ncclSuccess) return ncclf(g, e, "ncclGroupStart");
        for (int r = 1; r < n; ++r) {
            GHIP(hipSetDevice(g->devices[r]), "hipSetDevice");
            e = g->rccl.send(g->slab[r], slab_floats, ncclFloat32, 0, g->comms[r], g->streams[r]);
            if (e != ncclSuccess) break;
        }
        if (e == ncclSuccess) {
            GHIP(hipSetDevice(g->devices[0]), "hipSetDevice");
            for (int r = 1; r < n && e == ncclSuccess; ++r)
                e = g->rccl.recv(g->d_recv + (size_t)(r - 1) * slab_floats, slab_floats, ncclFloat32, r, g->comms[0],
                                 g->streams[0]);
        }
        ncclResult_t e2 = g->rccl.group_end();
        if (e != ncclSuccess) return ncclf(g, e, "ncclSend/ncclRecv");
        if (e2 != ncclSuccess) return ncclf(g, e2, "ncclGroupEnd");
    } else if (n > 1) {  // ranks sharing a GPU: device copies once every share is done
        for (int r = 1; r < n; ++r) {
            GHIP(hipSetDevice(g->devices[r]), "hipSetDevice");
            GHIP(hipStreamSynchronize(g->streams[r]), "rank render");
        }
        GHIP(hipSetDevice(g->devices[0]), "hipSetDevice");
        for (int r = 1; r < n; ++r)
            GHIP(hipMemcpyPeerAsync(g->d_recv + (size_t)(r - 1) * slab_floats, g->devices[0], g->slab[r], g->devices[r],
                                    slab_floats * sizeof(float), g->streams[0]),
                 "hipMemcpyPeerAsync(slab)");
    }
    // 3) unshuffle the gathered slabs (ranks 1 .. n-1) into the frame on the root and copy it out
    GHIP(hipSetDevice(g->devices[0]), "hipSetDevice");
    if (n > 1)
        GHIP(launch_unshuffle_part(g->d_recv, 1, (uint32_t)(n - 1), (uint32_t)n, per, (W + kTile - 1) / kTile, W, H, g->d_frame,
                                   g->streams[0]),
             "unshuffle");
    GHIP(hipMemcpyAsync(rgb, g->d_frame, (size_t)W * H * 3 * sizeof(float), hipMemcpyDeviceToHost, g->streams[0]),
         "hipMemcpyAsync(frame)");
    for (int r = 0; r < n; ++r) {
        GHIP(hipSetDevice(g->devices[r]), "hipSetDevice");
        GHIP(hipStreamSynchronize(g->streams[r]), "frame");
    }
    // 4) every rank's outcome (vr_synchronize: capacity reports, per-ray capacity errors)
    *again = false;
    for (int r = 0; r < n; ++r) {
        st = vr_synchronize(g->ranks[r]);
        if (st == VR_OK) continue;
        if (st == VR_ERR_RETRY) {
            *again = true;
            continue;
        }
        return fail(st, "rank " + std::to_string(r) + ": " + vr_last_error());
    }
    return VR_OK;
}

}  // namespace

namespace vr {

vr_status group_create(int ndev, const int* devices, vr_group** out) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(VR_ERR_HIP, "vr_init_multi: no HIP device available");
    if (ndev < 1 || ndev > 64) return fail(VR_ERR_INVALID, "vr_init_multi: ndev must be in [1, 64]");
    auto* g = new vr_group();
    for (int r = 0; r < ndev; ++r) {
        const int d = devices ? devices[r] : r;
        if (d < 0 || d >= count) {
            delete g;
            return fail(VR_ERR_INVALID, "vr_init_multi: device " + std::to_string(d) + " out of range");
        }
        g->devices.push_back(d);
    }
    g->use_rccl = std::set<int>(g->devices.begin(), g->devices.end()).size() == g->devices.size();
    g->ranks.assign(ndev, nullptr);
    g->streams.assign(ndev, nullptr);
    g->slab.assign(ndev, nullptr);
    auto bail = [&](vr_status st) {
        std::string m = vr_last_error();
        group_destroy(g);
        return fail(st, m);
    };
    for (int r = 0; r < ndev; ++r) {
        vr_status st = vr_init(g->devices[r], &g->ranks[r]);
        if (st != VR_OK) return bail(st);
        if (hipSetDevice(g->devices[r]) != hipSuccess || hipStreamCreateWithFlags(&g->streams[r], hipStreamNonBlocking) != hipSuccess) {
            fail(VR_ERR_HIP, "vr_init_multi: stream creation failed");
            return bail(VR_ERR_HIP);
        }
    }
    if (g->use_rccl) {
        std::string e = g->rccl.load();
        if (!e.empty()) {
            fail(VR_ERR_UNSUPPORTED, "vr_init_multi: " + e);
            return bail(VR_ERR_UNSUPPORTED);
        }
        g->comms.assign(ndev, nullptr);
        ncclResult_t r = g->rccl.init_all(g->comms.data(), ndev, g->devices.data());
        if (r != ncclSuccess) {
            ncclf(g, r, "vr_init_multi: ncclCommInitAll");
            g->comms.clear();
            return bail(VR_ERR_HIP);
        }
    }
    *out = g;
    return VR_OK;
}

void group_destroy(vr_group* g) {
    if (!g) return;
    for (size_t r = 0; r < g->ranks.size(); ++r) {
        if (g->ranks[r]) {
            (void)hipSetDevice(g->devices[r]);
            (void)hipDeviceSynchronize();
        }
    }
    for (ncclComm_t c : g->comms)
        if (c && g->rccl.destroy) g->rccl.destroy(c);
    for (size_t r = 0; r < g->ranks.size(); ++r) {
        (void)hipSetDevice(g->devices[r]);
        if (g->slab[r]) (void)hipFree(g->slab[r]);
        if (g->streams[r]) (void)hipStreamDestroy(g->streams[r]);
        if (g->ranks[r]) vr_destroy(g->ranks[r]);
    }
    if (!g->devices.empty()) {
        (void)hipSetDevice(g->devices[0]);
        if (g->d_recv) (void)hipFree(g->d_recv);
        if (g->d_frame) (void)hipFree(g->d_frame);
    }
    // the RCCL library stays loaded: its runtime may hold threads and device state until exit
    delete g;
}

int group_size(const vr_group* g) { return g ? (int)g->ranks.size() : 0; }
vr_ctx* group_rank(vr_group* g, int r) { return (g && r >= 0 && r < (int)g->ranks.size()) ? g->ranks[r] : nullptr; }

vr_status group_upload(vr_group* g, const vr_scene* s) {
    return each_rank_parallel(g, [&](int r) { return vr_upload_scene(g->ranks[r], s); });
}

vr_status group_render(vr_group* g, const vr_camera* cam, const vr_render_params* p, uint32_t W, uint32_t H, float* rgb) {
    if (!cam || !p || !rgb) return fail(VR_ERR_INVALID, "vr_render: NULL argument");
    if (W == 0 || H == 0 || W > 65535 || H > 65535) return fail(VR_ERR_INVALID, "width/height must be in [1, 65535]");
    for (int attempt = 1;; ++attempt) {  // the same schedule as one context's render_sync (kFrameAttempts)
        bool again = false;
        vr_status st = group_frame(g, cam, p, W, H, rgb, &again);
        if (st != VR_OK) return st;
        if (!again) return VR_OK;
        if (attempt >= kFrameAttempts)
            return fail(VR_ERR_OVERFLOW, "scatter-record / shadow-ray queue capacity could not be sized");
    }
}

vr_status group_set_option(vr_group* g, int32_t option, int64_t value) {
    for (vr_ctx* c : g->ranks) {
        vr_status st = vr_set_option(c, option, value);
        if (st != VR_OK) return st;
    }
    return VR_OK;
}

vr_status group_synchronize(vr_group* g) {
    vr_status first = VR_OK;  // every rank is synchronised (and its sticky frame outcome cleared); the first failure is returned
    std::string msg;
    for (vr_ctx* c : g->ranks) {
        vr_status st = vr_synchronize(c);
        if (first == VR_OK && st != VR_OK) {
            first = st;
            msg = vr_last_error();
        }
    }
    return first == VR_OK ? VR_OK : fail(first, msg);
}

// Whole-group statistics of the last frame: counts summed over ranks, times the slowest rank's.
vr_status group_stats(vr_group* g, vr_render_stats* o) {
    std::memset(o, 0, sizeof(*o));
    for (vr_ctx* c : g->ranks) {
        vr_render_stats s{};
        vr_status st = vr_get_stats(c, &s);
        if (st != VR_OK) return st;
        o->kernel_ms = std::max(o->kernel_ms, s.kernel_ms);
        for (size_t i = 0; i < std::size(o->stage_ms); ++i) o->stage_ms[i] = std::max(o->stage_ms[i], s.stage_ms[i]);
        o->pixels += s.pixels;
        o->fallback_pixels += s.fallback_pixels;
        o->error_pixels += s.error_pixels;
        o->scatter_records += s.scatter_records;
        o->secondary_rays += s.secondary_rays;
        o->record_overflow |= s.record_overflow;
        o->deep_pixels += s.deep_pixels;
        o->slow_rays += s.slow_rays;
        o->band_rays += s.band_rays;
    }
    return VR_OK;
}

bool group_uses_rccl(const vr_group* g) { return g && g->use_rccl; }

}  // namespace vr
