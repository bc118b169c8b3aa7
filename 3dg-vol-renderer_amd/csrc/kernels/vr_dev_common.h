// Device helpers shared by the kernel translation units: output addressing, tile mapping, the
// active-set list, and the work counters of the instrumented build.
#pragma once
#include "../../../include/vr_hip.h"
#include "vr_march.h"

namespace vr {
namespace dev {

constexpr float kInv4Pi = (float)(1.0 / (4.0 * 3.14159265358979323846));  // Vector3f * double -> float
constexpr float k4Pi = (float)(4.0 * 3.14159265358979323846);
constexpr float kTPad = 1e-5f;

enum { kOK = 0, kOverflow = 1, kError = 2 };

// Sorted list of Gaussian (leaf-order) ids with a 64-bit bloom mask for membership tests.
// Element i lives at act[i * stride] (LDS with a per-thread stride, or a global array, stride 1).
struct ActList {
    int* act;
    int stride;
    int n;
    uint64_t bloom;
    __device__ __forceinline__ int get(int i) const { return act[i * stride]; }
    __device__ __forceinline__ void set(int i, int v) { act[i * stride] = v; }
    __device__ __forceinline__ void rebuild_bloom() {
        bloom = 0;
        for (int i = 0; i < n; ++i) bloom |= 1ull << (get(i) & 63);
    }
    __device__ __forceinline__ int find(int j) const {
        if (!((bloom >> (j & 63)) & 1ull)) return -1;
        for (int i = 0; i < n; ++i)
            if (get(i) == j) return i;
        return -1;
    }
};

// Work counters of the instrumented (S = true) kernels; with S = false every update vanishes.
enum { kCtrNodes = 0, kCtrPrims, kCtrOD, kCtrMu, kCtrSecRays, kCtrSteps, kCtrPrimQueries, kCtrPixels, kNumCtr };
struct Ctr {
    uint32_t v[kNumCtr];
};
template <bool S>
struct NodeCount {
    Ctr* c;
    __device__ __forceinline__ void operator()() const {
        if constexpr (S) c->v[kCtrNodes]++;
    }
};
// Wave-reduce and add to the global 64-bit totals. Every lane of the wave must call it.
__device__ __forceinline__ void flush_counters(unsigned long long* work, const Ctr& c) {
    for (int i = 0; i < kNumCtr; ++i) {
        unsigned long long v = c.v[i];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(work + i, v);
    }
}

// ---- output addressing ----
__device__ __forceinline__ void store_px(const RenderArgs& A, uint32_t tile_local, int lx, int ly, int x, int y, float r,
                                         float g, float b) {
    if (A.packed) {
        size_t o = ((size_t)tile_local * 256u + (size_t)(ly * kTile + lx)) * 3u;
        A.out[o] = r;
        A.out[o + 1] = g;
        A.out[o + 2] = b;
    } else if (x < (int)A.width && y < (int)A.height) {
        size_t o = ((size_t)y * A.width + (size_t)x) * 3u;
        A.out[o] = r;
        A.out[o + 1] = g;
        A.out[o + 2] = b;
    }
}

// lane l of a 256-thread tile workgroup: wave w covers the 8x8 quadrant (w & 1, w >> 1)
__device__ __forceinline__ void tile_pixel(const RenderArgs& A, uint32_t tile_local, int lane_id, int& lx, int& ly, int& x,
                                           int& y) {
    int wv = lane_id >> 6, ln = lane_id & 63;
    lx = (wv & 1) * 8 + (ln & 7);
    ly = (wv >> 1) * 8 + (ln >> 3);
    uint32_t tile = A.first_tile + tile_local * A.tile_stride;
    x = (int)((tile % A.tiles_x) * kTile) + lx;
    y = (int)((tile / A.tiles_x) * kTile) + ly;
}

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so give each XCD a
// contiguous run of tiles (neighbouring tiles share BVH paths and records in that XCD's L2).
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    if (nb % 8u != 0u) return b;
    return (b % 8u) * (nb / 8u) + b / 8u;
}

}  // namespace dev
}  // namespace vr
