// Device BVH build (the reference rebuilds its midpoint-split BVH on the host at
// every parameter update, gmm.h:231-446 via apply_params_to_gmm_local, gmm.h:673).
//
// A linear BVH in the Karras (2012) formulation, written for the layouts the traversal kernels read:
//   1. morton_kernel: 63-bit Morton code (21 bits per axis) of every box centroid in the centroid
//      bounds; hipcub radix sort of (code, index) pairs -> primitive order;
//   2. karras_kernel: internal node i of the binary radix tree over the sorted codes (ties broken by
//      index) -> its range [first, last], split and children; parents recorded;
//   3. depth_kernel: node depth by walking parent links (and the tree's maximum depth);
//   4. box_kernel, one launch per depth, deepest first: the boxes of every *reachable* node (range
//      larger than kLeafMax: smaller ranges are leaves of <= kLeafMax contiguous primitives, as the
//      host builder's); a child's box is its range's primitive boxes (leaf) or its node box;
//   5. emit_kernel: the child-pair BVHNode of every reachable node (index = Karras index, root 0),
//      its outward-rounded half-precision copy (HNode), and the 4-wide HNode4 of every reachable node
//      at even depth (its grandchildren, compacted by a scan) — the same three trees the host
//      builder uploads, so every traversal kernel runs unchanged.
// The event set a ray collects does not depend on the tree (boxes are conservative), so renders are
// identical up to summation order whichever builder made it.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>

#include "../vr_internal.h"
#include "../vr_lbvh.h"

namespace vr {
namespace lbvh {

constexpr uint32_t kNone = 0xffffffffu;

__device__ __forceinline__ uint64_t spread21(uint64_t v) {  // 21 bits -> every third bit of 63
    v &= 0x1fffffull;
    v = (v | v << 32) & 0x1f00000000ffffull;
    v = (v | v << 16) & 0x1f0000ff0000ffull;
    v = (v | v << 8) & 0x100f00f00f00f00full;
    v = (v | v << 4) & 0x10c30c30c30c30c3ull;
    v = (v | v << 2) & 0x1249249249249249ull;
    return v;
}

__global__ void morton_kernel(const float* __restrict__ boxes, uint32_t n, float3 lo, float3 inv_ext, uint64_t* keys,
                              uint32_t* vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* b = boxes + 6 * (size_t)i;
    const float c[3] = {0.5f * (b[0] + b[3]), 0.5f * (b[1] + b[4]), 0.5f * (b[2] + b[5])};
    const float l[3] = {lo.x, lo.y, lo.z}, s[3] = {inv_ext.x, inv_ext.y, inv_ext.z};
    uint64_t q[3];
    for (int k = 0; k < 3; ++k) {
        float u = (c[k] - l[k]) * s[k];
        u = fminf(fmaxf(u, 0.0f), 1.0f);
        q[k] = (uint64_t)fminf(u * 2097152.0f, 2097151.0f);
    }
    keys[i] = spread21(q[0]) << 2 | spread21(q[1]) << 1 | spread21(q[2]);
    vals[i] = i;
}

__device__ __forceinline__ int delta(const uint64_t* __restrict__ k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint64_t a = k[i], b = k[j];
    if (a == b) return 64 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clzll((long long)(a ^ b));
}

struct Tree {
    uint32_t* first;   // per internal node: range [first, last] of sorted primitives
    uint32_t* last;
    uint32_t* split;   // left child covers [first, split], right [split + 1, last]
    uint32_t* parent;  // per internal node (root: kNone)
    uint32_t* depth;   // per internal node (root 0)
    float* box;        // per internal node: min xyz, max xyz (reachable nodes only)
    uint32_t* map4;    // per internal node: exclusive count of reachable even-depth nodes before it
    uint32_t* maxdepth;
};

__global__ void karras_kernel(const uint64_t* __restrict__ keys, int n, Tree T) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(keys, n, i, i - d);
    int lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(keys, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) / 2;
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + min(d, 0);
    const int first = min(i, j), last = max(i, j);
    T.first[i] = (uint32_t)first;
    T.last[i] = (uint32_t)last;
    T.split[i] = (uint32_t)gamma;
    if (first != gamma) T.parent[gamma] = (uint32_t)i;          // left child is internal node gamma
    if (last != gamma + 1) T.parent[gamma + 1] = (uint32_t)i;   // right child is internal node gamma + 1
    if (i == 0) T.parent[0] = kNone;
}

__device__ __forceinline__ bool reachable(const Tree& T, uint32_t i) {
    return i == 0 || T.last[i] - T.first[i] + 1u > (uint32_t)kLeafMax;
}

__global__ void depth_kernel(int n, Tree T) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint32_t)(n - 1)) return;
    uint32_t d = 0;
    for (uint32_t p = T.parent[i]; p != kNone && d < 4096u; p = T.parent[p]) ++d;
    T.depth[i] = d;
    if (reachable(T, i)) atomicMax(T.maxdepth, d);
}

__device__ __forceinline__ void range_box(const float* __restrict__ sb, uint32_t a, uint32_t b, float* out) {
    for (int k = 0; k < 3; ++k) {
        out[k] = INFINITY;
        out[3 + k] = -INFINITY;
    }
    for (uint32_t j = a; j <= b; ++j)
        for (int k = 0; k < 3; ++k) {
            out[k] = fminf(out[k], sb[6 * (size_t)j + k]);
            out[3 + k] = fmaxf(out[3 + k], sb[6 * (size_t)j + 3 + k]);
        }
}

// Box of child `side` of node i: its range's primitives (leaf) or its own node box (computed at the
// deeper level already).
__device__ __forceinline__ void child_box(const Tree& T, const float* __restrict__ sb, uint32_t i, int side, float* out) {
    const uint32_t a = side == 0 ? T.first[i] : T.split[i] + 1u;
    const uint32_t b = side == 0 ? T.split[i] : T.last[i];
    const uint32_t node = side == 0 ? T.split[i] : T.split[i] + 1u;
    if (b - a + 1u <= (uint32_t)kLeafMax) {
        range_box(sb, a, b, out);
    } else {
        for (int k = 0; k < 6; ++k) out[k] = T.box[6 * (size_t)node + k];
    }
}

__global__ void box_kernel(int n, uint32_t level, const float* __restrict__ sb, Tree T) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint32_t)(n - 1) || T.depth[i] != level || !reachable(T, i)) return;
    float l[6], r[6];
    child_box(T, sb, i, 0, l);
    child_box(T, sb, i, 1, r);
    for (int k = 0; k < 3; ++k) {
        T.box[6 * (size_t)i + k] = fminf(l[k], r[k]);
        T.box[6 * (size_t)i + 3 + k] = fmaxf(l[3 + k], r[3 + k]);
    }
}

__global__ void flag4_kernel(int n, const Tree T, uint32_t* flags) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint32_t)(n - 1)) return;
    flags[i] = (reachable(T, i) && (T.depth[i] & 1u) == 0u) ? 1u : 0u;
}

// half-precision conversion with outward rounding (as the host's f16_directed, vr_device.cpp)
__device__ __forceinline__ uint16_t f16_bits(_Float16 h) { return __builtin_bit_cast(uint16_t, h); }
__device__ __forceinline__ double f16_val(uint16_t b) { return (double)__builtin_bit_cast(_Float16, b); }
__device__ __forceinline__ uint16_t f16_step(uint16_t h, bool up) {
    const bool neg = h & 0x8000u;
    if ((h & 0x7fffu) == 0) return up ? 0x0001u : 0x8001u;
    return (uint16_t)((neg != up) ? h + 1 : h - 1);
}
__device__ __forceinline__ uint16_t f16_directed(double v, bool up) {
    if (isinf(v)) return v > 0 ? 0x7c00u : 0xfc00u;
    uint16_t h = f16_bits((_Float16)(float)v);
    if (up) {
        while (f16_val(h) < v) h = f16_step(h, true);
    } else {
        while (f16_val(h) > v) h = f16_step(h, false);
    }
    return h;
}

struct Emit {
    BVHNode* nodes;
    HNode* hnodes;    // nullptr: f32 nodes only
    HNode4* hnodes4;  // nullptr: f32 nodes only
    float3 hc;        // half-node normalisation: u = (x - hc) * hs, in double
    double hs;
};

__device__ __forceinline__ int32_t child_ref(const Tree& T, uint32_t i, int side) {
    const uint32_t a = side == 0 ? T.first[i] : T.split[i] + 1u;
    const uint32_t b = side == 0 ? T.split[i] : T.last[i];
    if (b - a + 1u <= (uint32_t)kLeafMax) return make_leaf(a, b - a + 1u);
    return (int32_t)(side == 0 ? T.split[i] : T.split[i] + 1u);
}

__global__ void emit_kernel(int n, const float* __restrict__ sb, Tree T, Emit E) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint32_t)(n - 1)) return;
    BVHNode nd;
    HNode hn;
    if (!reachable(T, i)) {  // never referenced: an empty node keeps the array well-formed
        for (int k = 0; k < 12; ++k) nd.f[k] = (k % 6) < 3 ? INFINITY : -INFINITY;
        nd.c[0] = nd.c[1] = nd.c[2] = nd.c[3] = 0;
        E.nodes[i] = nd;
        if (E.hnodes) {
            for (int k = 0; k < 12; ++k) hn.h[k] = (k % 6) < 3 ? 0x7c00u : 0xfc00u;
            hn.c[0] = hn.c[1] = 0;
            E.hnodes[i] = hn;
        }
        return;
    }
    for (int side = 0; side < 2; ++side) {
        float b[6];
        child_box(T, sb, i, side, b);
        for (int k = 0; k < 6; ++k) nd.f[6 * side + k] = b[k];
        nd.c[side] = child_ref(T, i, side);
        if (E.hnodes) {
            const double c3[3] = {(double)E.hc.x, (double)E.hc.y, (double)E.hc.z};
            for (int k = 0; k < 3; ++k) {
                const double ulo = isinf(b[k]) ? (double)b[k] : ((double)b[k] - c3[k]) * E.hs;
                const double uhi = isinf(b[3 + k]) ? (double)b[3 + k] : ((double)b[3 + k] - c3[k]) * E.hs;
                hn.h[6 * side + k] = f16_directed(ulo, false);
                hn.h[6 * side + 3 + k] = f16_directed(uhi, true);
            }
            hn.c[side] = nd.c[side];
        }
    }
    nd.c[2] = nd.c[3] = 0;
    E.nodes[i] = nd;
    if (E.hnodes) E.hnodes[i] = hn;
}

// 4-wide nodes: every reachable node at even depth holds its children's children (a leaf child
// stays one slot). Reads the half nodes written by emit_kernel (previous launch).
__global__ void emit4_kernel(int n, Tree T, Emit E) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint32_t)(n - 1) || !reachable(T, i) || (T.depth[i] & 1u)) return;
    HNode4 w;
    int m = 0;
    const HNode& p = E.hnodes[i];
    for (int side = 0; side < 2; ++side) {
        const int32_t ref = p.c[side];
        if (ref < 0) {
            for (int k = 0; k < 6; ++k) w.h[m][k] = p.h[6 * side + k];
            w.c[m++] = ref;
        } else {
            const HNode& q = E.hnodes[ref];
            for (int s2 = 0; s2 < 2; ++s2) {
                for (int k = 0; k < 6; ++k) w.h[m][k] = q.h[6 * s2 + k];
                w.c[m++] = q.c[s2] < 0 ? q.c[s2] : (int32_t)T.map4[q.c[s2]];
            }
        }
    }
    for (; m < 4; ++m) {
        for (int k = 0; k < 6; ++k) w.h[m][k] = 0x7e00u;  // NaN box: no slab test reports a hit
        w.c[m] = 0;
    }
    E.hnodes4[T.map4[i]] = w;
}

__global__ void gather_records_kernel(const GaussianRecord* __restrict__ src, const float* __restrict__ boxes,
                                      const uint32_t* __restrict__ perm, uint32_t n, GaussianRecord* dst, float* sboxes) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t p = perm[j];
    dst[j] = src[p];
    for (int k = 0; k < 6; ++k) sboxes[6 * (size_t)j + k] = boxes[6 * (size_t)p + k];
}

}  // namespace lbvh

// lbvh_build (vr_lbvh.h): all device pointers of the result are owned by the caller afterwards.
hipError_t lbvh_build(const GaussianRecord* d_rec, const float* d_boxes, uint32_t n, const float cmin[3],
                      const float cmax[3], bool half, const float hc[3], float hs, hipStream_t s, LbvhResult& R) {
    using namespace lbvh;
    hipError_t e = hipSuccess;
    const int N = (int)n;
    const unsigned nb = (n + 255) / 256;
    uint64_t *keys = nullptr, *keys2 = nullptr;
    uint32_t *vals = nullptr, *flags = nullptr;
    float* sboxes = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0, scan_bytes = 0;
    Tree T{};
    uint32_t h_max = 0, h_count4 = 0, h_last_flag = 0;
    auto ck = [&](hipError_t x) {
        if (e == hipSuccess && x != hipSuccess) e = x;
        return e == hipSuccess;
    };
    float3 lo = make_float3(cmin[0], cmin[1], cmin[2]);
    float3 ie;
    {
        float ex[3];
        for (int k = 0; k < 3; ++k) ex[k] = cmax[k] - cmin[k];
        ie = make_float3(ex[0] > 0 ? 1.0f / ex[0] : 0.0f, ex[1] > 0 ? 1.0f / ex[1] : 0.0f, ex[2] > 0 ? 1.0f / ex[2] : 0.0f);
    }
    ck(hipMalloc(&keys, n * 8ull)) && ck(hipMalloc(&keys2, n * 8ull)) && ck(hipMalloc(&vals, n * 4ull)) &&
        ck(hipMalloc(&R.order, n * 4ull)) && ck(hipMalloc(&R.gauss, n * sizeof(GaussianRecord))) &&
        ck(hipMalloc(&sboxes, n * 24ull)) && ck(hipMalloc(&T.first, n * 4ull)) && ck(hipMalloc(&T.last, n * 4ull)) &&
        ck(hipMalloc(&T.split, n * 4ull)) && ck(hipMalloc(&T.parent, n * 4ull)) && ck(hipMalloc(&T.depth, n * 4ull)) &&
        ck(hipMalloc(&T.box, n * 24ull)) && ck(hipMalloc(&T.map4, n * 4ull)) && ck(hipMalloc(&flags, n * 4ull)) &&
        ck(hipMalloc(&T.maxdepth, 4)) && ck(hipMalloc(&R.nodes, (n - 1) * sizeof(BVHNode)));
    if (e == hipSuccess && half) ck(hipMalloc(&R.hnodes, (n - 1) * sizeof(HNode)));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(morton_kernel, dim3(nb), dim3(256), 0, s, d_boxes, n, lo, ie, keys, vals);
        ck(hipGetLastError());
    }
    if (e == hipSuccess) ck(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys2, vals, R.order, N, 0, 63, s));
    if (e == hipSuccess) ck(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, flags, T.map4, N - 1, s));
    if (e == hipSuccess) ck(hipMalloc(&tmp, std::max(tmp_bytes, scan_bytes)));
    if (e == hipSuccess) ck(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys2, vals, R.order, N, 0, 63, s));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(gather_records_kernel, dim3(nb), dim3(256), 0, s, d_rec, d_boxes, R.order, n, R.gauss, sboxes);
        ck(hipGetLastError());
    }
    if (e == hipSuccess) ck(hipMemsetAsync(T.maxdepth, 0, 4, s));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(karras_kernel, dim3(nb), dim3(256), 0, s, keys2, N, T);
        ck(hipGetLastError());
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(depth_kernel, dim3(nb), dim3(256), 0, s, N, T);
        ck(hipGetLastError());
    }
    if (e == hipSuccess) ck(hipMemcpyAsync(&h_max, T.maxdepth, 4, hipMemcpyDeviceToHost, s));
    if (e == hipSuccess) ck(hipStreamSynchronize(s));
    if (e == hipSuccess && h_max + 2 > (uint32_t)kMaxDepth + 1) e = hipErrorNotSupported;  // too deep: host build
    for (int lv = (int)h_max; e == hipSuccess && lv >= 0; --lv) {
        hipLaunchKernelGGL(box_kernel, dim3(nb), dim3(256), 0, s, N, (uint32_t)lv, sboxes, T);
        ck(hipGetLastError());
    }
    Emit E{R.nodes, R.hnodes, nullptr, make_float3(hc[0], hc[1], hc[2]), (double)hs};
    if (e == hipSuccess) {
        hipLaunchKernelGGL(emit_kernel, dim3(nb), dim3(256), 0, s, N, sboxes, T, E);
        ck(hipGetLastError());
    }
    if (e == hipSuccess && half) {
        hipLaunchKernelGGL(flag4_kernel, dim3(nb), dim3(256), 0, s, N, T, flags);
        ck(hipGetLastError());
        if (e == hipSuccess) ck(hipcub::DeviceScan::ExclusiveSum(tmp, scan_bytes, flags, T.map4, N - 1, s));
        if (e == hipSuccess) ck(hipMemcpyAsync(&h_count4, T.map4 + (N - 2), 4, hipMemcpyDeviceToHost, s));
        if (e == hipSuccess) ck(hipMemcpyAsync(&h_last_flag, flags + (N - 2), 4, hipMemcpyDeviceToHost, s));
        if (e == hipSuccess) ck(hipStreamSynchronize(s));
        const uint32_t n4 = h_count4 + h_last_flag;
        if (e == hipSuccess) ck(hipMalloc(&R.hnodes4, std::max<uint32_t>(n4, 1) * sizeof(HNode4)));
        E.hnodes4 = R.hnodes4;
        if (e == hipSuccess) {
            hipLaunchKernelGGL(emit4_kernel, dim3(nb), dim3(256), 0, s, N, T, E);
            ck(hipGetLastError());
        }
        R.num_nodes4 = n4;
    }
    if (e == hipSuccess) ck(hipStreamSynchronize(s));
    for (void* p : {(void*)keys, (void*)keys2, (void*)vals, (void*)flags, (void*)sboxes, tmp, (void*)T.first, (void*)T.last,
                    (void*)T.split, (void*)T.parent, (void*)T.depth, (void*)T.box, (void*)T.map4, (void*)T.maxdepth})
        if (p) (void)hipFree(p);
    R.num_nodes = n - 1;
    R.max_depth = (int)h_max + 2;
    if (e != hipSuccess) {
        for (void* p : {(void*)R.gauss, (void*)R.order, (void*)R.nodes, (void*)R.hnodes, (void*)R.hnodes4})
            if (p) (void)hipFree(p);
        R = LbvhResult{};
    }
    return e;
}

}  // namespace vr
