// Host BVH builder for the device traversal kernels.
//
// The reference builds a midpoint-split binary BVH with leaves of <= 4 Gaussians
// (gmm.h:231-446; SAH compiled out at gmm.h:162) and traverses it with a per-thread std::vector
// stack. Only the *event set* a ray collects matters to the integrators, and that set does not
// depend on the tree (boxes are conservative), so the device tree is built for GPU traversal
// instead:
//   * binned SAH (16 bins x 3 axes) on centroids, leaves <= kLeafMax primitives;
//   * depth bounded by kMaxDepth (median splits take over when the remaining count could not
//     otherwise fit), so a fixed kStackSize LDS stack can never overflow;
//   * child-pair node layout (vr_internal.h): 64 B per node holding BOTH children's boxes, nodes
//     numbered in depth-first pre-order (left subtree adjacent to its parent);
//   * primitives reordered so every leaf is a contiguous run of 48-B records.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>

#include "vr_common.h"

namespace vr {

namespace {

struct Box {
    float mn[3] = {INFINITY, INFINITY, INFINITY};
    float mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const float* b) {
        for (int k = 0; k < 3; ++k) {
            mn[k] = std::min(mn[k], b[k]);
            mx[k] = std::max(mx[k], b[3 + k]);
        }
    }
    void grow(const Box& o) {
        for (int k = 0; k < 3; ++k) {
            mn[k] = std::min(mn[k], o.mn[k]);
            mx[k] = std::max(mx[k], o.mx[k]);
        }
    }
    float area() const {
        float d0 = mx[0] - mn[0], d1 = mx[1] - mn[1], d2 = mx[2] - mn[2];
        if (!(d0 >= 0.0f) || !(d1 >= 0.0f) || !(d2 >= 0.0f)) return 0.0f;
        return 2.0f * (d0 * d1 + d0 * d2 + d1 * d2);
    }
};

struct TNode {
    Box box;
    int32_t left = -1, right = -1;  // tmp children (internal)
    uint32_t first = 0, count = 0;  // leaf range when left < 0
};

int ceil_log2(uint64_t x) {
    int r = 0;
    while ((1ull << r) < x) ++r;
    return r;
}

}  // namespace

BVHBuild build_bvh(const std::vector<float>& boxes) {
    const uint32_t N = (uint32_t)(boxes.size() / 6);
    BVHBuild out;
    out.order.resize(N);
    for (uint32_t i = 0; i < N; ++i) out.order[i] = i;
    std::vector<float> cen(3 * (size_t)N);
    for (uint32_t i = 0; i < N; ++i)
        for (int k = 0; k < 3; ++k) cen[3 * i + k] = 0.5f * (boxes[6 * i + k] + boxes[6 * i + 3 + k]);

    std::vector<TNode> t;
    t.reserve(N ? 2 * (N / kLeafMax + 1) : 1);
    struct Work { int32_t node; int depth; };
    std::vector<Work> work;
    if (N > 0) {
        TNode root;
        root.first = 0;
        root.count = N;
        for (uint32_t i = 0; i < N; ++i) root.box.grow(&boxes[6 * i]);
        t.push_back(root);
        work.push_back({0, 1});
    }
    uint32_t* ord = out.order.data();
#ifndef VR_BVH_BINS
#define VR_BVH_BINS 16
#endif
    constexpr int kBins = VR_BVH_BINS;   // SAH bins per axis (<= 64)
    constexpr uint32_t leaf_max = kLeafMax;
    // Depth budget: SAH may go kSlack levels deeper than a perfectly balanced tree, but never past
    // kMaxDepth. Shallow trees let the march kernel use a 24-entry LDS stack (more waves per CU);
    // very large scenes fall back to the 32-entry stack.
    constexpr int kSlack = 6;
    const int depth_cap = std::min(kMaxDepth, std::max(kShallowDepth, ceil_log2((N + leaf_max - 1) / leaf_max + 1) + kSlack));
    while (!work.empty()) {
        Work w = work.back();
        work.pop_back();
        const uint32_t first = t[w.node].first, count = t[w.node].count;
        out.max_depth = std::max(out.max_depth, w.depth);
        if (count <= leaf_max) continue;
        Box cb;
        for (uint32_t j = first; j < first + count; ++j) {
            const float* c = &cen[3 * ord[j]];
            float b6[6] = {c[0], c[1], c[2], c[0], c[1], c[2]};
            cb.grow(b6);
        }
        int axis = 0;
        float ext[3];
        for (int k = 0; k < 3; ++k) ext[k] = cb.mx[k] - cb.mn[k];
        if (ext[1] > ext[axis]) axis = 1;
        if (ext[2] > ext[axis]) axis = 2;
        uint32_t mid = 0;
        const bool balanced = w.depth + ceil_log2((count + leaf_max - 1) / leaf_max) >= depth_cap - 1;
        if (!balanced && ext[axis] > 0.0f) {
            // binned SAH over all three axes
            float best_cost = INFINITY;
            int best_axis = -1, best_split = -1;
            for (int a = 0; a < 3; ++a) {
                if (!(ext[a] > 0.0f)) continue;
                Box bb[64];
                uint32_t bn[64] = {0};
                const float scale = kBins / ext[a];
                for (uint32_t j = first; j < first + count; ++j) {
                    uint32_t p = ord[j];
                    int b = (int)((cen[3 * p + a] - cb.mn[a]) * scale);
                    b = std::min(std::max(b, 0), kBins - 1);
                    bb[b].grow(&boxes[6 * p]);
                    bn[b]++;
                }
                float ra[64];
                uint32_t rn[64];
                Box acc;
                uint32_t n = 0;
                for (int b = kBins - 1; b > 0; --b) {
                    acc.grow(bb[b]);
                    n += bn[b];
                    ra[b] = acc.area();
                    rn[b] = n;
                }
                Box lacc;
                uint32_t ln = 0;
                for (int b = 0; b < kBins - 1; ++b) {
                    lacc.grow(bb[b]);
                    ln += bn[b];
                    if (ln == 0 || rn[b + 1] == 0) continue;
                    float c = lacc.area() * ln + ra[b + 1] * rn[b + 1];
                    if (c < best_cost) {
                        best_cost = c;
                        best_axis = a;
                        best_split = b;
                    }
                }
            }
            if (best_axis >= 0) {
                const float scale = kBins / ext[best_axis];
                uint32_t* beg = ord + first;
                uint32_t* it = std::partition(beg, beg + count, [&](uint32_t p) {
                    int b = (int)((cen[3 * p + best_axis] - cb.mn[best_axis]) * scale);
                    b = std::min(std::max(b, 0), kBins - 1);
                    return b <= best_split;
                });
                mid = (uint32_t)(it - beg);
            }
        }
        if (mid == 0 || mid == count) {  // median split (balanced mode or degenerate SAH)
            if (!(ext[axis] > 0.0f) && count <= 16u) continue;  // identical centroids: one leaf
            mid = count / 2;
            uint32_t* beg = ord + first;
            std::nth_element(beg, beg + mid, beg + count, [&](uint32_t a, uint32_t b) {
                return cen[3 * a + axis] < cen[3 * b + axis];
            });
        }
        TNode L, R;
        L.first = first;
        L.count = mid;
        R.first = first + mid;
        R.count = count - mid;
        for (uint32_t j = L.first; j < L.first + L.count; ++j) L.box.grow(&boxes[6 * ord[j]]);
        for (uint32_t j = R.first; j < R.first + R.count; ++j) R.box.grow(&boxes[6 * ord[j]]);
        int32_t li = (int32_t)t.size();
        t.push_back(L);
        int32_t ri = (int32_t)t.size();
        t.push_back(R);
        t[w.node].left = li;
        t[w.node].right = ri;
        work.push_back({ri, w.depth + 1});
        work.push_back({li, w.depth + 1});
    }

    // ---- emit child-pair nodes in DFS pre-order ----
    auto set_child = [&](BVHNode& pn, int side, const TNode& c, int32_t ref) {
        for (int k = 0; k < 3; ++k) {
            pn.f[6 * side + k] = c.box.mn[k];
            pn.f[6 * side + 3 + k] = c.box.mx[k];
        }
        pn.c[side] = ref;
    };
    auto set_empty = [&](BVHNode& pn, int side) {
        for (int k = 0; k < 3; ++k) {
            pn.f[6 * side + k] = INFINITY;
            pn.f[6 * side + 3 + k] = -INFINITY;
        }
        pn.c[side] = 0;
    };
    out.nodes.clear();
    if (N == 0) {
        BVHNode e{};
        set_empty(e, 0);
        set_empty(e, 1);
        out.nodes.push_back(e);
        return out;
    }
    if (t[0].left < 0) {  // whole scene is one leaf
        BVHNode e{};
        set_child(e, 0, t[0], make_leaf(t[0].first, t[0].count));
        set_empty(e, 1);
        out.nodes.push_back(e);
        return out;
    }
    std::vector<int32_t> pair_of(t.size(), -1);
    std::vector<int32_t> dfs{0};
    std::vector<int32_t> emit_order;
    while (!dfs.empty()) {
        int32_t n = dfs.back();
        dfs.pop_back();
        pair_of[n] = (int32_t)emit_order.size();
        emit_order.push_back(n);
        if (t[t[n].right].left >= 0) dfs.push_back(t[n].right);
        if (t[t[n].left].left >= 0) dfs.push_back(t[n].left);
    }
    out.nodes.resize(emit_order.size());
    for (size_t e = 0; e < emit_order.size(); ++e) {
        const TNode& n = t[emit_order[e]];
        BVHNode pn{};
        const TNode* kids[2] = {&t[n.left], &t[n.right]};
        for (int side = 0; side < 2; ++side) {
            const TNode& c = *kids[side];
            int32_t ref = c.left < 0 ? make_leaf(c.first, c.count) : pair_of[side == 0 ? n.left : n.right];
            set_child(pn, side, c, ref);
        }
        out.nodes[e] = pn;
    }
    return out;
}

}  // namespace vr
