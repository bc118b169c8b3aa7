// Device BVH builder interface (kernels/vr_lbvh.hip), shared by its definition and its caller
// (host/vr_device.cpp) so the result layout has exactly one definition.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>

#include "vr_internal.h"

namespace vr {

struct LbvhResult {
    GaussianRecord* gauss = nullptr;  // records in leaf order
    uint32_t* order = nullptr;        // leaf-order index -> scene index
    BVHNode* nodes = nullptr;         // N - 1 child-pair nodes (root 0)
    HNode* hnodes = nullptr;          // same tree at half precision (if requested)
    HNode4* hnodes4 = nullptr;        // 4-wide tree (if requested)
    size_t num_nodes = 0, num_nodes4 = 0;
    int max_depth = 0;                // as BVHBuild::max_depth: root = 1, a leaf child counts as a level
};

// d_rec: records in scene order, d_boxes: 6 floats per primitive (both device, n >= 2 primitives).
// cmin/cmax: centroid bounds; half: build the half-precision trees with normalisation (hc, hs).
// hipErrorNotSupported: the tree is deeper than the traversal stacks allow.
hipError_t lbvh_build(const GaussianRecord* d_rec, const float* d_boxes, uint32_t n, const float cmin[3], const float cmax[3],
                      bool half, const float hc[3], float hs, hipStream_t s, LbvhResult& R);

}  // namespace vr
