// Internal layouts shared by the host side (scene prep, BVH build, launch) and the HIP kernels.
// Everything here is plain data: it is the HBM image of a scene.
#pragma once
#include <hip/hip_runtime_api.h>
#include <hip/hip_vector_types.h>
#include <stdint.h>

namespace vr {

// ------------------------------------------------------------------------------------------
// Gaussian record: 48 B = 3 x float4 (three 16-B loads, one 64-B sector pair when aligned).
//   r0 = { mean.x, mean.y, mean.z, density }
//   r1 = { M00, M01, M02, M11 }         M = Sigma^-1 (exactly symmetric, see vr_scene.cpp)
//   r2 = { M12, M22, norm, albedo }     norm = (2pi)^-1.5 det^-0.5   (gaussian.h:52-55)
// Stored in BVH leaf order (contiguous per leaf).
// ------------------------------------------------------------------------------------------
struct GaussianRecord {
    float mx, my, mz, density;
    float m00, m01, m02, m11;
    float m12, m22, norm, albedo;
};
static_assert(sizeof(GaussianRecord) == 48, "record must be 48 B");

// Whitened copy of a record for the secondary rays (48 B, same leaf order): M = L^T L with L upper
// triangular (Cholesky of the inverse covariance, in double), so a ray's quadratic is that of a unit
// sphere in the coordinates L (x - mean): A = |L d|^2, B/2 = L p . L d, Cq = |L p|^2. dn = density *
// norm * sqrt(pi / 2): the optical depth's prefactor density * norm * sqrt(pi / (2A)) is dn * A^-1/2.
struct WRecord {
    float mx, my, mz, dn;
    float l00, l01, l02, l11;
    float l12, l22, pad0, pad1;
};
static_assert(sizeof(WRecord) == 48, "whitened record must be 48 B");

// ------------------------------------------------------------------------------------------
// BVH node, child-pair layout, 64 B: one node fetch tests both children.
//   f[0..5]  = left  child box (min xyz, max xyz)
//   f[6..11] = right child box
//   c[0], c[1] = child refs: >= 0 internal node index; < 0 leaf:
//                 leaf = 0x80000000 | (first << 4) | (count - 1), count <= 16, first < 2^27
//   c[2], c[3] = unused (0)
// Node 0 is the root pair. An empty child has an inverted box (+inf, -inf) and ref 0 (never hit).
// ------------------------------------------------------------------------------------------
struct BVHNode {
    float f[12];
    int32_t c[4];
};
static_assert(sizeof(BVHNode) == 64, "node must be 64 B");

// The same child-pair node at half precision (secondary rays): the two children's boxes in
// scene-normalised coordinates u = (x - hn_center) * hn_scale, rounded outward to f16 (min down,
// max up), so every box still contains the f32 one. Ray parameters t are unchanged by the
// normalisation (o' + t d' = (o + t d - c) s), so the slab test is the f32 one on a wider box.
struct HNode {
    uint16_t h[12];  // [6 side + k]: min xyz, [6 side + 3 + k]: max xyz, side 0 = left
    int32_t c[2];
};
static_assert(sizeof(HNode) == 32, "half node must be 32 B");

// 4-wide half-precision node for the secondary rays: up to 4 children (boxes as in HNode, same
// normalisation and outward rounding), collapsed from the child-pair tree. c == 0: empty slot, whose
// box is NaN (no slab test reports a hit for it).
struct HNode4 {
    uint16_t h[4][6];  // child i: min xyz, max xyz
    int32_t c[4];      // > 0: HNode4 index, < 0: leaf ref, 0: empty
};
static_assert(sizeof(HNode4) == 64, "4-wide half node must be 64 B");

#ifndef VR_SEC_SOA
#define VR_SEC_SOA 1  // the secondary rays' node step reads a per-axis copy of their tree (sign-selected slabs; A/B)
#endif

#ifndef VR_LEAF_MAX
#define VR_LEAF_MAX 2  // A/B (round 3, every line): 2 beats 3 by 0.8-2.8 % (C4 +1.7 %), 1 and 4 lose
#endif
constexpr int kLeafMax = VR_LEAF_MAX;  // primitives per leaf (<= 16: leaf refs hold count - 1 in 4 bits)
constexpr int kMaxDepth = 30;        // builder guarantees node depth <= kMaxDepth
// Per-lane traversal-stack capacity of the 4-wide walk (up to 3 pushes per level; the collapsed
// tree is no deeper than the pair tree): sizes the persistent kernel's global stack overflow.
constexpr int kWideStackMax = 3 * kMaxDepth + 1;
constexpr int kStackSize = 32;       // traversal stack entries (>= kMaxDepth + 1)
constexpr int kShallowDepth = 24;    // trees this shallow use the 24-entry stack variant
constexpr int kShallowStack = 24;    // (a child-pair traversal pushes at most depth - 1 entries)
constexpr int kTile = 16;            // pixel tile edge (one 256-thread workgroup per tile)

__host__ __device__ inline bool ref_is_leaf(int32_t r) { return r < 0; }
__host__ __device__ inline uint32_t leaf_first(int32_t r) { return ((uint32_t)r & 0x7fffffffu) >> 4; }
__host__ __device__ inline uint32_t leaf_count(int32_t r) { return ((uint32_t)r & 15u) + 1u; }
__host__ __device__ inline int32_t make_leaf(uint32_t first, uint32_t count) {
    return (int32_t)(0x80000000u | (first << 4) | (count - 1u));
}

struct SphereRecord {  // 32 B
    float cx, cy, cz, radius;
    float sigma_a, sigma_s, pad0, pad1;
};

struct LightRecord {
    float px, py, pz, ix, iy, iz;
};

constexpr int kMaxLights = 16;
constexpr int kEnvOrderMax = 240;  // environment rays are direction-ordered up to this many samples (LDS bound)
constexpr uint32_t kNoRecord = 0xffffffffu;
constexpr int kActInline = 4;  // active-list slots stored with each scatter record
// Ray-march pixels whose active set outgrows the 64-slot LDS fallback: a global-memory active list of
// kActDeep slots per thread, kDeepThreads threads (march_deep_kernel), up to kDeepQueue such pixels per frame.
constexpr int kActDeep = 2048, kDeepThreads = 256, kDeepBlock = 64;
constexpr uint32_t kDeepQueue = 65536;
// march_wide_kernel: the fallback queue one pixel per lane, kActWide active-list slots per lane in global
// memory ([slot][thread] rows), kWideThreads lanes; used when the queue holds at least A.wide_min pixels.
#ifndef VR_WIDE_THREADS
#define VR_WIDE_THREADS 262144  // lanes of march_wide_kernel (4 waves per SIMD; 64 MB of active-list slots)
#endif
constexpr int kActWide = 64, kWideThreads = VR_WIDE_THREADS, kWideBlock = 64;

constexpr int kMaxSpheres = 64;
// Deferred NEE (free-flight): a path's queued shadow rays are a linked list in the queue (kFFNone ends
// it); ff_tail's flag bit says its inline radiance follows them.
constexpr uint32_t kFFNone = 0x7fffffffu;
constexpr uint32_t kFFTailAfter = 0x80000000u;
constexpr uint32_t kFFNeeMaxPerPath = 16;  // VR_OPT_FF_NEE_QUEUE bound (queue rays per path of a launch)
// Renders of one frame before a capacity report becomes VR_ERR_OVERFLOW, shared by a context
// (render_sync) and a group (group_render). A frame over its record buffers fits the next time (they are
// grown to the counted need + 1/8). The shadow-ray queue starts at >= 1 ray per path and at most doubles
// per render up to its bound (<= kFFNeeMaxPerPath rays per path: log2 16 = 4 doublings), then one
// render traces every shadow ray inline: 1 + 4 + 1 renders, + 1 for a record-capacity retry.
constexpr int kFrameAttempts = 7;
constexpr int32_t kFFBigCap = 1024;          // ff_fallback_kernel: Gaussians overlapping one point it can sweep
constexpr uint32_t kFFBigThreads = 1024;     // ff_fallback_kernel: threads (scratch row stride)

// Kernel launch parameters (passed by value).
struct RenderArgs {
    // camera
    int32_t cam_type;
    float cam_pos[3], cam_view[3], cam_right[3], cam_up[3], cam_pinhole[3];
    // frame / tiles
    uint32_t width, height, tiles_x, first_tile, tile_stride, num_tiles;
    int32_t packed;
    float* out;
    // scene
    const GaussianRecord* gauss;
    const WRecord* wrec;      // whitened copy of gauss (secondary rays of RayMarchingGaussians)
    // tile bins of the binned march (VR_OPT_MARCH_BINNED; nullptr: the BVH march): bin (tile_local,
    // depth bucket b) = entries bin_ent[bin_off[tile_local * bin_nb + b] ..), each a record index:
    // the records whose 3.15-sigma box may hold a point of the tile's pixel rays at ray distance
    // >= b * bin_dz (the bucket's lower bound of every entry distance of those rays)
    const uint32_t* bin_off;
    const uint32_t* bin_ent;
    uint32_t* bin_cnt;        // binning scratch: per-bin counts, then per-bin cursors
    uint32_t* bin_out;        // binning output (bin_ent while it is being written)
    uint32_t bin_nb;
    float bin_dz;
    const BVHNode* nodes;
    const HNode* hnodes;      // nullptr: the scene is not suited to half-precision boxes (see vr_device.cpp)
    const HNode4* hnodes4;    // 4-wide collapse of the same tree (secondary rays); nullptr with hnodes
    const HNode4* hnodes4s;   // the secondary rays' copy with tight boxes (gauss_refit_secondary), else hnodes4
    const HNode4* hnodes4t;   // hnodes4s's nodes with the boxes laid out per axis (soa_nodes_kernel), or nullptr
    const HNode4* hnodes4w;   // hnodes4's nodes laid out per axis (soa_nodes_kernel; read by wide_children), with hnodes4
    const int32_t* prim_node4;  // the 4-wide node whose child is each record's leaf (record starts), or nullptr
    const int32_t* hn4_parent;  // parent of every HNode4 | (its slot + 1) << 28 (root: -1); nullptr: walks start at the root
    uint32_t num_nodes4;        // HNode4 count
    float hn_center[3], hn_scale;
    const SphereRecord* spheres;
    int32_t num_prims;
    int32_t bvh_depth;  // deepest node level of the uploaded BVH (root = 1)
    int32_t num_lights;
    LightRecord lights[kMaxLights];
    float env[3];
    // march
    float step_size;
    int32_t env_samples;
    float t_eps;
    float tau_cut;        // secondary rays: Tr := 0 once the optical depth reaches this (see vr_device.cpp)
    int32_t pure;         // PureRayMarching: marched (point-sampled) transmittance, integrator.h:100-267
    const float* tsteps;  // iterated float step sequence t_k (test_integrators.h:184,289)
    int32_t num_tsteps;
    // fallback queue (active-set overflow) and error counters
    uint32_t* queue;       // [0] = count, [1..] = packed pixel ids (tile_local << 8 | lane)
    uint32_t queue_cap;
    uint32_t* deepq;       // [0] = count, [1..] = pixels for march_deep_kernel (active set > 64)
    uint32_t deepq_cap;
    int32_t* deep_act;     // march_deep_kernel's active lists, [slot][thread]
    int32_t* wide_act;     // march_wide_kernel's active lists, [slot][thread]
    uint32_t wide_min;     // fallback pixels from which the per-lane wide pass takes the queue (VR_OPT_MARCH_WIDE_MIN)
    int32_t march_big;     // 1: the primary march with kActBig LDS slots (a scene whose earlier frame overflowed 16 often)
    uint32_t* counters;    // [0] = error pixels / paths, [2] = free-flight paths re-run in ff_fallback_kernel,
                           // [3] = the most shadow rays a free-flight launch of the frame tried to queue
    unsigned long long* work;  // instrumented build only: [0..7] march-kernel counters, [8..15] secondary-kernel counters

    // ---- wavefront buffers (RayMarchingGaussians), pixel-local index p = tile_local * 256 + lane ----
    uint32_t* px_first; // first scatter record of pixel p (kNoRecord: none); later ones via rec_next
    float* px_T;        // transmittance left after the march (multiplies env_color at the end)
    float4* rec_pos;    // per record: pos.xyz, T * sigma_s
    uint4* rec_meta;    // per record: x | y << 16, step index k, act offset, act count
    uint32_t* rec_next; // per record: the pixel's next record in step order (kNoRecord: last)
    int32_t* rec_act;   // active Gaussians (leaf-order ids) of each record, sorted: kActInline slots per
                        // record, longer lists in the overflow pool after rec_cap * kActInline
    float* tr;          // per secondary ray: transmittance, slot = chunk * rays-per-chunk + hand-out index
    float4* rec_rad;    // per record: Li + Le (record_radiance_kernel), the radiance the accumulation weighs
    uint32_t* rec_alloc;  // [0] records allocated, [1] overflow-pool entries allocated, [2] capacity exceeded
    uint32_t rec_cap, act_ovf_cap;
    unsigned long long* rec_bloom;  // per record: 64-bit membership mask of its active list
    uint32_t* slowq;                // light rays needing the exact stopping event: [0] count, [1..] ray ids
    uint32_t slowq_cap;
    uint32_t* fixq;                 // env rays with one chord in the f32 error band: [0] count, [1 + 3i] ray id, [2 + 3i] tau, [3 + 3i] Gaussian
    uint32_t fixq_cap;
    unsigned long long* ray_next;   // persistent secondary kernel: next unclaimed ray id
    int32_t* stack_ovf;             // persistent secondary kernel: traversal-stack entries past its LDS stack
    uint32_t stack_ovf_lanes;       // lanes (grid x block) the overflow buffer holds
    uint16_t* env_order;            // per record chunk: its environment rays (record-in-chunk << 8 | sample), direction order
    uint64_t* env_base;             // with env_order: per record, the generator state its environment samples jump from
    uint32_t chunk_rec;             // records per secondary-ray chunk (power of 2; 64 without env_order)
    uint32_t chunk_shift;           // log2(chunk_rec)
    float* rec_cut;                 // per record: optical-depth cut-off of its secondary rays (nullptr: tau_cut)
    int32_t* rec_start;             // per record: the HNode4 subtree its secondary rays walk first (nullptr: the root)
    // ---- free-flight integrators (vr_freeflight.hip): one (tile chunk, sample batch) step ----
    int32_t ff_multi;        // 0 FreeFlightGaussians, 1 MultiScatterGaussians
    int32_t ff_samples;      // samples per pixel (integrator num_samples)
    int32_t ff_n;            // int(sqrt(num_samples)): strata per axis (integrator.h:564)
    int32_t ff_min_bounces;  // MultiScatterGaussians min_scatter (Russian roulette after it)
    int32_t ff_max_bounces;  // safety bound on a path's bounces (exceeded: error path)
    int32_t ff_solver;       // distance solver (VR_OPT_FF_SOLVER, distance_solvers.h:143-187): 0 ANALYTIC_PLUS_NEWTON,
                             // 1 BISECTION, 2 NEWTON, 3 ANALYTIC_PLUS_BISECTION, 4 UNIFORM
    uint32_t ff_si0, ff_nsb; // first sample index of the batch, samples in the batch
    uint32_t ff_tile_base;   // first tile (tile-local index) of the chunk
    uint32_t ff_threads;     // threads of one step = row stride of the scratch arrays
    int32_t ff_hit_cap, ff_act_cap;  // per-thread hit-buffer / active-list capacities
    int32_t ff_hit_cap0;     // first window's capacity (doubles per window up to ff_hit_cap)
    float4* ff_hit;          // scratch [hit_cap][threads]: entry key, exit t1, record id, -
    float4* ff_act0;         // scratch [act_cap][threads]: per active entry P, B, 2A, den
    float4* ff_act1;         // scratch [act_cap][threads]: per active entry F, F_next, t1, hit slot
    unsigned long long* ff_next;  // persistent path kernel: next unclaimed path of the launch
    unsigned long long ff_total;  // paths of the launch (tiles of the chunk x samples x 256)
    float* ff_sum;           // [tile-local pixel][3] running sum over sample batches
    // Paths over the path kernel's hit-buffer capacity (more than ff_hit_cap Gaussians overlapping one
    // point): queued and re-run whole by ff_fallback_kernel with kFFBigCap-entry rows (inline NEE).
    uint32_t* ff_fbq;        // [0] count, [1..] path indices of the launch (nullptr: no fallback pass)
    uint32_t ff_fbq_cap;
    float4* ff_big;          // the fallback's scratch rows: hit, act0, act1, each [kFFBigCap][kFFBigThreads]
    // Deferred next-event estimation: the path kernel queues a bounce's shadow ray instead of tracing
    // it; ff_nee_kernel traces the queue and writes each contribution into its path's slot; the
    // accumulation adds a path's slots in bounce order (see vr_freeflight.hip).
    float4* ff_nee;          // queue, 3 float4 per ray: {o, tmax}, {d, next ray of the path (bits)},
                             // {m0 m1 m2, light bits (-1: env)}; ff_nee_kernel overwrites m with m * Li
    uint32_t* ff_nee_n;      // [0] rays queued in the launch (may pass ff_nee_cap: those rays went inline)
    uint32_t ff_nee_cap;     // queue capacity in rays (0: every shadow ray is traced inline)
    int32_t ff_nee_refill;   // idle lanes of a wave that trigger its refill in ff_nee_kernel
    float4* ff_tail;         // [path of the launch]: {inline radiance xyz, first queued ray | kFFTailAfter}
    int32_t ff_sm;           // persistent path kernel: 1 the phase-scheduled ff_path_sm_kernel, 0 ff_path_kernel
    const uint32_t* gauss_order;  // record (leaf order) -> scene index
    uint32_t* rec_bits;      // RECORD_PIXEL_GAUSSIANS bitset [word][pixel] (nullptr: not recording)
    uint32_t rec_npix;       // W * H
    const unsigned long long* pcg_jump;  // [2k] = A^k, [2k+1] = inc (A^(k-1) + ... + 1): PCG32 state after k draws
};

}  // namespace vr
