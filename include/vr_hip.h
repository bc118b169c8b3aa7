/*
 * vr_hip.h — C ABI of the MI355X-native forward volume renderer (libvr_hip.so).
 *
 * This is the drop-in boundary for the reference's forward render call
 *     Integrator::render(const Scene&, Image&)            (include/integrator.h:49-57)
 * of wantonsushi/3DG-vol-renderer. Plain C: opaque handles, plain structs, pointers and sizes,
 * integer status codes, no exceptions and no C++/torch types across the boundary. The header-only
 * C++ mirror of the reference API (3dg-vol-renderer_amd/include/vr/: Scene, Camera, Image,
 * Integrator, HipRayMarchingGaussians ...) and the Python ctypes mirror (vr_amd) both sit on top
 * of exactly these entry points. INTEGRATION.md shows the bindings.
 *
 * Every entry point returns VR_OK (0) on success; on failure it returns a non-zero vr_status and
 * vr_last_error() (thread-local) describes why. The C++ wrappers turn a non-zero status into
 * std::runtime_error, which is the reference's error convention (scene.h:47,79; image.h:26,30).
 */
#ifndef VR_HIP_H_
#define VR_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VR_ABI_VERSION 7

typedef enum vr_status {
    VR_OK = 0,
    VR_ERR_INVALID = 1,     /* bad argument / inconsistent request */
    VR_ERR_IO = 2,          /* cannot open / read / write a file */
    VR_ERR_PARSE = 3,       /* malformed scene / XML / PPM */
    VR_ERR_HIP = 4,         /* HIP runtime error (includes "no GPU") */
    VR_ERR_NOSCENE = 5,     /* render before vr_upload_scene */
    VR_ERR_OVERFLOW = 6,    /* a per-ray capacity (active set, stack, step table) was exceeded */
    VR_ERR_UNSUPPORTED = 7, /* valid request the device path does not implement */
    VR_ERR_RETRY = 8        /* vr_synchronize only: the last frame outgrew the scatter-record buffers
                               sized from earlier frames; they have been grown, render it again */
} vr_status;

/* scene.h:18-22 Scene::VolumeType */
typedef enum vr_volume_type { VR_VOLUME_GAUSSIANS = 0, VR_VOLUME_SPHERES = 1 } vr_volume_type;

/* camera.h:31 Pinhole_Camera, camera.h:58 Orthographic_Camera */
typedef enum vr_camera_type { VR_CAMERA_PINHOLE = 0, VR_CAMERA_ORTHOGRAPHIC = 1 } vr_camera_type;

/* Integrators with a device implementation. */
typedef enum vr_integrator {
    VR_RAYMARCH_GAUSSIANS = 0, /* RayMarchingGaussians  test_integrators.h:143-297 */
    VR_RAYMARCH_SPHERES = 1,   /* RayMarchingSpheres    test_integrators.h:11-136  */
    VR_TEST_HITMASK = 2,       /* TestIntegrator        integrator.h:65-94         */
    VR_PURE_RAYMARCH = 3,      /* PureRayMarching       integrator.h:100-267       */
    VR_FREE_FLIGHT = 4,        /* FreeFlightGaussians   integrator.h:273-408 (single scattering) */
    VR_MULTI_SCATTER = 5       /* MultiScatterGaussians integrator.h:416-720 (ANALYTIC_PLUS_NEWTON) */
} vr_integrator;

/* Light (scene.h:12-15). */
typedef struct vr_light {
    float position[3];
    float intensity[3];
} vr_light;

/* One 'g' record of a scene file / arguments of Gaussian(mean, cov, density, albedo, emission)
 * (scene.h:91-113, gaussian.h:75-92). cov = {xx, xy, xz, yy, yz, zz}. Emission is carried for API
 * parity but is never read by any reference integrator. */
typedef struct vr_gaussian {
    float mean[3];
    float cov[6];
    float density;
    float albedo;
    float emission[3];
} vr_gaussian;

/* Sphere(center, radius, sigma_a, sigma_s) (smm.h:17-27). */
typedef struct vr_sphere {
    float center[3];
    float radius;
    float sigma_a;
    float sigma_s;
} vr_sphere;

/* Camera state after the reference constructors ran (camera.h:15-22, 38-43, 60-62). */
typedef struct vr_camera {
    int32_t type;        /* vr_camera_type */
    float position[3];
    float view_dir[3];   /* normalised member Camera::view_dir */
    float right[3];
    float up[3];
    float pinhole[3];    /* pinhole cameras only */
    float fov;
    float focal_length;  /* 1 / tan(fov / 2) */
} vr_camera;

/* Render parameters = the integrator constructor arguments (test_integrators.h:17,149-153;
 * integrator.h:278-281, 501-505). */
typedef struct vr_render_params {
    int32_t integrator;   /* vr_integrator */
    float step_size;      /* ray-march step (reference default 0.01) */
    int32_t env_samples;  /* environment directions per scattering step (20 Gaussians, 5 spheres) */
    float t_eps;          /* stop a ray once T <= t_eps; 0 = exact (stop only when T == 0) */
    uint32_t flags;       /* reserved, must be 0 */
    int32_t num_samples;  /* free-flight integrators: paths per pixel (FreeFlightGaussians 256,
                             MultiScatterGaussians 16; set_num_samples, integrator.h:719) */
    int32_t min_bounces;  /* MultiScatterGaussians min_scatter (default 5): Russian roulette after it */
} vr_render_params;

typedef struct vr_scene_info {
    int32_t volume_type;  /* vr_volume_type */
    int64_t num_primitives;
    int64_t num_lights;
    float env_color[3];
    float bounds_min[3];  /* union of the primitives' 3-sigma / sphere boxes */
    float bounds_max[3];
} vr_scene_info;

/* Statistics of the last vr_render / vr_render_tiles_device call on a context (waits for it). */
typedef struct vr_render_stats {
    double kernel_ms;         /* device time of the render kernels (HIP events) */
    int64_t pixels;           /* pixels rendered */
    int64_t fallback_pixels;  /* pixels re-run on the large-capacity path (active-set overflow);
                                 free-flight integrators: paths re-run with kFFBigCap-entry rows
                                 (more than 128 Gaussians overlapping one point) */
    int64_t error_pixels;     /* pixels that exceeded every capacity (output NaN) */
    /* Stages (HIP events on the render stream). RayMarchingGaussians: [0] primary march (scatter
     * records), [1] record-buffer sizing (one host sync; a re-run of the march if the capacity
     * carried over from the last frame was too small) and secondary-ray cut-offs, [2] secondary-ray
     * transmittance, [3] accumulate. FreeFlight / MultiScatterGaussians: [0] path kernel, [2]
     * deferred shadow rays, [3] accumulate. 0 for the other integrators. */
    double stage_ms[4];
    int64_t scatter_records;  /* march steps with sigma_s > 0 (each spawns lights + env_samples rays) */
    int64_t secondary_rays;   /* records * (lights + env_samples) */
    int64_t record_overflow;  /* 1: the frame outgrew the scatter-record buffers sized from earlier
                                 frames (its output is invalid; the buffers have been grown, render
                                 again). vr_render does that itself. */
    int64_t deep_pixels;      /* pixels re-run on the global-memory active-list pass (> 64 active) */
    int64_t slow_rays;        /* RayMarchingGaussians: secondary rays traced again on the exact slow path (a light
                                 ray's stopping event, a missed member, a member at its 3-sigma boundary, two
                                 chords or a member's within the reference f32 quadratic's error band) */
    int64_t band_rays;        /* RayMarchingGaussians: secondary rays with one non-member chord within that band,
                                 whose contribution the reference's M form recomputes (secondary_fix_kernel) */
} vr_render_stats;

typedef struct vr_scene vr_scene; /* host-side scene: primitives, lights, env colour */
typedef struct vr_ctx vr_ctx;     /* device context: one GPU, uploaded scene, workspaces */

/* ---------------- library ---------------- */
const char* vr_version(void);
/* Thread-local description of the last failure of any vr_* call on this thread. */
const char* vr_last_error(void);

/* ---------------- host scene (scene.h) ---------------- */
vr_status vr_scene_create(int32_t volume_type, vr_scene** out);
/* Scene::load_GMM (scene.h:72-120), incl. its skip-unknown-token and emission-peek behaviour. */
vr_status vr_scene_load_gmm(const char* path, vr_scene** out);
/* Scene::load_SMM (scene.h:38-68). */
vr_status vr_scene_load_smm(const char* path, vr_scene** out);
/* Mitsuba-3 subset used by tests/env_one_sphere_test_ortho.xml (no reference equivalent; the
 * reference rendered that XML in Mitsuba). Fills the scene, camera, film size and parameters.
 * Any output pointer may be NULL. */
vr_status vr_scene_load_xml(const char* path, vr_scene** out, vr_camera* camera, uint32_t* width,
                            uint32_t* height, vr_render_params* params);
vr_status vr_scene_add_gaussians(vr_scene* s, const vr_gaussian* g, size_t n);
/* Synthetic scenes of the reference generators' distribution (tests/make_random.py:21-45 for
 * variant 0, tests/make_nonuniform_random.py:19-30 (y biased towards 0) for variant 1): mean
 * x,z ~ U(-1,1), y ~ U(0,2); per-axis diameter ~ U(0.01, 0.035); covariance
 * Q diag((d/2)^2) Q^T with Q from the QR of a 3x3 standard-normal matrix (det fixed to +1);
 * density ~ U(0.2, 0.5); albedo ~ U(0.25, 0.95); emission ~ U(0,1)^3. Values are rounded exactly as
 * the generators print them (%.4f / %.6f) and then read back as floats, so a generated scene is
 * the scene load_GMM would produce from the generator's text file. Seeded PCG32 (rng.h). */
vr_status vr_scene_add_random_gaussians(vr_scene* s, uint64_t n, uint64_t seed, int32_t variant);
vr_status vr_scene_add_spheres(vr_scene* s, const vr_sphere* sp, size_t n);
vr_status vr_scene_add_lights(vr_scene* s, const vr_light* l, size_t n);
vr_status vr_scene_set_env_color(vr_scene* s, const float rgb[3]);
vr_status vr_scene_get_info(const vr_scene* s, vr_scene_info* out);
/* Gaussian precompute (gaussian.h:52-55): 12 floats per Gaussian, in scene order:
 * mean[3], density, inv_cov{00,01,02,11,12,22}, norm, albedo. */
vr_status vr_scene_get_records(const vr_scene* s, float* out, size_t n);
vr_status vr_scene_get_lights(const vr_scene* s, vr_light* out, size_t n);
vr_status vr_scene_get_gaussians(const vr_scene* s, vr_gaussian* out, size_t n);
vr_status vr_scene_get_spheres(const vr_scene* s, vr_sphere* out, size_t n);
void vr_scene_destroy(vr_scene* s);

/* ---------------- camera (camera.h) ---------------- */
vr_status vr_camera_pinhole(const float position[3], const float view_dir[3], float fov, vr_camera* out);
vr_status vr_camera_orthographic(const float position[3], const float forward[3], vr_camera* out);
/* Camera::sample_ray (camera.h:45-53, 64-73) followed by Ray's normalisation (ray.h:11-12). */
vr_status vr_camera_sample_ray(const vr_camera* c, double u, double v, float origin[3], float direction[3]);

/* ---------------- image (image.h) ---------------- */
/* Image::make_PPM (image.h:62-84): 8-bit P6 with clamp(v*255) truncation. rgb is 3*W*H floats. */
vr_status vr_image_write_ppm(const char* path, const float* rgb, uint32_t width, uint32_t height);
/* Image(const std::string&) (image.h:24-45): P6 reader; rgb must hold 3*W*H floats. Pass rgb=NULL
 * to query width/height only. */
vr_status vr_image_read_ppm(const char* path, float* rgb, uint32_t* width, uint32_t* height);

/* ---------------- animated GIF (tests/main.cpp:81-114 turntable; gif-h's role) ---------------- */
typedef struct vr_gif vr_gif;
/* GifBegin: a looping GIF89a of width x height frames (delay_cs: the default frame delay, 1/100 s). */
vr_status vr_gif_begin(const char* path, uint32_t width, uint32_t height, uint32_t delay_cs, vr_gif** out);
/* GifWriteFrame: one RGBA8 frame (Image::get_rgba_buffer, image.h:89-104) shown for delay_cs
 * hundredths of a second; its own 256-colour palette (median cut), LZW-compressed. */
vr_status vr_gif_write_frame(vr_gif* gif, const uint8_t* rgba, uint32_t delay_cs);
/* GifEnd: trailer, close, free. */
vr_status vr_gif_end(vr_gif* gif);

/* ---------------- device ---------------- */
vr_status vr_init(int device, vr_ctx** out);
/* Number of visible GPUs. */
vr_status vr_device_count(int32_t* n);
/* Multi-GPU context: one host thread drives `ndev` GPUs (devices[0..ndev-1], or
 * 0..ndev-1 if devices is NULL). vr_upload_scene replicates the scene on every device; vr_render cuts
 * the frame into 16x16 tiles, rank r renders tiles r, r+ndev, r+2ndev, ... into a packed slab on its
 * device, the slabs are gathered to devices[0] with RCCL (one ncclGroupStart/End of every rank's
 * ncclSend and the root's ncclRecv over xGMI; librccl is loaded at this call) and unshuffled there
 * into the row-major frame. A device listed more than once shares its GPU between ranks (rehearsal
 * of the split on one GPU; the slabs then move with device copies, RCCL holds one rank per device).
 * vr_synchronize / vr_set_option apply to every device; vr_get_stats sums counts over the ranks and
 * reports the slowest rank's times (vr_get_rank_stats: one rank). The other entry points act on the
 * first device. vr_destroy releases the whole group. */
vr_status vr_init_multi(int32_t ndev, const int32_t* devices, vr_ctx** out);
/* Devices a context drives (1 for vr_init contexts); whether its gather runs over RCCL. */
int32_t vr_ctx_num_devices(const vr_ctx* ctx);
int32_t vr_ctx_uses_rccl(const vr_ctx* ctx);
vr_status vr_get_rank_stats(vr_ctx* ctx, int32_t rank, vr_render_stats* out);
void vr_destroy(vr_ctx* ctx);
/* Prepare (BVH build) and upload the scene; replaces any previous one. Host copies are not kept. */
vr_status vr_upload_scene(vr_ctx* ctx, const vr_scene* s);
/* Integrator::render(scene, image): full W x H frame into rgb_host (3*W*H floats, row-major,
 * idx = 3*(y*W + x) as image.h:13-17). Synchronous. */
vr_status vr_render(vr_ctx* ctx, const vr_camera* cam, const vr_render_params* p, uint32_t width,
                    uint32_t height, float* rgb_host);
/* Multi-GPU building block (asynchronous on `stream`, a hipStream_t or NULL for the default; the
 * host never waits for the device inside a frame once the context has rendered one frame of this
 * kind — the first sizes the scatter-record buffers). The frame's outcome is reported by
 * vr_synchronize (VR_ERR_RETRY if the frame outgrew the record buffers, which are then grown:
 * render it again; VR_ERR_OVERFLOW if pixels exceeded a per-ray capacity) and by vr_get_stats.
 * The frame is cut into 16x16 tiles numbered row-major; this call renders tiles
 * first_tile, first_tile + tile_stride, ... (num_tiles of them). If `packed` is non-zero the
 * output is a slab of num_tiles * 256 pixels (tile-major, row-major inside a tile, 3 floats per
 * pixel; pixels outside the frame are written as 0); otherwise `d_out` is the full W x H frame and
 * only those tiles' pixels are written. d_out is device memory. */
vr_status vr_render_tiles_device(vr_ctx* ctx, const vr_camera* cam, const vr_render_params* p,
                                 uint32_t width, uint32_t height, uint32_t first_tile,
                                 uint32_t tile_stride, uint32_t num_tiles, int32_t packed,
                                 float* d_out, void* stream);
/* Scatter `nslabs` packed slabs (slab r = tiles r, r+nslabs, ...; each tiles_per_slab * 256 px)
 * into the row-major W x H frame d_image. Asynchronous on `stream`. */
vr_status vr_unshuffle_tiles_device(vr_ctx* ctx, const float* d_slabs, uint32_t nslabs,
                                    uint32_t tiles_per_slab, uint32_t width, uint32_t height,
                                    float* d_image, void* stream);
/* Scatter the packed slabs of ranks first .. first + nslabs - 1 of a stride-way split (slab k = tiles
 * first + k, first + k + stride, ...; each tiles_per_slab * 256 px) into the row-major W x H frame
 * d_image: the gather of a split whose root rendered its own tiles straight into the frame.
 * Asynchronous on `stream`. */
vr_status vr_unshuffle_tiles_part_device(vr_ctx* ctx, const float* d_slabs, uint32_t first, uint32_t nslabs,
                                         uint32_t stride, uint32_t tiles_per_slab, uint32_t width, uint32_t height,
                                         float* d_image, void* stream);
/* Diagnostics (untimed): render the given tiles once with the instrumented build of the same
 * kernels and return the work they executed. counts[0..7], the march kernels (both passes):
 * [0] BVH node tests (4-wide nodes, or child pairs on the fallback path), [1] ray-Gaussian
 * quadratic + intersect evaluations, [2] optical-depth evaluations, [3] density (mu_t)
 * evaluations, [4] unused, [5] active march steps, [6] primary-ray BVH queries, [7] pixels completed.
 * counts[8..15], the secondary-ray stage (the persistent kernel's own schedule + the exact slow path):
 * [8] BVH node steps, [9] tree-leaf primitive tests, [10] optical-depth evaluations, [11] active-
 * list primitive tests, [12] secondary rays started, [13] rays ended by the optical-depth cut-off,
 * [14] node steps of those rays, [15] node steps of the rays that ran to the end of the tree.
 * Free-flight integrators: counts[0..7], the path kernel: [0] paths, [1] free-flight distance
 * searches (bounces), [2] 4-wide node steps and [3] child-pair node steps of the hit-collection
 * walks, [4] ray-Gaussian quadratic + intersect evaluations, [5] erf evaluations of the event sweep,
 * the entries' cached factors and the distance solver, [6] shadow rays traced inline, [7] shadow
 * rays queued; counts[8..11], the shadow-ray kernel: [8] rays, [9] 4-wide node steps, [10] primitive
 * tests, [11] optical depths. Synchronous; Gaussian scenes only. Used for the roofline reports. */
vr_status vr_count_work(vr_ctx* ctx, const vr_camera* cam, const vr_render_params* p, uint32_t width,
                        uint32_t height, uint32_t first_tile, uint32_t tile_stride, uint32_t num_tiles,
                        uint64_t counts[16]);
/* MultiScatterGaussians::render(scene, image, &per_pixel_gaussians) under RECORD_PIXEL_GAUSSIANS
 * (integrator.h:532-536, 616-644): renders like vr_render (params->integrator must be
 * VR_MULTI_SCATTER) and records, per pixel, the Gaussians (scene order) with an event at or before
 * a path's scattering point (t <= t_scatter + 1e-6), or every Gaussian hit by a path segment that did
 * not scatter, as a bitset in the context's recording `slot` (0 or 1). Synchronous. */
vr_status vr_render_record(vr_ctx* ctx, const vr_camera* cam, const vr_render_params* p, uint32_t width,
                           uint32_t height, float* rgb_host, int32_t slot);
/* Copy a recording to the host: bits[w * W*H + p] bit b set <=> Gaussian 32w + b was recorded at
 * row-major pixel p. n_words must be ceil(N/32) * W * H. */
vr_status vr_get_pixel_gaussians(vr_ctx* ctx, int32_t slot, uint32_t* bits, size_t n_words);
/* Stochastic finite-difference statistic of StochasticFiniteDiffInverseIntegrator::optimize
 * (inverse_integrator.h:166-182): out[g] = sum over the union of the pixels recorded for Gaussian g
 * in slot 0 (base render) and slot 1 (perturbed render) of loss_plus[p] - loss_base[p] (double).
 * loss_* are host arrays of W*H per-pixel L1 losses (compute_pixel_losses, :21-30); n = N. */
vr_status vr_sfd_loss_diff(vr_ctx* ctx, const float* loss_base, const float* loss_plus, uint32_t width,
                           uint32_t height, double* out, size_t n);
/* ---------------- inverse rendering (gmm.h:583-706, optimizer.h, inverse_integrator.h) ---------------- */
/* GaussianMixtureModel::pack_parameters (gmm.h:583-628): 11 floats per Gaussian, scene order: mean(3),
 * Rodrigues rotation of the covariance eigenbasis (3), log scale (3), log density, logit albedo.
 * n_params must be 11 * N. (Eigenbasis from a Jacobi solver, made right-handed: DESIGN.md §3c.) */
vr_status vr_gmm_pack_parameters(const vr_scene* s, float* params, size_t n_params);
/* apply_params_to_gmm_local (gmm.h:634-674): a new scene with base's lights / environment and every
 * Gaussian rebuilt from params (covariance R S S^T R^T, density exp, albedo sigmoid). */
vr_status vr_gmm_apply_parameters(const vr_scene* base, const float* params, size_t n_params, vr_scene** out);
/* make_default_eps_for_params (gmm.h:678-706). */
vr_status vr_gmm_default_eps(float* eps, size_t n_params);
/* AdamOptimizer::step (optimizer.h:31-44) for step number t >= 1 (m, v: the moment vectors). */
vr_status vr_adam_step(float* params, const float* grads, float* m, float* v, size_t n, int32_t t, float lr, float beta1,
                       float beta2, float eps);
/* Sign vector k of vr_sfd_optimize's run with `seed` (+1 / -1 per parameter): the deterministic
 * stand-in for the reference's coin(mt19937(random_device)) (inverse_integrator.h:101-103, 139-141). */
vr_status vr_sfd_sign_vector(uint64_t seed, uint64_t k, float* signs, size_t n);

/* SFDDConfig (inverse_integrator.h:52-57) + run options. */
typedef struct vr_sfd_config {
    int32_t max_iters;          /* reference default 1000 */
    int32_t save_every;         /* 25: render + write out_dir/iter_NNNN.ppm every save_every iterations */
    int32_t num_stoch_samples;  /* 4: sign vectors per iteration */
    float lr;                   /* 1e-2 (Adam) */
    uint64_t seed;              /* sign-vector stream (vr_sfd_sign_vector) */
    int32_t final_samples;      /* 16384: paths per pixel of the final render (:229-238); 0 skips it */
    const char* out_dir;        /* NULL / "": write no images (the reference writes ./sfd_output) */
} vr_sfd_config;
typedef struct vr_sfd_result {
    float* params;         /* out, 11 * N: the optimised parameters (caller-allocated) */
    double* loss_history;  /* out, max_iters: mean L1 loss of every base render */
    double* last_grads;    /* out (may be NULL), 11 * N: the last iteration's SFD gradient estimate */
    float* final_image;    /* out (may be NULL), 3 * W * H: the final render */
    double final_loss;     /* out: its mean L1 loss (-1 if final_samples == 0) */
} vr_sfd_result;
/* StochasticFiniteDiffInverseIntegrator::optimize(scene_initial, I_ref) (inverse_integrator.h:61-238)
 * on the context's device: per iteration a recorded base render (RECORD_PIXEL_GAUSSIANS bitsets in
 * HBM), num_stoch_samples perturbed recorded renders, the per-Gaussian union-of-pixels loss
 * statistic and per-pixel L1 losses on the device, Adam on the host; every parameter update is
 * re-uploaded with the device BVH build. fwd: MultiScatterGaussians parameters; I_ref: 3 * W * H. */
vr_status vr_sfd_optimize(vr_ctx* ctx, const vr_camera* cam, const vr_render_params* fwd, const vr_scene* scene_initial,
                          const float* I_ref, uint32_t width, uint32_t height, const vr_sfd_config* cfg,
                          vr_sfd_result* result);
/* Number of 16x16 tiles of a W x H frame. */
uint32_t vr_num_tiles(uint32_t width, uint32_t height);
/* Per-context tuning options (defaults are the benchmark/product settings). Explicit and
 * re-entrant: the library reads no environment variables. */
typedef enum vr_option {
    VR_OPT_HALF_NODES = 1,       /* 1 (default): upload f16 copies of the BVH (pair + 4-wide) when the
                                    scene's leaf boxes suit them; 0: f32 nodes only. Applies at the next
                                    vr_upload_scene. Results are identical either way (boxes only
                                    propose candidates; every decision is the exact quadratic). */
    VR_OPT_SECONDARY_BUDGET = 2, /* 1 (default): with t_eps > 0, stop secondary rays at a per-record
                                    optical depth that keeps each pixel within t_eps (DESIGN.md error
                                    budget); 0: the frame-wide cut-off ln(1/t_eps) + ln(1000) only. */
    VR_OPT_FF_WINDOW0 = 3,       /* free-flight integrators: first hit-window capacity, 1..128, doubling per
                                    window; 0 (default): derived from the uploaded scene's typical optical
                                    depth per Gaussian (4..32). Results do not depend on it. */
    VR_OPT_RECORD_CAPACITY = 4,  /* scatter-record buffer capacity (records; the active-list pool gets the
                                    same) carried into the next frame: 0 (size it at the next frame, with one
                                    host sync) or >= 4096. The context normally sizes it from earlier frames;
                                    setting it lets a test drive a frame over capacity (reported, then
                                    rendered again with grown buffers). Results do not depend on it. */
    VR_OPT_DEVICE_BVH = 5,       /* 0 (default): vr_upload_scene builds the BVH on the host (binned SAH);
                                    1: on the device (linear BVH: Morton sort + radix tree, kernels/
                                    vr_lbvh.hip) for scenes of >= 256 Gaussians — the fast path for the
                                    inverse loop's re-upload after every parameter update. Results are
                                    identical up to summation order (the event set is tree-independent). */
    VR_OPT_FF_NEE_QUEUE = 6,     /* free-flight integrators: shadow-ray queue capacity, in rays per path of a
                                    launch, 0..16 (default 6). The path kernel queues each bounce's next-event
                                    shadow ray for a separate tracing kernel; 0 traces them inline. Results
                                    are identical (the same walk and sums). A frame whose launch found the
                                    queue full is reported (VR_ERR_RETRY from the asynchronous entry points;
                                    vr_render re-renders by itself) and rendered again with a grown queue, or,
                                    once the queue is at this bound, with every shadow ray inline (so for the
                                    context's later frames, until the next upload or a change of this option).
                                    Memory: the queue holds value x (paths of a launch, at most 2^23) rays
                                    of 48 B, 2.4 GB at the default 6 per path; it is grown, never shrunk,
                                    per context (lower it for many contexts on one device). */
    VR_OPT_MARCH_BINNED = 7,     /* RayMarchingGaussians / PureRayMarching primary march: 0 (default): BVH
                                    window queries per pixel; 1: Gaussians binned to 16x16 tiles by depth
                                    bucket, each tile's list streamed by its waves.
                                    Results are identical (the same exact intersect decides every entry). */
    VR_OPT_FF_SOLVER = 8,        /* free-flight integrators: the distance solver (distance_solvers.h:143-187, a
                                    compile-time #define in the reference): 0 (default) ANALYTIC_PLUS_NEWTON, the
                                    mode the reference compiles (:146); 1 BISECTION; 2 NEWTON; 3
                                    ANALYTIC_PLUS_BISECTION; 4 UNIFORM, whose rand01() (mt19937 seeded by
                                    random_device, not reproducible) is replaced by the textbook-PCG32 uniform of
                                    stream 2 + bounce of the path's derive_path_seed (documented deviation). */
    VR_OPT_START_SUBTREE = 9,    /* RayMarchingGaussians / PureRayMarching secondary rays (4-wide tree): 1 (default):
                                    a ray walks the deepest subtree holding its record's position first, then
                                    climbs to the root (no descent from the root for rays cut near their origin);
                                    0: every walk starts at the root. Same Gaussians, same decisions; only the
                                    order of the optical-depth sum differs (float association). */
    /* 10: retired (round 6): the staged free-flight pipeline, measured 2.3x slower than the persistent path kernel */
    VR_OPT_SEC_TIGHT = 11,       /* RayMarchingGaussians secondary rays, applied at the next upload: 1 (default):
                                    their own copy of the 4-wide tree with the exact boxes of the ellipsoids the
                                    whitened test accepts (the shared tree's boxes are padded by 5 % for the
                                    camera rays' M-form test); 0: the shared tree. Same Gaussians, same
                                    decisions; only the order of the optical-depth sum differs. */
    VR_OPT_MARCH_WIDE_MIN = 12,  /* RayMarchingGaussians / PureRayMarching: pixels whose active set outgrew the
                                    primary march's 16 LDS slots are marched again; a queue of at least this
                                    many pixels (default 2048) goes one pixel per lane with 64 slots in
                                    global memory, a shorter one one pixel per wave (64 LDS slots). Same
                                    operations either way: frames are identical. */
    VR_OPT_FF_KERNEL = 13        /* free-flight integrators, persistent path kernel: 0 (default) chosen from the
                                    uploaded scene: the phase-scheduled kernel for translucent scenes of many
                                    Gaussians (at least 256, median central-chord optical depth below 16: long
                                    hit collections and event sweeps per bounce), else the bounce kernel;
                                    1: the bounce kernel (a whole bounce per lane and wave iteration);
                                    2: the phase-scheduled kernel (each wave iteration runs the collection, sweep
                                    or shading phase most of its lanes are in). Frames are identical. */
} vr_option;
vr_status vr_set_option(vr_ctx* ctx, int32_t option, int64_t value);
vr_status vr_get_option(vr_ctx* ctx, int32_t option, int64_t* value);
/* Waits for the context's device work; returns VR_ERR_RETRY / VR_ERR_OVERFLOW if the last frame is
 * invalid (see vr_render_tiles_device). The outcome is reported once per frame, also when vr_get_stats
 * (or any other call) collected the frame's report first; a later frame's call replaces it. */
vr_status vr_synchronize(vr_ctx* ctx);
vr_status vr_get_stats(vr_ctx* ctx, vr_render_stats* out);
/* Diagnostics: the pixels of the last RayMarchingGaussians / PureRayMarching frame that were re-run
 * on the large-capacity fallback path (vr_render_stats.fallback_pixels of them). Writes up to `cap`
 * (x, y) pairs into xy[2*cap] (global frame coordinates, queue order) and the total count into *n. */
vr_status vr_get_fallback_pixels(vr_ctx* ctx, uint32_t* xy, size_t cap, size_t* n);
/* Diagnostics (slow: one copy per value): the scatter records of pixel (x, y) of the last
 * RayMarchingGaussians frame in step order, one row of 9 + S floats each (S = lights + env_samples):
 * step index k, record position xyz, T * sigma_s, Li + Le (rgb), active-list length, then the
 * transmittance of each secondary ray (lights first, then environment samples, in sample order).
 * Writes up to `cap` rows of `row` floats into out, the record count into *n and the frame's row
 * width 9 + S into *row_out (if not NULL). With cap > 0, `row` must equal that width (VR_ERR_INVALID
 * otherwise: a narrower buffer would be written past its end); call with cap = 0 to learn both. */
vr_status vr_debug_pixel_records(vr_ctx* ctx, uint32_t x, uint32_t y, float* out, size_t cap, size_t row, size_t* n,
                                 size_t* row_out);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* VR_HIP_H_ */
