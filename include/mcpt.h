/*
 * mcpt.h -- C ABI of the MI355X-native wavefront path-tracing backend.
 *
 * Drop-in for the reference's CUDA path (JakeKurtz/MC-Path-Tracer):
 *   wavefront_pathtrace(...)   CUDA-RayTracer/wavefront_kernels.cuh:24-31 (body :377-442)
 *   clear_dfilm(dFilm*)        CUDA-RayTracer/wavefront_kernels.cuh:18   (body :55-76)
 *   draw_to_surface            CUDA-RayTracer/wavefront_kernels.cu:6-40
 *   PathTracer::render_image   CUDA-RayTracer/PathTracer.cpp:112-130
 *   Scene::load / set_environment_light / add_light   CUDA-RayTracer/Scene.h:40-58
 *   Camera::update (matrices)  CUDA-RayTracer/Camera.cu:194-224, PerspectiveCamera.cpp:49
 *
 * Conventions: every call returns 0 on success or a negative MCPT_E* code and
 * stores a message retrievable with mcpt_last_error(); nothing calls exit()
 * (the reference's checkCudaErrors exits with 99, CudaHelpers.cpp:3-11).
 * Host buffers passed in are copied; device memory is owned by the context.
 * Plain pointers and sizes only.
 */
#ifndef MCPT_H
#define MCPT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCPT_ABI_VERSION 1

enum {
    MCPT_OK = 0,
    MCPT_E_INVALID = -1,   /* bad argument / state */
    MCPT_E_HIP = -2,       /* HIP runtime error */
    MCPT_E_IO = -3,        /* file could not be read / parsed */
    MCPT_E_NOMEM = -4,
    MCPT_E_NODEVICE = -5   /* no gfx950 device: the product never falls back to the CPU */
};

/* Integrator configuration.  Reference mode reproduces the hard-coded values of
 * wavefront_kernels.cu: max_depth 5 (:142), rr_depth 3 (:189), spp <= 250 (:124). */
typedef struct mcpt_config {
    uint64_t seed;       /* keyed RNG seed; default 0x5EED2026 */
    int32_t spp;         /* samples per pixel (<= 2^19 - 256): gates processing and new samples */
    int32_t max_depth;   /* 'path_length > max_depth' terminates */
    int32_t rr_depth;    /* Russian roulette when 'path_length > rr_depth' */
    int32_t tile_w;      /* film tile (Film.cu:17: 256x256) */
    int32_t tile_h;
    int32_t flags;       /* MCPT_FLAG_* (0 = reference mode) */
} mcpt_config;

/* Quality mode: fixes the reference quirks of Appendix A.4-A.7, A.9 and
 * A.11 -- background added once, Russian-roulette survivors reweighted by 1/(1-q) with q from
 * the updated throughput, light-selection pdf 1/N, MIS weight 1 for delta lights, textbook
 * Gram-Schmidt, env sampling and pdf on matched (clamped) cells.  An alternative integrator:
 * never compared against the reference, only against the oracle's fixed mode. */
#define MCPT_FLAG_FIXED 1
/* The film observes the camera and the scene as in the reference (Film::update -> clear(),
 * Film.cu:278-281): mcpt_camera_set with a different camera, or a scene re-upload, marks the
 * film stale and the next mcpt_iterate / mcpt_wavefront_step / mcpt_render clears it first.
 * This flag turns that off (the caller clears explicitly with mcpt_film_clear). */
#define MCPT_FLAG_NO_AUTO_CLEAR 2

/* Scene as flat, BVH-ordered arrays (the device data model of Scene.h:24-33,
 * BVH.h:63-72, Triangle.h:11-23, dMaterial.cuh:11-33, EnvironmentLight.h:17-40). */
typedef struct mcpt_scene_desc {
    int32_t ntri;
    const float *v0, *v1, *v2;    /* 3*ntri world-space positions */
    const float *n0, *n1, *n2;    /* 3*ntri vertex normals */
    const int32_t *mat;           /* ntri material ids */
    int32_t nnodes;               /* LinearBVHNode array, depth-first */
    const float *bmin, *bmax;     /* 3*nnodes */
    const int32_t *offset;        /* primitivesOffset (leaf) / secondChildOffset (interior) */
    const int32_t *nprims;        /* 0 => interior */
    const int32_t *axis;
    int32_t nmat;
    const float *mat_params;      /* nmat*8: base rgb, fresnel rgb, roughness, metallic */
    int32_t ndir;                 /* directional lights (light ids 1..ndir; env is light 0) */
    const float *dir_params;      /* ndir*7: dir xyz, color rgb, ls */
    int32_t env_mode;             /* 0 = Color, 1 = HRDI */
    float env_color[3];
    float env_ls;
    int32_t env_w, env_h;
    const float *env_tex;         /* env_h*env_w*4 RGBA32F, row 0 = top */
    const float *env_marginal_y;  /* env_h */
    const float *env_conds_y;     /* env_h*env_w */
    const float *env_pdf;         /* env_h*env_w */
    const int32_t *tri_id;        /* optional ntri original triangle ids (NULL = array position): the
                                     exact-t tie-break key and the id the trace API reports, so
                                     neither depends on the order a BVH builder stored triangles in */
} mcpt_scene_desc;

/* dCamera (Camera.h:34-46): column-major m[c][r] = m[c*4+r]. */
typedef struct mcpt_camera {
    float inv_view_proj[16];
    float inv_view[16];
    float lens_radius;
    float focal;
} mcpt_camera;

/* PerspectiveCamera parameters (Camera.h:98-117, PerspectiveCamera.cpp:30-49). */
typedef struct mcpt_camera_params {
    float position[3];
    float yaw_deg, pitch_deg;     /* Camera.cu:210-224 */
    float fovy_rad, aspect, znear, zfar;
    float lens_radius, focal;     /* defaults 1e-4, 35 (Camera.h:115-116) */
} mcpt_camera_params;

typedef struct mcpt_stage_stats {
    uint64_t extend_rays;   /* closest-hit rays traced */
    uint64_t shadow_rays;   /* light-sample shadow rays */
    uint64_t vis_rays;      /* BRDF-sample visibility rays (wavefront_kernels.cu:334-336) */
    uint64_t iterations;    /* wavefront iterations executed */
    uint64_t live_paths;    /* paths still in flight after the call */
    float ms_total;         /* device time of logic+generate+material+extend+shadow */
    float ms_shade;         /* k_shade: logic + generate + material (fused) */
    float ms_extend;        /* k_trace: extension AND any-hit rays (one fused persistent launch) */
    float ms_shadow;        /* 0: the any-hit rays are traced inside the k_trace launch */
    uint64_t ext_nodes;     /* closest-hit: child-pair nodes fetched (2 boxes each); this and the next five
                               are counted only under mcpt_set_work_counters(ctx, 1) */
    uint64_t ext_tests;     /* closest-hit: ray/triangle tests */
    uint64_t ext_hits;      /* closest-hit: rays that found a surface */
    uint64_t any_nodes, any_tests, any_hits;   /* any-hit (shadow + visibility) */
} mcpt_stage_stats;

enum { MCPT_STAGE_LOGIC = 0, MCPT_STAGE_GENERATE = 1, MCPT_STAGE_MATERIAL = 2,
       MCPT_STAGE_EXTEND = 3, MCPT_STAGE_SHADOW = 4 };

/* Path state at the shading stages' boundary, for mcpt_stage_run(LOGIC | GENERATE | MATERIAL)
 * (host SoA, n paths; SURVEY.md 8(b) per-stage parity harness).  Field meaning against the
 * reference's Paths (Wavefront.cuh:8-26):
 *   flags     bit 0 dead; bits 1..8 len (path_length); bits 9..12 the MIS conditions of the
 *             previous vertex (9 light term w > 0 && pdf > 0, 10 BRDF term, 11 f_sample == 0 or
 *             pdf_sample == 0, 12 a BRDF visibility ray was drawn: non-delta light); bits 13..31
 *             the sample index the path renders (keys its RNG draws)
 *   samples   dFilm.samples of the pixel (completed samples)
 *   hit_tri   the closest hit of `ray` (index into the uploaded scene's triangle arrays, -1 none)
 *   ray_o/_d  Paths.ray (3n each)
 *   beta      Paths.beta in xyz, (f_sample / pdf_sample).x in w (4n)
 *   nee0/1    the light-sample / BRDF-sample MIS terms f * Li * w / pdf (wavefront_kernels.cu:
 *             168-179) in xyz, (f_sample / pdf_sample).y / .z in w (4n)
 *   vis       light-sample / BRDF-sample visibility (Paths.visible; the BRDF one is the
 *             reference's inline visibility ray, :334-336) (2n)
 *   Ld        dFilm.Ld of the pixel (3n)
 *   light_o/_d, bvis_o/_d   MATERIAL out: the light-sample shadow ray (ray_light, :212-213) and the
 *             BRDF visibility ray (:334) it queued for the trace stage; NaN where none was
 *             queued (a delta light, or a ray resolved in place because it cannot hit the scene:
 *             its vis byte is then set to 1) (3n each)
 *   queued    out: bit 0 extension ray queued, bit 1 path continues into MATERIAL (LOGIC),
 *             bit 2 light ray queued, bit 3 BRDF visibility ray queued (n)
 * LOGIC (k_shade): wf_logic + wf_generate of a film of film_w x film_h pixels, path i = pixel
 * (i % film_w, i / film_w), one path per pixel, the context's camera and config.  In: flags,
 * samples, hit_tri, ray_d, beta, nee0, nee1, vis, Ld; a live path's sample index (flags bits
 * 13..31) must equal its samples, as in every state the reference or the oracle produces
 * (MCPT_E_INVALID otherwise: the device derives the count from the index).  Out: flags, samples,
 * Ld, ray_o/_d of new paths, beta (the updated throughput of continuing paths), hit_tri, queued.
 * GENERATE: LOGIC with every path dead (wf_generate for sample index `samples`).
 * MATERIAL (k_material): the light choice (:207-213) and wf_mat_mix (:295-375) of continuing path
 * i at pixel i.  In: flags (len, sample index), hit_tri, ray_o/_d, beta.  Out: flags, ray_o/_d
 * (the next extension ray), beta, nee0, nee1, hit_tri, vis, light/bvis rays, queued. */
typedef struct mcpt_path_view {
    uint32_t film_w, film_h;
    uint32_t *flags, *samples;
    int32_t *hit_tri;
    float *ray_o, *ray_d, *beta, *nee0, *nee1;
    uint8_t *vis;
    float *Ld;
    float *light_o, *light_d, *bvis_o, *bvis_d;
    uint8_t *queued;
} mcpt_path_view;

/* Caller SoA buffers for mcpt_stage_run (host memory). */
typedef struct mcpt_soa_view {
    const float *ray_o;     /* EXTEND / SHADOW in: 3*n */
    const float *ray_d;     /* EXTEND / SHADOW in: 3*n */
    float *hit_pos_t;       /* EXTEND out: 4*n pos.xyz, t */
    float *hit_nrm_mat;     /* EXTEND out: 4*n normal.xyz, (float)material (-1 miss) */
    int32_t *hit_tri;       /* EXTEND out: n triangle index or -1 */
    uint8_t *visible;       /* SHADOW out: n */
    uint32_t *steps;        /* optional out, unused since round 4 (was: per-ray node fetches + tests in diagnostics builds; left zero) */
    mcpt_path_view *paths;  /* LOGIC / GENERATE / MATERIAL: in->paths inputs, out->paths outputs */
} mcpt_soa_view;

typedef struct mcpt_ctx mcpt_ctx;     /* device context: one per GPU, not thread-safe */
typedef struct mcpt_scene mcpt_scene; /* host scene builder (Scene.cu) */

/* ---- device context (replaces wavefront_pathtrace / clear_dfilm) ---- */
int mcpt_create(int device, const mcpt_config *cfg, mcpt_ctx **out);
void mcpt_destroy(mcpt_ctx *ctx);
const char *mcpt_last_error(const mcpt_ctx *ctx);   /* ctx may be NULL: last global error */
int mcpt_scene_upload(mcpt_ctx *ctx, const mcpt_scene_desc *desc);
/* Same scene with the BVH built on the GPU instead of taken from desc (its
 * BVH arrays are ignored and may be empty); one triangle per leaf.  Hits and films are
 * identical to mcpt_scene_upload's: the traversal's result does not depend on the tree.
 * Builders (mcpt_set_gpu_bvh_builder):
 *   MCPT_GPU_BVH_PLOC (default): parallel locally-ordered clustering over Morton-sorted
 *     triangles -- surface-area agglomeration, quality close to a full SAH build;
 *   MCPT_GPU_BVH_LBVH: Karras' linear BVH (Morton-code splits; fastest build, slower trees). */
#define MCPT_GPU_BVH_LBVH 0
#define MCPT_GPU_BVH_PLOC 1
int mcpt_scene_upload_gpu_bvh(mcpt_ctx *ctx, const mcpt_scene_desc *desc);
int mcpt_set_gpu_bvh_builder(mcpt_ctx *ctx, int32_t builder);
int mcpt_camera_set(mcpt_ctx *ctx, const mcpt_camera *cam);
int mcpt_film_resize(mcpt_ctx *ctx, uint32_t w, uint32_t h, uint32_t tile_w, uint32_t tile_h);
int mcpt_film_clear(mcpt_ctx *ctx);                                          /* == clear_dfilm */
/* Paths in flight per pixel (default 1, the reference's one path per pixel,
 * wavefront_kernels.cu:108,114).  With S > 1, path slot k of a pixel renders its samples
 * k, k + S, k + 2S, ... into its own accumulator and the film readers sum the slots in
 * slot order: the same per-sample contributions, summed in another order (films agree to
 * float rounding, samples exactly).  More rays per iteration amortise each launch's ramp
 * and drain.  Re-allocates the path state, so a change CLEARS the film.  A rejected count
 * (W*H*slots >= 2^31, or out of memory) leaves the previous slot count in place. */
int mcpt_set_path_slots(mcpt_ctx *ctx, uint32_t slots);
/* Work partitions of the persistent traversal kernel (0 = device default: two per XCD, 16 on
 * MI355X; at most 64).  Each partition's rays are handed out by one counter; waves start on a
 * partition of their die and, once it is drained, join the others, so all settings trace every
 * ray and give identical results -- a tuning knob only (MCPT_TRACE_PARTS sets the default). */
int mcpt_set_trace_partitions(mcpt_ctx *ctx, uint32_t nparts);
/* Traversal work counters (mcpt_stage_stats ext_nodes / ext_tests / ext_hits / any_*): on = 1 runs
 * k_trace's counting build, off (0, the default) leaves them 0.  The counting build holds six more
 * per-lane registers, which the 64-VGPR 8-wave traversal cannot afford without spilling. */
int mcpt_set_work_counters(mcpt_ctx *ctx, int32_t on);
int mcpt_set_tiles(mcpt_ctx *ctx, const uint32_t *tile_xy, uint32_t ntiles); /* batch tile set; NULL = all */
/* Path-state layout (default 0, full: one path per pixel of the whole W x H film per slot, path id =
 * pixel id as in the reference, wavefront_kernels.cu:108,114; Film.cu:254-275 sizes the pool at
 * W x H).  on = 1, compact: the path state covers only the tile set, slots x (tiles x tile pixels)
 * paths -- a rank of a multi-GPU split that owns 1/N of the tiles holds 1/N of the state and clears
 * 1/N of it.  Results do not change (every sample is keyed by its pixel).  In the compact layout
 * mcpt_set_tiles re-allocates the path state and CLEARS the film (a tile listed twice is rejected),
 * mcpt_set_path_slots keeps the tile set, mcpt_film_resize resets it to every tile, and
 * mcpt_wavefront_step accepts only tiles of the set.  The film readers still return the W x H frame:
 * the tile set's pixels, pixels scattered in by mcpt_film_unpack_tiles / mcpt_gather, zero elsewhere.
 * A change re-allocates and clears the film. */
int mcpt_set_compact_paths(mcpt_ctx *ctx, int32_t on);
int mcpt_wavefront_step(mcpt_ctx *ctx, uint32_t tile_x, uint32_t tile_y, mcpt_stage_stats *st); /* one iteration, one tile */
int mcpt_iterate(mcpt_ctx *ctx, uint32_t iterations, mcpt_stage_stats *st);  /* batch iterations over the tile set */
int mcpt_render(mcpt_ctx *ctx, mcpt_stage_stats *st);                       /* iterate until every pixel has spp */
int mcpt_stage_run(mcpt_ctx *ctx, int stage, const mcpt_soa_view *in, mcpt_soa_view *out, uint32_t n);
int mcpt_film_read(mcpt_ctx *ctx, float *Ld_rgb, uint32_t *samples);         /* host copies, 3*W*H / W*H */
int mcpt_film_read_device(mcpt_ctx *ctx, void *d_Ld_rgb, void *d_samples);  /* device-to-device */
int mcpt_film_pack_tiles(mcpt_ctx *ctx, void *d_out, uint32_t *npix);       /* tile-set pixels -> packed 16 B/px (rgb f32, samples u32) */
/* The inverse on the gathering rank: scatter another rank's packed tile pixels (device memory on
 * ctx's GPU, 16 B/px in the order mcpt_film_pack_tiles wrote them for tiles tile_xy[0..ntiles))
 * into ctx's film accumulators.  The tiles must not be ctx's own (their other path slots would
 * be added in), and until the next film clear they cannot become ctx's own either: mcpt_set_tiles
 * rejects a set holding one (MCPT_E_INVALID; the compact layout's set_tiles clears the film
 * anyway).  Synchronous. */
int mcpt_film_unpack_tiles(mcpt_ctx *ctx, const void *d_in, const uint32_t *tile_xy, uint32_t ntiles);
int mcpt_film_tonemap_rgba8(mcpt_ctx *ctx, float exposure, uint8_t *out);   /* == draw_to_surface */
int mcpt_film_size(const mcpt_ctx *ctx, uint32_t *w, uint32_t *h);
/* Frame-end gather of a multi-GPU render in one process: the tile-set pixels of
 * every context (one per GPU, same film and tile size, tile sets disjoint from the root's) are
 * copied device-to-device over xGMI into ctxs[root]'s film, whose readers then return the whole
 * frame.  Processes with one GPU each send their mcpt_film_pack_tiles buffer to the root over
 * RCCL, which scatters it with mcpt_film_unpack_tiles (mcpt/parallel.py).  Synchronous. */
int mcpt_gather(mcpt_ctx *const *ctxs, int32_t n, int32_t root);
/* Film output (replaces stbi_write_png of the display buffer, RenderingContext.cpp:114-118):
 * PNG = tonemapped 8-bit RGB, row 0 = top; PFM = float RGB radiance Ld/samples (0 where no sample). */
int mcpt_film_write_png(mcpt_ctx *ctx, float exposure, const char *path);
int mcpt_film_write_pfm(mcpt_ctx *ctx, const char *path);
int mcpt_image_write_png(const char *path, uint32_t w, uint32_t h, const uint8_t *rgba8);
int mcpt_image_write_pfm(const char *path, uint32_t w, uint32_t h, const float *rgb);
int mcpt_sync(mcpt_ctx *ctx);
int mcpt_device_name(mcpt_ctx *ctx, char *buf, int32_t len);
/* diagnostics: rays of the current extension (which=0) or any-hit (which=1) queue, and the
 * device time of the last mcpt_stage_run kernel. */
int mcpt_debug_queue_rays(mcpt_ctx *ctx, int which, float *ray_o, float *ray_d, uint32_t *n_inout);
float mcpt_debug_last_stage_ms(const mcpt_ctx *ctx);
/* Tests: on = 1 runs the traversal with a 2-entry LDS stack per lane (deeper entries in scratch)
 * instead of the 8 / 10 entries the tree depth selects, so that the scratch path is exercised on
 * every tree.  Same results, slower. */
int mcpt_debug_tiny_lds_stack(mcpt_ctx *ctx, int32_t on);
float mcpt_debug_last_build_ms(const mcpt_ctx *ctx);  /* device time of the last GPU BVH build */
/* HRDI tables: an upload whose desc has env_tex but no env_marginal_y / env_conds_y / env_pdf builds
 * them on the device (build_environment_light, light_initialization_kernels.cu:3-161; bit-identical to
 * the host build).  Device time of the last such build, and a copy of the uploaded scene's device
 * tables (any output may be NULL; *flags bit 0 = built on the device, bit 1 = env_cell search guides on). */
float mcpt_debug_last_env_build_ms(const mcpt_ctx *ctx);
int mcpt_debug_env_tables(mcpt_ctx *ctx, float *marginal_y, float *conds_y, float *pdf, int32_t *flags);
/* pair-node numbering of the last uploaded tree: 0 depth-first, 1 depth-first by sibling pairs,
 * 2 breadth-first, 3 line pairs (a node and its larger-area child per 128-B line, pad nodes where a
 * node has no interior child; opt-in) (default 2 for trees of <= 2 MiB of nodes, else 0;
 * MCPT_SIBLING_LAYOUT=0/1/2/3 at upload forces one; inputs that are not a tree -- a shared child --
 * always get 0). */
int mcpt_debug_node_layout(const mcpt_ctx *ctx);
/* any-hit occluder cache: any-hit rays resolved by it since the film was
 * last cleared (counted in shadow_rays / vis_rays as traced rays; they skip the traversal), and
 * whether the uploaded scene has the cache (MCPT_OCC_G=0 at upload turns it off). */
int mcpt_debug_occ_stats(const mcpt_ctx *ctx, uint64_t *resolved, int32_t *enabled);
/* Ray counts since the last film clear (5 values): extension rays, of them traversed by k_trace
 * (the rest: NaN / zero directions and root-box misses resolved where the ray was made), any-hit
 * (shadow + BRDF visibility) rays, of them traversed, and of them resolved by the occluder cache. */
int mcpt_debug_ray_counts(const mcpt_ctx *ctx, uint64_t *out);
/* The traversal's loop-phase counts, recorded by the counting build (mcpt_set_work_counters on)
 * since the last film clear or reset (reset = 1 starts a new count after reading): out12[0] loop
 * trips, [1] refills, [2] lanes refilled, [3] node-phase wave iterations, [4] triangle phases,
 * [5] lanes testing a triangle in them, [6] / [7] / [8] lanes with node work / a parked leaf / no
 * ray at a trip's start, [9] trips in which a lane finished its ray, [10] node-phase iterations in
 * which a lane popped its stack; [11] 0.  With the node steps of mcpt_stage_stats they split the
 * lane utilisation by phase, and with the kernel's ISA sections its VALU (tools/trace_attrib.py).
 * Returns the number of words filled (11), 0 when none were recorded. */
int mcpt_debug_trace_profile(mcpt_ctx *ctx, uint64_t *out12, int reset);
/* k_shade's per-section wave entries and active lanes, summed over the
 * launches since the last reset, in a build with -DMCPT_DIAG_SHADE: out[2k] entries and out[2k+1]
 * lanes of section k (waves, valid paths, logic, MIS terms, generate, continuing, background), up to
 * n words.  Returns the words available (14); the product build fills zeros and returns 0. */
int mcpt_debug_shade_sections(mcpt_ctx *ctx, uint64_t *out, int n, int reset);
/* diagnostics: the kernels' shared-denominator division (mcpt::quot3, mcpt_core.hpp) on the
 * device for n host pairs: out[i] = a[i] / b[i] as the kernels compute it (must equal IEEE fp32). */
int mcpt_debug_quot(mcpt_ctx *ctx, const float *a, const float *b, uint32_t n, float *out);
/* Measured HBM ceiling for the roofline: a hand-written dwordx4 copy of `bytes`
 * between two device buffers, `iters` launches timed with HIP events; *gbps = (read + write) bytes / s. */
int mcpt_debug_hbm_copy(mcpt_ctx *ctx, uint64_t bytes, uint32_t iters, double *gbps);

/* ---- host scene builder (Scene.cu:24-470, EnvironmentLight.cu:329-452, BVH.cu) ---- */
mcpt_scene *mcpt_scene_new(void);
void mcpt_scene_free(mcpt_scene *s);
int mcpt_scene_load_glb(mcpt_scene *s, const char *path, const float *xform16);  /* xform may be NULL */
int mcpt_scene_add_mesh(mcpt_scene *s, int32_t ntri, const float *v0, const float *v1, const float *v2,
                        const float *n0, const float *n1, const float *n2, const float *base_rgb);
int mcpt_scene_set_env_hdr(mcpt_scene *s, const char *path, int32_t mode);
/* flags MCPT_ENV_DEVICE_TABLES: keep the texture only; mcpt_scene_upload then builds the tables on
 * the device (for large maps: the host build is several serial passes over every texel). */
#define MCPT_ENV_DEVICE_TABLES 1
int mcpt_scene_set_env_hdr_ex(mcpt_scene *s, const char *path, int32_t mode, uint32_t flags);
int mcpt_scene_set_env_color(mcpt_scene *s, const float *rgb, float ls);
int mcpt_scene_add_dir_light(mcpt_scene *s, const float *dir, const float *rgb, float ls);
int mcpt_scene_transform(mcpt_scene *s, const float *xform16);   /* bake a transform into all meshes */
int mcpt_scene_make_proxy(mcpt_scene *s, int32_t config_id, const char *asset_dir); /* SURVEY.md 8d proxies */
int mcpt_scene_build(mcpt_scene *s, int32_t max_prims_in_node);  /* SAH BVH (BVH.cu:84-333) + env tables */
/* BVH builder choice.  Topology is not a parity contract (hits are tree-independent: conservative
 * culling + (t, scene index) ties), so any builder gives identical films.
 *   MCPT_BVH_REFERENCE: BVHAccel's SAH (BVH.cu:84-333) -- 12 buckets on the largest centroid axis,
 *     cost .125 + (n0 A0 + n1 A1) / A; what mcpt_scene_build runs.
 *   MCPT_BVH_SAH3: binned SAH over all three axes (buckets per axis), cost
 *     trav_cost + isect_cost (n0 A0 + n1 A1) / A against a leaf cost isect_cost n. */
#define MCPT_BVH_REFERENCE 0
#define MCPT_BVH_SAH3 1
typedef struct mcpt_bvh_params {
    int32_t builder;      /* MCPT_BVH_* */
    int32_t max_prims;    /* 1..8 triangles per leaf */
    int32_t buckets;      /* SAH3: bins per axis (2..256) */
    float trav_cost;      /* SAH3: cost of a node visit, relative to ... */
    float isect_cost;     /* ... a triangle test */
} mcpt_bvh_params;
int mcpt_scene_build_ex(mcpt_scene *s, const mcpt_bvh_params *p); /* BVH + env tables */
int mcpt_scene_get_desc(const mcpt_scene *s, mcpt_scene_desc *out); /* pointers owned by s */
int mcpt_scene_bvh_depth(const mcpt_scene *s);
int mcpt_camera_make(const mcpt_camera_params *p, mcpt_camera *out);

#ifdef __cplusplus
}
#endif
#endif
