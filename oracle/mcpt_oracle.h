/*
 * mcpt_oracle.h -- CPU restatement of the MC-Path-Tracer wavefront hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (mc-path-tracer_amd/) may
 * include, link or call this.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py load liboracle.so, and only as the checker.
 *
 * Parity status: PARTIALLY PINNED.  The reference (CUDA 11.8 / MSVC / OpenGL)
 * cannot be compiled or run in this image, and it ships
 * no tests or golden vectors.  The restatement is pinned by:
 *   - the reference's only self-check, sum(env pdf) ~= 1
 *     (light_initialization_kernels.cu:113-133),
 *   - the README BRDF formulas (README.md:74-124) as known-answer tests,
 *   - independent re-derivations in tests/ (numpy lowerbias32/splitmix64,
 *     glibc transcendentals within a stated ULP bound, brute-force ray casts).
 * Third-party arithmetic the reference delegates (CUDA texture filtering,
 * stb_image, glm, CUDA fast-math transcendentals) is restated and UNPINNED.
 *
 * Every function cites the reference file:line it restates, relative to
 * /root/reference/CUDA-RayTracer/ (cuda_math/ for the math core).
 */
#ifndef MCPT_ORACLE_H
#define MCPT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Scene arrays (already BVH-ordered).  Triangles are in world space: the
 * reference bakes node transforms into vertices (Scene.cu:224) and keeps an
 * identity dTransform, so Triangle.cu:69/82/86 transforms are exact no-ops. */
typedef struct or_scene {
    int32_t ntri;
    const float *v0, *v1, *v2;      /* 3*ntri positions                   */
    const float *n0, *n1, *n2;      /* 3*ntri vertex normals              */
    const int32_t *mat;             /* ntri material id                   */
    int32_t nnodes;                 /* LinearBVHNode (BVH.h:63-72)        */
    const float *bmin, *bmax;       /* 3*nnodes                           */
    const int32_t *offset;          /* primitivesOffset / secondChildOffset */
    const int32_t *nprims;          /* 0 => interior                      */
    const int32_t *axis;
    int32_t nmat;
    const float *mat_params;        /* nmat*8: base rgb, fresnel rgb, roughness, metallic */
    int32_t ndir;                   /* directional lights after the env light */
    const float *dir_params;        /* ndir*7: dir xyz, color rgb, ls     */
    int32_t env_mode;               /* 0 = Color, 1 = HRDI (EnvironmentLight.h:11-15) */
    float env_color[3];
    float env_ls;
    int32_t env_w, env_h;
    const float *env_tex;           /* env_h*env_w*4 RGBA32F, row 0 = top */
    const float *env_marginal_y;    /* env_h                              */
    const float *env_conds_y;       /* env_h*env_w                        */
    const float *env_pdf;           /* env_h*env_w                        */
    const int32_t *tri_id;          /* optional ntri triangle ids (tie key, reported id); NULL = index */
} or_scene;

typedef struct or_camera {
    float inv_view_proj[16];        /* column-major m[c][r] = m[c*4+r] (Matrix.h:12-95) */
    float inv_view[16];
    float lens_radius;
    float focal;
} or_camera;

typedef struct or_config {
    uint64_t seed;
    int32_t spp;          /* gates processing and new samples (wavefront_kernels.cu:124,219) */
    int32_t max_depth;    /* 'path_length > 5' (wavefront_kernels.cu:142,148) */
    int32_t rr_depth;     /* 'path_length > 3' (wavefront_kernels.cu:189)      */
    int32_t tile_w, tile_h;
    int32_t nthreads;
    int32_t traversal;    /* 0 = reference stack traversal, 1 = brute force, 2 = stack traversal with
                             the literal reference leaf rule (no own-box check, first visited wins) */
    int32_t row_begin, row_end;  /* restrict to rows [begin,end); 0,0 = all */
    int32_t fixed;        /* 1 = quality mode (product MCPT_FLAG_FIXED) */
    int32_t tile_mod, tile_rank;  /* tile_mod > 0: only tiles with (tx+ty) % tile_mod == tile_rank
                                     (one rank's share of the multi-GPU partition) */
} or_config;

/* counters[0]=extension rays, [1]=shadow rays, [2]=BRDF visibility rays,
 * [3]=wavefront iterations (summed over tiles), [4]=BVH nodes visited,
 * [5]=triangle tests. */
int or_render(const or_scene *sc, const or_camera *cam, const or_config *cfg,
              int32_t W, int32_t H, float *Ld, uint32_t *samples, uint64_t *counters);

/* Batch ray casts (Triangle.cu:144-203 / 204-243).  hit_f4 per ray:
 * pos.xyz, t ; nrm_f4: normal.xyz, (float)mat (mat=-1 on miss); tri: index or -1 */
void or_trace_closest(const or_scene *sc, int32_t n, const float *ro, const float *rd,
                      int32_t traversal, float *pos_t, float *nrm_mat, int32_t *tri);
void or_trace_any(const or_scene *sc, int32_t n, const float *ro, const float *rd,
                  int32_t traversal, uint8_t *visible);

/* Env tables (light_initialization_kernels.cu:3-112). out_pdf_denom may be NULL. */
void or_env_build(int32_t W, int32_t H, const float *tex, float *marginal_y,
                  float *marginal_p, float *conds_y, float *pdf, float *out_pdf_denom);

/* Known-answer hooks. */
float or_sinf(float x);
float or_cosf(float x);
float or_asinf(float x);
float or_acosf(float x);
float or_atan2f(float y, float x);
uint32_t or_lowerbias32(uint32_t x);
uint64_t or_splitmix64(uint64_t z);
float or_rand(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t len, uint32_t slot);
void or_env_fetch(const or_scene *sc, float u, float v, float *rgb);
float or_env_pdf(const or_scene *sc, float dx, float dy, float dz);
void or_env_dir(const or_scene *sc, float ex, float ey, float *wi);
/* BRDF hooks: params = base rgb, fresnel rgb, roughness, metallic.
 * out: f_spec rgb, f_diff rgb, pdf_spec, pdf_diff. */
void or_brdf_eval(const float *params, const float *n, const float *wi, const float *wo, float *out);
float or_power_heuristic(float f, float g);
int32_t or_upper_bound(const float *list, int32_t size, float val);
/* Per-stage restatements at the product's shading-stage boundary (include/mcpt.h mcpt_path_view;
 * SURVEY.md section 4 item 2): the same logic_core / mis_terms / pick_light / mat_mix_core the
 * full render runs.  Arrays are host SoA over n paths, path i = pixel i.
 * or_stage_logic: wf_logic + wf_generate (wavefront_kernels.cu:90-251) of a W x H film (n = W*H),
 *   one path per pixel.  In: flags, samples, hit_tri, ray_d (3n), beta/nee0/nee1 (4n), vis (2n),
 *   Ld (3n).  Out (may alias the inputs): flags, samples, Ld, ray_o/ray_d of generated paths,
 *   beta (xyz updated for continuing paths), queued (bit 1: continues into the material stage).
 * or_stage_material: the light choice (:207-213) + wf_mat_mix (:295-375) of continuing paths.
 *   In: flags (len, sample index), hit_tri, ray_o/ray_d, beta.  Out: flags, ray_o/ray_d (next
 *   extension ray), beta (xyz, ratio.x), nee0/nee1 (4n), light_o/light_d and bvis_o/bvis_d
 *   (3n; NaN for a delta light's absent visibility ray). */
void or_stage_logic(const or_scene *sc, const or_camera *cam, const or_config *cfg, int32_t W, int32_t H,
                    uint32_t *flags, uint32_t *samples, const int32_t *hit_tri, float *ray_o, float *ray_d,
                    float *beta, const float *nee0, const float *nee1, const uint8_t *vis, float *Ld,
                    uint8_t *queued);
void or_stage_material(const or_scene *sc, const or_config *cfg, int32_t n, uint32_t *flags, const int32_t *hit_tri,
                       float *ray_o, float *ray_d, float *beta, float *nee0, float *nee1, float *light_o,
                       float *light_d, float *bvis_o, float *bvis_d);
void or_gen_ray(const or_camera *cam, int32_t W, int32_t H, int32_t x, int32_t y,
                uint64_t seed, uint32_t pixel, uint32_t sample, float *o, float *d);
const char *or_version(void);

/* trav_model.c (test infrastructure): a model of the product traversal's box culling, checked
 * against or_trace_closest / or_trace_any on adversarial rays (tests/test_cull_model.py).
 * or_model_margins: per desc node and per triangle own-box margins and the far coefficient P;
 * returns 0 when a node box does not contain its subtree's vertices.  or_model_trace: mode 0
 * culls nothing, 1 the round-3 rule, 2 the round-4 rule; tri = closest triangle id or -1,
 * t = its t, visible = any-hit result; *nodes = boxes tested. */
int32_t or_model_margins(const or_scene *sc, float *node_w, float *tri_w, float *p);
void or_model_set_safe(double c); /* modes 6 / 7: margins and planes (0: the product's) */
uint64_t or_model_tri_tests(void); /* triangle tests of the last or_model_trace call */
void or_model_trace(const or_scene *sc, int32_t n, const float *ro, const float *rd, int32_t mode,
                    const float *node_w, const float *tri_w, float p, int32_t *tri, float *t, uint8_t *visible,
                    uint64_t *nodes);
/* traversal study (trav_model.c): per-ray steps / origin-box steps / triangle tests / outcome and
 * the 128-B lines fetched under a node numbering; or_lru_sim: LRU misses over those line streams */
void or_model_study(const or_scene *sc, int32_t n, const float *ro, const float *rd, int32_t mode, int32_t kind,
                    const float *node_w, const float *tri_w, float p, const int32_t *pair_line, int32_t tri_line0,
                    int32_t *steps, int32_t *origin_steps, int32_t *tris, uint8_t *hit, int32_t *lines, int64_t cap,
                    int64_t *off);
void or_model_set_any_order(int32_t m); /* study: any-hit visiting order (0 near-first) */
int64_t or_lru_sim(const int32_t *lines, const int64_t *off, int32_t n, int32_t batch, int32_t sets, int32_t ways);

#ifdef __cplusplus
}
#endif

#endif
