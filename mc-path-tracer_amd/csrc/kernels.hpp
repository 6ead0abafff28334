// kernels.hpp -- device data layout shared by kernels.hip and runtime.hip.
//
// HBM layout (P = slots * W*H paths; slot 0 is the reference's one path per pixel, path_id ==
// pixel_id, wavefront_kernels.cu:108,114).  The reference's Paths is an array-of-structs with a
// 128-B Isect and a 32-B dRay per path (Wavefront.cuh:8-26); here every field is a separate
// 16-B-aligned stream so a wave64 access is one coalesced 1 KiB dwordx4 transaction.  (Records
// that pack a path's fields together -- 32-B rays, 64-B {beta, nee0, nee1, Ld} -- move fewer HBM
// bytes on the sparse accesses but cost more lines per wave instruction, and measured slower:
// k_material 248 -> 302 ms, k_shade 139 -> 193 ms per three config-2 frames)
//   ray_o/ray_d   float4 [P]    extension ray (xyz, pad)
//   hit_tri       i32    [P]    closest triangle of the extension ray (-1 = miss); the hit
//                               record (isect) is rebuilt from it where it is consumed
//   sray_o/sray_d float4 [2Q]   any-hit rays at their any-queue position (Q = queue entries,
//                               allocated with the queues): written densely by k_material after
//                               its block push, read densely by k_trace; the queue entry itself
//                               holds the result index 2p (light sample) / 2p+1 (BRDF visibility).
//   beta          float4 [P]    throughput, (f_sample/pdf_sample).x
//   nee0 / nee1   float4 [P]    precomputed light / BRDF MIS terms, ratio .y / .z
//   flags         u32    [P]    dead, len, MIS condition bits, the path's sample index (bits 13..31)
//   vis           u8     [2P]   any-hit results
//   samples       u32    [P]    film sample count (dFilm.samples)
//   Ld            float4 [P]    film radiance (dFilm.Ld)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device/mcpt_core.hpp"

namespace mcpt_dev {

constexpr int kBlock = 256;
constexpr int kTraceBlock = 64;  // one wave per traversal block
#ifndef MCPT_LDS_STACK
#define MCPT_LDS_STACK 8
#endif
constexpr int kLdsStack = MCPT_LDS_STACK;  // traversal stack entries per lane kept in LDS (deeper: scratch)
#ifndef MCPT_LDS_STACK_DEEP
#define MCPT_LDS_STACK_DEEP 10
#endif
constexpr int kLdsStackDeep = MCPT_LDS_STACK_DEEP;  // the same for trees deeper than kDeepTree levels
constexpr int kLdsStackTiny = 2;  // test instantiation (mcpt_debug_tiny_lds_stack): pushes beyond 2 go to scratch
#ifndef MCPT_DEEP_TREE
#define MCPT_DEEP_TREE 20
#endif
constexpr int kDeepTree = MCPT_DEEP_TREE;  // stack pushes beyond which the deep-stack k_trace runs
constexpr int kMaxStack = 64;  // total (reference: int nodesToVisit[64], Triangle.cu:161)

enum : uint32_t {
    F_DEAD = 1u,
    F_LEN_SHIFT = 1,        // bits 1..8
    F_CONDL = 1u << 9,      // light-sample MIS term valid (w > 0 && pdf > 0)
    F_CONDB = 1u << 10,     // BRDF-sample MIS term valid when visible
    F_FZERO = 1u << 11,     // f_sample == 0 || pdf_sample == 0
    F_HASVIS = 1u << 12,    // non-delta light: a BRDF visibility ray was traced
    F_SIDX_SHIFT = 13       // bits 13..31: the sample index the path renders (RNG key); a dead
                            // path's next one (k_shade derives the film's sample count from it)
};
constexpr uint32_t kMaxSpp = 1u << (32 - F_SIDX_SHIFT);  // sample indices must fit the flags word
constexpr int kRecLenShift = 24;  // material record word 2: sample index (< kMaxSpp) | len << 24 (len < 256)
static_assert(kMaxSpp <= (1u << kRecLenShift), "sample index and len share a record word");

// k_shade blocks: kBlock consecutive pixels of one path slot; slot k's blocks follow slot k-1's
__host__ __device__ constexpr int shade_blocks_per_tile(int tile_px, int slots) {
    return (tile_px + kBlock - 1) / kBlock * slots;
}

// BVH node width of the traversal, per scene (DevScene::width): width 2, child-pair
// nodes, 4 x float4 (per axis (mn0, mn1, mx0, mx1), then refs); width 4, 8 x float4:
// mn.x[4], mx.x[4], mn.y[4], mx.y[4], mn.z[4], mx.z[4], refs[4] (kEnd = empty), pad.
// float4 per triangle intersection record: 3 (48 B, packed) or 4 (64 B: a record never
// straddles two 64-B halves of a cache line; MCPT_TRI_F4)
#ifndef MCPT_TRI_F4
#define MCPT_TRI_F4 3
#endif
constexpr int kTriF4 = MCPT_TRI_F4;

struct DevScene {
    const float4* nodes;    // BVH nodes (width children each: 4 or 8 float4)
    const float4* tri;      // kTriF4 x float4: (v0.xyz, e1.x) (e1.yz, e2.xy) (e2.z, id, -, -) [pad]; id = tri_id bits
    const float4* tri_sh;   // 3 x float4: (n0.xyz, n1.x) (n1.yz, n2.xy) (n2.z, mat, -, -)
    float root_mn[3], root_mx[3];
    int root_ref;           // >= 0 pair node, < 0 leaf (0x80000000 | (count-1)<<24 | offset)
    int depth;              // bound on stack pushes of the uploaded tree: picks the k_trace instantiation
    int width;              // node width: 2 (child pairs) or 4 (quads)
    int nlights;            // 1 + ndir (Scene.cu:370-388)
    const float* mats;      // 8 floats per material
    const float* dirs;      // 7 floats per directional light
    mcpt::EnvView env;
    // Any-hit occluder cache: occ[kOccWays i + w] is a triangle record
    // that occluded an any-hit ray of cell i (origin cell of the root box x direction bin), or
    // kOccEmpty; occ_rec[kOccRecF4 t ..] is triangle t's occluder record: the box of the BVH leaf
    // that holds it with that leaf's culling margin, and the triangle (v0, e1, e2), 64 B.
    // k_material tests an any-hit ray against its cell's triangle under that leaf box first:
    // a hit there is one the traversal would find too, so the ray is resolved as occluded.
    // occ == nullptr: off.
    uint32_t* occ;
    // The lookup gate, kOccGateWords words kept with the table (all reset at upload and with the film): [0] skip: k_material skips the lookups while nonzero; k_accumulate
    // sets it to [1] after an iteration whose lookups resolved under 1 in kOccMinRate of the rays
    // tested and counts it down one per iteration; k_trace records occluders only while it is <= 1,
    // so the next lookups meet a fresh table.  [1] backoff: 15, 31, 63, ... 255 after consecutive
    // failed lookup iterations, 0 while they pay.  [2] warm: set by the first iteration that traced
    // any-hit rays (and so recorded occluders into the table the film clear emptied); k_material
    // looks nothing up before it.  (Round 6: the lookups against the empty table used to be judged,
    // which closed the gate for the frame's biggest iterations, 2-4 -- at N = 8 most of a rank's
    // frame.)
    uint32_t* occ_gate;
    const float4* occ_rec;
    uint32_t ntri;
    int occ_g, occ_b;       // origin cells per axis, direction bins per face coordinate
    float occ_inv[3];       // occ_g / root box extent, per axis
    // Conservative culling (mcpt_core.hpp "conservative box culling"): every node holds each
    // child's margin W (pair nodes: q3.z / q3.w; 4-wide nodes: float4 7; occ_rec[4t].w), P is the
    // scene's far coefficient, root_w the root box's margin.  cull_ok = 0 (a caller BVH whose boxes
    // do not contain their triangles, or MCPT_CULL=0): nothing is culled.
    float cull_p, root_w;
    int cull_ok;
};
constexpr uint32_t kOccEmpty = 0xffffffffu;
constexpr uint32_t kOccWays = 2;      // entries per cell: k_trace writes way tri mod 2, k_material tests both
                                      // (1 way resolved 52 % of config 2's any-hit rays, 2 ways 64 %)
constexpr uint32_t kOccGateWords = 3;  // DevScene::occ_gate
constexpr uint32_t kOccMinRate = 10;  // lookups pay when >= 1 in kOccMinRate resolves a ray (see occ_skip)
__host__ __device__ constexpr size_t occ_entries(int g, int b) { return (size_t)g * g * g * 6 * b * b * kOccWays; }

struct DevPaths {
    float4 *ray_o, *ray_d, *sray_o, *sray_d, *beta, *nee0, *nee1, *Ld;
    int32_t* hit_tri;  // closest hit of the extension ray (-1: none); k_shade rebuilds the hit record
    uint32_t *flags, *samples;
    uint8_t* vis;
};

// Queue counters and statistics are sharded over kShards cache lines (one
// shard per k_shade block mod kShards): a single counter word serialises at
// roughly 90 atomics per microsecond, which is what ~24K pushes and ~100K
// statistics adds per iteration would otherwise cost.
constexpr int kShards = 64;
constexpr int kMaxParts = kShards;  // k_trace work partitions (at most one per queue shard)
enum : int { C_EXT = 0, C_ANY = 1, C_VIS = 2, C_STATS = 3, C_EXT_RAYS = 9, C_ANY_RAYS = 10, C_MAT = 11, C_OCC = 12,
              C_OCC_TRY = 13, C_PH = 14, C_WORDS = 32 };  // C_STATS..+5; C_OCC / C_OCC_TRY: any-hit rays resolved by /
                                                          // tested against the occluder cache; C_PH..+kPhaseWords-1:
                                                          // k_trace's loop-phase counts (counting build, PH_*)
// k_trace loop-phase counts of the counting instantiation (mcpt_debug_trace_profile), per wave summed:
enum : int {
    PH_TRIPS = 0,          // loop trips with a ray in the wave
    PH_REFILLS = 1,        // refill events
    PH_REFILL_LANES = 2,   // lanes handed a ray by them
    PH_NODE_ITERS = 3,     // node-phase wave iterations (per trip: the most steps any lane took, <= kNodeSteps)
    PH_TRI_PHASES = 4,     // triangle phases run
    PH_TRI_LANES = 5,      // lanes that tested a triangle in them
    PH_TRIP_NODE = 6,      // lanes with node work at a trip's start
    PH_TRIP_LEAF = 7,      // lanes holding a parked leaf at a trip's start
    PH_TRIP_IDLE = 8,      // lanes without a ray at a trip's start (after the refill)
    PH_FINISH_TRIPS = 9,   // trips in which at least one lane finished its ray
    PH_POP_ITERS = 10,     // node-phase wave iterations in which at least one lane popped the stack
    kPhaseWords = 11
};
struct CounterBlock {
    uint32_t shard[kShards][C_WORDS];  // [0] ext pushes [1] any-hit pushes [2] vis rays [3..8] traversal stats [9,10] rays [11] material pushes
    uint32_t last_ext, last_live;
    uint32_t trace_short;  // k_trace launches that left a partition's rays untraced (k_accumulate; must stay 0)
    uint32_t idle;         // set by k_accumulate after an iteration with no ray: the tile set is complete, so
                           // the remaining iterations of the call skip their kernels (run_iterations resets it)
    uint32_t pad[28];
    uint32_t last_ext_shard[kShards];  // per-shard extension pushes of the last iteration
    uint32_t grab[kMaxParts][C_WORDS];  // k_trace ray hand-out, one counter line per partition
    unsigned long long tot_ext, tot_any, tot_vis, tot_occ;
    unsigned long long tot_stats[6];
    unsigned long long tot_ext_q, tot_any_q;  // rays queued to k_trace (the rest were resolved in place)
    unsigned long long tot_phase[kPhaseWords];  // k_trace loop-phase counts (PH_*; counting build only)
};

struct ShadeArgs {
    DevScene scene;
    mcpt::CamView cam;
    DevPaths p;
    const int2* tiles;
    int ntiles, tile_w, tile_h, W, H;
    int spp, max_depth, rr_depth;
    int slots;  // path slots per pixel (paths in flight per pixel; slot k runs samples k, k + slots, ...)
    float slots_rcp;  // RN32(1 / slots) (k_shade's udiv_small)
    // Path index of a pixel: slot * npx + its index within the slot.  Full layout (compact 0): npx =
    // W * H and the index is the pixel id (the reference's path_id = pixel_id, wavefront_kernels.cu:
    // 108,114).  Compact layout (mcpt_set_compact_paths): the path state covers only the context's tile
    // set, npx = tile-set tiles * tile pixels and the index is set_tile * tile_w * tile_h + the pixel's
    // index in its tile, where set_tile = tile_base[t] for launch tile t (nullptr: t itself, the launch
    // runs the whole set in its order).
    uint32_t npx;
    int compact;
    const int* tile_base;
    uint64_t seed;
    uint32_t *ext_q, *any_q;
    // material queue (continuing paths, k_shade -> k_material, ext_cap per shard): dense records
    // {pid, pixel, sample index | len << kRecLenShift, hit_tri} + the updated throughput, so
    // k_material reads its per-path inputs from k_shade's coalesced loads instead of gathering them
    // again at pid (the pixel keys its RNG draws: the path index need not be the pixel id)
    uint4* mat_rec;
    float4* mat_beta;
    uint32_t ext_cap, any_cap;  // per-shard queue capacity
    CounterBlock* cnt;
    // k_shade block done flags, per (slot, film tile, block of the tile): set once every path of
    // the block is dead with its last sample finished, so later launches skip the block's loads
    // (cleared with the film; nullptr: off)
    uint8_t* blk_done;
    uint32_t shade_vblocks;  // k_shade: shading blocks of the launch (launch_shade sets it and the grid)
    // Per-pixel camera records of the W x H film (k_cam_table; gen_ray_pixel of every pixel): the
    // pixel's focal point (thin lens) or pinhole origin in cam_px, the pinhole direction in cam_dir
    const float4* cam_px;
    const float4* cam_dir;
};

// One ray set of a trace launch: rays ro/rd[rid] for queue entries
// queue[s * shard_cap + k], k < count of shard s.
struct TraceSet {
    const float4 *ro, *rd;
    const uint32_t* queue;      // nullptr => identity
    const uint32_t* count_ptr;  // device count of shard s at count_ptr[s * C_WORDS] (nullptr => count)
    uint32_t count;
    uint32_t shard_cap;         // queue entries per shard
    uint32_t* stats;            // optional: shard s counters at stats[s * C_WORDS + 0..2] (nodes, tests, hits)
    uint32_t* ray_steps;        // optional per-queue-entry node fetches + triangle tests (diagnostics)
    int prefiltered;            // 1: every ray has a valid direction and enters the root box (k_shade checked)
    int ray_at_slot;            // 1: the ray of queue position k is ro/rd[k] (dense); queue[k] is only the
                                //    result index.  0: the ray is ro/rd[queue[k]]
};
struct TraceArgs {
    DevScene scene;
    TraceSet set[2];            // [0] closest hit -> hit_tri, [1] any hit -> vis
    int nshards;
    int32_t* hit_tri;           // closest-hit output: triangle index or -1
    uint8_t* vis;               // any-hit output: 1 = unoccluded
    uint32_t refill_min;        // refill when at least this many lanes are idle (set by launch_trace)
    uint32_t tri_min;           // run the triangle phase when this many lanes hold a leaf (set by launch_trace)
    uint32_t nparts;            // work partitions (default: the device's XCDs; set by launch_trace)
    uint32_t ndies;             // XCDs of the device (set by launch_trace)
    uint32_t* grab;             // nparts chunk counters, C_WORDS apart, zero at launch (k_accumulate resets)
    const uint32_t* idle;       // optional: nonzero = the tile set is complete, exit at once (CounterBlock::idle)
    int tiny_stack;             // host side: launch the kLdsStackTiny instantiation (mcpt_debug_tiny_lds_stack)
    uint32_t* phase;            // counting build: loop-phase counts of shard s at phase[s * C_WORDS + PH_*] (or nullptr)
};

struct HitRecordArgs { DevScene scene; const float4 *ro, *rd; const int32_t* tri; float4 *hit_p, *hit_n; int32_t* scene_tri; uint32_t n; };
struct ClearArgs { uint32_t* flags; uint32_t* samples; float4* Ld; uint32_t n, npx; };  // n = npx * slots
// n accumulators per slot.  tiles == nullptr: n = W * H pixels in pixel order (full layout); else the
// compact layout's order (tile-set tile i's pixels at i * tile_w * tile_h, row by row), scattered to
// out[y * W + x] for the pixels inside the W x H film
struct ResolveArgs {
    const float4* Ld; const uint32_t* samples; float4* out_Ld; uint32_t* out_samples; uint32_t n; int slots;
    const int2* tiles; int tile_w, tile_h, W, H;
};
struct TonemapArgs { const float4* Ld; const uint32_t* samples; uchar4* out; float exposure; uint32_t n; };
struct PackArgs { const float4* Ld; const uint32_t* samples; const int2* tiles; int ntiles, tile_w, tile_h, W, H; float4* out; };
struct UnpackArgs { const float4* in; const int2* tiles; int ntiles, tile_w, tile_h, W, H; float4* Ld; uint32_t* samples; };

// Launch geometry of one device (mcpt_create): persistent grids from the occupancy
// calculator and the device's XCD count, with environment overrides for sweeps.
struct LaunchGeom {
    uint32_t trace_waves[2][2];  // k_trace grid (waves) per [node width 2/4][LDS stack normal/deep];
                                 // at most 28 waves per CU (MCPT_TRACE_WAVES overrides)
    uint32_t trace_parts;    // k_trace work partitions, MCPT_TRACE_PARTS (1..kMaxParts)
    uint32_t ndies;          // XCDs
    uint32_t mat_blocks[2];  // k_material grid [reference mode, fixed mode]
    uint32_t shade_grid;     // k_shade grid cap (resident blocks x MCPT_SHADE_GRID; 0: one block per shading block)
    uint32_t refill_min, tri_min;  // MCPT_REFILL_MIN, MCPT_TRI_MIN
};
int launch_geometry(int device, LaunchGeom& g);  // device must be current
void launch_shade(const ShadeArgs& a, int nblocks, const LaunchGeom& g, bool fixed_mode, hipStream_t s);
void launch_shade_stage(bool material_stage, const ShadeArgs& a, int nblocks, const LaunchGeom& g, bool fixed_mode,
                        hipStream_t s);
void launch_trace(const TraceArgs& a, const LaunchGeom& g, hipStream_t s);
void launch_clear(const ClearArgs& a, hipStream_t s);
// Occluder records (DevScene::occ_rec): for each triangle record t, {leaf mn, margin} {leaf mx,
// v0.x} {v0.yz, e1.xy} {e1.z, e2} of the leaf that holds it (nodes: nnodes nodes of the given
// width; a root that is itself a leaf gets the root box)
constexpr int kOccRecF4 = 4;
void launch_occ_records(const DevScene& sc, uint32_t nnodes, float4* rec, hipStream_t s);
void launch_occ_probes(const DevScene& sc, float4* ro, float4* rd, uint32_t nkeys, hipStream_t s);
// Culling margins of a child-pair tree (mcpt_core.hpp cull_*): tri_w[t] = W'_T of record t,
// *pmax = the far coefficient P's bits (max), then `passes` bottom-up passes writing every
// child's subtree maximum into q3.z / q3.w (passes >= tree depth + 1 reach the fixed point).
// plane: the axis-plane bound (cull_plane_b) where it applies (false: the general bound only).
void launch_cull_margins(float4* nodes, uint32_t npairs, const float4* tri, uint32_t ntri, float* tri_w,
                         uint32_t* pmax, int passes, bool plane, hipStream_t s);
// tex[i].w = pdf[i], i < n (EnvView::tex: the pdf in the texture's alpha plane)
void launch_env_pack(float4* tex, const float* pdf, size_t n, hipStream_t s);
void launch_env_table(const mcpt::EnvView& e, bool fixed_mode, float4* out, float2* row, float2* col, hipStream_t s);
// HRDI tables on the device (env_build.hip), bit-identical to the host build: scratch holds
// env_build_scratch_floats(W, H) floats; W * H < 2^31.
size_t env_build_scratch_floats(int W, int H);
void launch_env_build(const float4* tex, int W, int H, float* scratch, float* marginal_y, float* conds_y,
                      float* pdf, hipStream_t s);
// CDF check (*bad |= 1 unless the guides are valid) + the env_cell search guides
void launch_env_guides(const float* marginal_y, const float* conds_y, int W, int H, uint16_t* gm, uint16_t* gc,
                       uint32_t* bad, hipStream_t s);

// GPU linear BVH (bvh_build.hip).  Inputs: host vertex arrays (3 floats per
// triangle each) and the device triangle / shading records in scene order.
struct LbvhInput { int ntri; const float *v0, *v1, *v2; const float4 *d_tri, *d_sh; };
struct LbvhOutput {
    float4 *nodes = nullptr, *tri = nullptr, *tri_sh = nullptr;  // hipMalloc'ed, owned by the caller
    int nnodes = 0, root_ref = 0, depth = 0, rounds = 0;
    float root_mn[3], root_mx[3];
};
// PLOC cluster record: subtree height (low 8 bits, saturated at 255) and the subtree's
// interior-node count (bits 8..31).  Unsigned with logical shifts: a count below 2^24 (every
// scene mcpt_scene_upload accepts) packs and unpacks exactly (tests/native/core_identities.cpp).
__host__ __device__ constexpr uint32_t ploc_pack(uint32_t height, uint32_t count) {
    return (height < 255u ? height : 255u) | (count << 8);
}
__host__ __device__ constexpr uint32_t ploc_height(uint32_t h) { return h & 0xffu; }
__host__ __device__ constexpr uint32_t ploc_count(uint32_t h) { return h >> 8; }
// the record of a merge of clusters a and b
__host__ __device__ constexpr uint32_t ploc_merge(uint32_t a, uint32_t b) {
    return ploc_pack((ploc_height(a) > ploc_height(b) ? ploc_height(a) : ploc_height(b)) + 1u,
                     ploc_count(a) + ploc_count(b) + 1u);
}
int build_lbvh(const LbvhInput& in, LbvhOutput& out, hipStream_t s);
int build_ploc(const LbvhInput& in, LbvhOutput& out, hipStream_t s);
int trace_profile(unsigned long long* out, int reset);
int wave_times(unsigned long long* out, int n);
int shade_sections(unsigned long long* out, int n, int reset);  // -DMCPT_DIAG_SHADE builds (else 0)
void launch_cam_table(const mcpt::CamView& cam, int W, int H, float4* px, float4* dir, hipStream_t s);
void launch_quot(const float* a, const float* b, float* out, uint32_t n, hipStream_t s);
void launch_copy(const float4* src, float4* dst, size_t n, hipStream_t s);
void launch_hit_record(const HitRecordArgs& a, hipStream_t s);
void launch_tonemap(const TonemapArgs& a, hipStream_t s);
void launch_resolve(const ResolveArgs& a, hipStream_t s);
void launch_accumulate(CounterBlock* c, uint32_t nparts, uint32_t* occ_gate, hipStream_t s);
void launch_pack(const PackArgs& a, hipStream_t s);
void launch_unpack(const UnpackArgs& a, hipStream_t s);

}  // namespace mcpt_dev
