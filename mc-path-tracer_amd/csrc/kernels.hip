// kernels.hip -- gfx950 kernels of the wavefront path tracer.
//
// One wavefront iteration (= one reference wavefront_pathtrace call,
// wavefront_kernels.cu:377-442, widened from one 256x256 tile to a tile set):
//   k_shade     fused wf_logic + wf_generate, one thread per path (wavefront_kernels.cu:90-251);
//               pushes the continuing paths as dense material records
//   k_material  light choice + wf_mat_mix over the material records (:207-215, 295-375)
//   k_trace     one persistent launch for both ray sets: wf_extend closest hit
//               (wavefront_kernels.cu:253-272, Triangle.cu:144-203) and wf_shadow + the BRDF
//               visibility ray that the reference traces inline in wf_mat_mix
//               (wavefront_kernels.cu:274-293, 334-336; Triangle.cu:204-243)
// The material stage evaluates the BRDF-sample terms unconditionally and the
// visibility bit selects them in the next k_shade; this is exactly the
// reference's result (f_brdf = Li_brdf = 0, pdf_brdf.x = pdf_light.y = 1 when
// occluded, wavefront_kernels.cu:311).  Queues are compacted per block with
// wave64 ballot + mbcnt + an LDS prefix and one atomic per block and queue.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>

#include "device/mcpt_core.hpp"
#include "kernels.hpp"

using namespace mcpt;

namespace mcpt_dev {

// ---------------------------------------------------------------------------
// block-level stream compaction (replaces per-thread atomicAdd pushes,
// wavefront_kernels.cu:215,221,250,373,374)
// ---------------------------------------------------------------------------
template <int NQ>
__device__ inline void block_push(const bool (&want)[NQ], uint32_t* const (&counters)[NQ], uint32_t (&slot)[NQ],
                                  uint32_t (&total)[NQ]) {
    __shared__ uint32_t s_wave[NQ][kBlock / 64];
    __shared__ uint32_t s_base[NQ];
    __shared__ uint32_t s_tot[NQ];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t prefix[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
        uint64_t m = __ballot(want[q]);
        prefix[q] = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (lane == 0) s_wave[q][wave] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x < NQ) {
        const int q = threadIdx.x;
        uint32_t tot = 0;
        for (int w = 0; w < kBlock / 64; w++) { uint32_t c = s_wave[q][w]; s_wave[q][w] = tot; tot += c; }
        s_base[q] = tot ? atomicAdd(counters[q], tot) : 0u;
        s_tot[q] = tot;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NQ; q++) {
        slot[q] = s_base[q] + s_wave[q][wave] + prefix[q];
        total[q] = s_tot[q];
    }
}

__device__ inline V3 xyz(float4 a) { return v3(a.x, a.y, a.z); }

// The kernel's by-value argument struct read through an opaque copy of the kernarg segment
// pointer.  Kernel arguments are invariant loads, so the compiler hoists every field a persistent
// loop uses into SGPRs at kernel entry; ShadeArgs' ~60 uniform words then exceed the SGPR file and
// spill into VGPR lanes (k_material: 78 SGPRs, 76 v_writelane / 281 v_readlane).  Behind the empty
// asm the pointer is a new value wherever this is called, so the fields are loaded (s_load from the
// scalar cache) where they are used.  The struct stays in the constant address space: the cast to
// a generic reference is undone by address-space inference after inlining (scalar loads, no flat).
// k_material: 128 -> 112 VGPRs, no SGPR spill, shade stage 142.9 -> 141.1 ms per config-2 frame
// (interleaved A/B, two rounds).  The same re-read per k_trace loop trip removed its 12 SGPR spills
// but cost 2.52 -> 2.59 ms per launch (scalar-load latency on every trip): not used there.
template <class T>
__device__ inline const T& kernarg_fresh() {
    typedef const __attribute__((address_space(4))) T KT;
    KT* p = (KT*)__builtin_amdgcn_kernarg_segment_ptr();
    __asm__ volatile("" : "+s"(p));
    return *(const T*)p;
}


// Path-state streams of the shading kernels (k_shade, k_material): every word is touched once per
// kernel and iteration, over a state many times the L2 and MALL, so MCPT_NT marks these loads (bit
// 1) and stores (bit 2) non-temporal -- streaming, not retained -- for the env tables, BVH and
// occluder records to keep the caches.  Bit 4: k_trace's ray loads and result stores too; bit 8:
// the queue entries and staged any-hit rays the shading kernels store.  Measured (config 2 / 3,
// interleaved, two rounds): loads and stores (3) shade stage 144.6 -> 138.4 ms / 107.5 -> 101.4 ms
// per frame, stores alone (2) nearly as good, loads alone (1) 0.5-3 % slower.
#ifndef MCPT_NT
#define MCPT_NT 3
#endif
template <class T>
__device__ inline void st_q(T* p, T v) {  // queue entries (MCPT_NT bit 8)
    if constexpr (MCPT_NT & 8) __builtin_nontemporal_store(v, p);
    else *p = v;
}
typedef float f4v_t __attribute__((ext_vector_type(4)));
typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
template <class T>
__device__ inline T ld_s(const T* p) {
    if constexpr (MCPT_NT & 1) return __builtin_nontemporal_load(p);
    else return *p;
}
__device__ inline float4 ld_s(const float4* p) {
    if constexpr (MCPT_NT & 1) {
        const f4v_t v = __builtin_nontemporal_load(reinterpret_cast<const f4v_t*>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}
__device__ inline uint4 ld_s(const uint4* p) {
    if constexpr (MCPT_NT & 1) {
        const u4v_t v = __builtin_nontemporal_load(reinterpret_cast<const u4v_t*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}
template <class T>
__device__ inline void st_s(T* p, T v) {
    if constexpr (MCPT_NT & 2) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ inline void st_s(float4* p, float4 v) {
    if constexpr (MCPT_NT & 2) __builtin_nontemporal_store(f4v_t{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v_t*>(p));
    else *p = v;
}
__device__ inline void st_s(uint4* p, uint4 v) {
    if constexpr (MCPT_NT & 2) __builtin_nontemporal_store(u4v_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u4v_t*>(p));
    else *p = v;
}
// the xyz of a float4 element with one dwordx3 load (one VGPR fewer than the float4)
__device__ inline V3 ld3f4(const float4* p) {
    const float* f = reinterpret_cast<const float*>(p);
    return v3(f[0], f[1], f[2]);
}
__device__ inline float4 f4(V3 v, float w) { return make_float4(v.x, v.y, v.z, w); }

// Diagnostics of the shading kernels' instruction attribution, off in the product:
//  * -DMCPT_ISA_MARKERS: assembly comments at the section boundaries (MCPT_MARK, mcpt_core.hpp;
//    tools/isa_sections.py counts the VALU instructions between them in hipcc -S output);
//  * -DMCPT_DIAG_SHADE: per-section wave entries and active lanes, summed over a run in a device
//    global (mcpt_debug_shade_sections reads it).
enum : int { SD_WAVES = 0, SD_VALID, SD_LOGIC, SD_NEE, SD_GEN, SD_CONT, SD_BG, SD_N };
#ifdef MCPT_DIAG_SHADE
__device__ unsigned long long g_shade_diag[2 * SD_N];
#define SHADE_DIAG(k, cond)                                                      \
    do {                                                                         \
        const uint64_t m_ = __ballot(cond);                                      \
        if ((threadIdx.x & 63) == 0 && m_) {                                     \
            atomicAdd(&g_shade_diag[2 * (k)], 1ull);                             \
            atomicAdd(&g_shade_diag[2 * (k) + 1], (unsigned long long)__popcll(m_)); \
        }                                                                        \
    } while (0)
#else
#define SHADE_DIAG(k, cond) \
    do {                    \
    } while (0)
#endif
int shade_sections(unsigned long long* out, int n, int reset) {
#ifdef MCPT_DIAG_SHADE
    unsigned long long h[2 * SD_N];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_shade_diag), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < n && i < 2 * SD_N; i++) out[i] = h[i];
    if (reset) {
        memset(h, 0, sizeof(h));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_shade_diag), h, sizeof(h)) != hipSuccess) return -1;
    }
    return 2 * SD_N;
#else
    for (int i = 0; i < n; i++) out[i] = 0;
    (void)reset;
    return 0;
#endif
}

__device__ inline V3 light_L(const DevScene& sc, int id, V3 wi) {
    if (id == 0) return env_L(sc.env, wi);
    const float* p = sc.dirs + 7 * (id - 1);  // DirectionalLight.cu:34
    return v3(p[3], p[4], p[5]) * p[6];
}
template <bool FIXED>
__device__ inline void light_L_pdf(const DevScene& sc, int id, V3 wi, V3& L, float& pdf) {
    if (id == 0) {
        env_L_pdf<FIXED>(sc.env, wi, L, pdf);
    } else {
        const float* p = sc.dirs + 7 * (id - 1);  // DirectionalLight.cu:34, :40-43
        L = v3(p[3], p[4], p[5]) * p[6];
        pdf = 1.f;
    }
}
__device__ inline float light_pdf(const DevScene& sc, int id, V3 wi) {
    if (id == 0) return env_pdf(sc.env, wi);
    return 1.f;  // DirectionalLight.cu:40-43
}

// Reference slab test (Bounds3f.h:121-153) written branch-free: the same six
// products and the same comparison sequence, evaluated unconditionally so the
// whole node is fetched up front (the early-out form let the compiler sink the
// z loads behind the x/y test: two dependent round trips per node).  NaN slabs
// compare false and pass, exactly as in the reference.
__device__ inline bool slab(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, V3 o, V3 inv,
                            int nx, int ny, int nz, float& t0, float& t1) {
    float bx0 = nx ? mxx : mnx, bx1 = nx ? mnx : mxx;
    float by0 = ny ? mxy : mny, by1 = ny ? mny : mxy;
    float bz0 = nz ? mxz : mnz, bz1 = nz ? mnz : mxz;
    float tmin = (bx0 - o.x) * inv.x;
    float tmax = (bx1 - o.x) * inv.x;
    float tymin = (by0 - o.y) * inv.y;
    float tymax = (by1 - o.y) * inv.y;
    float tzmin = (bz0 - o.z) * inv.z;
    float tzmax = (bz1 - o.z) * inv.z;
    bool miss = (tmin > tymax) || (tymin > tmax);
    float a = (tymin > tmin) ? tymin : tmin;
    float b = (tymax < tmax) ? tymax : tmax;
    miss = miss || (a > tzmax) || (tzmin > b);
    t0 = (tzmin > a) ? tzmin : a;
    t1 = (tzmax < b) ? tzmax : b;
    return !miss;
}
constexpr float K_INF_F = __builtin_huge_valf();
#ifndef MCPT_OCC_LAYOUT
#define MCPT_OCC_LAYOUT 0  // occluder-table key order (occ_index): 0 origin-cell major, 1 direction-bin major
#endif
constexpr int kEnd = -1;  // not a valid leaf: offset + count <= ntri < 2^24

// Culling scale of a ray (mcpt_core.hpp "conservative box culling"): iota = max_a |1/d_a| (1 + 2^-18)
// for the rays the bound covers -- finite inverse, |d| <= 1 + 2^-10, a scene whose boxes contain
// their triangles.  The sign says whether the behind cut applies: +iota when iota P <= 1 (no
// direction component below P |d|), -iota when not.  Rays the bound does not cover get -FLT_MAX:
// W iota is then beyond every t for any box holding a triangle that can be accepted at all (det
// >= 1e-6 needs |e1| |e2| |d| >= 1e-6, so such a box has W > 1e-9), i.e. nothing is culled.  A
// ray with an infinite inverse component gets -inf (it takes slab(): |iota| = inf is the test).
// One register per ray holds all of it.
__device__ inline float cull_iota(const DevScene& sc, V3 d, V3 inv) {
    const float ax = __builtin_fabsf(inv.x), ay = __builtin_fabsf(inv.y), az = __builtin_fabsf(inv.z);
    if (!(ax < K_INF_F && ay < K_INF_F && az < K_INF_F)) return -K_INF_F;
    const float n2 = d.x * d.x + d.y * d.y + d.z * d.z;
    if (!sc.cull_ok || !(n2 <= kCullNormMax)) return -3.4028235e38f;
    const float io = __builtin_fmaxf(__builtin_fmaxf(ax, ay), az) * kCullSlackF;
    return io * sc.cull_p <= 1.f ? io : -io;
}
// The cull of a box whose slab test passed, with m = W iota (W: the box's margin, iota signed as
// cull_iota returns it).  key = t0 - |m|: no triangle in the box can be accepted with t below it,
// so it orders the stack and is re-tested against the cut on pop.  The behind cut needs m >= 0 (a
// NaN m, from W = 0 with iota = inf, culls nothing).  Any-hit rays pass cut = +inf.
__device__ inline bool keep_box(float t0, float t1, float m, float cut, float& key) {
    key = t0 - __builtin_fabsf(m);
    return !(m >= 0.f && __builtin_fmaf(t1, kCullBehindF, m) < 0.f) && !(key > cut);
}

// Both child boxes of a pair node at once, for rays whose inverse direction is
// finite in all three components (then no slab product can be NaN).  The six
// plane differences and products per box run as packed fp32 pairs (one
// v_pk_add_f32 + one v_pk_mul_f32 per axis and plane: the two boxes' planes
// sit side by side in the node).  Entry/exit per axis are min/max of the two
// products: by monotone rounding they equal the reference's sign-selected near
// and far products (Bounds3f.h:121-153), and the reference's pairwise overlap
// tests reduce to max3(entries) <= min3(exits) (Helly in 1-D); t0/t1 equal its
// running max/min up to the sign of zero.  Rays with an infinite inverse
// component take slab().
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ inline void pair_slab(float4 qx, float4 qy, float4 qz, V3 o, V3 inv, float& t0a, float& t1a, float& t0b,
                                 float& t1b) {
    const f2v ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
    const f2v ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
    const f2v ax = (f2v{qx.x, qx.y} - ox) * ix, bx = (f2v{qx.z, qx.w} - ox) * ix;
    const f2v ay = (f2v{qy.x, qy.y} - oy) * iy, by = (f2v{qy.z, qy.w} - oy) * iy;
    const f2v az = (f2v{qz.x, qz.y} - oz) * iz, bz = (f2v{qz.z, qz.w} - oz) * iz;
    t0a = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(ax.x, bx.x), __builtin_fminf(ay.x, by.x)),
                          __builtin_fminf(az.x, bz.x));
    t1a = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(ax.x, bx.x), __builtin_fmaxf(ay.x, by.x)),
                          __builtin_fmaxf(az.x, bz.x));
    t0b = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(ax.y, bx.y), __builtin_fminf(ay.y, by.y)),
                          __builtin_fminf(az.y, bz.y));
    t1b = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(ax.y, bx.y), __builtin_fmaxf(ay.y, by.y)),
                          __builtin_fmaxf(az.y, bz.y));
}

// The four child boxes of a 4-wide node, same arithmetic as pair_slab (packed
// pairs of boxes per axis and plane; entry/exit = min/max of the two products),
// folded axis by axis (max/min are exact, so the order does not change t0/t1).
__device__ inline void quad_axis(const float4& mn, const float4& mx, float o, float inv, float (&lo)[4],
                                 float (&hi)[4], bool first) {
    const f2v oo = {o, o}, ii = {inv, inv};
    const f2v a0 = (f2v{mn.x, mn.y} - oo) * ii, a1 = (f2v{mn.z, mn.w} - oo) * ii;
    const f2v b0 = (f2v{mx.x, mx.y} - oo) * ii, b1 = (f2v{mx.z, mx.w} - oo) * ii;
    const float l[4] = {__builtin_fminf(a0.x, b0.x), __builtin_fminf(a0.y, b0.y), __builtin_fminf(a1.x, b1.x),
                        __builtin_fminf(a1.y, b1.y)};
    const float h[4] = {__builtin_fmaxf(a0.x, b0.x), __builtin_fmaxf(a0.y, b0.y), __builtin_fmaxf(a1.x, b1.x),
                        __builtin_fmaxf(a1.y, b1.y)};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        lo[k] = first ? l[k] : __builtin_fmaxf(lo[k], l[k]);
        hi[k] = first ? h[k] : __builtin_fminf(hi[k], h[k]);
    }
}

// The same slab tests with the ray held as (o_a, 1 / d_a) register pairs, one per axis: the packed
// subtract takes o_a from the pair's low half for both lanes (op_sel_hi) and the packed multiply
// 1 / d_a from its high half (op_sel), so no duplicated {o_a, o_a} / {inv_a, inv_a} pairs are built
// per trip (9 VALU moves per k_trace loop trip were the compiler's copies for pair_slab's
// broadcasts).  The operations and their order are pair_slab's: q + (-o) is q - o exactly; min and
// max are exact.  Written as inline assembly because the compiler neither folds the broadcasts into
// op_sel nor knows an asm result is a canonical float (it would canonicalise each before min / max);
// the operands are finite here (finite inverse: no NaN product).
__device__ inline f2v pk_slab(f2v q, f2v p) {  // ((q.x - p.x) * p.y, (q.y - p.x) * p.y)
    f2v r;
    __asm__("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
            "v_pk_mul_f32 %0, %0, %2 op_sel:[0,1] op_sel_hi:[1,1]"
            : "=&v"(r)
            : "v"(q), "v"(p));
    return r;
}
// entry / exit of one box from its six plane products: max3 of the per-axis minima, min3 of the maxima
__device__ inline void box_t(float ax, float bx, float ay, float by, float az, float bz, float& t0, float& t1) {
    float m0, m1, m2, n0, n1, n2;
    __asm__("v_min_f32 %2, %8, %9\n\t"
            "v_min_f32 %3, %10, %11\n\t"
            "v_min_f32 %4, %12, %13\n\t"
            "v_max_f32 %5, %8, %9\n\t"
            "v_max_f32 %6, %10, %11\n\t"
            "v_max_f32 %7, %12, %13\n\t"
            "v_max3_f32 %0, %2, %3, %4\n\t"
            "v_min3_f32 %1, %5, %6, %7"
            : "=v"(t0), "=v"(t1), "=&v"(m0), "=&v"(m1), "=&v"(m2), "=&v"(n0), "=&v"(n1), "=&v"(n2)
            : "v"(ax), "v"(bx), "v"(ay), "v"(by), "v"(az), "v"(bz));
}
__device__ inline void pair_slab2(float4 qx, float4 qy, float4 qz, f2v px, f2v py, f2v pz, float& t0a, float& t1a,
                                  float& t0b, float& t1b) {
    const f2v ax = pk_slab(f2v{qx.x, qx.y}, px), bx = pk_slab(f2v{qx.z, qx.w}, px);
    const f2v ay = pk_slab(f2v{qy.x, qy.y}, py), by = pk_slab(f2v{qy.z, qy.w}, py);
    const f2v az = pk_slab(f2v{qz.x, qz.y}, pz), bz = pk_slab(f2v{qz.z, qz.w}, pz);
    box_t(ax.x, bx.x, ay.x, by.x, az.x, bz.x, t0a, t1a);
    box_t(ax.y, bx.y, ay.y, by.y, az.y, bz.y, t0b, t1b);
}
// quad_axis with the (o_a, 1 / d_a) pair (pk_slab); the folds over the axes as quad_axis (min / max in
// asm as well: their inputs are asm results)
__device__ inline float vmin(float a, float b) {
    float r;
    __asm__("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ inline float vmax(float a, float b) {
    float r;
    __asm__("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ inline void quad_axis2(const float4& mn, const float4& mx, f2v p, float (&lo)[4], float (&hi)[4], bool first) {
    const f2v a0 = pk_slab(f2v{mn.x, mn.y}, p), a1 = pk_slab(f2v{mn.z, mn.w}, p);
    const f2v b0 = pk_slab(f2v{mx.x, mx.y}, p), b1 = pk_slab(f2v{mx.z, mx.w}, p);
    const float l[4] = {vmin(a0.x, b0.x), vmin(a0.y, b0.y), vmin(a1.x, b1.x), vmin(a1.y, b1.y)};
    const float h[4] = {vmax(a0.x, b0.x), vmax(a0.y, b0.y), vmax(a1.x, b1.x), vmax(a1.y, b1.y)};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        lo[k] = first ? l[k] : vmax(lo[k], l[k]);
        hi[k] = first ? h[k] : vmin(hi[k], h[k]);
    }
}

// The first test the traversal makes: a NaN/zero direction or a ray that misses
// the root box (after the cull) can hit nothing.  k_shade resolves such rays in
// place instead of queueing them.
__device__ inline bool ray_misses_scene(const DevScene& sc, V3 o, V3 d) {
    if (!(d.x == d.x && d.y == d.y && d.z == d.z) || (d.x == 0.f && d.y == 0.f && d.z == 0.f)) return true;
    // An origin inside the root box cannot miss it: per axis (mn - o) <= 0 <= (mx - o)
    // exactly, so entry <= 0 <= exit (or NaN, which passes), and the cull keeps the
    // box.  Skips the three IEEE divisions for every bounce ray inside the scene.
    if (o.x >= sc.root_mn[0] && o.x <= sc.root_mx[0] && o.y >= sc.root_mn[1] && o.y <= sc.root_mx[1] &&
        o.z >= sc.root_mn[2] && o.z <= sc.root_mx[2])
        return false;
    const V3 inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
    const float m = sc.root_w * cull_iota(sc, d, inv);
    float t0, t1, key;
    return !(slab(sc.root_mn[0], sc.root_mn[1], sc.root_mn[2], sc.root_mx[0], sc.root_mx[1], sc.root_mx[2], o, inv,
                  inv.x < 0.f, inv.y < 0.f, inv.z < 0.f, t0, t1) &&
             keep_box(t0, t1, m, K_INF_F, key));
}

// Hit record of ray (o, d) on triangle tri, as dTriangle::hit builds it
// (Triangle.cu:66-92): Moller-Trumbore t/u/v, the interpolated normal
// normalised twice (identity transform), position o + t d, material id.
__device__ inline void hit_record(const DevScene& sc, V3 o, V3 d, int tri, V3& pos, V3& nrm, int& mat, float& t_out) {
    const float4* tp = sc.tri + kTriF4 * tri;
    const float4 w0 = tp[0], w1 = tp[1], w2 = tp[2];
    const float4* sp4 = sc.tri_sh + 3 * tri;
    const float4 s0 = sp4[0], s1 = sp4[1], s2 = sp4[2];
    // All six loads in one round trip: the compiler otherwise issues the vertex load after
    // the determinant test and the shading record after the whole test (three serialised
    // fetches; the hit is known to exist, so every value is used).
    __asm__ volatile("" ::"v"(w0.x), "v"(w0.y), "v"(w0.z), "v"(w0.w), "v"(w1.x), "v"(w1.y), "v"(w1.z), "v"(w1.w),
                     "v"(w2.x), "v"(s0.x), "v"(s0.y), "v"(s0.z), "v"(s0.w), "v"(s1.x), "v"(s1.y), "v"(s1.z),
                     "v"(s1.w), "v"(s2.x), "v"(s2.y));
    float t, u, v;
    tri_test(o, d, v3(w0.x, w0.y, w0.z), v3(w0.w, w1.x, w1.y), v3(w1.z, w1.w, w2.x), t, u, v);
    const V3 n0 = v3(s0.x, s0.y, s0.z), n1 = v3(s0.w, s1.x, s1.y), n2 = v3(s1.z, s1.w, s2.x);
    const float w = (1.f - u) - v;
    nrm = normalize((n1 * u + n2 * v) + n0 * w);  // Triangle.cu:76
    nrm = normalize(nrm);                          // identity transform, :82
    pos = o + d * t;                               // :86
    mat = __float_as_int(s2.y);                    // material id bits
    t_out = t;
}

// ---------------------------------------------------------------------------
// Any-hit occluder cache.  An any-hit ray's outcome is one bit (wf_shadow,
// wavefront_kernels.cu:274-293): occluded iff some triangle passes the traversal's
// acceptance -- its leaf box and every ancestor box pass the slab test and the cull,
// and Moller-Trumbore accepts it with 0 <= t < K_HUGE (Triangle.cu:157-205).  Which
// occluder is found does not matter.  k_trace records the occluder of each occluded
// ray in a small table keyed by (origin cell, direction bin), and k_material tests a new
// any-hit ray against its cell's entry first, under that triangle's own leaf box with
// the traversal's arithmetic (pair_slab's products, keep_box with the any-hit cut).
// Every ancestor box contains the leaf box and the rounded slab interval is monotone in
// the box, so an ancestor passes whenever the leaf does: a cache hit is a triangle the
// traversal accepts as well, and the ray is resolved as occluded exactly as the
// traversal would resolve it.  A miss costs the test and the ray is traced as before.
// The table's contents (racy plain stores) only decide how much work is skipped, never
// a result.  Rays with an infinite inverse component (slab(), NaN slabs) are not tested.
// ---------------------------------------------------------------------------
__device__ inline uint32_t occ_index(const DevScene& sc, V3 o, V3 d) {
    const float gm = (float)(sc.occ_g - 1), bm = (float)(sc.occ_b - 1), hb = 0.5f * (float)sc.occ_b;
    // fmaxf(NaN, 0) = 0: a NaN coordinate falls in cell / bin 0
    const uint32_t cx = (uint32_t)__builtin_fminf(__builtin_fmaxf((o.x - sc.root_mn[0]) * sc.occ_inv[0], 0.f), gm);
    const uint32_t cy = (uint32_t)__builtin_fminf(__builtin_fmaxf((o.y - sc.root_mn[1]) * sc.occ_inv[1], 0.f), gm);
    const uint32_t cz = (uint32_t)__builtin_fminf(__builtin_fmaxf((o.z - sc.root_mn[2]) * sc.occ_inv[2], 0.f), gm);
    const float ax = __builtin_fabsf(d.x), ay = __builtin_fabsf(d.y), az = __builtin_fabsf(d.z);
    uint32_t face;
    float u, v, m;
    if (ax >= ay && ax >= az) {
        face = d.x < 0.f ? 1u : 0u; u = d.y; v = d.z; m = ax;
    } else if (ay >= az) {
        face = d.y < 0.f ? 3u : 2u; u = d.x; v = d.z; m = ay;
    } else {
        face = d.z < 0.f ? 5u : 4u; u = d.x; v = d.y; m = az;
    }
    const float r = hb * __builtin_amdgcn_rcpf(m);  // cube-map coordinates in [-1, 1] -> [0, B)
    const uint32_t ub = (uint32_t)__builtin_fminf(__builtin_fmaxf(u * r + hb, 0.f), bm);
    const uint32_t vb = (uint32_t)__builtin_fminf(__builtin_fmaxf(v * r + hb, 0.f), bm);
    const uint32_t G = (uint32_t)sc.occ_g, B = (uint32_t)sc.occ_b;
    // one table cell per key (hashing the keys into a 2^21- or 2^23-cell table measured 43 % / 60 %
    // of config 2's any-hit rays resolved against 72 % direct: the keys that occur collide heavily)
#if MCPT_OCC_LAYOUT == 1
    // direction major: lanes whose rays share a direction bin and lie in neighbouring origin cells
    // (along x) read one 128-B line (A/B knob)
    return (((face * B + ub) * B + vb) * G + cz) * G * G + cy * G + cx;
#else
    return ((((cz * G + cy) * G + cx) * 6u + face) * B + ub) * B + vb;
#endif
}

// true: (o, d) (reciprocal inv, all finite; signed culling scale io) is occluded by the triangle of
// occluder record r0..r3 (kOccRecF4: {leaf box mn, margin} {leaf box mx, v0.x} {v0.yz, e1.xy}
// {e1.z, e2}) under its leaf box
__device__ inline bool occ_test(V3 o, V3 d, V3 inv, float io, float4 bmn, float4 bmx, float4 r2, float4 r3) {
    // pair_slab's arithmetic for one box (its first lane)
    const float ax = (bmn.x - o.x) * inv.x, bx = (bmx.x - o.x) * inv.x;
    const float ay = (bmn.y - o.y) * inv.y, by = (bmx.y - o.y) * inv.y;
    const float az = (bmn.z - o.z) * inv.z, bz = (bmx.z - o.z) * inv.z;
    const float t0 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(ax, bx), __builtin_fminf(ay, by)),
                                     __builtin_fminf(az, bz));
    const float t1 = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(ax, bx), __builtin_fmaxf(ay, by)),
                                     __builtin_fmaxf(az, bz));
    float key;
    if (!(t0 <= t1) || !keep_box(t0, t1, bmn.w * io, K_INF_F, key)) return false;  // k_trace's any-hit cull
    float th;
    return tri_test_t(o, d, v3(bmx.w, r2.x, r2.y), v3(r2.z, r2.w, r3.x), v3(r3.y, r3.z, r3.w), th) && !(th < 0.f) &&
           th < K_HUGE;
}
// The cell's entries of (o, d): kOccWays triangle records (k_trace writes way tri mod kOccWays).
// MCPT_NT bit 16: the table's random 8-B reads and the occluder stores are non-temporal (the 96 MB
// table cannot stay in L2; its lines would evict the env tables' and occluder records').
__device__ inline uint2 occ_entry(const DevScene& sc, uint32_t cell) {
    const uint2* e = reinterpret_cast<const uint2*>(sc.occ) + cell;
    if constexpr (MCPT_NT & 16) {
        typedef uint32_t u2v_t __attribute__((ext_vector_type(2)));
        const u2v_t v = __builtin_nontemporal_load(reinterpret_cast<const u2v_t*>(e));
        return make_uint2(v.x, v.y);
    } else {
        return *e;
    }
}
// An any-hit ray against its cell's entries: both candidates' occluder records (leaf box, margin
// and triangle in one aligned 64-B record: one half line each, where the leaf box and the 48-B
// triangle record used to cost two or three) are fetched in one round trip (an empty way reads
// record 0 and is not tested).  k_material calls it for the light ray, then the BRDF ray: 32
// VGPRs of records at a time, next to the BRDF sample's deferred state.
__device__ inline bool occ_hit1(const DevScene& sc, V3 o, V3 d, uint2 e) {
    const bool v0 = e.x < sc.ntri, v1 = e.y < sc.ntri;
    if (!(v0 || v1)) return false;
    const float4* p0 = sc.occ_rec + kOccRecF4 * (size_t)(v0 ? e.x : 0u);
    const float4* p1 = sc.occ_rec + kOccRecF4 * (size_t)(v1 ? e.y : 0u);
    const float4 bn0 = p0[0], bx0 = p0[1], r20 = p0[2], r30 = p0[3];
    const float4 bn1 = p1[0], bx1 = p1[1], r21 = p1[2], r31 = p1[3];
    const V3 inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);  // k_trace's
    if (!(__builtin_fabsf(inv.x) < K_INF_F && __builtin_fabsf(inv.y) < K_INF_F && __builtin_fabsf(inv.z) < K_INF_F))
        return false;
    const float io = cull_iota(sc, d, inv);
    return (v0 && occ_test(o, d, inv, io, bn0, bx0, r20, r30)) || (v1 && occ_test(o, d, inv, io, bn1, bx1, r21, r31));
}

// ---------------------------------------------------------------------------
// k_shade: the first half of one wavefront iteration's shading, for one block of
// 256 pixels of a path slot.
//   phase 1, one thread per pixel: wf_logic (MIS combine, throughput update,
//     Russian roulette, termination, sample count) and wf_generate for pixels
//     whose path ended (wavefront_kernels.cu:90-251);
//   phase 2: one block-wide push (ballot + mbcnt + per-wave LDS prefix, one atomic
//     per queue) of the generated extension rays and of the continuing paths as
//     material records, which k_material (below) runs densely: the light choice
//     and wf_mat_mix are most of the shading instructions, and on the pixel-ordered
//     threads they ran with the terminating / regenerating lanes masked off.
// Per path the arithmetic is the reference's, so which thread evaluates a path
// does not change any result.
// ---------------------------------------------------------------------------
struct MatOut {
    bool want_ext, want_l, want_b, trivial_ext, vis_ray, need_cb;
    uint32_t trivial_any;
    uint2 el, eb;  // occluder-cache entries of the light / BRDF rays (loads issued inside material())
    // the BRDF sample's light terms are finished by material_brdf_terms after the occluder cache
    // (a visibility ray it resolves as occluded needs none: k_shade reads nee1.xyz only when
    // vis = 1, wavefront_kernels.cu:336-343)
    V3 n, wo, wi_b;
    int matid, light_id;
    uint32_t flags;  // the flags word (F_CONDB added by material_brdf_terms)
    float rrz;       // nee1.w
};

// Light choice + wf_mat_mix for the continuing path pid of pixel `pix` (vertex len, sample
// index `sidx`, throughput `beta_store` after the logic update).
//
// FIXED (quality mode, mcpt_config.flags & MCPT_FLAG_FIXED) changes, each
// a reference quirk of Appendix A: light-selection pdf 1/N folded into both light pdfs
// (A.6), delta lights get MIS weight 1 (pdf_brdf.y = 0 instead of 1, A.7), textbook
// Gram-Schmidt (A.9), env sampling/pdf on matched, clamped cells (A.11).
template <bool FIXED>
__device__ inline MatOut material(const ShadeArgs& a, uint32_t pid, uint32_t pix, uint32_t sidx, uint32_t len,
                                 V3 beta_store, int32_t htri, float4* stage, bool occ_on) {
    const DevScene& sc = a.scene;
    const uint2 none = make_uint2(kOccEmpty, kOccEmpty);
    MatOut mo{};
    mo.el = mo.eb = none;
    // the pixel and the sample index come with the record (k_shade: slot k of a pixel runs
    // samples k, k + S, k + 2S, ...)
    MCPT_MARK("m_hit");
    const Rng r{rng_key(a.seed, pix, sidx), len};
    const V3 ro = xyz(ld_s(a.p.ray_o + pid)), rdir = xyz(ld_s(a.p.ray_d + pid));
    V3 pos, n;
    int mat;
    float t_hit;
    hit_record(sc, ro, rdir, htri, pos, n, mat, t_hit);
    const V3 wo = -rdir;
    const Mat m = load_mat(sc.mats + 8 * mat);
    // The three parts of wf_mat_mix draw from disjoint RNG slots and share only the hit
    // record, so they are evaluated in the order that lets each store its results at
    // once (short register live ranges): the continuation first (:353-358, its ratio
    // f_s/pdf_s rides in the .w slots of beta/nee0/nee1), then the light sample
    // (:316-329), then the BRDF sample's direction (:331-334); its light terms
    // (:335-343) wait for the occluder cache (material_brdf_terms).
    uint32_t nf = 0;
    V3 rr;
    {
        MCPT_MARK("m_cont");
        V3 wi_s = brdf_sample_wi<FIXED>(m, n, wo, r, SL_CONT_E0, r(SL_CONT_LOBE) < 0.5f);  // spec : diff
        float pdf_s;
        V3 f_s;
        brdf_f_pdf(m, n, wi_s, wo, f_s, pdf_s);
        if ((f_s.x == 0.f && f_s.y == 0.f && f_s.z == 0.f) || pdf_s == 0.f) nf |= F_FZERO;
        rr = f_s / pdf_s;
        const V3 new_o = pos + n * 0.001f;  // :358
        st_s(a.p.beta + pid, f4(beta_store, rr.x));
        st_s(a.p.ray_o + pid, f4(new_o, 0.f));
        st_s(a.p.ray_d + pid, f4(wi_s, 0.f));
        mo.want_ext = true;
        if (ray_misses_scene(sc, new_o, wi_s)) {  // resolved here: isect stays "not found"
            a.p.hit_tri[pid] = -1;
            mo.want_ext = false;
            mo.trivial_ext = true;
        }
    }
    MCPT_MARK("m_light");
    int l_id = (int)(r(SL_LIGHT) * (float)(sc.nlights - 0) + (float)0);
    const int light_id = (l_id == sc.nlights) ? 0 : l_id;
    const bool delta = light_id > 0;
    const float sel = FIXED ? 1.f / (float)sc.nlights : 1.f;  // light-selection pdf
    {
        V3 ldir, Li_l;
        float pdfl_x;
        const float4* lt = sc.env.ltab[FIXED ? 1 : 0];
        if (light_id == 0 && lt) {
            // HRDI env sample: direction, radiance and pdf are functions of the sampled cell
            // alone, tabulated at upload by the same code (k_env_table): a 16-B cell fetch and
            // the direction's row / column factors instead of the spherical direction, map,
            // bilinear fetch and pdf of every sample (16 B per cell keeps the table at 2 MiB
            // for a 512x256 map: half the L2 footprint of the previous {dir, pdf, L} cells)
            int cx, cy;
            env_cell<FIXED>(sc.env, r, cx, cy);
            const float4 t0 = lt[(int64_t)cy * (sc.env.w + 1) + cx + 1];
            const float2 rs = sc.env.lrow[FIXED ? 1 : 0][cy], cs = sc.env.lcol[FIXED ? 1 : 0][cx + 1];
            ldir = v3(cs.y * rs.x, rs.y, cs.x * rs.x);  // spherical_direction's products
            pdfl_x = t0.w;
            Li_l = xyz(t0);
        } else {
            if (light_id == 0) ldir = env_dir<FIXED>(sc.env, r);
            else ldir = ld3(sc.dirs + 7 * (light_id - 1), 0);
            light_L_pdf<FIXED>(sc, light_id, ldir, Li_l, pdfl_x);
        }
        V3 f_l;
        float pdf_bl;
        brdf_f_pdf(m, n, ldir, wo, f_l, pdf_bl);
        if (FIXED) pdfl_x = pdfl_x * sel;
        float pdfb_y = !delta ? pdf_bl : (FIXED ? 0.f : 1.f);
        float wL = power_heuristic(pdfl_x, pdfb_y);
        V3 cL = ((f_l * Li_l) * wL) / pdfl_x;
        if (wL > 0.f && pdfl_x > 0.f) nf |= F_CONDL;
        st_s(a.p.nee0 + pid, f4(cL, rr.y));
        const V3 so_l = pos + n * 0.01f;
        if (ray_misses_scene(sc, so_l, ldir)) {
            a.p.vis[2 * pid] = 1;
            mo.trivial_any++;
        } else {
            // staged: stored at its any-queue position after the block push, with the ray's
            // result index (vis) in o.w (k_trace's refill keeps it for the finish)
            stage[0 * kBlock + threadIdx.x] = f4(so_l, __uint_as_float(2 * pid));
            stage[1 * kBlock + threadIdx.x] = f4(ldir, 0.f);
            mo.want_l = true;
            // the occluder-cache entry, loaded now and used after material()
            if (occ_on) mo.el = occ_entry(sc, occ_index(sc, so_l, ldir));
        }
    }
    // the BRDF sample's direction and visibility ray (its light terms come after the occluder
    // cache, material_brdf_terms)
    MCPT_MARK("m_bsdir");
    if (!delta) {
        const V3 wi_b = brdf_sample_wi<FIXED>(m, n, wo, r, SL_MAT_E0, r(SL_MAT_LOBE) < 0.5f);  // spec : diff
        const V3 so_b = pos + wi_b * 0.001f;
        nf |= F_HASVIS;
        mo.vis_ray = true;
        mo.need_cb = true;
        mo.wi_b = wi_b;
        if (ray_misses_scene(sc, so_b, wi_b)) {
            a.p.vis[2 * pid + 1] = 1;
            mo.trivial_any++;
        } else {
            if (occ_on) mo.eb = occ_entry(sc, occ_index(sc, so_b, wi_b));
            stage[2 * kBlock + threadIdx.x] = f4(so_b, __uint_as_float(2 * pid + 1));
            stage[3 * kBlock + threadIdx.x] = f4(wi_b, 0.f);
            mo.want_b = true;
        }
    }
    MCPT_MARK("m_ret");
    mo.n = n;
    mo.wo = wo;
    mo.matid = mat;
    mo.light_id = light_id;
    mo.rrz = rr.z;
    mo.flags = nf | ((len + 1) << F_LEN_SHIFT) | (sidx << F_SIDX_SHIFT);  // extend increments len (:270)
    return mo;
}
// The BRDF sample's light terms (wavefront_kernels.cu:331-343) and the path's last two words:
// nee1 = (cB, f_s / pdf_s .z) and the flags word (F_CONDB).  cB is evaluated only for a
// visibility ray that may be unoccluded (need_cb): one the occluder cache resolved is never read.
template <bool FIXED>
__device__ inline void material_brdf_terms(const ShadeArgs& a, uint32_t pid, const MatOut& mo) {
    const DevScene& sc = a.scene;
    V3 cB = v3(0.f, 0.f, 0.f);
    uint32_t nf = mo.flags;
    if (mo.need_cb) {
        const Mat m = load_mat(sc.mats + 8 * mo.matid);
        V3 f_b;
        float pdfb_x;
        brdf_f_pdf(m, mo.n, mo.wi_b, mo.wo, f_b, pdfb_x);
        V3 Li_b;
        float pdfl_y;
        light_L_pdf<FIXED>(sc, mo.light_id, mo.wi_b, Li_b, pdfl_y);
        if (FIXED) pdfl_y = pdfl_y * (1.f / (float)sc.nlights);
        float wB = power_heuristic(pdfb_x, pdfl_y);
        cB = ((f_b * Li_b) * wB) / pdfb_x;
        if (wB > 0.f && pdfb_x > 0.f) nf |= F_CONDB;
    }
    st_s(a.p.nee1 + pid, f4(cB, mo.rrz));
    st_s(a.p.flags + pid, nf);
}

// k_shade: 8 waves per SIMD (<= 64 VGPRs; the virtual-block loop left alone allocates 67, no spill at 64)
#ifndef MCPT_SHADE_WPE
#define MCPT_SHADE_WPE 8
#endif
#if MCPT_SHADE_WPE > 0
#define MCPT_SHADE_ATTR __attribute__((amdgpu_waves_per_eu(MCPT_SHADE_WPE, MCPT_SHADE_WPE)))
#else
#define MCPT_SHADE_ATTR
#endif
#ifndef MCPT_MAT_WPE
#define MCPT_MAT_WPE 4  // 4 waves per SIMD (<= 128 VGPRs): without it the occluder-cache prefetch tips it to 130
#endif
#ifdef MCPT_MAT_WPE
#define MCPT_MAT_ATTR __attribute__((amdgpu_waves_per_eu(MCPT_MAT_WPE, MCPT_MAT_WPE)))
#else
#define MCPT_MAT_ATTR
#endif
// Shading block vb (k_shade's virtual block: kBlock consecutive pixels of one path slot and tile),
// decomposed once per launch by the k_shade workgroup that runs it (thread k for its k-th block, in
// the prologue, into LDS): the per-block integer divisions by the slot and tile sizes are VALU
// sequences (no scalar divide), which the block loop would otherwise repeat per wave and block.
//   x0, y0: film position of the block's first pixel (with tile_w a multiple of kBlock a block is one
//           run of a tile row, pixel x0 + k; otherwise x0, y0 are the tile's corner);
//   loc0:   path index within the slot of the first pixel (ShadeArgs::npx);
//   sr:     path slot | pixels of the block inside its tile << 8 (kBlock for all but a tile's last);
//   li0:    the first pixel's index in its tile;
//   done:   its finished-block flag, kept per slot, film tile and block so it outlives a change of
//           tile set.
struct VBlk { int x0, y0; uint32_t loc0, sr, li0, done; };
__device__ inline VBlk vblock_of(const ShadeArgs& a, int vb) {
    const int tile_px = a.tile_w * a.tile_h;
    const int bpt = (tile_px + kBlock - 1) / kBlock;
    // path slots: blocks [k * ntiles * bpt, (k + 1) * ntiles * bpt) run slot k of every pixel
    const int per_slot = a.ntiles * bpt;
    const int slot = a.slots > 1 ? vb / per_slot : 0;
    const int bs = vb - slot * per_slot;
    const int tile = bs / bpt;
    const int bib = bs - tile * bpt;
    const int li0 = bib * kBlock;
    const int2 t = a.tiles[tile];
    VBlk r;
    if (a.tile_w % kBlock == 0) {
        const int row = li0 / a.tile_w;
        r.x0 = t.x * a.tile_w + (li0 - row * a.tile_w);
        r.y0 = t.y * a.tile_h + row;
    } else {
        r.x0 = t.x * a.tile_w;
        r.y0 = t.y * a.tile_h;
    }
    // path index (ShadeArgs::npx): the pixel id, or its place in the compact tile-set layout
    r.loc0 = a.compact ? (uint32_t)(a.tile_base ? a.tile_base[tile] : tile) * (uint32_t)tile_px + (uint32_t)li0 : 0u;
    r.sr = (uint32_t)slot | ((uint32_t)min(tile_px - li0, kBlock) << 8);
    r.li0 = (uint32_t)li0;
    const uint32_t ntx = (uint32_t)((a.W + a.tile_w - 1) / a.tile_w), nty = (uint32_t)((a.H + a.tile_h - 1) / a.tile_h);
    r.done = (((uint32_t)slot * nty + (uint32_t)t.y) * ntx + (uint32_t)t.x) * (uint32_t)bpt + (uint32_t)bib;
    return r;
}
// floor(n / d) for n < 2^23, d >= 1, from rcp = RN32(1 / d): the truncated float product is q or
// q - 1 (relative error < 2^-22 on n / d, and 1 - frac(n / d) >= 1 / d), one correction
__device__ inline uint32_t udiv_small(uint32_t n, uint32_t d, float rcp) {
    uint32_t q = (uint32_t)((float)n * rcp);
    if (n - __umul24(q, d) >= d) q++;
    return q;
}

// One shading block: logic + generate for kBlock pixels of a path slot, then the block's pushes.
template <bool FIXED>
__device__ __attribute__((always_inline)) inline void shade_vblock(const ShadeArgs& a, int vb, const VBlk& v) {
    const DevScene& sc = a.scene;
    const int slot = (int)(v.sr & 0xffu);
    const int lane = threadIdx.x & 63;
    bool valid = (int)threadIdx.x < (int)(v.sr >> 8);
    uint32_t pid = 0, pix = 0;  // path id (slot * pixels + pixel) and pixel id
    int x = 0, y = 0;
    if (valid) {
        if (a.tile_w % kBlock == 0) {
            x = v.x0 + (int)threadIdx.x;
            y = v.y0;
        } else {
            const int li = (int)v.li0 + (int)threadIdx.x;
            x = v.x0 + li % a.tile_w;
            y = v.y0 + li / a.tile_w;
        }
        valid = x < a.W - 1 && y < a.H - 1;  // last column and row never rendered (wavefront_kernels.cu:110)
        pix = (uint32_t)y * (uint32_t)a.W + (uint32_t)x;
        pid = (uint32_t)slot * a.npx + (a.compact ? v.loc0 + threadIdx.x : pix);
    }
    // ---- phase 1: logic + generate (one thread per pixel)
    MCPT_MARK("load");
    bool gen_ext = false, gen_trivial = false, cont = false;
    bool d_logic = false, d_nee = false, d_gen = false;  // (MCPT_DIAG_SHADE)
    (void)d_logic; (void)d_nee; (void)d_gen;
    uint32_t cont_len = 0, cont_sidx = 0;
    int32_t cont_htri = -1;
    V3 beta_store = v3(0.f, 0.f, 0.f);
    // A primary ray that missed adds the background (env_L of its direction) to the film.
    // That is done after the pushes, where the logic's state is dead: the env lookup's
    // temporaries on top of the logic's live values set the kernel's register peak (81 VGPRs,
    // 5 waves per SIMD, against 48 without it).  Nothing else touches such a path's film in
    // this iteration, so the order of the two film updates does not change a bit.
    bool bg = false;
    V3 bg_film = v3(0.f, 0.f, 0.f), bg_dir = bg_film;
    bool finished = true;  // dead with its last sample done (or no pixel): see blk_done
    if (valid) {
        // Every load the logic may need is issued up front, in one round: the
        // per-path state unconditionally, the len-dependent streams (ray_d for a
        // primary miss, the MIS terms and visibility for len > 1) at pid when needed
        // and at a shared dummy index 0 otherwise (no extra bandwidth).
        const uint32_t fl = ld_s(a.p.flags + pid);
        const int32_t htri = ld_s(a.p.hit_tri + pid);
        const float4 b4 = ld_s(a.p.beta + ((((fl >> F_LEN_SHIFT) & 0xffu) > 1u) ? pid : 0u));  // len 1: beta is (1,1,1), not loaded
        const uint32_t len = (fl >> F_LEN_SHIFT) & 0xffu;
        const bool need_rd = len == 1 && htri < 0;
        const bool need_nee = len <= (uint32_t)a.max_depth && len > 1;
        // The film is read only where the logic can add to it: a primary miss (background)
        // or a vertex with MIS terms.  Elsewhere the update is film + 0 * beta, which leaves
        // the film's bits unchanged (Ld is never -0: it starts at +0 and every update adds to
        // it), so neither the load nor the store is needed.
        const bool need_ld = !(fl & F_DEAD) && (need_rd || need_nee);
        const V3 ld4 = ld3f4(a.p.Ld + (need_ld ? pid : 0u));  // .w is always 0 (k_clear, k_resolve): xyz only
        const V3 rd = ld3f4(a.p.ray_d + (need_rd ? pid : 0u));
        const float4 n0 = ld_s(a.p.nee0 + (need_nee ? pid : 0u)), n1 = ld_s(a.p.nee1 + (need_nee ? pid : 0u));
        const uchar2 vv = reinterpret_cast<const uchar2*>(a.p.vis)[need_nee ? pid : 0u];
        bool dead = (fl & F_DEAD) != 0;
        const uint32_t spp = (uint32_t)a.spp;
        // this slot's sample index (slot k runs samples k, k + S, ...; S = 1: the count itself):
        // the flags word carries it, the one in progress for a live path (k_material keys its
        // draws with it) and the next one for a dead path (k_clear: the slot's first), so the
        // film's sample count is (sidx - slot) / S and its stream is only written
        uint32_t sidx = fl >> F_SIDX_SHIFT;
        uint32_t samples = a.slots > 1 ? udiv_small(sidx - (uint32_t)slot, (uint32_t)a.slots, a.slots_rcp) : sidx;
        if (!dead && sidx < spp) {  // wavefront_kernels.cu:124
            MCPT_MARK("logic");
            d_logic = true;
            d_nee = need_nee;
            const Rng r{rng_key(a.seed, pix, sidx), len};
            const bool found = htri >= 0;
            const V3 B = len == 1 ? v3(1.f, 1.f, 1.f) : xyz(b4);  // wf_generate's beta (:245)
            V3 film = ld4;
            bool terminate = false;
            beta_store = B;
            if (len == 1) {  // :129-140
                if (found) {
                    film = film + v3(0.f, 0.f, 0.f) * B;
                } else {  // background (:135-138): added below, after the pushes
                    bg = true;
                    bg_film = film;
                    bg_dir = rd;
                }
            }
            if (len > (uint32_t)a.max_depth || !found) terminate = true;  // :142-146
            if (need_nee) {                                                // :150-197
                const uint8_t vl = vv.x, vb = vv.y;
                V3 acc = v3(0.f, 0.f, 0.f);
                if ((fl & F_CONDL) && vl) acc = acc + xyz(n0);
                if (fl & F_HASVIS) {
                    if (vb) { if (fl & F_CONDB) acc = acc + xyz(n1); }
                    else acc = acc + v3(0.f, 0.f, 0.f);
                } else {
                    acc = acc + v3(0.f, 0.f, 0.f);  // delta light: f_brdf = 0, weights 0.5
                }
                film = film + acc * B;
                if (fl & F_FZERO) {
                    terminate = true;
                } else {
                    beta_store = B * v3(b4.w, n0.w, n1.w);  // paths->beta *= f_sample / pdf_sample (:187)
                    if (len > (uint32_t)a.rr_depth) {        // :189-196
                        if (FIXED) {  // q from the updated throughput, survivors reweighted (A.5)
                            float q = fmx(0.05f, 1.f - beta_store.y);
                            if (r(SL_RR) < q) terminate = true;
                            else beta_store = beta_store / (1.f - q);
                        } else {
                            float q = fmx(0.05f, 1.f - B.y);
                            if (r(SL_RR) < q) terminate = true;
                        }
                    }
                }
            }
            // film unchanged bit for bit (a zero contribution): the store would rewrite the same bytes
            if (need_ld && (__float_as_uint(film.x) != __float_as_uint(ld4.x) ||
                            __float_as_uint(film.y) != __float_as_uint(ld4.y) ||
                            __float_as_uint(film.z) != __float_as_uint(ld4.z)))
                st_s(a.p.Ld + pid, f4(film, 0.f));
            if (terminate) {  // :199-204
                dead = true;
                samples++;
                sidx += (uint32_t)a.slots;
                st_s(a.p.samples + pid, samples);
            } else {
                cont = true;
                cont_len = len;
                cont_sidx = sidx;
                cont_htri = htri;
            }
        }
        uint32_t nflags = fl;
        if (dead) nflags = F_DEAD | (sidx << F_SIDX_SHIFT);
        if (dead && sidx < spp) {  // :219-222 + wf_generate (:225-251)
            MCPT_MARK("generate");
            d_gen = true;
            // dCamera::gen_ray (Camera.cu:18-45): the pixel's part from its camera record
            // (k_cam_table), the thin lens per sample
            V3 new_o = ld3f4(a.cam_px + pix), new_d;
            if (a.cam.lens_radius > 0.f) {
                const Rng r0{rng_key(a.seed, pix, sidx), 0u};
                gen_ray_lens(a.cam, new_o, r0, new_o, new_d);
            } else {
                new_d = ld3f4(a.cam_dir + pix);
            }
            // beta = (1,1,1) (:245) is implied by len 1: k_shade does not load it for len-1 paths
            nflags = (1u << F_LEN_SHIFT) | (sidx << F_SIDX_SHIFT);
            st_s(a.p.ray_o + pid, f4(new_o, 0.f));
            st_s(a.p.ray_d + pid, f4(new_d, 0.f));
            gen_ext = true;
            if (ray_misses_scene(sc, new_o, new_d)) {  // resolved here: isect stays "not found"
                a.p.hit_tri[pid] = -1;
                gen_ext = false;
                gen_trivial = true;
            }
        }
        MCPT_MARK("flags");
        if (!cont && nflags != fl) st_s(a.p.flags + pid, nflags);  // continuing paths: written by material()
        finished = dead && !(sidx < spp);
    }
    SHADE_DIAG(SD_WAVES, true);
    SHADE_DIAG(SD_VALID, valid);
    SHADE_DIAG(SD_LOGIC, d_logic);
    SHADE_DIAG(SD_NEE, d_nee);
    SHADE_DIAG(SD_GEN, d_gen);
    SHADE_DIAG(SD_CONT, cont);
    SHADE_DIAG(SD_BG, bg);
    MCPT_MARK("push");
    // ---- pushes: generated extension rays and continuing paths (material queue); one
    // atomic per block and queue.  A continuing path's record and updated throughput go
    // to k_material densely (it writes p.beta with f_s/pdf_s in .w).
    const int shard = vb % kShards;  // the queues' capacity assumes <= kBlock pushes per block and shard
    uint32_t* sc_ctr = a.cnt->shard[shard];
    {
        bool want[2] = {gen_ext, cont};
        uint32_t* ctr[2] = {sc_ctr + C_EXT, sc_ctr + C_MAT};
        uint32_t slot[2], total[2];
        block_push<2>(want, ctr, slot, total);
        if (gen_ext) st_q(a.ext_q + shard * a.ext_cap + slot[0], pid);
        if (cont) {
            const uint32_t qi = shard * a.ext_cap + slot[1];
            st_s(a.mat_rec + qi, make_uint4(pid, pix, cont_sidx | (cont_len << kRecLenShift), (uint32_t)cont_htri));
            st_s(a.mat_beta + qi, f4(beta_store, 0.f));
        }
    }
    uint32_t n_ext = (gen_ext || gen_trivial) ? 1u : 0u;  // queued + resolved-in-place rays
    for (int off = 32; off > 0; off >>= 1) n_ext += __shfl_xor(n_ext, off);
    if (lane == 0 && n_ext) atomicAdd(sc_ctr + C_EXT_RAYS, n_ext);
    MCPT_MARK("background");
    if (bg) {  // wavefront_kernels.cu:129-140, len 1 and no hit: beta is (1,1,1)
        const int nbg = FIXED ? 1 : sc.nlights;  // the reference adds it once per light (A.4)
        V3 film = bg_film;
        for (int i = 0; i < nbg; i++) film = film + env_L(sc.env, bg_dir) * v3(1.f, 1.f, 1.f);
        if (__float_as_uint(film.x) != __float_as_uint(bg_film.x) || __float_as_uint(film.y) != __float_as_uint(bg_film.y) ||
            __float_as_uint(film.z) != __float_as_uint(bg_film.z))
            a.p.Ld[pid] = f4(film, 0.f);
    }
    MCPT_MARK("done");
    if (a.blk_done && __syncthreads_and(finished ? 1 : 0) && threadIdx.x == 0) a.blk_done[v.done] = 1;
    MCPT_MARK("end");
}

// k_shade: a bounded grid of G blocks; block b runs shading blocks b, b + G, b + 2G, ... (at most
// kBlock of them: launch_shade sizes G).  A block whose paths have all finished their last sample
// stays so until the film is cleared, so it is skipped: thread k reads the flag of the block's k-th
// shading block, all in one round trip, and the block loops over the live ones.  A one-pass grid
// (one workgroup per shading block, G = the block count) paid ~0.2 ms per launch just to dispatch
// and retire config 2's 246K workgroups once they had all finished (the frame's last ~20
// iterations; 64 iterations per frame).
template <bool FIXED>
__global__ __launch_bounds__(kBlock) MCPT_SHADE_ATTR void k_shade(ShadeArgs a) {
    if (a.cnt->idle) return;  // the tile set is complete (an earlier iteration of the call traced no ray)
    __shared__ uint64_t s_live[kBlock / 64];
    const uint32_t G = gridDim.x, nvb = a.shade_vblocks;
    const uint32_t mine = (nvb - blockIdx.x + G - 1) / G;  // <= kBlock
    const uint32_t k = threadIdx.x;
    bool live = false;
    __shared__ VBlk s_vb[kBlock];  // thread k: the block's k-th shading block (vblock_of)
    if (k < mine) {
        const VBlk v = vblock_of(a, (int)(blockIdx.x + k * G));
        live = !a.blk_done || a.blk_done[v.done] == 0;
        s_vb[k] = v;
    }
    const uint64_t m = __ballot(live);
    if ((threadIdx.x & 63) == 0) s_live[threadIdx.x >> 6] = m;
    __syncthreads();
    for (uint32_t j = 0; j < mine; j++) {
        if (!((s_live[j >> 6] >> (j & 63)) & 1ull)) continue;
        // the arguments re-read per shading block (kernarg_fresh): hoisted out of the loop, the
        // struct's fields took the SGPR file and spilled (89 SGPRs, 54 -> 86 VGPRs)
        shade_vblock<FIXED>(kernarg_fresh<ShadeArgs>(), (int)(blockIdx.x + j * G), s_vb[j]);
    }
}

// ---------------------------------------------------------------------------
// k_material: light choice + wf_mat_mix (wavefront_kernels.cu:207-215, 295-375) for
// the paths k_shade found continuing, dense over the material queue: 256 paths per
// block and trip, so every wave of a block has the same (heavy) work and the block
// pushes meet at the barrier together.  Block b serves shard b mod kShards, chunks
// b / kShards, + gridDim.x / kShards, ... of it (grid from the occupancy calculator).
// ---------------------------------------------------------------------------
template <bool FIXED>
__global__ __launch_bounds__(kBlock) MCPT_MAT_ATTR void k_material(ShadeArgs a_kernarg) {
    (void)a_kernarg;  // read through kernarg_fresh (the same bytes: it is the kernel's only argument)
    const ShadeArgs& a = kernarg_fresh<ShadeArgs>();
    if (a.cnt->idle) return;  // the tile set is complete
    const uint32_t shard = blockIdx.x % kShards, w_in = blockIdx.x / kShards, bps = gridDim.x / kShards;
    uint32_t* sc_ctr = a.cnt->shard[shard];
    const uint32_t n = sc_ctr[C_MAT];
    const int lane = threadIdx.x & 63;
    uint32_t n_ext = 0, n_any = 0, n_vis = 0, n_occ = 0, occ_try = 0;
    const bool occ_on = a.scene.occ && a.scene.occ_gate[0] == 0 && a.scene.occ_gate[2] != 0;  // see DevScene::occ_gate
    // Any-hit rays are staged here (light ray o/d, BRDF visibility ray o/d) and stored after
    // the block push at their queue positions: the block's rays of one kind land contiguously,
    // so k_trace reads them densely and without the queue-entry hop (the pid-indexed layout
    // wrote and read 32-B pieces of partly used lines).
    __shared__ float4 s_any[4][kBlock];
    for (uint32_t base = w_in * kBlock; base < n; base += bps * kBlock) {  // block-uniform trip count
        const ShadeArgs& a = kernarg_fresh<ShadeArgs>();  // this trip's loads (see kernarg_fresh)
        const uint32_t i = base + threadIdx.x;
        MatOut mo{};
        uint32_t mpid = 0;
        bool occ_l = false, occ_b = false, try_l = false, try_b = false;  // resolved by / tested against the occluder cache
        if (i < n) {
            const uint4 q = ld_s(a.mat_rec + shard * a.ext_cap + i);  // {pid, pixel, sample index | len << 24, hit_tri}
            const float4 b4 = ld_s(a.mat_beta + shard * a.ext_cap + i);
            mpid = q.x;
            mo = material<FIXED>(a, mpid, q.y, q.z & ((1u << kRecLenShift) - 1u), q.z >> kRecLenShift, xyz(b4),
                                 (int32_t)q.w, &s_any[0][0], occ_on);
            // the occluder cache (see occ_hit1), before the BRDF sample's light terms: a ray it
            // resolves gets its wf_shadow result here and is not queued
            MCPT_MARK("m_occ");
            if (occ_on) {
                try_l = mo.want_l;
                try_b = mo.want_b;
                const V3 ol = xyz(s_any[0][threadIdx.x]), dl = xyz(s_any[1][threadIdx.x]);
                const V3 ob = xyz(s_any[2][threadIdx.x]), db = xyz(s_any[3][threadIdx.x]);
                if (mo.want_l) occ_l = occ_hit1(a.scene, ol, dl, mo.el);
                if (mo.want_b) occ_b = occ_hit1(a.scene, ob, db, mo.eb);
                if (occ_l) {
                    a.p.vis[2 * mpid] = 0;
                    mo.want_l = false;
                    mo.trivial_any++;
                }
                if (occ_b) {
                    a.p.vis[2 * mpid + 1] = 0;
                    mo.want_b = false;
                    mo.need_cb = false;
                    mo.trivial_any++;
                }
            }
            MCPT_MARK("m_bterms");
            material_brdf_terms<FIXED>(a, mpid, mo);
        }
        MCPT_MARK("m_push");
        bool want[3] = {mo.want_ext, mo.want_l, mo.want_b};
        uint32_t* ctr[3] = {sc_ctr + C_EXT, sc_ctr + C_ANY, sc_ctr + C_ANY};
        uint32_t slot[3], total[3];
        block_push<3>(want, ctr, slot, total);
        if (mo.want_ext) st_q(a.ext_q + shard * a.ext_cap + slot[0], mpid);
        // (the any-hit rays carry their result index in o.w: no queue entries)
        if (mo.want_l) {
            const uint32_t k = shard * a.any_cap + slot[1];
            if constexpr (MCPT_NT & 8) {
                st_s(a.p.sray_o + k, s_any[0][threadIdx.x]);
                st_s(a.p.sray_d + k, s_any[1][threadIdx.x]);
            } else {
                a.p.sray_o[k] = s_any[0][threadIdx.x];
                a.p.sray_d[k] = s_any[1][threadIdx.x];
            }
        }
        if (mo.want_b) {
            const uint32_t k = shard * a.any_cap + slot[2];
            if constexpr (MCPT_NT & 8) {
                st_s(a.p.sray_o + k, s_any[2][threadIdx.x]);
                st_s(a.p.sray_d + k, s_any[3][threadIdx.x]);
            } else {
                a.p.sray_o[k] = s_any[2][threadIdx.x];
                a.p.sray_d[k] = s_any[3][threadIdx.x];
            }
        }
        MCPT_MARK("m_count");
        // per-wave ray counts from lane masks (wave-uniform scalars: no registers held across the
        // next trip's material())
        n_occ += (uint32_t)(__popcll(__ballot(occ_l)) + __popcll(__ballot(occ_b)));
        occ_try += (uint32_t)(__popcll(__ballot(try_l)) + __popcll(__ballot(try_b)));
        n_ext += (uint32_t)__popcll(__ballot(mo.want_ext || mo.trivial_ext));  // queued + resolved-in-place rays
        n_any += (uint32_t)(__popcll(__ballot(mo.want_l)) + __popcll(__ballot(mo.want_b)) +
                            __popcll(__ballot(mo.trivial_any >= 1u)) + __popcll(__ballot(mo.trivial_any >= 2u)));
        n_vis += (uint32_t)__popcll(__ballot(mo.vis_ray));
    }
    if (lane == 0) {
        if (n_ext) atomicAdd(sc_ctr + C_EXT_RAYS, n_ext);
        if (n_any) atomicAdd(sc_ctr + C_ANY_RAYS, n_any);
        if (n_vis) atomicAdd(sc_ctr + C_VIS, n_vis);
        if (n_occ) atomicAdd(sc_ctr + C_OCC, n_occ);
        if (occ_try) atomicAdd(sc_ctr + C_OCC_TRY, occ_try);
    }
}

// ---------------------------------------------------------------------------
// BVH traversal (BVH.cu:115-207 closest hit, Triangle.cu:157-205 any hit).
// Child-pair nodes (both child boxes in the parent, 64 B) with the reference's
// slab arithmetic per box (Bounds3f.h:121-153).  Culling beyond the reference
// (which visits every box the infinite line crosses) is provably conservative: a box
// is skipped only when no triangle in it can be accepted with t >= 0 or below the
// best t, for any angle between the ray and the triangle, by the Moller-Trumbore
// error bound of mcpt_core.hpp ("conservative box culling": each child carries its
// margin W, keep_box).  Ties on t go to the lower triangle index, so the visit order
// is free (near child first here, by the cull key t0 - W iota).
//
// One persistent kernel traces both ray sets of an iteration: set 0 closest hit
// (extension rays -> hit_tri), set 1 any hit (light and BRDF visibility rays ->
// vis).  The grid is sized to the resident wave count.  The queue shards are
// grouped into partitions (two per XCD); a partition's set-0 entries followed by
// its set-1 entries are read as one sequence of rays, handed out by one atomic
// counter per partition whenever enough lanes of a wave are idle at the top of
// the loop (waves whose partition ran dry join another one; see below).  Each
// loop trip a lane does up to kNodeSteps child-pair (or 4-wide) node tests, then
// (in the wave-uniform triangle phase) one triangle of its parked leaf.  Reaching
// a leaf parks it and traversal continues speculatively from the stack, so node
// and triangle work are executed by full waves rather than interleaved per lane.
// Stack: kLdsStack entries per lane in LDS ([entry][lane], conflict-free), deeper
// entries in private scratch.
// ---------------------------------------------------------------------------
// Inclusive scan over the 64 lanes of a wave with DPP moves (no ds_bpermute address
// registers): Hillis-Steele within each 16-lane row (row_shr 1/2/4/8; lanes shifted past
// their row's start add the 0 'old' operand), then row 15's total into rows 1 and 3
// (row_bcast:15) and lane 31's into rows 2 and 3 (row_bcast:31).
__device__ inline uint32_t wave_scan_incl(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Traversal work counters: wave-reduce, one atomic per counter per wave.
__device__ inline void wave_stats(uint32_t* stats, int lane, uint32_t nodes, uint32_t tests, uint32_t hits) {
    if (!stats) return;
    for (int off = 32; off > 0; off >>= 1) {
        nodes += __shfl_xor(nodes, off);
        tests += __shfl_xor(tests, off);
        hits += __shfl_xor(hits, off);
    }
    if (lane == 0) {
        uint32_t* st = stats + (blockIdx.x % kShards) * C_WORDS;
        atomicAdd(st + 0, nodes);
        atomicAdd(st + 1, tests);
        atomicAdd(st + 2, hits);
    }
}

#ifndef MCPT_NODE_STEPS
#define MCPT_NODE_STEPS 4
#endif
// Shared triangle phase (MCPT_TRI_SHARE=1; measured and not kept): a triangle
// phase tests every triangle of every parked leaf of the wave, dealt over all 64 lanes (a lane tests
// another lane's ray against one of that lane's triangles), instead of one triangle per lane holding
// a leaf.  Parity held (110 GPU tests), but config 2's k_trace went 2.47 -> 2.79 ms per launch: the
// upload expands every multi-triangle leaf into pair nodes over one-triangle leaves (their own
// boxes: the tree-independent acceptance), so a parked leaf is one triangle and a phase holds 36 of
// them on average (6.91 G tests in 190 M phases, the same with and without sharing); one round per
// phase then does the same tests with the owner search and ray exchange on top.  Applies to the instantiations with an LDS stack of <= kShareMaxStack
// entries (its 512-B result slots per wave would cost the deep-stack kernels a resident wave per CU).
#ifndef MCPT_TRI_SHARE
#define MCPT_TRI_SHARE 0
#endif
constexpr int kShareMaxStack = 8;
constexpr int kNodeSteps = MCPT_NODE_STEPS;
#ifndef MCPT_GRAB_MAX
#define MCPT_GRAB_MAX 0
#endif
constexpr int kGrabMax = MCPT_GRAB_MAX;  // rays one hand-out atomic may reserve for a wave (<= 64: only the idle lanes)
// Order of a partition's ray sequence: extension rays first (MCPT_ANY_FIRST=1: the costlier
// any-hit rays first, so the tail is made of cheap rays -- measured mixed: config 2 k_trace
// 0.779 -> 0.791 ms, config 3 1.149 -> 1.129, config 5 17.09 -> 17.27).
#ifndef MCPT_ANY_FIRST
#define MCPT_ANY_FIRST 0
#endif
constexpr bool kAnyFirst = MCPT_ANY_FIRST != 0;
// A trip's node phase ends for every lane once fewer than this many lanes still have node work (0:
// each lane takes its kNodeSteps steps); the others resume next trip, after the triangle phase and
// a refill of the idle lanes.  Per instantiation, from a sweep of 0/24/32/40/48 (interleaved A/B,
// one box, whole frames; profiles/ab_r05_node_min.txt): child pairs with the 8-entry stack
// (config 2) 32: k_trace 2.54 -> 2.47 ms, frame -1.9 %; 4-wide nodes (configs 3, 5) 24: config 3
// 2.70 -> 2.45 ms (-6 % frame), config 5 17.7 -> 16.9 ms (-3.4 %); child pairs with the deep stack
// (config 4, 26 pair steps per ray) 0: 24 / 32 were 1.2 / 2.6 % slower.
#ifndef MCPT_NODE_MIN_LANES2
#define MCPT_NODE_MIN_LANES2 32
#endif
#ifndef MCPT_NODE_MIN_LANES2_DEEP
#define MCPT_NODE_MIN_LANES2_DEEP 0
#endif
#ifndef MCPT_NODE_MIN_LANES4
#define MCPT_NODE_MIN_LANES4 24
#endif

// Waves per SIMD: 7 (<= 72 VGPRs) for child pairs with either LDS stack, 6 (80) for 4-wide nodes
// (8 float4 of node data per step).  The attribute lets the register allocator park the
// partition scan's loop-invariant lane addresses (and a few scalars) in scratch -- reloaded only
// by the scan -- instead of giving up a wave.  Round 2 ran the pair kernel at 8 waves (64 VGPRs:
// config 2 0.758 ms against 0.777 at 7); the culling bound's per-ray scale (cull_iota, round 4)
// is one register too many there: 8 spilled VGPRs in the loop, config 2 2.74 against 2.52 ms
// per launch at 7 (interleaved, one box).
#ifndef MCPT_TRACE_WPE
#define MCPT_TRACE_WPE 7
#endif
#ifndef MCPT_TRACE_WPE_DEEP
#define MCPT_TRACE_WPE_DEEP 7
#endif
#ifndef MCPT_TRACE_WPE4
#define MCPT_TRACE_WPE4 6
#endif
#define MCPT_TRACE_WPE_OF(kW, kS) \
    ((kW) == 4 ? MCPT_TRACE_WPE4 : ((kS) > ::mcpt_dev::kLdsStack ? MCPT_TRACE_WPE_DEEP : MCPT_TRACE_WPE))
#define MCPT_TRACE_ATTR \
    __attribute__((amdgpu_waves_per_eu(MCPT_TRACE_WPE_OF(kW, kLdsStack), MCPT_TRACE_WPE_OF(kW, kLdsStack))))
// node width (2: child pairs, 4: quads), LDS stack entries per lane, work counters (TraceSet::stats)
template <int kW, int kLdsStack, bool kCount>
__global__ __launch_bounds__(kTraceBlock) MCPT_TRACE_ATTR void k_trace(TraceArgs a) {
    if (a.idle && *a.idle) return;  // the tile set is complete
    constexpr bool kShare = MCPT_TRI_SHARE != 0 && kLdsStack <= kShareMaxStack;
    __shared__ int2 stk[kLdsStack][kTraceBlock];
    // shared triangle phase: each lane's best (t, scene id, leaf position) key, min-combined by the
    // lanes testing its triangles
    __shared__ uint64_t s_key[kShare ? kTraceBlock : 1];
    const int lane = threadIdx.x;
    // ---- work distribution.  The queue shards are split into nparts partitions
    // (shard s -> partition s mod nparts; by default one per XCD) and each partition's
    // rays are handed out by one agent-scope atomic counter (gfx950 performs these at
    // the memory side: the same instruction as a workgroup-scope add, coherent across
    // XCDs).  A wave starts on the partition of the die it runs on (hardware XCC id:
    // the counter's line and the partition's rays stay in that die's L2 -- a speed
    // choice only).  Once that partition is drained and the wave has no ray left, it
    // reads every partition's counter and joins the first one (after its own, in
    // rotation) that still holds rays; it exits when all of them read drained.  So
    // every queued ray is traced whatever the placement of waves on dies (a die with
    // no waves, more partitions than dies), and k_accumulate checks per launch that
    // every counter reached its partition's ray count.  A static split left the waves
    // of a launch finishing anywhere between 52 % and 100 % of its duration
    // (tools/wave_times.py).
    const uint32_t nsh = (uint32_t)a.nshards, nparts = a.nparts;
    uint32_t home = 0;
    if (nparts > 1) {
        uint32_t xcc;
        __asm__ volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        // several partitions per die (nparts a multiple of the die count): consecutive
        // blocks of a die (blocks are dealt round-robin over the dies) alternate between them
        const uint32_t nd = a.ndies >= 1 && a.ndies <= nparts && nparts % a.ndies == 0 ? a.ndies : nparts;
        home = (xcc & 15u) % nd + nd * ((blockIdx.x / nd) % (nparts / nd));  // (nd: XCC ids 0..7)
    }
    // rays per partition (s_tot), for the drained test of the partition scan
    __shared__ uint32_t s_tot[kMaxParts];
    if (lane < kMaxParts) s_tot[lane] = 0;
    __syncthreads();
    if ((uint32_t)lane < nsh) {
        uint32_t n = 0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const TraceSet& ts = a.set[k];
            n += ts.count_ptr ? ts.count_ptr[lane * C_WORDS] : (lane == 0 ? ts.count : 0u);
        }
        if (n) atomicAdd(&s_tot[lane % nparts], n);
    }
    __syncthreads();
    // Partition entries: its shards part, part + nparts, ... (spart of them) of set 0,
    // then the same shards of set 1 (at most 2 * 64 entries: one per lane and half),
    // read as one sequence of rays.  pre(e) = first position of entry e (exclusive prefix;
    // entries past the last and pre(128)
    // give the total), kept in LDS (s_pre): the kernel has to stay at <= 72 VGPRs for 7
    // waves per SIMD (gfx950 allocates VGPRs in blocks of 8 here: 73..80 -> 6 waves).
    // Rays are handed out exactly as lanes fall idle (an atomic add of the idle count):
    // a wave reserves no rays ahead, so when the partition runs dry each wave only
    // finishes its lanes.  (The block is one wave: s_pre is rewritten in program order
    // after its last read.)
    __shared__ uint32_t s_pre[129];
    uint32_t part = home, spart = 0, T = 0;  // T: rays in the current partition
    uint32_t* grab = a.grab;
    bool more = false;  // the current partition may still hold rays
    // join partition p: its entry prefix into s_pre, its ray count into T
    auto enter = [&](uint32_t p) {
        part = __builtin_amdgcn_readfirstlane(p);  // (wave-uniform: keep it, spart and T in SGPRs)
        spart = __builtin_amdgcn_readfirstlane(nsh > part ? (nsh - part + nparts - 1) / nparts : 0u);
        // the two halves one after the other: this code sits inside the traversal loop,
        // where every temporary counts against the VGPR budget of 7 waves per SIMD
        uint32_t base = 0;
#pragma unroll 1
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t e = (uint32_t)lane + 64u * h;
            const bool k1 = kAnyFirst ? e < spart : e >= spart;  // entry e belongs to set 1 (any hit)
            const uint32_t j = e >= spart ? e - spart : e;
            uint32_t ne = 0;
            if (e < 2 * spart) {
                const TraceSet& ts = k1 ? a.set[1] : a.set[0];
                const uint32_t sh = part + j * nparts;
                ne = ts.count_ptr ? ts.count_ptr[sh * C_WORDS] : (sh == 0 ? ts.count : 0u);
            }
            const uint32_t inc = wave_scan_incl(ne);
            s_pre[e] = base + inc - ne;
            base += __builtin_amdgcn_readlane(inc, 63);
        }
        T = __builtin_amdgcn_readfirstlane(base);
        if (lane == 0) s_pre[128] = T;
        __syncthreads();
        grab = a.grab + part * C_WORDS;
        more = T > 0;
    };
    enter(home);
    const DevScene& sc = a.scene;
    // occluder-cache records (see occ_hit1): off while k_material's lookups are gated off, except in
    // the iteration before the next lookups (DevScene::occ_gate)
    const bool occ_rec = sc.occ && sc.occ_gate[0] <= 1u;

    // Work counters (only the kCount instantiation: six long-lived per-lane registers cost the
    // 64-VGPR, 8-wave kernel its spill-free hot loop).  tot_* count every node step, triangle
    // test and hit; the any-hit set's share is attributed per ray (tot_n1 -= tot_n when an
    // any-hit ray starts, += when it finishes), so a step costs one add.
    uint32_t tot_n = 0, tot_t = 0, tot_h = 0, tot_n1 = 0, tot_t1 = 0, tot_h1 = 0;
    uint32_t ph[kPhaseWords] = {};  // loop-phase counts (kCount only; wave-uniform)
    uint64_t drained = 0;  // partitions this wave saw run dry (by an atomic: never stale)
    for (;;) {  // one trip per partition joined
    // Per-lane ray state is declared per partition trip: when the trip ends no lane holds a
    // ray, so none of it is live across the partition scan below (VGPR budget).
    uint32_t buf_lo = 0, buf_hi = 0, last_p = 0;  // wave-uniform reservation of the partition (refill)
    bool act = false;
    uint32_t rid = 0;
    // origin and inverse direction axis by axis as (o_a, 1 / d_a) register pairs (pair_slab2)
    f2v px = {0.f, 0.f}, py = px, pz = px;
    V3 d = v3(0.f, 0.f, 0.f);
#define RAY_O v3(px.x, py.x, pz.x)
#define RAY_INV v3(px.y, py.y, pz.y)
    int ref = kEnd, leaf = kEnd, sp = 0, tri = -1;
    // best: the closest hit's t, or -1 for an any-hit ray (its kind: best < 0; an accepted t is never
    // below +-0); io: the ray's signed culling scale (cull_iota; |io| = inf: an infinite inverse
    // component, the slab() path)
    float best = K_HUGE, cut = K_HUGE, io = K_INF_F;
    uint32_t bsid = 0;  // shared triangle phase: scene id of the closest hit so far (tri >= 0)
    int2 spill[kMaxStack - kLdsStack];
    // Pop the next entry still in front of the current cut (any-hit rays keep
    // cut = +inf, so for them every entry is taken).
    auto pop = [&]() -> int {
        while (sp > 0) {
            sp--;
            int2 e;
            if (sp < kLdsStack) {
                e = stk[sp][lane];
            } else {
                e = spill[sp - kLdsStack];
                __asm__ volatile("" : "+v"(e.x), "+v"(e.y));  // keep the LDS load an LDS load (no flat merge)
            }
            if (__int_as_float(e.y) > cut) continue;
            return e.x;
        }
        return kEnd;
    };
    auto finish = [&]() {
        const bool kind = best < 0.f;
        if constexpr (kCount) {
            tot_h += tri >= 0 ? 1u : 0u;
            if (kind) {
                tot_n1 += tot_n;
                tot_t1 += tot_t;
                tot_h1 += tri >= 0 ? 1u : 0u;
            }
        }
        if (kind) {
            // (rid: the result index -- a dense set's ray carried it in o.w, see the refill)
            if constexpr (MCPT_NT & 4) __builtin_nontemporal_store((uint8_t)(tri < 0), a.vis + rid);
            else a.vis[rid] = (uint8_t)(tri < 0);  // wf_shadow (wavefront_kernels.cu:274-293)
            if (tri >= 0 && occ_rec) {  // the cell's occluder (occ_hit1)
                // (hashed again here rather than kept from d.w: a register held over the whole
                // traversal, or a reload of the record, costs more than the hash on occluded rays)
                uint32_t* w = sc.occ + (size_t)occ_index(sc, RAY_O, d) * kOccWays + (uint32_t)tri % kOccWays;
                if constexpr (MCPT_NT & 16) __builtin_nontemporal_store((uint32_t)tri, w);
                else *w = (uint32_t)tri;
            }
        } else {
            if constexpr (MCPT_NT & 4) __builtin_nontemporal_store(tri, a.hit_tri + rid);
            else a.hit_tri[rid] = tri;  // hit record rebuilt by the consumer (hit_record())
        }
        act = false;
    };
    for (;;) {
        // ---- refill idle lanes with the partition's next rays
        MCPT_MARK("t_top");
        const uint64_t idle = __ballot(!act);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if ((more || buf_lo < buf_hi) && (nidle >= a.refill_min || nidle == 64u)) {
            // Positions come from a per-wave reservation [buf_lo, buf_hi) of the partition,
            // refilled by one atomic when empty.  By default (kGrabMax 0) an atomic reserves
            // exactly the idle lanes' rays.  Reserving more (a share of what is left, up to
            // kGrabMax, so later refills skip the atomic's round trip: a refill is three
            // dependent memory round trips, 7.3K cycles in the profile build) measured slower
            // on config 2: k_trace 0.775 / 0.785 / 0.812 / 0.874 ms at 0 / 128 / 256 / 512 --
            // other waves hide the refill latency, the reserved backlog lengthens the tail.
            if (buf_lo >= buf_hi) {
                uint32_t G = nidle;
                if (kGrabMax > 64) {
                    const uint32_t rem = T > last_p ? T - last_p : 0u;
                    const uint32_t wpp = max(1u, gridDim.x / nparts);
                    G = max(nidle, min((uint32_t)kGrabMax, rem / (2u * wpp)));
                }
                uint32_t g0 = 0;
                if (lane == 0) g0 = __hip_atomic_fetch_add(grab, G, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                g0 = __builtin_amdgcn_readfirstlane(g0);
                last_p = g0 + G;
                if (g0 + G >= T) {  // the rest of the partition is taken
                    more = false;
                    drained |= 1ull << part;
                }
                buf_lo = g0;
                buf_hi = g0 < T ? min(g0 + G, T) : g0;
            }
            MCPT_MARK("t_refill");
            const uint32_t p0 = buf_lo;
            const uint32_t take = min(nidle, buf_hi - buf_lo);
            buf_lo += take;
            if constexpr (kCount) {
                ph[PH_REFILLS]++;
                ph[PH_REFILL_LANES] += take;
            }
            const uint32_t q = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            const uint32_t pos = p0 + q;  // meaningful on idle lanes
            // entry of the first position: the last e with pre(e) <= p0 (a non-empty one)
            const uint32_t e0 = take ? (uint32_t)__popcll(__ballot(s_pre[lane] <= p0)) +
                                           (uint32_t)__popcll(__ballot(s_pre[64 + lane] <= p0)) - 1u
                                     : 0u;
            if (!act) {
                if (q < take) {
                    uint32_t my_e = e0;
                    while (pos >= s_pre[my_e + 1]) my_e++;  // the grab spans entries (rarely a step)
                    const uint32_t my_pre = s_pre[my_e];
                    const bool kind = kAnyFirst ? my_e < spart : my_e >= spart;
                    const uint32_t sh = part + (my_e >= spart ? my_e - spart : my_e) * nparts;
                    const uint32_t qslot = sh * (kind ? a.set[1].shard_cap : a.set[0].shard_cap) + (pos - my_pre);
                    // select the set's fields with ternaries: indexing a.set[kind] with a
                    // per-lane kind makes hipcc fetch them from kernarg memory per lane
                    const uint32_t* qp = kind ? a.set[1].queue : a.set[0].queue;
                    const float4* rop = kind ? a.set[1].ro : a.set[0].ro;
                    const float4* rdp = kind ? a.set[1].rd : a.set[0].rd;
                    // a dense set (ray_at_slot: the any-hit rays k_material stores at their queue
                    // positions) issues its ray loads with the queue-entry load, not after it
                    const bool at_slot = kind ? a.set[1].ray_at_slot : a.set[0].ray_at_slot;
                    float4 o4, d4;
                    if constexpr (MCPT_NT & 4) {
                        rid = at_slot ? qslot : (qp ? __builtin_nontemporal_load(qp + qslot) : qslot);
                        o4 = ld_s(rop + rid);
                        d4 = ld_s(rdp + rid);
                    } else {
                        rid = at_slot ? qslot : (qp ? qp[qslot] : qslot);
                        o4 = rop[rid];
                        d4 = rdp[rid];
                    }
                    // a dense set's ray carries its result index in o.w (k_material): the finish
                    // writes there, with no queue entry loaded or record re-read
                    if (at_slot) rid = __float_as_uint(o4.w);
                    px.x = o4.x;
                    py.x = o4.y;
                    pz.x = o4.z;
                    d = xyz(d4);
                    tri = -1;
                    best = kind ? -1.f : K_HUGE;
                    if constexpr (kCount) {
                        if (kind) {  // the any-hit set's counts start here (see tot_n)
                            tot_n1 -= tot_n;
                            tot_t1 -= tot_t;
                        }
                    }
                    sp = 0;
                    leaf = kEnd;
                    act = true;
                    const bool pre = kind ? a.set[1].prefiltered : a.set[0].prefiltered;
                    // NaN / zero direction: a miss / visible
                    if (!pre &&
                        (!(d.x == d.x && d.y == d.y && d.z == d.z) || (d.x == 0.f && d.y == 0.f && d.z == 0.f))) {
                        finish();
                    } else {
                        px.y = 1.f / d.x;
                        py.y = 1.f / d.y;
                        pz.y = 1.f / d.z;
                        io = cull_iota(sc, d, RAY_INV);
                        cut = kind ? K_INF_F : best * __builtin_fmaf(__builtin_fabsf(io), sc.cull_p, kCullSlackF);
                        float t0, t1, key;
                        // (k_shade resolved the rays that miss the root box in place, so the
                        // queued sets skip this test: same outcome, ray_misses_scene())
                        if (!pre && (!slab(sc.root_mn[0], sc.root_mn[1], sc.root_mn[2], sc.root_mx[0],
                                           sc.root_mx[1], sc.root_mx[2], RAY_O, RAY_INV, px.y < 0.f, py.y < 0.f, pz.y < 0.f,
                                           t0, t1) ||
                                     !keep_box(t0, t1, sc.root_w * io, cut, key)))
                            finish();
                        else
                            ref = sc.root_ref;
                    }
                }
            }
        }
        // (a trip without rays continues the loop.  The single-back-edge form -- skip the phases
        // instead -- removes ~20 register moves per trip from the listing but measured 0.7 % slower
        // on config 2: 2.478 / 2.493 vs 2.461 / 2.465 ms per launch, interleaved on one box)
        if (__ballot(act) == 0) {
            if (!more && buf_lo >= buf_hi) break;  // partition drained, every lane idle
            continue;
        }
        {
        MCPT_MARK("t_trip");
        uint32_t itc = 0, ipop = 0;  // node steps / iterations with a pop in the wave, this trip (kCount)
        if constexpr (kCount) {
            ph[PH_TRIPS]++;
            ph[PH_TRIP_NODE] += (uint32_t)__popcll(__ballot(act && ref >= 0));
            ph[PH_TRIP_LEAF] += (uint32_t)__popcll(__ballot(act && leaf != kEnd));
            ph[PH_TRIP_IDLE] += (uint32_t)__popcll(__ballot(!act));
        }
        // ---- node phase: up to kNodeSteps child-pair tests per lane holding an
        // interior node (amortises the per-trip bookkeeping over several steps)
        if (act) {
#pragma unroll 1
          for (int it = 0; it < kNodeSteps; it++) {
            MCPT_MARK("t_node");
            if constexpr (kCount) itc++;
            bool need_pop = false;
            if (ref >= 0) {
              if constexpr (kCount) tot_n++;
              const int nx = px.y < 0.f, ny = py.y < 0.f, nz = pz.y < 0.f;  // slow-path slab only
              if constexpr (kW == 4) {
                // 4-wide node: test the four child boxes, visit the nearest hit, push the
                // other hits far-to-near with their entry t (popped nearest-first)
                const float4* nd = sc.nodes + 8 * ref;
                const float4 mnx = nd[0], mxx = nd[1], mny = nd[2], mxy = nd[3], mnz = nd[4], mxz = nd[5], rf = nd[6];
                const float4 wq = nd[7];  // the children's margins
                float t0[4], t1[4];
                bool hk[4];
                if (__builtin_fabsf(io) < K_INF_F) {  // finite inverse: pair arithmetic
                    quad_axis2(mnx, mxx, px, t0, t1, true);
                    quad_axis2(mny, mxy, py, t0, t1, false);
                    quad_axis2(mnz, mxz, pz, t0, t1, false);
#pragma unroll
                    for (int k = 0; k < 4; k++) hk[k] = t0[k] <= t1[k];
                } else {
                    V3 so = RAY_O, si = RAY_INV;
                    __asm__ volatile("" : "+v"(so.x), "+v"(so.y), "+v"(so.z), "+v"(si.x), "+v"(si.y), "+v"(si.z));
                    const float* fmnx = &mnx.x; const float* fmxx = &mxx.x;
                    const float* fmny = &mny.x; const float* fmxy = &mxy.x;
                    const float* fmnz = &mnz.x; const float* fmxz = &mxz.x;
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        hk[k] = slab(fmnx[k], fmny[k], fmnz[k], fmxx[k], fmxy[k], fmxz[k], so, si, nx, ny, nz, t0[k],
                                     t1[k]);
                }
                int rr[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
                const float wk[4] = {wq.x, wq.y, wq.z, wq.w};
                float key[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    float ck;
                    const bool kb = keep_box(t0[k], t1[k], wk[k] * io, cut, ck);
                    const bool h = hk[k] && rr[k] != kEnd && kb;
                    // sort key: the cull key t0 - W iota (a NaN key from the NaN-passing slab sorts
                    // first and is never culled on pop), misses last
                    key[k] = h ? (ck == ck ? ck : -K_INF_F) : K_INF_F;
                    rr[k] = h ? rr[k] : kEnd;
                }
#define MCPT_CAS(i, j)                                                   \
                if (key[j] < key[i]) {                                    \
                    const float tk = key[i]; key[i] = key[j]; key[j] = tk; \
                    const int tr = rr[i]; rr[i] = rr[j]; rr[j] = tr;       \
                }
                MCPT_CAS(0, 1) MCPT_CAS(2, 3) MCPT_CAS(0, 2) MCPT_CAS(1, 3) MCPT_CAS(1, 2)
#undef MCPT_CAS
                need_pop = rr[0] == kEnd;
                if (!need_pop) {
#pragma unroll
                    for (int k = 3; k >= 1; k--) {
                        if (rr[k] != kEnd) {
                            const int2 e = make_int2(rr[k], __float_as_int(key[k]));
                            if (sp < kLdsStack) stk[sp][lane] = e;
                            else spill[sp - kLdsStack] = e;
                            sp++;
                        }
                    }
                    ref = rr[0];
                }
              } else {
                const float4* nd = sc.nodes + 4 * ref;
                const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
                float a0, b0, a1, b1;
                bool h0, h1;
                // node layout (SoA pairs): q0 = (mn.x, mn.x', mx.x, mx.x'), q1 = y, q2 = z,
                // q3 = (child ref, child ref', margin, margin'); unprimed = first child
                if (__builtin_fabsf(io) < K_INF_F) {  // finite inverse: pair arithmetic
                    pair_slab2(q0, q1, q2, px, py, pz, a0, b0, a1, b1);
                    h0 = a0 <= b0;
                    h1 = a1 <= b1;
                } else {
                    MCPT_MARK("rare");  // (an infinite inverse component: the reference's slab)
                    // the ray through opaque copies made here: the compiler would otherwise build its
                    // vectorised slab's operand pairs once per trip, for this rarely taken branch
                    V3 so = RAY_O, si = RAY_INV;
                    __asm__ volatile("" : "+v"(so.x), "+v"(so.y), "+v"(so.z), "+v"(si.x), "+v"(si.y), "+v"(si.z));
                    h0 = slab(q0.x, q1.x, q2.x, q0.z, q1.z, q2.z, so, si, nx, ny, nz, a0, b0);
                    h1 = slab(q0.y, q1.y, q2.y, q0.w, q1.w, q2.w, so, si, nx, ny, nz, a1, b1);
                }
                MCPT_MARK("t_node2");
                // the children's margins ride in q3.z / q3.w (see keep_box)
                // (evaluated unconditionally: a key assigned only under h0 / h1 costs the
                // allocator a live range per step -- 7 -> 23 spilled VGPRs)
                float k0, k1;
                const bool kb0 = keep_box(a0, b0, q3.z * io, cut, k0);
                const bool kb1 = keep_box(a1, b1, q3.w * io, cut, k1);
                h0 = h0 && kb0;
                h1 = h1 && kb1;
                const int c0 = __float_as_int(q3.x), c1 = __float_as_int(q3.y);
                need_pop = !(h0 | h1);
                if (h0 && h1) {
                    const bool first0 = !(k1 < k0);
                    const int2 e = make_int2(first0 ? c1 : c0, __float_as_int(first0 ? k1 : k0));
                    if (sp < kLdsStack) stk[sp][lane] = e;
                    else spill[sp - kLdsStack] = e;
                    sp++;
                    ref = first0 ? c0 : c1;
                } else {
                    ref = h0 ? c0 : c1;
                }
              }
            }
            // a reached leaf is parked in the lane's leaf slot and traversal
            // continues speculatively with the next stack entry
            if (!need_pop && ref < 0 && ref != kEnd) {
                if (leaf == kEnd) {
                    leaf = ref;
                    need_pop = true;
                }
            }
            MCPT_MARK("t_pop");
            if constexpr (kCount) ipop += __ballot(need_pop) != 0 ? 1u : 0u;  // (the active lanes agree)
            if (need_pop) ref = pop();
            if (ref < 0) break;  // parked-leaf slot full or traversal done: wait for the triangle phase
            // the node phase ends for every lane once fewer than kNodeMin still have node work
            // (they resume next trip, after the triangle phase and a refill)
            constexpr int kNodeMin =
                kW == 4 ? MCPT_NODE_MIN_LANES4 : (kLdsStack > ::mcpt_dev::kLdsStack ? MCPT_NODE_MIN_LANES2_DEEP : MCPT_NODE_MIN_LANES2);
            if constexpr (kNodeMin > 0)
                if ((uint32_t)__popcll(__ballot(true)) < (uint32_t)kNodeMin) break;
          }
        }
        if constexpr (kCount) {  // the node phase ran as many wave iterations as its busiest lane
            uint32_t m = itc, mp = ipop;
            for (int off = 32; off > 0; off >>= 1) {
                m = max(m, (uint32_t)__shfl_xor((int)m, off));
                mp = max(mp, (uint32_t)__shfl_xor((int)mp, off));
            }
            ph[PH_NODE_ITERS] += m;
            ph[PH_POP_ITERS] += mp;
        }
        // ---- triangle phase (wave-uniform): when enough lanes have a parked
        // leaf, or no lane has node work left, each parked leaf tests one triangle
        MCPT_MARK("t_tri");
        const uint32_t n_tri = (uint32_t)__popcll(__ballot(leaf != kEnd));
        const uint32_t n_node = (uint32_t)__popcll(__ballot(act && ref >= 0));
        if constexpr (kShare) {
          if (n_tri != 0 && (n_tri >= a.tri_min || n_tri >= n_node)) {
            // ---- shared triangle phase: the wave's parked leaves hold T triangles in all; lane
            // segment [excl, excl + cnt) of positions 0..T-1 is its leaf's, and position p is tested
            // by lane p mod 64 in round p / 64 against the segment owner's ray.  A test that accepts
            // min-combines the key (t, scene id, position in the leaf) into the owner's LDS slot:
            // the closest hit keeps the smallest t with ties to the lower scene id, exactly as the
            // one-at-a-time loop (Triangle.cu:174-179; the order of tests does not matter), and an
            // any-hit ray takes any acceptance (Triangle.cu:222-224).  t is the same value and
            // non-negative (-0 made +0, which compares equal), so its bits order as the floats.
            const bool own = leaf != kEnd;
            const uint32_t cnt = own ? (((uint32_t)leaf >> 24) & 7u) + 1u : 0u;
            const uint32_t incl = wave_scan_incl(cnt);
            const uint32_t excl = incl - cnt;
            const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
            // the owner's current best: any hit: none; closest hit: (best, its scene id, 7), or
            // (K_HUGE, 0) without a hit, so that t == K_HUGE is rejected as by t < best
            const uint64_t init = !own || best < 0.f
                                      ? ~0ull
                                      : ((uint64_t)__float_as_uint(best) << 32) | (tri >= 0 ? (bsid << 3) | 7u : 0u);
            s_key[lane] = init;
            __syncthreads();  // (one wave: orders the LDS writes before the other lanes' atomics)
            if constexpr (kCount) {
                if (own) tot_t += cnt;
                ph[PH_TRI_LANES] += total;
            }
#pragma unroll 1
            for (uint32_t base = 0; base < total; base += 64u) {
                if constexpr (kCount) ph[PH_TRI_PHASES]++;
                const uint32_t p = base + (uint32_t)lane;
                // owner: the last lane whose segment starts at or before p (excl is non-decreasing;
                // lanes after the owner start past p, empty segments before it do not matter)
                uint32_t ow = 0;
#pragma unroll
                for (uint32_t sh = 32; sh > 0; sh >>= 1) {
                    const uint32_t e = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((ow + sh) << 2), (int)excl);
                    if (e <= p) ow += sh;
                }
                const int oa = (int)(ow << 2);
                const uint32_t k = p - (uint32_t)__builtin_amdgcn_ds_bpermute(oa, (int)excl);
                const int oleaf = __builtin_amdgcn_ds_bpermute(oa, leaf);
                const V3 po = v3(__int_as_float(__builtin_amdgcn_ds_bpermute(oa, __float_as_int(px.x))),
                                 __int_as_float(__builtin_amdgcn_ds_bpermute(oa, __float_as_int(py.x))),
                                 __int_as_float(__builtin_amdgcn_ds_bpermute(oa, __float_as_int(pz.x))));
                const V3 pd = v3(__int_as_float(__builtin_amdgcn_ds_bpermute(oa, __float_as_int(d.x))),
                                 __int_as_float(__builtin_amdgcn_ds_bpermute(oa, __float_as_int(d.y))),
                                 __int_as_float(__builtin_amdgcn_ds_bpermute(oa, __float_as_int(d.z))));
                if (p < total) {
                    const int id = (oleaf & 0xffffff) + (int)k;
                    const float4* tp = sc.tri + kTriF4 * id;
                    const float4 w0 = tp[0], w1 = tp[1], w2 = tp[2];
                    __asm__ volatile("" ::"v"(w0.x), "v"(w0.y), "v"(w0.z), "v"(w0.w), "v"(w1.x), "v"(w1.y), "v"(w1.z),
                                     "v"(w1.w), "v"(w2.x), "v"(w2.y));
                    float t;
                    if (tri_test_t(po, pd, v3(w0.x, w0.y, w0.z), v3(w0.w, w1.x, w1.y), v3(w1.z, w1.w, w2.x), t) &&
                        !(t < 0.f) && t < K_HUGE) {
                        const uint64_t key = ((uint64_t)__float_as_uint(t + 0.f) << 32) |
                                             (((uint32_t)__float_as_int(w2.y) << 3) | k);
                        __hip_atomic_fetch_min(&s_key[ow], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
            __syncthreads();  // the atomics before the owners' reads
            if (own) {
                const uint64_t key = s_key[lane];
                if (key < init) {
                    tri = (leaf & 0xffffff) + (int)(key & 7u);
                    if (best < 0.f) {
                        ref = kEnd;  // occluded (tmax 1e32): drop the rest of the traversal
                    } else {
                        best = __uint_as_float((uint32_t)(key >> 32));
                        bsid = (uint32_t)key >> 3;
                        cut = best * __builtin_fmaf(__builtin_fabsf(io), sc.cull_p, kCullSlackF);
                    }
                }
                leaf = kEnd;
            }
          }
        } else if (n_tri != 0 && (n_tri >= a.tri_min || n_tri >= n_node)) {
            if constexpr (kCount) {
                ph[PH_TRI_PHASES]++;
                ph[PH_TRI_LANES] += n_tri;
            }
            if (leaf != kEnd) {
                if constexpr (kCount) tot_t++;
                const int id = leaf & 0xffffff;
                const float4* tp = sc.tri + kTriF4 * id;
                const float4 w0 = tp[0], w1 = tp[1], w2 = tp[2];
                // One memory round trip per test: without this the compiler sinks the vertex
                // load (w0.xyz) below the determinant test, so every front-facing test waits
                // for a second, dependent fetch of the same record.
                __asm__ volatile("" ::"v"(w0.x), "v"(w0.y), "v"(w0.z), "v"(w0.w), "v"(w1.x), "v"(w1.y), "v"(w1.z),
                                 "v"(w1.w), "v"(w2.x), "v"(w2.y));
                float t;
                bool done = false;
                const bool acc = tri_test_t(RAY_O, d, v3(w0.x, w0.y, w0.z), v3(w0.w, w1.x, w1.y), v3(w1.z, w1.w, w2.x), t);
                MCPT_MARK("t_tri2");
                if (acc && !(t < 0.f) &&
                    (best < 0.f ? t < K_HUGE
                          : (t < best ||
                             (t == best && tri >= 0 && __float_as_int(w2.y) < __float_as_int(sc.tri[kTriF4 * tri + 2].y))))) {
                    if (best < 0.f) {
                        tri = id;  // occluded (tmax 1e32)
                        done = true;
                    } else {
                        // exact-t ties go to the lower triangle id (tri record .y of the
                        // third float4), whatever order the BVH build stored triangles in
                        best = t;
                        tri = id;
                        cut = best * __builtin_fmaf(__builtin_fabsf(io), sc.cull_p, kCullSlackF);
                    }
                }
                if (done) {  // any hit: drop the rest of the traversal
                    leaf = kEnd;
                    ref = kEnd;
                } else if ((leaf & 0x07000000) != 0) {
                    leaf = leaf + 1 - (1 << 24);  // offset + 1, count - 1
                } else {
                    leaf = kEnd;
                }
            }
        }
        MCPT_MARK("t_finish");
        if constexpr (kCount) ph[PH_FINISH_TRIPS] += __ballot(act && ref == kEnd && leaf == kEnd) != 0 ? 1u : 0u;
        if (act && ref == kEnd && leaf == kEnd) finish();
        }
        MCPT_MARK("t_end");
    }
    MCPT_MARK("t_scan");
    // ---- partition scan: read every counter (one lane each) and join the first
    // partition after the current one that still holds rays.  A stale read (this die's
    // L2 holding an old copy of a counter line) can only be lower than the true count, so
    // a partition that reads drained is drained.  One that reads open but is not costs
    // one atomic, which marks it in `drained`; every other join takes rays.  So the scans
    // end, with every partition's counter at or past its ray count.
    {
        uint32_t g = 0;
        const bool cand = (uint32_t)lane < nparts && !((drained >> lane) & 1ull);
        if (cand) g = __hip_atomic_load(a.grab + lane * C_WORDS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t open = __ballot(cand && g < s_tot[lane]);
        if (open == 0) break;  // every partition drained
        // the open partition with the most rays left (lowest index on ties): waves that
        // run dry spread over the remaining work instead of queueing on one counter
        const uint32_t rem = min(s_tot[lane] - g, (1u << 25) - 1u);
        uint32_t key = (open >> lane) & 1ull ? (rem << 6) | (63u - (uint32_t)lane) : 0u;
        for (int off = 32; off > 0; off >>= 1) key = max(key, (uint32_t)__shfl_xor((int)key, off));
        enter(63u - (__builtin_amdgcn_readfirstlane(key) & 63u));
    }
    }
#undef RAY_O
#undef RAY_INV
    if constexpr (kCount) {
        wave_stats(a.set[0].stats, lane, tot_n - tot_n1, tot_t - tot_t1, tot_h - tot_h1);
        wave_stats(a.set[1].stats, lane, tot_n1, tot_t1, tot_h1);
        if (a.phase && lane == 0) {
            uint32_t* pw = a.phase + (blockIdx.x % kShards) * C_WORDS;
#pragma unroll
            for (int k = 0; k < kPhaseWords; k++)
                if (ph[k]) atomicAdd(pw + k, ph[k]);
        }
    }
}

// Camera records of a W x H film: gen_ray_pixel of every pixel (ShadeArgs::cam_px / cam_dir)
__global__ void k_cam_table(mcpt::CamView cam, int W, int H, float4* px, float4* dir) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint32_t)W * (uint32_t)H) return;
    const int x = (int)(i % (uint32_t)W), y = (int)(i / (uint32_t)W);
    V3 o, d;
    gen_ray_pixel(cam, W, H, x, y, o, d);
    px[i] = f4(cam.lens_radius > 0.f ? gen_ray_focal(cam, o, d) : o, 0.f);
    dir[i] = f4(d, 0.f);
}
void launch_cam_table(const mcpt::CamView& cam, int W, int H, float4* px, float4* dir, hipStream_t s) {
    const uint32_t n = (uint32_t)W * (uint32_t)H;
    if (n) hipLaunchKernelGGL(k_cam_table, dim3((n + 255) / 256), dim3(256), 0, s, cam, W, H, px, dir);
}

// The env texture's device copy takes the pdf table into its alpha plane (EnvView::tex)
__global__ void k_env_pack(float4* tex, const float* __restrict__ pdf, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) tex[i].w = pdf[i];
}
void launch_env_pack(float4* tex, const float* pdf, size_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_env_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tex, pdf, n);
}

// Light-sample table of an HRDI env light (EnvView::ltab / lrow / lcol): entry (y, x + 1)
// holds env_L / env_pdf at the direction env_dir returns for cell (x, y) -- computed by the
// very functions the per-sample path calls, so the values are the same -- and the row /
// column tables the direction's two factors (spherical_theta / spherical_phi of the cell's
// v / u, the arithmetic of spherical_direction).
template <bool FIXED>
__global__ void k_env_table(EnvView e, float4* out, float2* row, float2* col) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int W1 = e.w + 1;
    if (i < e.h) {
        float st, ct;
        spherical_theta(env_cell_v<FIXED>(e, i), st, ct);
        row[i] = make_float2(st, ct);
    }
    if (i < W1) {
        const int x = i - 1;
        float sp, cp;
        spherical_phi(env_cell_u<FIXED>(e, FIXED && x < 0 ? 0 : x), sp, cp);
        col[i] = make_float2(sp, cp);
    }
    if (i >= W1 * e.h) return;
    const int y = i / W1, x = i - y * W1 - 1;
    const V3 d = env_cell_dir<FIXED>(e, FIXED && x < 0 ? 0 : x, y);
    V3 L;
    float pdf;
    env_L_pdf<FIXED>(e, d, L, pdf);
    out[i] = make_float4(L.x, L.y, L.z, pdf);
}
void launch_env_table(const EnvView& e, bool fixed_mode, float4* out, float2* row, float2* col, hipStream_t s) {
    const int n = (e.w + 1) * e.h;
    if (fixed_mode) hipLaunchKernelGGL(k_env_table<true>, dim3((n + 255) / 256), dim3(256), 0, s, e, out, row, col);
    else hipLaunchKernelGGL(k_env_table<false>, dim3((n + 255) / 256), dim3(256), 0, s, e, out, row, col);
}

__global__ void k_hit_record(HitRecordArgs a) {  // stage_run(EXTEND) outputs
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int tri = a.tri[i];
    if (tri < 0) {
        a.hit_p[i] = make_float4(0.f, 0.f, 0.f, K_HUGE);
        a.hit_n[i] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
        a.scene_tri[i] = -1;
        return;
    }
    a.scene_tri[i] = __float_as_int(a.scene.tri[kTriF4 * tri + 2].y);  // storage position -> scene index
    V3 pos, nrm;
    int mat;
    float t;
    hit_record(a.scene, xyz(a.ro[i]), xyz(a.rd[i]), tri, pos, nrm, mat, t);
    a.hit_p[i] = make_float4(pos.x, pos.y, pos.z, t);
    a.hit_n[i] = make_float4(nrm.x, nrm.y, nrm.z, __int_as_float(mat));
}

__global__ void k_clear(ClearArgs a) {  // g_clear_dfilm (wavefront_kernels.cu:55-66)
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    a.flags[i] = F_DEAD | ((i / a.npx) << F_SIDX_SHIFT);  // dead, next sample: the slot's first
    a.samples[i] = 0;
    a.Ld[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ void k_resolve(ResolveArgs a) {  // film = sum of the path slots' accumulators, in slot order
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    uint32_t o = i;  // the pixel
    if (a.tiles) {   // compact layout: accumulator i is pixel li of tile-set tile ti
        const uint32_t tpx = (uint32_t)(a.tile_w * a.tile_h), ti = i / tpx, li = i - ti * tpx;
        const int2 t = a.tiles[ti];
        const uint32_t x = (uint32_t)t.x * a.tile_w + li % (uint32_t)a.tile_w, y = (uint32_t)t.y * a.tile_h + li / (uint32_t)a.tile_w;
        if (x >= (uint32_t)a.W || y >= (uint32_t)a.H) return;
        o = y * (uint32_t)a.W + x;
    }
    float4 L = a.Ld[i];
    uint32_t n = a.samples[i];
    for (int k = 1; k < a.slots; k++) {
        const float4 l = a.Ld[(size_t)k * a.n + i];
        L = make_float4(L.x + l.x, L.y + l.y, L.z + l.z, 0.f);
        n += a.samples[(size_t)k * a.n + i];
    }
    a.out_Ld[o] = L;
    a.out_samples[o] = n;
}

__global__ void k_tonemap(TonemapArgs a) {  // draw_to_surface (wavefront_kernels.cu:6-40)
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    float4 L = a.Ld[i];
    float s = (float)a.samples[i];
    V3 c = v3(L.x / s, L.y / s, L.z / s);
    c = c * a.exposure;
    c = v3(c.x / (c.x + 1.0f), c.y / (c.y + 1.0f), c.z / (c.z + 1.0f));
    float cc[3] = {255 * c.x, 255 * c.y, 255 * c.z};
    uchar4 o;
    unsigned char b[3];
    for (int k = 0; k < 3; k++) {
        float v = cc[k];
        b[k] = (v == v && v >= 0.f && v < 4294967296.f) ? (unsigned char)(unsigned int)v : (unsigned char)0;
    }
    o.x = b[0]; o.y = b[1]; o.z = b[2]; o.w = 255;
    a.out[i] = o;
}

// the occluder gate's first backoff (iterations without lookups after the first that did not pay):
// 3 / 7 / 15 measured interleaved (profiles/ab_r06_occ_gate.txt): config 3 247.1 / 245.2 / 244.6 ms,
// config 5 (64 spp) 729.9 / - / 727.6 ms, config 2 (whose lookups pay) unchanged
#ifndef MCPT_OCC_BACKOFF0
#define MCPT_OCC_BACKOFF0 15
#endif
__global__ void k_accumulate(CounterBlock* c, uint32_t nparts, uint32_t* occ_gate) {  // fold per-iteration shard counts into 64-bit totals
    if (c->idle) return;  // nothing ran since the iteration that set it; every counter is zero
    const int t = threadIdx.x;  // one lane per shard
    uint32_t v[C_STATS + 6];
#pragma unroll
    for (int k = 0; k < C_STATS + 6; k++) {
        v[k] = c->shard[t][k];
        c->shard[t][k] = 0;
    }
    c->last_ext_shard[t] = v[C_EXT];
    // drain check of the k_trace launch: every partition's hand-out counter must have
    // reached the partition's queued rays (shards t = p mod nparts)
    __shared__ uint32_t s_part[kMaxParts];
    if (t < kMaxParts) s_part[t] = 0;
    __syncthreads();
    atomicAdd(&s_part[t % nparts], v[C_EXT] + v[C_ANY]);
    __syncthreads();
    uint32_t g = 0;
    if (t < kMaxParts) g = c->grab[t][0];
    const bool short_part = t < (int)nparts && g < s_part[t];
#pragma unroll
    for (int k = 0; k < C_STATS + 6; k++)
        for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
    if (__ballot(short_part) != 0 && t == 0) c->trace_short += 1;
    if (t < kMaxParts) c->grab[t][0] = 0;  // k_trace chunk hand-out counters
    uint32_t phw[kPhaseWords];  // k_trace loop-phase counts (counting build; zero otherwise)
#pragma unroll
    for (int k = 0; k < kPhaseWords; k++) {
        phw[k] = c->shard[t][C_PH + k];
        c->shard[t][C_PH + k] = 0;
        for (int off = 32; off > 0; off >>= 1) phw[k] += __shfl_xor(phw[k], off);
    }
    uint32_t er = c->shard[t][C_EXT_RAYS], ar = c->shard[t][C_ANY_RAYS], oc = c->shard[t][C_OCC],
             ot = c->shard[t][C_OCC_TRY];
    c->shard[t][C_EXT_RAYS] = 0;
    c->shard[t][C_ANY_RAYS] = 0;
    c->shard[t][C_MAT] = 0;
    c->shard[t][C_OCC] = 0;
    c->shard[t][C_OCC_TRY] = 0;
    for (int off = 32; off > 0; off >>= 1) {
        er += __shfl_xor(er, off);
        ar += __shfl_xor(ar, off);
        oc += __shfl_xor(oc, off);
        ot += __shfl_xor(ot, off);
    }
    if (t == 0) {
        c->tot_ext += er;
        c->tot_any += ar;
        c->tot_occ += oc;
        // occluder-cache gate for the next iterations' k_material (a speed choice only)
        if (occ_gate) {
            if (occ_gate[0]) {
                occ_gate[0]--;
            } else if (!occ_gate[2]) {
                // the table is empty until the first iteration that traced any-hit rays has
                // recorded their occluders: k_material starts its lookups after it
                if (v[C_ANY]) occ_gate[2] = 1;
            } else if (ot >= 4096u) {
                if ((unsigned long long)oc * kOccMinRate < ot) {
                    occ_gate[1] = occ_gate[1] ? min(2u * occ_gate[1] + 1u, 255u) : (uint32_t)MCPT_OCC_BACKOFF0;
                    occ_gate[0] = occ_gate[1];
                } else {
                    occ_gate[1] = 0;
                }
            }
        }
        c->tot_vis += v[C_VIS];
        c->tot_ext_q += v[C_EXT];
        c->tot_any_q += v[C_ANY];
        c->last_ext = v[C_EXT];
        c->last_live = er;
        if (er == 0) c->idle = 1;  // no path alive and none generated: every later iteration is a no-op
        for (int k = 0; k < 6; k++) c->tot_stats[k] += v[C_STATS + k];
        for (int k = 0; k < kPhaseWords; k++) c->tot_phase[k] += phw[k];
    }
}

__global__ void k_pack(PackArgs a) {  // tile-set pixels -> packed 16 B/px (for the RCCL gather)
    const int tile_px = a.tile_w * a.tile_h;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint32_t)(a.ntiles * tile_px)) return;
    const int tile = i / tile_px, li = i % tile_px;
    int2 t = a.tiles[tile];
    int x = t.x * a.tile_w + li % a.tile_w, y = t.y * a.tile_h + li / a.tile_w;
    float4 o = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
    if (x < a.W && y < a.H) {
        uint32_t pid = (uint32_t)y * a.W + x;
        float4 L = a.Ld[pid];
        o = make_float4(L.x, L.y, L.z, __uint_as_float(a.samples[pid]));
    }
    a.out[i] = o;
}

__global__ void k_unpack(UnpackArgs a) {  // packed 16 B/px of a tile set -> film accumulators (mcpt_gather)
    const int tile_px = a.tile_w * a.tile_h;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint32_t)(a.ntiles * tile_px)) return;
    const int tile = i / tile_px, li = i % tile_px;
    const int2 t = a.tiles[tile];
    const int x = t.x * a.tile_w + li % a.tile_w, y = t.y * a.tile_h + li / a.tile_w;
    if (x >= a.W || y >= a.H) return;
    const uint32_t pid = (uint32_t)y * a.W + x;
    const float4 v = a.in[i];
    a.Ld[pid] = make_float4(v.x, v.y, v.z, 0.f);
    a.samples[pid] = __float_as_uint(v.w);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// Material grid: resident blocks (occupancy calculator x CUs) rounded down to a multiple of
// the shard count (at least one block per shard).
static uint32_t env_u32(const char* name, int def, int lo, int hi) {
    const char* e = getenv(name);
    int v = e ? atoi(e) : def;
    return (uint32_t)std::min(hi, std::max(lo, v));
}
// Per-device launch geometry, computed once per context (mcpt_create) for the device
// the context owns.
//  * k_material: resident blocks (occupancy calculator x CUs) rounded down to a multiple
//    of the shard count (at least one block per shard).
//  * k_trace: resident waves per CU from the occupancy calculator (32 for the 64-VGPR
//    child-pair instantiation, 28 deep-stack, 24 quads).  Round 1 measured 28 best on an
//    earlier kernel (0.406 / 0.368 / 0.354 / 0.329 / 0.382 ms at 16 / 20 / 24 / 28 / 32 waves
//    per CU); the round-2 kernel at 64 VGPRs runs 0.758 ms at 32 against 0.784 at 28 and
//    0.777 for the 72-VGPR build at 28.  MCPT_TRACE_WAVES caps the waves per CU.
//  * k_trace partitions: two per XCD, MCPT_TRACE_PARTS overrides.
int launch_geometry(int dev, LaunchGeom& g) {
    int cus = 0, nx = 1, per_cu = 0, mat0 = 0, mat1 = 0, sh0 = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&nx, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess) nx = 1;
    int occ[2][2] = {};  // [width 2 / 4][LDS stack 8 / deep]
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[0][0], k_trace<2, kLdsStack, false>, kTraceBlock, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[0][1], k_trace<2, kLdsStackDeep, false>, kTraceBlock, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[1][0], k_trace<4, kLdsStack, false>, kTraceBlock, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[1][1], k_trace<4, kLdsStackDeep, false>, kTraceBlock, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&mat0, k_material<false>, kBlock, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&mat1, k_material<true>, kBlock, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&sh0, k_shade<false>, kBlock, 0) != hipSuccess)
        return -1;
    if (cus <= 0) cus = 256;
    per_cu = 32;
    if (const char* e = getenv("MCPT_TRACE_WAVES")) per_cu = atoi(e);
    if (per_cu <= 0) per_cu = 16;
    for (int w = 0; w < 2; w++)
        for (int k = 0; k < 2; k++) g.trace_waves[w][k] = (uint32_t)(cus * std::max(1, std::min(per_cu, occ[w][k])));
    g.ndies = (uint32_t)std::max(1, nx);
    // Two partitions (hand-out counters) per die: one counter per die serialised the
    // returning atomics (config 2 k_trace 0.82 ms at 8 partitions, 0.767 at 16, 0.766 at
    // 32, 0.779 at 64; interleaved runs on one box)
    g.trace_parts = env_u32("MCPT_TRACE_PARTS", std::min(kMaxParts, 2 * std::max(1, nx)), 1, kMaxParts);
    if (const char* e = getenv("MCPT_MAT_BLOCKS_PER_CU")) {  // diagnostics: a smaller persistent grid
        const int m = atoi(e);                               // (4 -> 3 / 2 blocks: shade stage +5 % / +18 %)
        if (m > 0) { mat0 = std::min(mat0, m); mat1 = std::min(mat1, m); }
    }
    g.mat_blocks[0] = (uint32_t)std::max(1, cus * std::max(1, mat0) / kShards) * (uint32_t)kShards;
    g.mat_blocks[1] = (uint32_t)std::max(1, cus * std::max(1, mat1) / kShards) * (uint32_t)kShards;
    // k_shade grid: MCPT_SHADE_GRID times the resident blocks (0: one workgroup per shading block)
    g.shade_grid = (uint32_t)std::max(1, cus * std::max(1, sh0)) * env_u32("MCPT_SHADE_GRID", 16, 0, 1024);
    if (getenv("MCPT_SHADE_WGS")) g.shade_grid = env_u32("MCPT_SHADE_WGS", 0, 1, 1 << 30);  // tests: an absolute cap
    g.refill_min = env_u32("MCPT_REFILL_MIN", 0, 0, 64);  // 0: per instantiation (launch_trace)
    g.tri_min = env_u32("MCPT_TRI_MIN", 16, 0, 64);
    return 0;
}
// k_shade's grid: nblocks shading blocks over at most g.shade_grid workgroups, and never fewer
// than nblocks / kBlock (a workgroup reads its blocks' done flags one per thread)
static uint32_t shade_grid(uint32_t nblocks, const LaunchGeom& g) {
    uint32_t G = g.shade_grid ? std::min(nblocks, g.shade_grid) : nblocks;
    return std::max(G, (nblocks + kBlock - 1) / kBlock);
}
void launch_shade(const ShadeArgs& args, int nblocks, const LaunchGeom& g, bool fixed_mode, hipStream_t s) {
    ShadeArgs a = args;
    a.shade_vblocks = (uint32_t)nblocks;
    const uint32_t G = shade_grid((uint32_t)nblocks, g);
    if (fixed_mode) {
        hipLaunchKernelGGL(k_shade<true>, dim3(G), dim3(kBlock), 0, s, a);
        hipLaunchKernelGGL(k_material<true>, dim3(g.mat_blocks[1]), dim3(kBlock), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_shade<false>, dim3(G), dim3(kBlock), 0, s, a);
        hipLaunchKernelGGL(k_material<false>, dim3(g.mat_blocks[0]), dim3(kBlock), 0, s, a);
    }
}
// One of the two shading kernels alone (mcpt_stage_run's LOGIC / GENERATE and MATERIAL stages).
void launch_shade_stage(bool material_stage, const ShadeArgs& args, int nblocks, const LaunchGeom& g, bool fixed_mode,
                        hipStream_t s) {
    ShadeArgs a = args;
    a.shade_vblocks = (uint32_t)nblocks;
    if (!material_stage) {
        const uint32_t G = shade_grid((uint32_t)nblocks, g);
        if (fixed_mode) hipLaunchKernelGGL(k_shade<true>, dim3(G), dim3(kBlock), 0, s, a);
        else hipLaunchKernelGGL(k_shade<false>, dim3(G), dim3(kBlock), 0, s, a);
    } else {
        if (fixed_mode) hipLaunchKernelGGL(k_material<true>, dim3(g.mat_blocks[1]), dim3(kBlock), 0, s, a);
        else hipLaunchKernelGGL(k_material<false>, dim3(g.mat_blocks[0]), dim3(kBlock), 0, s, a);
    }
}
// Persistent grid: the device's resident waves rounded to a multiple of the shard count.
void launch_trace(const TraceArgs& args, const LaunchGeom& g, hipStream_t s) {
    if (args.nshards <= 0) return;
    TraceArgs a = args;
    a.tri_min = g.tri_min;
    a.nparts = std::min<uint32_t>(kMaxParts, std::max<uint32_t>(1, g.trace_parts));
    a.ndies = g.ndies;
    const uint32_t nsh = (uint32_t)a.nshards;
    // Deep trees (beyond kDeepTree levels) take the deeper LDS stack: fewer pushes spill to
    // scratch, at one resident wave per CU less (LDS-limited).  Config 5 (depth 25): 17.3 ->
    // 16.5 ms per launch; config 2 (depth 16) 0.781 -> 0.815 ms with it, so shallow trees keep 8.
    // The node width is the scene's (DevScene::width, chosen at upload).
    const int w = a.scene.width == 4 ? 1 : 0, k = a.scene.depth > kDeepTree ? 1 : 0;
    // Refill threshold (idle lanes before a wave takes new rays), per instantiation, measured
    // on the config that uses it (k_trace ms per launch, interleaved rounds on one box):
    //   child pairs, 8-entry stack (config 2): 20 -- 0.7267 at 16, 0.7237 at 20; 8 / 12 / 24 /
    //     28 / 32: 0.750 / 0.734 / 0.725 / 0.729 / 0.732;
    //   child pairs, deep stack (config 4): 32 -- 16 / 24 / 28 / 32 / 40: 7.55 / 7.31 / 7.27 /
    //     7.25 / 7.40;
    //   4-wide, 8-entry (config 3): 24 -- 16 / 20 / 24 / 28 / 32: 1.110 / 1.105 / 1.109 / 1.106
    //     / 1.114 (flat);
    //   4-wide, deep stack (config 5): 24 -- 16 / 20 / 24 / 28 / 32 / 40: 15.16 / 15.14 / 14.87
    //     / 14.88 / 14.99 / 15.61.
    // Waves that refill less often spend fewer trips on the refill's dependent loads; too high
    // a threshold leaves lanes idle (round-2 sweeps; tools/gpu/run.sh abenv repeats them).
    static const uint32_t kRefill[2][2] = {{20u, 32u}, {24u, 24u}};  // [width 2/4][stack 8/deep]
    a.refill_min = g.refill_min ? g.refill_min : kRefill[w][k];
    const uint32_t wps = std::max<uint32_t>(1, g.trace_waves[w][k] / nsh);
    const dim3 grid(wps * nsh), block(kTraceBlock);
    // Test instantiation with a 2-entry LDS stack (mcpt_debug_tiny_lds_stack): every push past the
    // second takes the scratch entries, so parity tests cover that path on every tree.
    if (a.tiny_stack) {
        if (w == 0) hipLaunchKernelGGL((k_trace<2, kLdsStackTiny, false>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_trace<4, kLdsStackTiny, false>), grid, block, 0, s, a);
        return;
    }
    // The counting instantiation (work counters, mcpt_set_work_counters) runs on the same grid;
    // a persistent wave that finds its partitions drained simply exits.
    if (a.set[0].stats || a.set[1].stats) {
        if (w == 0 && k == 0) hipLaunchKernelGGL((k_trace<2, kLdsStack, true>), grid, block, 0, s, a);
        else if (w == 0) hipLaunchKernelGGL((k_trace<2, kLdsStackDeep, true>), grid, block, 0, s, a);
        else if (k == 0) hipLaunchKernelGGL((k_trace<4, kLdsStack, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_trace<4, kLdsStackDeep, true>), grid, block, 0, s, a);
        return;
    }
    if (w == 0 && k == 0) hipLaunchKernelGGL((k_trace<2, kLdsStack, false>), grid, block, 0, s, a);
    else if (w == 0) hipLaunchKernelGGL((k_trace<2, kLdsStackDeep, false>), grid, block, 0, s, a);
    else if (k == 0) hipLaunchKernelGGL((k_trace<4, kLdsStack, false>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_trace<4, kLdsStackDeep, false>), grid, block, 0, s, a);
}
__global__ void k_quot(const float* a, const float* b, float* out, uint32_t n) {  // mcpt_debug_quot
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float q0, q1, q2;
    quot3(a[i], 1.0f, -a[i], b[i], q0, q1, q2);
    out[i] = q0;
}
void launch_quot(const float* a, const float* b, float* out, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_quot, dim3((n + 255) / 256), dim3(256), 0, s, a, b, out, n);
}

// HBM copy ceiling (mcpt_debug_hbm_copy; SURVEY.md 8(d) "re-measure a STREAM-copy ceiling"): one
// dwordx4 per lane, one pass (a block per 256 float4).  tools/hbm/copy_sweep.hip measured the
// variants: one-pass grids reach 6.25-6.39 TB/s on 1-4 GiB, persistent grid-stride loops
// 4.5-5.0 TB/s whatever the unroll or cache policy.
__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ src, float4* __restrict__ dst, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}
void launch_copy(const float4* src, float4* dst, size_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_copy, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, n);
}

// The round-2/3 diagnostics builds (per-section wave clocks of k_shade / k_material, k_trace loop
// profiles, wave lifetimes, per-ray step counts) are gone from the kernels (they are in git
// history); rocprofv3 counter passes (tools/gpu/run.sh pmc) replace them.  The ABI entries stay
// and report that nothing was collected.
int wave_times(unsigned long long* out, int n) {
    (void)out;
    (void)n;
    return 0;
}
int trace_profile(unsigned long long* out, int reset) {  // (replaced by the counting build's phase counts)
    (void)out;
    (void)reset;
    return 0;
}
__global__ void k_occ_records(DevScene sc, uint32_t nnodes, float4* out) {  // see launch_occ_records
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    auto put = [&](int ref, float mnx, float mny, float mnz, float mxx, float mxy, float mxz, float w) {
        if (ref >= 0 || ref == kEnd) return;
        const uint32_t off = (uint32_t)ref & 0xffffffu, cnt = (((uint32_t)ref >> 24) & 7u) + 1u;
        for (uint32_t k = off; k < off + cnt && k < sc.ntri; k++) {
            const float4* tr = sc.tri + kTriF4 * (size_t)k;  // (v0.xyz, e1.x) (e1.yz, e2.xy) (e2.z, ...)
            const float4 a = tr[0], b = tr[1], c = tr[2];
            float4* o = out + kOccRecF4 * (size_t)k;
            o[0] = make_float4(mnx, mny, mnz, w);  // .w: the leaf's culling margin
            o[1] = make_float4(mxx, mxy, mxz, a.x);
            o[2] = make_float4(a.y, a.z, a.w, b.x);
            o[3] = make_float4(b.y, b.z, b.w, c.x);
        }
    };
    if (i == 0 && sc.root_ref < 0)  // the whole tree is one leaf: its box is the root box
        put(sc.root_ref, sc.root_mn[0], sc.root_mn[1], sc.root_mn[2], sc.root_mx[0], sc.root_mx[1], sc.root_mx[2],
            sc.root_w);
    if (i >= nnodes) return;
    if (sc.width == 4) {  // mn.x[4], mx.x[4], mn.y[4], mx.y[4], mn.z[4], mx.z[4], refs[4], margins[4]
        const float4* nd = sc.nodes + 8 * (size_t)i;
        const float4 mnx = nd[0], mxx = nd[1], mny = nd[2], mxy = nd[3], mnz = nd[4], mxz = nd[5], rf = nd[6], wq = nd[7];
        const float* a0 = &mnx.x; const float* a1 = &mxx.x; const float* b0 = &mny.x;
        const float* b1 = &mxy.x; const float* c0 = &mnz.x; const float* c1 = &mxz.x; const float* r = &rf.x;
        const float* w = &wq.x;
        for (int k = 0; k < 4; k++) put(__float_as_int(r[k]), a0[k], b0[k], c0[k], a1[k], b1[k], c1[k], w[k]);
    } else {  // per axis (mn0, mn1, mx0, mx1), then (ref0, ref1, margin0, margin1)
        const float4* nd = sc.nodes + 4 * (size_t)i;
        const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
        put(__float_as_int(q3.x), q0.x, q1.x, q2.x, q0.z, q1.z, q2.z, q3.z);
        put(__float_as_int(q3.y), q0.y, q1.y, q2.y, q0.w, q1.w, q2.w, q3.w);
    }
}

// Culling margins (mcpt_core.hpp "conservative box culling").  k_cull_tri: W'_T of every triangle
// record (float, rounded up) and the far coefficient P (positive floats order as their bits).
__global__ void k_cull_tri(const float4* tri, uint32_t ntri, float* tw, uint32_t* pmax, int plane) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ntri) return;
    const float4* r = tri + kTriF4 * (size_t)i;
    const float4 r0 = r[0], r1 = r[1], r2 = r[2];
    double far;
    tw[i] = cull_to_float_up(cull_tri_margin(v3(r0.w, r1.x, r1.y), v3(r1.z, r1.w, r2.x), &far, plane != 0));
    if (far > 0.0) atomicMax(pmax, __float_as_uint(cull_to_float_up(far)));
}
// One bottom-up pass over child-pair nodes: each child's word (q3.z / q3.w) = the largest W'_T
// under it -- its triangles for a leaf, the child node's two words for an interior child.  Words
// start at 0 and only grow toward the subtree maxima, so a word read before or after its own
// update in the same pass is either way a lower bound, and depth + 1 passes reach the fixed point.
__global__ void k_cull_pairs(float4* nodes, uint32_t npairs, const float* tw, uint32_t ntri) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npairs) return;
    const float4 q3 = nodes[4 * (size_t)i + 3];
    float w[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int ref = __float_as_int(k ? q3.y : q3.x);
        float v = 0.f;
        if (ref >= 0) {
            const float4 c = nodes[4 * (size_t)ref + 3];
            v = __builtin_fmaxf(c.z, c.w);
        } else if (ref != kEnd) {
            const uint32_t off = (uint32_t)ref & 0xffffffu, cnt = (((uint32_t)ref >> 24) & 7u) + 1u;
            for (uint32_t t = off; t < off + cnt && t < ntri; t++) v = __builtin_fmaxf(v, tw[t]);
        }
        w[k] = v;
    }
    nodes[4 * (size_t)i + 3] = make_float4(q3.x, q3.y, w[0], w[1]);
}
__global__ void k_cull_zero(float4* nodes, uint32_t npairs) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npairs) return;
    float4 q3 = nodes[4 * (size_t)i + 3];
    q3.z = q3.w = 0.f;
    nodes[4 * (size_t)i + 3] = q3;
}
void launch_cull_margins(float4* nodes, uint32_t npairs, const float4* tri, uint32_t ntri, float* tri_w,
                         uint32_t* pmax, int passes, bool plane, hipStream_t s) {
    if (ntri) hipLaunchKernelGGL(k_cull_tri, dim3((ntri + 255) / 256), dim3(256), 0, s, tri, ntri, tri_w, pmax, plane ? 1 : 0);
    if (!npairs) return;
    hipLaunchKernelGGL(k_cull_zero, dim3((npairs + 255) / 256), dim3(256), 0, s, nodes, npairs);
    for (int p = 0; p < passes; p++)
        hipLaunchKernelGGL(k_cull_pairs, dim3((npairs + 255) / 256), dim3(256), 0, s, nodes, npairs, tri_w, ntri);
}
// One probe ray per occluder-table key (the pre-fill at upload, runtime.cpp): from the centre of
// the key's origin cell along the centre of its direction bin, so that occ_index maps the probe back
// to its own key.  Tracing the probes as any-hit rays records an occluder in every key whose probe
// is occluded -- a property of the scene alone, like the BVH.
__global__ void k_occ_probes(DevScene sc, float4* ro, float4* rd, uint32_t nkeys) {
    const uint32_t key = blockIdx.x * blockDim.x + threadIdx.x;
    if (key >= nkeys) return;
    const uint32_t G = (uint32_t)sc.occ_g, B = (uint32_t)sc.occ_b;
    uint32_t t = key, cx, cy, cz, face, ub, vb;
#if MCPT_OCC_LAYOUT == 1
    cx = t % G; t /= G; cy = t % G; t /= G; cz = t % G; t /= G; vb = t % B; t /= B; ub = t % B; face = t / B;
#else
    vb = t % B; t /= B; ub = t % B; t /= B; face = t % 6u; t /= 6u; cx = t % G; t /= G; cy = t % G; cz = t / G;
#endif
    const uint32_t c[3] = {cx, cy, cz};
    float o[3];
    for (int k = 0; k < 3; k++)
        o[k] = sc.occ_inv[k] > 0.f ? sc.root_mn[k] + ((float)c[k] + 0.5f) / sc.occ_inv[k] : sc.root_mn[k];
    const float hb = 0.5f * (float)B;
    const float u = ((float)ub + 0.5f) / hb - 1.f, v = ((float)vb + 0.5f) / hb - 1.f;
    const float sg = (face & 1u) ? -1.f : 1.f;
    float d[3];
    if (face < 2u) { d[0] = sg; d[1] = u; d[2] = v; }
    else if (face < 4u) { d[0] = u; d[1] = sg; d[2] = v; }
    else { d[0] = u; d[1] = v; d[2] = sg; }
    const float inv_n = 1.f / __builtin_sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    ro[key] = make_float4(o[0], o[1], o[2], 0.f);
    rd[key] = make_float4(d[0] * inv_n, d[1] * inv_n, d[2] * inv_n, 0.f);
}
void launch_occ_probes(const DevScene& sc, float4* ro, float4* rd, uint32_t nkeys, hipStream_t s) {
    if (nkeys == 0) return;
    hipLaunchKernelGGL(k_occ_probes, dim3((nkeys + 255) / 256), dim3(256), 0, s, sc, ro, rd, nkeys);
}
void launch_occ_records(const DevScene& sc, uint32_t nnodes, float4* rec, hipStream_t s) {
    hipLaunchKernelGGL(k_occ_records, dim3(nnodes / 256 + 1), dim3(256), 0, s, sc, nnodes, rec);
}
void launch_clear(const ClearArgs& a, hipStream_t s) {
    if (a.n == 0) return;  // an empty tile set (compact layout): nothing to launch, no zero-sized grid
    hipLaunchKernelGGL(k_clear, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}
void launch_hit_record(const HitRecordArgs& a, hipStream_t s) {
    if (a.n == 0) return;
    hipLaunchKernelGGL(k_hit_record, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}
void launch_resolve(const ResolveArgs& a, hipStream_t s) {
    if (a.n == 0) return;
    hipLaunchKernelGGL(k_resolve, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}
void launch_tonemap(const TonemapArgs& a, hipStream_t s) {
    if (a.n == 0) return;
    hipLaunchKernelGGL(k_tonemap, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}
void launch_accumulate(CounterBlock* c, uint32_t nparts, uint32_t* occ_gate, hipStream_t s) {
    hipLaunchKernelGGL(k_accumulate, dim3(1), dim3(kShards), 0, s, c, std::min<uint32_t>(kMaxParts, std::max<uint32_t>(1, nparts)),
                       occ_gate);
}
void launch_unpack(const UnpackArgs& a, hipStream_t s) {
    const uint32_t n = (uint32_t)(a.ntiles * a.tile_w * a.tile_h);
    if (n) hipLaunchKernelGGL(k_unpack, dim3((n + 255) / 256), dim3(256), 0, s, a);
}
void launch_pack(const PackArgs& a, hipStream_t s) {
    uint32_t n = (uint32_t)(a.ntiles * a.tile_w * a.tile_h);
    if (n == 0) return;
    hipLaunchKernelGGL(k_pack, dim3((n + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace mcpt_dev
