// env_build.hip -- HRDI light tables built on the device.
//
// The reference builds the environment light's sampling tables with four CUDA
// kernels, three of them <<<1,1>>> loops (light_initialization_kernels.cu:3-112):
//   pdf_denom   = sum over texels, row-major, of lum * sin(pi v)           (float)
//   marginal_p  = per row, sum of lum * (sin(pi v) / pdf_denom)             (double terms,
//                 float accumulator), marginal_y = running sum over rows
//   conds_y     = per row, running sum of lum * sin(pi v) / (denom * marginal_p[y])
//   pdf         = lum * sin(pi v) / pdf_denom                               (per texel)
// Every result depends on the order of its float additions, so the device build
// keeps each chain's order and parallelises everything around the chains:
//   k_env_lum     one thread per texel: luminance of the bilinear texel fetch (the
//                 texture unit's 8-bit weights) and lum * sin(pi v);
//   k_env_denom   the one global chain: one lane adds the products in row-major order
//                 from LDS, while three waves stage the next chunk from HBM;
//   k_env_rows    one thread per row: the marginal_p chain, then the conds_y chain;
//   k_env_marginal one thread: marginal_y over the rows;
//   k_env_pdf     one thread per texel.
// The tables are bit-identical to the host restatement (host/scene.cpp
// build_env_tables) and the oracle's or_env_build: the same shared functions
// (mcpt_core.hpp: tex_bilinear, luminance, dsin) and the same rounding (IEEE
// division, no contraction).  k_env_check + k_env_guides then validate the CDFs and
// build the search guides for either source of tables (uploaded or built here).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"

namespace mcpt_dev {

using mcpt::kEnvGuide;

namespace {

constexpr int kB = 256;
constexpr uint32_t kDenChunk = 8192;  // floats per LDS stage of the denominator chain (2 x 32 KiB)

__global__ void k_env_lum(const float4* __restrict__ tex, int W, int H, float* __restrict__ lum,
                          float* __restrict__ prod, float* __restrict__ srow) {
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (uint32_t)W * (uint32_t)H) return;
    const int j = (int)(id / (uint32_t)W), i = (int)(id - (uint32_t)j * (uint32_t)W);
    const float u = (float)i / (float)W;
    const float v = (float)j / (float)H;
    const float s = mcpt::dsin(mcpt::PI_F * v);
    const float l = mcpt::luminance(mcpt::tex_bilinear(tex, W, H, u, v));
    lum[id] = l;
    prod[id] = l * s;
    if (i == 0) srow[j] = s;
}

// g_compute_pdf_denom (light_initialization_kernels.cu:3-26): wave 0's lane 0 adds,
// waves 1-3 stage chunk c+1 into the other LDS buffer meanwhile.
__global__ __launch_bounds__(kB) void k_env_denom(const float* __restrict__ prod, uint32_t n, float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float buf[2][kDenChunk];
    const uint32_t nch = (n + kDenChunk - 1) / kDenChunk;
    const uint32_t t = threadIdx.x;
    // staging: every load of a chunk issued before the LDS stores (one HBM round trip per
    // chunk, hidden behind the previous chunk's adds)
    auto stage = [&](uint32_t c) {
        constexpr uint32_t kS = kB - 64;                         // staging threads
        constexpr int kPer = (int)((kDenChunk / 4 + kS - 1) / kS);  // float4 loads per thread
        const uint32_t base = c * kDenChunk;
        const uint32_t len = n - base < kDenChunk ? n - base : kDenChunk;
        const uint32_t n4 = len / 4;
        const float4* src = reinterpret_cast<const float4*>(prod + base);
        float4* dst = reinterpret_cast<float4*>(buf[c & 1]);
        float4 v[kPer];
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            const uint32_t k = (t - 64) + q * kS;
            if (k < n4) v[q] = src[k];
        }
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            const uint32_t k = (t - 64) + q * kS;
            if (k < n4) dst[k] = v[q];
        }
        for (uint32_t k = n4 * 4 + (t - 64); k < len; k += kS) buf[c & 1][k] = prod[base + k];
    };
    if (t >= 64 && nch > 0) stage(0);
    __syncthreads();
    float denom = 0.0f;
    for (uint32_t c = 0; c < nch; c++) {
        if (t >= 64) {
            if (c + 1 < nch) stage(c + 1);
        } else if (t == 0) {
            // the adds in order; the LDS reads of the next two groups (kG float4 each, three
            // register sets, at most 3 kG <= 15 reads outstanding: the LDS counter's range) are
            // in flight while a group is added
            constexpr uint32_t kG = 4;
            const uint32_t len = n - c * kDenChunk < kDenChunk ? n - c * kDenChunk : kDenChunk;
            const float* b = buf[c & 1];
            const float4* b4 = reinterpret_cast<const float4*>(b);
            const uint32_t ng = len / (4 * kG);
            float4 A[kG], B[kG], D[kG];
            auto add = [&](const float4* x) {
#pragma unroll
                for (uint32_t q = 0; q < kG; q++) { denom += x[q].x; denom += x[q].y; denom += x[q].z; denom += x[q].w; }
            };
            // loads are unconditional (group index clamped into the buffer), so no register
            // copies are needed between the sets
            const uint32_t last = ng ? ng - 1 : 0;
            auto load = [&](float4* x, uint32_t g) {
                g = g < last ? g : last;
#pragma unroll
                for (uint32_t q = 0; q < kG; q++) x[q] = b4[g * kG + q];
            };
            load(A, 0);
            load(B, 1);
            for (uint32_t g = 0; g < ng; g += 3) {
                load(D, g + 2);
                add(A);
                load(A, g + 3);
                if (g + 1 < ng) add(B);
                load(B, g + 4);
                if (g + 2 < ng) add(D);
            }
            for (uint32_t k = ng * 4 * kG; k < len; k++) denom += b[k];
        }
        __syncthreads();
    }
    if (t == 0) out[0] = denom;
}

// g_compute_marginal_dist's per-row sums and g_compute_conditional_dist
// (light_initialization_kernels.cu:27-86), one thread per row.
__global__ void k_env_rows(const float* __restrict__ lum, const float* __restrict__ srow,
                           const float* __restrict__ denom_p, int W, int H, float* __restrict__ marginal_p,
                           float* __restrict__ conds_y) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= H) return;
    const float denom = denom_p[0];
    const float s = srow[j];
    const float* L = lum + (size_t)j * W;
    const double st = (double)(s / denom);
    float mp = 0.f;
    for (int i = 0; i < W; i++) mp = (float)((double)mp + (double)L[i] * st);
    marginal_p[j] = mp;
    const float val = s / (denom * mp);
    float* R = conds_y + (size_t)j * W;
    float prev = 0.f;
    for (int x = 0; x < W; x++) {
        float r = L[x] * val;
        if (x != 0) r = r + prev;
        R[x] = r;
        prev = r;
    }
}

__global__ void k_env_marginal(const float* __restrict__ marginal_p, int H, float* __restrict__ marginal_y) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    float prev = 0.f;
    for (int j = 0; j < H; j++) {
        float y = marginal_p[j];
        if (j != 0) y = y + prev;
        marginal_y[j] = y;
        prev = y;
    }
}

__global__ void k_env_pdf(const float* __restrict__ prod, const float* __restrict__ denom_p, uint32_t n,
                          float* __restrict__ pdf) {
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id < n) pdf[id] = prod[id] / denom_p[0];
}

// Guide validity: the marginal CDF sorted and NaN-free; every conditional row sorted
// and NaN-free or NaN throughout (row 0 of every map: 0 / (denom * 0)).  Thread H
// checks the marginal; bit 0 of *bad is set on failure.
__global__ void k_env_check(const float* __restrict__ marginal_y, const float* __restrict__ conds_y, int W, int H,
                            uint32_t* __restrict__ bad) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > H) return;
    const bool marg = j == H;
    const float* a = marg ? marginal_y : conds_y + (size_t)j * W;
    const int n = marg ? H : W;
    bool all_nan = !marg, sorted = true;
    for (int i = 0; i < n; i++) {
        const float x = a[i];
        all_nan = all_nan && !(x == x);
        sorted = sorted && (x == x) && (i == 0 || !(x < a[i - 1]));
    }
    if (!(all_nan || sorted)) atomicOr(bad, 1u);
}

// guide_m[k] = upper_bound(marginal_y, H, k / G); guide_c[y (G+1) + k] the same per row
__global__ void k_env_guides(const float* __restrict__ marginal_y, const float* __restrict__ conds_y, int W, int H,
                             uint16_t* __restrict__ gm, uint16_t* __restrict__ gc) {
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t G1 = kEnvGuide + 1;
    if (id >= (uint32_t)(H + 1) * G1) return;
    const int r = (int)(id / G1), k = (int)(id - (uint32_t)r * G1);
    const float val = (float)k / (float)kEnvGuide;
    if (r == H) gm[k] = (uint16_t)mcpt::upper_bound(marginal_y, H, val);
    else gc[id] = (uint16_t)mcpt::upper_bound(conds_y + (size_t)r * W, W, val);
}

inline dim3 grid(size_t n) { return dim3((unsigned)((n + kB - 1) / kB)); }

}  // namespace

// The luminance region is rounded up to a multiple of 4 floats so that `prod` (read as float4
// by k_env_denom) starts 16-B aligned whatever W * H is.
static size_t env_lum_floats(int W, int H) { return ((size_t)W * H + 3) & ~(size_t)3; }
size_t env_build_scratch_floats(int W, int H) { return env_lum_floats(W, H) + (size_t)W * H + 2 * (size_t)H + 4; }

void launch_env_build(const float4* tex, int W, int H, float* scratch, float* marginal_y, float* conds_y,
                      float* pdf, hipStream_t s) {
    const size_t n = (size_t)W * H;
    float* lum = scratch;
    float* prod = lum + env_lum_floats(W, H);
    float* srow = prod + n;
    float* mp = srow + H;
    float* denom = mp + H;
    hipLaunchKernelGGL(k_env_lum, grid(n), dim3(kB), 0, s, tex, W, H, lum, prod, srow);
    hipLaunchKernelGGL(k_env_denom, dim3(1), dim3(kB), 0, s, prod, (uint32_t)n, denom);
    hipLaunchKernelGGL(k_env_rows, dim3((H + 63) / 64), dim3(64), 0, s, lum, srow, denom, W, H, mp, conds_y);
    hipLaunchKernelGGL(k_env_marginal, dim3(1), dim3(64), 0, s, mp, H, marginal_y);
    hipLaunchKernelGGL(k_env_pdf, grid(n), dim3(kB), 0, s, prod, denom, (uint32_t)n, pdf);
}

void launch_env_guides(const float* marginal_y, const float* conds_y, int W, int H, uint16_t* gm, uint16_t* gc,
                       uint32_t* bad, hipStream_t s) {
    hipLaunchKernelGGL(k_env_check, grid((size_t)H + 1), dim3(kB), 0, s, marginal_y, conds_y, W, H, bad);
    hipLaunchKernelGGL(k_env_guides, grid((size_t)(H + 1) * (kEnvGuide + 1)), dim3(kB), 0, s, marginal_y, conds_y,
                       W, H, gm, gc);
}

}  // namespace mcpt_dev
