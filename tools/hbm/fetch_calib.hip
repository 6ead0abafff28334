// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 against known byte counts, per
// access pattern (VERDICT r02 "validate the x2 FETCH_SIZE correction per access pattern").
// Every kernel runs once on buffers far larger than the 4 MiB per-XCD L2, so each touched line
// leaves L2 exactly once; the program prints one JSON line per kernel with the bytes the pattern
// moves (`logical`: bytes the lanes load or store; `lines`: distinct 128-B lines touched x 128).
// tools/fetch_calib.py joins them with the counter passes:
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d D -o f --output-format csv -- tools/hbm/fetch_calib
//   rocprofv3 --pmc WRITE_SIZE --kernel-trace -d D -o w --output-format csv -- tools/hbm/fetch_calib
// Patterns: the path-state streams of k_shade / k_material (16 B/lane coalesced), 4 B/lane
// coalesced streams (flags, samples, queue entries), 4 B/lane and 16 B/lane gathers at distinct
// lines (BVH nodes, triangle records, pid-indexed hit data), pairs of float4 in one line (a 32-B
// ray), sparse pid-indexed float4 reads at ~38 % lane density (k_material's pid gathers), and the
// store counterparts.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

// bijection on [0, 2^k): odd multiplier mod a power of two
__device__ inline uint64_t perm(uint64_t i, uint64_t mask) { return (i * 0x9E3779B97F4A7C15ull) & mask; }

__global__ __launch_bounds__(256) void k_rd_stream16(const f4* __restrict__ a, size_t n, float* out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    f4 v = i < n ? a[i] : f4{0, 0, 0, 0};
    if (v.x == 1234.5f && v.y == -1.f) out[0] = v.z;  // never true: keeps the load
}
__global__ __launch_bounds__(256) void k_rd_stream4(const float* __restrict__ a, size_t n, float* out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    float v = i < n ? a[i] : 0.f;
    if (v == 1234.5f) out[0] = v;
}
// lane i reads 4 B at the start of line perm(i): n distinct lines
__global__ __launch_bounds__(256) void k_rd_gather4(const float* __restrict__ a, size_t n, uint64_t lmask, float* out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float v = a[perm(i, lmask) * 32];
    if (v == 1234.5f) out[0] = v;
}
__global__ __launch_bounds__(256) void k_rd_gather16(const f4* __restrict__ a, size_t n, uint64_t lmask, float* out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    f4 v = a[perm(i, lmask) * 8];
    if (v.x == 1234.5f && v.w == 2.f) out[0] = v.y;
}
// a 32-B ray: two float4 of one line per lane
__global__ __launch_bounds__(256) void k_rd_gather32(const f4* __restrict__ a, size_t n, uint64_t lmask, float* out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const f4* p = a + perm(i, lmask) * 8;
    f4 v = p[0], w = p[1];
    if (v.x == 1234.5f && w.w == 2.f) out[0] = v.y + w.y;
}
// a 64-B node: four float4 of one line (child-pair node fetch)
__global__ __launch_bounds__(256) void k_rd_gather64(const f4* __restrict__ a, size_t n, uint64_t lmask, float* out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const f4* p = a + perm(i, lmask) * 8;
    f4 v = p[0], w = p[1], x = p[2], y = p[3];
    if (v.x == 1234.5f && w.w == 2.f && x.x == 3.f && y.y == 4.f) out[0] = v.y + w.y;
}
// k_material-like: a wave's lanes read float4 at increasing pids with ~38 % density (pid =
// floor(k * 2.6) for the k-th lane overall), so lines are partly used
__global__ __launch_bounds__(256) void k_rd_sparse16(const f4* __restrict__ a, size_t n, float* out) {
    const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    f4 v = a[(k * 13) / 5];
    if (v.x == 1234.5f) out[0] = v.y;
}
__global__ __launch_bounds__(256) void k_wr_stream16(f4* __restrict__ a, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) a[i] = f4{1.f, 2.f, 3.f, (float)i};
}
__global__ __launch_bounds__(256) void k_wr_stream4(float* __restrict__ a, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) a[i] = (float)i;
}
__global__ __launch_bounds__(256) void k_wr_scatter4(float* __restrict__ a, size_t n, uint64_t lmask) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) a[perm(i, lmask) * 32] = (float)i;
}
__global__ __launch_bounds__(256) void k_wr_scatter16(f4* __restrict__ a, size_t n, uint64_t lmask) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) a[perm(i, lmask) * 8] = f4{1.f, 2.f, 3.f, (float)i};
}
__global__ __launch_bounds__(256) void k_wr_sparse16(f4* __restrict__ a, size_t n) {
    const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (k < n) a[(k * 13) / 5] = f4{1.f, 2.f, 3.f, (float)k};
}

static unsigned blocks(size_t n) { return (unsigned)((n + 255) / 256); }
static void report(const char* name, double logical, double lines) {
    std::printf("{\"kernel\": \"%s\", \"logical\": %.0f, \"lines\": %.0f}\n", name, logical, lines);
}

int main() {
    const size_t bytes = (size_t)2 << 30;  // 2 GiB: 8x the 256 MiB MALL
    float* a = nullptr;
    float* out = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 256) != hipSuccess) return 1;
    if (hipMemset(a, 0, bytes) != hipSuccess) return 1;
    const uint64_t nlines = bytes / 128, lmask = nlines - 1;  // 2^24 lines
    const size_t n16 = bytes / 16, n4 = bytes / 4;
    const size_t ng = (size_t)4 << 20;  // gathers: 4 M distinct lines (512 MiB of lines)
    const size_t ns = (size_t)((bytes / 16) * 5 / 13);  // sparse: indices up to bytes / 16
    hipLaunchKernelGGL(k_rd_stream16, dim3(blocks(n16)), dim3(256), 0, 0, (const f4*)a, n16, out);
    report("k_rd_stream16", 16.0 * n16, (double)bytes);
    hipLaunchKernelGGL(k_rd_stream4, dim3(blocks(n4)), dim3(256), 0, 0, a, n4, out);
    report("k_rd_stream4", 4.0 * n4, (double)bytes);
    hipLaunchKernelGGL(k_rd_gather4, dim3(blocks(ng)), dim3(256), 0, 0, a, ng, lmask, out);
    report("k_rd_gather4", 4.0 * ng, 128.0 * ng);
    hipLaunchKernelGGL(k_rd_gather16, dim3(blocks(ng)), dim3(256), 0, 0, (const f4*)a, ng, lmask, out);
    report("k_rd_gather16", 16.0 * ng, 128.0 * ng);
    hipLaunchKernelGGL(k_rd_gather32, dim3(blocks(ng)), dim3(256), 0, 0, (const f4*)a, ng, lmask, out);
    report("k_rd_gather32", 32.0 * ng, 128.0 * ng);
    hipLaunchKernelGGL(k_rd_gather64, dim3(blocks(ng)), dim3(256), 0, 0, (const f4*)a, ng, lmask, out);
    report("k_rd_gather64", 64.0 * ng, 128.0 * ng);
    hipLaunchKernelGGL(k_rd_sparse16, dim3(blocks(ns)), dim3(256), 0, 0, (const f4*)a, ns, out);
    report("k_rd_sparse16", 16.0 * ns, (double)bytes);  // every line of the range is touched
    hipLaunchKernelGGL(k_wr_stream16, dim3(blocks(n16)), dim3(256), 0, 0, (f4*)a, n16);
    report("k_wr_stream16", 16.0 * n16, (double)bytes);
    hipLaunchKernelGGL(k_wr_stream4, dim3(blocks(n4)), dim3(256), 0, 0, a, n4);
    report("k_wr_stream4", 4.0 * n4, (double)bytes);
    hipLaunchKernelGGL(k_wr_scatter4, dim3(blocks(ng)), dim3(256), 0, 0, a, ng, lmask);
    report("k_wr_scatter4", 4.0 * ng, 128.0 * ng);
    hipLaunchKernelGGL(k_wr_scatter16, dim3(blocks(ng)), dim3(256), 0, 0, (f4*)a, ng, lmask);
    report("k_wr_scatter16", 16.0 * ng, 128.0 * ng);
    hipLaunchKernelGGL(k_wr_sparse16, dim3(blocks(ns)), dim3(256), 0, 0, (f4*)a, ns);
    report("k_wr_sparse16", 16.0 * ns, (double)bytes);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    (void)hipFree(a);
    (void)hipFree(out);
    return 0;
}
