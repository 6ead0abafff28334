// HBM copy-ceiling sweep: variants of a dwordx4 copy (plain / nontemporal loads+stores, grid-stride
// persistent vs one-pass grids, elements per lane).  Prints read+write GB/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_gs(const f4* __restrict__ s, f4* __restrict__ d, size_t n) {
    const size_t st = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * st < n; i += U * st) {
        f4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++) v[k] = NT ? __builtin_nontemporal_load(s + i + k * st) : s[i + k * st];
#pragma unroll
        for (int k = 0; k < U; k++) { if (NT) __builtin_nontemporal_store(v[k], d + i + k * st); else d[i + k * st] = v[k]; }
    }
    for (; i < n; i += st) d[i] = s[i];
}
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_blk(const f4* __restrict__ s, f4* __restrict__ d, size_t n) {
    // one pass: block b copies U*256 consecutive float4s
    size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    f4 v[U];
#pragma unroll
    for (int k = 0; k < U; k++) if (base + k * 256 < n) v[k] = NT ? __builtin_nontemporal_load(s + base + k * 256) : s[base + k * 256];
#pragma unroll
    for (int k = 0; k < U; k++) if (base + k * 256 < n) { if (NT) __builtin_nontemporal_store(v[k], d + base + k * 256); else d[base + k * 256] = v[k]; }
}
template <typename K>
static void run(const char* name, K kern, unsigned grid, const f4* a, f4* b, size_t n) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, b, n);
    hipEventRecord(e0);
    const int it = 20;
    for (int i = 0; i < it; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, (i & 1) ? (const f4*)b : a, (i & 1) ? (f4*)a : b, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s grid %7u  %8.1f GB/s\n", name, grid, 2.0 * n * 16 * it / (ms * 1e-3) / 1e9);
}
int main() {
    for (size_t bytes : {(size_t)1 << 30, (size_t)4 << 30}) {
        size_t n = bytes / 16;
        f4 *a, *b;
        if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
        hipMemset(a, 0, bytes); hipMemset(b, 0, bytes);
        printf("== %zu MiB\n", bytes >> 20);
        for (unsigned w : {8u, 16u, 32u}) {
            run("gs U4 plain", k_gs<4, false>, 256 * w / 4, a, b, n);
            run("gs U4 nt", k_gs<4, true>, 256 * w / 4, a, b, n);
        }
        run("gs U8 plain 16w", k_gs<8, false>, 256 * 4, a, b, n);
        run("blk U1 plain", k_blk<1, false>, (unsigned)((n + 255) / 256), a, b, n);
        run("blk U4 plain", k_blk<4, false>, (unsigned)((n + 1023) / 1024), a, b, n);
        run("blk U4 nt", k_blk<4, true>, (unsigned)((n + 1023) / 1024), a, b, n);
        run("blk U8 plain", k_blk<8, false>, (unsigned)((n + 2047) / 2048), a, b, n);
        hipFree(a); hipFree(b);
    }
    return 0;
}
