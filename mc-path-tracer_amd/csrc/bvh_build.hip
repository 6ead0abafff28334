// bvh_build.hip -- GPU BVH builder for large scenes.
//
// The reference builds its BVH on the host (BVHAccel, BVH.cu:53-333: SAH with 12
// buckets, then a depth-first flatten), which for the 2 M-triangle configs takes
// seconds.  This is a linear BVH (Morton order + Karras 2012 radix tree) built
// entirely on the device:
//   1. per-triangle boxes from the uploaded vertices (exact min/max, the same
//      leaf boxes the host builder produces) and centroids;
//   2. centroid bounds (two-level block reduction);
//   3. 30-bit Morton codes, stable radix sort of (code, triangle) pairs (hipCUB);
//   4. Karras' parallel radix-tree construction over the sorted codes (ties in the
//      code broken by position, so every key is distinct);
//   5. node boxes bottom-up in kernel-synchronous passes (one pass per tree level:
//      a node is finished when both children are; kernel boundaries make the
//      writes of one pass visible to every XCD in the next, no cross-XCD flags);
//   6. emission in the traversal's child-pair node layout, with the triangle
//      records permuted into Morton order.
// One triangle per leaf, like the host builder at these sizes.  The traversal's
// hits do not depend on the tree: a leaf is reached iff its own box passes the
// slab test (every ancestor box contains it, and the rounded slab intervals are
// monotone in the box), leaf boxes are bit-identical to the host builder's, the
// culling is conservative and exact-t ties go to the lower scene index (carried
// in each triangle record), so films match the oracle's (which uses the host
// SAH tree) bit for bit -- tested in tests/test_gpu.py.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "kernels.hpp"

namespace mcpt_dev {

namespace {

constexpr int kB = 256;

__global__ void k_prim_boxes(int n, const float* __restrict__ v0, const float* __restrict__ v1,
                             const float* __restrict__ v2, float4* __restrict__ bmn, float4* __restrict__ bmx,
                             float4* __restrict__ cen) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float mn[3], mx[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float a = v0[3 * i + k], b = v1[3 * i + k], c = v2[3 * i + k];
        mn[k] = fminf(fminf(a, b), c);  // Bounds3f Union of the three vertices
        mx[k] = fmaxf(fmaxf(a, b), c);
    }
    bmn[i] = make_float4(mn[0], mn[1], mn[2], 0.f);
    bmx[i] = make_float4(mx[0], mx[1], mx[2], 0.f);
    cen[i] = make_float4(0.5f * (mn[0] + mx[0]), 0.5f * (mn[1] + mx[1]), 0.5f * (mn[2] + mx[2]), 0.f);
}

// block reduction of centroid bounds into partial[blockIdx] (mn in .xyz of [2b], mx of [2b+1])
__global__ void k_cen_bounds(int n, const float4* __restrict__ cen, float4* __restrict__ partial) {
    __shared__ float s[6][kB];
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) {
        const float4 c = cen[i];
        mn[0] = fminf(mn[0], c.x); mn[1] = fminf(mn[1], c.y); mn[2] = fminf(mn[2], c.z);
        mx[0] = fmaxf(mx[0], c.x); mx[1] = fmaxf(mx[1], c.y); mx[2] = fmaxf(mx[2], c.z);
    }
    for (int k = 0; k < 3; k++) { s[k][threadIdx.x] = mn[k]; s[3 + k][threadIdx.x] = mx[k]; }
    __syncthreads();
    for (int w = kB / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int k = 0; k < 3; k++) {
                s[k][threadIdx.x] = fminf(s[k][threadIdx.x], s[k][threadIdx.x + w]);
                s[3 + k][threadIdx.x] = fmaxf(s[3 + k][threadIdx.x], s[3 + k][threadIdx.x + w]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = make_float4(s[0][0], s[1][0], s[2][0], 0.f);
        partial[2 * blockIdx.x + 1] = make_float4(s[3][0], s[4][0], s[5][0], 0.f);
    }
}

__device__ inline uint32_t expand_bits(uint32_t v) {  // 10 bits -> every third bit
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ void k_morton(int n, int nparts, const float4* __restrict__ partial, const float4* __restrict__ cen,
                         uint32_t* __restrict__ code, uint32_t* __restrict__ idx) {
    __shared__ float sb[6];
    if (threadIdx.x == 0) {
        float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int p = 0; p < nparts; p++) {
            const float4 a = partial[2 * p], b = partial[2 * p + 1];
            mn[0] = fminf(mn[0], a.x); mn[1] = fminf(mn[1], a.y); mn[2] = fminf(mn[2], a.z);
            mx[0] = fmaxf(mx[0], b.x); mx[1] = fmaxf(mx[1], b.y); mx[2] = fmaxf(mx[2], b.z);
        }
        for (int k = 0; k < 3; k++) { sb[k] = mn[k]; sb[3 + k] = mx[k]; }
    }
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 c = cen[i];
    const float cc[3] = {c.x, c.y, c.z};
    uint32_t q[3];
    for (int k = 0; k < 3; k++) {
        const float ext = sb[3 + k] - sb[k];
        float f = ext > 0.f ? (cc[k] - sb[k]) / ext : 0.f;
        f = fminf(fmaxf(f * 1024.f, 0.f), 1023.f);
        q[k] = (uint32_t)f;
    }
    code[i] = (expand_bits(q[0]) << 2) | (expand_bits(q[1]) << 1) | expand_bits(q[2]);
    idx[i] = (uint32_t)i;
}

// longest common prefix of sorted keys i and j (position breaks code ties)
__device__ inline int delta(const uint32_t* __restrict__ code, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t a = code[i], b = code[j];
    if (a == b) return 32 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clz(a ^ b);
}

// Karras 2012, Fig. 4: internal node i of N-1; children encoded as
// internal k -> k, leaf k -> (N - 1) + k.
__global__ void k_karras(int n, const uint32_t* __restrict__ code, int2* __restrict__ child) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(code, n, i, i + 1) - delta(code, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(code, n, i, i - d);
    int lmax = 2;
    while (delta(code, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(code, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(code, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(code, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + min(d, 0);
    const int left = (min(i, j) == gamma) ? (n - 1) + gamma : gamma;
    const int right = (max(i, j) == gamma + 1) ? (n - 1) + gamma + 1 : gamma + 1;
    child[i] = make_int2(left, right);
}

// Bottom-up pass `pass`: an internal node whose two children were finished in
// EARLIER passes (or are leaves) gets its box; done[i] = pass + 1, which is its
// height.  Reading only results of earlier launches keeps every read behind a
// kernel boundary (the per-XCD L2s are not coherent within a launch).
__global__ void k_bounds_pass(int n, int pass, const int2* __restrict__ child, const float4* __restrict__ pmn,
                              const float4* __restrict__ pmx, const uint32_t* __restrict__ idx,
                              float4* __restrict__ nmn, float4* __restrict__ nmx, int* __restrict__ done) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1 || done[i]) return;
    const int2 c = child[i];
    float4 amn, amx, bmn, bmx;
    if (c.x >= n - 1) { const uint32_t p = idx[c.x - (n - 1)]; amn = pmn[p]; amx = pmx[p]; }
    else { const int h = done[c.x]; if (h == 0 || h > pass) return; amn = nmn[c.x]; amx = nmx[c.x]; }
    if (c.y >= n - 1) { const uint32_t p = idx[c.y - (n - 1)]; bmn = pmn[p]; bmx = pmx[p]; }
    else { const int h = done[c.y]; if (h == 0 || h > pass) return; bmn = nmn[c.y]; bmx = nmx[c.y]; }
    nmn[i] = make_float4(fminf(amn.x, bmn.x), fminf(amn.y, bmn.y), fminf(amn.z, bmn.z), 0.f);
    nmx[i] = make_float4(fmaxf(amx.x, bmx.x), fmaxf(amx.y, bmx.y), fmaxf(amx.z, bmx.z), 0.f);
    done[i] = pass + 1;
}

// child-pair node i (SoA pairs, see k_trace) + permuted triangle records
__global__ void k_emit(int n, const int2* __restrict__ child, const float4* __restrict__ pmn,
                       const float4* __restrict__ pmx, const uint32_t* __restrict__ idx,
                       const float4* __restrict__ nmn, const float4* __restrict__ nmx,
                       float4* __restrict__ nodes) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int2 c = child[i];
    float4 mn[2], mx[2];
    int ref[2];
    const int cc[2] = {c.x, c.y};
    for (int k = 0; k < 2; k++) {
        if (cc[k] >= n - 1) {
            const int leaf = cc[k] - (n - 1);
            const uint32_t p = idx[leaf];
            mn[k] = pmn[p];
            mx[k] = pmx[p];
            ref[k] = (int)(0x80000000u | (uint32_t)leaf);  // one triangle at sorted position `leaf`
        } else {
            mn[k] = nmn[cc[k]];
            mx[k] = nmx[cc[k]];
            ref[k] = cc[k];
        }
    }
    float4* q = nodes + 4 * i;
    q[0] = make_float4(mn[0].x, mn[1].x, mx[0].x, mx[1].x);
    q[1] = make_float4(mn[0].y, mn[1].y, mx[0].y, mx[1].y);
    q[2] = make_float4(mn[0].z, mn[1].z, mx[0].z, mx[1].z);
    q[3] = make_float4(__int_as_float(ref[0]), __int_as_float(ref[1]), 0.f, 0.f);
}

__global__ void k_permute(int n, const uint32_t* __restrict__ idx, const float4* __restrict__ tri_in,
                          const float4* __restrict__ sh_in, float4* __restrict__ tri_out, float4* __restrict__ sh_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = idx[i];
    for (int k = 0; k < kTriF4; k++) tri_out[kTriF4 * i + k] = tri_in[kTriF4 * p + k];
    for (int k = 0; k < 3; k++) sh_out[3 * i + k] = sh_in[3 * p + k];
}

// ---------------------------------------------------------------------------
// PLOC (Meister & Bittner 2018, "Parallel Locally-Ordered Clustering"): start from
// one cluster per triangle in Morton order; each round every cluster finds its
// nearest neighbour within +-r positions (smallest surface area of the union box),
// mutual nearest neighbours merge into a new node, and the surviving clusters are
// compacted in order.  Bottom-up agglomeration by surface area gives trees close to
// a full SAH build (the LBVH splits at Morton-code bits regardless of geometry).
// Ties are broken by the pair's indices (a strict total order on pairs), so the
// globally closest pair is always mutual and every round merges at least once.
// Deterministic: node indices come from prefix sums (the last merge, the root, is
// node 0), not from atomics.
constexpr int kPlocR = 16;  // search radius (the paper's default)

__device__ inline float union_area(float4 amn, float4 amx, float4 bmn, float4 bmx) {
    const float dx = fmaxf(amx.x, bmx.x) - fminf(amn.x, bmn.x);
    const float dy = fmaxf(amx.y, bmx.y) - fminf(amn.y, bmn.y);
    const float dz = fmaxf(amx.z, bmx.z) - fminf(amn.z, bmn.z);
    return dx * dy + dy * dz + dz * dx;  // half the surface area (same order both ways)
}

// chgt: per cluster, tree height and interior nodes in its subtree (ploc_pack, kernels.hpp)
__global__ void k_ploc_init(int n, const uint32_t* __restrict__ idx, const float4* __restrict__ pmn,
                            const float4* __restrict__ pmx, int* __restrict__ cref, float4* __restrict__ cmn,
                            float4* __restrict__ cmx, uint32_t* __restrict__ chgt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = idx[i];
    cref[i] = (int)(0x80000000u | (uint32_t)i);  // leaf: one triangle at sorted position i
    cmn[i] = pmn[p];
    cmx[i] = pmx[p];
    chgt[i] = ploc_pack(0u, 0u);
}

// nearest neighbour of every cluster within +-r (boxes of the block's range + halo in LDS)
__global__ __launch_bounds__(kB) void k_ploc_nn(int nc, const float4* __restrict__ cmn, const float4* __restrict__ cmx,
                                               int* __restrict__ nn) {
    __shared__ float4 smn[kB + 2 * kPlocR], smx[kB + 2 * kPlocR];
    const int base = blockIdx.x * kB - kPlocR;
    for (int t = threadIdx.x; t < kB + 2 * kPlocR; t += kB) {
        const int g = base + t;
        if (g >= 0 && g < nc) { smn[t] = cmn[g]; smx[t] = cmx[g]; }
    }
    __syncthreads();
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= nc) return;
    const int li = threadIdx.x + kPlocR;
    const float4 amn = smn[li], amx = smx[li];
    float best = INFINITY;
    int bj = -1;
    const int j0 = max(0, i - kPlocR), j1 = min(nc - 1, i + kPlocR);
    for (int j = j0; j <= j1; j++) {
        if (j == i) continue;
        float a = union_area(amn, amx, smn[j - base], smx[j - base]);
        if (!(a == a)) a = INFINITY;  // NaN coordinates: still a strict order (by indices)
        // order on pairs: area, then index distance, then the parity of the lower index,
        // then the lower index ((distance, lower index) identify the pair: a strict total
        // order).  On equal areas (coincident triangles) this pairs (0,1), (2,3), ... -- a
        // balanced merge -- where a plain lower-index order would chain one pair per round.
        const uint32_t kd = (uint32_t)abs(j - i), kl = (uint32_t)min(i, j);
        const uint32_t bd = (uint32_t)abs(bj - i), bl = (uint32_t)min(i, bj);
        const uint64_t key = ((uint64_t)kd << 32) | ((uint64_t)(kl & 1u) << 31) | (kl >> 1);
        const uint64_t bkey = ((uint64_t)bd << 32) | ((uint64_t)(bl & 1u) << 31) | (bl >> 1);
        if (bj < 0 || a < best || (a == best && key < bkey)) { best = a; bj = j; }
    }
    nn[i] = bj;
}

// flags: low word = this cluster starts a merge (mutual pair, i < j), high word = it survives
__global__ void k_ploc_mark(int nc, const int* __restrict__ nn, unsigned long long* __restrict__ flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nc) return;
    const int j = nn[i];
    const bool mutual = j >= 0 && nn[j] == i;
    const bool merge = mutual && i < j, survive = !(mutual && i > j);
    flag[i] = (merge ? 1ull : 0ull) | (survive ? (1ull << 32) : 0ull);
}

// apply one round: merged pairs become node (top - merge rank) in the child-pair layout,
// survivors are written at their compacted positions
__global__ void k_ploc_apply(int nc, int top, const int* __restrict__ nn, const unsigned long long* __restrict__ flag,
                             const unsigned long long* __restrict__ scan, const int* __restrict__ cref,
                             const float4* __restrict__ cmn, const float4* __restrict__ cmx,
                             const uint32_t* __restrict__ chgt, int* __restrict__ oref, float4* __restrict__ omn,
                             float4* __restrict__ omx, uint32_t* __restrict__ ohgt, float4* __restrict__ nodes,
                             int* __restrict__ ncnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nc) return;
    const unsigned long long f = flag[i];
    if (!(f >> 32)) return;  // absorbed by its partner
    const unsigned long long sc = scan[i];
    const int pos = (int)(sc >> 32);
    if (f & 1ull) {
        const int j = nn[i];
        const int k = top - (int)(sc & 0xffffffffull);
        const float4 amn = cmn[i], amx = cmx[i], bmn = cmn[j], bmx = cmx[j];
        float4* q = nodes + 4 * k;
        q[0] = make_float4(amn.x, bmn.x, amx.x, bmx.x);
        q[1] = make_float4(amn.y, bmn.y, amx.y, bmx.y);
        q[2] = make_float4(amn.z, bmn.z, amx.z, bmx.z);
        q[3] = make_float4(__int_as_float(cref[i]), __int_as_float(cref[j]), 0.f, 0.f);
        oref[pos] = k;
        omn[pos] = make_float4(fminf(amn.x, bmn.x), fminf(amn.y, bmn.y), fminf(amn.z, bmn.z), 0.f);
        omx[pos] = make_float4(fmaxf(amx.x, bmx.x), fmaxf(amx.y, bmx.y), fmaxf(amx.z, bmx.z), 0.f);
        const uint32_t h = ploc_merge(chgt[i], chgt[j]);
        ohgt[pos] = h;
        ncnt[k] = (int)ploc_count(h);
    } else {
        oref[pos] = cref[i];
        omn[pos] = cmn[i];
        omx[pos] = cmx[i];
        ohgt[pos] = chgt[i];
    }
}

// Re-number the PLOC nodes for locality, top-down, one launch per clustering round in
// reverse (a node's parent was created in a later round, so its new index is known):
//   layout 0, depth-first: interior children at p + 1 and p + 1 + count(first child);
//   layout 1, depth-first by sibling pairs: a node's interior children side by side at the
//     start of its descendants' range (one 128-B line holds both), then their subtrees.
// newidx / dstart hold each node's new index and (layout 1) descendant range start.
__global__ void k_relabel(int lo, int hi, int layout, const float4* __restrict__ raw, const int* __restrict__ ncnt,
                          int* __restrict__ newidx, int* __restrict__ dstart, float4* __restrict__ nodes) {
    const int k = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= hi) return;
    const int p = newidx[k];
    const float4* q = raw + 4 * k;
    const float4 q3 = q[3];
    int c[2] = {__float_as_int(q3.x), __float_as_int(q3.y)};
    int nc[2] = {c[0], c[1]};
    if (layout == 0) {
        int next = p + 1;
        for (int t = 0; t < 2; t++)
            if (c[t] >= 0) { nc[t] = next; newidx[c[t]] = next; next += ncnt[c[t]]; }
    } else {
        int ds = dstart[k];
        const int ni = (c[0] >= 0) + (c[1] >= 0);
        int sub = ds + ni;
        for (int t = 0; t < 2; t++)
            if (c[t] >= 0) { nc[t] = ds++; newidx[c[t]] = nc[t]; dstart[c[t]] = sub; sub += ncnt[c[t]] - 1; }
    }
    float4* o = nodes + 4 * p;
    o[0] = q[0];
    o[1] = q[1];
    o[2] = q[2];
    o[3] = make_float4(__int_as_float(nc[0]), __int_as_float(nc[1]), q3.z, q3.w);
}

struct Bufs {
    std::vector<void*> v;
    ~Bufs() { for (void* p : v) (void)hipFree(p); }
    template <class T>
    T* get(size_t count) {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(count * sizeof(T), 16)) != hipSuccess) return nullptr;
        v.push_back(p);
        return (T*)p;
    }
};

}  // namespace

// Steps 1-3 shared by both builders: primitive boxes, Morton codes, sorted (code, triangle)
// pairs; allocates the caller-owned node and permuted triangle arrays.
static int sort_prims(const LbvhInput& in, LbvhOutput& out, Bufs& tmp, hipStream_t s, float4*& pmn, float4*& pmx,
                      uint32_t*& code_s, uint32_t*& idx_s) {
    const int n = in.ntri;
    float *dv0 = tmp.get<float>(3 * (size_t)n), *dv1 = tmp.get<float>(3 * (size_t)n), *dv2 = tmp.get<float>(3 * (size_t)n);
    pmn = tmp.get<float4>(n);
    pmx = tmp.get<float4>(n);
    float4* cen = tmp.get<float4>(n);
    const int nparts = 512;
    float4* partial = tmp.get<float4>(2 * nparts);
    uint32_t *code = tmp.get<uint32_t>(n), *idx = tmp.get<uint32_t>(n);
    code_s = tmp.get<uint32_t>(n);
    idx_s = tmp.get<uint32_t>(n);
    if (!dv0 || !dv1 || !dv2 || !pmn || !pmx || !cen || !partial || !code || !idx || !code_s || !idx_s) return -2;
    const size_t vb = 3 * (size_t)n * sizeof(float);
    if (hipMemcpyAsync(dv0, in.v0, vb, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(dv1, in.v1, vb, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(dv2, in.v2, vb, hipMemcpyHostToDevice, s) != hipSuccess)
        return -3;
    const int g = (n + kB - 1) / kB;
    hipLaunchKernelGGL(k_prim_boxes, dim3(g), dim3(kB), 0, s, n, dv0, dv1, dv2, pmn, pmx, cen);
    hipLaunchKernelGGL(k_cen_bounds, dim3(nparts), dim3(kB), 0, s, n, cen, partial);
    hipLaunchKernelGGL(k_morton, dim3(g), dim3(kB), 0, s, n, nparts, partial, cen, code, idx);
    size_t tbytes = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, tbytes, code, code_s, idx, idx_s, n, 0, 30, s) != hipSuccess)
        return -4;
    void* tstore = tmp.get<uint8_t>(tbytes);
    if (!tstore) return -2;
    if (hipcub::DeviceRadixSort::SortPairs(tstore, tbytes, code, code_s, idx, idx_s, n, 0, 30, s) != hipSuccess)
        return -4;
    // nodes + permuted triangles (owned by the caller's scene allocation)
    const int ni = std::max(n - 1, 1);
    out.nodes = nullptr;
    if (hipMalloc(&out.nodes, std::max<size_t>((size_t)ni * 4 * sizeof(float4), 16)) != hipSuccess) return -2;
    if (hipMalloc(&out.tri, kTriF4 * (size_t)n * sizeof(float4)) != hipSuccess) return -2;
    if (hipMalloc(&out.tri_sh, 3 * (size_t)n * sizeof(float4)) != hipSuccess) return -2;
    hipLaunchKernelGGL(k_permute, dim3(g), dim3(kB), 0, s, n, idx_s, in.d_tri, in.d_sh, out.tri, out.tri_sh);
    return 0;
}

static int single_leaf(const float4* pmn, const float4* pmx, LbvhOutput& out, hipStream_t s) {
    std::vector<float4> pm(2);
    if (hipMemcpyAsync(pm.data(), pmn, sizeof(float4), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(pm.data() + 1, pmx, sizeof(float4), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess)
        return -3;
    out.root_ref = (int)0x80000000u;
    out.depth = 0;
    out.root_mn[0] = pm[0].x; out.root_mn[1] = pm[0].y; out.root_mn[2] = pm[0].z;
    out.root_mx[0] = pm[1].x; out.root_mx[1] = pm[1].y; out.root_mx[2] = pm[1].z;
    out.nnodes = 0;
    return 0;
}

int build_ploc(const LbvhInput& in, LbvhOutput& out, hipStream_t s) {
    const int n = in.ntri;
    if (n <= 0) return -1;
    Bufs tmp;
    float4 *pmn, *pmx;
    uint32_t *code_s, *idx_s;
    int rc = sort_prims(in, out, tmp, s, pmn, pmx, code_s, idx_s);
    if (rc) return rc;
    if (n == 1) return single_leaf(pmn, pmx, out, s);
    int* cref[2] = {tmp.get<int>(n), tmp.get<int>(n)};
    uint32_t* chgt[2] = {tmp.get<uint32_t>(n), tmp.get<uint32_t>(n)};
    float4* cmn[2] = {tmp.get<float4>(n), tmp.get<float4>(n)};
    float4* cmx[2] = {tmp.get<float4>(n), tmp.get<float4>(n)};
    int* nn = tmp.get<int>(n);
    unsigned long long *flag = tmp.get<unsigned long long>(n), *scan = tmp.get<unsigned long long>(n);
    unsigned long long* tail = nullptr;  // pinned readback of the last scan entry + flag
    if (!cref[0] || !cref[1] || !chgt[0] || !chgt[1] || !cmn[0] || !cmn[1] || !cmx[0] || !cmx[1] || !nn || !flag || !scan ||
        hipHostMalloc(&tail, 2 * sizeof(unsigned long long)) != hipSuccess)
        return -2;
    struct PinnedFree { unsigned long long* p; ~PinnedFree() { (void)hipHostFree(p); } } pf{tail};
    size_t sbytes = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, sbytes, flag, scan, n, s) != hipSuccess) return -4;
    void* sstore = tmp.get<uint8_t>(sbytes);
    if (!sstore) return -2;
    hipLaunchKernelGGL(k_ploc_init, dim3((n + kB - 1) / kB), dim3(kB), 0, s, n, idx_s, pmn, pmx, cref[0], cmn[0], cmx[0],
                       chgt[0]);
    float4* raw = tmp.get<float4>(4 * (size_t)(n - 1));
    int *ncnt = tmp.get<int>(n - 1), *newidx = tmp.get<int>(n - 1), *dstart = tmp.get<int>(n - 1);
    if (!raw || !ncnt || !newidx || !dstart) return -2;
    std::vector<std::pair<int, int>> round_rng;  // node index range [lo, hi) created by each round
    int nc = n, top = n - 2, cur = 0, rounds = 0;
    while (nc > 1) {
        const int g = (nc + kB - 1) / kB;
        hipLaunchKernelGGL(k_ploc_nn, dim3(g), dim3(kB), 0, s, nc, cmn[cur], cmx[cur], nn);
        hipLaunchKernelGGL(k_ploc_mark, dim3(g), dim3(kB), 0, s, nc, nn, flag);
        if (hipcub::DeviceScan::ExclusiveSum(sstore, sbytes, flag, scan, nc, s) != hipSuccess) return -4;
        hipLaunchKernelGGL(k_ploc_apply, dim3(g), dim3(kB), 0, s, nc, top, nn, flag, scan, cref[cur], cmn[cur], cmx[cur],
                           chgt[cur], cref[cur ^ 1], cmn[cur ^ 1], cmx[cur ^ 1], chgt[cur ^ 1], raw, ncnt);
        if (hipMemcpyAsync(tail, scan + (nc - 1), sizeof(unsigned long long), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(tail + 1, flag + (nc - 1), sizeof(unsigned long long), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -3;
        const unsigned long long tot = tail[0] + tail[1];
        const int merges = (int)(tot & 0xffffffffull), survivors = (int)(tot >> 32);
        if (merges <= 0 || survivors != nc - merges) return -5;  // no progress: cannot happen with a strict order
        round_rng.push_back({top - merges + 1, top + 1});
        top -= merges;
        nc = survivors;
        cur ^= 1;
        rounds++;
    }
    uint32_t root_h = 0;
    std::vector<float4> pm(2);
    if (hipMemcpyAsync(&root_h, chgt[cur], sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(pm.data(), cmn[cur], sizeof(float4), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(pm.data() + 1, cmx[cur], sizeof(float4), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess)
        return -3;
    if (top != -1) return -5;
    root_h = ploc_height(root_h);
    // locality layout (as the host upload chooses: sibling pairs for trees that stay in L2)
    const int layout = (size_t)(n - 1) * 64 <= ((size_t)2 << 20) ? 1 : 0;
    const int zero = 0, one = 1;
    if (hipMemcpyAsync(newidx, &zero, sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(dstart, &one, sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess)
        return -3;
    for (int r = (int)round_rng.size() - 1; r >= 0; r--) {
        const int lo = round_rng[r].first, hi = round_rng[r].second;
        hipLaunchKernelGGL(k_relabel, dim3((hi - lo + kB - 1) / kB), dim3(kB), 0, s, lo, hi, layout, raw, ncnt, newidx,
                           dstart, out.nodes);
    }
    if (hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess) return -3;
    out.root_ref = 0;
    out.depth = (int)root_h;
    out.root_mn[0] = pm[0].x; out.root_mn[1] = pm[0].y; out.root_mn[2] = pm[0].z;
    out.root_mx[0] = pm[1].x; out.root_mx[1] = pm[1].y; out.root_mx[2] = pm[1].z;
    out.nnodes = n - 1;
    out.rounds = rounds;
    return 0;
}

int build_lbvh(const LbvhInput& in, LbvhOutput& out, hipStream_t s) {
    const int n = in.ntri;
    if (n <= 0) return -1;
    Bufs tmp;
    float4 *pmn, *pmx;
    uint32_t *code_s, *idx_s;
    int rc = sort_prims(in, out, tmp, s, pmn, pmx, code_s, idx_s);
    if (rc) return rc;
    const int ni = std::max(n - 1, 1);
    int2* child = tmp.get<int2>(ni);
    float4 *nmn = tmp.get<float4>(ni), *nmx = tmp.get<float4>(ni);
    int* done = tmp.get<int>(ni);
    if (!child || !nmn || !nmx || !done) return -2;
    std::vector<float4> pm(2);
    if (n == 1) {  // a single leaf: no interior node; the root ref is the leaf
        if (hipMemcpyAsync(pm.data(), pmn, sizeof(float4), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(pm.data() + 1, pmx, sizeof(float4), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -3;
        out.root_ref = (int)0x80000000u;
        out.depth = 0;
    } else {
        hipLaunchKernelGGL(k_karras, dim3((ni + kB - 1) / kB), dim3(kB), 0, s, n, code_s, child);
        if (hipMemsetAsync(done, 0, (size_t)ni * sizeof(int), s) != hipSuccess) return -3;
        // one pass per level; the Karras tree of 30-bit codes + position ties is at most ~62 deep
        int root_h = 0;
        for (int pass = 0; pass < 128; pass += 16) {
            for (int k = 0; k < 16; k++)
                hipLaunchKernelGGL(k_bounds_pass, dim3((ni + kB - 1) / kB), dim3(kB), 0, s, n, pass + k, child,
                                   pmn, pmx, idx_s, nmn, nmx, done);
            if (hipMemcpyAsync(&root_h, done, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return -3;
            if (root_h) break;
        }
        if (!root_h) return -5;
        hipLaunchKernelGGL(k_emit, dim3((ni + kB - 1) / kB), dim3(kB), 0, s, n, child, pmn, pmx, idx_s, nmn, nmx,
                           out.nodes);
        if (hipMemcpyAsync(pm.data(), nmn, sizeof(float4), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(pm.data() + 1, nmx, sizeof(float4), hipMemcpyDeviceToHost, s) != hipSuccess)
            return -3;
        out.root_ref = 0;
        out.depth = (int)root_h;  // interior levels = maximal stack pushes + 1
    }
    if (hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess) return -3;
    out.root_mn[0] = pm[0].x; out.root_mn[1] = pm[0].y; out.root_mn[2] = pm[0].z;
    out.root_mx[0] = pm[1].x; out.root_mx[1] = pm[1].y; out.root_mx[2] = pm[1].z;
    out.nnodes = n - 1;
    return 0;
}

}  // namespace mcpt_dev
