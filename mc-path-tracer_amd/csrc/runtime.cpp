// runtime.cpp -- device context behind the mcpt_* C ABI (include/mcpt.h).
//
// Replaces the reference's orchestration: PathTracer (PathTracer.cpp:112-187),
// Film device state (Film.cu:121-276), Scene::transfer_data_to_device
// (Scene.cu:363-470) and wavefront_pathtrace (wavefront_kernels.cu:377-442).
// Differences by design: one stream, no host sync or managed-memory counter
// readback between stages (counts stay on the device and the trace kernels are
// persistent), a whole tile set per iteration instead of one 256x256 tile, and
// error codes instead of exit(99).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "kernels.hpp"
#include "mcpt.h"

using namespace mcpt_dev;

namespace mcpt_host {
void set_global_error(const std::string& e);
const char* global_error();
}  // namespace mcpt_host

struct mcpt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    mcpt_config cfg{};
    char devname[256] = {0};
    int num_cu = 0;
    LaunchGeom geom{};             // persistent grids and k_trace partitions of this device
    uint32_t trace_parts_default = 1;
    // scene
    std::vector<void*> scene_bufs;
    DevScene scene{};
    bool has_scene = false;
    bool has_scene_before = false;  // set at the start of a re-upload
    int32_t ntri = 0;               // triangles of the uploaded scene
    size_t occ_entries_n = 0;       // occluder-cache table entries (DevScene::occ; + kOccGateWords gate words)
    uint32_t* occ_init = nullptr;   // the table as the upload's pre-fill left it (film clears restore it); nullptr: empty
    int pair_depth = 0;
    bool cull_ok = true, occ_nest_ok = true;  // last upload: boxes contain their triangles / nest (scene_upload)
    // traversal work counters (mcpt_set_work_counters): k_trace's counting instantiation, whose six
    // per-lane counters cost the fast one its spill-free registers -- off by default
    bool count_work = getenv("MCPT_WORK_COUNTERS") != nullptr;
    int node_layout = 0;  // pair-node numbering the last upload used (mcpt_debug_node_layout)
    // camera
    mcpt::CamView cam{};
    bool has_cam = false;
    // per-pixel camera records (cam_table): for the film size and camera they were built for
    float4* cam_tab = nullptr;
    size_t cam_tab_cap = 0;  // pixels allocated
    uint32_t cam_tab_W = 0, cam_tab_H = 0;
    mcpt::CamView cam_tab_cam{};
    bool cam_tab_ok = false;
    // Film observes camera and scene (Film::update -> clear(), Film.cu:278-281; notified by
    // Camera::update, Camera.cu:207, and Scene::notify, Scene.cu:534-545): a change marks the
    // film stale and the next iteration clears it first (unless MCPT_FLAG_NO_AUTO_CLEAR).
    bool film_stale = false;
    // film + paths
    uint32_t W = 0, H = 0, tile_w = 256, tile_h = 256;
    size_t P = 0;      // pixels (W * H)
    uint32_t slots = 1;  // path slots per pixel (mcpt_set_path_slots); path state holds slots * npx paths
    // Path layout (mcpt_set_compact_paths).  Full: npx = P, path index = slot * P + pixel id.  Compact:
    // the path state covers the tile set only, npx = tile-set tiles x tile pixels (ShadeArgs::npx).
    bool compact = false;
    size_t npx = 0;
    float4* film_Ld = nullptr;     // slots > 1 or compact: the film, W x H (sum of the slot accumulators)
    uint32_t* film_samples = nullptr;
    std::vector<void*> film_bufs;
    uint8_t* blk_done = nullptr;  // k_shade block done flags (ShadeArgs::blk_done), in film_bufs
    size_t blk_done_n = 0;
    bool blk_done_off = getenv("MCPT_NO_BLOCK_DONE") != nullptr;  // A/B switch: every block runs
    DevPaths p{};
    uint32_t *ext_q = nullptr, *any_q = nullptr, *mat_q = nullptr;
    float4* any_ray = nullptr;          // any-hit rays at their queue positions: o [2 queue_alloc], then d
    uint32_t ext_cap = 0, any_cap = 0;  // per-shard capacities
    size_t queue_alloc = 0;             // entries allocated for ext_q (any_q holds twice)
    CounterBlock* cnt = nullptr;
    CounterBlock* cnt_host = nullptr;  // pinned
    CounterBlock totals{};             // host copy of the counters after the last call (valid: totals_ok)
    bool totals_ok = false;
    int2* step_tile = nullptr;         // mcpt_wavefront_step's one-tile set: device + pinned staging (16 B:
    int2* step_tile_h = nullptr;       // the tile, then its index in the tile set, ShadeArgs::tile_base)
    int2* tiles = nullptr;
    std::vector<int2> tiles_h;
    // tiles holding pixels scattered in from another context (mcpt_film_unpack_tiles, mcpt_gather)
    // since the last film clear: the full layout's slot 0 holds them, so they may not become own
    // tiles before a clear (their sample count restarts from the flags word while Ld accumulates)
    std::vector<int2> unpacked;
    uint32_t tiles_cap = 0;
    std::vector<hipEvent_t> events;
    // stage_run scratch
    std::vector<void*> tmp_bufs;
    float last_stage_ms = 0.f;
    float last_build_ms = 0.f;  // last GPU BVH build (mcpt_scene_upload_gpu_bvh)
    float last_env_build_ms = 0.f;  // last device build of the HRDI tables (env_build.hip)
    bool env_device_built = false;  // the uploaded scene's HRDI tables were built on the device
    bool env_guides = false;        // env_cell uses the search guides
    int gpu_bvh_builder = MCPT_GPU_BVH_PLOC;  // mcpt_set_gpu_bvh_builder
    bool tiny_stack = false;  // mcpt_debug_tiny_lds_stack: k_trace with a 2-entry LDS stack (tests)
    unsigned long long phase_base[kPhaseWords] = {};  // mcpt_debug_trace_profile's reset point
};

static int set_err(mcpt_ctx* c, int rc, const std::string& msg) {
    if (c) c->err = msg;
    mcpt_host::set_global_error(msg);
    return rc;
}
#define HIPCHK(c, x)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess)                                                                 \
            return set_err((c), MCPT_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_));  \
    } while (0)

static void free_list(std::vector<void*>& v) {
    for (void* q : v)
        if (q) (void)hipFree(q);
    v.clear();
}
template <class T>
static int dalloc(mcpt_ctx* c, std::vector<void*>& list, T** out, size_t count) {
    void* q = nullptr;
    size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess) return set_err(c, MCPT_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    list.push_back(q);
    *out = (T*)q;
    return MCPT_OK;
}
template <class T>
static int dupload(mcpt_ctx* c, std::vector<void*>& list, T** out, const T* src, size_t count) {
    int rc = dalloc(c, list, out, count);
    if (rc) return rc;
    if (count) HIPCHK(c, hipMemcpy(*out, src, count * sizeof(T), hipMemcpyHostToDevice));
    return MCPT_OK;
}

extern "C" {

const char* mcpt_last_error(const mcpt_ctx* c) { return c ? c->err.c_str() : mcpt_host::global_error(); }

int mcpt_create(int device, const mcpt_config* cfg, mcpt_ctx** out) {
    if (!out) return set_err(nullptr, MCPT_E_INVALID, "out is null");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return set_err(nullptr, MCPT_E_NODEVICE, "no HIP device visible (the backend has no CPU fallback)");
    if (device < 0 || device >= n) return set_err(nullptr, MCPT_E_INVALID, "device index out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return set_err(nullptr, MCPT_E_HIP, "hipGetDeviceProperties failed");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_err(nullptr, MCPT_E_NODEVICE, std::string("device is ") + prop.gcnArchName + ", code objects are gfx950 only");
    mcpt_ctx* c = new mcpt_ctx();
    c->device = device;
    c->num_cu = prop.multiProcessorCount;
    snprintf(c->devname, sizeof(c->devname), "%s (%s, %d CUs)", prop.name, prop.gcnArchName, prop.multiProcessorCount);
    if (cfg) c->cfg = *cfg;
    else { c->cfg.seed = 0x5EED2026ull; c->cfg.spp = 16; c->cfg.max_depth = 5; c->cfg.rr_depth = 3; c->cfg.tile_w = 256; c->cfg.tile_h = 256; }
    // a dead path's flags word holds its next sample index, up to spp - 1 + 256 path slots
    if (c->cfg.max_depth < 1 || c->cfg.max_depth > 200 || c->cfg.spp < 0 || (uint32_t)c->cfg.spp > kMaxSpp - 256) {
        delete c;
        return set_err(nullptr, MCPT_E_INVALID, "bad config (max_depth 1..200, spp 0..2^19-256)");
    }
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return set_err(nullptr, MCPT_E_HIP, "stream creation failed");
    }
    if (hipMalloc(&c->cnt, sizeof(CounterBlock)) != hipSuccess || hipHostMalloc(&c->cnt_host, sizeof(CounterBlock)) != hipSuccess) {
        delete c;
        return set_err(nullptr, MCPT_E_NOMEM, "counter allocation failed");
    }
    (void)hipMemset(c->cnt, 0, sizeof(CounterBlock));
    if (launch_geometry(device, c->geom) != 0) {
        mcpt_destroy(c);
        return set_err(nullptr, MCPT_E_HIP, "occupancy query failed");
    }
    c->trace_parts_default = c->geom.trace_parts;
    *out = c;
    return MCPT_OK;
}

void mcpt_destroy(mcpt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_list(c->scene_bufs);
    free_list(c->film_bufs);
    free_list(c->tmp_bufs);
    if (c->cnt) (void)hipFree(c->cnt);
    if (c->cnt_host) (void)hipHostFree(c->cnt_host);
    if (c->tiles) (void)hipFree(c->tiles);
    if (c->step_tile) (void)hipFree(c->step_tile);
    if (c->step_tile_h) (void)hipHostFree(c->step_tile_h);
    if (c->ext_q) (void)hipFree(c->ext_q);
    if (c->any_q) (void)hipFree(c->any_q);
    if (c->mat_q) (void)hipFree(c->mat_q);
    if (c->any_ray) (void)hipFree(c->any_ray);
    if (c->cam_tab) (void)hipFree(c->cam_tab);
    for (auto e : c->events) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int mcpt_device_name(mcpt_ctx* c, char* buf, int32_t len) {
    if (!c || !buf || len <= 0) return MCPT_E_INVALID;
    snprintf(buf, (size_t)len, "%s", c->devname);
    return MCPT_OK;
}

// Scene upload: LinearBVHNode (BVH.h:63-72) -> child-pair nodes, dTriangle
// (Triangle.h:11-23, 288 B) -> 48-B intersection + 48-B shading records.

// Collapse a child-pair BVH into 4-wide nodes (DevScene::width 4): every 4-wide node
// is a pair node at even depth; its slots are the children of its two children
// (a leaf child takes one slot itself).  Boxes are copied, never recomputed, so
// every leaf box is the pair tree's (and the reference builder's) exact box.
// Breadth-first numbering keeps the top levels together.  Returns the new root
// ref and the largest number of stack pushes along any root-to-leaf path.
static int pairs_to_quads(const std::vector<float4>& pn, int root_ref, std::vector<float4>& qn, int& new_root,
                          int& max_push) {
    qn.clear();
    max_push = 0;
    if (root_ref < 0) { new_root = root_ref; return 0; }
    auto ref_at = [&](int p, int k) { int r; memcpy(&r, k ? &pn[4 * p + 3].y : &pn[4 * p + 3].x, 4); return r; };
    auto comp = [](const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; };
    std::vector<int> quad_of(pn.size() / 4, -1), order;
    std::vector<int> push_depth;  // pushes accumulated on the path to each quad node
    order.push_back(root_ref);
    quad_of[root_ref] = 0;
    push_depth.push_back(0);
    for (size_t h = 0; h < order.size(); h++) {
        const int p = order[h];
        struct Slot { float mn[3], mx[3], w; int ref; };  // w: the child's culling margin (q3.z / q3.w)
        Slot sl[4];
        int n = 0;
        for (int k = 0; k < 2; k++) {
            const int r = ref_at(p, k);
            if (r < 0) {  // leaf child of the pair node: its box is in p
                for (int a = 0; a < 3; a++) { sl[n].mn[a] = comp(pn[4 * p + a], k); sl[n].mx[a] = comp(pn[4 * p + a], 2 + k); }
                sl[n].w = comp(pn[4 * p + 3], 2 + k);
                sl[n++].ref = r;
            } else {      // interior child: take its two children
                for (int j = 0; j < 2; j++) {
                    for (int a = 0; a < 3; a++) { sl[n].mn[a] = comp(pn[4 * r + a], j); sl[n].mx[a] = comp(pn[4 * r + a], 2 + j); }
                    sl[n].w = comp(pn[4 * r + 3], 2 + j);
                    sl[n++].ref = ref_at(r, j);
                }
            }
        }
        const int pd = push_depth[h] + (n - 1);
        max_push = std::max(max_push, pd);
        for (int k = 0; k < n; k++) {
            if (sl[k].ref >= 0) {
                const int g = sl[k].ref;
                if (quad_of[g] < 0) {
                    quad_of[g] = (int)order.size();
                    order.push_back(g);
                    push_depth.push_back(pd);
                }
                sl[k].ref = quad_of[g];
            }
        }
        float4 q[8];
        float* f = reinterpret_cast<float*>(q);
        for (int i = 0; i < 32; i++) f[i] = 0.f;
        for (int k = 0; k < 4; k++) {
            const bool used = k < n;
            for (int a = 0; a < 3; a++) {
                f[(2 * a) * 4 + k] = used ? sl[k].mn[a] : 0.f;      // mn.a[k]
                f[(2 * a + 1) * 4 + k] = used ? sl[k].mx[a] : 0.f;  // mx.a[k]
            }
            int r = used ? sl[k].ref : -1;  // kEnd: empty slot
            memcpy(&f[6 * 4 + k], &r, 4);
            f[7 * 4 + k] = used ? sl[k].w : 0.f;  // margins (float4 7)
        }
        qn.insert(qn.end(), q, q + 8);
    }
    new_root = 0;
    return 0;
}

static hipEvent_t ev(mcpt_ctx* c, size_t i);
static int scene_upload(mcpt_ctx* c, const mcpt_scene_desc* d, bool gpu_bvh) {
    if (!c || !d) return set_err(c, MCPT_E_INVALID, "null argument");
    if (d->ntri < 0 || d->nnodes < 0 || d->nmat < 0 || d->ndir < 0) return set_err(c, MCPT_E_INVALID, "negative sizes");
    if (d->ntri >= (1 << 24)) return set_err(c, MCPT_E_INVALID, "more than 2^24 triangles");
    if (d->ntri > 0 && d->nnodes == 0 && !gpu_bvh) return set_err(c, MCPT_E_INVALID, "triangles without BVH");
    for (int32_t i = 0; i < d->ntri; i++)
        if (d->mat[i] < 0 || d->mat[i] >= d->nmat) return set_err(c, MCPT_E_INVALID, "material id out of range");
    if (d->env_mode == 1) {
        // tables: all three given (host build), or none (built on the device from env_tex)
        const int given = !!d->env_marginal_y + !!d->env_conds_y + !!d->env_pdf;
        if (!d->env_tex || d->env_w < 2 || d->env_h < 2 || (given != 0 && given != 3))
            return set_err(c, MCPT_E_INVALID, "HRDI env light without texture or with partial tables");
        if ((int64_t)d->env_w * d->env_h >= ((int64_t)1 << 31)) return set_err(c, MCPT_E_INVALID, "env map too large");
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    free_list(c->scene_bufs);
    c->has_scene_before = c->has_scene_before || c->has_scene;
    c->has_scene = false;
    const int N = gpu_bvh ? 0 : d->nnodes;  // gpu_bvh: the desc's BVH arrays are ignored
    // pair-node numbering of interior nodes + validation
    std::vector<int> pair_of(N, -1);
    int npair = 0;
    for (int i = 0; i < N; i++) {
        if (d->nprims[i] == 0) {
            if (i + 1 >= N || d->offset[i] <= i || d->offset[i] >= N) return set_err(c, MCPT_E_INVALID, "bad BVH child offset");
            pair_of[i] = npair++;  // depth-first numbering (renumbered below)
        } else {
            if (d->nprims[i] < 0 || d->nprims[i] > 8) return set_err(c, MCPT_E_INVALID, "leaf with more than 8 primitives");
            if (d->offset[i] < 0 || d->offset[i] + d->nprims[i] > d->ntri) return set_err(c, MCPT_E_INVALID, "bad leaf range");
        }
    }
    // Sibling-contiguous numbering for trees that stay in L2: the interior children of a
    // node get consecutive pair indices (one 128-B line holds both, so a popped far child is
    // often already cached), level by level (layout 2, breadth-first: the hot top levels
    // share lines) or depth-first by sibling pairs (layout 1).  Measured against plain
    // depth-first numbering (layout 0: parent next to its first child) on config 2 (4.8 K
    // pairs): k_trace 0.808 -> 0.786 (1) -> 0.781 ms (2); configs 3-5 (0.1-2 M pairs, beyond
    // L2) run 1-2 % slower with 1 or 2, so they keep 0.  MCPT_SIBLING_LAYOUT=0/1/2 forces a
    // layout (other values are ignored).  Layout only: hits are unchanged (tested).
    //
    // Layout 3 (line pairs, round 6): every 128-B line holds a node and its
    // larger-area interior child (a node without one leaves the line's second half as a pad node
    // that nothing references), lines in depth-first order.  Modelled on config 4
    // (tools/trav_study.py): distinct lines per ray 28.5 -> 25.5, L2 misses per ray unchanged
    // (4.77 -> 4.79); measured on the GPU before it becomes anyone's default.
    const char* sl_env = getenv("MCPT_SIBLING_LAYOUT");
    int layout = (size_t)npair * 64 <= ((size_t)2 << 20) ? 2 : 0;
    if (sl_env && sl_env[0] >= '0' && sl_env[0] <= '3' && sl_env[1] == 0) layout = sl_env[0] - '0';
    c->node_layout = 0;
    std::vector<uint8_t> is_pad;  // layout 3: pair indices that are pads
    if (N > 0 && d->nprims[0] == 0 && layout == 3) {
        auto area = [&](int i) {
            float e[3];
            for (int k = 0; k < 3; k++) e[k] = std::fmax(d->bmax[3 * i + k] - d->bmin[3 * i + k], 0.f);
            return (double)e[0] * e[1] + (double)e[1] * e[2] + (double)e[2] * e[0];
        };
        auto inner = [&](int i, int out[2]) {
            int n = 0;
            for (int ch : {i + 1, d->offset[i]})
                if (d->nprims[ch] == 0) out[n++] = ch;
            return n;
        };
        std::vector<int> po(N, -1), st{0};
        int next = 0;
        bool tree = true;
        while (tree && !st.empty()) {
            const int i = st.back();
            st.pop_back();
            if (po[i] >= 0) { tree = false; break; }
            next += next & 1;  // a line starts with a head
            po[i] = next++;
            int ks[2], rest[3], nr = 0;
            const int nk = inner(i, ks);
            if (nk > 0) {
                const int cb = nk == 2 && area(ks[1]) > area(ks[0]) ? ks[1] : ks[0];
                if (po[cb] >= 0) { tree = false; break; }
                po[cb] = next++;  // the head's line partner
                for (int k = 0; k < nk; k++)
                    if (ks[k] != cb) rest[nr++] = ks[k];
                int gk[2];
                const int ng = inner(cb, gk);
                for (int k = 0; k < ng; k++) rest[nr++] = gk[k];
            }
            // the larger-area subtree comes next (popped first)
            std::sort(rest, rest + nr, [&](int x, int y) { return area(x) < area(y); });
            for (int k = 0; k < nr; k++) st.push_back(rest[k]);
        }
        int reached = 0;
        for (int i = 0; i < N; i++) reached += d->nprims[i] == 0 && po[i] >= 0;
        if (tree && reached == npair) {
            is_pad.assign(next, 1);
            for (int i = 0; i < N; i++)
                if (d->nprims[i] == 0) is_pad[po[i]] = 0;
            pair_of.swap(po);
            npair = next;  // pads included
            c->node_layout = 3;
        }
    } else if (N > 0 && d->nprims[0] == 0 && layout != 0) {
        // Renumber by walking the tree from the root.  The walk must reach every interior
        // node exactly once (a tree); a shared child (a DAG, which the validation above
        // accepts and layout 0 traverses correctly) or an unreachable node would give two
        // nodes one pair index, so such inputs keep layout 0.
        std::vector<int> po(pair_of);
        std::vector<uint8_t> seen(N, 0);
        int next = 0;
        po[0] = next++;
        seen[0] = 1;
        bool tree = true;
        std::vector<int> st{0};  // layout 1: stack (depth-first by sibling pairs); 2: FIFO (breadth-first)
        size_t head = 0;
        while (tree && (layout == 2 ? head < st.size() : !st.empty())) {
            int i;
            if (layout == 2) {
                i = st[head++];
            } else {
                i = st.back();
                st.pop_back();
            }
            const int ch[2] = {i + 1, d->offset[i]};
            for (int k = 0; k < 2 && tree; k++) {
                if (d->nprims[ch[k]] != 0) continue;
                if (seen[ch[k]]) tree = false;  // reached twice
                seen[ch[k]] = 1;
                po[ch[k]] = next++;
            }
            if (layout == 2) {
                for (int k = 0; k < 2; k++)
                    if (d->nprims[ch[k]] == 0) st.push_back(ch[k]);
            } else {
                for (int k = 1; k >= 0; k--)
                    if (d->nprims[ch[k]] == 0) st.push_back(ch[k]);
            }
        }
        if (tree && next == npair) {  // every interior node reached exactly once: a permutation
            pair_of.swap(po);
            c->node_layout = layout;
        }
    }
    // A leaf with several triangles becomes a small subtree of pair nodes whose leaves
    // hold one triangle each, boxed by its own bounds (the vertex union,
    // g_init_BVH_triangle_info).  A triangle then counts only if the line passes the
    // leaf box and its own box -- BVHAccel's one-triangle-leaf semantics -- so results
    // do not depend on how a builder grouped triangles (Moller-Trumbore alone can
    // accept a grazing line just outside a triangle's box).  The oracle applies the
    // same own-box test to multi-triangle leaves.
    std::vector<float4> xn;  // expansion pairs, appended after the desc's pairs
    auto tri_box = [&](int t0, int n, float mn[3], float mx[3]) {
        for (int k = 0; k < 3; k++) { mn[k] = 3.402823466e+38f; mx[k] = -3.402823466e+38f; }
        for (int t = t0; t < t0 + n; t++)
            for (const float* v : {d->v0 + 3 * (size_t)t, d->v1 + 3 * (size_t)t, d->v2 + 3 * (size_t)t})
                for (int k = 0; k < 3; k++) { mn[k] = std::fmin(mn[k], v[k]); mx[k] = std::fmax(mx[k], v[k]); }
    };
    std::function<int(int, int)> expand = [&](int t0, int n) -> int {
        if (n == 1) return (int)(0x80000000u | (uint32_t)t0);
        const int m = n / 2;
        const int me = npair + (int)(xn.size() / 4);
        xn.resize(xn.size() + 4);
        const int r0 = expand(t0, m), r1 = expand(t0 + m, n - m);
        float a0[3], b0[3], a1[3], b1[3];
        tri_box(t0, m, a0, b0);
        tri_box(t0 + m, n - m, a1, b1);
        float4* q = &xn[(size_t)(me - npair) * 4];
        q[0] = make_float4(a0[0], a1[0], b0[0], b1[0]);
        q[1] = make_float4(a0[1], a1[1], b0[1], b1[1]);
        q[2] = make_float4(a0[2], a1[2], b0[2], b1[2]);
        float fr0, fr1;
        memcpy(&fr0, &r0, 4);
        memcpy(&fr1, &r1, 4);
        q[3] = make_float4(fr0, fr1, 0.f, 0.f);
        return me;
    };
    std::vector<int> leaf_ref(N, 0);
    int xdepth = 0;  // extra levels under a desc leaf
    for (int i = 0; i < N; i++) {
        if (d->nprims[i] == 0) continue;
        leaf_ref[i] = expand(d->offset[i], d->nprims[i]);
        int lv = 0;
        while ((1 << lv) < d->nprims[i]) lv++;
        xdepth = std::max(xdepth, lv);
    }
    auto ref_of = [&](int j) -> int { return d->nprims[j] == 0 ? pair_of[j] : leaf_ref[j]; };
    std::vector<float4> pn((size_t)npair * 4);
    for (size_t k = 0; k < is_pad.size(); k++) {
        if (!is_pad[k]) continue;
        float fe;
        const int e = -1;  // kEnd: no child (the pad is never referenced)
        memcpy(&fe, &e, 4);
        pn[4 * k + 3] = make_float4(fe, fe, 0.f, 0.f);
    }
    for (int i = 0; i < N; i++) {
        if (d->nprims[i] != 0) continue;
        int c0 = i + 1, c1 = d->offset[i];
        const float *a0 = d->bmin + 3 * c0, *b0 = d->bmax + 3 * c0, *a1 = d->bmin + 3 * c1, *b1 = d->bmax + 3 * c1;
        float4* q = &pn[(size_t)pair_of[i] * 4];
        // SoA pairs: per axis (min child 0, min child 1, max child 0, max child 1)
        q[0] = make_float4(a0[0], a1[0], b0[0], b1[0]);
        q[1] = make_float4(a0[1], a1[1], b0[1], b1[1]);
        q[2] = make_float4(a0[2], a1[2], b0[2], b1[2]);
        int r0 = ref_of(c0), r1 = ref_of(c1);
        float fr0, fr1;
        memcpy(&fr0, &r0, 4);
        memcpy(&fr1, &r1, 4);
        q[3] = make_float4(fr0, fr1, 0.f, 0.f);  // .z / .w: the children's culling margins (launch_cull_margins)
    }
    pn.insert(pn.end(), xn.begin(), xn.end());
    // depth of the tree = bound on stack pushes
    int depth = 0;
    if (N > 0) {
        std::vector<std::pair<int, int>> st{{0, 0}};
        while (!st.empty()) {
            auto [n, dd] = st.back();
            st.pop_back();
            depth = std::max(depth, dd);
            if (d->nprims[n] == 0) { st.push_back({n + 1, dd + 1}); st.push_back({d->offset[n], dd + 1}); }
        }
    }
    depth += xdepth;
    if (depth > kMaxStack) return set_err(c, MCPT_E_INVALID, "BVH deeper than the 64-entry traversal stack");
    c->pair_depth = depth;
    std::vector<float4> tri((size_t)d->ntri * kTriF4, make_float4(0.f, 0.f, 0.f, 0.f)), sh((size_t)d->ntri * 3);
    for (int32_t i = 0; i < d->ntri; i++) {
        mcpt::V3 p0 = mcpt::ld3(d->v0, i), p1 = mcpt::ld3(d->v1, i), p2 = mcpt::ld3(d->v2, i);
        mcpt::V3 e1 = p1 - p0, e2 = p2 - p0;  // Triangle.cu:13-14
        tri[kTriF4 * i + 0] = make_float4(p0.x, p0.y, p0.z, e1.x);
        tri[kTriF4 * i + 1] = make_float4(e1.y, e1.z, e2.x, e2.y);
        const int32_t id = d->tri_id ? d->tri_id[i] : i;
        float fi;
        memcpy(&fi, &id, 4);  // triangle id: the traversal's tie-break key and the API's triangle id
        tri[kTriF4 * i + 2] = make_float4(e2.z, fi, 0.f, 0.f);
        mcpt::V3 n0 = mcpt::ld3(d->n0, i), n1 = mcpt::ld3(d->n1, i), n2 = mcpt::ld3(d->n2, i);
        float fm;
        int mm = d->mat[i];
        memcpy(&fm, &mm, 4);
        sh[3 * i + 0] = make_float4(n0.x, n0.y, n0.z, n1.x);
        sh[3 * i + 1] = make_float4(n1.y, n1.z, n2.x, n2.y);
        sh[3 * i + 2] = make_float4(n2.z, fm, 0.f, 0.f);
    }
    DevScene s{};
    float4 *dn, *dt, *dsh;
    float *dm, *dd;
    int rc;
    if ((rc = dupload(c, c->scene_bufs, &dn, pn.data(), pn.size()))) return rc;
    if ((rc = dupload(c, c->scene_bufs, &dt, tri.data(), tri.size()))) return rc;
    if ((rc = dupload(c, c->scene_bufs, &dsh, sh.data(), sh.size()))) return rc;
    LbvhOutput lb;
    c->last_build_ms = 0.f;
    if (gpu_bvh && d->ntri > 0) {
        HIPCHK(c, hipEventRecord(ev(c, 0), c->stream));
        LbvhInput li{d->ntri, d->v0, d->v1, d->v2, dt, dsh};
        const int brc = c->gpu_bvh_builder == MCPT_GPU_BVH_LBVH ? build_lbvh(li, lb, c->stream) : build_ploc(li, lb, c->stream);
        for (void* q : {(void*)lb.nodes, (void*)lb.tri, (void*)lb.tri_sh})
            if (q) c->scene_bufs.push_back(q);
        if (brc) return set_err(c, MCPT_E_HIP, "GPU BVH build failed (" + std::to_string(brc) + ")");
        HIPCHK(c, hipEventRecord(ev(c, 1), c->stream));
        HIPCHK(c, hipEventSynchronize(c->events[1]));
        HIPCHK(c, hipEventElapsedTime(&c->last_build_ms, c->events[0], c->events[1]));
        if (lb.depth > kMaxStack) return set_err(c, MCPT_E_INVALID, "GPU BVH deeper than the 64-entry traversal stack");
        dn = lb.nodes;
        dt = lb.tri;
        dsh = lb.tri_sh;
        c->pair_depth = lb.depth;
    }
    // Conservative culling (mcpt_core.hpp "conservative box culling").  The bound holds for a box
    // that contains its triangles: a caller BVH whose node boxes miss some of their subtree's
    // vertices is traversed without culling (cull_ok 0).  The occluder cache also needs every box
    // inside its parent's (occ_test tests a leaf box in place of its ancestors): nest_ok.
    bool cull_ok = true, nest_ok = true;
    if (!gpu_bvh && N > 0) {
        std::vector<float> lo(3 * (size_t)N, 3.402823466e+38f), hi(3 * (size_t)N, -3.402823466e+38f);
        for (int i = N - 1; i >= 0; i--) {  // children follow their parent (offset[i] > i, i + 1)
            float* l = &lo[3 * (size_t)i];
            float* h = &hi[3 * (size_t)i];
            if (d->nprims[i] > 0) {
                for (int t = d->offset[i]; t < d->offset[i] + d->nprims[i]; t++)
                    for (const float* v : {d->v0 + 3 * (size_t)t, d->v1 + 3 * (size_t)t, d->v2 + 3 * (size_t)t})
                        for (int k = 0; k < 3; k++) { l[k] = std::fmin(l[k], v[k]); h[k] = std::fmax(h[k], v[k]); }
            } else {
                for (int ch : {i + 1, d->offset[i]}) {
                    for (int k = 0; k < 3; k++) {
                        l[k] = std::fmin(l[k], lo[3 * (size_t)ch + k]);
                        h[k] = std::fmax(h[k], hi[3 * (size_t)ch + k]);
                        if (!(d->bmin[3 * (size_t)ch + k] >= d->bmin[3 * (size_t)i + k]) ||
                            !(d->bmax[3 * (size_t)ch + k] <= d->bmax[3 * (size_t)i + k]))
                            nest_ok = false;
                    }
                }
            }
            for (int k = 0; k < 3; k++)
                if (!(l[k] >= d->bmin[3 * (size_t)i + k]) || !(h[k] <= d->bmax[3 * (size_t)i + k])) cull_ok = false;
        }
        nest_ok = nest_ok && cull_ok;
    }
    if (const char* e = getenv("MCPT_CULL"))  // 0: no culling at all (A/B, and a reference-order traversal)
        if (e[0] == '0' && e[1] == 0) cull_ok = false;
    c->cull_ok = cull_ok;
    c->occ_nest_ok = nest_ok;
    float cull_p = 0.f, root_w = __builtin_huge_valf();
    {
        const uint32_t npairs = (uint32_t)(gpu_bvh ? lb.nnodes : pn.size() / 4);
        const int proot = gpu_bvh ? lb.root_ref : (N > 0 ? ref_of(0) : 0);
        float* tw = nullptr;
        uint32_t* pm = nullptr;
        if (d->ntri > 0) {
            if ((rc = dalloc(c, c->tmp_bufs, &tw, (size_t)d->ntri)) || (rc = dalloc(c, c->tmp_bufs, &pm, 1))) return rc;
            HIPCHK(c, hipMemsetAsync(pm, 0, sizeof(uint32_t), c->stream));
            // MCPT_CULL_PLANE=0: the general bound for axis-plane triangles too (A/B; the host
            // builder's isolation of unbounded triangles reads the same variable)
            const char* pl = std::getenv("MCPT_CULL_PLANE");
            const bool plane = !(pl && pl[0] == '0' && pl[1] == 0);
            mcpt_dev::launch_cull_margins(dn, npairs, dt, (uint32_t)d->ntri, tw, pm, c->pair_depth + 2, plane, c->stream);
            HIPCHK(c, hipGetLastError());
            uint32_t pb = 0;
            HIPCHK(c, hipMemcpyAsync(&pb, pm, sizeof(pb), hipMemcpyDeviceToHost, c->stream));
            float4 rq = make_float4(0.f, 0.f, 0.f, 0.f);
            std::vector<float> leaf_w;
            if (proot >= 0 && npairs > 0) {
                HIPCHK(c, hipMemcpyAsync(&rq, dn + 4 * (size_t)proot + 3, sizeof(rq), hipMemcpyDeviceToHost, c->stream));
            } else if (proot < 0) {  // the whole tree is one leaf
                const uint32_t off = (uint32_t)proot & 0xffffffu, cnt = (((uint32_t)proot >> 24) & 7u) + 1u;
                leaf_w.resize(cnt);
                HIPCHK(c, hipMemcpyAsync(leaf_w.data(), tw + off, cnt * sizeof(float), hipMemcpyDeviceToHost, c->stream));
            }
            HIPCHK(c, hipStreamSynchronize(c->stream));
            memcpy(&cull_p, &pb, 4);
            root_w = proot >= 0 ? std::fmax(rq.z, rq.w) : 0.f;
            for (float w : leaf_w) root_w = std::fmax(root_w, w);
            free_list(c->tmp_bufs);
        }
    }
    if ((rc = dupload(c, c->scene_bufs, &dm, d->mat_params, (size_t)d->nmat * 8))) return rc;
    if ((rc = dupload(c, c->scene_bufs, &dd, d->dir_params, (size_t)d->ndir * 7))) return rc;
    s.nodes = dn; s.tri = dt; s.tri_sh = dsh; s.mats = dm; s.dirs = dd;
    // Node width: 4-wide nodes (one 128-B line tests four boxes, half the levels) for trees
    // of more than 32 MB of pair nodes, child pairs otherwise.  Per launch, interleaved on one
    // box: config 5 (2 M tris, 128 MB) 16.7 -> 15.6 ms and config 3 (871K, 55 MB) 1.154 ->
    // 1.148 ms with quads; config 4 (252K, 16 MB) 7.69 -> 7.79 ms and config 2 (4.8K) 0.783 ->
    // 0.848 ms, so those keep pairs.  MCPT_BVH_WIDTH=2/4 forces a width.
    const size_t tree_pairs = gpu_bvh ? (size_t)lb.nnodes : pn.size() / 4;
    uint32_t nnodes = (uint32_t)tree_pairs;  // nodes of the uploaded width (the leaf-box pass)
    int width = tree_pairs * 64 > ((size_t)32 << 20) ? 4 : 2;
    if (const char* we = getenv("MCPT_BVH_WIDTH"))
        if ((we[0] == '2' || we[0] == '4') && we[1] == 0) width = we[0] - '0';
    int quad_root = 0, quad_push = 0;
    if (width == 4) {
        // 4-wide traversal: collapse the pair tree (host SAH or GPU LBVH) into 4-wide nodes
        std::vector<float4> pairs;
        int proot;
        if (gpu_bvh && d->ntri > 0) {
            pairs.resize((size_t)lb.nnodes * 4);
            if (lb.nnodes) HIPCHK(c, hipMemcpy(pairs.data(), lb.nodes, pairs.size() * sizeof(float4), hipMemcpyDeviceToHost));
            proot = lb.root_ref;
        } else {  // the uploaded pairs, with the margins launch_cull_margins wrote
            pairs.resize(pn.size());
            if (!pn.empty()) HIPCHK(c, hipMemcpy(pairs.data(), dn, pairs.size() * sizeof(float4), hipMemcpyDeviceToHost));
            proot = N > 0 ? ref_of(0) : 0;
        }
        std::vector<float4> quads;
        int max_push = 0;
        if (d->ntri > 0) {
            pairs_to_quads(pairs, proot, quads, quad_root, max_push);
            if (max_push > kMaxStack) return set_err(c, MCPT_E_INVALID, "4-wide BVH needs more than 64 stack entries");
            quad_push = max_push;
            float4* dq;
            if ((rc = dupload(c, c->scene_bufs, &dq, quads.data(), quads.size()))) return rc;
            s.nodes = dq;
            nnodes = (uint32_t)(quads.size() / 8);
        }
    }
    s.nlights = 1 + d->ndir;
    if (gpu_bvh && d->ntri > 0) {
        for (int k = 0; k < 3; k++) { s.root_mn[k] = lb.root_mn[k]; s.root_mx[k] = lb.root_mx[k]; }
        s.root_ref = width == 4 ? (lb.root_ref < 0 ? lb.root_ref : quad_root) : lb.root_ref;
    } else if (N > 0) {
        for (int k = 0; k < 3; k++) { s.root_mn[k] = d->bmin[k]; s.root_mx[k] = d->bmax[k]; }
        s.root_ref = width == 4 ? (ref_of(0) < 0 ? ref_of(0) : quad_root) : ref_of(0);
    } else {
        // empty scene: a root box that no ray can enter
        for (int k = 0; k < 3; k++) { s.root_mn[k] = 1.f; s.root_mx[k] = -1.f; }
        s.root_ref = 0;
    }
    s.env.mode = d->env_mode;
    for (int k = 0; k < 3; k++) s.env.color[k] = d->env_color[k];
    s.env.ls = d->env_ls;
    s.env.w = d->env_w;
    s.env.h = d->env_h;
    s.env.tex = nullptr;
    s.env.guide_m = s.env.guide_c = nullptr;
    s.env.ltab[0] = s.env.ltab[1] = nullptr;
    s.env.lrow[0] = s.env.lrow[1] = nullptr;
    s.env.lcol[0] = s.env.lcol[1] = nullptr;
    if (d->env_mode == 1) {
        float4* tx;
        float *my, *cy, *pd;
        const int W = d->env_w, H = d->env_h;
        size_t WH = (size_t)W * H;
        if ((rc = dupload(c, c->scene_bufs, &tx, reinterpret_cast<const float4*>(d->env_tex), WH))) return rc;
        c->env_device_built = !d->env_marginal_y;
        c->last_env_build_ms = 0.f;
        if (!c->env_device_built) {
            if ((rc = dupload(c, c->scene_bufs, &my, d->env_marginal_y, (size_t)H))) return rc;
            if ((rc = dupload(c, c->scene_bufs, &cy, d->env_conds_y, WH))) return rc;
            if ((rc = dupload(c, c->scene_bufs, &pd, d->env_pdf, WH))) return rc;
        } else {
            // build_environment_light (light_initialization_kernels.cu:134-161) on the device
            if ((rc = dalloc(c, c->scene_bufs, &my, (size_t)H)) || (rc = dalloc(c, c->scene_bufs, &cy, WH)) ||
                (rc = dalloc(c, c->scene_bufs, &pd, WH)))
                return rc;
            float* scratch = nullptr;
            hipError_t e = hipMalloc(&scratch, mcpt_dev::env_build_scratch_floats(W, H) * sizeof(float));
            if (e != hipSuccess) return set_err(c, MCPT_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
            HIPCHK(c, hipEventRecord(ev(c, 0), c->stream));
            mcpt_dev::launch_env_build(tx, W, H, scratch, my, cy, pd, c->stream);
            HIPCHK(c, hipEventRecord(ev(c, 1), c->stream));
            e = hipGetLastError();
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            (void)hipFree(scratch);
            if (e != hipSuccess) return set_err(c, MCPT_E_HIP, std::string("env build: ") + hipGetErrorString(e));
            float ms = 0.f;
            HIPCHK(c, hipEventElapsedTime(&ms, ev(c, 0), ev(c, 1)));
            c->last_env_build_ms = ms;
        }
        s.env.tex = tx; s.env.marginal_y = my; s.env.conds_y = cy; s.env.pdf = pd;
        mcpt_dev::launch_env_pack(tx, pd, WH, c->stream);  // before the tables below read env_pdf
        HIPCHK(c, hipGetLastError());
        // search guides for env_cell, on the device for either source of tables: valid on
        // a sorted, NaN-free marginal CDF and conditional rows that are sorted and NaN-free
        // or NaN throughout (upper_bound returns 0 on such a row for every value, and so
        // does the guided search with its all-zero guide).  Every HRDI map has one: row 0's
        // sin(0) = 0 makes it 0 / (denom * 0) (light_initialization_kernels.cu:72).
        // Otherwise the plain bisection is used.
        s.env.guide_m = s.env.guide_c = nullptr;
        c->env_guides = false;
        if (W <= 65535 && H <= 65535) {
            const size_t G1 = mcpt::kEnvGuide + 1;
            uint16_t *dgm, *dgc;
            uint32_t* dbad;
            if ((rc = dalloc(c, c->scene_bufs, &dgm, G1)) || (rc = dalloc(c, c->scene_bufs, &dgc, (size_t)H * G1)) ||
                (rc = dalloc(c, c->scene_bufs, &dbad, 1)))
                return rc;
            HIPCHK(c, hipMemsetAsync(dbad, 0, sizeof(uint32_t), c->stream));
            mcpt_dev::launch_env_guides(my, cy, W, H, dgm, dgc, dbad, c->stream);
            HIPCHK(c, hipGetLastError());
            uint32_t bad = 1;
            HIPCHK(c, hipMemcpyAsync(&bad, dbad, sizeof(bad), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            bool ok = bad == 0;
            if (const char* g = std::getenv("MCPT_ENV_GUIDES")) ok = ok && g[0] != '0';  // 0: plain bisection (A/B, tests)
            if (ok) {
                s.env.guide_m = dgm;
                s.env.guide_c = dgc;
                c->env_guides = true;
            }
        }
        // light-sample tables, reference and quality mode (k_env_table)
        if ((size_t)(d->env_w + 1) * d->env_h < ((size_t)1 << 28)) {
            const size_t ne = (size_t)(d->env_w + 1) * d->env_h;
            float4 *lt0, *lt1;
            float2 *rc0, *rc1;  // row table (h entries) then column table (w + 1)
            const size_t nrc = (size_t)d->env_h + d->env_w + 1;
            if ((rc = dalloc(c, c->scene_bufs, &lt0, ne)) || (rc = dalloc(c, c->scene_bufs, &lt1, ne)) ||
                (rc = dalloc(c, c->scene_bufs, &rc0, nrc)) || (rc = dalloc(c, c->scene_bufs, &rc1, nrc)))
                return rc;
            launch_env_table(s.env, false, lt0, rc0, rc0 + d->env_h, c->stream);
            launch_env_table(s.env, true, lt1, rc1, rc1 + d->env_h, c->stream);
            HIPCHK(c, hipGetLastError());
            HIPCHK(c, hipStreamSynchronize(c->stream));
            s.env.ltab[0] = lt0;
            s.env.ltab[1] = lt1;
            s.env.lrow[0] = rc0;
            s.env.lrow[1] = rc1;
            s.env.lcol[0] = rc0 + d->env_h;
            s.env.lcol[1] = rc1 + d->env_h;
        }
    }
    s.depth = width == 4 ? quad_push : c->pair_depth;
    s.width = width;
    s.cull_p = cull_p;
    s.root_w = root_w;
    s.cull_ok = cull_ok ? 1 : 0;
    // Any-hit occluder cache (kernels.hip occ_hit1): every triangle record's leaf box and the
    // (origin cell x direction bin) table, empty at upload.  MCPT_OCC_G=0 turns it off;
    // MCPT_OCC_G / MCPT_OCC_B set the cells per axis / bins per face coordinate.
    s.ntri = (uint32_t)d->ntri;
    s.occ = nullptr;
    s.occ_rec = nullptr;
    {
        // 24^3 cells x 6 x 12^2 bins x 2 ways = 96 MB.  Config 2 with the table emptied at every film
        // clear: 62 % of the any-hit rays resolved (16^3 x 8^2: 60 %, 32^3 x 16^2: 64 %; frame rates
        // within 1 %: the bigger tables resolve more but warm up more slowly and miss L2 more)
        int G = 24, B = 12;
        if (const char* e = getenv("MCPT_OCC_G")) G = atoi(e);
        if (const char* e = getenv("MCPT_OCC_B")) B = atoi(e);
        // the index G^3 * 6 * B^2 must fit 32 bits
        // (off unless every box nests in its parent's: occ_test relies on it, see cull_ok above)
        if (G > 0 && G <= 64 && B > 0 && B <= 64 && (uint64_t)G * G * G * 6 * B * B <= 0xffffffffull && d->ntri > 0 &&
            c->occ_nest_ok) {
            float4* lbx;
            uint32_t* occ;
            const size_t ne = occ_entries(G, B);
            if ((rc = dalloc(c, c->scene_bufs, &lbx, kOccRecF4 * (size_t)d->ntri)) ||
                (rc = dalloc(c, c->scene_bufs, &occ, ne + kOccGateWords)))
                return rc;
            // NaN boxes (all-ones bytes) for a record no leaf holds: occ_test's slab then fails
            HIPCHK(c, hipMemsetAsync(lbx, 0xff, kOccRecF4 * (size_t)d->ntri * sizeof(float4), c->stream));
            HIPCHK(c, hipMemsetAsync(occ, 0xff, ne * sizeof(uint32_t), c->stream));
            HIPCHK(c, hipMemsetAsync(occ + ne, 0, kOccGateWords * sizeof(uint32_t), c->stream));  // the lookup gate: on
            launch_occ_records(s, nnodes, lbx, c->stream);
            HIPCHK(c, hipGetLastError());
            HIPCHK(c, hipStreamSynchronize(c->stream));
            s.occ_rec = lbx;
            s.occ = occ;
            s.occ_gate = occ + ne;
            c->occ_entries_n = ne;
            s.occ_g = G;
            s.occ_b = B;
            for (int k = 0; k < 3; k++) {
                const float ext = s.root_mx[k] - s.root_mn[k];
                s.occ_inv[k] = ext > 0.f && ext < 3.4e38f ? (float)G / ext : 0.f;
            }
        }
    }
    c->scene = s;
    c->ntri = d->ntri;
    c->occ_init = nullptr;  // (the previous scene's copy went with scene_bufs)
    if (s.occ) {
        // Occluder-table pre-fill: one any-hit probe ray per table key (origin cell centre, direction
        // bin centre; k_occ_probes) traced with occluder recording on, so every key whose probe is
        // occluded starts with a triangle -- derived from the scene alone, like the BVH.  Film
        // clears restore this table, so every frame starts from the same one and no frame depends
        // on another.  MCPT_OCC_PREFILL=0: frames start from an empty table.
        const char* pe = getenv("MCPT_OCC_PREFILL");
        if (!(pe && pe[0] == '0' && pe[1] == 0)) {
            const uint32_t nkeys = (uint32_t)(c->occ_entries_n / kOccWays);
            float4 *pro, *prd;
            uint8_t* pvis;
            free_list(c->tmp_bufs);
            if ((rc = dalloc(c, c->tmp_bufs, &pro, nkeys)) || (rc = dalloc(c, c->tmp_bufs, &prd, nkeys)) ||
                (rc = dalloc(c, c->tmp_bufs, &pvis, nkeys)) || (rc = dalloc(c, c->scene_bufs, &c->occ_init, c->occ_entries_n)))
                return rc;
            launch_occ_probes(s, pro, prd, nkeys, c->stream);
            TraceArgs ta{};
            ta.scene = s;  // occ on, gate words 0: the finish records the occluder of every occluded probe
            ta.nshards = 1;
            TraceSet& ts = ta.set[1];
            ts.ro = pro;
            ts.rd = prd;
            ts.count = nkeys;
            ts.shard_cap = nkeys;
            ta.vis = pvis;
            ta.grab = &c->cnt->grab[0][0];
            launch_trace(ta, c->geom, c->stream);
            HIPCHK(c, hipMemsetAsync(c->cnt->grab, 0, sizeof(c->cnt->grab), c->stream));  // hand-out counters back to 0
            HIPCHK(c, hipMemcpyAsync(c->occ_init, s.occ, c->occ_entries_n * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                     c->stream));
            const uint32_t warm[kOccGateWords] = {0u, 0u, 1u};  // the table holds occluders: lookups from the start
            HIPCHK(c, hipMemcpyAsync(s.occ_gate, warm, sizeof(warm), hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipGetLastError());
            HIPCHK(c, hipStreamSynchronize(c->stream));
            free_list(c->tmp_bufs);
        }
    }
    if (c->has_scene_before) c->film_stale = true;  // a re-upload notifies the film
    c->has_scene = true;
    return MCPT_OK;
}

int mcpt_scene_upload(mcpt_ctx* c, const mcpt_scene_desc* d) { return scene_upload(c, d, false); }
int mcpt_scene_upload_gpu_bvh(mcpt_ctx* c, const mcpt_scene_desc* d) { return scene_upload(c, d, true); }
int mcpt_set_gpu_bvh_builder(mcpt_ctx* c, int32_t builder) {
    if (!c || (builder != MCPT_GPU_BVH_LBVH && builder != MCPT_GPU_BVH_PLOC))
        return set_err(c, MCPT_E_INVALID, "unknown GPU BVH builder");
    c->gpu_bvh_builder = builder;
    return MCPT_OK;
}
float mcpt_debug_last_build_ms(const mcpt_ctx* c) { return c ? c->last_build_ms : -1.f; }
float mcpt_debug_last_env_build_ms(const mcpt_ctx* c) { return c ? c->last_env_build_ms : -1.f; }

int mcpt_debug_env_tables(mcpt_ctx* c, float* marginal_y, float* conds_y, float* pdf, int32_t* flags) {
    if (!c) return set_err(c, MCPT_E_INVALID, "null context");
    if (!c->has_scene || c->scene.env.mode != 1 || !c->scene.env.tex) return set_err(c, MCPT_E_INVALID, "no HRDI scene uploaded");
    const mcpt::EnvView& e = c->scene.env;
    const size_t WH = (size_t)e.w * e.h;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (marginal_y) HIPCHK(c, hipMemcpy(marginal_y, e.marginal_y, (size_t)e.h * sizeof(float), hipMemcpyDeviceToHost));
    if (conds_y) HIPCHK(c, hipMemcpy(conds_y, e.conds_y, WH * sizeof(float), hipMemcpyDeviceToHost));
    if (pdf) HIPCHK(c, hipMemcpy(pdf, e.pdf, WH * sizeof(float), hipMemcpyDeviceToHost));
    if (flags) *flags = (c->env_device_built ? 1 : 0) | (c->env_guides ? 2 : 0);
    return MCPT_OK;
}
int mcpt_debug_node_layout(const mcpt_ctx* c) { return c ? c->node_layout : MCPT_E_INVALID; }
int mcpt_debug_ray_counts(const mcpt_ctx* c, uint64_t* out) {
    if (!c || !out) return MCPT_E_INVALID;
    const CounterBlock& t = c->totals;
    const bool ok = c->totals_ok;
    out[0] = ok ? t.tot_ext : 0;    // extension rays (queued + resolved in place)
    out[1] = ok ? t.tot_ext_q : 0;  // extension rays k_trace traversed
    out[2] = ok ? t.tot_any : 0;    // shadow + BRDF visibility rays
    out[3] = ok ? t.tot_any_q : 0;  // any-hit rays k_trace traversed
    out[4] = ok ? t.tot_occ : 0;    // any-hit rays the occluder cache resolved in k_material
    return MCPT_OK;
}
int mcpt_debug_occ_stats(const mcpt_ctx* c, uint64_t* resolved, int32_t* enabled) {
    if (!c) return MCPT_E_INVALID;
    if (resolved) *resolved = c->totals_ok ? c->totals.tot_occ : 0;
    if (enabled) *enabled = c->scene.occ != nullptr;
    return MCPT_OK;
}

int mcpt_camera_set(mcpt_ctx* c, const mcpt_camera* cam) {
    if (!c || !cam) return set_err(c, MCPT_E_INVALID, "null argument");
    mcpt::CamView nc = c->cam;
    memcpy(nc.ivp, cam->inv_view_proj, sizeof(nc.ivp));
    memcpy(nc.iv, cam->inv_view, sizeof(nc.iv));
    nc.lens_radius = cam->lens_radius;
    nc.focal = cam->focal;
    if (c->has_cam && memcmp(&nc, &c->cam, sizeof(nc)) != 0) c->film_stale = true;
    c->cam = nc;
    c->has_cam = true;
    return MCPT_OK;
}

static int set_tiles_internal(mcpt_ctx* c, const std::vector<int2>& t) {
    // per-shard queue capacity: shard = k_shade block mod kShards (a block pushes <= one ray per thread)
    const uint32_t nblocks = (uint32_t)t.size() * (uint32_t)shade_blocks_per_tile((int)(c->tile_w * c->tile_h), (int)c->slots);
    c->ext_cap = std::max<uint32_t>(1, (nblocks + kShards - 1) / kShards) * kBlock;
    c->any_cap = 2 * c->ext_cap;
    const size_t need = (size_t)kShards * c->ext_cap;
    if (need > c->queue_alloc) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->ext_q) (void)hipFree(c->ext_q);
        if (c->any_q) (void)hipFree(c->any_q);
        if (c->mat_q) (void)hipFree(c->mat_q);
        if (c->any_ray) (void)hipFree(c->any_ray);
        c->ext_q = c->any_q = c->mat_q = nullptr;
        c->any_ray = nullptr;
        c->queue_alloc = 0;
        if (hipMalloc(&c->ext_q, need * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&c->any_q, 2 * need * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&c->mat_q, need * 8 * sizeof(uint32_t)) != hipSuccess ||  // MatRec + beta per slot
            hipMalloc(&c->any_ray, 4 * need * sizeof(float4)) != hipSuccess)    // o + d per any-queue entry
            return set_err(c, MCPT_E_NOMEM, "queue allocation failed");
        c->queue_alloc = need;
    }
    c->p.sray_o = c->any_ray;  // indexed by any-queue position (kShards * any_cap = 2 * need entries)
    c->p.sray_d = c->any_ray + 2 * c->queue_alloc;
    if (t.size() > c->tiles_cap) {
        if (c->tiles) HIPCHK(c, hipFree(c->tiles));
        c->tiles = nullptr;
        HIPCHK(c, hipMalloc(&c->tiles, std::max<size_t>(t.size(), 1) * sizeof(int2)));
        c->tiles_cap = (uint32_t)t.size();
    }
    if (!t.empty()) HIPCHK(c, hipMemcpyAsync(c->tiles, t.data(), t.size() * sizeof(int2), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->tiles_h = t;
    return MCPT_OK;
}
static std::vector<int2> all_tiles(const mcpt_ctx* c) {
    std::vector<int2> t;
    uint32_t nx = (c->W + c->tile_w - 1) / c->tile_w, ny = (c->H + c->tile_h - 1) / c->tile_h;
    for (uint32_t y = 0; y < ny; y++)
        for (uint32_t x = 0; x < nx; x++) t.push_back(make_int2((int)x, (int)y));
    return t;
}

int mcpt_film_clear(mcpt_ctx* c) {
    if (!c || !c->P) return set_err(c, MCPT_E_INVALID, "film not allocated");
    HIPCHK(c, hipSetDevice(c->device));
    ClearArgs a{c->p.flags, c->p.samples, c->p.Ld, (uint32_t)(c->npx * c->slots), (uint32_t)c->npx};
    launch_clear(a, c->stream);
    HIPCHK(c, hipGetLastError());
    if (c->compact) {  // the W x H film also holds pixels unpacked from other contexts (mcpt_film_unpack_tiles)
        HIPCHK(c, hipMemsetAsync(c->film_Ld, 0, c->P * sizeof(float4), c->stream));
        HIPCHK(c, hipMemsetAsync(c->film_samples, 0, c->P * sizeof(uint32_t), c->stream));
    }
    if (c->blk_done) HIPCHK(c, hipMemsetAsync(c->blk_done, 0, c->blk_done_n, c->stream));
    // The occluder cache starts every film from the same table -- the upload's pre-fill, or empty --
    // with its lookup gate on, so a frame's work never depends on the frames before it.  (It only
    // ever chooses which triangle an any-hit ray tests first; the 96 MB copy takes ~0.04 ms.)
    if (c->scene.occ) {
        if (c->occ_init) {  // the upload's pre-filled table (scene-derived), the same for every frame
            HIPCHK(c, hipMemcpyAsync(c->scene.occ, c->occ_init, c->occ_entries_n * sizeof(uint32_t),
                                     hipMemcpyDeviceToDevice, c->stream));
            static const uint32_t warm[kOccGateWords] = {0u, 0u, 1u};
            HIPCHK(c, hipMemcpyAsync(c->scene.occ_gate, warm, sizeof(warm), hipMemcpyHostToDevice, c->stream));
        } else {
            HIPCHK(c, hipMemsetAsync(c->scene.occ, 0xff, c->occ_entries_n * sizeof(uint32_t), c->stream));
            HIPCHK(c, hipMemsetAsync(c->scene.occ_gate, 0, kOccGateWords * sizeof(uint32_t), c->stream));
        }
    }
    c->film_stale = false;
    c->unpacked.clear();
    HIPCHK(c, hipMemsetAsync(c->cnt, 0, sizeof(CounterBlock), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    memset(&c->totals, 0, sizeof(c->totals));  // the counters are now zero on the device too
    memset(c->phase_base, 0, sizeof(c->phase_base));
    c->totals_ok = true;
    return MCPT_OK;
}

// Film state for the current film size, path slots, layout and tile set: the path streams (slots x
// npx paths), the k_shade block flags and the W x H film of the slot sums (slots > 1 or compact).
// Frees the previous film state first; the caller clears the film.
static int alloc_film_state(mcpt_ctx* c) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    free_list(c->film_bufs);
    {
        DevPaths keep{};  // the queue-owned any-hit ray buffers stay
        keep.sray_o = c->p.sray_o;
        keep.sray_d = c->p.sray_d;
        c->p = keep;
    }
    c->film_Ld = nullptr;
    c->film_samples = nullptr;
    c->blk_done = nullptr;
    c->blk_done_n = 0;
    const uint32_t w = c->W, h = c->H, tw = c->tile_w, th = c->tile_h;
    const size_t npix = (size_t)w * h;
    const size_t npx = c->compact ? c->tiles_h.size() * (size_t)tw * th : npix;
    const size_t P = npx * c->slots;  // P: paths
    c->npx = 0;
    if (P >= (1ull << 31)) return set_err(c, MCPT_E_INVALID, "film too large for the path slots");
    DevPaths p{};
    int rc;
    if ((rc = dalloc(c, c->film_bufs, &p.ray_o, P)) || (rc = dalloc(c, c->film_bufs, &p.ray_d, P)) ||
        (rc = dalloc(c, c->film_bufs, &p.hit_tri, P)) ||
        (rc = dalloc(c, c->film_bufs, &p.beta, P)) || (rc = dalloc(c, c->film_bufs, &p.nee0, P)) ||
        (rc = dalloc(c, c->film_bufs, &p.nee1, P)) || (rc = dalloc(c, c->film_bufs, &p.Ld, P)) ||
        (rc = dalloc(c, c->film_bufs, &p.flags, P)) || (rc = dalloc(c, c->film_bufs, &p.samples, P)) ||
        (rc = dalloc(c, c->film_bufs, &p.vis, 2 * P)))
        return rc;
    {  // k_shade block done flags: slots x film tiles x blocks per tile
        const size_t ntiles = (size_t)((w + tw - 1) / tw) * ((h + th - 1) / th);
        c->blk_done_n = c->slots * ntiles * (size_t)shade_blocks_per_tile((int)(tw * th), 1);
        if ((rc = dalloc(c, c->film_bufs, &c->blk_done, c->blk_done_n))) return rc;
    }
    if ((c->slots > 1 || c->compact) && ((rc = dalloc(c, c->film_bufs, &c->film_Ld, npix)) ||
                                         (rc = dalloc(c, c->film_bufs, &c->film_samples, npix))))
        return rc;
    HIPCHK(c, hipMemset(p.hit_tri, 0xff, P * sizeof(int32_t)));
    HIPCHK(c, hipMemset(p.vis, 0, 2 * P));
    p.sray_o = c->p.sray_o;  // the any-hit rays live with the queues (set_tiles_internal)
    p.sray_d = c->p.sray_d;
    c->p = p;
    c->npx = npx;
    return MCPT_OK;
}

int mcpt_film_resize(mcpt_ctx* c, uint32_t w, uint32_t h, uint32_t tw, uint32_t th) {
    if (!c || w == 0 || h == 0 || tw == 0 || th == 0) return set_err(c, MCPT_E_INVALID, "bad film size");
    if ((uint64_t)w * h >= (1ull << 31)) return set_err(c, MCPT_E_INVALID, "film too large");
    if ((uint64_t)tw * th > (1ull << 26)) return set_err(c, MCPT_E_INVALID, "tile too large");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    free_list(c->film_bufs);
    c->P = 0;
    c->npx = 0;
    c->p = DevPaths{};  // (set_tiles_internal below re-points the any-hit ray buffers)
    c->blk_done = nullptr;
    c->blk_done_n = 0;
    c->W = w; c->H = h; c->tile_w = tw; c->tile_h = th;
    for (uint32_t** q : {&c->ext_q, &c->any_q, &c->mat_q}) {  // re-sized for the new tile set below
        if (*q) (void)hipFree(*q);
        *q = nullptr;
    }
    if (c->any_ray) (void)hipFree(c->any_ray);
    c->any_ray = nullptr;
    c->queue_alloc = 0;
    int rc = set_tiles_internal(c, all_tiles(c));
    if (rc) return rc;
    if ((rc = alloc_film_state(c))) return rc;
    c->P = (size_t)w * h;
    return mcpt_film_clear(c);
}

// A new tile set.  In the compact layout the path state follows the tile set: it is re-allocated and
// the film cleared (a tile listed twice would share its paths: rejected).
static bool has_tile(const std::vector<int2>& v, int2 t) {
    for (const int2& o : v)
        if (o.x == t.x && o.y == t.y) return true;
    return false;
}
static int set_tiles_checked(mcpt_ctx* c, const std::vector<int2>& t) {
    if (!c->compact) {
        for (const int2& x : t)
            if (has_tile(c->unpacked, x))
                return set_err(c, MCPT_E_INVALID, "a tile of the set holds pixels unpacked from another context: clear the film first");
        return set_tiles_internal(c, t);
    }
    for (size_t i = 0; i < t.size(); i++)
        for (size_t j = 0; j < i; j++)
            if (t[i].x == t[j].x && t[i].y == t[j].y)
                return set_err(c, MCPT_E_INVALID, "compact paths: a tile is listed twice");
    const std::vector<int2> old = c->tiles_h;
    int rc = set_tiles_internal(c, t);
    if (rc) return rc;
    const size_t P = c->P;
    c->P = 0;  // the film is not allocated until the new path state is
    if ((rc = alloc_film_state(c))) {  // e.g. out of memory: back to the previous tile set, as
        const std::string err = c->err;  // mcpt_set_path_slots / mcpt_set_compact_paths do
        if (set_tiles_internal(c, old) == MCPT_OK && alloc_film_state(c) == MCPT_OK) {
            c->P = P;
            (void)mcpt_film_clear(c);
        }
        return set_err(c, rc, err);
    }
    c->P = P;
    return mcpt_film_clear(c);
}

int mcpt_set_tiles(mcpt_ctx* c, const uint32_t* xy, uint32_t n) {
    if (!c || !c->P) return set_err(c, MCPT_E_INVALID, "film not allocated");
    HIPCHK(c, hipSetDevice(c->device));
    if (!xy) return set_tiles_checked(c, all_tiles(c));
    std::vector<int2> t;
    uint32_t nx = (c->W + c->tile_w - 1) / c->tile_w, ny = (c->H + c->tile_h - 1) / c->tile_h;
    for (uint32_t i = 0; i < n; i++) {
        if (xy[2 * i] >= nx || xy[2 * i + 1] >= ny) return set_err(c, MCPT_E_INVALID, "tile out of range");
        t.push_back(make_int2((int)xy[2 * i], (int)xy[2 * i + 1]));
    }
    return set_tiles_checked(c, t);
}

int mcpt_set_compact_paths(mcpt_ctx* c, int32_t on) {
    if (!c) return MCPT_E_INVALID;
    const bool v = on != 0;
    if (v == c->compact) return MCPT_OK;
    c->compact = v;
    if (!c->P) return MCPT_OK;  // takes effect with the film's allocation
    HIPCHK(c, hipSetDevice(c->device));
    const size_t P = c->P;
    c->P = 0;
    int rc = alloc_film_state(c);
    if (rc) {  // e.g. out of memory: back to the previous layout
        const std::string err = c->err;
        c->compact = !v;
        if (alloc_film_state(c) == MCPT_OK) {
            c->P = P;
            (void)mcpt_film_clear(c);
        }
        return set_err(c, rc, err);
    }
    c->P = P;
    return mcpt_film_clear(c);
}

static hipEvent_t ev(mcpt_ctx* c, size_t i) {
    while (c->events.size() <= i) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->events.push_back(e);
    }
    return c->events[i];
}

// The camera records of a W x H film under the current camera (k_cam_table: gen_ray_pixel of every
// pixel, 32 B each), rebuilt on the context's stream when the film size or the camera changed.
static int cam_table(mcpt_ctx* c, uint32_t W, uint32_t H, const float4** px, const float4** dir) {
    const size_t n = (size_t)W * H;
    if (!(c->cam_tab_ok && c->cam_tab_W == W && c->cam_tab_H == H && memcmp(&c->cam_tab_cam, &c->cam, sizeof(c->cam)) == 0)) {
        if (n > c->cam_tab_cap) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            if (c->cam_tab) (void)hipFree(c->cam_tab);
            c->cam_tab = nullptr;
            c->cam_tab_cap = 0;
            c->cam_tab_ok = false;
            if (hipMalloc(&c->cam_tab, 2 * n * sizeof(float4)) != hipSuccess)
                return set_err(c, MCPT_E_NOMEM, "camera table allocation failed");
            c->cam_tab_cap = n;
        }
        launch_cam_table(c->cam, (int)W, (int)H, c->cam_tab, c->cam_tab + n, c->stream);
        HIPCHK(c, hipGetLastError());
        c->cam_tab_W = W;
        c->cam_tab_H = H;
        c->cam_tab_cam = c->cam;
        c->cam_tab_ok = true;
    }
    *px = c->cam_tab;
    *dir = c->cam_tab + n;
    return MCPT_OK;
}

static int check_ready(mcpt_ctx* c) {
    if (!c) return MCPT_E_INVALID;
    if (!c->has_scene) return set_err(c, MCPT_E_INVALID, "no scene uploaded");
    if (!c->has_cam) return set_err(c, MCPT_E_INVALID, "no camera set");
    if (!c->P) return set_err(c, MCPT_E_INVALID, "film not allocated");
    if (!c->ext_q || !c->any_q || !c->mat_q || !c->any_ray)  // a failed (re)allocation left none
        return set_err(c, MCPT_E_NOMEM, "ray queues not allocated");
    return MCPT_OK;
}

// One wavefront iteration over the current tile set: shade -> extend -> any-hit.
static int enqueue_iteration(mcpt_ctx* c, size_t evbase, bool timing, const int2* tiles, int ntiles, const int* tile_base) {
    ShadeArgs sa;
    sa.scene = c->scene;
    sa.cam = c->cam;
    sa.p = c->p;
    sa.tiles = tiles;
    sa.ntiles = ntiles;
    sa.tile_w = (int)c->tile_w;
    sa.tile_h = (int)c->tile_h;
    sa.W = (int)c->W;
    sa.H = (int)c->H;
    sa.spp = c->cfg.spp;
    sa.max_depth = c->cfg.max_depth;
    sa.rr_depth = c->cfg.rr_depth;
    sa.seed = c->cfg.seed;
    sa.slots = (int)c->slots;
    sa.slots_rcp = 1.0f / (float)c->slots;
    sa.npx = (uint32_t)c->npx;
    sa.compact = c->compact ? 1 : 0;
    sa.tile_base = tile_base;
    sa.ext_q = c->ext_q;
    sa.any_q = c->any_q;
    sa.mat_rec = reinterpret_cast<uint4*>(c->mat_q);
    sa.mat_beta = reinterpret_cast<float4*>(c->mat_q) + (size_t)kShards * c->ext_cap;
    sa.ext_cap = c->ext_cap;
    sa.any_cap = c->any_cap;
    sa.cnt = c->cnt;
    sa.blk_done = c->blk_done_off ? nullptr : c->blk_done;
    if (int rc = cam_table(c, c->W, c->H, &sa.cam_px, &sa.cam_dir)) return rc;
    const int bpt = shade_blocks_per_tile((int)(c->tile_w * c->tile_h), (int)c->slots);
    if (timing) HIPCHK(c, hipEventRecord(ev(c, evbase + 0), c->stream));
    if (sa.ntiles > 0)
        launch_shade(sa, sa.ntiles * bpt, c->geom, (c->cfg.flags & MCPT_FLAG_FIXED) != 0, c->stream);
    if (timing) HIPCHK(c, hipEventRecord(ev(c, evbase + 1), c->stream));
    // extension (closest hit) and any-hit rays in one persistent launch
    TraceArgs ta{};
    ta.scene = c->scene;
    ta.nshards = kShards;
    TraceSet& e = ta.set[0];
    e.ro = c->p.ray_o;
    e.rd = c->p.ray_d;
    e.queue = c->ext_q;
    e.count_ptr = &c->cnt->shard[0][C_EXT];
    e.shard_cap = c->ext_cap;
    e.stats = c->count_work ? &c->cnt->shard[0][C_STATS] : nullptr;  // mcpt_set_work_counters
    e.prefiltered = 1;  // k_shade queues only rays that enter the root box
    TraceSet& v = ta.set[1];
    v.ro = c->p.sray_o;
    v.rd = c->p.sray_d;
    v.queue = c->any_q;
    v.count_ptr = &c->cnt->shard[0][C_ANY];
    v.shard_cap = c->any_cap;
    v.stats = c->count_work ? &c->cnt->shard[0][C_STATS + 3] : nullptr;
    v.prefiltered = 1;
    v.ray_at_slot = 1;  // k_material stores the any-hit rays at their queue positions
    ta.phase = c->count_work ? &c->cnt->shard[0][C_PH] : nullptr;  // loop-phase counts (mcpt_debug_trace_profile)
    ta.hit_tri = c->p.hit_tri;
    ta.vis = c->p.vis;
    ta.grab = &c->cnt->grab[0][0];  // reset by k_accumulate below
    ta.idle = &c->cnt->idle;
    ta.tiny_stack = c->tiny_stack ? 1 : 0;
    launch_trace(ta, c->geom, c->stream);
    if (timing) HIPCHK(c, hipEventRecord(ev(c, evbase + 2), c->stream));
    launch_accumulate(c->cnt, c->geom.trace_parts, c->scene.occ ? c->scene.occ_gate : nullptr, c->stream);
    HIPCHK(c, hipGetLastError());
    return MCPT_OK;
}

// n iterations over a tile set (the context's, or one tile for mcpt_wavefront_step).  One
// host synchronisation per call: the counter totals before the call are the host copy the
// previous call (or the film clear) left.
static int run_iterations(mcpt_ctx* c, uint32_t n, mcpt_stage_stats* st, const int2* tiles = nullptr, int ntiles = -1,
                          const int* tile_base = nullptr) {
    int rc = check_ready(c);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    if (c->film_stale && !(c->cfg.flags & MCPT_FLAG_NO_AUTO_CLEAR) && (rc = mcpt_film_clear(c))) return rc;
    if (!tiles) {
        tiles = c->tiles;
        ntiles = (int)c->tiles_h.size();
    }
    if (!c->totals_ok) {
        HIPCHK(c, hipMemcpyAsync(c->cnt_host, c->cnt, sizeof(CounterBlock), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->totals = *c->cnt_host;
        c->totals_ok = true;
    }
    const CounterBlock before = c->totals;
    // iterations after one that traced no ray skip their kernels (k_accumulate sets the flag):
    // mcpt_render's last batch of 32 no longer pays full launches for the finished film
    HIPCHK(c, hipMemsetAsync(&c->cnt->idle, 0, sizeof(uint32_t), c->stream));
    for (uint32_t i = 0; i < n; i++) {
        // events for at most the first 4096 iterations of a call
        bool timing = i < 4096;
        if ((rc = enqueue_iteration(c, (size_t)3 * i, timing, tiles, ntiles, tile_base))) {
            c->totals_ok = false;
            return rc;
        }
    }
    c->totals_ok = false;
    HIPCHK(c, hipMemcpyAsync(c->cnt_host, c->cnt, sizeof(CounterBlock), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->totals = *c->cnt_host;
    c->totals_ok = true;
    const CounterBlock& after = c->totals;
    if (after.trace_short != before.trace_short)  // k_accumulate's drain check (never expected)
        return set_err(c, MCPT_E_HIP, "k_trace left queued rays untraced in " +
                                          std::to_string(after.trace_short - before.trace_short) + " launch(es)");
    if (st) {
        memset(st, 0, sizeof(*st));
        st->extend_rays = after.tot_ext - before.tot_ext;
        st->vis_rays = after.tot_vis - before.tot_vis;
        st->shadow_rays = (after.tot_any - before.tot_any) - st->vis_rays;
        st->iterations = n;
        st->live_paths = after.last_live;
        st->ext_nodes = after.tot_stats[0] - before.tot_stats[0];
        st->ext_tests = after.tot_stats[1] - before.tot_stats[1];
        st->ext_hits = after.tot_stats[2] - before.tot_stats[2];
        st->any_nodes = after.tot_stats[3] - before.tot_stats[3];
        st->any_tests = after.tot_stats[4] - before.tot_stats[4];
        st->any_hits = after.tot_stats[5] - before.tot_stats[5];
        uint32_t tn = std::min<uint32_t>(n, 4096);
        for (uint32_t i = 0; i < tn; i++) {
            float a = 0, b = 0;
            HIPCHK(c, hipEventElapsedTime(&a, c->events[3 * i + 0], c->events[3 * i + 1]));
            HIPCHK(c, hipEventElapsedTime(&b, c->events[3 * i + 1], c->events[3 * i + 2]));
            st->ms_shade += a;
            st->ms_extend += b;  // extension + any-hit rays: one k_trace launch (ms_shadow stays 0)
        }
        st->ms_total = st->ms_shade + st->ms_extend + st->ms_shadow;
    }
    return MCPT_OK;
}

int mcpt_iterate(mcpt_ctx* c, uint32_t n, mcpt_stage_stats* st) { return run_iterations(c, n, st); }

int mcpt_wavefront_step(mcpt_ctx* c, uint32_t tx, uint32_t ty, mcpt_stage_stats* st) {
    int rc = check_ready(c);
    if (rc) return rc;
    uint32_t nx = (c->W + c->tile_w - 1) / c->tile_w, ny = (c->H + c->tile_h - 1) / c->tile_h;
    if (tx >= nx || ty >= ny) return set_err(c, MCPT_E_INVALID, "tile out of range");
    // compact layout: the tile's paths are those of its place in the tile set
    int base = 0;
    if (c->compact) {
        base = -1;
        for (size_t i = 0; i < c->tiles_h.size() && base < 0; i++)
            if (c->tiles_h[i].x == (int)tx && c->tiles_h[i].y == (int)ty) base = (int)i;
        if (base < 0) return set_err(c, MCPT_E_INVALID, "compact paths: the tile is not in the tile set");
    }
    // The one-tile set goes through its own small buffer (pinned staging, stream-ordered
    // copy): the context's tile set and queues stay as they are when their per-shard queue
    // capacity covers one tile, which it does unless the tile set is empty.
    const uint32_t bpt = (uint32_t)shade_blocks_per_tile((int)(c->tile_w * c->tile_h), (int)c->slots);
    const uint32_t need = std::max<uint32_t>(1, (bpt + kShards - 1) / kShards) * kBlock;
    if (c->ext_cap >= need) {
        if (!c->step_tile) {
            HIPCHK(c, hipSetDevice(c->device));
            HIPCHK(c, hipMalloc(&c->step_tile, 2 * sizeof(int2)));
            HIPCHK(c, hipHostMalloc(&c->step_tile_h, 2 * sizeof(int2)));
        }
        c->step_tile_h[0] = make_int2((int)tx, (int)ty);  // the previous call's copy has completed
        c->step_tile_h[1] = make_int2(base, 0);
        HIPCHK(c, hipMemcpyAsync(c->step_tile, c->step_tile_h, 2 * sizeof(int2), hipMemcpyHostToDevice, c->stream));
        return run_iterations(c, 1, st, c->step_tile, 1, reinterpret_cast<const int*>(c->step_tile + 1));
    }
    std::vector<int2> saved = c->tiles_h;
    if ((rc = set_tiles_internal(c, {make_int2((int)tx, (int)ty)}))) return rc;
    rc = run_iterations(c, 1, st);
    int rc2 = set_tiles_internal(c, saved);
    return rc ? rc : rc2;
}

int mcpt_render(mcpt_ctx* c, mcpt_stage_stats* st) {
    int rc = check_ready(c);
    if (rc) return rc;
    mcpt_stage_stats acc{}, one{};
    const uint64_t cap = (uint64_t)(c->cfg.spp + 1) * (uint64_t)(c->cfg.max_depth + 2) + 16;
    uint64_t done = 0;
    // Iterations per batch (one host synchronisation each).  Once the film is done, the rest of a
    // batch are no-op launches (~24 us per iteration, mostly dispatching k_shade's grid), so the
    // first batch is sized to the expected frame -- samples per path slot x (max depth + 1)
    // iterations, the lockstep schedule of paths that all start together -- and later ones are
    // short.  (Config 2 at N = 8: 12 iterations of work ran in a batch of 32.)
    const uint64_t expect = (uint64_t)((c->cfg.spp + c->slots - 1) / c->slots) * (uint64_t)(c->cfg.max_depth + 1);
    for (;;) {
        const uint32_t batch = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(8, expect > done ? expect - done : 0));
        if ((rc = run_iterations(c, batch, &one))) return rc;
        acc.extend_rays += one.extend_rays;
        acc.shadow_rays += one.shadow_rays;
        acc.vis_rays += one.vis_rays;
        acc.iterations += one.iterations;
        acc.ms_shade += one.ms_shade;
        acc.ms_extend += one.ms_extend;
        acc.ms_shadow += one.ms_shadow;
        acc.ms_total += one.ms_total;
        acc.live_paths = one.live_paths;
        acc.ext_nodes += one.ext_nodes; acc.ext_tests += one.ext_tests; acc.ext_hits += one.ext_hits;
        acc.any_nodes += one.any_nodes; acc.any_tests += one.any_tests; acc.any_hits += one.any_hits;
        done += one.iterations;
        if (one.live_paths == 0 || done > cap) break;
    }
    if (st) *st = acc;
    if (acc.live_paths != 0) return set_err(c, MCPT_E_INVALID, "render did not converge within the iteration cap");
    return MCPT_OK;
}

int mcpt_sync(mcpt_ctx* c) {
    if (!c) return MCPT_E_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MCPT_OK;
}

// mcpt_stage_run(LOGIC | GENERATE | MATERIAL): the product's shading kernels (k_shade: wf_logic
// + wf_generate; k_material: light choice + wf_mat_mix) over caller path state of n paths in
// scratch device buffers -- the per-stage parity harness of SURVEY.md 8(b) / section 4 item 2.
// The context's film, queues and counters are not touched.
static int stage_run_paths(mcpt_ctx* c, int stage, const mcpt_path_view* in, mcpt_path_view* out, uint32_t n) {
    const bool mat = stage == MCPT_STAGE_MATERIAL, gen = stage == MCPT_STAGE_GENERATE;
    if (!in || !out) return set_err(c, MCPT_E_INVALID, "stage needs in->paths and out->paths");
    uint32_t W = n, H = 1;
    if (!mat) {
        W = in->film_w;
        H = in->film_h;
        if (!c->has_cam) return set_err(c, MCPT_E_INVALID, "no camera set");
        if ((uint64_t)W * H != n || W < 2 || H < 2) return set_err(c, MCPT_E_INVALID, "film_w * film_h must equal n (>= 2 x 2)");
    }
    if (n >= (1u << 26)) return set_err(c, MCPT_E_INVALID, "too many paths for one stage call");
    if (mat && in->hit_tri)  // k_material rebuilds the hit record from the triangle: it must exist
        for (uint32_t i = 0; i < n; i++)
            if (in->hit_tri[i] < 0 || in->hit_tri[i] >= c->ntri)
                return set_err(c, MCPT_E_INVALID, "MATERIAL: every path needs a hit (0 <= hit_tri < ntri)");
    if (!in->hit_tri || !in->flags || (!gen && (!in->ray_d || !in->beta)) || (!mat && !in->samples) ||
        (mat && !in->ray_o) || (stage == MCPT_STAGE_LOGIC && (!in->nee0 || !in->nee1 || !in->vis || !in->Ld)))
        return set_err(c, MCPT_E_INVALID, "missing path-state input");
    HIPCHK(c, hipSetDevice(c->device));
    free_list(c->tmp_bufs);
    auto& L = c->tmp_bufs;
    // shard capacity: LOGIC blocks of 256 paths push into shard block mod 64; MATERIAL records are
    // dealt to shards i mod 64
    const uint32_t nblocks = (uint32_t)shade_blocks_per_tile((int)n, 1);
    const uint32_t per_shard = mat ? (n + kShards - 1) / kShards : ((nblocks + kShards - 1) / kShards) * kBlock;
    const uint32_t ext_cap = std::max<uint32_t>(kBlock, (per_shard + kBlock - 1) / kBlock * kBlock), any_cap = 2 * ext_cap;
    const size_t qn = (size_t)kShards * ext_cap;
    DevPaths p{};
    uint32_t *ext_q, *any_q;
    uint4* mrec;
    float4* mbeta;
    CounterBlock* cnt;
    int2* tl;
    int rc;
    if ((rc = dalloc(c, L, &p.ray_o, n)) || (rc = dalloc(c, L, &p.ray_d, n)) || (rc = dalloc(c, L, &p.beta, n)) ||
        (rc = dalloc(c, L, &p.nee0, n)) || (rc = dalloc(c, L, &p.nee1, n)) || (rc = dalloc(c, L, &p.Ld, n)) ||
        (rc = dalloc(c, L, &p.hit_tri, n)) || (rc = dalloc(c, L, &p.flags, n)) || (rc = dalloc(c, L, &p.samples, n)) ||
        (rc = dalloc(c, L, &p.vis, 2 * (size_t)n)) ||
        (rc = dalloc(c, L, &p.sray_o, 2 * qn)) || (rc = dalloc(c, L, &p.sray_d, 2 * qn)) ||
        (rc = dalloc(c, L, &ext_q, qn)) || (rc = dalloc(c, L, &any_q, 2 * qn)) || (rc = dalloc(c, L, &mrec, qn)) ||
        (rc = dalloc(c, L, &mbeta, qn)) || (rc = dalloc(c, L, &cnt, 1)) || (rc = dalloc(c, L, &tl, 1)))
        return rc;
    auto f4v = [n](const float* a, int k, float w) {  // host k-float SoA -> float4 (w pad)
        std::vector<float4> v(n, make_float4(0.f, 0.f, 0.f, w));
        if (a)
            for (uint32_t i = 0; i < n; i++)
                v[i] = make_float4(a[k * i], a[k * i + 1], a[k * i + 2], k == 4 ? a[4 * i + 3] : w);
        return v;
    };
    auto up = [&](void* d, const void* h, size_t bytes) -> hipError_t {
        return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream);
    };
    std::vector<float4> ro = f4v(in->ray_o, 3, 0.f), rd = f4v(in->ray_d, 3, 0.f), be = f4v(in->beta, 4, 0.f),
                        n0 = f4v(in->nee0, 4, 0.f), n1 = f4v(in->nee1, 4, 0.f), ld = f4v(in->Ld, 3, 0.f);
    std::vector<uint32_t> fl(in->flags, in->flags + n), sm(n, 0u);
    if (in->samples) sm.assign(in->samples, in->samples + n);
    if (gen) std::fill(fl.begin(), fl.end(), (uint32_t)F_DEAD);
    if (!mat) {
        // The device's flags word carries a dead path's next sample index too, and k_shade derives
        // the film's sample count from it (one path slot here: sample index = count).  In: a dead
        // path's index is its samples; a live path's must equal them (the oracle's and the
        // reference's states always agree: samples changes only when a path ends).  Out: dead
        // paths' flags as the interface has them (F_DEAD alone).
        for (uint32_t i = 0; i < n; i++) {
            if (fl[i] & F_DEAD) fl[i] = (uint32_t)F_DEAD | (sm[i] << F_SIDX_SHIFT);
            else if ((fl[i] >> F_SIDX_SHIFT) != sm[i])
                return set_err(c, MCPT_E_INVALID, "LOGIC: a live path's sample index (flags) must equal its samples");
            if (sm[i] >= kMaxSpp) return set_err(c, MCPT_E_INVALID, "samples must be < 2^19");
        }
    }
    std::vector<uint8_t> vis(2 * (size_t)n, 0);
    if (in->vis) vis.assign(in->vis, in->vis + 2 * (size_t)n);
    CounterBlock* hc = c->cnt_host;  // pinned staging (the context's counters stay on the device)
    memset(hc, 0, sizeof(CounterBlock));
    std::vector<uint4> rec;
    std::vector<float4> rbeta;
    if (mat) {  // records {pid, len, sample index, hit_tri} + throughput, path i in shard i mod 64
        rec.assign(qn, make_uint4(0, 0, 0, 0));
        rbeta.assign(qn, make_float4(0.f, 0.f, 0.f, 0.f));
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t sh = i % kShards, k = i / kShards;
            rec[(size_t)sh * ext_cap + k] = make_uint4(i, i, (fl[i] >> F_SIDX_SHIFT) | (((fl[i] >> F_LEN_SHIFT) & 0xffu) << kRecLenShift),
                                                       (uint32_t)in->hit_tri[i]);
            rbeta[(size_t)sh * ext_cap + k] = make_float4(be[i].x, be[i].y, be[i].z, 0.f);
            hc->shard[sh][C_MAT]++;
        }
    }
    const int2 tile0 = make_int2(0, 0);
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = up(p.ray_o, ro.data(), n * sizeof(float4));
    if (e == hipSuccess) e = up(p.ray_d, rd.data(), n * sizeof(float4));
    if (e == hipSuccess) e = up(p.beta, be.data(), n * sizeof(float4));
    if (e == hipSuccess) e = up(p.nee0, n0.data(), n * sizeof(float4));
    if (e == hipSuccess) e = up(p.nee1, n1.data(), n * sizeof(float4));
    if (e == hipSuccess) e = up(p.Ld, ld.data(), n * sizeof(float4));
    if (e == hipSuccess) e = up(p.hit_tri, in->hit_tri, n * sizeof(int32_t));
    if (e == hipSuccess) e = up(p.flags, fl.data(), n * sizeof(uint32_t));
    if (e == hipSuccess) e = up(p.samples, sm.data(), n * sizeof(uint32_t));
    if (e == hipSuccess) e = up(p.vis, vis.data(), 2 * (size_t)n);
    if (e == hipSuccess) e = up(cnt, hc, sizeof(CounterBlock));
    if (e == hipSuccess) e = up(tl, &tile0, sizeof(int2));
    if (e == hipSuccess && mat) e = up(mrec, rec.data(), qn * sizeof(uint4));
    if (e == hipSuccess && mat) e = up(mbeta, rbeta.data(), qn * sizeof(float4));
    if (e != hipSuccess) return set_err(c, MCPT_E_HIP, std::string("stage upload: ") + hipGetErrorString(e));
    ShadeArgs sa{};
    sa.scene = c->scene;
    sa.scene.occ = nullptr;  // stage runs: outputs of the stage alone (no occluder cache)
    sa.cam = c->cam;
    sa.p = p;
    sa.tiles = tl;
    sa.ntiles = 1;
    sa.tile_w = (int)W;
    sa.tile_h = (int)H;
    sa.W = (int)W;
    sa.H = (int)H;
    sa.spp = c->cfg.spp;
    sa.max_depth = c->cfg.max_depth;
    sa.rr_depth = c->cfg.rr_depth;
    sa.seed = c->cfg.seed;
    sa.slots = 1;
    sa.slots_rcp = 1.0f;
    sa.npx = n;  // path i is pixel i of the W x H stage film
    if ((rc = cam_table(c, W, H, &sa.cam_px, &sa.cam_dir))) return rc;
    sa.ext_q = ext_q;
    sa.any_q = any_q;
    sa.mat_rec = mrec;
    sa.mat_beta = mbeta;
    sa.ext_cap = ext_cap;
    sa.any_cap = any_cap;
    sa.cnt = cnt;
    HIPCHK(c, hipEventRecord(ev(c, 0), c->stream));
    launch_shade_stage(mat, sa, (int)nblocks, c->geom, (c->cfg.flags & MCPT_FLAG_FIXED) != 0, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(ev(c, 1), c->stream));
    HIPCHK(c, hipMemcpyAsync(hc, cnt, sizeof(CounterBlock), hipMemcpyDeviceToHost, c->stream));
    std::vector<float4> o_ro(n), o_rd(n), o_be(n), o_n0(n), o_n1(n), o_ld(n);
    std::vector<uint32_t> o_fl(n), o_sm(n), o_eq(qn);
    std::vector<int32_t> o_ht(n);
    std::vector<uint8_t> o_vis(2 * (size_t)n);
    std::vector<uint4> o_rec(qn);
    std::vector<float4> o_rb(qn), o_so(2 * qn), o_sd(2 * qn);
    auto dn = [&](void* h, const void* d, size_t bytes) -> hipError_t {
        return hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, c->stream);
    };
    if (e == hipSuccess) e = dn(o_ro.data(), p.ray_o, n * sizeof(float4));
    if (e == hipSuccess) e = dn(o_rd.data(), p.ray_d, n * sizeof(float4));
    if (e == hipSuccess) e = dn(o_be.data(), p.beta, n * sizeof(float4));
    if (e == hipSuccess) e = dn(o_n0.data(), p.nee0, n * sizeof(float4));
    if (e == hipSuccess) e = dn(o_n1.data(), p.nee1, n * sizeof(float4));
    if (e == hipSuccess) e = dn(o_ld.data(), p.Ld, n * sizeof(float4));
    if (e == hipSuccess) e = dn(o_fl.data(), p.flags, n * sizeof(uint32_t));
    if (e == hipSuccess) e = dn(o_sm.data(), p.samples, n * sizeof(uint32_t));
    if (e == hipSuccess) e = dn(o_ht.data(), p.hit_tri, n * sizeof(int32_t));
    if (e == hipSuccess) e = dn(o_vis.data(), p.vis, 2 * (size_t)n);
    if (e == hipSuccess) e = dn(o_eq.data(), ext_q, qn * sizeof(uint32_t));
    if (e == hipSuccess) e = dn(o_rec.data(), mrec, qn * sizeof(uint4));
    if (e == hipSuccess) e = dn(o_rb.data(), mbeta, qn * sizeof(float4));
    if (e == hipSuccess) e = dn(o_so.data(), p.sray_o, 2 * qn * sizeof(float4));
    if (e == hipSuccess) e = dn(o_sd.data(), p.sray_d, 2 * qn * sizeof(float4));
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return set_err(c, MCPT_E_HIP, std::string("stage run: ") + hipGetErrorString(e));
    HIPCHK(c, hipEventElapsedTime(&c->last_stage_ms, c->events[0], c->events[1]));
    const float qnan = __builtin_nanf("");
    std::vector<uint8_t> queued(n, 0);
    std::vector<float> lo(3 * (size_t)n, qnan), ldr(3 * (size_t)n, qnan), bo(3 * (size_t)n, qnan), bd(3 * (size_t)n, qnan);
    for (int sh = 0; sh < kShards; sh++) {
        for (uint32_t k = 0; k < hc->shard[sh][C_EXT]; k++) queued[o_eq[(size_t)sh * ext_cap + k]] |= 1;
        if (!mat)
            for (uint32_t k = 0; k < hc->shard[sh][C_MAT]; k++) {  // continuing paths: their updated throughput
                const size_t q = (size_t)sh * ext_cap + k;
                const uint32_t pid = o_rec[q].x;
                queued[pid] |= 2;
                o_be[pid] = make_float4(o_rb[q].x, o_rb[q].y, o_rb[q].z, o_be[pid].w);
            }
        for (uint32_t k = 0; k < hc->shard[sh][C_ANY]; k++) {
            const size_t q = (size_t)sh * any_cap + k;
            uint32_t r;  // the ray's result index (2 pid + BRDF ray) rides in its origin's .w
            memcpy(&r, &o_so[q].w, sizeof(r));
            const uint32_t pid = r >> 1;
            float* so = (r & 1) ? bo.data() : lo.data();
            float* sd = (r & 1) ? bd.data() : ldr.data();
            queued[pid] |= (r & 1) ? 8 : 4;
            so[3 * pid] = o_so[q].x; so[3 * pid + 1] = o_so[q].y; so[3 * pid + 2] = o_so[q].z;
            sd[3 * pid] = o_sd[q].x; sd[3 * pid + 1] = o_sd[q].y; sd[3 * pid + 2] = o_sd[q].z;
        }
    }
    auto put3 = [n](float* dst, const std::vector<float4>& v) {
        if (dst)
            for (uint32_t i = 0; i < n; i++) { dst[3 * i] = v[i].x; dst[3 * i + 1] = v[i].y; dst[3 * i + 2] = v[i].z; }
    };
    auto put4 = [n](float* dst, const std::vector<float4>& v) {
        if (dst) memcpy(dst, v.data(), n * sizeof(float4));
    };
    if (!mat)
        for (uint32_t& f : o_fl)
            if (f & F_DEAD) f = F_DEAD;  // the interface's dead flags (the index lives in samples)
    if (out->flags) memcpy(out->flags, o_fl.data(), n * sizeof(uint32_t));
    if (out->samples) memcpy(out->samples, o_sm.data(), n * sizeof(uint32_t));
    if (out->hit_tri) memcpy(out->hit_tri, o_ht.data(), n * sizeof(int32_t));
    put3(out->ray_o, o_ro);
    put3(out->ray_d, o_rd);
    put4(out->beta, o_be);
    put4(out->nee0, o_n0);
    put4(out->nee1, o_n1);
    if (out->vis) memcpy(out->vis, o_vis.data(), 2 * (size_t)n);
    put3(out->Ld, o_ld);
    if (out->light_o) memcpy(out->light_o, lo.data(), 3 * (size_t)n * sizeof(float));
    if (out->light_d) memcpy(out->light_d, ldr.data(), 3 * (size_t)n * sizeof(float));
    if (out->bvis_o) memcpy(out->bvis_o, bo.data(), 3 * (size_t)n * sizeof(float));
    if (out->bvis_d) memcpy(out->bvis_d, bd.data(), 3 * (size_t)n * sizeof(float));
    if (out->queued) memcpy(out->queued, queued.data(), n);
    free_list(c->tmp_bufs);
    return MCPT_OK;
}

int mcpt_stage_run(mcpt_ctx* c, int stage, const mcpt_soa_view* in, mcpt_soa_view* out, uint32_t n) {
    if (!c || !in || !out) return set_err(c, MCPT_E_INVALID, "null argument");
    if (!c->has_scene) return set_err(c, MCPT_E_INVALID, "no scene uploaded");
    if (stage < MCPT_STAGE_LOGIC || stage > MCPT_STAGE_SHADOW) return set_err(c, MCPT_E_INVALID, "unknown stage");
    if (n == 0) return MCPT_OK;
    if (stage == MCPT_STAGE_LOGIC || stage == MCPT_STAGE_GENERATE || stage == MCPT_STAGE_MATERIAL)
        return stage_run_paths(c, stage, in->paths, out->paths, n);
    if (!in->ray_o || !in->ray_d) return set_err(c, MCPT_E_INVALID, "null rays");
    if (stage == MCPT_STAGE_EXTEND && (!out->hit_pos_t || !out->hit_nrm_mat)) return set_err(c, MCPT_E_INVALID, "null outputs");
    if (stage == MCPT_STAGE_SHADOW && !out->visible) return set_err(c, MCPT_E_INVALID, "null outputs");
    HIPCHK(c, hipSetDevice(c->device));
    free_list(c->tmp_bufs);
    std::vector<float4> ro(n), rd(n);
    for (uint32_t i = 0; i < n; i++) {
        ro[i] = make_float4(in->ray_o[3 * i], in->ray_o[3 * i + 1], in->ray_o[3 * i + 2], 0.f);
        rd[i] = make_float4(in->ray_d[3 * i], in->ray_d[3 * i + 1], in->ray_d[3 * i + 2], 0.f);
    }
    float4 *dro, *drd, *hp = nullptr, *hn = nullptr;
    int32_t* ht = nullptr;
    uint8_t* vis = nullptr;
    int rc;
    if ((rc = dupload(c, c->tmp_bufs, &dro, ro.data(), n)) || (rc = dupload(c, c->tmp_bufs, &drd, rd.data(), n)))
        return rc;
    TraceArgs ta{};
    ta.scene = c->scene;
    ta.scene.occ = nullptr;  // stage runs: outputs of the stage alone (no occluder cache)
    ta.nshards = 1;
    TraceSet& ts = ta.set[stage == MCPT_STAGE_SHADOW ? 1 : 0];
    ts.ro = dro;
    ts.rd = drd;
    ts.count = n;
    ts.shard_cap = n;
    if (stage == MCPT_STAGE_EXTEND) {
        if ((rc = dalloc(c, c->tmp_bufs, &hp, n)) || (rc = dalloc(c, c->tmp_bufs, &hn, n)) || (rc = dalloc(c, c->tmp_bufs, &ht, n)))
            return rc;
        ta.hit_tri = ht;
    } else {
        if ((rc = dalloc(c, c->tmp_bufs, &vis, n))) return rc;
        ta.vis = vis;
    }
    uint32_t* steps = nullptr;
    if (out->steps) {
        if ((rc = dalloc(c, c->tmp_bufs, &steps, n))) return rc;
        ts.ray_steps = steps;
    }
    ta.grab = &c->cnt->grab[0][0];
    HIPCHK(c, hipEventRecord(ev(c, 0), c->stream));
    ta.tiny_stack = c->tiny_stack ? 1 : 0;
    launch_trace(ta, c->geom, c->stream);
    HIPCHK(c, hipEventRecord(ev(c, 1), c->stream));
    uint32_t grab0 = 0;  // drain check: the one shard is partition 0's
    HIPCHK(c, hipMemcpyAsync(&c->cnt_host->grab[0][0], &c->cnt->grab[0][0], sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemsetAsync(c->cnt->grab, 0, sizeof(c->cnt->grab), c->stream));  // hand-out counters back to 0
    if (stage == MCPT_STAGE_EXTEND) {
        HitRecordArgs ha{c->scene, dro, drd, ht, hp, hn, ht, n};  // ht: positions in, scene indices out
        launch_hit_record(ha, c->stream);
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipEventElapsedTime(&c->last_stage_ms, c->events[0], c->events[1]));
    grab0 = c->cnt_host->grab[0][0];
    if (grab0 < n) return set_err(c, MCPT_E_HIP, "k_trace left rays untraced");
    if (steps) HIPCHK(c, hipMemcpy(out->steps, steps, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (stage == MCPT_STAGE_EXTEND) {
        std::vector<float4> a(n), b(n);
        HIPCHK(c, hipMemcpy(a.data(), hp, n * sizeof(float4), hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(b.data(), hn, n * sizeof(float4), hipMemcpyDeviceToHost));
        std::vector<int32_t> t(n);
        HIPCHK(c, hipMemcpy(t.data(), ht, n * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; i++) {
            out->hit_pos_t[4 * i + 0] = a[i].x; out->hit_pos_t[4 * i + 1] = a[i].y;
            out->hit_pos_t[4 * i + 2] = a[i].z; out->hit_pos_t[4 * i + 3] = a[i].w;
            int m;
            memcpy(&m, &b[i].w, 4);
            out->hit_nrm_mat[4 * i + 0] = b[i].x; out->hit_nrm_mat[4 * i + 1] = b[i].y;
            out->hit_nrm_mat[4 * i + 2] = b[i].z; out->hit_nrm_mat[4 * i + 3] = (float)m;
            if (out->hit_tri) out->hit_tri[i] = t[i];
        }
    } else {
        HIPCHK(c, hipMemcpy(out->visible, vis, n, hipMemcpyDeviceToHost));
    }
    free_list(c->tmp_bufs);
    return MCPT_OK;
}

// The film (dFilm.Ld / samples): the path state's accumulators with one slot per pixel,
// else their per-pixel sum in slot order (k_resolve) -- enqueued on the context stream.
static int film_view(mcpt_ctx* c, const float4** Ld, const uint32_t** samples) {
    if (c->slots <= 1 && !c->compact) {
        *Ld = c->p.Ld;
        *samples = c->p.samples;
        return MCPT_OK;
    }
    ResolveArgs a{c->p.Ld, c->p.samples, c->film_Ld, c->film_samples, (uint32_t)c->npx, (int)c->slots,
                  c->compact ? c->tiles : nullptr, (int)c->tile_w, (int)c->tile_h, (int)c->W, (int)c->H};
    launch_resolve(a, c->stream);
    HIPCHK(c, hipGetLastError());
    *Ld = c->film_Ld;
    *samples = c->film_samples;
    return MCPT_OK;
}

// Where another context's tile pixels are scattered (mcpt_film_unpack_tiles, mcpt_gather): the
// pixel-indexed accumulators the film view reads beside the context's own tiles
static void unpack_target(mcpt_ctx* c, float4** Ld, uint32_t** samples) {
    *Ld = c->compact ? c->film_Ld : c->p.Ld;
    *samples = c->compact ? c->film_samples : c->p.samples;
}

int mcpt_set_path_slots(mcpt_ctx* c, uint32_t slots) {
    if (!c || slots < 1 || slots > 256) return set_err(c, MCPT_E_INVALID, "path slots must be 1..256");
    if (slots == c->slots) return MCPT_OK;
    if (!c->P) {
        c->slots = slots;
        return MCPT_OK;
    }
    // check the new size before touching anything: a rejected count leaves the film as it was
    if ((uint64_t)c->npx * slots >= (1ull << 31)) return set_err(c, MCPT_E_INVALID, "film too large for the path slots");
    const uint32_t old = c->slots;
    c->slots = slots;
    if (c->compact) {  // the path state of the current tile set (its queues too: their capacity follows the slots)
        HIPCHK(c, hipSetDevice(c->device));
        const std::vector<int2> t = c->tiles_h;
        const size_t P = c->P;
        c->P = 0;
        int rc = set_tiles_internal(c, t);
        if (!rc) rc = alloc_film_state(c);
        if (rc != MCPT_OK) {
            const std::string err = c->err;
            c->slots = old;
            if (set_tiles_internal(c, t) == MCPT_OK && alloc_film_state(c) == MCPT_OK) {
                c->P = P;
                (void)mcpt_film_clear(c);
            }
            return set_err(c, rc, err);
        }
        c->P = P;
        return mcpt_film_clear(c);
    }
    int rc = mcpt_film_resize(c, c->W, c->H, c->tile_w, c->tile_h);  // clears the film
    if (rc != MCPT_OK) {  // e.g. out of memory: back to the old slot count and its (cleared) film
        const std::string err = c->err;
        c->slots = old;
        (void)mcpt_film_resize(c, c->W, c->H, c->tile_w, c->tile_h);
        return set_err(c, rc, err);
    }
    return MCPT_OK;
}

int mcpt_set_work_counters(mcpt_ctx* c, int32_t on) {
    if (!c) return MCPT_E_INVALID;
    c->count_work = on != 0;
    return MCPT_OK;
}

int mcpt_set_trace_partitions(mcpt_ctx* c, uint32_t nparts) {
    if (!c || nparts > (uint32_t)kMaxParts)
        return set_err(c, MCPT_E_INVALID, "trace partitions must be 0 (device default) .. " + std::to_string(kMaxParts));
    c->geom.trace_parts = nparts ? nparts : c->trace_parts_default;
    return MCPT_OK;
}

int mcpt_film_read(mcpt_ctx* c, float* Ld, uint32_t* samples) {
    if (!c || !c->P) return set_err(c, MCPT_E_INVALID, "film not allocated");
    HIPCHK(c, hipSetDevice(c->device));
    const float4* fL;
    const uint32_t* fs;
    int rc = film_view(c, &fL, &fs);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (Ld) {
        std::vector<float4> tmp(c->P);
        HIPCHK(c, hipMemcpy(tmp.data(), fL, c->P * sizeof(float4), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < c->P; i++) { Ld[3 * i] = tmp[i].x; Ld[3 * i + 1] = tmp[i].y; Ld[3 * i + 2] = tmp[i].z; }
    }
    if (samples) HIPCHK(c, hipMemcpy(samples, fs, c->P * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return MCPT_OK;
}

int mcpt_film_read_device(mcpt_ctx* c, void* dLd, void* dsamples) {
    if (!c || !c->P) return set_err(c, MCPT_E_INVALID, "film not allocated");
    HIPCHK(c, hipSetDevice(c->device));
    const float4* fL;
    const uint32_t* fs;
    int rc = film_view(c, &fL, &fs);
    if (rc) return rc;
    if (dLd) HIPCHK(c, hipMemcpyAsync(dLd, fL, c->P * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
    if (dsamples) HIPCHK(c, hipMemcpyAsync(dsamples, fs, c->P * sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MCPT_OK;
}

int mcpt_film_pack_tiles(mcpt_ctx* c, void* d_out, uint32_t* npix) {
    if (!c || !c->P) return set_err(c, MCPT_E_INVALID, "film not allocated");
    uint32_t n = (uint32_t)(c->tiles_h.size() * c->tile_w * c->tile_h);
    if (npix) *npix = n;
    if (!d_out) return MCPT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const float4* fL;
    const uint32_t* fs;
    int rc = film_view(c, &fL, &fs);
    if (rc) return rc;
    PackArgs a{fL, fs, c->tiles, (int)c->tiles_h.size(), (int)c->tile_w, (int)c->tile_h, (int)c->W, (int)c->H, (float4*)d_out};
    if (n) launch_pack(a, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MCPT_OK;
}

int mcpt_film_unpack_tiles(mcpt_ctx* c, const void* d_in, const uint32_t* xy, uint32_t n) {
    if (!c || !c->P) return set_err(c, MCPT_E_INVALID, "film not allocated");
    if (n == 0) return MCPT_OK;
    if (!d_in || !xy) return set_err(c, MCPT_E_INVALID, "null argument");
    const uint32_t nx = (c->W + c->tile_w - 1) / c->tile_w, ny = (c->H + c->tile_h - 1) / c->tile_h;
    std::vector<int2> t(n);
    for (uint32_t i = 0; i < n; i++) {
        if (xy[2 * i] >= nx || xy[2 * i + 1] >= ny) return set_err(c, MCPT_E_INVALID, "tile out of range");
        t[i] = make_int2((int)xy[2 * i], (int)xy[2 * i + 1]);
        if (has_tile(c->tiles_h, t[i]))  // the context's own pixels would mix with its other slots
            return set_err(c, MCPT_E_INVALID, "unpack into one of the context's own tiles");
    }
    HIPCHK(c, hipSetDevice(c->device));
    int2* dt = nullptr;
    HIPCHK(c, hipMalloc(&dt, n * sizeof(int2)));
    hipError_t e = hipMemcpyAsync(dt, t.data(), n * sizeof(int2), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        // scattered into slot 0 of the path state (its other slots of a pixel the context never
        // renders stay zero, so the film view's slot sum returns these values); compact layout: into
        // the W x H film, where the film view's resolve writes only the context's own tiles
        float4* tL;
        uint32_t* ts;
        unpack_target(c, &tL, &ts);
        UnpackArgs ua{(const float4*)d_in, dt, (int)n, (int)c->tile_w, (int)c->tile_h, (int)c->W, (int)c->H, tL, ts};
        launch_unpack(ua, c->stream);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(dt);
    if (e != hipSuccess) return set_err(c, MCPT_E_HIP, std::string("unpack: ") + hipGetErrorString(e));
    for (const int2& x : t)
        if (!has_tile(c->unpacked, x)) c->unpacked.push_back(x);
    return MCPT_OK;
}

// Frame-end gather of a multi-GPU render inside one process (SURVEY.md 8(b) mcpt_gather, 8(e)):
// every context's tile-set pixels, resolved over its path slots and packed 16 B/px, are copied
// device-to-device onto the root's device (hipMemcpyPeerAsync: SDMA over xGMI between MI355X
// dies of a node) and scattered into the root's film accumulators, so the root's film readers
// return the whole frame.  Tile sets must not overlap the root's own tiles (the interleaved
// partition of mcpt/parallel.py); the multi-process form sends the same packed buffers to the
// root over RCCL and scatters them with mcpt_film_unpack_tiles (mcpt/parallel.py).
int mcpt_gather(mcpt_ctx* const* ctxs, int32_t n, int32_t root) {
    if (!ctxs || n < 1 || root < 0 || root >= n || !ctxs[root]) return set_err(nullptr, MCPT_E_INVALID, "bad gather arguments");
    mcpt_ctx* R = ctxs[root];
    for (int32_t i = 0; i < n; i++) {
        mcpt_ctx* c = ctxs[i];
        if (!c || !c->P) return set_err(R, MCPT_E_INVALID, "gather: a context has no film");
        if (c->W != R->W || c->H != R->H || c->tile_w != R->tile_w || c->tile_h != R->tile_h)
            return set_err(R, MCPT_E_INVALID, "gather: film or tile sizes differ between contexts");
        for (int32_t j = 0; j < i; j++)
            if (ctxs[j] == c) return set_err(R, MCPT_E_INVALID, "gather: a context is listed twice");
        if (c != R)
            for (const int2& x : c->tiles_h)
                if (has_tile(R->tiles_h, x)) return set_err(R, MCPT_E_INVALID, "gather: a tile set overlaps the root's own tiles");
    }
    for (int32_t i = 0; i < n; i++) {
        mcpt_ctx* c = ctxs[i];
        if (c == R || c->tiles_h.empty()) continue;
        const size_t npix = c->tiles_h.size() * (size_t)c->tile_w * c->tile_h;
        // pack on the source device (its film view resolves the path slots)
        HIPCHK(R, hipSetDevice(c->device));
        const float4* fL;
        const uint32_t* fs;
        int rc = film_view(c, &fL, &fs);
        if (rc) return set_err(R, rc, c->err);
        float4* src = nullptr;
        if (hipMalloc(&src, npix * sizeof(float4)) != hipSuccess) return set_err(R, MCPT_E_NOMEM, "gather: pack buffer");
        PackArgs pa{fL, fs, c->tiles, (int)c->tiles_h.size(), (int)c->tile_w, (int)c->tile_h, (int)c->W, (int)c->H, src};
        launch_pack(pa, c->stream);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        // copy to the root's device and scatter into its accumulators (slot 0; the other slots
        // of pixels the root does not render are zero, so its slot sum returns these values)
        float4* dst = nullptr;
        int2* dt = nullptr;
        if (e == hipSuccess) e = hipSetDevice(R->device);
        if (e == hipSuccess && c->device != R->device) {
            // direct xGMI access where the pair supports it; hipMemcpyPeerAsync also works
            // without it (staged), so a refusal here is not an error
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, R->device, c->device) == hipSuccess && can)
                (void)hipDeviceEnablePeerAccess(c->device, 0);
            (void)hipGetLastError();
        }
        if (e == hipSuccess) e = hipMalloc(&dst, npix * sizeof(float4));
        if (e == hipSuccess) e = hipMalloc(&dt, c->tiles_h.size() * sizeof(int2));
        if (e == hipSuccess)
            e = hipMemcpyPeerAsync(dst, R->device, src, c->device, npix * sizeof(float4), R->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(dt, c->tiles_h.data(), c->tiles_h.size() * sizeof(int2), hipMemcpyHostToDevice, R->stream);
        if (e == hipSuccess) {
            float4* tL;
            uint32_t* ts;
            unpack_target(R, &tL, &ts);
            UnpackArgs ua{dst, dt, (int)c->tiles_h.size(), (int)R->tile_w, (int)R->tile_h, (int)R->W, (int)R->H, tL, ts};
            launch_unpack(ua, R->stream);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipStreamSynchronize(R->stream);
        (void)hipFree(dst);
        (void)hipFree(dt);
        (void)hipSetDevice(c->device);
        (void)hipFree(src);
        if (e != hipSuccess) return set_err(R, MCPT_E_HIP, std::string("gather: ") + hipGetErrorString(e));
        for (const int2& x : c->tiles_h)
            if (!has_tile(R->unpacked, x)) R->unpacked.push_back(x);
    }
    (void)hipSetDevice(R->device);
    return MCPT_OK;
}

int mcpt_film_size(const mcpt_ctx* c, uint32_t* w, uint32_t* h) {
    if (!c || !w || !h) return MCPT_E_INVALID;
    if (!c->P) return set_err(const_cast<mcpt_ctx*>(c), MCPT_E_INVALID, "film not allocated");
    *w = c->W;
    *h = c->H;
    return MCPT_OK;
}

int mcpt_film_tonemap_rgba8(mcpt_ctx* c, float exposure, uint8_t* out) {
    if (!c || !c->P || !out) return set_err(c, MCPT_E_INVALID, "bad argument");
    HIPCHK(c, hipSetDevice(c->device));
    const float4* fL;
    const uint32_t* fs;
    int rc = film_view(c, &fL, &fs);
    if (rc) return rc;
    uchar4* d = nullptr;
    HIPCHK(c, hipMalloc(&d, c->P * sizeof(uchar4)));
    TonemapArgs a{fL, fs, d, exposure, (uint32_t)c->P};
    launch_tonemap(a, c->stream);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out, d, c->P * sizeof(uchar4), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return set_err(c, MCPT_E_HIP, std::string("tonemap: ") + hipGetErrorString(e));
    return MCPT_OK;
}

}  // extern "C"

extern "C" {
int mcpt_debug_queue_rays(mcpt_ctx* c, int which, float* ro, float* rd, uint32_t* n_inout) {
    if (!c || !c->P || !n_inout || (which != 0 && which != 1)) return set_err(c, MCPT_E_INVALID, "bad argument");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    CounterBlock cb;
    HIPCHK(c, hipMemcpy(&cb, c->cnt, sizeof(cb), hipMemcpyDeviceToHost));
    // k_accumulate reset the live counters; the queues still hold the last iteration's entries
    uint32_t n = which == 0 ? cb.last_ext : 0;
    if (which == 1) return set_err(c, MCPT_E_INVALID, "any-hit queue length is not retained");
    if (!ro || !rd) { *n_inout = n; return MCPT_OK; }
    n = std::min(n, *n_inout);
    std::vector<uint32_t> all((size_t)kShards * c->ext_cap), q;
    HIPCHK(c, hipMemcpy(all.data(), c->ext_q, all.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (int sh = 0; sh < kShards; sh++)
        for (uint32_t k = 0; k < cb.last_ext_shard[sh] && q.size() < n; k++) q.push_back(all[(size_t)sh * c->ext_cap + k]);
    n = (uint32_t)q.size();
    const size_t np = c->npx * c->slots;
    std::vector<float4> o(np), d(np);
    HIPCHK(c, hipMemcpy(o.data(), c->p.ray_o, np * sizeof(float4), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(d.data(), c->p.ray_d, np * sizeof(float4), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; i++) {
        float4 a = o[q[i]], b = d[q[i]];
        ro[3 * i] = a.x; ro[3 * i + 1] = a.y; ro[3 * i + 2] = a.z;
        rd[3 * i] = b.x; rd[3 * i + 1] = b.y; rd[3 * i + 2] = b.z;
    }
    *n_inout = n;
    return MCPT_OK;
}
float mcpt_debug_last_stage_ms(const mcpt_ctx* c) { return c ? c->last_stage_ms : -1.f; }
int mcpt_debug_tiny_lds_stack(mcpt_ctx* c, int32_t on) {
    if (!c) return MCPT_E_INVALID;
    c->tiny_stack = on != 0;
    return MCPT_OK;
}

int mcpt_debug_quot(mcpt_ctx* c, const float* a, const float* b, uint32_t n, float* out) {
    if (!c || (n && (!a || !b || !out))) return set_err(c, MCPT_E_INVALID, "null argument");
    HIPCHK(c, hipSetDevice(c->device));
    float* d = nullptr;
    if (n == 0) return MCPT_OK;
    if (hipMalloc(&d, (size_t)3 * n * sizeof(float)) != hipSuccess) return set_err(c, MCPT_E_NOMEM, "quot buffers");
    int rc = MCPT_OK;
    if (hipMemcpyAsync(d, a, n * sizeof(float), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(d + n, b, n * sizeof(float), hipMemcpyHostToDevice, c->stream) != hipSuccess)
        rc = set_err(c, MCPT_E_HIP, "copy");
    if (!rc) {
        launch_quot(d, d + n, d + 2 * (size_t)n, n, c->stream);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(out, d + 2 * (size_t)n, n * sizeof(float), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            rc = set_err(c, MCPT_E_HIP, "quot kernel");
    }
    (void)hipFree(d);
    return rc;
}

int mcpt_debug_hbm_copy(mcpt_ctx* c, uint64_t bytes, uint32_t iters, double* gbps) {
    if (!c || !gbps || bytes < 4096 || iters == 0) return set_err(c, MCPT_E_INVALID, "bad argument");
    HIPCHK(c, hipSetDevice(c->device));
    const size_t n = (size_t)(bytes / sizeof(float4));
    float4* d = nullptr;
    if (hipMalloc(&d, 2 * n * sizeof(float4)) != hipSuccess) return set_err(c, MCPT_E_NOMEM, "copy buffers");
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = MCPT_OK;
    if (hipMemsetAsync(d, 0, 2 * n * sizeof(float4), c->stream) != hipSuccess ||
        hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
        rc = set_err(c, MCPT_E_HIP, "copy setup");
    } else {
        launch_copy(d, d + n, n, c->stream);  // warm-up
        (void)hipEventRecord(e0, c->stream);
        for (uint32_t i = 0; i < iters; i++) launch_copy(i & 1 ? d + n : d, i & 1 ? d : d + n, n, c->stream);
        (void)hipEventRecord(e1, c->stream);
        float ms = 0.f;
        if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
            hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.f)
            rc = set_err(c, MCPT_E_HIP, "copy kernel");
        else
            *gbps = 2.0 * (double)n * sizeof(float4) * iters / (ms * 1e-3) / 1e9;  // read + write bytes
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d);
    return rc;
}

// k_trace's loop-phase counts (PH_*, counting build: mcpt_set_work_counters on) since the last film
// clear or reset, from the host copy of the counters the last call left: returns kPhaseWords
int mcpt_debug_trace_profile(mcpt_ctx* c, uint64_t* out12, int reset) {
    if (!c || !out12) return MCPT_E_INVALID;
    for (int i = 0; i < 12; i++) out12[i] = 0;
    if (!c->totals_ok) return 0;
    for (int i = 0; i < kPhaseWords; i++) out12[i] = c->totals.tot_phase[i] - c->phase_base[i];
    if (reset)
        for (int i = 0; i < kPhaseWords; i++) c->phase_base[i] = c->totals.tot_phase[i];
    return kPhaseWords;
}
// Diagnostics builds (-DMCPT_WAVE_TIMES) only, not part of mcpt.h: entry / exit s_memrealtime (100 MHz)
// stamps of the last k_trace launch's first n waves (out: 4n words: entry, exit, partition,
// time the partition ran dry); returns n or 0.
int mcpt_debug_wave_times(mcpt_ctx* c, uint64_t* out, int n) {
    if (!c || !out || n < 0) return MCPT_E_INVALID;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return wave_times(reinterpret_cast<unsigned long long*>(out), n);
}
// Diagnostics builds (-DMCPT_DIAG_SHADE) only, not part of mcpt.h: k_shade's per-section wave entries
// and active lanes (SD_* pairs, kernels.hip) summed since the last reset; returns the word count or 0.
int mcpt_debug_shade_sections(mcpt_ctx* c, uint64_t* out, int n, int reset) {
    if (!c || !out || n < 0) return MCPT_E_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return shade_sections(reinterpret_cast<unsigned long long*>(out), n, reset);
}
}
