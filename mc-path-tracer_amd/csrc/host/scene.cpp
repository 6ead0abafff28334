// scene.cpp -- host scene builder behind the mcpt_scene_* C ABI.
//
// Re-designs the reference's host-side scene assembly for the MI355X backend:
//   Scene::load (assimp)          CUDA-RayTracer/Scene.cu:24-66, 187-324 -> minimal glTF-2.0 .glb reader
//   stbi_loadf HDR                 CUDA-RayTracer/dTexture.cu:205-283     -> Radiance RGBE (new-RLE) reader
//   build_environment_light        CUDA-RayTracer/light_initialization_kernels.cu:3-161 -> host tables
//   BVHAccel (SAH, 12 buckets)     CUDA-RayTracer/BVH.cu:53-333           -> host SAH build + flatten
//   Scene::transfer_data_to_device CUDA-RayTracer/Scene.cu:363-470        -> flat SoA arrays (mcpt_scene_desc)
// Everything here is setup; the per-bounce hot path lives in kernels.hip.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../device/mcpt_core.hpp"
#include "host_internal.hpp"
#include "mcpt.h"

using mcpt::V3;

namespace mcpt_host {

// ---------------------------------------------------------------------------
// Minimal JSON (enough for glTF 2.0 headers).
// ---------------------------------------------------------------------------
struct Json {
    enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
    double num = 0;
    bool b = false;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;
    const Json* get(const char* k) const {
        if (kind != Obj) return nullptr;
        for (auto& kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    double numv(const char* k, double dflt) const {
        const Json* j = get(k);
        return (j && j->kind == Num) ? j->num : dflt;
    }
};
struct JsonParser {
    const char* p;
    const char* end;
    bool ok = true;
    void ws() { while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) p++; }
    Json parse() {
        ws();
        Json j;
        if (p >= end) { ok = false; return j; }
        char c = *p;
        if (c == '{') {
            j.kind = Json::Obj; p++; ws();
            if (p < end && *p == '}') { p++; return j; }
            while (ok && p < end) {
                ws();
                Json k = parse();
                if (k.kind != Json::Str) { ok = false; break; }
                ws();
                if (p >= end || *p != ':') { ok = false; break; }
                p++;
                Json v = parse();
                j.obj.emplace_back(k.str, std::move(v));
                ws();
                if (p < end && *p == ',') { p++; continue; }
                if (p < end && *p == '}') { p++; break; }
                ok = false;
            }
        } else if (c == '[') {
            j.kind = Json::Arr; p++; ws();
            if (p < end && *p == ']') { p++; return j; }
            while (ok && p < end) {
                j.arr.push_back(parse());
                ws();
                if (p < end && *p == ',') { p++; continue; }
                if (p < end && *p == ']') { p++; break; }
                ok = false;
            }
        } else if (c == '"') {
            j.kind = Json::Str; p++;
            while (p < end && *p != '"') {
                if (*p == '\\' && p + 1 < end) { p++; char e = *p; j.str.push_back(e == 'n' ? '\n' : e); p++; continue; }
                j.str.push_back(*p++);
            }
            if (p < end) p++;
        } else if (c == 't' || c == 'f') {
            j.kind = Json::Bool; j.b = (c == 't');
            p += (c == 't') ? 4 : 5;
        } else if (c == 'n') {
            p += 4;
        } else {
            j.kind = Json::Num;
            char* q = nullptr;
            j.num = strtod(p, &q);
            if (q == p) ok = false;
            p = q;
        }
        return j;
    }
};

// ---------------------------------------------------------------------------
// 4x4 column-major helpers (glm semantics: m[c][r] = m[c*4+r]).
// ---------------------------------------------------------------------------
struct M4 { float m[16]; };
static M4 m4_identity() { M4 r{}; r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1.f; return r; }
static M4 m4_mul(const M4& a, const M4& b) {  // glm operator*(mat4, mat4)
    M4 r{};
    for (int c = 0; c < 4; c++)
        for (int row = 0; row < 4; row++)
            r.m[c * 4 + row] = a.m[0 * 4 + row] * b.m[c * 4 + 0] + a.m[1 * 4 + row] * b.m[c * 4 + 1] +
                               a.m[2 * 4 + row] * b.m[c * 4 + 2] + a.m[3 * 4 + row] * b.m[c * 4 + 3];
    return r;
}
// glm::inverse (detail::compute_inverse<4,4>), same operation order.
static M4 m4_inverse(const M4& M) {
    auto m = [&](int c, int r) { return M.m[c * 4 + r]; };
    float C00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3), C02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
    float C03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3), C04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3);
    float C06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3), C07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
    float C08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2), C10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
    float C11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2), C12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3);
    float C14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3), C15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
    float C16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2), C18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
    float C19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2), C20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1);
    float C22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1), C23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
    float F0[4] = {C00, C00, C02, C03}, F1[4] = {C04, C04, C06, C07}, F2[4] = {C08, C08, C10, C11};
    float F3[4] = {C12, C12, C14, C15}, F4[4] = {C16, C16, C18, C19}, F5[4] = {C20, C20, C22, C23};
    float V0[4] = {m(1, 0), m(0, 0), m(0, 0), m(0, 0)}, V1[4] = {m(1, 1), m(0, 1), m(0, 1), m(0, 1)};
    float V2[4] = {m(1, 2), m(0, 2), m(0, 2), m(0, 2)}, V3_[4] = {m(1, 3), m(0, 3), m(0, 3), m(0, 3)};
    float I0[4], I1[4], I2[4], I3[4];
    for (int i = 0; i < 4; i++) {
        I0[i] = V1[i] * F0[i] - V2[i] * F1[i] + V3_[i] * F2[i];
        I1[i] = V0[i] * F0[i] - V2[i] * F3[i] + V3_[i] * F4[i];
        I2[i] = V0[i] * F1[i] - V1[i] * F3[i] + V3_[i] * F5[i];
        I3[i] = V0[i] * F2[i] - V1[i] * F4[i] + V2[i] * F5[i];
    }
    const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    M4 inv;
    for (int i = 0; i < 4; i++) {
        inv.m[0 * 4 + i] = I0[i] * SA[i];
        inv.m[1 * 4 + i] = I1[i] * SB[i];
        inv.m[2 * 4 + i] = I2[i] * SA[i];
        inv.m[3 * 4 + i] = I3[i] * SB[i];
    }
    float Row0[4] = {inv.m[0], inv.m[4], inv.m[8], inv.m[12]};
    float D0[4];
    for (int i = 0; i < 4; i++) D0[i] = M.m[0 * 4 + i] * Row0[i];
    float D1 = (D0[0] + D0[1]) + (D0[2] + D0[3]);
    float ood = 1.f / D1;
    for (int i = 0; i < 16; i++) inv.m[i] = inv.m[i] * ood;
    return inv;
}
static V3 m4_point(const M4& a, V3 p) {
    float v[4] = {p.x, p.y, p.z, 1.f}, o[4];
    mcpt::mat_vec4(a.m, v[0], v[1], v[2], v[3], o);
    return mcpt::v3(o[0], o[1], o[2]);
}
static M4 m4_transpose(const M4& a) {
    M4 r;
    for (int c = 0; c < 4; c++)
        for (int row = 0; row < 4; row++) r.m[c * 4 + row] = a.m[row * 4 + c];
    return r;
}
// glm::normalize: v * inversesqrt(dot(v, v))
static V3 glm_normalize(V3 v) {
    float d = v.x * v.x + v.y * v.y + v.z * v.z;
    float s = 1.f / std::sqrt(d);
    return mcpt::v3(v.x * s, v.y * s, v.z * s);
}
static V3 glm_cross(V3 a, V3 b) { return mcpt::cross(a, b); }
static float glm_dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

static M4 trs_matrix(const float* t, const float* q, const float* s) {  // glTF node TRS -> T*R*S
    float x = q[0], y = q[1], z = q[2], w = q[3];
    M4 R = m4_identity();
    R.m[0] = 1 - 2 * (y * y + z * z); R.m[1] = 2 * (x * y + z * w); R.m[2] = 2 * (x * z - y * w);
    R.m[4] = 2 * (x * y - z * w); R.m[5] = 1 - 2 * (x * x + z * z); R.m[6] = 2 * (y * z + x * w);
    R.m[8] = 2 * (x * z + y * w); R.m[9] = 2 * (y * z - x * w); R.m[10] = 1 - 2 * (x * x + y * y);
    M4 S = m4_identity();
    S.m[0] = s[0]; S.m[5] = s[1]; S.m[10] = s[2];
    M4 T = m4_identity();
    T.m[12] = t[0]; T.m[13] = t[1]; T.m[14] = t[2];
    return m4_mul(T, m4_mul(R, S));
}

// ---------------------------------------------------------------------------
// Scene
// ---------------------------------------------------------------------------
void Scene::add_mesh(const std::vector<V3>& pos, const std::vector<V3>& nrm, const std::vector<uint32_t>& idx,
                     V3 base) {
    int mat_id = (int)(materials.size() / 8);
    float mp[8] = {base.x, base.y, base.z, 0.04f, 0.04f, 0.04f, 1.f, 0.f};  // dMaterial.cuh:13-18, Scene.cu:306-307
    materials.insert(materials.end(), mp, mp + 8);
    for (size_t i = 0; i + 2 < idx.size(); i += 3) {
        Tri t;
        for (int k = 0; k < 3; k++) { t.p[k] = pos[idx[i + k]]; t.n[k] = nrm[idx[i + k]]; }
        t.mat = mat_id;
        tris.push_back(t);
    }
    built = false;
}

void Scene::transform(const float* xf16) {
    M4 M;
    memcpy(M.m, xf16, sizeof(M.m));
    M4 N = m4_transpose(m4_inverse(M));  // Scene.cu:212
    for (auto& t : tris)
        for (int k = 0; k < 3; k++) {
            t.p[k] = m4_point(M, t.p[k]);
            float o[4];
            mcpt::mat_vec4(N.m, t.n[k].x, t.n[k].y, t.n[k].z, 1.f, o);  // w = 1 quirk (Scene.cu:232)
            t.n[k] = glm_normalize(mcpt::v3(o[0], o[1], o[2]));
        }
    built = false;
}

static bool read_file(const char* path, std::vector<uint8_t>& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    f.seekg(0, std::ios::end);
    std::streamoff n = f.tellg();
    f.seekg(0);
    out.resize((size_t)n);
    if (n > 0) f.read((char*)out.data(), n);
    return (bool)f;
}

// glTF 2.0 binary reader: POSITION, NORMAL, indices, node TRS/matrix, base
// colour.  Mirrors Scene::load_model/load_mesh/load_material (Scene.cu:187-324):
// node transforms baked into positions, normals by transpose(inverse(M)),
// roughness forced to 1, metallic to 0; no material => base colour (1,1,1)
// (assimp's glTF2 default material; parity unpinned).
int Scene::load_glb(const char* path, const float* xf16, std::string& err) {
    std::vector<uint8_t> buf;
    if (!read_file(path, buf)) { err = std::string("cannot read ") + path; return MCPT_E_IO; }
    if (buf.size() < 20 || memcmp(buf.data(), "glTF", 4) != 0) { err = "not a glb file"; return MCPT_E_IO; }
    uint32_t jlen, jtype;
    memcpy(&jlen, &buf[12], 4);
    memcpy(&jtype, &buf[16], 4);
    if (jtype != 0x4E4F534Au || 20 + (size_t)jlen > buf.size()) { err = "bad glb json chunk"; return MCPT_E_IO; }
    JsonParser jp{(const char*)&buf[20], (const char*)&buf[20] + jlen};
    Json root = jp.parse();
    if (!jp.ok) { err = "bad glb json"; return MCPT_E_IO; }
    const uint8_t* bin = nullptr;
    size_t binlen = 0;
    size_t off = 20 + jlen;
    if (off + 8 <= buf.size()) {
        uint32_t blen, btype;
        memcpy(&blen, &buf[off], 4);
        memcpy(&btype, &buf[off + 4], 4);
        if (btype == 0x004E4942u && off + 8 + blen <= buf.size()) { bin = &buf[off + 8]; binlen = blen; }
    }
    const Json* accessors = root.get("accessors");
    const Json* views = root.get("bufferViews");
    const Json* meshes = root.get("meshes");
    const Json* nodes = root.get("nodes");
    const Json* mats = root.get("materials");
    if (!accessors || !views || !meshes || !nodes || !bin) { err = "glb missing arrays"; return MCPT_E_IO; }

    auto read_accessor = [&](int ai, std::vector<float>& fout, std::vector<uint32_t>& iout, int& ncomp) -> bool {
        if (ai < 0 || ai >= (int)accessors->arr.size()) return false;
        const Json& a = accessors->arr[ai];
        int vi = (int)a.numv("bufferView", -1);
        if (vi < 0 || vi >= (int)views->arr.size()) return false;
        const Json& v = views->arr[vi];
        size_t boff = (size_t)v.numv("byteOffset", 0) + (size_t)a.numv("byteOffset", 0);
        size_t stride = (size_t)v.numv("byteStride", 0);
        int ctype = (int)a.numv("componentType", 0);
        size_t count = (size_t)a.numv("count", 0);
        const Json* type = a.get("type");
        std::string ts = type ? type->str : "SCALAR";
        ncomp = ts == "SCALAR" ? 1 : ts == "VEC2" ? 2 : ts == "VEC3" ? 3 : ts == "VEC4" ? 4 : 0;
        if (!ncomp) return false;
        size_t csize = (ctype == 5126 || ctype == 5125) ? 4 : (ctype == 5123 || ctype == 5122) ? 2 : 1;
        if (!stride) stride = csize * ncomp;
        if (boff + (count ? (count - 1) * stride + csize * ncomp : 0) > binlen) return false;
        for (size_t i = 0; i < count; i++)
            for (int c = 0; c < ncomp; c++) {
                const uint8_t* src = bin + boff + i * stride + c * csize;
                if (ctype == 5126) { float f; memcpy(&f, src, 4); fout.push_back(f); }
                else if (ctype == 5125) { uint32_t u; memcpy(&u, src, 4); iout.push_back(u); }
                else if (ctype == 5123) { uint16_t u; memcpy(&u, src, 2); iout.push_back(u); }
                else if (ctype == 5121) { iout.push_back(*src); }
                else return false;
            }
        return true;
    };

    M4 base = m4_identity();
    if (xf16) memcpy(base.m, xf16, sizeof(base.m));
    int status = MCPT_OK;
    // Scene.cu:187-199: accTransform = node * acc, recursive over children.
    std::function<void(int, const M4&)> visit = [&](int ni, const M4& acc) {
        if (status != MCPT_OK || ni < 0 || ni >= (int)nodes->arr.size()) return;
        const Json& n = nodes->arr[ni];
        M4 local = m4_identity();
        if (const Json* mj = n.get("matrix")) {
            for (int i = 0; i < 16 && i < (int)mj->arr.size(); i++) local.m[i] = (float)mj->arr[i].num;
        } else {
            float t[3] = {0, 0, 0}, q[4] = {0, 0, 0, 1}, s[3] = {1, 1, 1};
            if (const Json* tj = n.get("translation")) for (int i = 0; i < 3; i++) t[i] = (float)tj->arr[i].num;
            if (const Json* qj = n.get("rotation")) for (int i = 0; i < 4; i++) q[i] = (float)qj->arr[i].num;
            if (const Json* sj = n.get("scale")) for (int i = 0; i < 3; i++) s[i] = (float)sj->arr[i].num;
            local = trs_matrix(t, q, s);
        }
        M4 M = m4_mul(acc, local);
        M4 N = m4_transpose(m4_inverse(M));
        if (const Json* mi = n.get("mesh")) {
            int meshi = (int)mi->num;
            if (meshi >= 0 && meshi < (int)meshes->arr.size()) {
                const Json* prims = meshes->arr[meshi].get("primitives");
                for (size_t pi = 0; prims && pi < prims->arr.size(); pi++) {
                    const Json& pr = prims->arr[pi];
                    if ((int)pr.numv("mode", 4) != 4) continue;
                    const Json* attrs = pr.get("attributes");
                    std::vector<float> P, Nn;
                    std::vector<uint32_t> dummy, idx;
                    int nc = 0;
                    if (!attrs || !read_accessor((int)attrs->numv("POSITION", -1), P, dummy, nc) || nc != 3) {
                        err = "glb: bad POSITION"; status = MCPT_E_IO; return;
                    }
                    size_t nv = P.size() / 3;
                    bool has_n = attrs->get("NORMAL") && read_accessor((int)attrs->numv("NORMAL", -1), Nn, dummy, nc) && nc == 3;
                    if (pr.get("indices")) {
                        std::vector<float> fdummy;
                        if (!read_accessor((int)pr.numv("indices", -1), fdummy, idx, nc)) {
                            err = "glb: bad indices"; status = MCPT_E_IO; return;
                        }
                    } else {
                        for (uint32_t i = 0; i < nv; i++) idx.push_back(i);
                    }
                    std::vector<V3> pos(nv), nrm(nv);
                    for (size_t i = 0; i < nv; i++) {
                        pos[i] = m4_point(M, mcpt::v3(P[3 * i], P[3 * i + 1], P[3 * i + 2]));
                        V3 nn = has_n ? mcpt::v3(Nn[3 * i], Nn[3 * i + 1], Nn[3 * i + 2]) : mcpt::v3(0, 1, 0);
                        float o[4];
                        mcpt::mat_vec4(N.m, nn.x, nn.y, nn.z, 1.f, o);
                        nrm[i] = glm_normalize(mcpt::v3(o[0], o[1], o[2]));
                    }
                    if (!has_n) {  // aiProcess_GenSmoothNormals: area-weighted vertex normals
                        std::vector<V3> acc(nv, mcpt::v3(0, 0, 0));
                        for (size_t i = 0; i + 2 < idx.size(); i += 3) {
                            V3 a = pos[idx[i]], b = pos[idx[i + 1]], c = pos[idx[i + 2]];
                            V3 fn = glm_cross(b - a, c - a);
                            for (int k = 0; k < 3; k++) acc[idx[i + k]] = acc[idx[i + k]] + fn;
                        }
                        for (size_t i = 0; i < nv; i++) nrm[i] = glm_normalize(acc[i]);
                    }
                    for (uint32_t ix : idx)
                        if (ix >= nv) { err = "glb: index out of range"; status = MCPT_E_IO; return; }
                    V3 bc = mcpt::v3(1.f, 1.f, 1.f);
                    int mati = (int)pr.numv("material", -1);
                    if (mats && mati >= 0 && mati < (int)mats->arr.size()) {
                        const Json* pbr = mats->arr[mati].get("pbrMetallicRoughness");
                        const Json* bcf = pbr ? pbr->get("baseColorFactor") : nullptr;
                        if (bcf && bcf->arr.size() >= 3)
                            bc = mcpt::v3((float)bcf->arr[0].num, (float)bcf->arr[1].num, (float)bcf->arr[2].num);
                    }
                    add_mesh(pos, nrm, idx, bc);
                }
            }
        }
        if (const Json* ch = n.get("children"))
            for (auto& c : ch->arr) visit((int)c.num, M);
    };
    std::vector<int> roots;
    const Json* scenes = root.get("scenes");
    int si = (int)root.numv("scene", 0);
    if (scenes && si >= 0 && si < (int)scenes->arr.size() && scenes->arr[si].get("nodes")) {
        for (auto& r : scenes->arr[si].get("nodes")->arr) roots.push_back((int)r.num);
    } else {
        for (int i = 0; i < (int)nodes->arr.size(); i++) roots.push_back(i);
    }
    for (int r : roots) visit(r, base);
    return status;
}

// Radiance .hdr (RGBE, flat or new-RLE) -> RGBA32F, restating stb_image's
// stbi__hdr_load/stbi__hdr_convert (rgb * ldexp(1, e-136), 0 when e == 0).
// stb_image itself is not vendored in the reference (parity unpinned).
int load_hdr(const char* path, int& W, int& H, std::vector<float>& rgba, std::string& err) {
    std::vector<uint8_t> b;
    if (!read_file(path, b)) { err = std::string("cannot read ") + path; return MCPT_E_IO; }
    size_t p = 0;
    auto line = [&]() {
        std::string s;
        while (p < b.size() && b[p] != '\n') s.push_back((char)b[p++]);
        if (p < b.size()) p++;
        return s;
    };
    std::string l = line();
    if (l.rfind("#?RADIANCE", 0) != 0 && l.rfind("#?RGBE", 0) != 0) { err = "not a radiance hdr"; return MCPT_E_IO; }
    bool fmt_ok = false;
    for (;;) {
        if (p >= b.size()) { err = "hdr: truncated header"; return MCPT_E_IO; }
        l = line();
        if (l.empty()) break;
        if (l == "FORMAT=32-bit_rle_rgbe") fmt_ok = true;
    }
    if (!fmt_ok) { err = "hdr: unsupported format"; return MCPT_E_IO; }
    l = line();
    char ya[3] = {0}, xa[3] = {0};
    if (sscanf(l.c_str(), "%2s %d %2s %d", ya, &H, xa, &W) != 4 || std::string(ya) != "-Y" || std::string(xa) != "+X" ||
        W <= 0 || H <= 0) {
        err = "hdr: unsupported orientation"; return MCPT_E_IO;
    }
    rgba.assign((size_t)W * H * 4, 0.f);
    std::vector<uint8_t> scan((size_t)W * 4);
    auto convert = [&](size_t pix, const uint8_t* in) {
        float* o = &rgba[pix * 4];
        if (in[3] != 0) {
            float f1 = (float)std::ldexp(1.0f, (int)in[3] - (128 + 8));
            o[0] = in[0] * f1; o[1] = in[1] * f1; o[2] = in[2] * f1;
        } else {
            o[0] = o[1] = o[2] = 0.f;
        }
        o[3] = 0.f;  // dTexture.cu:233 pads alpha with 0
    };
    for (int y = 0; y < H; y++) {
        if (p + 4 > b.size()) { err = "hdr: truncated"; return MCPT_E_IO; }
        bool rle = W >= 8 && W < 32768 && b[p] == 2 && b[p + 1] == 2 && !(b[p + 2] & 0x80) &&
                   (((int)b[p + 2] << 8) | b[p + 3]) == W;
        if (!rle) {  // flat RGBE
            for (int x = 0; x < W; x++) {
                if (p + 4 > b.size()) { err = "hdr: truncated"; return MCPT_E_IO; }
                convert((size_t)y * W + x, &b[p]);
                p += 4;
            }
            continue;
        }
        p += 4;
        for (int c = 0; c < 4; c++) {
            int x = 0;
            while (x < W) {
                if (p >= b.size()) { err = "hdr: truncated rle"; return MCPT_E_IO; }
                int count = b[p++];
                if (count > 128) {
                    count -= 128;
                    if (p >= b.size() || x + count > W) { err = "hdr: bad rle run"; return MCPT_E_IO; }
                    uint8_t v = b[p++];
                    for (int i = 0; i < count; i++) scan[(size_t)(x++) * 4 + c] = v;
                } else {
                    if (count == 0 || p + count > b.size() || x + count > W) { err = "hdr: bad rle dump"; return MCPT_E_IO; }
                    for (int i = 0; i < count; i++) scan[(size_t)(x++) * 4 + c] = b[p++];
                }
            }
        }
        for (int x = 0; x < W; x++) convert((size_t)y * W + x, &scan[(size_t)x * 4]);
    }
    return MCPT_OK;
}

// Env tables (light_initialization_kernels.cu:3-112), same serial order as the
// reference's <<<1,1>>> kernels; computed once on the host.
void build_env_tables(int W, int H, const std::vector<float>& tex, std::vector<float>& marginal_y,
                      std::vector<float>& marginal_p, std::vector<float>& conds_y, std::vector<float>& pdf,
                      float& denom_out) {
    const float4* t = reinterpret_cast<const float4*>(tex.data());
    marginal_y.assign(H, 0.f);
    marginal_p.assign(H, 0.f);
    conds_y.assign((size_t)W * H, 0.f);
    pdf.assign((size_t)W * H, 0.f);
    float denom = 0.0f;
    for (int j = 0; j < H; j++) {
        float v = (float)j / (float)H;
        float s = mcpt::dsin(mcpt::PI_F * v);
        for (int i = 0; i < W; i++) {
            float u = (float)i / (float)W;
            float lum = mcpt::luminance(mcpt::tex_bilinear(t, W, H, u, v));
            denom += lum * s;
        }
    }
    for (int j = 0; j < H; j++) {
        float v = (float)j / (float)H;
        double st = (double)(mcpt::dsin(mcpt::PI_F * v) / denom);
        float mp = 0.f;
        for (int i = 0; i < W; i++) {
            float u = (float)i / (float)W;
            double lum = (double)mcpt::luminance(mcpt::tex_bilinear(t, W, H, u, v));
            mp = (float)((double)mp + lum * st);
        }
        marginal_p[j] = mp;
        marginal_y[j] = (j != 0) ? mp + marginal_y[j - 1] : mp;
    }
    for (int y = 0; y < H; y++) {
        float v = (float)y / (float)H;
        float st = mcpt::dsin(mcpt::PI_F * v);
        float val = st / (denom * marginal_p[y]);
        float* row = &conds_y[(size_t)y * W];
        for (int x = 0; x < W; x++) {
            float u = (float)x / (float)W;
            float lum = mcpt::luminance(mcpt::tex_bilinear(t, W, H, u, v));
            row[x] = lum * val;
            if (x != 0) row[x] = row[x] + row[x - 1];
        }
    }
    for (int y = 0; y < H; y++) {
        float v = (float)y / (float)H;
        float st = mcpt::dsin(mcpt::PI_F * v);
        for (int x = 0; x < W; x++) {
            float u = (float)x / (float)W;
            float lum = mcpt::luminance(mcpt::tex_bilinear(t, W, H, u, v));
            pdf[(size_t)y * W + x] = (lum * st) / denom;
        }
    }
    denom_out = denom;
}

int Scene::set_env_hdr(const char* path, int mode, std::string& err, bool host_tables) {
    int W = 0, H = 0;
    std::vector<float> tex;
    int rc = load_hdr(path, W, H, tex, err);
    if (rc) return rc;
    env_w = W;
    env_h = H;
    env_tex.swap(tex);
    env_mode = mode;
    if (!host_tables) {  // built on the device at upload (env_build.hip)
        env_marginal_y.clear(); env_marginal_p.clear(); env_conds_y.clear(); env_pdf.clear();
        env_pdf_denom = 0.f;
        return MCPT_OK;
    }
    float denom;
    build_env_tables(W, H, env_tex, env_marginal_y, env_marginal_p, env_conds_y, env_pdf, denom);
    env_pdf_denom = denom;
    return MCPT_OK;
}

// ---------------------------------------------------------------------------
// SAH BVH (BVH.cu:84-333): 12 buckets, cost .125 + (n0 A0 + n1 A1) / A,
// depth-first flatten into LinearBVHNode order, triangles gathered by
// orderedPrims (Scene.cu:459-469).  Topology is implementation-defined in the
// reference (MSVC std::partition); only closest-hit results are a contract.
// Deviation for robustness: leaves never exceed max_prims (degenerate centroid
// sets are split by index instead of becoming one huge leaf).
// ---------------------------------------------------------------------------
struct Bounds {
    V3 mn, mx;
    Bounds() {
        float lo = -3.402823466e+38f, hi = 3.402823466e+38f;
        mn = mcpt::v3(hi, hi, hi);
        mx = mcpt::v3(lo, lo, lo);
    }
    void add(V3 p) {
        mn = mcpt::v3(std::fmin(mn.x, p.x), std::fmin(mn.y, p.y), std::fmin(mn.z, p.z));
        mx = mcpt::v3(std::fmax(mx.x, p.x), std::fmax(mx.y, p.y), std::fmax(mx.z, p.z));
    }
    void add(const Bounds& b) {
        mn = mcpt::v3(std::fmin(mn.x, b.mn.x), std::fmin(mn.y, b.mn.y), std::fmin(mn.z, b.mn.z));
        mx = mcpt::v3(std::fmax(mx.x, b.mx.x), std::fmax(mx.y, b.mx.y), std::fmax(mx.z, b.mx.z));
    }
    double area() const {  // Bounds3f.h:59-63
        V3 d = mx - mn;
        return 2.0 * (d.x * d.y + d.x * d.z + d.y * d.z);
    }
    int max_extent() const {
        V3 d = mx - mn;
        if (d.x > d.y && d.x > d.z) return 0;
        if (d.y > d.z) return 1;
        return 2;
    }
};
static float comp(V3 v, int a) { return a == 0 ? v.x : a == 1 ? v.y : v.z; }
struct PrimInfo { int prim; Bounds b; V3 c; };
struct BuildNode { Bounds b; int child[2] = {-1, -1}; int axis = 0, first = 0, n = 0; };

struct Builder {
    std::vector<PrimInfo>& info;
    std::vector<BuildNode> nodes;
    std::vector<int> ordered;
    int max_prims;
    int max_depth = 0;
    // mode 1 (MCPT_BVH_SAH3): binned SAH over all three axes with prefix/suffix sweeps,
    // cost ct + ci (n0 A0 + n1 A1) / A against leaf cost ci n
    int mode = 0, nb = 32;
    double ct = 1.0, ci = 1.0;
    Builder(std::vector<PrimInfo>& i, int mp) : info(i), max_prims(mp) {}

    // Leaves are created left to right over disjoint ranges, so the final orderedPrims is
    // info's prim order and a leaf's first triangle is its range start.
    int leaf(int start, int end, const Bounds& b) {
        BuildNode n;
        n.b = b; n.first = start; n.n = end - start;
        nodes.push_back(n);
        return (int)nodes.size() - 1;
    }
    int median_split(int start, int end, int dim) {
        const int mid = (start + end) / 2;
        std::nth_element(info.begin() + start, info.begin() + mid, info.begin() + end,
                         [dim](const PrimInfo& a, const PrimInfo& c) {
                             return comp(a.c, dim) < comp(c.c, dim) || (comp(a.c, dim) == comp(c.c, dim) && a.prim < c.prim);
                         });
        return mid;
    }
    int inner(int start, int mid, int end, int depth, int dim) {
        int me = (int)nodes.size();
        nodes.push_back(BuildNode());
        int c0 = build(start, mid, depth + 1);
        int c1 = build(mid, end, depth + 1);
        nodes[me].child[0] = c0;
        nodes[me].child[1] = c1;
        nodes[me].axis = dim;
        nodes[me].b = nodes[c0].b;
        nodes[me].b.add(nodes[c1].b);
        nodes[me].n = 0;
        return me;
    }
    // The split decision for info[start, end), partitioning the range in place: a leaf, or
    // the split position and axis.  Depends on the range's contents alone, so subtrees can
    // be built concurrently with the same result (build_parallel).
    struct Split { bool leaf; int mid, dim; Bounds b; };
    Split decide_sah3(int start, int end) {
        Bounds b;
        for (int i = start; i < end; i++) b.add(info[i].b);
        const int np = end - start;
        if (np == 1) return {true, 0, 0, b};
        Bounds cb;
        for (int i = start; i < end; i++) cb.add(info[i].c);
        const double A = b.area();
        double best = 1e300;
        int bdim = -1, bsplit = 0;
        std::vector<int> cnt(nb);
        std::vector<Bounds> bb(nb), right(nb);
        for (int dim = 0; dim < 3; dim++) {
            const float lo = comp(cb.mn, dim), hi = comp(cb.mx, dim);
            if (!(hi > lo)) continue;
            std::fill(cnt.begin(), cnt.end(), 0);
            std::fill(bb.begin(), bb.end(), Bounds());
            const double scale = (double)nb / ((double)hi - (double)lo);
            for (int i = start; i < end; i++) {
                int k = (int)(((double)comp(info[i].c, dim) - lo) * scale);
                k = k < 0 ? 0 : (k >= nb ? nb - 1 : k);
                cnt[k]++;
                bb[k].add(info[i].b);
            }
            Bounds acc;
            int rc = 0;
            std::vector<int> rcnt(nb);
            for (int k = nb - 1; k > 0; k--) {
                acc.add(bb[k]);
                rc += cnt[k];
                right[k] = acc;
                rcnt[k] = rc;
            }
            Bounds left;
            int lc = 0;
            for (int k = 0; k < nb - 1; k++) {
                left.add(bb[k]);
                lc += cnt[k];
                const int r = rcnt[k + 1];
                if (lc == 0 || r == 0) continue;
                const double cost = ct + ci * ((double)lc * left.area() + (double)r * right[k + 1].area()) / A;
                if (cost < best) { best = cost; bdim = dim; bsplit = k; }
            }
        }
        if (bdim < 0) {  // all centroids coincide (or one bin): leaf, or an index split to bound leaf size
            if (np <= max_prims) return {true, 0, 0, b};
            const int dim = b.max_extent();
            return {false, median_split(start, end, dim), dim, b};
        }
        if (np <= max_prims && ci * np <= best) return {true, 0, 0, b};
        const float lo = comp(cb.mn, bdim), hi = comp(cb.mx, bdim);
        const double scale = (double)nb / ((double)hi - (double)lo);
        auto it = std::partition(info.begin() + start, info.begin() + end, [&](const PrimInfo& p) {
            int k = (int)(((double)comp(p.c, bdim) - lo) * scale);
            k = k < 0 ? 0 : (k >= nb ? nb - 1 : k);
            return k <= bsplit;
        });
        int mid = (int)(it - info.begin());
        if (mid == start || mid == end) mid = median_split(start, end, bdim);
        return {false, mid, bdim, b};
    }
    Split decide(int start, int end) {
        if (mode == 1) return decide_sah3(start, end);
        Bounds b;
        for (int i = start; i < end; i++) b.add(info[i].b);
        int np = end - start;
        if (np == 1) return {true, 0, 0, b};
        Bounds cb;
        for (int i = start; i < end; i++) cb.add(info[i].c);
        int dim = cb.max_extent();
        int mid = (start + end) / 2;
        float cmin = comp(cb.mn, dim), cmax = comp(cb.mx, dim);
        if (cmax == cmin) {
            if (np <= max_prims) return {true, 0, 0, b};
            mid = (start + end) / 2;  // deviation: index split keeps leaves small
        } else if (np <= 2) {
            std::nth_element(info.begin() + start, info.begin() + mid, info.begin() + end,
                             [dim](const PrimInfo& a, const PrimInfo& c) { return comp(a.c, dim) < comp(c.c, dim); });
        } else {
            constexpr int NB = 12;
            int count[NB] = {0};
            Bounds bb[NB];
            auto bucket = [&](const PrimInfo& p) {
                float o = comp(p.c, dim) - cmin;
                if (cmax > cmin) o /= cmax - cmin;  // Bounds3f::offset (Bounds3f.h:80-86)
                int k = (int)(NB * o);
                if (k == NB) k = NB - 1;
                return k;
            };
            for (int i = start; i < end; i++) { int k = bucket(info[i]); count[k]++; bb[k].add(info[i].b); }
            float cost[NB - 1];
            for (int i = 0; i < NB - 1; i++) {
                Bounds b0, b1;
                int c0 = 0, c1 = 0;
                for (int j = 0; j <= i; j++) { b0.add(bb[j]); c0 += count[j]; }
                for (int j = i + 1; j < NB; j++) { b1.add(bb[j]); c1 += count[j]; }
                double a0 = c0 ? b0.area() : 0.0, a1 = c1 ? b1.area() : 0.0;
                cost[i] = (float)(.125f + (c0 * a0 + c1 * a1) / b.area());
            }
            float minCost = cost[0];
            int split = 0;
            for (int i = 1; i < NB - 1; i++)
                if (cost[i] < minCost) { minCost = cost[i]; split = i; }
            float leafCost = (float)np;
            if (np > max_prims || minCost < leafCost) {
                auto it = std::partition(info.begin() + start, info.begin() + end,
                                         [&](const PrimInfo& p) { return bucket(p) <= split; });
                mid = (int)(it - info.begin());
                if (mid == start || mid == end) {
                    mid = (start + end) / 2;
                    std::nth_element(info.begin() + start, info.begin() + mid, info.begin() + end,
                                     [dim](const PrimInfo& a, const PrimInfo& c) { return comp(a.c, dim) < comp(c.c, dim); });
                }
            } else {
                return {true, 0, 0, b};
            }
        }
        return {false, mid, dim, b};
    }
    int build(int start, int end, int depth) {
        max_depth = std::max(max_depth, depth);
        const Split sp = decide(start, end);
        if (sp.leaf) return leaf(start, end, sp.b);
        return inner(start, sp.mid, end, depth, sp.dim);
    }
    // Same tree as build(0, T, 0), with the subtrees below a cut built by worker threads:
    // the top of the tree is split here; ranges of at most `grain` triangles become tasks,
    // each a Builder of its own over its disjoint range of info (every decision depends on
    // the range alone, so the tree -- and the flattened arrays -- are identical).  Task
    // nodes are appended afterwards and the cut's child links re-pointed.
    int build_parallel(int start0, int end0, int depth0, int nthreads) {
        struct Task { int start, end, depth, parent, slot; Builder* b; int root; };
        std::vector<Task> tasks;
        const int grain = std::max(4096, (end0 - start0) / (8 * nthreads));
        std::function<int(int, int, int, int, int)> top = [&](int start, int end, int depth, int parent, int slot) -> int {
            max_depth = std::max(max_depth, depth);
            if (end - start <= grain) {
                tasks.push_back({start, end, depth, parent, slot, nullptr, -1});
                return -1;  // filled in after the tasks ran
            }
            const Split sp = decide(start, end);
            if (sp.leaf) return leaf(start, end, sp.b);
            const int me = (int)nodes.size();
            nodes.push_back(BuildNode());
            const int c0 = top(start, sp.mid, depth + 1, me, 0);
            const int c1 = top(sp.mid, end, depth + 1, me, 1);
            nodes[me].child[0] = c0;
            nodes[me].child[1] = c1;
            nodes[me].axis = sp.dim;
            nodes[me].n = 0;
            return me;
        };
        const int root = top(start0, end0, depth0, -1, 0);
        std::vector<std::unique_ptr<Builder>> owned;
        for (Task& t : tasks) {
            owned.emplace_back(new Builder(info, max_prims));
            t.b = owned.back().get();
            t.b->mode = mode; t.b->nb = nb; t.b->ct = ct; t.b->ci = ci;
        }
        std::atomic<size_t> next{0};
        auto work = [&]() {
            for (size_t k; (k = next.fetch_add(1)) < tasks.size();)
                tasks[k].root = tasks[k].b->build(tasks[k].start, tasks[k].end, tasks[k].depth);
        };
        std::vector<std::thread> pool;
        for (int i = 1; i < nthreads; i++) pool.emplace_back(work);
        work();
        for (auto& th : pool) th.join();
        const int cut_end = (int)nodes.size();
        int rootref = root;
        for (Task& t : tasks) {
            const int off = (int)nodes.size();
            for (BuildNode n : t.b->nodes) {
                if (n.n == 0) { n.child[0] += off; n.child[1] += off; }
                nodes.push_back(n);
            }
            max_depth = std::max(max_depth, t.b->max_depth);
            if (t.parent < 0) rootref = t.root + off;
            else nodes[t.parent].child[t.slot] = t.root + off;
        }
        // boxes of the interior nodes above the cut, bottom-up
        std::function<void(int)> fix = [&](int i) {
            if (i >= cut_end || nodes[i].n > 0) return;
            fix(nodes[i].child[0]);
            fix(nodes[i].child[1]);
            nodes[i].b = nodes[nodes[i].child[0]].b;
            nodes[i].b.add(nodes[nodes[i].child[1]].b);
        };
        fix(rootref);
        return rootref;
    }
};

int Scene::build(int max_prims, std::string& err) {
    mcpt_bvh_params p{};
    p.builder = MCPT_BVH_REFERENCE;
    p.max_prims = max_prims;
    return build(p, err);
}

int Scene::build(const mcpt_bvh_params& prm, std::string& err) {
    const int max_prims = prm.max_prims;
    if (max_prims < 1 || max_prims > 8) { err = "max_prims must be 1..8"; return MCPT_E_INVALID; }
    if (prm.builder != MCPT_BVH_REFERENCE && prm.builder != MCPT_BVH_SAH3) { err = "unknown BVH builder"; return MCPT_E_INVALID; }
    if (prm.builder == MCPT_BVH_SAH3 && (prm.buckets < 2 || prm.buckets > 256 || !(prm.trav_cost >= 0.f) || !(prm.isect_cost > 0.f))) {
        err = "SAH3 needs 2..256 buckets, trav_cost >= 0, isect_cost > 0";
        return MCPT_E_INVALID;
    }
    size_t T = tris.size();
    std::vector<PrimInfo> info(T);
    for (size_t i = 0; i < T; i++) {  // g_init_BVH_triangle_info (mesh_initialization_kernels.cu:63-83)
        info[i].prim = (int)i;
        for (int k = 0; k < 3; k++) info[i].b.add(tris[i].p[k]);
        info[i].c = info[i].b.mn * 0.5f + info[i].b.mx * 0.5f;
    }
    Builder bld(info, max_prims);
    if (prm.builder == MCPT_BVH_SAH3) {
        bld.mode = 1;
        bld.nb = prm.buckets;
        bld.ct = prm.trav_cost;
        bld.ci = prm.isect_cost;
    }
    node_bmin.clear(); node_bmax.clear(); node_offset.clear(); node_nprims.clear(); node_axis.clear();
    bvh_depth = 0;
    if (T > 0) {
        // MCPT_BVH_THREADS: worker threads for the subtrees (default min(16, cores); 1 = sequential)
        int nth = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
        if (const char* e = std::getenv("MCPT_BVH_THREADS")) nth = std::max(1, std::atoi(e));
        // SAH3: triangles whose boxes the traversal may never cull (mcpt_core.hpp cull_tri_margin:
        // large against the det >= 1e-6 threshold and not in an axis plane) get a subtree of
        // their own under the root.  Every ancestor of such a triangle is unbounded too, so mixed
        // into the tree they would keep whole subtrees of small triangles from being culled
        // (config 2's ten wall triangles sat under 7 interior nodes).  MCPT_BVH_ISOLATE=0: off.
        int nbig = 0;
        if (bld.mode == 1) {
            const char* iso = std::getenv("MCPT_BVH_ISOLATE");
            const char* pl = std::getenv("MCPT_CULL_PLANE");  // as runtime.cpp's margins
            const bool plane = !(pl && pl[0] == '0' && pl[1] == 0);
            if (!(iso && iso[0] == '0' && iso[1] == 0)) {
                auto unbounded = [&](const PrimInfo& p) {
                    const V3* P = tris[(size_t)p.prim].p;
                    const V3 e1 = P[1] - P[0], e2 = P[2] - P[0];  // as the triangle record stores them
                    return mcpt::cull_tri_unbounded(e1, e2, plane);
                };
                auto it = std::stable_partition(info.begin(), info.end(), unbounded);
                nbig = (int)(it - info.begin());
                if (nbig == (int)T) nbig = 0;  // every triangle unbounded: nothing to isolate
            }
        }
        auto sub = [&](int start, int end, int depth) {
            return (end - start >= 65536 && nth > 1) ? bld.build_parallel(start, end, depth, nth) : bld.build(start, end, depth);
        };
        int root;
        if (nbig > 0) {
            root = (int)bld.nodes.size();
            bld.nodes.push_back(BuildNode());
            const int c0 = sub(0, nbig, 1), c1 = sub(nbig, (int)T, 1);
            bld.nodes[root].child[0] = c0;
            bld.nodes[root].child[1] = c1;
            bld.nodes[root].b = bld.nodes[c0].b;
            bld.nodes[root].b.add(bld.nodes[c1].b);
            bld.nodes[root].n = 0;
            bld.max_depth = std::max(bld.max_depth, 1);
        } else {
            root = sub(0, (int)T, 0);
        }
        bvh_depth = bld.max_depth;
        // flatten_tree (BVH.cu:312-333): depth-first, first child adjacent.
        std::function<int(int)> flatten = [&](int ni) -> int {
            const BuildNode& n = bld.nodes[ni];
            int my = (int)node_nprims.size();
            node_bmin.insert(node_bmin.end(), {n.b.mn.x, n.b.mn.y, n.b.mn.z});
            node_bmax.insert(node_bmax.end(), {n.b.mx.x, n.b.mx.y, n.b.mx.z});
            node_offset.push_back(0);
            node_nprims.push_back(n.n);
            node_axis.push_back(n.axis);
            if (n.n > 0) {
                node_offset[my] = n.first;
            } else {
                flatten(n.child[0]);
                node_offset[my] = flatten(n.child[1]);
            }
            return my;
        };
        flatten(root);
    }
    // gather triangles in orderedPrims order (Scene.cu:459-469)
    bld.ordered.resize(T);
    for (size_t i = 0; i < T; i++) bld.ordered[i] = info[i].prim;  // orderedPrims (leaf ranges in order)
    size_t N = T;
    f_v0.resize(3 * N); f_v1.resize(3 * N); f_v2.resize(3 * N);
    f_n0.resize(3 * N); f_n1.resize(3 * N); f_n2.resize(3 * N);
    f_mat.resize(N);
    f_id.resize(N);
    for (size_t i = 0; i < N; i++) {
        f_id[i] = bld.ordered.empty() ? (int32_t)i : bld.ordered[i];
        const Tri& t = tris[(size_t)f_id[i]];
        const V3* P = t.p;
        const V3* Nn = t.n;
        float* dst[6] = {&f_v0[3 * i], &f_v1[3 * i], &f_v2[3 * i], &f_n0[3 * i], &f_n1[3 * i], &f_n2[3 * i]};
        V3 src[6] = {P[0], P[1], P[2], Nn[0], Nn[1], Nn[2]};
        for (int k = 0; k < 6; k++) { dst[k][0] = src[k].x; dst[k][1] = src[k].y; dst[k][2] = src[k].z; }
        f_mat[i] = t.mat;
    }
    built = true;
    return MCPT_OK;
}

void Scene::desc(mcpt_scene_desc* d) const {
    memset(d, 0, sizeof(*d));
    d->ntri = (int32_t)f_mat.size();
    d->v0 = f_v0.data(); d->v1 = f_v1.data(); d->v2 = f_v2.data();
    d->n0 = f_n0.data(); d->n1 = f_n1.data(); d->n2 = f_n2.data();
    d->mat = f_mat.data();
    d->nnodes = (int32_t)node_nprims.size();
    d->bmin = node_bmin.data(); d->bmax = node_bmax.data();
    d->offset = node_offset.data(); d->nprims = node_nprims.data(); d->axis = node_axis.data();
    d->nmat = (int32_t)(materials.size() / 8);
    d->mat_params = materials.data();
    d->ndir = (int32_t)(dir_lights.size() / 7);
    d->dir_params = dir_lights.data();
    d->env_mode = env_mode;
    for (int i = 0; i < 3; i++) d->env_color[i] = env_color[i];
    d->env_ls = env_ls;
    d->env_w = env_w; d->env_h = env_h;
    d->env_tex = env_tex.empty() ? nullptr : env_tex.data();
    d->env_marginal_y = env_marginal_y.empty() ? nullptr : env_marginal_y.data();
    d->env_conds_y = env_conds_y.empty() ? nullptr : env_conds_y.data();
    d->env_pdf = env_pdf.empty() ? nullptr : env_pdf.data();
    d->tri_id = f_id.empty() ? nullptr : f_id.data();
}

// ---------------------------------------------------------------------------
// Camera (Camera.cu:194-224, PerspectiveCamera.cpp:49; glm semantics).
// ---------------------------------------------------------------------------
void make_camera(const mcpt_camera_params& p, mcpt_camera& out) {
    const float deg = 0.01745329251994329576923690768489f;  // glm::radians
    float yaw = p.yaw_deg * deg, pitch = p.pitch_deg * deg;
    V3 front = mcpt::v3(std::cos(yaw) * std::cos(pitch), std::sin(pitch), std::sin(yaw) * std::cos(pitch));
    front = glm_normalize(front);
    V3 worldUp = mcpt::v3(0.f, 1.f, 0.f);
    V3 right = glm_normalize(glm_cross(front, worldUp));
    V3 up = glm_normalize(glm_cross(right, front));
    V3 eye = mcpt::v3(p.position[0], p.position[1], p.position[2]);
    V3 center = eye + front;
    // glm::lookAtRH
    V3 f = glm_normalize(center - eye);
    V3 s = glm_normalize(glm_cross(f, up));
    V3 u = glm_cross(s, f);
    M4 view = m4_identity();
    view.m[0] = s.x; view.m[4] = s.y; view.m[8] = s.z;
    view.m[1] = u.x; view.m[5] = u.y; view.m[9] = u.z;
    view.m[2] = -f.x; view.m[6] = -f.y; view.m[10] = -f.z;
    view.m[12] = -glm_dot(s, eye); view.m[13] = -glm_dot(u, eye); view.m[14] = glm_dot(f, eye);
    // glm::perspectiveRH_NO
    float tanHalf = std::tan(p.fovy_rad / 2.f);
    M4 proj{};
    proj.m[0] = 1.f / (p.aspect * tanHalf);
    proj.m[5] = 1.f / tanHalf;
    proj.m[10] = -(p.zfar + p.znear) / (p.zfar - p.znear);
    proj.m[11] = -1.f;
    proj.m[14] = -(2.f * p.zfar * p.znear) / (p.zfar - p.znear);
    M4 ivp = m4_inverse(m4_mul(proj, view));
    M4 iv = m4_inverse(view);
    memcpy(out.inv_view_proj, ivp.m, sizeof(ivp.m));
    memcpy(out.inv_view, iv.m, sizeof(iv.m));
    out.lens_radius = p.lens_radius;
    out.focal = p.focal;
}

}  // namespace mcpt_host
