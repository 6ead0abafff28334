// proxies.cpp -- deterministic stand-ins for the BASELINE configs whose assets are
// missing from the reference snapshot (.MISSING_LARGE_BLOBS): SURVEY.md section 8(d).
//   C1  models/sphere.glb + hrdi/HDR_029_Sky_Cloudy_Env.hdr          (real assets)
//   C2  Cornell box [-1,1]^3 open at +z + 5 sphere.glb instances      (scene_show_off_spheres.glb)
//   C3  displaced icosphere, 871,414 tris + ground quad              (scene_show_off_dragon.glb)
//   C4  Suzanne.glb midpoint-subdivided x2 = 251,904 tris             (scene_show_off_head.glb)
//   C5  C3 generator at 2,000,000 tris (seed 13) + ground quad        (greek_sculpture.glb)
// C2-C5 are baked with a 1 degree rotation about normalize(1,1,1) so no surface
// normal has an exactly-zero component (gram_schmidt NaN quirk, Vector.h:1128-1139).
#include <cmath>
#include <cstring>
#include <map>
#include <unordered_map>

#include "host_internal.hpp"

using mcpt::V3;
using mcpt::v3;

namespace mcpt_host {

static uint64_t sm_state;
static double urand() {  // splitmix64 stream in [0,1)
    uint64_t z = mcpt::splitmix64(sm_state);
    sm_state += 0x9E3779B97F4A7C15ull;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

static void rotation_1deg(float out[16]) {  // axis-angle about normalize(1,1,1), 1 degree
    double a = 1.0 * M_PI / 180.0, c = cos(a), s = sin(a), t = 1 - c;
    double k = 1.0 / sqrt(3.0), x = k, y = k, z = k;
    double R[3][3] = {{t * x * x + c, t * x * y - s * z, t * x * z + s * y},
                      {t * x * y + s * z, t * y * y + c, t * y * z - s * x},
                      {t * x * z - s * y, t * y * z + s * x, t * z * z + c}};
    memset(out, 0, 16 * sizeof(float));
    for (int r = 0; r < 3; r++)
        for (int cc = 0; cc < 3; cc++) out[cc * 4 + r] = (float)R[r][cc];
    out[15] = 1.f;
}

// quad a,b,c,d (in order) with front faces (e1 x e2) pointing along 'facing'.
static void add_quad(Scene& s, V3 a, V3 b, V3 c, V3 d, V3 facing, V3 color) {
    V3 n = mcpt::cross(b - a, c - a);
    if (mcpt::dot(n, facing) < 0.f) std::swap(b, d);
    std::vector<V3> pos = {a, b, c, d}, nrm(4, facing);
    std::vector<uint32_t> idx = {0, 1, 2, 0, 2, 3};
    s.add_mesh(pos, nrm, idx, color);
}

static void add_ground(Scene& s, float half, V3 color) {
    add_quad(s, v3(-half, 0, -half), v3(half, 0, -half), v3(half, 0, half), v3(-half, 0, half), v3(0, 1, 0), color);
}

// value noise on an integer lattice, trilinear with smoothstep (seeded)
static float lattice(uint64_t seed, int x, int y, int z) {
    uint64_t h = mcpt::splitmix64(seed ^ ((uint64_t)(uint32_t)x * 0x9E3779B1ull) ^
                                  ((uint64_t)(uint32_t)y * 0x85EBCA77ull << 20) ^ ((uint64_t)(uint32_t)z * 0xC2B2AE3Dull << 40));
    return (float)((double)(h >> 11) * (1.0 / 9007199254740992.0)) * 2.f - 1.f;
}
static float value_noise(uint64_t seed, V3 p) {
    float fx = std::floor(p.x), fy = std::floor(p.y), fz = std::floor(p.z);
    int ix = (int)fx, iy = (int)fy, iz = (int)fz;
    float tx = p.x - fx, ty = p.y - fy, tz = p.z - fz;
    tx = tx * tx * (3 - 2 * tx); ty = ty * ty * (3 - 2 * ty); tz = tz * tz * (3 - 2 * tz);
    float r = 0;
    for (int k = 0; k < 8; k++) {
        int dx = k & 1, dy = (k >> 1) & 1, dz = (k >> 2) & 1;
        float w = (dx ? tx : 1 - tx) * (dy ? ty : 1 - ty) * (dz ? tz : 1 - tz);
        r += w * lattice(seed, ix + dx, iy + dy, iz + dz);
    }
    return r;
}

// Icosphere subdivided until >= ntarget triangles, truncated to ntarget,
// displaced radially by amp * fbm(p), smooth normals, centred at c.
static void add_displaced_icosphere(Scene& s, int64_t ntarget, uint64_t seed, float amp, V3 c, V3 color) {
    const float t = (1.f + std::sqrt(5.f)) / 2.f;
    std::vector<V3> P = {v3(-1, t, 0), v3(1, t, 0), v3(-1, -t, 0), v3(1, -t, 0), v3(0, -1, t), v3(0, 1, t),
                         v3(0, -1, -t), v3(0, 1, -t), v3(t, 0, -1), v3(t, 0, 1), v3(-t, 0, -1), v3(-t, 0, 1)};
    for (auto& p : P) p = mcpt::normalize(p);
    std::vector<uint32_t> F = {0, 11, 5, 0, 5, 1, 0, 1, 7, 0, 7, 10, 0, 10, 11, 1, 5, 9, 5, 11, 4, 11, 10, 2, 10, 7, 6,
                               7, 1, 8, 3, 9, 4, 3, 4, 2, 3, 2, 6, 3, 6, 8, 3, 8, 9, 4, 9, 5, 2, 4, 11, 6, 2, 10, 8, 6, 7, 9, 8, 1};
    while ((int64_t)(F.size() / 3) < ntarget) {
        std::unordered_map<uint64_t, uint32_t> mid;
        auto midpoint = [&](uint32_t a, uint32_t b) {
            uint64_t key = a < b ? ((uint64_t)a << 32 | b) : ((uint64_t)b << 32 | a);
            auto it = mid.find(key);
            if (it != mid.end()) return it->second;
            P.push_back(mcpt::normalize((P[a] + P[b]) * 0.5f));
            uint32_t id = (uint32_t)P.size() - 1;
            mid.emplace(key, id);
            return id;
        };
        std::vector<uint32_t> G;
        G.reserve(F.size() * 4);
        for (size_t i = 0; i < F.size(); i += 3) {
            uint32_t a = F[i], b = F[i + 1], cc = F[i + 2];
            uint32_t ab = midpoint(a, b), bc = midpoint(b, cc), ca = midpoint(cc, a);
            uint32_t tri[12] = {a, ab, ca, b, bc, ab, cc, ca, bc, ab, bc, ca};
            G.insert(G.end(), tri, tri + 12);
        }
        F.swap(G);
    }
    F.resize((size_t)ntarget * 3);
    std::vector<V3> Q(P.size());
    for (size_t i = 0; i < P.size(); i++) {
        V3 q = P[i] * 3.0f;
        float d = value_noise(seed, q) * 0.6f + value_noise(seed + 1, q * 2.3f) * 0.3f + value_noise(seed + 2, q * 5.1f) * 0.1f;
        Q[i] = c + P[i] * (1.f + amp * d);
    }
    std::vector<V3> N(P.size(), v3(0, 0, 0));
    for (size_t i = 0; i < F.size(); i += 3) {
        V3 fn = mcpt::cross(Q[F[i + 1]] - Q[F[i]], Q[F[i + 2]] - Q[F[i]]);
        for (int k = 0; k < 3; k++) N[F[i + k]] = N[F[i + k]] + fn;
    }
    for (auto& n : N) n = mcpt::normalize(n);
    // orient outward: e1 x e2 along the radial direction
    V3 fn0 = mcpt::cross(Q[F[1]] - Q[F[0]], Q[F[2]] - Q[F[0]]);
    if (mcpt::dot(fn0, Q[F[0]] - c) < 0.f) {
        for (size_t i = 0; i < F.size(); i += 3) std::swap(F[i + 1], F[i + 2]);
        for (auto& n : N) n = -n;
    }
    s.add_mesh(Q, N, F, color);
}

// Midpoint subdivision (x2 per level) of every mesh triangle: 4^levels tris each.
static void subdivide_all(Scene& s, int levels) {
    for (int l = 0; l < levels; l++) {
        std::vector<Tri> out;
        out.reserve(s.tris.size() * 4);
        for (const Tri& t : s.tris) {
            V3 mp[3], mn[3];
            for (int k = 0; k < 3; k++) {
                mp[k] = (t.p[k] + t.p[(k + 1) % 3]) * 0.5f;
                mn[k] = mcpt::normalize(t.n[k] + t.n[(k + 1) % 3]);
            }
            Tri a = t, b = t, c = t, d = t;
            a.p[0] = t.p[0]; a.p[1] = mp[0]; a.p[2] = mp[2]; a.n[0] = t.n[0]; a.n[1] = mn[0]; a.n[2] = mn[2];
            b.p[0] = mp[0]; b.p[1] = t.p[1]; b.p[2] = mp[1]; b.n[0] = mn[0]; b.n[1] = t.n[1]; b.n[2] = mn[1];
            c.p[0] = mp[2]; c.p[1] = mp[1]; c.p[2] = t.p[2]; c.n[0] = mn[2]; c.n[1] = mn[1]; c.n[2] = t.n[2];
            d.p[0] = mp[0]; d.p[1] = mp[1]; d.p[2] = mp[2]; d.n[0] = mn[0]; d.n[1] = mn[1]; d.n[2] = mn[2];
            out.push_back(a); out.push_back(b); out.push_back(c); out.push_back(d);
        }
        s.tris.swap(out);
    }
}

int make_proxy(Scene& s, int config_id, const std::string& dir, std::string& err) {
    std::string sep = (dir.empty() || dir.back() == '/') ? "" : "/";
    std::string sphere = dir + sep + "sphere.glb", suzanne = dir + sep + "Suzanne.glb";
    std::string hdr029 = dir + sep + "HDR_029_Sky_Cloudy_Env.hdr", night = dir + sep + "night_free_Env.hdr";
    float rot[16];
    rotation_1deg(rot);
    int rc = MCPT_OK;
    switch (config_id) {
    case 1:
        rc = s.load_glb(sphere.c_str(), nullptr, err);
        if (!rc) rc = s.set_env_hdr(hdr029.c_str(), 1, err);
        return rc;
    case 2: {
        V3 grey = v3(0.73f, 0.73f, 0.73f), red = v3(0.63f, 0.065f, 0.05f), green = v3(0.14f, 0.45f, 0.09f);
        add_quad(s, v3(-1, -1, -1), v3(1, -1, -1), v3(1, 1, -1), v3(-1, 1, -1), v3(0, 0, 1), grey);  // back
        add_quad(s, v3(-1, -1, -1), v3(1, -1, -1), v3(1, -1, 1), v3(-1, -1, 1), v3(0, 1, 0), grey);  // floor
        add_quad(s, v3(-1, 1, -1), v3(1, 1, -1), v3(1, 1, 1), v3(-1, 1, 1), v3(0, -1, 0), grey);     // ceiling
        add_quad(s, v3(-1, -1, -1), v3(-1, 1, -1), v3(-1, 1, 1), v3(-1, -1, 1), v3(1, 0, 0), red);   // left
        add_quad(s, v3(1, -1, -1), v3(1, 1, -1), v3(1, 1, 1), v3(1, -1, 1), v3(-1, 0, 0), green);    // right
        const float radii[5] = {0.3f, 0.35f, 0.4f, 0.5f, 0.6f};
        V3 cen[5];
        sm_state = 11;
        for (int i = 0; i < 5; i++) {
            float r = radii[i];
            V3 c = v3(0, 0, 0);
            for (int attempt = 0; attempt < 2000; attempt++) {
                c = v3((float)(-1 + r + (2 - 2 * r) * urand()), -1 + r, (float)(-1 + r + (2 - 2 * r) * urand()));
                bool ok = true;
                for (int j = 0; j < i; j++) {
                    V3 d = c - cen[j];
                    if (std::sqrt(mcpt::dot(d, d)) < r + radii[j] + 0.02f) ok = false;
                }
                if (ok) break;
            }
            cen[i] = c;
            float xf[16] = {r, 0, 0, 0, 0, r, 0, 0, 0, 0, r, 0, c.x, c.y, c.z, 1};
            rc = s.load_glb(sphere.c_str(), xf, err);
            if (rc) return rc;
            // spheres get distinct albedos so the image is not all grey
            const float alb[5][3] = {{0.9f, 0.9f, 0.9f}, {0.8f, 0.6f, 0.2f}, {0.2f, 0.4f, 0.8f}, {0.7f, 0.7f, 0.7f}, {0.5f, 0.8f, 0.5f}};
            float* m = &s.materials[s.materials.size() - 8];
            m[0] = alb[i][0]; m[1] = alb[i][1]; m[2] = alb[i][2];
        }
        s.transform(rot);
        return s.set_env_hdr(night.c_str(), 1, err);
    }
    case 3:
    case 5: {
        int64_t n = config_id == 3 ? 871414 : 2000000;
        uint64_t seed = config_id == 3 ? 7 : 13;
        add_displaced_icosphere(s, n, seed, 0.15f, v3(0, 1, 0), v3(0.8f, 0.8f, 0.8f));
        add_ground(s, 5.f, v3(0.6f, 0.6f, 0.6f));
        s.transform(rot);
        return s.set_env_hdr(night.c_str(), 1, err);
    }
    case 4: {
        rc = s.load_glb(suzanne.c_str(), nullptr, err);
        if (rc) return rc;
        subdivide_all(s, 2);
        s.transform(rot);
        return s.set_env_hdr(hdr029.c_str(), 1, err);
    }
    default:
        err = "unknown proxy config";
        return MCPT_E_INVALID;
    }
}

}  // namespace mcpt_host
