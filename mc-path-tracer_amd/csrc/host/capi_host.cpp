// capi_host.cpp -- extern "C" entry points of the host scene builder (mcpt_scene_*).
#include <cstring>
#include <new>

#include "host_internal.hpp"
#include "mcpt.h"

struct mcpt_scene {
    mcpt_host::Scene s;
};

namespace mcpt_host {
thread_local std::string g_last_error;
void set_global_error(const std::string& e) { g_last_error = e; }
const char* global_error() { return g_last_error.c_str(); }
}  // namespace mcpt_host

static int fail(mcpt_scene* s, int rc, const std::string& msg) {
    if (s) s->s.err = msg;
    mcpt_host::set_global_error(msg);
    return rc;
}

extern "C" {

mcpt_scene* mcpt_scene_new(void) { return new (std::nothrow) mcpt_scene(); }
void mcpt_scene_free(mcpt_scene* s) { delete s; }

int mcpt_scene_load_glb(mcpt_scene* s, const char* path, const float* xform16) {
    if (!s || !path) return fail(s, MCPT_E_INVALID, "null argument");
    std::string err;
    int rc = s->s.load_glb(path, xform16, err);
    return rc ? fail(s, rc, err) : MCPT_OK;
}

int mcpt_scene_add_mesh(mcpt_scene* s, int32_t ntri, const float* v0, const float* v1, const float* v2,
                        const float* n0, const float* n1, const float* n2, const float* base_rgb) {
    if (!s || ntri < 0 || (ntri > 0 && (!v0 || !v1 || !v2 || !n0 || !n1 || !n2)))
        return fail(s, MCPT_E_INVALID, "bad mesh arguments");
    std::vector<mcpt::V3> pos, nrm;
    std::vector<uint32_t> idx;
    const float* P[3] = {v0, v1, v2};
    const float* N[3] = {n0, n1, n2};
    for (int32_t t = 0; t < ntri; t++)
        for (int k = 0; k < 3; k++) {
            pos.push_back(mcpt::ld3(P[k], t));
            nrm.push_back(mcpt::ld3(N[k], t));
            idx.push_back((uint32_t)idx.size());
        }
    mcpt::V3 bc = base_rgb ? mcpt::v3(base_rgb[0], base_rgb[1], base_rgb[2]) : mcpt::v3(1.f, 1.f, 1.f);
    s->s.add_mesh(pos, nrm, idx, bc);
    return MCPT_OK;
}

int mcpt_scene_set_env_hdr(mcpt_scene* s, const char* path, int32_t mode) {
    if (!s || !path || (mode != 0 && mode != 1)) return fail(s, MCPT_E_INVALID, "bad env arguments");
    std::string err;
    int rc = s->s.set_env_hdr(path, mode, err);
    return rc ? fail(s, rc, err) : MCPT_OK;
}

int mcpt_scene_set_env_hdr_ex(mcpt_scene* s, const char* path, int32_t mode, uint32_t flags) {
    if (!s || !path || (mode != 0 && mode != 1) || (flags & ~(uint32_t)MCPT_ENV_DEVICE_TABLES))
        return fail(s, MCPT_E_INVALID, "bad env arguments");
    std::string err;
    int rc = s->s.set_env_hdr(path, mode, err, !(flags & MCPT_ENV_DEVICE_TABLES));
    return rc ? fail(s, rc, err) : MCPT_OK;
}

int mcpt_scene_set_env_color(mcpt_scene* s, const float* rgb, float ls) {
    if (!s || !rgb) return fail(s, MCPT_E_INVALID, "null argument");
    for (int i = 0; i < 3; i++) s->s.env_color[i] = rgb[i];
    s->s.env_ls = ls;
    s->s.env_mode = 0;
    return MCPT_OK;
}

int mcpt_scene_add_dir_light(mcpt_scene* s, const float* dir, const float* rgb, float ls) {
    if (!s || !dir || !rgb) return fail(s, MCPT_E_INVALID, "null argument");
    // device copy is NOT normalised (DirectionalLight.cu:82-88)
    float p[7] = {dir[0], dir[1], dir[2], rgb[0], rgb[1], rgb[2], ls};
    s->s.dir_lights.insert(s->s.dir_lights.end(), p, p + 7);
    return MCPT_OK;
}

int mcpt_scene_transform(mcpt_scene* s, const float* xform16) {
    if (!s || !xform16) return fail(s, MCPT_E_INVALID, "null argument");
    s->s.transform(xform16);
    return MCPT_OK;
}

int mcpt_scene_make_proxy(mcpt_scene* s, int32_t config_id, const char* asset_dir) {
    if (!s || !asset_dir) return fail(s, MCPT_E_INVALID, "null argument");
    std::string err;
    int rc = mcpt_host::make_proxy(s->s, config_id, asset_dir, err);
    return rc ? fail(s, rc, err) : MCPT_OK;
}

int mcpt_scene_build(mcpt_scene* s, int32_t max_prims_in_node) {
    if (!s) return fail(s, MCPT_E_INVALID, "null scene");
    std::string err;
    int rc = s->s.build(max_prims_in_node, err);
    return rc ? fail(s, rc, err) : MCPT_OK;
}

int mcpt_scene_build_ex(mcpt_scene* s, const mcpt_bvh_params* p) {
    if (!s || !p) return fail(s, MCPT_E_INVALID, "null argument");
    std::string err;
    int rc = s->s.build(*p, err);
    return rc ? fail(s, rc, err) : MCPT_OK;
}

int mcpt_scene_get_desc(const mcpt_scene* s, mcpt_scene_desc* out) {
    if (!s || !out) return MCPT_E_INVALID;
    if (!s->s.built) return fail(const_cast<mcpt_scene*>(s), MCPT_E_INVALID, "scene not built");
    s->s.desc(out);
    return MCPT_OK;
}

int mcpt_scene_bvh_depth(const mcpt_scene* s) { return s ? s->s.bvh_depth : MCPT_E_INVALID; }

int mcpt_camera_make(const mcpt_camera_params* p, mcpt_camera* out) {
    if (!p || !out) return MCPT_E_INVALID;
    mcpt_host::make_camera(*p, *out);
    return MCPT_OK;
}

}  // extern "C"
