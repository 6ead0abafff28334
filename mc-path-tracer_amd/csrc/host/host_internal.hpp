// host_internal.hpp -- host-side scene model (Scene.h / Mesh.h / EnvironmentLight.h
// of the reference, reduced to what the path-tracing backend consumes).
#pragma once
#include <functional>
#include <string>
#include <vector>

#include "../device/mcpt_core.hpp"
#include "mcpt.h"

namespace mcpt_host {

struct Tri {
    mcpt::V3 p[3];
    mcpt::V3 n[3];
    int mat;
};

struct Scene {
    // meshes (Scene::render_objects, Mesh.cu:35-60), world space
    std::vector<Tri> tris;
    std::vector<float> materials;   // 8 floats per material (dMaterial.cuh:11-33)
    std::vector<float> dir_lights;  // 7 floats per light (DirectionalLight.h)
    // environment light (EnvironmentLight.h:17-40); default Color 0.8 (Scene.cu:21)
    int env_mode = 0;
    float env_color[3] = {0.8f, 0.8f, 0.8f};
    float env_ls = 1.f;
    int env_w = 0, env_h = 0;
    float env_pdf_denom = 0.f;
    std::vector<float> env_tex, env_marginal_y, env_marginal_p, env_conds_y, env_pdf;
    // built, BVH-ordered arrays (mcpt_scene_desc)
    bool built = false;
    int bvh_depth = 0;
    std::vector<float> f_v0, f_v1, f_v2, f_n0, f_n1, f_n2;
    std::vector<int32_t> f_mat;
    std::vector<int32_t> f_id;  // original triangle index of each BVH-ordered slot
    std::vector<float> node_bmin, node_bmax;
    std::vector<int32_t> node_offset, node_nprims, node_axis;
    std::string err;

    void add_mesh(const std::vector<mcpt::V3>& pos, const std::vector<mcpt::V3>& nrm,
                  const std::vector<uint32_t>& idx, mcpt::V3 base);
    void transform(const float* xf16);
    int load_glb(const char* path, const float* xf16, std::string& err);
    int set_env_hdr(const char* path, int mode, std::string& err, bool host_tables = true);
    int build(int max_prims, std::string& err);
    int build(const mcpt_bvh_params& p, std::string& err);
    void desc(mcpt_scene_desc* d) const;
};

int load_hdr(const char* path, int& W, int& H, std::vector<float>& rgba, std::string& err);
void build_env_tables(int W, int H, const std::vector<float>& tex, std::vector<float>& marginal_y,
                      std::vector<float>& marginal_p, std::vector<float>& conds_y, std::vector<float>& pdf,
                      float& denom);
void make_camera(const mcpt_camera_params& p, mcpt_camera& out);
int make_proxy(Scene& s, int config_id, const std::string& asset_dir, std::string& err);

}  // namespace mcpt_host
