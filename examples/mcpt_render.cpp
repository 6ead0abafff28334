// mcpt_render.cpp -- the reference's render loop written against the C ABI only
// (what a maintainer's PathTracer::render_image + RenderingContext "Save" become,
// INTEGRATION.md): build a BASELINE config scene with the host builder, upload it,
// run the wavefront iterations until every pixel has its samples, write PNG + PFM.
//
//   mcpt_render <config 1-5> [spp] [out_prefix] [--gpu-bvh] [--reference-bvh] [--fixed] [--tiles-per-call] [--slots S]
//
// --tiles-per-call uses the reference orchestration (one 256x256 tile per call,
// wavefront_kernels.cu:377-442 + Film::update_tile_position) instead of batch mode.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "mcpt.h"

struct Cfg { int w, h, spp, depth; float pos[3], pitch; const char* env; };

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <config 1-5> [spp] [out_prefix] [--gpu-bvh] [--reference-bvh] [--fixed] [--tiles-per-call] [--slots S]\n", argv[0]);
        return 2;
    }
    const Cfg cfgs[6] = {{0, 0, 0, 0, {0, 0, 0}, 0, ""},
                         {256, 256, 16, 3, {0.f, 0.f, 4.f}, 0.f, "HDR_029_Sky_Cloudy_Env.hdr"},
                         {1920, 1080, 256, 5, {0.f, 0.f, 3.5f}, 0.f, "night_free_Env.hdr"},
                         {1920, 1080, 256, 5, {0.f, 1.5f, 4.5f}, -10.f, "night_free_Env.hdr"},
                         {3840, 2160, 1024, 8, {0.f, 0.f, 2.5f}, 0.f, "HDR_029_Sky_Cloudy_Env.hdr"},
                         {4096, 4096, 4096, 12, {0.f, 1.2f, 3.f}, -5.f, "night_free_Env.hdr"}};
    const int id = atoi(argv[1]);
    if (id < 1 || id > 5) { fprintf(stderr, "config must be 1..5\n"); return 2; }
    Cfg c = cfgs[id];
    if (argc > 2 && argv[2][0] != '-') c.spp = atoi(argv[2]);
    std::string out = (argc > 3 && argv[3][0] != '-') ? argv[3] : "mcpt_render";
    bool gpu_bvh = false, ref_bvh = false, fixed = false, per_tile = false;
    uint32_t slots = 1;
    for (int i = 2; i < argc; i++) {
        if (!strcmp(argv[i], "--gpu-bvh")) gpu_bvh = true;
        if (!strcmp(argv[i], "--reference-bvh")) ref_bvh = true;
        if (!strcmp(argv[i], "--fixed")) fixed = true;
        if (!strcmp(argv[i], "--tiles-per-call")) per_tile = true;
        if (!strcmp(argv[i], "--slots") && i + 1 < argc) slots = (uint32_t)atoi(argv[++i]);
    }
    const char* assets = getenv("MCPT_ASSETS") ? getenv("MCPT_ASSETS") : "assets";

    // Scene::load + BVHAccel + EnvironmentLight (host builder)
    mcpt_scene* s = mcpt_scene_new();
    // host BVH: binned 3-axis SAH (default) or BVHAccel's builder; films are identical either way
    mcpt_bvh_params bp = {MCPT_BVH_SAH3, 8, 128, 0.5f, 1.0f};
    if (!s || mcpt_scene_make_proxy(s, id, assets) || (ref_bvh ? mcpt_scene_build(s, 8) : mcpt_scene_build_ex(s, &bp))) {
        fprintf(stderr, "scene: %s\n", mcpt_last_error(nullptr));
        return 1;
    }
    mcpt_scene_desc d;
    mcpt_scene_get_desc(s, &d);

    // PathTracer::PathTracer
    mcpt_config cfg{0x5EED2026ull, c.spp, c.depth, 3, 256, 256, fixed ? MCPT_FLAG_FIXED : 0};
    mcpt_ctx* ctx = nullptr;
    if (mcpt_create(0, &cfg, &ctx) != MCPT_OK) {
        fprintf(stderr, "mcpt_create: %s\n", mcpt_last_error(nullptr));
        return 1;
    }
    int rc = gpu_bvh ? mcpt_scene_upload_gpu_bvh(ctx, &d) : mcpt_scene_upload(ctx, &d);
    // Camera::update
    mcpt_camera_params cp{{c.pos[0], c.pos[1], c.pos[2]}, -90.f, c.pitch, 0.785398163f, (float)c.w / (float)c.h,
                          0.01f, 1e4f, 1e-4f, 35.f};
    mcpt_camera cam;
    if (!rc) rc = mcpt_camera_make(&cp, &cam);
    if (!rc) rc = mcpt_camera_set(ctx, &cam);
    if (!rc) rc = mcpt_set_path_slots(ctx, slots);  // paths in flight per pixel (default 1)
    if (!rc) rc = mcpt_film_resize(ctx, c.w, c.h, 256, 256);
    if (rc) { fprintf(stderr, "setup: %s\n", mcpt_last_error(ctx)); return 1; }

    mcpt_stage_stats st{};
    if (per_tile) {  // reference orchestration: one iteration of one tile per call, tiles round-robin
        const uint32_t tx_n = (c.w + 255) / 256, ty_n = (c.h + 255) / 256;
        uint64_t rays = 0;
        double ms = 0;
        for (uint32_t round = 0; round < 1000000u && !rc; round++) {
            uint64_t round_rays = 0;
            for (uint32_t t = 0; t < tx_n * ty_n && !rc; t++) {  // Film::update_tile_position
                mcpt_stage_stats one{};
                rc = mcpt_wavefront_step(ctx, t % tx_n, t / tx_n, &one);
                round_rays += one.extend_rays + one.shadow_rays + one.vis_rays;
                ms += one.ms_total;
            }
            rays += round_rays;
            if (round_rays == 0) break;  // every pixel has its samples
        }
        st.extend_rays = rays;
        st.ms_total = (float)ms;
    } else {
        rc = mcpt_render(ctx, &st);  // batch: every tile per iteration until all pixels have spp
    }
    if (rc) { fprintf(stderr, "render: %s\n", mcpt_last_error(ctx)); return 1; }
    const uint64_t rays = per_tile ? st.extend_rays : st.extend_rays + st.shadow_rays + st.vis_rays;
    printf("config %d %dx%d %d spp depth %d%s%s: %llu rays, %.1f ms device time, %.0f Mray/s\n", id, c.w, c.h,
           c.spp, c.depth, gpu_bvh ? " gpu-bvh" : "", fixed ? " fixed" : "", (unsigned long long)rays,
           st.ms_total, rays / (st.ms_total * 1e-3) / 1e6);
    if ((rc = mcpt_film_write_png(ctx, 1.f, (out + ".png").c_str())) ||
        (rc = mcpt_film_write_pfm(ctx, (out + ".pfm").c_str()))) {
        fprintf(stderr, "write: %s\n", mcpt_last_error(ctx));
        return 1;
    }
    mcpt_destroy(ctx);
    mcpt_scene_free(s);
    return 0;
}
