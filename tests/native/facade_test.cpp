// facade_test.cpp -- the C++ host facade (include/mcpt.hpp) driven the way the reference's
// render loop drives its objects (RenderEngine.cpp:19-20 -> PathTracer::render_image).
//
//   facade_test cpu <assets>                  host logic only (no GPU needed): Film tiles,
//                                             Camera::update / rotate / move, Scene lights and
//                                             environment, errors; PathTracer must refuse to
//                                             start without a gfx950 device (no CPU fallback).
//   facade_test render <assets> <out.bin>     GPU: BASELINE config 1 at 32x32, 2 spp, depth 3
//                                             through render_image (one tile iteration per
//                                             call) until the frame is done; the film and the
//                                             camera it used go to out.bin for the oracle
//                                             comparison in tests/test_facade.py.  Also checks
//                                             batch mode == tile loop bit for bit, and the
//                                             observer clears (camera edit, light edit).
#include <cstdio>
#include <unistd.h>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mcpt.hpp"

using namespace mcpt;

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                         \
        }                                                                     \
    } while (0)

static int run_cpu(const std::string& assets) {
    // Film: tiles round-robin in row-major order (Film.cu:94-103, :172-178); clear restarts
    auto film = std::make_shared<Film>();
    film->set_size(600, 300);
    CHECK(film->get_nmb_tiles() == 6);
    const uint32_t want[7][2] = {{1, 0}, {2, 0}, {0, 1}, {1, 1}, {2, 1}, {0, 0}, {1, 0}};
    for (auto& w : want) {
        film->update_tile_position();
        CHECK(film->get_tile_x_pos() == w[0] && film->get_tile_y_pos() == w[1]);
    }
    const uint64_t clears = film->clear_count();
    film->clear();
    CHECK(film->get_tile_x_pos() == 0 && film->get_tile_y_pos() == 0 && film->clear_count() == clears + 1);
    uint32_t tw, th;
    film->get_tile_size(tw, th);
    CHECK(tw == 256 && th == 256);

    // Camera::update: the facade's dCamera equals mcpt_camera_make on the same parameters
    auto cam = std::make_shared<PerspectiveCamera>(vec3(0.f, 0.f, 4.f), radians(45.f), 0.01f, 1e4f);
    cam->set_aspect_ratio(1.f);
    mcpt_camera_params p{{0.f, 0.f, 4.f}, -90.f, 0.f, radians(45.f), 1.f, 0.01f, 1e4f, 1e-4f, 35.f};
    mcpt_camera ref;
    CHECK(mcpt_camera_make(&p, &ref) == MCPT_OK);
    CHECK(std::memcmp(&ref, &cam->get_dptr(), sizeof(ref)) == 0);
    const uint64_t r0 = cam->revision();
    cam->rotate(0.f, 5000.f);  // pitch clamped at 89 (Camera.cu:85-92)
    float yaw, pitch;
    cam->get_yaw_pitch(yaw, pitch);
    CHECK(yaw == -90.f && pitch == 89.f && cam->revision() > r0);
    cam->set_yaw_pitch(-90.f, 0.f);
    cam->move(FORWARD, 1.f);  // 2.5 units along front = -z
    CHECK(std::fabs(cam->get_position().z - 1.5f) < 1e-6f && std::fabs(cam->get_position().x) < 1e-6f);
    bool threw = false;
    try {
        PerspectiveCamera bad(std::nanf(""), 0.01f, 1e4f);
    } catch (const Error& e) {
        threw = e.code() == MCPT_E_INVALID;
    }
    CHECK(threw);

    // Scene: geometry + HRDI env from the builder, lights from the light objects
    auto scene = std::make_shared<Scene>();
    CHECK(scene->get_environment_light()->get_light_type() == Color);  // Scene.cu:13
    scene->load(assets + "/sphere.glb");
    auto env = std::make_shared<EnvironmentLight>(assets + "/HDR_029_Sky_Cloudy_Env.hdr");
    scene->set_environment_light(env);
    auto sun = std::make_shared<DirectionalLight>(vec3(0.f, 2.f, 0.f), vec3(1.f, 0.9f, 0.8f));
    scene->add_light(sun);
    scene->add_light(sun);  // once only
    std::vector<float> dp;
    mcpt_scene_desc d = scene->desc(dp);
    CHECK(d.ntri == 960 && d.env_mode == 1 && d.env_w == 512 && d.env_h == 256 && d.ndir == 1);
    CHECK(d.dir_params[1] == 2.f && d.dir_params[3] == 1.f && d.dir_params[6] == 1.f);  // device dir as given
    auto st0 = scene->state();
    sun->set_dir(vec3(0.f, 3.f, 0.f));
    CHECK(sun->get_dir().y == 1.f);  // host copy normalised (DirectionalLight.cu:82-88)
    sun->set_ls(2.f);
    CHECK(scene->state() != st0);
    d = scene->desc(dp);
    CHECK(d.dir_params[1] == 3.f && d.dir_params[6] == 2.f);
    auto grey = std::make_shared<EnvironmentLight>(vec3(0.5f));
    grey->set_ls(3.f);
    scene->set_environment_light(grey);
    d = scene->desc(dp);
    CHECK(d.env_mode == 0 && d.env_color[0] == 0.5f && d.env_ls == 3.f && d.ntri == 960);
    scene->remove_light(sun);
    d = scene->desc(dp);
    CHECK(d.ndir == 0);

    // env texture reload: keyed on the light object and its texture revision, not the path
    {
        const std::string tmp = "/tmp/mcpt_facade_env_" + std::to_string((long)getpid()) + ".hdr";
        auto write_hdr = [&](int w, int h) {  // flat (width < 8) RGBE, all texels (128, 64, 32) e 129
            FILE* f = std::fopen(tmp.c_str(), "wb");
            std::fprintf(f, "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y %d +X %d\n", h, w);
            for (int i = 0; i < w * h; i++) std::fputc(128, f), std::fputc(64, f), std::fputc(32, f), std::fputc(129, f);
            std::fclose(f);
        };
        write_hdr(4, 2);
        auto e1 = std::make_shared<EnvironmentLight>(tmp);
        scene->set_environment_light(e1);
        d = scene->desc(dp);
        CHECK(d.env_mode == 1 && d.env_w == 4 && d.env_h == 2);
        write_hdr(6, 3);  // the file changes on disk
        e1->set_ls(2.f);  // not a texture edit: no re-read
        d = scene->desc(dp);
        CHECK(d.env_w == 4 && d.env_h == 2);
        e1->set_texture_filepath(tmp);  // the same path set again: re-read
        d = scene->desc(dp);
        CHECK(d.env_w == 6 && d.env_h == 3);
        write_hdr(2, 1);
        scene->set_environment_light(std::make_shared<EnvironmentLight>(tmp));  // another object, same path
        d = scene->desc(dp);
        CHECK(d.env_w == 2 && d.env_h == 1);
        // copies keep the original's light id: two copies re-pointed the same number of times at
        // different files must still reload when swapped
        {
            const std::string tmp2 = tmp + ".b.hdr";
            auto base = std::make_shared<EnvironmentLight>(tmp);
            auto ca = std::make_shared<EnvironmentLight>(*base), cb = std::make_shared<EnvironmentLight>(*base);
            CHECK(ca->get_id() == cb->get_id());
            write_hdr(4, 2);
            ca->set_texture_filepath(tmp);
            {
                FILE* f = std::fopen(tmp2.c_str(), "wb");
                std::fprintf(f, "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y %d +X %d\n", 5, 7);
                for (int i = 0; i < 35; i++) std::fputc(128, f), std::fputc(64, f), std::fputc(32, f), std::fputc(129, f);
                std::fclose(f);
            }
            cb->set_texture_filepath(tmp2);
            scene->set_environment_light(ca);
            d = scene->desc(dp);
            CHECK(d.env_w == 4 && d.env_h == 2);
            scene->set_environment_light(cb);
            d = scene->desc(dp);
            CHECK(d.env_w == 7 && d.env_h == 5);
            scene->set_environment_light(ca);
            d = scene->desc(dp);
            CHECK(d.env_w == 4 && d.env_h == 2);
            std::remove(tmp2.c_str());
        }
        std::remove(tmp.c_str());
        scene->set_environment_light(grey);
    }
    threw = false;
    try {
        grey->set_type(Atmosphere);
    } catch (const Error& e) {
        threw = e.code() == MCPT_E_INVALID;
    }
    CHECK(threw);
    threw = false;
    try {
        scene->load(assets + "/no_such_file.glb");
    } catch (const Error& e) {
        threw = e.code() == MCPT_E_IO;
    }
    CHECK(threw);

    // no gfx950 device here: the product refuses to start instead of falling back to the CPU
    threw = false;
    try {
        PathTracer pt(0);
    } catch (const Error& e) {
        threw = e.code() == MCPT_E_NODEVICE;
    }
    CHECK(threw);
    std::printf("facade cpu %s (%d failures)\n", g_fail ? "FAILED" : "ok", g_fail);
    return g_fail ? 1 : 0;
}

static int run_render(const std::string& assets, const std::string& out) {
    const uint32_t W = 32, H = 32;
    mcpt_config cfg = default_config();
    cfg.spp = 2;
    cfg.max_depth = 3;  // BASELINE config 1 depth
    PathTracer pt(0, cfg);
    auto scene = std::make_shared<Scene>();
    scene->load(assets + "/sphere.glb");
    scene->set_environment_light(std::make_shared<EnvironmentLight>(assets + "/HDR_029_Sky_Cloudy_Env.hdr"));
    auto camera = std::make_shared<PerspectiveCamera>(vec3(0.f, 0.f, 4.f), radians(45.f), 0.01f, 1e4f);
    camera->set_aspect_ratio((float)W / (float)H);
    auto film = std::make_shared<Film>();
    film->set_size(W, H);

    // the reference loop: render_image per displayed frame, one tile iteration per call
    uint64_t rays = 0;
    int calls = 0;
    for (; calls < 1000; calls++) {
        pt.render_image(scene, camera, film);
        const mcpt_stage_stats& s = pt.last_stats();
        rays += s.extend_rays + s.shadow_rays + s.vis_rays;
        if (s.extend_rays + s.shadow_rays + s.vis_rays == 0) break;
    }
    CHECK(calls < 1000 && rays > 0);
    const mcpt_camera cam0 = camera->get_dptr();  // the camera of this film (edited below)
    CHECK(film->get_image().size() == (size_t)W * H * 4);
    std::vector<float> Ld;
    std::vector<uint32_t> smp;
    pt.read_film(Ld, smp);
    for (uint32_t i = 0; i < W * H; i++) {
        const uint32_t x = i % W, y = i / W;
        CHECK(smp[i] == ((x == W - 1 || y == H - 1) ? 0u : 2u));  // last row/column never rendered (A.3)
    }

    // batch mode on a second film of the same size: bit-identical (tile-partition invariance)
    auto film2 = std::make_shared<Film>();
    film2->set_size(W, H);
    pt.render_frame(scene, camera, film2);
    std::vector<float> Ld2;
    std::vector<uint32_t> smp2;
    pt.read_film(Ld2, smp2);
    CHECK(smp2 == smp && std::memcmp(Ld2.data(), Ld.data(), Ld.size() * sizeof(float)) == 0);

    // observers: a camera edit clears the film (Film::update), so one call later a pixel has
    // at most one sample again; so does a light edit
    camera->set_position(vec3(0.f, 0.f, 4.5f));
    pt.render_image(scene, camera, film2);
    CHECK(film2->get_tile_x_pos() == 0);  // cleared to tile 0, then advanced (1 tile: back to 0)
    std::vector<float> Ld3;
    std::vector<uint32_t> smp3;
    for (int k = 0; k < 3; k++) pt.render_image(scene, camera, film2);
    pt.read_film(Ld3, smp3);
    uint32_t mx = 0;
    for (uint32_t v : smp3) mx = v > mx ? v : mx;
    CHECK(mx <= 2);
    scene->get_environment_light()->set_ls(2.f);
    pt.render_image(scene, camera, film2);
    pt.read_film(Ld3, smp3);
    mx = 0;
    for (uint32_t v : smp3) mx = v > mx ? v : mx;
    CHECK(mx == 0);  // one iteration after a clear: no sample has finished yet

    FILE* f = std::fopen(out.c_str(), "wb");
    if (!f) return 2;
    const uint32_t hdr[4] = {W, H, 2u, 3u};
    std::fwrite(hdr, 4, 4, f);
    std::fwrite(&cam0, sizeof(mcpt_camera), 1, f);
    std::fwrite(Ld.data(), sizeof(float), Ld.size(), f);
    std::fwrite(smp.data(), sizeof(uint32_t), smp.size(), f);
    std::fclose(f);
    std::printf("facade render %s: %s, %d calls, %llu rays (%d failures)\n", g_fail ? "FAILED" : "ok",
                pt.device_name().c_str(), calls, (unsigned long long)rays, g_fail);
    return g_fail ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s cpu <assets> | render <assets> <out.bin>\n", argv[0]);
        return 2;
    }
    try {
        if (!std::strcmp(argv[1], "cpu")) return run_cpu(argv[2]);
        if (!std::strcmp(argv[1], "render") && argc > 3) return run_render(argv[2], argv[3]);
    } catch (const Error& e) {
        std::fprintf(stderr, "mcpt::Error %d: %s\n", e.code(), e.what());
        return 1;
    }
    return 2;
}
