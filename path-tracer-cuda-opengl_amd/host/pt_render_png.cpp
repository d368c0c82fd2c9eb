// pt_render_png — command-line renderer, the counterpart of the reference's main() ->
// renderToPng() (main.cu:462-487, 530-535): build a scene, build the LBVH, initialise the
// per-pixel RNG streams, render, quantise and write a PNG.  Runtime flags replace the
// reference's compile-time constants (global_variables.h:28-35, macros.h:8-12).
// With --gpus N the frame is split into interleaved row stripes, one host thread per GPU.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "pt.h"

static void usage() {
    std::fprintf(stderr,
                 "usage: pt_render_png [--scene NAME] [--models DIR] [--width W] [--height H] [--spp N]\n"
                 "                     [--depth D] [--seed S] [--gpus N] [--stripe ROWS] [--out FILE]\n"
                 "                     [--rng compat|sample] [--frames K]\n"
                 "--frames K: progressive rendering, K frames of --spp samples accumulated per pixel (the\n"
                 "            headless counterpart of the reference's interactive loop); PNG of the last one\n"
                 "scenes: triangle_world (default, as the reference), random_world, test_world, rtiow,\n"
                 "        cornell, bunny_cornell, bunny_field\n");
}

#define CHECK(x)                                                                      \
    do {                                                                              \
        int _rc = (x);                                                                \
        if (_rc != PT_OK) {                                                           \
            std::fprintf(stderr, "%s failed (%d): %s\n", #x, _rc, pt_last_error());   \
            std::exit(99);                                                            \
        }                                                                             \
    } while (0)

int main(int argc, char** argv) {
    std::string scene = "triangle_world", models = "models", out = "debug.png";
    int width = 0, height = 0, spp = -1, depth = -1, gpus = 1, stripe = 8, frames = 1, rng = PT_RNG_COMPAT;
    unsigned long long seed = 1;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { usage(); std::exit(2); }
            return argv[++i];
        };
        if (a == "--scene") scene = next();
        else if (a == "--models") models = next();
        else if (a == "--width") width = std::atoi(next());
        else if (a == "--height") height = std::atoi(next());
        else if (a == "--spp") spp = std::atoi(next());
        else if (a == "--depth") depth = std::atoi(next());
        else if (a == "--seed") seed = std::strtoull(next(), nullptr, 10);
        else if (a == "--gpus") gpus = std::atoi(next());
        else if (a == "--stripe") stripe = std::atoi(next());
        else if (a == "--out") out = next();
        else if (a == "--frames") frames = std::atoi(next());
        else if (a == "--rng") {
            std::string r = next();
            if (r == "compat") rng = PT_RNG_COMPAT;
            else if (r == "sample") rng = PT_RNG_SAMPLE;
            else { usage(); return 2; }
        }
        else { usage(); return 2; }
    }
    pt_scene_desc d;
    CHECK(pt_preset_scene(scene.c_str(), models.c_str(), width, height, &d));
    if (spp > 0) d.spp = spp;
    if (depth >= 0) d.max_depth = depth;
    int ndev = 0;
    CHECK(pt_device_count(&ndev));
    if (ndev <= 0) { std::fprintf(stderr, "no GPU visible\n"); return 99; }
    if (gpus > ndev) gpus = ndev;
    std::printf("scene %s: %lld objects, %dx%d @%dspp depth %d on %d GPU(s)\n", d.name, (long long)d.n_objects,
                d.width, d.height, d.spp, d.max_depth, gpus);

    if (frames < 1) frames = 1;
    // The frame is quantised on the device (PT_OUT_RGBA8: PngImage::saveColor per pixel), so each
    // GPU hands back 4 bytes per pixel of its row stripes.
    std::vector<uint8_t> frame((size_t)d.width * d.height * 4);
    std::vector<pt_stats> stats(gpus);
    std::vector<double> kms(gpus, 0.0);
    std::vector<std::thread> th;
    auto t0 = std::chrono::steady_clock::now();
    for (int g = 0; g < gpus; g++) {
        th.emplace_back([&, g]() {
            pt_scene* s = nullptr;
            pt_film* f = nullptr;
            CHECK(pt_scene_create(g, d.objects, d.n_objects, d.materials, d.n_materials, &s));
            CHECK(pt_scene_build_bvh(s, PT_BVH_ORIGIN_BOUNDS));
            CHECK(pt_film_create(g, d.width, d.height, stripe, gpus, g, seed, &f));
            int nrows = 0;
            int64_t npix = 0;
            CHECK(pt_film_info(f, &nrows, &npix));
            std::vector<int32_t> rows(nrows);
            CHECK(pt_film_rows(f, rows.data()));
            std::vector<uint8_t> part((size_t)npix * 4);
            pt_render_opts o{};
            o.rng = rng;
            o.out_format = PT_OUT_RGBA8;
            o.flags = frames > 1 ? PT_RENDER_ACCUMULATE : 0;
            pt_stats st{};
            for (int k = 0; k < frames; k++) {
                CHECK(pt_render_ex(s, f, &d.camera, d.spp, d.max_depth, reinterpret_cast<float*>(part.data()), 0,
                                   nullptr, &o, &st));
                kms[g] += st.kernel_ms;
                stats[g].rays += st.rays;
                if (frames > 1 && g == 0)
                    std::printf("frame %d: %d spp accumulated, %.2f ms kernel on GPU 0\n", k + 1, (k + 1) * d.spp,
                                st.kernel_ms);
            }
            for (int r = 0; r < nrows; r++)
                std::memcpy(&frame[(size_t)rows[r] * d.width * 4], &part[(size_t)r * d.width * 4], 4 * (size_t)d.width);
            pt_film_destroy(f);
            pt_scene_destroy(s);
        });
    }
    for (auto& t : th) t.join();
    double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    unsigned long long rays = 0;
    double kmax = 0;
    for (int g = 0; g < gpus; g++) {
        rays += stats[g].rays;
        kmax = kms[g] > kmax ? kms[g] : kmax;
    }
    std::printf("Time Cost: %.3f s kernel (max over GPUs), %.3f s wall incl. setup; %.1f Mray/s\n", kmax / 1e3, wall,
                rays / (kmax * 1e3));
    CHECK(pt_write_png_rgba8(out.c_str(), frame.data(), d.width, d.height));
    pt_scene_desc_free(&d);
    return 0;
}
