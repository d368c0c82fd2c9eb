// Sanitizer driver (TEST INFRASTRUCTURE: compiled and run by tests/test_sanitizers.py with
// -fsanitize=address,undefined and, separately, -fsanitize=thread; the product never uses it).
// Exercises the host code of libpt (host/pt_host.cpp: scene presets, OBJ loading, Morton keys,
// quantisation, PNG writing; host/pt_wide8.cpp: the 16-thread binned-SAH wide build) and the CPU
// restatement (oracle/pt_oracle.cpp: LBVH, closest hits, threaded compat and sample-mode renders)
// on the BASELINE scenes at small frame sizes.  SURVEY §5 asks for ASan/UBSan on the CPU build and
// TSan on its threaded code.  usage: sanitize_main models_dir out_dir [light]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pt.h"
#include "pt_oracle.h"
#include "pt_wide8.hpp"

namespace {
int failures = 0;
void check(bool ok, const char* what) {
    if (!ok) {
        std::fprintf(stderr, "CHECK FAILED: %s\n", what);
        failures++;
    }
}

// The wide build's inputs from the oracle's LBVH, as the device's leafGatherKernel writes them.
void wideBuild(const pt_object* objs, int64_t n, const std::vector<uint64_t>& keys, const std::vector<orc_node>& nd) {
    std::vector<uint32_t> prims((size_t)n * pt::kW8PrimDwords, 0u);
    std::vector<float> boxes((size_t)n * 6);
    for (int64_t k = 0; k < n; k++) {
        const pt_object& o = objs[keys[(size_t)k] & 0xffffffffu];
        uint32_t* r = &prims[(size_t)k * 12];
        float* f = reinterpret_cast<float*>(r);
        float* b = &boxes[(size_t)k * 6];
        r[3] = (uint32_t)o.mat;
        r[7] = (uint32_t)(keys[(size_t)k] & 0xffffffffu);
        if (o.type == PT_SPHERE) {
            f[0] = o.v[0]; f[1] = o.v[1]; f[2] = o.v[2]; f[4] = o.v[3]; r[11] = 1u;
            const float rr = std::fabs(o.v[3]);
            for (int a = 0; a < 3; a++) { b[a] = o.v[a] - rr; b[3 + a] = o.v[a] + rr; }
        } else {
            for (int v = 0; v < 3; v++)
                for (int a = 0; a < 3; a++) f[4 * v + a] = o.v[3 * v + a];
            for (int a = 0; a < 3; a++) {
                b[a] = std::fmin(std::fmin(o.v[a], o.v[3 + a]), o.v[6 + a]);
                b[3 + a] = std::fmax(std::fmax(o.v[a], o.v[3 + a]), o.v[6 + a]);
            }
        }
    }
    std::vector<uint32_t> lref((size_t)(n > 1 ? n - 1 : 1)), rref(lref.size());
    for (int64_t i = 0; i + 1 < n; i++) {
        auto ref = [&](int32_t c) { return c >= n - 1 ? (0x80000000u | (uint32_t)(c - (n - 1))) : (uint32_t)c; };
        lref[(size_t)i] = ref(nd[(size_t)i].left);
        rref[(size_t)i] = ref(nd[(size_t)i].right);
    }
    const std::vector<uint32_t> rank = pt::referenceRanks(lref.data(), rref.data(), 1, n);
    pt::Wide8 w;
    std::string err;
    check(pt::buildWide8(prims.data(), boxes.data(), rank.data(), n, w, err), "buildWide8");
    check(w.depth > 0 && w.usedNodes > 0, "wide tree non-empty");
}

void scene(const char* name, const char* models, const std::string& outDir, bool light) {
    pt_scene_desc d{};
    const int w = 32, h = 18;
    check(pt_preset_scene(name, models, w, h, &d) == PT_OK, "pt_preset_scene");
    const int64_t n = d.n_objects;
    const auto* objs = reinterpret_cast<const orc_object*>(d.objects);
    const auto* mats = reinterpret_cast<const orc_material*>(d.materials);
    const auto* cam = reinterpret_cast<const orc_camera*>(&d.camera);
    // Morton keys: host (libpt) and oracle agree
    std::vector<uint64_t> keys((size_t)n), okeys((size_t)n);
    check(pt_morton_keys(d.objects, n, 1, keys.data()) == PT_OK, "pt_morton_keys");
    check(orc_morton_keys(objs, n, 1, okeys.data()) == 0, "orc_morton_keys");
    check(keys == okeys, "Morton keys equal");
    std::vector<orc_node> nodes((size_t)(2 * n - 1)), refNodes(nodes.size());
    check(orc_build_lbvh(objs, n, okeys.data(), 1, nodes.data()) == 0, "orc_build_lbvh tight");
    check(orc_build_lbvh(objs, n, okeys.data(), 0, refNodes.data()) == 0, "orc_build_lbvh reference boxes");
    check(orc_bvh_depth(nodes.data(), n) > 0 || n == 1, "depth");
    // closest hits from the camera through the frame, BVH and brute force
    std::vector<float> rays;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const float u = (x + 0.5f) / w, v = (y + 0.5f) / h;
            float dir[3];
            for (int a = 0; a < 3; a++)
                dir[a] = d.camera.lower_left[a] + u * d.camera.horizontal[a] + v * d.camera.vertical[a] - d.camera.origin[a];
            rays.insert(rays.end(), {d.camera.origin[0], d.camera.origin[1], d.camera.origin[2], dir[0], dir[1], dir[2]});
        }
    const int64_t nr = (int64_t)rays.size() / 6;
    std::vector<orc_hit> hb((size_t)nr), hf((size_t)nr);
    orc_stats st{};
    check(orc_trace(objs, n, nodes.data(), rays.data(), nr, 0.001f, INFINITY, 0, hb.data(), &st) == 0, "orc_trace");
    if (n <= 20000)
        check(orc_trace(objs, n, nodes.data(), rays.data(), nr, 0.001f, INFINITY, 1, hf.data(), &st) == 0, "brute");
    // threaded renders: compat (per-pixel XORWOW) and sample mode
    std::vector<int32_t> rows((size_t)h);
    for (int r = 0; r < h; r++) rows[(size_t)r] = r;
    std::vector<uint32_t> states((size_t)w * h * 6);
    orc_xorwow_init_range(1, 0, (int64_t)w * h, states.data());
    std::vector<float> rgb((size_t)w * h * 3), srgb(rgb.size());
    const int spp = light ? 1 : 2;
    check(orc_render(objs, n, mats, d.n_materials, nodes.data(), cam, w, h, rows.data(), h, spp, d.max_depth,
                     states.data(), rgb.data(), &st, 4) == 0, "orc_render");
    check(orc_render_sample(objs, n, mats, d.n_materials, nodes.data(), cam, w, h, rows.data(), h, spp, d.max_depth,
                            3, 2, srgb.data(), &st, 4) == 0, "orc_render_sample");
    // quantise + PNG (host)
    std::vector<uint8_t> rgba((size_t)w * h * 4);
    check(pt_quantize_rgba8(rgb.data(), w, h, rgba.data()) == PT_OK, "pt_quantize_rgba8");
    const std::string png = outDir + "/" + name + ".png";
    check(pt_write_png(png.c_str(), rgb.data(), w, h) == PT_OK, "pt_write_png");
    check(pt_write_png_rgba8(png.c_str(), rgba.data(), w, h) == PT_OK, "pt_write_png_rgba8");
    // the host wide build (threads)
    if (!light || n < 20000) wideBuild(d.objects, n, okeys, nodes);
    pt_scene_desc_free(&d);
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const char* models = argv[1];
    const std::string out = argv[2];
    const bool light = argc > 3;   // (TSan: ~10x slower; the 1M-primitive field is skipped)
    for (const char* name : {"rtiow", "triangle_world", "random_world", "test_world", "cornell", "bunny_cornell"})
        scene(name, models, out, light);
    if (!light) scene("bunny_field", models, out, light);
    // OBJ loading and camera movement (host surface)
    pt_object* objs = nullptr;
    int64_t count = 0;
    const float t[3] = {0.0f, 0.0f, 0.0f};
    const std::string bunny = std::string(models) + "/bunny/bunny.obj";
    check(pt_load_obj(bunny.c_str(), 1500.0f, t, 0, &objs, &count) == PT_OK && count == 4968, "pt_load_obj");
    pt_free(objs);
    check(pt_load_obj("/nonexistent.obj", 1.0f, t, 0, &objs, &count) != PT_OK, "missing OBJ fails");
    pt_camera cam;
    const float from[3] = {278, 273, -800}, at[3] = {278, 273, 0};
    check(pt_camera_make(from, at, 40.0f, 1.0f, 0.0f, 10.0f, 0.0f, 1.0f, &cam) == PT_OK, "pt_camera_make");
    for (int k = 0; k < 12; k++) check(pt_camera_move(&cam, k % 6, 0.1f) == PT_OK, "pt_camera_move");
    std::printf(failures ? "FAILED %d\n" : "ok\n", failures);
    return failures ? 1 : 0;
}
