// pt_host.cpp — host-side surface: camera, PNG, OBJ, scene builders, Morton keys, and the
// host-only entry points of include/pt.h.  No GPU is touched here.
#include "pt_host.hpp"

#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>

#include "pt_error.hpp"

namespace pt {

// ------------------------------------------------------------------------ camera
camera::camera(point3 lookFrom, point3 lookAt, float vfov, float aspect_ratio, float aperture, float focus_dist,
               float t0, float t1) {
    const float kDegToRad = 0.01745329252f;              // global_variables.h:20
    float theta = vfov * kDegToRad;                       // utility.h:28-30
    float h = std::tan(theta / 2.0f);
    float viewport_height = 2.0f * h;
    float viewport_width = aspect_ratio * viewport_height;
    mFront = normalize(lookFrom - lookAt);
    mRight = normalize(cross(vec3(0, 1, 0), mFront));
    mUp = cross(mFront, mRight);
    mPosition = lookFrom;
    mHorizontalViewportSize = (focus_dist * viewport_width) * mRight;
    mVerticalViewportSize = (focus_dist * viewport_height) * mUp;
    mViewportLowLeftCorner =
        ((mPosition - mHorizontalViewportSize / 2.0f) - mVerticalViewportSize / 2.0f) - focus_dist * mFront;
    mLensRadius = aperture / 2.0f;
    time0 = t0;
    time1 = t1;
    mFocusDist = focus_dist;
}

void camera::processKeyboard(directions dir, float deltaTime) {   // camera.h:41-56
    const float kCameraSpeed = 2.5f;                                 // global_variables.h:36
    float velocity = kCameraSpeed * deltaTime;
    if (dir == FORWARD) mPosition -= mFront * velocity;
    if (dir == BACKWARD) mPosition += mFront * velocity;
    if (dir == LEFT) mPosition -= mRight * velocity;
    if (dir == RIGHT) mPosition += mRight * velocity;
    if (dir == UP) mPosition += mUp * velocity;
    if (dir == DOWN) mPosition -= mUp * velocity;
    mViewportLowLeftCorner =
        ((mPosition - mHorizontalViewportSize / 2.0f) - mVerticalViewportSize / 2.0f) - mFocusDist * mFront;
}

static void put3(float* d, const vec3& v) { d[0] = v.e[0]; d[1] = v.e[1]; d[2] = v.e[2]; }
static vec3 get3(const float* s) { return {s[0], s[1], s[2]}; }

pt_camera camera::abi() const {
    pt_camera c{};
    put3(c.origin, mPosition);
    put3(c.lower_left, mViewportLowLeftCorner);
    put3(c.horizontal, mHorizontalViewportSize);
    put3(c.vertical, mVerticalViewportSize);
    put3(c.right, mRight);
    put3(c.up, mUp);
    put3(c.front, mFront);
    c.focus_dist = mFocusDist;
    c.lens_radius = mLensRadius;
    c.time0 = time0;
    c.time1 = time1;
    return c;
}

// ---------------------------------------------------------------------- PngImage
PngImage::PngImage(int w, int h, int n) : mData((size_t)w * h * n, 0), mDataW(w), mDataH(h), mDataN(n) {}

static inline float clampf(float x, float lo, float hi) {   // utility.h:40-44
    if (x < lo) return lo;
    if (x > hi) return hi;
    return x;
}

void PngImage::saveColor(color clr, int row, int col, int spp) {   // png_image.h:24-30
    float crate = 1.0f / (float)spp;
    uint8_t* p = mData.data() + ((size_t)row * mDataW + col) * mDataN;
    p[0] = (uint8_t)(clampf(clr.x() * crate, 0.0f, 0.999f) * 256.0f);
    p[1] = (uint8_t)(clampf(clr.y() * crate, 0.0f, 0.999f) * 256.0f);
    p[2] = (uint8_t)(clampf(clr.z() * crate, 0.0f, 0.999f) * 256.0f);
    if (mDataN > 3) p[3] = 255;   // alpha_scale 255.999 -> 255
}

static void pngChunk(std::string& out, const char* type, const uint8_t* data, size_t len) {
    uint8_t be[4] = {(uint8_t)(len >> 24), (uint8_t)(len >> 16), (uint8_t)(len >> 8), (uint8_t)len};
    out.append((const char*)be, 4);
    out.append(type, 4);
    if (len) out.append((const char*)data, len);
    uLong crc = crc32(0L, (const Bytef*)type, 4);
    if (len) crc = crc32(crc, data, (uInt)len);
    uint8_t c[4] = {(uint8_t)(crc >> 24), (uint8_t)(crc >> 16), (uint8_t)(crc >> 8), (uint8_t)crc};
    out.append((const char*)c, 4);
}

bool PngImage::write(const char* filename) const {   // stbi_write_png(filename, w, h, n, data, w*4)
    const size_t stride = (size_t)mDataW * mDataN;
    std::vector<uint8_t> raw((stride + 1) * mDataH);
    for (int y = 0; y < mDataH; y++) {
        raw[y * (stride + 1)] = 0;   // filter: none
        std::memcpy(&raw[y * (stride + 1) + 1], &mData[y * stride], stride);
    }
    uLongf zlen = compressBound(raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), raw.size(), 6) != Z_OK) return false;
    std::string png("\x89PNG\r\n\x1a\n", 8);
    uint8_t ihdr[13] = {(uint8_t)(mDataW >> 24), (uint8_t)(mDataW >> 16), (uint8_t)(mDataW >> 8), (uint8_t)mDataW,
                        (uint8_t)(mDataH >> 24), (uint8_t)(mDataH >> 16), (uint8_t)(mDataH >> 8), (uint8_t)mDataH,
                        8, (uint8_t)(mDataN == 4 ? 6 : (mDataN == 3 ? 2 : 0)), 0, 0, 0};
    pngChunk(png, "IHDR", ihdr, 13);
    pngChunk(png, "IDAT", z.data(), zlen);
    pngChunk(png, "IEND", nullptr, 0);
    FILE* f = std::fopen(filename, "wb");
    if (!f) return false;
    bool ok = std::fwrite(png.data(), 1, png.size(), f) == png.size();
    return std::fclose(f) == 0 && ok;
}

// ------------------------------------------------------------------------ OBJ loader
bool objl::Loader::LoadFile(const std::string& path) {
    std::ifstream in(path);
    if (!in) return false;
    LoadedMeshes.clear();
    LoadedVertices.clear();
    LoadedIndices.clear();
    std::vector<Vector3> pos, nrm;
    std::vector<Vector2> tc;
    Mesh cur;
    auto flush = [&]() {
        if (!cur.Indices.empty() && !cur.Vertices.empty()) LoadedMeshes.push_back(cur);
        cur = Mesh();
    };
    auto resolve = [](long idx, size_t n) -> long { return idx < 0 ? (long)n + idx : idx - 1; };
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string tag;
        if (!(ls >> tag)) continue;
        if (tag == "v" || tag == "vn") {
            std::string a, b, c;
            ls >> a >> b >> c;
            Vector3 v{std::strtof(a.c_str(), nullptr), std::strtof(b.c_str(), nullptr), std::strtof(c.c_str(), nullptr)};
            (tag == "v" ? pos : nrm).push_back(v);
        } else if (tag == "vt") {
            std::string a, b;
            ls >> a >> b;
            tc.push_back({std::strtof(a.c_str(), nullptr), std::strtof(b.c_str(), nullptr)});
        } else if (tag == "o" || tag == "g") {
            flush();
            std::getline(ls >> std::ws, cur.MeshName);
        } else if (tag == "f") {
            std::vector<Vertex> face;
            std::string tok;
            while (ls >> tok) {
                Vertex vx;
                long vi = 0, ti = 0, ni = 0;
                int parts = std::sscanf(tok.c_str(), "%ld/%ld/%ld", &vi, &ti, &ni);
                if (parts < 3 && std::sscanf(tok.c_str(), "%ld//%ld", &vi, &ni) == 2) parts = 3, ti = 0;
                if (parts < 1) return false;
                long p = resolve(vi, pos.size());
                if (p < 0 || (size_t)p >= pos.size()) return false;
                vx.Position = pos[p];
                if (ti) { long t = resolve(ti, tc.size()); if (t >= 0 && (size_t)t < tc.size()) vx.TextureCoordinate = tc[t]; }
                if (ni) { long q = resolve(ni, nrm.size()); if (q >= 0 && (size_t)q < nrm.size()) vx.Normal = nrm[q]; }
                face.push_back(vx);
            }
            if (face.size() < 3) continue;
            unsigned base = (unsigned)cur.Vertices.size(), gbase = (unsigned)LoadedVertices.size();
            for (auto& v : face) { cur.Vertices.push_back(v); LoadedVertices.push_back(v); }
            for (size_t i = 1; i + 1 < face.size(); i++) {
                for (unsigned k : {0u, (unsigned)i, (unsigned)i + 1}) {
                    cur.Indices.push_back(base + k);
                    LoadedIndices.push_back(gbase + k);
                }
            }
        }
    }
    flush();
    return !LoadedMeshes.empty();
}

// -------------------------------------------------------------------- builders
pt_material lambertian(const color& a) {
    pt_material m{};
    m.type = PT_LAMBERTIAN;
    put3(m.albedo, a);
    return m;
}
pt_material metal(const color& a, float f) {
    pt_material m{};
    m.type = PT_METAL;
    put3(m.albedo, a);
    m.fuzz = f < 1 ? f : 1;
    return m;
}
pt_material dielectric(float ir) {
    pt_material m{};
    m.type = PT_DIELECTRIC;
    m.ir = ir;
    return m;
}
pt_object sphere(const point3& c, float r, int mat) {
    pt_object o{};
    o.type = PT_SPHERE;
    o.mat = mat;
    put3(o.v, c);
    o.v[3] = r;
    return o;
}
pt_object triangle(const point3& v0, const point3& v1, const point3& v2, int mat) {
    pt_object o{};
    o.type = PT_TRIANGLE;
    o.mat = mat;
    put3(o.v, v0);
    put3(o.v + 3, v1);
    put3(o.v + 6, v2);
    return o;
}

static size_t appendMeshes(Scene& s, const objl::Loader& ld, float scale, const vec3& t, int mat);
size_t appendObj(Scene& s, const std::string& path, float scale, const vec3& t, int mat) {
    objl::Loader ld;
    if (!ld.LoadFile(path)) throw std::runtime_error("cannot load OBJ " + path);
    return appendMeshes(s, ld, scale, t, mat);
}
// one parsed OBJ placed many times (the bunny fields): parsed once
static const objl::Loader& loadOnce(std::unique_ptr<objl::Loader>& ld, const std::string& path) {
    if (!ld) {
        ld.reset(new objl::Loader());
        if (!ld->LoadFile(path)) throw std::runtime_error("cannot load OBJ " + path);
    }
    return *ld;
}
static size_t appendMeshes(Scene& s, const objl::Loader& ld, float scale, const vec3& t, int mat) {
    size_t added = 0;
    for (const auto& m : ld.LoadedMeshes) {
        for (size_t i = 0; i + 2 < m.Indices.size(); i += 3) {
            vec3 v[3];
            for (int k = 0; k < 3; k++) {
                const auto& p = m.Vertices[m.Indices[i + k]].Position;
                v[k] = vec3(p.X * scale + t.x(), p.Y * scale + t.y(), p.Z * scale + t.z());
            }
            s.objects.push_back(triangle(v[0], v[1], v[2], mat));
            added++;
        }
    }
    return added;
}

static void cornellBox(Scene& s, const std::string& dir) {
    // Build-chosen materials (the reference ships geometry only).
    int white = (int)s.materials.size();
    s.materials.push_back(lambertian(color(0.725f, 0.71f, 0.68f)));
    int red = (int)s.materials.size();
    s.materials.push_back(lambertian(color(0.63f, 0.065f, 0.05f)));
    int green = (int)s.materials.size();
    s.materials.push_back(lambertian(color(0.14f, 0.45f, 0.091f)));
    const vec3 zero(0, 0, 0);
    appendObj(s, dir + "/cornellbox/floor.obj", 1.0f, zero, white);
    appendObj(s, dir + "/cornellbox/left.obj", 1.0f, zero, red);
    appendObj(s, dir + "/cornellbox/right.obj", 1.0f, zero, green);
    appendObj(s, dir + "/cornellbox/light.obj", 1.0f, zero, white);
    appendObj(s, dir + "/cornellbox/shortbox.obj", 1.0f, zero, white);
    appendObj(s, dir + "/cornellbox/tallbox.obj", 1.0f, zero, white);
}

static float aspectOf(int w, int h) { return (float)w / (float)h; }

Scene buildPreset(const std::string& name, const std::string& dir, int width, int height) {
    Scene s;
    s.name = name;
    auto frame = [&](int w, int h, int spp, int depth) {
        s.width = width > 0 ? width : w;
        s.height = height > 0 ? height : h;
        s.spp = spp;
        s.max_depth = depth;
    };
    if (name == "triangle_world") {                       // main.cu:119-196, camera main.cu:438-442
        frame(800, 450, 100, 50);
        HostRng rng;
        const int total = 600;
        const float radius = 10;
        for (int i = 0; i < total; i++) {
            float choose = rng.uniform() * 2;
            point3 center = rng.inUnitSphereDiscard() * radius;
            vec3 r1 = rng.vec3_args();
            vec3 r2 = rng.vec3_args();
            if (choose < 1) {
                s.objects.push_back(sphere(center, 0.5f, (int)s.materials.size()));
                if (choose < 0.6) s.materials.push_back(lambertian(r1 * r2));
                else if (choose < 0.9) s.materials.push_back(metal(r1 / 2.0f + vec3(0.5f, 0.5f, 0.5f), r2.x() / 2.0f));
                else s.materials.push_back(dielectric(1.5f));
            } else {
                point3 v0 = rng.inUnitSphereDiscard() + center;
                point3 v1 = rng.inUnitSphereDiscard() + center;
                point3 v2 = rng.inUnitSphereDiscard() + center;
                s.objects.push_back(triangle(v0, v1, v2, (int)s.materials.size()));
                if (choose < 1.6) s.materials.push_back(lambertian(r1 * r2));
                else if (choose < 1.9) s.materials.push_back(metal(r1 / 2.0f + vec3(0.5f, 0.5f, 0.5f), r2.x() / 2.0f));
                else s.materials.push_back(dielectric(1.5f));
            }
        }
        s.objects.push_back(sphere(point3(0, 0, -1010), 1000.0f, (int)s.materials.size()));
        s.materials.push_back(lambertian(color(0.5f, 0.5f, 0.5f)));
        s.cam = camera(vec3(0, 0, 25), vec3(0, 0, 0), 40, 16.0f / 9.0f, 0, 10, 0.0f, 1.0f).abi();
    } else if (name == "random_world") {                  // main.cu:198-256, camera main.cu:412-416
        frame(800, 450, 100, 50);
        HostRng rng;
        s.objects.push_back(sphere(point3(0, -1000, 0), 1000.0f, (int)s.materials.size()));
        s.materials.push_back(lambertian(color(0.5f, 0.5f, 0.5f)));
        for (int i = -10; i < 10; i++) {
            for (int j = -10; j < 10; j++) {
                float choose = rng.uniform();
                point3 center((float)i, 0.2f, (float)j);
                vec3 r1 = rng.vec3_args();
                vec3 r2 = rng.vec3_args();
                s.objects.push_back(sphere(center, 0.2f, (int)s.materials.size()));
                if (choose < 0.8) s.materials.push_back(lambertian(r1 * r2));
                else if (choose < 0.95) s.materials.push_back(metal(r1 / 2.0f + vec3(0.5f, 0.5f, 0.5f), r2.x() / 2.0f));
                else s.materials.push_back(dielectric(1.5f));
            }
        }
        s.objects.push_back(sphere(point3(4, 1, 0), 1.0f, (int)s.materials.size()));
        s.objects.push_back(sphere(point3(4, 1, 0), -0.9f, (int)s.materials.size()));
        s.materials.push_back(dielectric(1.5f));
        s.objects.push_back(sphere(point3(-4, 1, 0), 1.0f, (int)s.materials.size()));
        s.materials.push_back(lambertian(color(1, 0, 0.4f)));
        s.objects.push_back(sphere(point3(0, 1, 0), 1.0f, (int)s.materials.size()));
        s.materials.push_back(metal(color(0.7f, 0.6f, 0.5f), 0.0f));
        s.cam = camera(vec3(0, 30, 0.1f), vec3(0, 0, 0), 20, 16.0f / 9.0f, 0, 10, 0.0f, 1.0f).abi();
    } else if (name == "test_world") {                    // main.cu:57-117, camera main.cu:430-434
        frame(800, 450, 100, 50);
        s.objects.push_back(triangle(vec3(0, -2, 0), vec3(1, 0, 5), vec3(0, 2, 0), (int)s.materials.size()));
        s.materials.push_back(metal(color(0.7f, 0.6f, 0.5f), 0));
        s.objects.push_back(triangle(vec3(0, -2, 0), vec3(-1, 0, 5), vec3(0, 2, 0), (int)s.materials.size()));
        s.materials.push_back(metal(color(0.7f, 0.6f, 0.5f), 0));
        s.objects.push_back(sphere(point3(1005, 0, 0), 1000.0f, (int)s.materials.size()));
        s.materials.push_back(lambertian(color(0, 0, 1)));
        s.cam = camera(vec3(0, 0, 15), vec3(0, 0, 0), 20, 16.0f / 9.0f, 0, 10, 0.0f, 1.0f).abi();
    } else if (name == "rtiow") {                         // C1: ground + the three big spheres of main.cu:231-242
        frame(400, 225, 8, 50);
        s.objects.push_back(sphere(point3(0, -1000, 0), 1000.0f, (int)s.materials.size()));
        s.materials.push_back(lambertian(color(0.5f, 0.5f, 0.5f)));
        s.objects.push_back(sphere(point3(4, 1, 0), 1.0f, (int)s.materials.size()));
        s.objects.push_back(sphere(point3(4, 1, 0), -0.9f, (int)s.materials.size()));
        s.materials.push_back(dielectric(1.5f));
        s.objects.push_back(sphere(point3(-4, 1, 0), 1.0f, (int)s.materials.size()));
        s.materials.push_back(lambertian(color(1, 0, 0.4f)));
        s.objects.push_back(sphere(point3(0, 1, 0), 1.0f, (int)s.materials.size()));
        s.materials.push_back(metal(color(0.7f, 0.6f, 0.5f), 0.0f));
        s.cam = camera(vec3(13, 2, 3), vec3(0, 0, 0), 20, aspectOf(s.width, s.height), 0, 10, 0.0f, 1.0f).abi();
    } else if (name == "cornell" || name == "bunny_cornell" || name == "bunny_field" || name == "bunny_field_x4") {
        if (name == "cornell") frame(800, 800, 256, 8);
        else if (name == "bunny_cornell") frame(1920, 1080, 1024, 50);
        else if (name == "bunny_field_x4") frame(1920, 1080, 128, 16);
        else frame(1920, 1080, 512, 16);
        cornellBox(s, dir);
        const int white = 0;
        if (name == "bunny_cornell") {
            // Build-chosen placement: x1500, resting on the floor in the free front-right
            // region (clear of both boxes), facing the open side of the box.
            appendObj(s, dir + "/bunny/bunny.obj", 1500.0f, vec3(438.0f, -49.96f, 113.0f), white);
        } else if (name == "bunny_field") {
            // 15 x 14 = 210 instances at x250 on the floor: 210 * 4968 + 32 = 1,043,312 triangles.
            std::unique_ptr<objl::Loader> ld;
            for (int i = 0; i < 15; i++)
                for (int j = 0; j < 14; j++)
                    appendMeshes(s, loadOnce(ld, dir + "/bunny/bunny.obj"), 250.0f,
                                 vec3(24.0f + 35.5f * (float)i, -8.33f, 16.0f + 38.0f * (float)j), white);
        } else if (name == "bunny_field_x4") {
            // C5 at 4x the triangles (an HBM-resident stress case beyond the BASELINE configs): the same
            // floor covered by 30 x 28 = 840 half-size bunnies (x125, half the spacing),
            // 840 * 4968 + 32 = 4,173,152 triangles -- a flattened tree and records well beyond the
            // 256 MB Infinity Cache
            std::unique_ptr<objl::Loader> ld;
            for (int i = 0; i < 30; i++)
                for (int j = 0; j < 28; j++)
                    appendMeshes(s, loadOnce(ld, dir + "/bunny/bunny.obj"), 125.0f,
                                 vec3(12.0f + 17.75f * (float)i, -4.165f, 8.0f + 19.0f * (float)j), white);
        }
        s.cam = camera(vec3(278, 273, -800), vec3(278, 273, 0), 40, aspectOf(s.width, s.height), 0, 10, 0.0f,
                       1.0f).abi();
    } else {
        throw std::runtime_error("unknown preset '" + name + "'");
    }
    return s;
}

// ------------------------------------------------------------------------ Morton keys
static uint32_t expandBits(uint32_t v) {   // morton_code.h:19-27
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

struct HBox { vec3 mn, mx; };

static HBox objBox(const pt_object& o) {   // cuda_object.h:21-42
    if (o.type == PT_SPHERE) {
        vec3 c = get3(o.v);
        float r = std::fabs(o.v[3]);
        return {c - vec3(r, r, r), c + vec3(r, r, r)};
    }
    vec3 mn = get3(o.v), mx = mn;
    for (int k = 1; k < 3; k++) {
        vec3 p = get3(o.v + 3 * k);
        for (int a = 0; a < 3; a++) {
            if (mn.e[a] > p.e[a]) mn.e[a] = p.e[a];
            if (mx.e[a] < p.e[a]) mx.e[a] = p.e[a];
        }
    }
    return {mn, mx};
}

void mortonKeys(const pt_object* objs, int64_t n, bool includeOrigin, uint64_t* keys) {
    if (n <= 0) return;
    HBox mb = includeOrigin ? HBox{} : objBox(objs[0]);
    for (int64_t i = 0; i < n; i++) {   // aabb::unionBoxInPlace, aabb.h:36-44
        HBox b = objBox(objs[i]);
        for (int a = 0; a < 3; a++) {
            mb.mn.e[a] = std::fmin(mb.mn.e[a], b.mn.e[a]);
            mb.mx.e[a] = std::fmax(mb.mx.e[a], b.mx.e[a]);
        }
    }
    vec3 range = mb.mx - mb.mn;
    std::vector<std::pair<uint32_t, uint32_t>> m((size_t)n);
    for (int64_t i = 0; i < n; i++) {   // mortonCode3D, morton_code.h:29-45
        HBox b = objBox(objs[i]);
        vec3 c = (b.mn + b.mx) * 0.5f;
        float q[3];
        for (int a = 0; a < 3; a++) {
            float x = 0;
            if ((double)range.e[a] > 1e-7) x = (c.e[a] - mb.mn.e[a]) / range.e[a];
            q[a] = std::fmin(std::fmax(x * 1024.0f, 0.0f), 1023.0f);
        }
        uint32_t code = (expandBits((uint32_t)q[0]) << 2) + (expandBits((uint32_t)q[1]) << 1) + expandBits((uint32_t)q[2]);
        m[(size_t)i] = {code, (uint32_t)i};
    }
    std::stable_sort(m.begin(), m.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (int64_t i = 0; i < n; i++) keys[i] = ((uint64_t)m[(size_t)i].first << 32) | m[(size_t)i].second;
}

}  // namespace pt

// ================================================================== C ABI (host part)
using namespace pt;

extern "C" {

const char* pt_last_error(void) { return pt::lastError().c_str(); }
int pt_abi_version(void) { return PT_ABI_VERSION; }

int pt_camera_make(const float from[3], const float at[3], float vfov, float aspect, float aperture, float focus,
                   float t0, float t1, pt_camera* out) {
    if (!from || !at || !out) return fail(PT_ERR_INVALID, "pt_camera_make: null argument");
    *out = camera(get3(from), get3(at), vfov, aspect, aperture, focus, t0, t1).abi();
    return PT_OK;
}

int pt_camera_move(pt_camera* c, int dir, float dt) {
    if (!c || dir < 0 || dir > 5) return fail(PT_ERR_INVALID, "pt_camera_move: bad argument");
    camera cam(vec3(0, 0, 1), vec3(0, 0, 0), 90, 1, 0, 1);
    cam.mPosition = get3(c->origin);
    cam.mViewportLowLeftCorner = get3(c->lower_left);
    cam.mHorizontalViewportSize = get3(c->horizontal);
    cam.mVerticalViewportSize = get3(c->vertical);
    cam.mRight = get3(c->right);
    cam.mUp = get3(c->up);
    cam.mFront = get3(c->front);
    cam.mFocusDist = c->focus_dist;
    cam.mLensRadius = c->lens_radius;
    cam.time0 = c->time0;
    cam.time1 = c->time1;
    cam.processKeyboard((directions)dir, dt);
    *c = cam.abi();
    return PT_OK;
}

int pt_preset_instanced(const char* name, const char* models_dir, int width, int height, pt_instanced_desc* out) {
    if (!name || !out) return fail(PT_ERR_INVALID, "pt_preset_instanced: null argument");
    std::memset(out, 0, sizeof(*out));
    const std::string n = name, dir = models_dir ? models_dir : "models";
    if (n != "bunny_field" && n != "bunny_cornell" && n != "cornell")
        return fail(PT_ERR_INVALID, "pt_preset_instanced: no instanced form of '" + n + "'");
    try {
        // the flat preset for the frame, camera and materials; the meshes rebuilt in object space
        Scene flat = buildPreset(n, dir, width, height);
        Scene box, bunny;
        cornellBox(box, dir);   // (its own materials: the same 3 as the flat preset's first ones)
        std::vector<pt_instance> inst;
        auto translate = [](float x, float y, float z, int mesh) {
            pt_instance i{};
            i.m[0] = 1.0f; i.m[5] = 1.0f; i.m[10] = 1.0f;
            i.m[3] = x; i.m[7] = y; i.m[11] = z;
            i.mesh = mesh;
            return i;
        };
        inst.push_back(translate(0.0f, 0.0f, 0.0f, 0));   // the box, identity
        if (n == "bunny_cornell") {
            appendObj(bunny, dir + "/bunny/bunny.obj", 1500.0f, vec3(0, 0, 0), 0);
            inst.push_back(translate(438.0f, -49.96f, 113.0f, 1));
        } else if (n == "bunny_field") {   // pt_preset_scene's 15 x 14 grid, same order
            appendObj(bunny, dir + "/bunny/bunny.obj", 250.0f, vec3(0, 0, 0), 0);
            for (int i = 0; i < 15; i++)
                for (int j = 0; j < 14; j++)
                    inst.push_back(translate(24.0f + 35.5f * (float)i, -8.33f, 16.0f + 38.0f * (float)j, 1));
        }
        std::vector<pt_object> objs = box.objects;
        objs.insert(objs.end(), bunny.objects.begin(), bunny.objects.end());
        const int nm = bunny.objects.empty() ? 1 : 2;
        out->n_objects = (int64_t)objs.size();
        out->objects = (pt_object*)std::malloc(sizeof(pt_object) * std::max<size_t>(1, objs.size()));
        out->n_meshes = nm;
        out->mesh_first = (int64_t*)std::malloc(sizeof(int64_t) * 2);
        out->mesh_count = (int64_t*)std::malloc(sizeof(int64_t) * 2);
        out->n_instances = (int64_t)inst.size();
        out->instances = (pt_instance*)std::malloc(sizeof(pt_instance) * inst.size());
        out->n_materials = (int64_t)flat.materials.size();
        out->materials = (pt_material*)std::malloc(sizeof(pt_material) * std::max<size_t>(1, flat.materials.size()));
        if (!out->objects || !out->mesh_first || !out->mesh_count || !out->instances || !out->materials) {
            pt_instanced_desc_free(out);   // (what was allocated; the descriptor is left zeroed)
            return fail(PT_ERR_NOMEM, "pt_preset_instanced: out of memory");
        }
        std::memcpy(out->objects, objs.data(), sizeof(pt_object) * objs.size());
        out->mesh_first[0] = 0;
        out->mesh_count[0] = (int64_t)box.objects.size();
        out->mesh_first[1] = (int64_t)box.objects.size();
        out->mesh_count[1] = (int64_t)bunny.objects.size();
        std::memcpy(out->instances, inst.data(), sizeof(pt_instance) * inst.size());
        std::memcpy(out->materials, flat.materials.data(), sizeof(pt_material) * flat.materials.size());
        out->camera = flat.cam;
        out->width = flat.width;
        out->height = flat.height;
        out->spp = flat.spp;
        out->max_depth = flat.max_depth;
        std::snprintf(out->name, sizeof(out->name), "%s", flat.name.c_str());
    } catch (const std::exception& e) {
        pt_instanced_desc_free(out);
        return fail(PT_ERR_IO, std::string("pt_preset_instanced: ") + e.what());
    }
    return PT_OK;
}

void pt_instanced_desc_free(pt_instanced_desc* d) {
    if (!d) return;
    std::free(d->objects);
    std::free(d->mesh_first);
    std::free(d->mesh_count);
    std::free(d->instances);
    std::free(d->materials);
    std::memset(d, 0, sizeof(*d));
}

int pt_preset_scene(const char* name, const char* models_dir, int width, int height, pt_scene_desc* out) {
    if (!name || !out) return fail(PT_ERR_INVALID, "pt_preset_scene: null argument");
    std::memset(out, 0, sizeof(*out));
    try {
        Scene s = buildPreset(name, models_dir ? models_dir : "models", width, height);
        out->n_objects = (int64_t)s.objects.size();
        out->n_materials = (int64_t)s.materials.size();
        out->objects = (pt_object*)std::malloc(sizeof(pt_object) * std::max<size_t>(1, s.objects.size()));
        out->materials = (pt_material*)std::malloc(sizeof(pt_material) * std::max<size_t>(1, s.materials.size()));
        if (!out->objects || !out->materials) return fail(PT_ERR_NOMEM, "pt_preset_scene: out of memory");
        std::memcpy(out->objects, s.objects.data(), sizeof(pt_object) * s.objects.size());
        std::memcpy(out->materials, s.materials.data(), sizeof(pt_material) * s.materials.size());
        out->camera = s.cam;
        out->width = s.width;
        out->height = s.height;
        out->spp = s.spp;
        out->max_depth = s.max_depth;
        std::snprintf(out->name, sizeof(out->name), "%s", s.name.c_str());
    } catch (const std::exception& e) {
        return fail(PT_ERR_IO, std::string("pt_preset_scene: ") + e.what());
    }
    return PT_OK;
}

void pt_scene_desc_free(pt_scene_desc* d) {
    if (!d) return;
    std::free(d->objects);
    std::free(d->materials);
    d->objects = nullptr;
    d->materials = nullptr;
    d->n_objects = d->n_materials = 0;
}

int pt_load_obj(const char* path, float scale, const float t[3], int32_t mat, pt_object** out, int64_t* count) {
    if (!path || !out || !count) return fail(PT_ERR_INVALID, "pt_load_obj: null argument");
    Scene s;
    try {
        appendObj(s, path, scale, t ? get3(t) : vec3(), mat);
    } catch (const std::exception& e) {
        return fail(PT_ERR_IO, e.what());
    }
    *count = (int64_t)s.objects.size();
    *out = (pt_object*)std::malloc(sizeof(pt_object) * std::max<size_t>(1, s.objects.size()));
    if (!*out) return fail(PT_ERR_NOMEM, "pt_load_obj: out of memory");
    std::memcpy(*out, s.objects.data(), sizeof(pt_object) * s.objects.size());
    return PT_OK;
}

void pt_free(void* p) { std::free(p); }

int pt_morton_keys(const pt_object* objs, int64_t n, int include_origin, uint64_t* keys) {
    if (n < 0 || (n > 0 && (!objs || !keys))) return fail(PT_ERR_INVALID, "pt_morton_keys: bad argument");
    mortonKeys(objs, n, include_origin != 0, keys);
    return PT_OK;
}

int pt_quantize_rgba8(const float* rgb, int w, int h, uint8_t* rgba) {
    if (!rgb || !rgba || w <= 0 || h <= 0) return fail(PT_ERR_INVALID, "pt_quantize_rgba8: bad argument");
    PngImage png(w, h);
    for (int row = 0; row < h; row++)   // main.cu:477-483
        for (int col = 0; col < w; col++) {
            const float* c = rgb + 3 * ((size_t)row * w + col);
            png.saveColor(color(c[0], c[1], c[2]), h - row - 1, col);
        }
    std::memcpy(rgba, png.data().data(), png.data().size());
    return PT_OK;
}

int pt_write_png(const char* path, const float* rgb, int w, int h) {
    if (!path || !rgb || w <= 0 || h <= 0) return fail(PT_ERR_INVALID, "pt_write_png: bad argument");
    PngImage png(w, h);
    for (int row = 0; row < h; row++)
        for (int col = 0; col < w; col++) {
            const float* c = rgb + 3 * ((size_t)row * w + col);
            png.saveColor(color(c[0], c[1], c[2]), h - row - 1, col);
        }
    if (!png.write(path)) return fail(PT_ERR_IO, std::string("pt_write_png: cannot write ") + path);
    return PT_OK;
}

int pt_write_png_rgba8(const char* path, const uint8_t* rgba, int w, int h) {
    if (!path || !rgba || w <= 0 || h <= 0) return fail(PT_ERR_INVALID, "pt_write_png_rgba8: bad argument");
    PngImage png(w, h);
    const size_t stride = (size_t)w * 4;
    for (int row = 0; row < h; row++)   // row flip of main.cu:481
        std::memcpy(png.pixels() + (size_t)(h - row - 1) * stride, rgba + (size_t)row * stride, stride);
    if (!png.write(path)) return fail(PT_ERR_IO, std::string("pt_write_png_rgba8: cannot write ") + path);
    return PT_OK;
}

}  // extern "C"
