// pt_host.hpp — host-side C++ surface of the MI355X path tracer.
//
// Keeps the reference's host interfaces so scenes load and PNGs write unchanged:
//   vec3                (utils/vec3.h:10-104)        camera      (simulation/camera.h:10-76)
//   PngImage            (utils/png_image.h:15-49)    objl::Loader (outsource/OBJ_Loader.hpp, the
//                                                                 subset the reference would call)
//   Material / CudaObj constructors as plain builders (simulation/material.h:19-26,
//                                                      simulation/cuda_object.h:21-42)
//   scene builders      (main.cu:57-256 plus the benchmark configs of BASELINE.json)
// Everything here is host code; the device path is reached only through include/pt.h.
#pragma once
#include <cmath>
#include <cstdint>
#include <random>
#include <string>
#include <vector>

#include "pt.h"

namespace pt {

// ------------------------------------------------------------------- vec3 (utils/vec3.h)
struct vec3 {
    float e[3];
    vec3() : e{0, 0, 0} {}
    vec3(float a, float b, float c) : e{a, b, c} {}
    float x() const { return e[0]; }
    float y() const { return e[1]; }
    float z() const { return e[2]; }
    vec3 operator-() const { return {-e[0], -e[1], -e[2]}; }
    vec3& operator+=(const vec3& v) { e[0] += v.e[0]; e[1] += v.e[1]; e[2] += v.e[2]; return *this; }
    vec3& operator-=(const vec3& v) { e[0] -= v.e[0]; e[1] -= v.e[1]; e[2] -= v.e[2]; return *this; }
    float length_squared() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
    float length() const { return std::sqrt(length_squared()); }
};
using point3 = vec3;
using color = vec3;
inline vec3 operator+(const vec3& u, const vec3& v) { return {u.e[0] + v.e[0], u.e[1] + v.e[1], u.e[2] + v.e[2]}; }
inline vec3 operator-(const vec3& u, const vec3& v) { return {u.e[0] - v.e[0], u.e[1] - v.e[1], u.e[2] - v.e[2]}; }
inline vec3 operator*(const vec3& u, const vec3& v) { return {u.e[0] * v.e[0], u.e[1] * v.e[1], u.e[2] * v.e[2]}; }
inline vec3 operator*(float t, const vec3& v) { return {t * v.e[0], t * v.e[1], t * v.e[2]}; }
inline vec3 operator*(const vec3& v, float t) { return t * v; }
inline vec3 operator/(const vec3& v, float t) { return (1.0f / t) * v; }
inline float dot(const vec3& u, const vec3& v) { return u.e[0] * v.e[0] + u.e[1] * v.e[1] + u.e[2] * v.e[2]; }
inline vec3 cross(const vec3& u, const vec3& v) {
    return {u.e[1] * v.e[2] - u.e[2] * v.e[1], u.e[2] * v.e[0] - u.e[0] * v.e[2], u.e[0] * v.e[1] - u.e[1] * v.e[0]};
}
inline vec3 normalize(const vec3& v) {
    float l = v.length();
    if (l == 0) return {};
    return v / l;
}

// ---------------------------------------------------------------- camera (camera.h:10-76)
enum directions { FORWARD, BACKWARD, LEFT, RIGHT, UP, DOWN };   // utility.h:18-25

class camera {
public:
    camera(point3 lookFrom, point3 lookAt, float vfov, float aspect_ratio, float aperture, float focus_dist,
           float time0 = 0, float time1 = 0);
    void processKeyboard(directions dir, float deltaTime);
    pt_camera abi() const;

    point3 mPosition, mViewportLowLeftCorner;
    vec3 mHorizontalViewportSize, mVerticalViewportSize;
    vec3 mRight, mUp, mFront;
    float mFocusDist, mLensRadius, time0, time1;
};

// ------------------------------------------------------------ PngImage (png_image.h:15-49)
class PngImage {
public:
    PngImage(int w, int h, int n = 4);
    PngImage(const PngImage&) = delete;
    PngImage& operator=(const PngImage&) = delete;
    void saveColor(color clr, int row, int col, int samples_per_pixel = 1);
    int width() const { return mDataW; }
    int height() const { return mDataH; }
    int channel() const { return mDataN; }
    bool write(const char* filename) const;
    const std::vector<uint8_t>& data() const { return mData; }
    uint8_t* pixels() { return mData.data(); }   // raw RGBA8 rows, top row first (as written)

private:
    std::vector<uint8_t> mData;
    int mDataW, mDataH, mDataN;
};

// --------------------------------------------- objl::Loader surface (OBJ_Loader.hpp:407-717)
namespace objl {
struct Vector2 { float X = 0, Y = 0; };
struct Vector3 { float X = 0, Y = 0, Z = 0; };
struct Vertex { Vector3 Position; Vector3 Normal; Vector2 TextureCoordinate; };
struct Mesh {
    std::string MeshName;
    std::vector<Vertex> Vertices;
    std::vector<unsigned int> Indices;
};
class Loader {
public:
    // Parses v/vt/vn/f (and o/g mesh splits); polygons are fan-triangulated, which equals the
    // reference loader's split for the triangles and convex quads the bundled models contain.
    bool LoadFile(const std::string& path);
    std::vector<Mesh> LoadedMeshes;
    std::vector<Vertex> LoadedVertices;
    std::vector<unsigned int> LoadedIndices;
};
}  // namespace objl

// ------------------------------------------------------------------- scene assembly
// Material constructors: material.h:21-26 (the overload is the type tag; metal fuzz clamps to 1).
pt_material lambertian(const color& albedo);
pt_material metal(const color& albedo, float fuzz);
pt_material dielectric(float ir);
// CudaObj constructors: cuda_object.h:21-42.
pt_object sphere(const point3& c, float r, int mat);
pt_object triangle(const point3& v0, const point3& v1, const point3& v2, int mat);

// The reference's host RNG: one static mt19937 + uniform_real_distribution<float>(0,1)
// (utility.h:103-108).  vec3(f(), f(), f()) arguments are evaluated right to left by the
// compilers the reference was built with (MSVC / g++), i.e. z is drawn first.
class HostRng {
public:
    float uniform() { return dist(gen); }
    vec3 vec3_args() {   // vec3(randomUniformOnHost(), randomUniformOnHost(), randomUniformOnHost())
        float z = uniform(), y = uniform(), x = uniform();
        return {x, y, z};
    }
    vec3 inUnitSphereDiscard() {   // host randomInUnitSphereDiscard, utility.h:110-119
        vec3 res;
        do {
            float z = uniform() - 0.5f, y = uniform() - 0.5f, x = uniform() - 0.5f;
            res = 2.0f * vec3(x, y, z);
        } while (res.length_squared() >= 1.0f);
        return res;
    }

private:
    std::mt19937 gen;
    std::uniform_real_distribution<float> dist{0.0f, 1.0f};
};

struct Scene {
    std::string name;
    std::vector<pt_object> objects;
    std::vector<pt_material> materials;
    pt_camera cam{};
    int width = 0, height = 0, spp = 0, max_depth = 0;
};

// Builds a preset (see pt_preset_scene in pt.h); throws std::runtime_error on failure.
Scene buildPreset(const std::string& name, const std::string& modelsDir, int width, int height);
// Appends one triangle object per mesh triangle; v' = v * scale + translate.
size_t appendObj(Scene& s, const std::string& path, float scale, const vec3& translate, int mat);

// Morton keys (morton_code.h:29-75).
void mortonKeys(const pt_object* objs, int64_t n, bool includeOrigin, uint64_t* keys);

}  // namespace pt
