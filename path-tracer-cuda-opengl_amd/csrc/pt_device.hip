// pt_device.hip — MI355X (gfx950) device path: LBVH build, closest-hit traversal, render.
//
// Hot path re-designed for CDNA4:
//  * render: one lane per pixel of an 8x8 tile (one wave per workgroup), path regeneration
//    (a lane whose path ends starts its next sample in the same loop iteration, so no lane
//    idles between samples), per-lane XORWOW state in registers, coalesced SoA state I/O.
//  * traversal: BVH2 whose internal-node record holds BOTH child boxes + child refs (64 B,
//    four dwordx4 loads per visit, one 64-B segment); leaves are folded into the parent's
//    child refs; the traversal stack lives in LDS, lane-interleaved (conflict-free).
//  * primitives are stored in Morton (leaf) order, 48 B each ({v0,v1,v2} / {c,r}: the exact
//    object box is recomputed from them); a 48-B shading record per primitive (normal or
//    sphere centre/radius + the material inline) is read once per closest hit, in one round trip.
//  * LBVH: Karras hierarchy kernel + atomic-counter bottom-up refit with tight boxes.
// All arithmetic follows the reference's operation order and is compiled with
// -ffp-contract=off, so results are bit-identical to oracle/ (the CPU restatement).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <type_traits>
#include <memory>
#include <string>
#include <vector>

#include "../host/pt_error.hpp"
#include "../host/pt_host.hpp"
#include "../host/pt_wide8.hpp"
#include "../host/pt_wide_dev.hpp"
#include "pt.h"
#include "pt_math.hpp"

using pt::fail;

#include "pt_prims.hpp"   // radixSortPairs (pt_sort.hip)

namespace pt {
int launchCompatWide(int stack, const void* params, hipStream_t st);   // pt_compat.hip
int compatWideWavesPerCU(int stack, int& n);                            // pt_compat.hip
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            return fail(PT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
    } while (0)

namespace {

constexpr int kWave = 64;
#ifndef PT_AB_NO_ATOMICS
#define PT_AB_NO_ATOMICS 0
#endif
// Time-only A/B switches (wrong images; DESIGN.md section 11's VALU budget): the Lambertian
// rejection loop cut to its first trial; the sample-mode Philox seeding replaced by a two-multiply
// hash; the ray start without its MIX-range check and with a bare v_rcp_f32.
#ifndef PT_FIXED_SMALL
#define PT_FIXED_SMALL 1   // sample mode: blockFixedSmall when every finishing lane's sums are in [0, 2^24)
#endif
#ifndef PT_AB_ONE_TRIAL
#define PT_AB_ONE_TRIAL 0
#endif
#ifndef PT_AB_CHEAP_SEED
#define PT_AB_CHEAP_SEED 0
#endif
#ifndef PT_AB_CHEAP_START
#define PT_AB_CHEAP_START 0
#endif
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kSphereBit = 0x40000000u;
constexpr uint32_t kPrimMask = 0x3fffffffu;
constexpr int kJumpMats = 32;
constexpr int kNumCounters = 32;                 // per-scene u64 counters: work counts, error word, diagnostics                    // XORWOW 2^(67+k) jump matrices, k < 32

// ------------------------------------------------------------------------ device structs
struct DevScene {
    const float4* nodes;     // 4 x float4 per internal node: child boxes as (min, max) pairs per axis, refs (nodeBoxIdx)
    const float4* prims;     // 3 x float4 per primitive (leaf order)
    const float4* shade;     // 3 x float4 per primitive: {n | c, r} {albedo, fuzz} {ir, type | sphere << 16, mat, obj}
    const float4* mats;      // 2 x float4 per material
    const float4* wnodes;    // compressed 8-wide nodes, 5 x float4 each (renderKernelWF<.., WIDE>; host/pt_wide8.cpp)
    const float4* wprims;    // primitive records in wide-tree leaf order, {v0, rank} {v1, objID} {v2, sphere}
    const float4* wshade;    // shading records in reference rank order (wide kernels)
    const uint32_t* rankOf;  // leaf k -> its rank in the reference's traversal order
    const int* iparent;      // parent of each internal LBVH node (-1 for the root)
    unsigned int* err;       // set (never cleared in-kernel) when a traversal guard trips
    int nprims;
    int hasSpheres;          // 0: triangles only (the wide kernels' LEAF tests drop the sphere tie rules)
    float cx, cy, cz, ext;   // tight scene box: centre and largest extent (the wide kernels' far-origin test)
    float mixLim;            // largest finite |1 / d| component the MIX plane arithmetic takes (wideHits, mixUnsafe)
    // instanced scenes (renderKernelWF<.., INST>): per instance {world-to-object rows r0, r1, r2}
    // {objBase, identity, 0, 0}; a hit's key is instance << gBits | its primitive's shading index
    const float4* winst;
    int gBits;
};
// Instancing: the stack entry that returns a lane from an instance's bottom-level tree to the world
// (a child base of 2^24 - 1 never exists); the exponent word of an instance record (pt_wide8.hpp).
constexpr uint32_t kInstMarker = 0xffffffffu;
constexpr uint32_t kInstFlag = 0xff000000u;

struct DevCamera {
    float3 pos, ll, hor, ver;
    float3 right, up;
    float lens;   // lens radius (aperture / 2); 0: a pinhole, no lens draws
};


struct Counters {
    uint32_t rays, visits, tris, spheres;
};

// ------------------------------------------------------------------------ math helpers
// Exact restatements of utils/vec3.h operators (no contraction: -ffp-contract=off).
__device__ __forceinline__ float3 f3(float a, float b, float c) { return make_float3(a, b, c); }
__device__ __forceinline__ float3 add(float3 a, float3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ float3 sub(float3 a, float3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float3 mul(float3 a, float3 b) { return f3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float3 scale(float t, float3 v) { return f3(t * v.x, t * v.y, t * v.z); }
__device__ __forceinline__ float3 neg(float3 v) { return f3(-v.x, -v.y, -v.z); }
__device__ __forceinline__ float dot3(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float3 cross3(float3 u, float3 v) {
    return f3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
__device__ __forceinline__ float len2(float3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
__device__ __forceinline__ float3 divs(float3 v, float t) { return scale(rcpRN(t), v); }
__device__ __forceinline__ float3 normalize3(float3 v) {
    float l = sqrtf(len2(v));
    if (l == 0.0f) return f3(0.0f, 0.0f, 0.0f);
    return divs(v, l);
}
__device__ __forceinline__ float3 xyz(float4 v) { return f3(v.x, v.y, v.z); }

// ------------------------------------------------------------------------ XORWOW
#ifndef PT_XORWOW_BITOP3
#define PT_XORWOW_BITOP3 1
#endif
struct Xorwow {
    uint32_t d, v0, v1, v2, v3, v4;
    __device__ __forceinline__ uint32_t next() {   // curand(curandStateXORWOW*)
        uint32_t t = v0 ^ (v0 >> 2);
        v0 = v1; v1 = v2; v2 = v3; v3 = v4;
#if PT_XORWOW_BITOP3   // the three-way XOR in one v_bitop3_b32 (gfx950): six VALU per draw instead of seven
        v4 = __builtin_amdgcn_bitop3_b32(v4, v4 << 4, t ^ (t << 1), 0x96);
#else
        v4 = (v4 ^ (v4 << 4)) ^ (t ^ (t << 1));
#endif
        d += 362437u;
        return v4 + d;
    }
    // curand_uniform: x * 2^-32 + 2^-33 in (0, 1] (one exact FMA, pt_math.hpp)
    __device__ __forceinline__ float uniform() { return uniformOf(next()); }
    // 2 * (uniform() - 0.5f): the unit-sphere coordinates (one exact FMA, pt_math.hpp)
    __device__ __forceinline__ float centered2() { return centered2Of(uniform()); }
};

// Sample mode stream of (pixel p, sample s): one Philox4x32-10 block (Salmon et al. 2011)
// with key = seed and counter = {s, p_lo, p_hi, "SAMP"} seeds a XORWOW state, whose draws
// then cost a few shifts each (the reference's generator family, curand_uniform mapping).
// Any sample of any pixel starts anywhere, in one block of work.
__device__ __forceinline__ Xorwow sampleStream(uint32_t k0, uint32_t k1, uint32_t sample, uint32_t pixel) {
#if PT_AB_CHEAP_SEED   // (A/B timing only: no Philox rounds)
    {
        const uint32_t a = (sample ^ k0) * 0x9E3779B9u, b = (pixel ^ k1) * 0x85EBCA6Bu;
        return Xorwow{a, a ^ b, b + 0x6C078965u, a + b, (a ^ 0x2545F491u) | 1u, b ^ 0x53414D50u};
    }
#endif
    uint32_t c0 = sample, c1 = pixel, c2 = 0u, c3 = 0x53414D50u;
#pragma unroll 2   // (pairs of rounds: no register moves; a full unroll raises the camera-ray site's pressure)
    for (int r = 0; r < 10; r++) {
        // one 32 x 32 -> 64 multiply per word (v_mad_u64_u32) instead of mul_hi + mul_lo
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#if PT_XORWOW_BITOP3   // (three-way XORs as one v_bitop3_b32 each)
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96), n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
#else
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
#endif
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return Xorwow{c3, c0, c1, c2, c3 ^ 0x6C078965u, c0 ^ c1 ^ 0x2545F491u};
}

// ------------------------------------------------------------------------ traversal
// aabb::hit (aabb.h:21-34): per axis t0=(min-o)*inv, t1=(max-o)*inv, swap if inv<0,
// tmin=max(tmin,t0), tmax=min(tmax,t1); miss if tmax<tmin.  The ternaries of the reference
// keep the old bound on NaN, which is exactly maxNum/minNum (v_max_f32 / v_min_f32).
// SlabHit also returns the entry distance lo = max(tmin, near planes).  For a box that
// passed with tmax = T, the same test with any tmax' <= T fails iff tmax' < lo: hi(T') =
// fminf(T', far planes) and fminf ignores NaN, so hi(T') < lo <=> T' < lo or far < lo, and
// the latter is false because the box passed.  (lo is never NaN: fmaxf(tmin, NaN) = tmin.)
struct SlabHit { bool hit; float lo; };

// Internal node record, 16 floats (4 x float4).  Each child box is stored as one (min, max)
// pair per axis, so every pair sits in an aligned 64-bit register pair and the six slab
// planes of a child cost three packed subtracts and three packed multiplies
// (v_pk_add_f32 / v_pk_mul_f32: the same IEEE operations, two per instruction):
//   [0..5]  left  {mnx, mxx, mny, mxy, mnz, mxz}     [6..11] right {mnx, mxx, mny, mxy, mnz, mxz}
//   [12] left ref  [13] right ref  [14..15] unused
__host__ __device__ constexpr int nodeBoxIdx(int child, int axis, int isMax) { return 6 * child + 2 * axis + isMax; }

typedef float v2f __attribute__((ext_vector_type(2)));

// slabLo on a box given as (min, max) pairs per axis (the node record layout).
__device__ __forceinline__ SlabHit slabPair(v2f X, v2f Y, v2f Z, float3 o, float3 inv, float tmin, float tmax) {
    const v2f tx = (X - o.x) * inv.x, ty = (Y - o.y) * inv.y, tz = (Z - o.z) * inv.z;
    float nx = inv.x < 0.0f ? tx.y : tx.x, fx = inv.x < 0.0f ? tx.x : tx.y;
    float ny = inv.y < 0.0f ? ty.y : ty.x, fy = inv.y < 0.0f ? ty.x : ty.y;
    float nz = inv.z < 0.0f ? tz.y : tz.x, fz = inv.z < 0.0f ? tz.x : tz.y;
    float lo = fmaxf(fmaxf(fmaxf(tmin, nx), ny), nz);
    float hi = fminf(fminf(fminf(tmax, fx), fy), fz);
    return SlabHit{!(hi < lo), lo};
}
// Both child boxes of a node record at once (the 12 plane distances first, then the selects).
struct SlabHit2 { SlabHit l, r; };
__device__ __forceinline__ SlabHit2 slabBoth(float4 a, float4 b, float4 q, float3 o, float3 inv, float tmin,
                                             float tmax) {
    const v2f lx = (v2f{a.x, a.y} - o.x) * inv.x, ly = (v2f{a.z, a.w} - o.y) * inv.y,
              lz = (v2f{b.x, b.y} - o.z) * inv.z;
    const v2f rx = (v2f{b.z, b.w} - o.x) * inv.x, ry = (v2f{q.x, q.y} - o.y) * inv.y,
              rz = (v2f{q.z, q.w} - o.z) * inv.z;
    const bool sx = inv.x < 0.0f, sy = inv.y < 0.0f, sz = inv.z < 0.0f;
    SlabHit2 h;
    {
        const float lo = fmaxf(fmaxf(fmaxf(tmin, sx ? lx.y : lx.x), sy ? ly.y : ly.x), sz ? lz.y : lz.x);
        const float hi = fminf(fminf(fminf(tmax, sx ? lx.x : lx.y), sy ? ly.x : ly.y), sz ? lz.x : lz.y);
        h.l = SlabHit{!(hi < lo), lo};
    }
    {
        const float lo = fmaxf(fmaxf(fmaxf(tmin, sx ? rx.y : rx.x), sy ? ry.y : ry.x), sz ? rz.y : rz.x);
        const float hi = fminf(fminf(fminf(tmax, sx ? rx.x : rx.y), sy ? ry.x : ry.y), sz ? rz.x : rz.y);
        h.r = SlabHit{!(hi < lo), lo};
    }
    return h;
}
// Both child boxes of a node record (a, b, q = its first three float4s).
__device__ __forceinline__ SlabHit slabLeft(float4 a, float4 b, float3 o, float3 inv, float tmin, float tmax) {
    return slabPair(v2f{a.x, a.y}, v2f{a.z, a.w}, v2f{b.x, b.y}, o, inv, tmin, tmax);
}
__device__ __forceinline__ SlabHit slabRight(float4 b, float4 q, float3 o, float3 inv, float tmin, float tmax) {
    return slabPair(v2f{b.z, b.w}, v2f{q.x, q.y}, v2f{q.z, q.w}, o, inv, tmin, tmax);
}

// Primitive record (leaf order), 3 x float4:
//   triangle {v0, mat} {v1, objID} {v2, 0}        sphere {c, mat} {r, 0, 0, objID} {0, 0, 0, 1}
struct Prim { float4 p0, p1, p2; };
// Raw gfx9 buffer resource over a device array (stride 0, DATA_FORMAT_32): per-lane loads then
// take a 32-bit offset instead of 64-bit address arithmetic.  Arrays stay below 4 GB (< 2^26
// primitives / nodes, pt_scene_create).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rawRsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, -1 /* 4 GB of records */, 0x00020000);
}
// Integer products by small constants as full-rate shifts.  v_mul_lo_u32 (and the 64-bit
// v_mad_u64_u32) issue at a quarter of the VALU rate; LLVM folds `(x << a) + (x << b)` back into
// a multiply and lowers it with v_mul_lo_u32, so one shift is done in an (empty-effect) asm
// statement the folder cannot see through.
template <int S>
__device__ __forceinline__ uint32_t shlOpaque(uint32_t x) {
    uint32_t t;
    asm("v_lshlrev_b32 %0, %1, %2" : "=v"(t) : "i"(S), "v"(x));
    return t;
}
// byte offset of node slot x (80-B slots: x < 2^26; 128-B slots, PT_NODE_DWORDS 32: x < 2^25)
__device__ __forceinline__ uint32_t mul80(uint32_t x) {
    if constexpr (pt::kW8NodeDwords == 32) return x << 7;
    return shlOpaque<6>(x) + (x << 4);
}
__device__ __forceinline__ uint32_t mul48(uint32_t x) { return shlOpaque<5>(x) + (x << 4); }   // x < 2^27
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

__device__ __forceinline__ Prim loadPrim(const DevScene& S, uint32_t k) {
    const float4* p = S.prims + 3 * (size_t)k;
    return Prim{p[0], p[1], p[2]};
}

// CudaObj::hit (cuda_object.h:44-92): returns the accepted t (> tmin > 0), or -1 on a miss.
// `closest` is the current t_max.  Values are returned, never written through references, so
// the compiler keeps every traversal variable in registers.
__device__ __forceinline__ float primHitT(const Prim& q, bool sphere, float3 o, float3 d, float tmin, float closest) {
    if (sphere) {
        float3 oc = sub(o, xyz(q.p0));
        float r = q.p1.x;
        float a = len2(d);
        float half_b = dot3(oc, d);
        float cc = len2(oc) - r * r;
        float disc = half_b * half_b - a * cc;
        if (disc < 0.0f) return -1.0f;
        float sq = sqrtf(disc);
        float root = (-half_b - sq) / a;
        if (root < tmin || closest < root) {
            root = (-half_b + sq) / a;
            if (root < tmin || closest < root) return -1.0f;
        }
        return root;
    }
    const float3 v0 = xyz(q.p0);
    float3 e1 = sub(xyz(q.p1), v0), e2 = sub(xyz(q.p2), v0);
    float3 s1 = cross3(d, e2);
    float det = dot3(s1, e1);
    if (det == 0.0f) return -1.0f;
    float3 s = sub(o, v0);
    float3 s2 = cross3(s, e1);
    float inv = rcpRN(det);
    float t = dot3(s2, e2) * inv;
    float b1 = dot3(s1, s) * inv;
    float b2 = dot3(s2, d) * inv;
    // The reference's strict tests (cuda_object.h:83) without `b1 + b2 <= 0`, which never decides:
    // a sum that is <= 0 is not NaN, so neither term is, and the rounded sum of two positive terms
    // is positive -- one of b1 <= 0, b2 <= 0 already rejected it.  (b1 >= 1 and b2 >= 1 stay: with
    // the other term NaN, the sum test would not see them.)
    if (b1 >= 1.0f || b1 <= 0.0f || b2 >= 1.0f || b2 <= 0.0f || b1 + b2 >= 1.0f || t <= tmin || t >= closest)
        return -1.0f;
    return t;
}

__device__ __forceinline__ void primTest(const DevScene& S, uint32_t ref, float3 o, float3 d, float tmin,
                                         float& closest, int& best, Counters& c) {
    const uint32_t k = ref & kPrimMask;
    const bool sph = (ref & kSphereBit) != 0;
    if (sph) c.spheres++;
    else c.tris++;
    const float t = primHitT(loadPrim(S, k), sph, o, d, tmin, closest);
    if (t >= 0.0f) {
        closest = t;
        best = (int)k;
    }
}

// ------------------------------------------------------------------------ wide tree
// The reference's closest hit does not depend on its traversal order except through ties:
// a primitive is accepted when t < closest (triangle, cuda_object.h:83) or t <= closest
// (sphere, :57-61), and its left-first DFS visits leaves in key order k.  So the reference's
// result over ANY set of visited primitives that contains every primitive it would accept is
// the minimum of (t, tie rank) with ranks: spheres before triangles, spheres by DESCENDING k
// (a later sphere at the same t replaces the earlier hit), triangles by ASCENDING k (a later
// triangle at the same t is rejected).  The wide tree's boxes are conservative (outward-rounded
// planes, pt_wide8.cpp), so every primitive the reference would accept is visited.

// Candidate distance of a primitive independent of the current closest hit: the sphere's
// first root when >= tmin, else its second (the reference tries them in this order against
// [tmin, closest]; the second is never smaller); triangles as primHitT.  -1 on a miss.
__device__ __forceinline__ float primHitAny(const Prim& q, bool sphere, float3 o, float3 d, float tmin) {
    if (sphere) {
        float3 oc = sub(o, xyz(q.p0));
        float r = q.p1.x;
        float a = len2(d);
        float half_b = dot3(oc, d);
        float cc = len2(oc) - r * r;
        float disc = half_b * half_b - a * cc;
        if (disc < 0.0f) return -1.0f;
        float sq = sqrtf(disc);
        float root = (-half_b - sq) / a;
        if (!(root < tmin)) return root;
        root = (-half_b + sq) / a;
        if (!(root < tmin)) return root;
        return -1.0f;
    }
    const float3 v0 = xyz(q.p0);
    float3 e1 = sub(xyz(q.p1), v0), e2 = sub(xyz(q.p2), v0);
    float3 s1 = cross3(d, e2);
    float det = dot3(s1, e1);
    if (det == 0.0f) return -1.0f;
    float3 s = sub(o, v0);
    float3 s2 = cross3(s, e1);
    float inv = rcpRN(det);
    float t = dot3(s2, e2) * inv;
    float b1 = dot3(s1, s) * inv;
    float b2 = dot3(s2, d) * inv;
    if (b1 >= 1.0f || b1 <= 0.0f || b2 >= 1.0f || b2 <= 0.0f || b1 + b2 >= 1.0f || t <= tmin)   // (as primHitT)
        return -1.0f;
    return t;
}

// aabb::hit (aabb.h:21-34) on the primitive's exact box (cuda_object.h:21-42: sphere c -/+ |r|,
// triangle min / max of its vertices): the test the reference's traversal applies to a leaf
// before its primitive test (render_manager.h:107-123).
__device__ __forceinline__ SlabHit refLeafBox(const Prim& q, bool sphere, float3 o, float3 inv, float tmin, float tmax) {
    float mn[3], mx[3];
    if (sphere) {
        const float r = fabsf(q.p1.x);
        mn[0] = q.p0.x - r; mn[1] = q.p0.y - r; mn[2] = q.p0.z - r;
        mx[0] = q.p0.x + r; mx[1] = q.p0.y + r; mx[2] = q.p0.z + r;
    } else {   // utils::unionPoints (aabb.h:68-79); vertices are never NaN, so v_min3 / v_max3
        // give the same planes (up to the sign of a zero, which no slab comparison sees)
        mn[0] = fminf(fminf(q.p0.x, q.p1.x), q.p2.x);
        mn[1] = fminf(fminf(q.p0.y, q.p1.y), q.p2.y);
        mn[2] = fminf(fminf(q.p0.z, q.p1.z), q.p2.z);
        mx[0] = fmaxf(fmaxf(q.p0.x, q.p1.x), q.p2.x);
        mx[1] = fmaxf(fmaxf(q.p0.y, q.p1.y), q.p2.y);
        mx[2] = fmaxf(fmaxf(q.p0.z, q.p1.z), q.p2.z);
    }
    return slabPair(v2f{mn[0], mx[0]}, v2f{mn[1], mx[1]}, v2f{mn[2], mx[2]}, o, inv, tmin, tmax);
}

// Test wide-order primitive record q ({v0, rank}{v1, obj}{v2, sphere}) and keep the minimum of
// (t, tie rank).  `best` = rank | kSphereBit for a sphere, -1 before the first hit.
// The reference only tests a primitive whose exact box passes with the closest hit of that
// moment (aabb::hit, render_manager.h:107-123; a single primitive is the root and has no box
// test, :92-98).  A hit inside its own box (entry lo <= t, as exact arithmetic guarantees) is
// tested by the reference whenever it could matter, in any order.  A grazing hit whose rounded
// box entry lies beyond it (t < lo) is tested only if the closest hit of that moment is >= lo:
// the outcome depends on the order exactly when another candidate's t lies in [t, lo).  Such a
// lane sets `redo` and its query is repeated in the reference's order (traceRefStackless);
// `bestLo` is the current best's window end (its box entry when t < lo, else -inf).
// SPH = false: the scene has no spheres (DevScene::hasSpheres), so neither q nor the current best
// is one and the tie rule reduces to the triangles' ascending rank -- the same decisions with
// fewer instructions.
template <bool SPH>
__device__ __forceinline__ void wideTest(const Prim& q, float3 o, float3 d, float3 inv, float tmin, float& closest,
                                         int& best, float& bestLo, bool leafBoxes, bool& redo, uint32_t keyHi = 0u) {
    const bool sph = SPH && __float_as_uint(q.p2.w) != 0u;
    const float t = primHitAny(q, sph, o, d, tmin);
    if (t >= 0.0f) {
        // (instanced scenes: the instance id above the shading index, keyHi = instance << gBits)
        const int k = (int)(keyHi | __float_as_uint(q.p0.w));
        const bool none = best < 0, bSph = SPH && (best & (int)kSphereBit) != 0;
        const int bk = SPH ? best & (int)kPrimMask : best;
        const bool tie = sph ? (none || !bSph || k > bk) : (!none && !bSph && k < bk);
        redo = redo || (t >= closest && t < bestLo);   // not better, but inside the current best's window
        if (t < closest || (t == closest && tie)) {
            bool take = true;
            float lo = -__builtin_inff();
            if (leafBoxes) {
                const SlabHit b = refLeafBox(q, sph, o, inv, tmin, __builtin_inff());
                take = b.hit && !(closest < b.lo);
                redo = redo || (b.hit && closest < b.lo);   // the current best inside this one's window
                lo = t < b.lo ? b.lo : lo;
            }
            if (take) {
                closest = t;
                best = k | (sph ? (int)kSphereBit : 0);
                bestLo = lo;
            }
        }
    }
}

// wideTest's decisions on a primitive another lane tested (the wave-cooperative LEAF step): t from
// primHitAny, key = its rank | kSphereBit for a sphere, blo = its exact leaf box's entry distance
// (aabb::hit with tmax = inf) or -1 when that box is missed (an entry is >= tmin > 0).  Applied in
// the group's order, the same updates of closest / best / bestLo / redo as wideTest.
template <bool SPH>
__device__ __forceinline__ void wideMerge(float t, uint32_t key, float blo, float& closest, int& best, float& bestLo,
                                          bool leafBoxes, bool& redo) {
    if (t >= 0.0f) {
        const bool sph = SPH && (key & kSphereBit) != 0u;
        const int k = (int)(key & kPrimMask);
        const bool none = best < 0, bSph = SPH && (best & (int)kSphereBit) != 0;
        const int bk = SPH ? best & (int)kPrimMask : best;
        const bool tie = sph ? (none || !bSph || k > bk) : (!none && !bSph && k < bk);
        redo = redo || (t >= closest && t < bestLo);
        if (t < closest || (t == closest && tie)) {
            bool take = true;
            float lo = -__builtin_inff();
            if (leafBoxes) {
                const bool bh = blo >= 0.0f;
                take = bh && !(closest < blo);
                redo = redo || (bh && closest < blo);
                lo = t < blo ? blo : lo;
            }
            if (take) {
                closest = t;
                best = k | (sph ? (int)kSphereBit : 0);
                bestLo = lo;
            }
        }
    }
}

// Lanes below this one whose bit is set in m (v_mbcnt_lo / v_mbcnt_hi).
__device__ __forceinline__ __attribute__((unused)) uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One compressed 8-wide node (five 16-B words, layout in host/pt_wide8.cpp) against the ray:
// returns the hit mask, internal children in bits 24 + (slot ^ oct), leaf primitives in bits
// 0..23 (offsets from the node's primitive base).  Plane distances t = q * (s * inv) + (p - o) *
// inv; the planes lie at least the tree's smallest quantum 2^emin outside the exact boxes (one
// node quantum up to round 6), beyond this arithmetic's rounding,
// and a NaN (0 * inf on an axis the ray is parallel to) only drops that plane: the test never
// rejects a box the exact slab test (aabb.h:21-34) accepts.
//
// The margin holds while |p - o| stays within about 11 times the larger of the scene's extent
// and its coordinates (the margin is >= 2^-18 of that, the rounding of the ray's plane distances
// about 2^-21.6 of |p - o|): a ray whose origin lies farther than 8 scene extents from the
// scene's centre (wideFar) skips this test and is traced in the reference's order instead.
//
// MIX: the plane bytes as fp16 denormals into v_fma_mix_f32 (pt_math.hpp fmaMixLo), the scales
// a = s * inv taken times 2^24 -- the same t bit for bit while |s * 2^24 * inv| stays finite,
// which holds for |inv| <= DevScene::mixLim (a ray with a larger finite |inv| component takes the
// reference-order query instead: mixUnsafe).
template <bool MIX = false>
__device__ __forceinline__ uint32_t wideHits(uint4 n0, uint4 n1, uint4 n2, uint4 n3, uint4 n4, float3 o, float3 inv,
                                             uint32_t oct, float tmin, float tmax) {
    constexpr uint32_t kMixExp = MIX ? 24u : 0u;   // s * 2^24: the exponent byte + 24 (< 255: mixLim's bound)
    const float ax = __uint_as_float(((n0.w & 0xffu) + kMixExp) << 23) * inv.x;
    const float ay = __uint_as_float((((n0.w >> 8) & 0xffu) + kMixExp) << 23) * inv.y;
    const float az = __uint_as_float((((n0.w >> 16) & 0xffu) + kMixExp) << 23) * inv.z;
    const float bx = (__uint_as_float(n0.x) - o.x) * inv.x;
    const float by = (__uint_as_float(n0.y) - o.y) * inv.y;
    const float bz = (__uint_as_float(n0.z) - o.z) * inv.z;
    // near / far planes per axis: qlo for a positive direction, qhi for a negative one
    const bool sx = (oct & 1u) != 0, sy = (oct & 2u) != 0, sz = (oct & 4u) != 0;
    const uint32_t nearX[2] = {sx ? n2.z : n2.x, sx ? n2.w : n2.y}, farX[2] = {sx ? n2.x : n2.z, sx ? n2.y : n2.w};
    const uint32_t nearY[2] = {sy ? n3.z : n3.x, sy ? n3.w : n3.y}, farY[2] = {sy ? n3.x : n3.z, sy ? n3.y : n3.w};
    const uint32_t nearZ[2] = {sz ? n4.z : n4.x, sz ? n4.w : n4.y}, farZ[2] = {sz ? n4.x : n4.z, sz ? n4.y : n4.w};
    // the octant in every byte (shifts: the multiply by 0x01010101 is a quarter-rate v_mul_lo_u32)
    const uint32_t oct2 = oct | shlOpaque<8>(oct);
    const uint32_t oct4 = oct2 | (oct2 << 16);
    uint32_t hits = 0u;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t meta4 = h ? n1.w : n1.z;
        // per byte: internal children (0b001_11xxx) get their slot bits XOR the ray octant
        const uint32_t inner4 = (meta4 & (meta4 << 1)) & 0x10101010u;
        // 0x07 in the bytes of internal children (oct4 <= 0x07070707): 8y - y, not a multiply
        const uint32_t inner1 = inner4 >> 4;
        const uint32_t innerMask4 = shlOpaque<3>(inner1) - inner1;
        const uint32_t bitIndex4 = (meta4 ^ (oct4 & innerMask4)) & 0x1f1f1f1fu;
        const uint32_t childBits4 = (meta4 >> 5) & 0x07070707u;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            float tnx, tny, tnz, tfx, tfy, tfz;
            if constexpr (MIX) {   // children j, j ^ 1 share an fp16 pair (the perms are redone per child:
                                   // cheaper in registers than six pairs live across two children)
                const bool hi = (j & 2) != 0;
                const uint32_t px = hi ? planePairHi(nearX[h]) : planePairLo(nearX[h]);
                const uint32_t py = hi ? planePairHi(nearY[h]) : planePairLo(nearY[h]);
                const uint32_t pz = hi ? planePairHi(nearZ[h]) : planePairLo(nearZ[h]);
                const uint32_t qx = hi ? planePairHi(farX[h]) : planePairLo(farX[h]);
                const uint32_t qy = hi ? planePairHi(farY[h]) : planePairLo(farY[h]);
                const uint32_t qz = hi ? planePairHi(farZ[h]) : planePairLo(farZ[h]);
                if (j & 1) {
                    tnx = fmaMixHi(px, ax, bx); tny = fmaMixHi(py, ay, by); tnz = fmaMixHi(pz, az, bz);
                    tfx = fmaMixHi(qx, ax, bx); tfy = fmaMixHi(qy, ay, by); tfz = fmaMixHi(qz, az, bz);
                } else {
                    tnx = fmaMixLo(px, ax, bx); tny = fmaMixLo(py, ay, by); tnz = fmaMixLo(pz, az, bz);
                    tfx = fmaMixLo(qx, ax, bx); tfy = fmaMixLo(qy, ay, by); tfz = fmaMixLo(qz, az, bz);
                }
            } else {
                tnx = __builtin_fmaf((float)((nearX[h] >> (8 * j)) & 0xffu), ax, bx);
                tny = __builtin_fmaf((float)((nearY[h] >> (8 * j)) & 0xffu), ay, by);
                tnz = __builtin_fmaf((float)((nearZ[h] >> (8 * j)) & 0xffu), az, bz);
                tfx = __builtin_fmaf((float)((farX[h] >> (8 * j)) & 0xffu), ax, bx);
                tfy = __builtin_fmaf((float)((farY[h] >> (8 * j)) & 0xffu), ay, by);
                tfz = __builtin_fmaf((float)((farZ[h] >> (8 * j)) & 0xffu), az, bz);
            }
            float lo, hi;
            if (MIX && (j & 1)) {
                lo = max3Raw(max3Raw(tnx, tny, tnz), tmin, tmin);
                hi = min3Raw(min3Raw(tfx, tfy, tfz), tmax, tmax);
            } else {
                lo = fmaxf(fmaxf(fmaxf(tnx, tny), tnz), tmin);
                hi = fminf(fminf(fminf(tfx, tfy), tfz), tmax);
            }
            const uint32_t bits = ((childBits4 >> (8 * j)) & 0xffu) << ((bitIndex4 >> (8 * j)) & 0xffu);
            hits |= lo <= hi ? bits : 0u;
        }
    }
    return hits;
}

// A direction parallel to an axis plane (a component +-0: |1/d| = inf; NaN counts too).
__device__ __forceinline__ bool zeroAxes(float3 inv) {
    return !(fmaxf(fmaxf(fabsf(inv.x), fabsf(inv.y)), fabsf(inv.z)) < __builtin_inff());
}
// One axis the ray is parallel to (d = +-0, 1/d = +-inf), for the 8 children of a wide node: aabb::hit
// (aabb.h:21-34) gives (plane - o) * (1/d) = -inf / +inf by the side of each plane o lies on (NaN when
// on it, which the reference's ternaries skip), so the axis bounds nothing when o lies between a
// child's two planes and rejects the child otherwise.  wideHits' decomposed form q * (s * inv) +
// (p - o) * inv is NaN for every plane of such an axis (never a wrong rejection, never a rejection
// at all: the ray would enter every child it overlaps in the other two axes -- round 4: 1,000-1,500
// node visits for C5 rays at the height of the origin).  Here the test itself, on the quantised
// planes p + q * s: u = (o - p) / s (1 / s a power of two), a child is kept when qlo <= u <= qhi.
// (The rounding of o - p is far below the planes' outward margin of >= 2^emin, as in wideHits.)
// k0 / k1: the children 0-3 / 4-7 byte masks, cleared (bits 5-7) for rejected children.
__device__ __forceinline__ void zeroAxisKeep(float oc, uint32_t pbits, uint32_t ebyte, uint32_t qlo0, uint32_t qlo1,
                                             uint32_t qhi0, uint32_t qhi1, uint32_t& k0, uint32_t& k1) {
    const float u = (oc - __uint_as_float(pbits)) * __uint_as_float((254u - ebyte) << 23);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const float l0 = (float)((qlo0 >> (8 * j)) & 0xffu), h0 = (float)((qhi0 >> (8 * j)) & 0xffu);
        const float l1 = (float)((qlo1 >> (8 * j)) & 0xffu), h1 = (float)((qhi1 >> (8 * j)) & 0xffu);
        if (u < l0 || u > h0) k0 &= ~(0xe0u << (8 * j));   // (NaN u: kept)
        if (u < l1 || u > h1) k1 &= ~(0xe0u << (8 * j));
    }
}
// Instanced scenes' node test (they have no reference-order query to hand such rays to): a wave with
// a lane whose ray -- in the current space -- is parallel to an axis plane clears the meta bytes of
// the children that lane's exact slab test rejects on that axis (zeroAxisKeep), then runs the usual
// test.  A wave-uniform branch: the common case pays the ballot only, and no registers stay live.
__device__ __forceinline__ uint32_t wideHitsInst(uint4 n0, uint4 n1, uint4 n2, uint4 n3, uint4 n4, float3 o,
                                                 float3 inv, uint32_t oct, float tmin, float tmax) {
    if (__ballot(zeroAxes(inv)) != 0) {
        const float inf = __builtin_inff();
        uint32_t k0 = 0xffffffffu, k1 = 0xffffffffu;
        if (!(fabsf(inv.x) < inf)) zeroAxisKeep(o.x, n0.x, n0.w & 0xffu, n2.x, n2.y, n2.z, n2.w, k0, k1);
        if (!(fabsf(inv.y) < inf)) zeroAxisKeep(o.y, n0.y, (n0.w >> 8) & 0xffu, n3.x, n3.y, n3.z, n3.w, k0, k1);
        if (!(fabsf(inv.z) < inf)) zeroAxisKeep(o.z, n0.z, (n0.w >> 16) & 0xffu, n4.x, n4.y, n4.z, n4.w, k0, k1);
        n1.z &= k0;
        n1.w &= k1;
    }
    return wideHits<false>(n0, n1, n2, n3, n4, o, inv, oct, tmin, tmax);
}

// The ray origin lies farther than 8 scene extents from the scene's centre on some axis, beyond
// the distance the wide boxes' margin covers (wideHits): the query runs in the reference's order.
#ifndef PT_WIDE_FAR_EXT
#define PT_WIDE_FAR_EXT 8.0f   // with the builders' PT_WIDE_EMIN_SHIFT 18 (host/pt_wide8.cpp)
#endif
constexpr float kWideFarExt = PT_WIDE_FAR_EXT;
__device__ __forceinline__ bool wideFar(float cx, float cy, float cz, float ext, float3 o) {
    const float m = fmaxf(fmaxf(fabsf(o.x - cx), fabsf(o.y - cy)), fabsf(o.z - cz));
    return !(m <= kWideFarExt * ext);   // (NaN: far)
}
__device__ __forceinline__ bool wideFar(const DevScene& S, float3 o) { return wideFar(S.cx, S.cy, S.cz, S.ext, o); }
// Instanced scenes draw the line at 2 world extents: their mesh trees are quantised for origins
// within that reach (buildInstanced), 4x finer planes than 8 extents would allow (c5i 503 -> 498
// ms); farther origins start at their entry into the world (instEntry).
#ifndef PT_INST_FAR_EXT
#define PT_INST_FAR_EXT 2.0f
#endif
constexpr float kInstFarExt = PT_INST_FAR_EXT;
static_assert(kInstFarExt >= 1.0f, "instEntry's cube (centre +- ext) must lie inside the quantised reach");
__device__ __forceinline__ bool instFar(const DevScene& S, float3 o) {
    const float m = fmaxf(fmaxf(fabsf(o.x - S.cx), fabsf(o.y - S.cy)), fabsf(o.z - S.cz));
    return !(m <= kInstFarExt * S.ext);   // (NaN: far)
}

// Instanced scenes have no reference-order query: a ray whose origin lies beyond the region the
// planes' margin covers (instFar) is moved along itself to its entry into the cube centre +- ext
// (ext = the world box's LARGEST extent, so the cube is the world box grown by at least ext / 2 on
// every side) -- no geometry lies before that point, and the new origin lies within 1 extent of the
// centre (max norm), inside the 2-extent reach every instanced tree was quantised for
// (buildInstanced; kInstFarExt >= 1 keeps the cube inside that reach).
// Returns the distance moved (0 when the ray misses that box or starts inside it).
__device__ __forceinline__ float instEntry(float cx, float cy, float cz, float ext, float3& o, float3 d, float3 inv) {
    const float lx = (cx - ext - o.x) * inv.x, hx = (cx + ext - o.x) * inv.x;
    const float ly = (cy - ext - o.y) * inv.y, hy = (cy + ext - o.y) * inv.y;
    const float lz = (cz - ext - o.z) * inv.z, hz = (cz + ext - o.z) * inv.z;
    const float t0 = fmaxf(fmaxf(fminf(lx, hx), fminf(ly, hy)), fminf(lz, hz));
    const float t1 = fminf(fminf(fmaxf(lx, hx), fmaxf(ly, hy)), fmaxf(lz, hz));
    if (!(t0 > 0.0f) || !(t0 <= t1)) return 0.0f;
    o = add(o, scale(t0, d));
    return t0;
}

// A reciprocal direction component larger than `lim` (DevScene::mixLim: a ray nearly parallel to
// an axis plane) would overflow the MIX plane scale s * 2^24 * inv (wideHits); such a ray takes the
// reference-order query.  So does an infinite component (a direction component of exactly 0): the
// decomposed plane distance fma(q, s * inv, (base - o) * inv) is then NaN for most planes, the
// NaN-ignoring min / max drop that axis's bound, and the ray would enter every box it overlaps in
// the other two axes (round 4: 1,000-1,500 node visits for C5 rays at the origin's height against a
// median of 1).  NaN: unsafe.
__device__ __forceinline__ bool mixUnsafe(float3 inv, float lim) {
    const float x = fabsf(inv.x), y = fabsf(inv.y), z = fabsf(inv.z);
    return !(x <= lim) || !(y <= lim) || !(z <= lim);
}

// RenderManager::hitBvh (render_manager.h:86-135): same visiting order (left child, right
// child, leaf children tested at once, internal children pushed left then right).
// Returns the leaf slot of the closest hit or -1; `closest` holds its t.
template <int STACK>
__device__ __forceinline__ int trace(const DevScene& S, float3 o, float3 d, float tmin, float& closest,
                                     uint32_t* stk, Counters& c) {
    int best = -1;
    if (S.nprims <= 0) return -1;
    if (S.nprims == 1) {   // root is a leaf: tested without a box test (:92-98)
        const uint32_t ref = kLeafBit | (__float_as_uint(S.prims[2].w) ? kSphereBit : 0u);
        primTest(S, ref, o, d, tmin, closest, best, c);
        return best;
    }
    const float3 inv = f3(rcpRN(d.x), rcpRN(d.y), rcpRN(d.z));
    int node = 0, sp = 0, guard = 0;
    for (;;) {
        // Each internal node is visited at most once per query; more means a corrupt tree.
        if (++guard > S.nprims) { atomicOr(S.err, 1u); break; }
        c.visits++;
        const float4* np = S.nodes + 4 * (size_t)node;
        const float4 a = np[0], b = np[1], q = np[2], r = np[3];
        const uint32_t lref = __float_as_uint(r.x), rref = __float_as_uint(r.y);
        if (slabLeft(a, b, o, inv, tmin, closest).hit) {
            if (lref & kLeafBit) primTest(S, lref, o, d, tmin, closest, best, c);
            else if (sp < STACK) { stk[sp * kWave] = lref; sp++; }
            else { atomicOr(S.err, 2u); break; }
        }
        if (slabRight(b, q, o, inv, tmin, closest).hit) {
            if (rref & kLeafBit) primTest(S, rref, o, d, tmin, closest, best, c);
            else if (sp < STACK) { stk[sp * kWave] = rref; sp++; }
            else { atomicOr(S.err, 2u); break; }
        }
        if (sp == 0) break;
        sp--;
        node = (int)stk[sp * kWave];
    }
    return best;
}

// RenderManager::hitBvh (render_manager.h:86-135) without a stack, for the wide kernels' rare
// order-dependent queries: the same primitive tests in the same order with the same `closest`.
// The reference pushes an internal child when its box passes at the parent's visit and pops
// right before left; here a child is entered when its box passes at the moment it would be
// popped (parent links lead back up).  A box that passed earlier but fails now has children
// that all fail now (their boxes are inside it; correctly rounded slab arithmetic is monotonic),
// so skipping it changes no primitive test.  Returns the leaf k of the closest hit or -1.
__device__ __forceinline__ int traceRefStackless(const DevScene& S, float3 o, float3 d, float tmin, float& closest) {
    int best = -1;
    if (S.nprims <= 0) return -1;
    if (S.nprims == 1) {   // root is a leaf: tested without a box test (:92-98)
        const float t1 = primHitT(loadPrim(S, 0), __float_as_uint(S.prims[2].w) != 0, o, d, tmin, closest);
        if (t1 >= 0.0f) { closest = t1; best = 0; }
        return best;
    }
    const float3 inv = f3(rcpRN(d.x), rcpRN(d.y), rcpRN(d.z));
    int node = 0, from = -1;   // from >= 0: returning from that child of `node`
    bool finished = false;
    for (int guard = 0; guard <= 4 * S.nprims; guard++) {   // each node is entered and left once
        const float4* np = S.nodes + 4 * (size_t)node;
        const float4 a = np[0], b = np[1], q = np[2], r = np[3];
        const uint32_t lref = __float_as_uint(r.x), rref = __float_as_uint(r.y);
        int next = -1;
        if (from < 0) {   // visit: the leaf children in order, then the right subtree, then the left
            const SlabHit hl = slabLeft(a, b, o, inv, tmin, closest);
            if (hl.hit && (lref & kLeafBit)) {
                const float t = primHitT(loadPrim(S, lref & kPrimMask), (lref & kSphereBit) != 0, o, d, tmin, closest);
                if (t >= 0.0f) { closest = t; best = (int)(lref & kPrimMask); }
            }
            const SlabHit hr = slabRight(b, q, o, inv, tmin, closest);
            if (hr.hit && (rref & kLeafBit)) {
                const float t = primHitT(loadPrim(S, rref & kPrimMask), (rref & kSphereBit) != 0, o, d, tmin, closest);
                if (t >= 0.0f) { closest = t; best = (int)(rref & kPrimMask); }
            }
            if (hr.hit && !(rref & kLeafBit)) next = (int)rref;
            else if (!(lref & kLeafBit) && slabLeft(a, b, o, inv, tmin, closest).hit) next = (int)lref;
        } else if ((uint32_t)from == rref && !(lref & kLeafBit) && slabLeft(a, b, o, inv, tmin, closest).hit) {
            next = (int)lref;
        }
        if (next >= 0) {
            node = next;
            from = -1;
        } else {
            if (node == 0) { finished = true; break; }
            from = node;
            node = S.iparent[node];
        }
    }
    if (!finished) atomicOr(S.err, 4u);   // a corrupt tree or parent links: reported, never silent
    return best;
}

// Hit record for leaf slot k at distance t (cuda_object.h:62-67 / 85-88, hit_record.h:21-24),
// with the hit object's material (material.h:17-68) carried along: the three independent 16-B
// loads of the shading record are one memory round trip (instead of prim -> normal -> material).
struct HitRec { float3 p, n; int mat, obj; bool front; float4 m0; float ir; int type; };

__device__ __forceinline__ HitRec makeHitFrom(const float4* shade, int k, float t, float3 o, float3 d) {
    HitRec h;
    const float4* r = shade + 3 * (size_t)k;
    const float4 s0 = r[0], s1 = r[1], s2 = r[2];
    const uint32_t tf = __float_as_uint(s2.y);
    h.p = add(o, scale(t, d));
    float3 outward;
    if (tf >> 16) {   // sphere: (p - c) / r
        outward = divs(sub(h.p, xyz(s0)), s0.w);
    } else {
        outward = xyz(s0);
    }
    h.front = dot3(d, outward) < 0.0f;
    h.n = h.front ? outward : neg(outward);
    h.mat = (int)__float_as_uint(s2.z);
    h.obj = (int)__float_as_uint(s2.w);
    h.m0 = s1;
    h.ir = s2.x;
    h.type = (int)(tf & 0xffffu);
    return h;
}
__device__ __forceinline__ HitRec makeHit(const DevScene& S, int k, float t, float3 o, float3 d) {
    return makeHitFrom(S.shade, k, t, o, d);
}

// Instanced scenes: the world ray (o, d) entering an instance, in its object space (rows r0..r2 of
// the world-to-object transform; the hit distance t is the same parameter in both spaces).
__device__ __forceinline__ float3 xformPoint(float4 r0, float4 r1, float4 r2, float3 p) {
    return f3(((r0.x * p.x + r0.y * p.y) + r0.z * p.z) + r0.w, ((r1.x * p.x + r1.y * p.y) + r1.z * p.z) + r1.w,
              ((r2.x * p.x + r2.y * p.y) + r2.z * p.z) + r2.w);
}
__device__ __forceinline__ float3 xformDir(float4 r0, float4 r1, float4 r2, float3 v) {
    return f3((r0.x * v.x + r0.y * v.y) + r0.z * v.z, (r1.x * v.x + r1.y * v.y) + r1.z * v.z,
              (r2.x * v.x + r2.y * v.y) + r2.z * v.z);
}
// Hit record of instance key `key` (instance << gBits | shading index) at distance t of the world
// ray: the object-space shading record, the outward normal returned to the world by the inverse
// transpose and normalised (cuda_object.h:62-67 / 85-88 in object space, hit_record.h:21-24 in the
// world); an instance whose linear part is the identity (a translation) keeps the record's normal as
// is, the flattened scene's arithmetic.
__device__ __forceinline__ HitRec makeHitInst(const DevScene& S, uint32_t key, float t, float3 o, float3 d, int& obj) {
    const uint32_t inst = key >> S.gBits, g = key & ((1u << S.gBits) - 1u);
    const float4* ir = S.winst + 4 * (size_t)inst;
    const float4 r0 = ir[0], r1 = ir[1], r2 = ir[2], ex = ir[3];
    const float4* r = S.wshade + 3 * (size_t)g;
    const float4 s0 = r[0], s1 = r[1], s2 = r[2];
    const uint32_t tf = __float_as_uint(s2.y);
    const bool ident = __float_as_uint(ex.y) == 1u, linIdent = __float_as_uint(ex.y) != 0u;
    HitRec h;
    h.p = add(o, scale(t, d));
    float3 outward;
    if (tf >> 16) {   // sphere: (p - c) / r in object space
        const float3 po = ident ? h.p : xformPoint(r0, r1, r2, h.p);
        outward = divs(sub(po, xyz(s0)), s0.w);
    } else {
        outward = xyz(s0);
    }
    if (!linIdent) {   // n_world = normalize(A^-T n_object): A^-1's columns dotted with n
        const float3 n = outward;
        outward = normalize3(f3((r0.x * n.x + r1.x * n.y) + r2.x * n.z, (r0.y * n.x + r1.y * n.y) + r2.y * n.z,
                                (r0.z * n.x + r1.z * n.y) + r2.z * n.z));
    }
    h.front = dot3(d, outward) < 0.0f;
    h.n = h.front ? outward : neg(outward);
    h.mat = (int)__float_as_uint(s2.z);
    obj = (int)(__float_as_uint(ex.x) + __float_as_uint(s2.w));   // the object's index in the flattened order
    h.obj = obj;
    h.m0 = s1;
    h.ir = s2.x;
    h.type = (int)(tf & 0xffffu);
    return h;
}

// ------------------------------------------------------------------------ BSDFs
// utility.h:51-62 / 73-82; vec3(...) arguments drawn x, y, z in order.
template <class G>
__device__ __forceinline__ float3 onUnitSphere(G& g) {
    float3 res;
    float norm;
    do {   // draws x, y, z in order; centered2() = 2 * (uniform() - 0.5f) exactly
        const float a = g.centered2();
        const float b = g.centered2();
        const float cz = g.centered2();
        res = f3(a, b, cz);
        norm = len2(res);
    } while (!PT_AB_ONE_TRIAL && norm >= 1.0f);
    return divs(res, sqrtf(norm));
}
template <class G>
__device__ __forceinline__ float3 inUnitSphere(G& g) {
    float3 res;
    do {
        const float a = g.centered2();
        const float b = g.centered2();
        const float cz = g.centered2();
        res = f3(a, b, cz);
    } while (len2(res) >= 1.0f);
    return res;
}
__device__ __forceinline__ float3 reflect3(float3 v, float3 n) { return sub(v, scale(2.0f * dot3(v, n), n)); }

// Material::scatter (material.h:28-61); returns false when the path is absorbed.
template <class G>
__device__ __forceinline__ bool scatter(const DevScene& S, const HitRec& h, float3& d, float3& atten, G& g) {
    (void)S;
    const float4 m0 = h.m0;
    const int type = h.type;
    if (type == PT_LAMBERTIAN) {
        float3 dir = add(h.n, onUnitSphere(g));
        if (fabsf(dir.x) < 1e-7f && fabsf(dir.y) < 1e-7f && fabsf(dir.z) < 1e-7f) dir = h.n;
        d = dir;
        atten = xyz(m0);
        return true;
    }
    if (type == PT_METAL) {
        float3 refl = reflect3(normalize3(d), h.n);
        float3 fz = inUnitSphere(g);
        d = add(refl, scale(m0.w, fz));
        atten = xyz(m0);
        return dot3(d, h.n) > 0.0f;
    }
    if (type == PT_DIELECTRIC) {
        atten = f3(1.0f, 1.0f, 1.0f);
        const float ir = h.ir;
        float ratio = h.front ? rcpRN(ir) : ir;
        float3 ud = normalize3(d);
        float cos_t = fminf(dot3(neg(ud), h.n), 1.0f);
        float sin_t = sqrtf(1.0f - cos_t * cos_t);
        bool cannot = ratio * sin_t > 1.0f;
        bool refl = cannot;
        if (!cannot) {   // reflectance (physical.h:20-25), pow(x,5) = ((x*x)*(x*x))*x
            float r0 = (1.0f - ratio) / (1.0f + ratio);
            r0 = r0 * r0;
            float x = 1.0f - cos_t;
            float x2 = x * x;
            float rf = r0 + (1.0f - r0) * ((x2 * x2) * x);
            refl = rf > g.uniform();
        }
        if (refl) {
            d = reflect3(ud, h.n);
        } else {   // refract (physical.h:14-19)
            float ct = fminf(dot3(neg(ud), h.n), 1.0f);
            float3 perp = scale(ratio, add(ud, scale(ct, h.n)));
            float3 par = scale(-sqrtf(fabsf(1.0f - len2(perp))), h.n);
            d = add(perp, par);
        }
        return true;
    }
    return false;
}

// scatter() with the attenuation applied in place (att *= albedo for Lambertian and metal): the
// dielectric's (1, 1, 1) is skipped, exactly (x * 1.0f == x for the finite attenuations of a
// path), and no attenuation value has to live across the material switch.
template <class G>
__device__ __forceinline__ bool scatterInto(const HitRec& h, float3& d, float3& att, G& g) {
    const float4 m0 = h.m0;
    const int type = h.type;
    if (type == PT_LAMBERTIAN) {
        float3 dir = add(h.n, onUnitSphere(g));
        if (fabsf(dir.x) < 1e-7f && fabsf(dir.y) < 1e-7f && fabsf(dir.z) < 1e-7f) dir = h.n;
        d = dir;
        att = mul(att, xyz(m0));
        return true;
    }
    if (type == PT_METAL) {
        float3 refl = reflect3(normalize3(d), h.n);
        float3 fz = inUnitSphere(g);
        d = add(refl, scale(m0.w, fz));
        att = mul(att, xyz(m0));
        return dot3(d, h.n) > 0.0f;
    }
    if (type == PT_DIELECTRIC) {
        const float ir = h.ir;
        float ratio = h.front ? rcpRN(ir) : ir;
        float3 ud = normalize3(d);
        float cos_t = fminf(dot3(neg(ud), h.n), 1.0f);
        float sin_t = sqrtf(1.0f - cos_t * cos_t);
        bool cannot = ratio * sin_t > 1.0f;
        bool refl = cannot;
        if (!cannot) {   // reflectance (physical.h:20-25), pow(x,5) = ((x*x)*(x*x))*x
            float r0 = (1.0f - ratio) / (1.0f + ratio);
            r0 = r0 * r0;
            float x = 1.0f - cos_t;
            float x2 = x * x;
            float rf = r0 + (1.0f - r0) * ((x2 * x2) * x);
            refl = rf > g.uniform();
        }
        if (refl) {
            d = reflect3(ud, h.n);
        } else {   // refract (physical.h:14-19)
            float ct = fminf(dot3(neg(ud), h.n), 1.0f);
            float3 perp = scale(ratio, add(ud, scale(ct, h.n)));
            float3 par = scale(-sqrtf(fabsf(1.0f - len2(perp))), h.n);
            d = add(perp, par);
        }
        return true;
    }
    return false;
}

// Sky (main.cu:34-36) times attenuation.
__device__ __forceinline__ float3 sky(float3 d, float3 att) {
    float3 ud = normalize3(d);
    float t = 0.5f * (ud.y + 1.0f);
    float3 c = add(scale(1.0f - t, f3(1.0f, 1.0f, 1.0f)), scale(t, f3(0.5f, 0.7f, 1.0f)));
    return mul(c, att);
}

// ------------------------------------------------------------------------ kernels
struct RenderParams {
    DevScene S;
    DevCamera cam;
    uint32_t *sd, *s0, *s1, *s2, *s3, *s4;   // film RNG state, SoA over local pixels
    float* out;
    unsigned long long* counters;             // rays, visits, tris, spheres, paths
    int width, nrows, stripe_h, nparts, part;
    int tiles_x, ntiles;
    int spp, max_depth;
    float invW, invH, invSpp;
    int leafBatch, shadeBatch;                // wavefront scheduler thresholds (lanes)
    int nodeMin;                              // compat: below this many NODE lanes, run the larger of LEAF / SHADE
    int kernel;                               // PT_KERNEL_*
    unsigned long long* waveTimes;            // optional (PT_WAVE_TIMES): {start, end, tile|xcc<<32} per wave
    const int* tileOrder;                     // launch order of tiles (longest first), or null = identity
    const uint32_t* tileXY;                   // sample mode: tile of each launch slot as tx | ty << 16 (the order decoded)
    int nblocksShift;                         // sample mode: log2(ngroups) when a power of two, else -1
    unsigned* tileCost;                       // out: per-tile wave duration (s_memrealtime ticks, 100 MHz)
    int prioTiles;                            // the first prioTiles tiles of the order run at s_setprio prioLevel
    int prioLevel;                            // 1-3 (s_setprio's user priority; added to the wave's age in issue arbitration)
    // sample mode (RNG_SAMPLE): samples are summed in fixed blocks of `block` samples.  Each
    // (pixel, block) is one task, summed in sample order (fp32) by whichever lane takes it; the
    // block sum is then added to the pixel's accumulator as a 32.32 fixed-point integer
    // (blockFixed), with atomics: integer addition is exact and order-free, so the image does
    // not depend on scheduling or on the stripe partition.  pixAcc[4 * pixel] = {x, y, z, rays}.
    int nblocks, block;
    // A task covers `group` consecutive summation blocks of one pixel (`span` = group x block samples;
    // ngroups spans per pixel): each block's fixed-point sum is added into the lane's LDS partial,
    // and the task adds the partial to the pixel's accumulator once (3 global atomics per task, not
    // per block).  The fixed-point additions are exact and order-free: the image does not change.
    int group, span, ngroups;
    unsigned long long* pixAcc;
    unsigned* taskCounter;                    // next task (zeroed before the launch)
    uint32_t* stackSpill;                     // sample mode, STACK > 32: stack entries >= 32 (per wave slot, lane)
    uint32_t ntasks;                          // tile slots x ngroups x 64
    int nwaves;                               // persistent waves launched
    uint32_t seed0, seed1;
    uint32_t sampleBase;                      // sample mode: index of the frame's first sample
    int measureCost;                          // sample mode: count rays per pixel for the tile order
    int camFar;                               // wide: the camera lies beyond the wide boxes' margin (wideFar)
    int rawOut;                               // compat: store the raw sample sum (resolveKernel follows)
    int stripeShift, blockShift;              // log2(stripe_h), log2(block) when powers of two, else -1
    int splitTiles, splitWays;                // compat: the longest tiles run as splitWays waves each
    int compatGrid;                           // compat (tile waves): critWaves + ntiles + splitTiles * (splitWays - 1)
    // compat, critical pixels (wide kernel): the nCrit pixels of critList (the previous launch's
    // longest chains) run first, critLanes per wave (blocks 0 .. critWaves - 1), each lane taking its
    // pixel's whole chain with a per-lane closest-hit traversal inside the ray start (no NODE / LEAF
    // steps); tile waves skip the pixels critFlag marks.  pixRays (optional): rays per pixel.
    int nCrit, critLanes, critWaves;
    const uint32_t* critList;
    const uint8_t* critFlag;
    uint32_t* pixRays;
};

// (blockFixed, blockFixedSmall, fixedToFloat: pt_math.hpp)
// One finished (pixel, block) task: its sum added to the pixel's accumulator, and -- on frames
// that measure tile costs (`cost`: the input of the next launches' longest-first order) -- its ray
// count; no-return atomics (device scope: 4 of them per task cost 5 % of a C3 frame, so the ray
// counts are taken on one frame in eight).
// compat critical pixels: how many (PT_CRIT_PIXELS) and how many per wave (PT_CRIT_LANES)
#ifndef PT_CRIT_PIXELS
#define PT_CRIT_PIXELS 256
#endif
#ifndef PT_CRIT_LANES
#define PT_CRIT_LANES 4
#endif
constexpr int kCritPixels = PT_CRIT_PIXELS;
constexpr int kCritLanes = PT_CRIT_LANES;
// which compat kernels have critical-pixel waves: the flattened wide tree on shallow trees (stack 8:
// the 4-waves/SIMD compat kernels, whose 128-VGPR budget holds the per-lane loop without spills)
__host__ __device__ constexpr bool critFor(bool sample, bool wide, bool inst, bool cq, int stack) {
    return !sample && wide && !inst && !cq && stack <= 8;
}
__device__ __forceinline__ __attribute__((unused)) void addFixed1(unsigned long long* acc, unsigned long long v) {
#if PT_AB_NO_ATOMICS
    return;
#endif
    __hip_atomic_fetch_add(acc, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void addBlock(unsigned long long* acc, float3 sum, uint32_t rays, bool cost) {
#if PT_AB_NO_ATOMICS
    return;
#endif
    // the common case -- every finishing lane's three sums in [0, 2^24), NaN excluded by the >= 0
    // tests -- takes blockFixedSmall (a wave-uniform branch on the ballot)
    const bool small = sum.x >= 0.0f && sum.y >= 0.0f && sum.z >= 0.0f &&
                       fmaxf(fmaxf(sum.x, sum.y), sum.z) < 16777216.0f;
    unsigned long long fx, fy, fz;
    if (PT_FIXED_SMALL && __ballot(!small) == 0) {
        fx = blockFixedSmall(sum.x); fy = blockFixedSmall(sum.y); fz = blockFixedSmall(sum.z);
    } else {
        fx = blockFixed(sum.x); fy = blockFixed(sum.y); fz = blockFixed(sum.z);
    }
    __hip_atomic_fetch_add(acc + 0, fx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(acc + 1, fy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(acc + 2, fz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cost) __hip_atomic_fetch_add(acc + 3, (unsigned long long)rays, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Compat mode end of a pixel: sqrt(sum / spp) (main.cu:290-293), or the raw sum when a resolve
// pass (accumulation / 8-bit output) follows.
__device__ __forceinline__ void storePixel(const RenderParams& P, size_t idx, float3 sum) {
    float* outp = P.out + 3 * idx;
    if (P.rawOut) {
        outp[0] = sum.x; outp[1] = sum.y; outp[2] = sum.z;
    } else {
        outp[0] = sqrtf(sum.x * P.invSpp);
        outp[1] = sqrtf(sum.y * P.invSpp);
        outp[2] = sqrtf(sum.z * P.invSpp);
    }
}

// shift: log2(sh) when sh is a power of two, else -1 (shifts instead of two VALU divisions)
__device__ __forceinline__ int globalRowFast(int lrow, int sh, int shift, int nparts, int part) {
    if (nparts == 1) return lrow;
    if (shift >= 0) return ((((lrow >> shift) * nparts + part)) << shift) + (lrow & (sh - 1));
    return ((lrow / sh) * nparts + part) * sh + lrow % sh;
}
__device__ __forceinline__ int globalRow(int lrow, int sh, int nparts, int part) {
    return ((lrow / sh) * nparts + part) * sh + lrow % sh;
}

// Tile scheduling.  Workgroups are dispatched in blockIdx order and dealt round-robin over the 8
// XCDs, so consecutive tiles land on different XCDs (balanced; the C3 BVH fits every L2).  When
// the film has measured per-tile costs from a previous launch, tiles are launched longest first
// (LPT): a tile's 1024 samples per pixel are sequential (per-pixel RNG stream), so the most
// expensive tiles are the critical path and must start first.  Scheduling never changes results.
__device__ __forceinline__ int tileOf(const RenderParams& P, int bid) {
    return P.tileOrder ? P.tileOrder[bid] : bid;
}

__device__ __forceinline__ void waveReduceAdd(unsigned long long* dst, uint32_t v) {
    unsigned long long x = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0 && x) atomicAdd(dst, x);
}

// SAMPLE: the sample-mode streams and block sums, one wave per tile, samples in order -- the
// same frame as renderKernelWF<STACK, true>, in the reference's traversal order (the bench
// counts algorithmic bytes with it).
// Lens sample of camera::get_ray (camera.h:58-62): a uniform point of the unit disk scaled by the
// lens radius, offset along right / up.  The reference draws it in polar form (utility.h:98-102:
// sqrtf, cosf, sinf) from the SHARED state randState[0] (main.cu:286, raced by every thread), so
// its lens samples are not reproducible; here they come from the path's own stream, right after
// the pixel jitter, by rejection (x, y in [-1, 1) until x^2 + y^2 < 1: the same uniform disk, and
// no transcendental, so the oracle's arithmetic is the kernel's bit for bit).
template <class G>
__device__ __forceinline__ void lensOffset(float3 right, float3 up, float lens, G& g, float3& o, float3& d) {
    float x, y;
    do {
        x = 2.0f * (g.uniform() - 0.5f);
        y = 2.0f * (g.uniform() - 0.5f);
    } while (x * x + y * y >= 1.0f);
    const float rx = lens * x, ry = lens * y;
    const float3 off = add(scale(rx, right), scale(ry, up));
    o = add(o, off);
    d = sub(d, off);
}

template <int STACK, bool SAMPLE>
__global__ __launch_bounds__(kWave) void renderKernel(RenderParams P) {
    __shared__ uint32_t stk[STACK * kWave];
    const int lane = threadIdx.x;
    const int tile = tileOf(P, blockIdx.x);
    const unsigned long long tStart = __builtin_amdgcn_s_memrealtime();
    const int tx = tile % P.tiles_x, ty = tile / P.tiles_x;
    const int col = tx * 8 + (lane & 7);
    const int lrow = ty * 8 + (lane >> 3);
    const bool valid = col < P.width && lrow < P.nrows;
    Counters c{0, 0, 0, 0};
    uint32_t paths = 0;
    if (valid) {
        const size_t idx = (size_t)lrow * P.width + col;
        const int row = globalRow(lrow, P.stripe_h, P.nparts, P.part);
        Xorwow g{};
        if constexpr (!SAMPLE) g = Xorwow{P.sd[idx], P.s0[idx], P.s1[idx], P.s2[idx], P.s3[idx], P.s4[idx]};
        const uint32_t gpix = (uint32_t)row * (uint32_t)P.width + (uint32_t)col;
        const float fcol = (float)col, frow = (float)row;
        float3 sum = f3(0.0f, 0.0f, 0.0f);
        float3 o, d, att;
        int depthLeft = 0, sample = 0;
        // newPath: main.cu:284-286 + camera::get_ray (camera.h:58-64): the lens sample from the
        // path's stream (lensOffset), the time draw skipped (no moving objects on the path).
        auto newPath = [&]() {
            if constexpr (SAMPLE) g = sampleStream(P.seed0, P.seed1, P.sampleBase + (uint32_t)sample, gpix);
            float u = (fcol + g.uniform()) * P.invW;
            float v = (frow + g.uniform()) * P.invH;
            o = P.cam.pos;
            d = sub(add(add(P.cam.ll, scale(u, P.cam.hor)), scale(v, P.cam.ver)), P.cam.pos);
            if (P.cam.lens != 0.0f) lensOffset(P.cam.right, P.cam.up, P.cam.lens, g, o, d);
            att = f3(1.0f, 1.0f, 1.0f);
            depthLeft = P.max_depth;
            paths++;
        };
        // sample mode: close summation block `b` after its last sample (its sum and its ray count,
        // the tile-cost input of the next launch's longest-first order)
        uint32_t blockRays0 = 0;
        auto flush = [&]() {
            if constexpr (SAMPLE) {
                if (sample % P.block == 0 || sample == P.spp) {
                    addBlock(P.pixAcc + 4 * idx, sum, c.rays - blockRays0 + 1u, P.measureCost != 0);
                    blockRays0 = c.rays;
                    sum = f3(0.0f, 0.0f, 0.0f);
                }
            }
        };
        if (P.max_depth <= 0) {
            while (sample < P.spp) { newPath(); sum = add(sum, sky(d, att)); sample++; flush(); }
        } else if (P.spp > 0) {
            newPath();
            uint32_t* my = stk + lane;
            for (;;) {
                // one bounce of rayTracing (main.cu:26-33) for this lane's current path
                c.rays++;
                depthLeft--;
                float closest = __builtin_inff();
                const int k = trace<STACK>(P.S, o, d, 0.001f, closest, my, c);
                bool done = false;
                float3 contrib;
                if (k < 0) {
                    contrib = sky(d, att);
                    done = true;
                } else {
                    HitRec h = makeHit(P.S, k, closest, o, d);
                    float3 na;
                    if (!scatter(P.S, h, d, na, g)) {
                        contrib = f3(0.0f, 0.0f, 0.0f);
                        done = true;
                    } else {
                        att = mul(att, na);
                        o = h.p;
                        if (depthLeft == 0) { contrib = sky(d, att); done = true; }
                    }
                }
                if (done) {
                    sum = add(sum, contrib);
                    ++sample;
                    flush();
                    if (sample == P.spp) break;
                    newPath();
                }
            }
        }
        if constexpr (!SAMPLE) {
            storePixel(P, idx, sum);
            P.sd[idx] = g.d; P.s0[idx] = g.v0; P.s1[idx] = g.v1; P.s2[idx] = g.v2; P.s3[idx] = g.v3; P.s4[idx] = g.v4;
        }
    }
    if (!SAMPLE && lane == 0) P.tileCost[tile] = (unsigned)min(__builtin_amdgcn_s_memrealtime() - tStart, 0xffffffffull);
    waveReduceAdd(P.counters + 0, c.rays);
    waveReduceAdd(P.counters + 1, c.visits);
    waveReduceAdd(P.counters + 2, c.tris);
    waveReduceAdd(P.counters + 3, c.spheres);
    waveReduceAdd(P.counters + 4, paths);
}


// Wavefront-scheduled render kernel (speculative while-while, exact).
// Each lane runs the same per-pixel program as renderKernel, decomposed into three step kinds;
// every loop iteration runs ONE kind, chosen from wave-wide __ballot counts (a uniform scalar
// branch), for all lanes that have that kind of work:
//   NODE : visit one internal node: test both child boxes against the lane's current `closest`;
//          hit leaves are appended to the lane's leaf queue (DFS order), hit internal children
//          are pushed / descended into (the reference's order: right subtree first).
//   LEAF : take the oldest queued leaf, RE-TEST its box against the current `closest`, then run
//          the primitive test (cuda_object.h:44-92).
//   SHADE: hit record + scatter + path bookkeeping + next ray (main.cu:26-36, 283-289).
// Exactness: leaves are tested in the reference's DFS order, each with the same `closest` the
// reference would use (only primitive tests change `closest`), and a box that fails with a
// stale (larger) `closest` also fails with the true one (the slab interval shrinks
// monotonically with tmax and with the box).  Node boxes tested with a stale `closest` only
// add visits.  So the sequence of primitive tests -- and every pixel -- is identical to the
// reference order; node visit counts may be higher.  Lanes keep traversing while leaves wait,
// so primitive tests run with many lanes active instead of one or two.
#ifndef PT_LEAF_QUEUE
#define PT_LEAF_QUEUE 4
#endif
constexpr int kLeafQ = PT_LEAF_QUEUE;
#ifndef PT_LEAF_QUEUE_SAMPLE
#define PT_LEAF_QUEUE_SAMPLE 2   // sample mode, binary tree, STACK <= 32; compat prefers 4 (C3 1774 vs 1959 ms)
#endif
#ifndef PT_TASK_POOL
#define PT_TASK_POOL 64
#endif
constexpr int kTaskPool = PT_TASK_POOL;   // sample mode: tasks a wave reserves per atomic
// Experiment (off): XCD-local task pools.  The tile slots are dealt to 8 counters (slot % 8), a
// wave drains the counter of its XCD (blockIdx % 8: workgroups are dispatched to the XCDs round
// robin) and then the others in turn, so each XCD's L2 sees the rays of an eighth of the tiles
// in flight.  Exact by construction: the image does not depend on which lane runs a task.
#ifndef PT_XCD_POOLS
#define PT_XCD_POOLS 0
#endif
static_assert(!PT_XCD_POOLS || PT_TASK_POOL == 64, "XCD pools hand out whole (tile, block) groups");
#ifndef PT_TASK_GROUPS
#define PT_TASK_GROUPS 0   // wide sample kernels: tasks of several summation blocks (LDS partials; measured slower)
#endif
#ifndef PT_TASK_BLOCKS
#define PT_TASK_BLOCKS 2
#endif
constexpr int kTaskBlocks = PT_TASK_BLOCKS;   // sample mode: summation blocks per task (PT_TASK_BLOCKS env overrides)
// Occupancy target of the wavefront kernel (waves per SIMD; 6 = at most 80 VGPRs).  The LDS
// stack (STACK x 256 B per wave, 160 KB per CU) allows 6 / 5 / 4 / 3 / 2 waves per SIMD at
// STACK 24 / 32 / 48 / 64 / 80, so deeper trees keep a larger register budget.  Compat tile
// mode measured best at 5 (C3 1,617 vs 1,675 ms at 6).  Sample mode on C3 (STACK 24):
// 4 waves 910 ms, 5 waves 815 ms, 6 waves 754 ms.
#ifndef PT_WAVES_PER_EU
#define PT_WAVES_PER_EU 6
#endif
#ifndef PT_STACK24
#define PT_STACK24 1   // STACK 24 instantiations (C3: depth + 1 <= 24): 6 waves per SIMD fit the LDS
#endif
#ifndef PT_LDS_STACK
#define PT_LDS_STACK 32   // sample mode: traversal stack entries per lane kept in LDS
#endif
template <int STACK, bool SAMPLE, bool WIDE>
constexpr int kLdsStack = (!WIDE && STACK > PT_LDS_STACK) ? PT_LDS_STACK : STACK;
#ifndef PT_AB_NO_SPLIT
#define PT_AB_NO_SPLIT 0   // (A/B only: compile the compat split-tile prologue out)
#endif
#ifndef PT_AB_COST_STORE
#define PT_AB_COST_STORE 0   // (A/B only: compat tile costs stored, not atomicMax'ed -- wrong with split tiles)
#endif
#ifndef PT_COMPAT_QUEUE
#define PT_COMPAT_QUEUE 0   // compat mode: persistent waves take pixels from a queue (else one wave per tile; 1 measured slower)
#endif
#ifndef PT_WIDE_SPEC
#define PT_WIDE_SPEC 1   // wide kernels: speculative traversal, primitive groups a lane may park while it keeps visiting nodes (0-3)
#endif
#ifndef PT_INST_SPEC
#define PT_INST_SPEC 0   // instanced wide kernels: speculative traversal within an instance's tree (0-1; 1 measured 3 % slower on C5 instanced)
#endif
#ifndef PT_WIDE_MIX
#define PT_WIDE_MIX 1   // wide kernels: plane distances by v_perm + v_fma_mix_f32 (wideHits<MIX>), bit-identical
#endif
#ifndef PT_MIX_CHECK
#define PT_MIX_CHECK 1   // (A/B timing only: 0 drops the per-ray mixUnsafe test -- not exact for near-axis rays)
#endif
#ifndef PT_LEAF_COOP
#define PT_LEAF_COOP 0   // wide kernels (not instanced): wave-cooperative LEAF steps, one (lane, primitive) pair per lane
#endif
#ifndef PT_LEAF_COOP_CAP
#define PT_LEAF_COOP_CAP 2   // pairs a lane offers per cooperative LEAF step (1-3)
#endif
#ifndef PT_WIDE_WAVES_PER_EU
#define PT_WIDE_WAVES_PER_EU 5   // wide tree (96 VGPRs; the stack never limits occupancy): C3 @64 spp 49.7 ms vs 68.8 at 6 (spills), 51.4 at 4
#endif
// Compat-mode wide kernels (pt_compat.hip) on shallow trees (STACK 8: C2, C3) at 4 waves per SIMD
// (104 VGPRs): C3 @1024 spp 806-825 -> 796-798 ms over three runs each, C2 @256 40.0-41.1 ->
// 41.0-41.4; deeper trees keep 5 (C5 @512: 552-558 at 5, 602-605 at 4).
#ifndef PT_COMPAT_WIDE_WAVES_PER_EU
#define PT_COMPAT_WIDE_WAVES_PER_EU 4
#endif
template <int STACK, bool SAMPLE, bool WIDE>
constexpr int kWavesPerEU = WIDE ? (SAMPLE || STACK > 8 ? PT_WIDE_WAVES_PER_EU : PT_COMPAT_WIDE_WAVES_PER_EU)
                                 : kLdsStack<STACK, SAMPLE, WIDE> <= 24
                                ? (SAMPLE ? PT_WAVES_PER_EU : 5)
                                : (kLdsStack<STACK, SAMPLE, WIDE> <= 32
                                       ? 5
                                       : (kLdsStack<STACK, SAMPLE, WIDE> <= 48 ? 4 : (STACK <= 64 ? 3 : 2)));

// WIDE: traverse the compressed 8-wide tree (wnodes / wprims, host/pt_wide8.cpp) instead of the
// binary LBVH.  Per lane: a node group `ng` (child base << 8 | hit internal slots, in slot ^ oct
// order, the nearest first), a primitive group (tgBase, tg = hit leaf primitives); NODE takes the
// next child of the group (pushing the rest), LEAF tests up to two primitives, keeping the
// minimum (t, tie rank) of wideTest -- the reference's closest hit, in any visiting order.
// Kernel arguments re-read from the kernarg segment where a rare step needs them (one scalar
// load) instead of being held in SGPRs across the step loop: the loop's uniform state exceeded
// the SGPR budget and the compiler parked the overflow in VGPR lanes, paying a v_readlane -- a
// VALU issue slot in an issue-bound kernel -- per use.  The empty asm hides the pointer's origin
// so the loads are not hoisted out of the loop again.
typedef const __attribute__((address_space(4))) RenderParams* KArgs;
__device__ __forceinline__ KArgs kargs() {
    KArgs k = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));
    return k;
}

typedef const __attribute__((address_space(4))) float KFloat;
typedef const __attribute__((address_space(4))) uint32_t* KU32;   // read-only launch tables, scalar loads
__device__ __forceinline__ float3 ld3(const __attribute__((address_space(4))) float3& v) {
    KFloat* f = (KFloat*)&v;
    return f3(f[0], f[1], f[2]);
}
__device__ __forceinline__ DevScene ldScene(KArgs k) {
    DevScene S;
    S.nodes = k->S.nodes; S.prims = k->S.prims; S.shade = k->S.shade; S.mats = k->S.mats;
    S.wnodes = k->S.wnodes; S.wprims = k->S.wprims; S.wshade = k->S.wshade; S.rankOf = k->S.rankOf;
    S.iparent = k->S.iparent; S.err = k->S.err; S.nprims = k->S.nprims;
    S.hasSpheres = k->S.hasSpheres;
    S.cx = k->S.cx; S.cy = k->S.cy; S.cz = k->S.cz; S.ext = k->S.ext;
    S.mixLim = k->S.mixLim;
    S.winst = k->S.winst; S.gBits = k->S.gBits;
    return S;
}

// INST (with WIDE): an instanced scene's two-level tree (pt_scene_create_instanced): a NODE step
// that reaches an instance record moves the lane's ray into the instance's object space and its
// bottom-level tree, a stack marker brings it back; no speculative traversal (a parked primitive
// group would belong to another space), no reference-order redo (instanced frames are held to a
// tolerance, not bit for bit).
template <int STACK, bool SAMPLE, bool WIDE, bool INST = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kWavesPerEU<STACK, SAMPLE, WIDE>))) void renderKernelWF(RenderParams P) {
    // Deep trees (binary kernels) keep 32 stack entries per lane in LDS (8 KB per wave: 5 waves
    // per SIMD) and the rare deeper entries in global memory (stackSpill, per wave slot and lane).
    constexpr int LS = kLdsStack<STACK, SAMPLE, WIDE>;
    __shared__ uint32_t stk[LS * kWave];
    // Wide kernels, speculative traversal: a lane whose primitive group waits for a LEAF step
    // keeps visiting nodes; the waiting group is parked here ({base, bits} per lane; oct bit 4
    // marks it) and comes back when the current group is empty.
    constexpr int SPECN = WIDE ? (INST ? PT_INST_SPEC : PT_WIDE_SPEC) : 0;   // parked groups per lane: a stack, count in oct bits 4-5
    constexpr bool SPEC = SPECN > 0;
    __shared__ uint32_t pend[SPEC ? 2 * SPECN * kWave : 1];
    // wave-cooperative LEAF steps: the step's queue of (owner lane, primitive) pairs
    constexpr bool COOP = WIDE && !INST && PT_LEAF_COOP != 0;
    __shared__ uint32_t leafQ[COOP ? kWave : 1];
    if constexpr (COOP) leafQ[threadIdx.x] = 0u;   // (every entry is a valid pair from here on)
    // instanced scenes: the lane's world ray {o, d} while it is inside an instance
    __shared__ float wray[INST ? 6 * kWave : 1];
    // sample mode: the lane's task {pixel col | local row << 16, next sample, end sample, rays}.
    // Only SHADE steps (per sample, not per node or primitive) touch it, so it lives in LDS, not
    // in four VGPRs carried through every step.
    __shared__ uint4 taskState[SAMPLE ? kWave : 1];
    // compat mode with the pixel queue (CQ): the lane's pixel {its tile, rays traced for it, its
    // index} (LDS: only a pixel's first and last sample touch it)
    constexpr bool CQ = !SAMPLE && PT_COMPAT_QUEUE != 0;
    __shared__ uint4 pixState[CQ ? kWave : 1];
    // sample mode, tasks of several blocks: the task's closed blocks so far, per lane (x, y, z)
    // (wide kernels; the binary ones take one block per task and keep their LDS for the stack)
    constexpr bool GROUPS = PT_TASK_GROUPS && SAMPLE && WIDE && STACK <= 16;   // (STACK 24: the LDS would cap occupancy)
    __shared__ unsigned long long accPart[GROUPS ? 3 * kWave : 1];
    if constexpr (GROUPS) {
        accPart[threadIdx.x] = 0ull; accPart[kWave + threadIdx.x] = 0ull; accPart[2 * kWave + threadIdx.x] = 0ull;
    }
    const int lane = threadIdx.x;
    // compat mode: all spp of a pixel in order (its per-pixel XORWOW stream).  Default: one wave =
    // one tile (the longest tiles split, below).  The pixel queue (CQ: PT_COMPAT_QUEUE=1, an
    // experiment, off: measured slower) makes the waves persistent and lets them
    // take pixels from a global counter (PT_TAKE_PIXELS): a lane whose pixel has all its samples
    // takes the next pixel.
    // sample mode: persistent waves; each lane repeatedly takes a task = (pixel, summation
    // block) from a global counter and sums that block's samples in order (see PT_TAKE_TASKS).
    // `sample` runs to nSamples (compat: spp; sample mode: the end of the task's block, and
    // `sample` is the absolute sample index)
    // Compat mode, split tiles: the first splitTiles tiles of the launch order (the longest: their
    // pixels' sequential chains are the frame's critical path) run as splitWays waves each, one slice
    // of 64 / splitWays pixels per wave (the other lanes idle), so a critical pixel shares its wave's
    // steps with fewer other pixels and its chain advances in more of them.
    int bidT = (int)blockIdx.x, slice = -1;
    // compat, critical-pixel waves (CRIT): the first critWaves blocks (wave-uniform)
    constexpr bool CRITK = critFor(SAMPLE, WIDE, INST, CQ, STACK);
    const bool crit = CRITK && bidT < P.critWaves;
    if constexpr (CRITK) {
        if (!crit) bidT -= P.critWaves;
    }
    if constexpr (!SAMPLE && !CQ && !PT_AB_NO_SPLIT) {
        const int ks = P.splitTiles * P.splitWays;   // (uniform)
        if (crit) {
        } else if (bidT < ks) { slice = bidT % P.splitWays; bidT /= P.splitWays; }
        else bidT -= ks - P.splitTiles;
    }
    int tile = (SAMPLE || CQ || crit) ? -1 : tileOf(P, bidT), nSamples = SAMPLE ? 0 : P.spp;
    int col = 0, lrow = 0;
    bool valid = false;
    uint32_t idx = 0u;
    if constexpr (!SAMPLE && !CQ) {
        if (crit) {   // a listed pixel per lane (lanes beyond critLanes or the list idle)
            const int k = bidT * P.critLanes + lane;
            valid = lane < P.critLanes && k < P.nCrit;
            idx = valid ? P.critList[k] : 0u;
            col = (int)(idx % (uint32_t)P.width);
            lrow = (int)(idx / (uint32_t)P.width);
        } else {
            col = (tile % P.tiles_x) * 8 + (lane & 7);
            lrow = (tile / P.tiles_x) * 8 + (lane >> 3);
            valid = col < P.width && lrow < P.nrows && (slice < 0 || (lane * P.splitWays) / kWave == slice);
            idx = valid ? (uint32_t)lrow * (uint32_t)P.width + (uint32_t)col : 0u;   // npix < 2^32
            if (CRITK && valid && P.critFlag && P.critFlag[idx]) valid = false;   // (a critical wave's pixel)
        }
    }
    const unsigned long long tStart = __builtin_amdgcn_s_memrealtime();
    if (!SAMPLE && !CQ && !crit && bidT < P.prioTiles) {   // wave-uniform condition (s_setprio takes an immediate)
        if (P.prioLevel >= 3) __builtin_amdgcn_s_setprio(3);
        else if (P.prioLevel == 2) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(1);
    }
    float fcol = (float)col;
    float frow = valid ? (float)globalRow(lrow, P.stripe_h, P.nparts, P.part) : 0.0f;
    const DevScene& S = P.S;
    // gfx9 buffer resource: base = the node array, raw (stride 0), DATA_FORMAT_32 in dword 3
    const __amdgpu_buffer_rsrc_t nodeRsrc = rawRsrc(WIDE ? (const void*)S.wnodes : (const void*)S.nodes);
    uint32_t* my = stk + lane;
    // Work counters are wave totals kept in scalar registers: each step adds the popcount of
    // a ballot of the lanes that did the work (no per-lane counter VGPRs).
    uint32_t sRays = 0, sVisits = 0, sTris = 0, sSph = 0, sPaths = 0;
#ifdef PT_DIAG
    uint32_t itN = 0, itL = 0, itS = 0, sPops = 0, sRedo = 0;   // scheduler diagnostics (iterations per kind)
    unsigned long long sSpecN = 0, sIdleN = 0;   // NODE steps: lanes waiting on primitives that have nodes left; lanes with no NODE work
    unsigned long long sAvoid = 0, sHalf = 0;    // LEAF (wide): tests whose exact box misses at test time; lanes testing one primitive
    unsigned long long sAvoidInf = 0, sParkT = 0, sParkA = 0;   // ... misses even with tmax = inf; tests / misses in parked groups
    unsigned long long cycN = 0, cycL = 0, cycS = 0, cycH = 0;   // and shader cycles per kind, loop head
    unsigned long long cycSh = 0, cycTk = 0, cycNp = 0, cycBr = 0;   // SHADE: shading, tasks, new path, ray start
#define PT_DIAG_ADD(v, x) (v) += (x)
#else
#define PT_DIAG_ADD(v, x) ((void)0)
#endif

    Xorwow g{};
    if constexpr (!SAMPLE) {
        if (valid) g = Xorwow{P.sd[idx], P.s0[idx], P.s1[idx], P.s2[idx], P.s3[idx], P.s4[idx]};
    }
    float3 sum = f3(0.0f, 0.0f, 0.0f), o = f3(0.0f, 0.0f, 0.0f), d = f3(0.0f, 0.0f, 1.0f);
    float3 inv = d, att = f3(1.0f, 1.0f, 1.0f);
    float closest = 0.0f;
    int best = -1, depthLeft = 0, sample = 0, node = -1, sp = 0, qn = 0;
    // leaf queue depth: sample mode on shallow trees (STACK <= 32: C2, C3) prefers 2, deep trees
    // (C5, STACK 48+) and compat mode 4 (C3 1068 vs 1088 ms, C2 67.4 vs 70.6, C5 1576 vs 1471)
    constexpr int LQ = (SAMPLE && !WIDE && STACK <= 32) ? PT_LEAF_QUEUE_SAMPLE : kLeafQ;
    uint32_t qref[LQ];   // leaf queue: leaf refs in DFS order (registers: constant indices only)
    float lq[LQ];     // their slab entry distances
#pragma unroll
    for (int i = 0; i < LQ; i++) { qref[i] = 0u; lq[i] = 0.0f; }
    // wide tree traversal state (WIDE): node group, primitive group, ray octant (| 8: redo the
    // query in the reference's order), the best hit's window end
    uint32_t ng = 0u, tgBase = 0u, tg = 0u, oct = 0u;
    float bestLo = 0.0f;
    bool active = false;
    // sample mode task state: summation block, its tile (cost accounting), rays traced for it
    uint32_t depthPaths = 0;
    uint32_t pxRays = 0;   // compat tile / critical lanes: rays traced for the lane's pixel (P.pixRays)
    bool needTask = SAMPLE || CQ;
    uint32_t poolBase = 0u, poolLeft = 0u;   // sample mode / CQ: the wave's reserved tasks (uniform)


    // Start the closest-hit query of (o, d).  (Macros, not lambdas: a [&] closure makes the
    // captured variables address-taken and they end up in scratch memory.)
#define PT_BEGIN_RAY()                                                                              \
    do {                                                                                          \
        depthLeft--;                                                                              \
        if constexpr (SAMPLE) {   /* rays per task: only frames that measure tile costs use them */ \
            if (kargs()->measureCost)                                                             \
                __hip_atomic_fetch_add(&taskState[lane].w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); \
        }                                                                                         \
        if constexpr (CQ) {   /* rays per pixel, likewise */                                     \
            if (kargs()->measureCost)                                                             \
                __hip_atomic_fetch_add(&pixState[lane].y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); \
        }                                                                                         \
        closest = __builtin_inff();                                                               \
        best = -1;                                                                                \
        sp = 0;                                                                                   \
        qn = 0;                                                                                   \
        if constexpr (CRITK) pxRays++;                                                            \
        if constexpr (WIDE) {   /* the root is slot 0 of a virtual node at base 0 */              \
            if (PT_AB_CHEAP_START) inv = f3(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z)); \
            else inv = f3(rcpRN(d.x), rcpRN(d.y), rcpRN(d.z));                                    \
            const uint32_t oc_ = (inv.x < 0.0f ? 1u : 0u) | (inv.y < 0.0f ? 2u : 0u) | (inv.z < 0.0f ? 4u : 0u); \
            oct = oc_;                                                                            \
            tg = 0u;                                                                              \
            bestLo = -__builtin_inff();                                                           \
            ng = S.nprims > 0 ? (1u << oc_) : 0u;                                                 \
            /* only camera rays can start far from the scene (a bounce starts on a primitive), and  \
               they all start at the camera: one uniform flag, set on the host (wideFar) */     \
            if (!INST && ((kargs()->camFar && depthLeft + 1 == kargs()->max_depth) ||              \
                          (PT_WIDE_MIX && PT_MIX_CHECK && !PT_AB_CHEAP_START && mixUnsafe(inv, kargs()->S.mixLim)))) {                  \
                ng = 0u;       /* origin far from the scene, or a direction the MIX planes */      \
                oct |= 8u;     /* cannot take: the query in the reference's order (SHADE's redo) */ \
            }                                                                                     \
            if (INST && kargs()->camFar && depthLeft + 1 == kargs()->max_depth) {                  \
                /* a far camera: the path starts where its ray enters the world (instEntry) */     \
                const auto& K_ = *kargs();                                                        \
                (void)instEntry(K_.S.cx, K_.S.cy, K_.S.cz, K_.S.ext, o, d, inv);                   \
            }                                                                                     \
            if (CRITK && crit) PT_CRIT_TRACE();                                                    \
        } else if (S.nprims <= 1) {                                                               \
            node = -1;                                                                            \
            if (S.nprims == 1) { /* root is a leaf: no box test (render_manager.h:92-98) */       \
                const float t1 = primHitT(loadPrim(S, 0), __float_as_uint(S.prims[2].w) != 0, o, d, \
                                          0.001f, closest);                                       \
                if (t1 >= 0.0f) { closest = t1; best = 0; }                                       \
            }                                                                                     \
        } else {                                                                                  \
            inv = f3(rcpRN(d.x), rcpRN(d.y), rcpRN(d.z));                                         \
            node = 0;                                                                             \
        }                                                                                         \
    } while (0)
    // Critical-pixel waves (compat, wide): the lane's whole closest-hit query at once, in a per-lane
    // loop (nearest child first, the NODE and LEAF steps' own tests and tie / window rules, no
    // speculation): a lane alone on its chain advances every iteration instead of waiting for the
    // wave's step kinds.  The result is the reference's closest hit either way;
    // a flagged order-dependent query is redone in the reference's order by the SHADE step as usual.
#define PT_CRIT_TRACE()                                                                             \
    do {                                                                                          \
        const bool lb_ = S.nprims > 1;                                                            \
        const bool sph_ = kargs()->S.hasSpheres != 0;                                             \
        bool redo_ = false;                                                                       \
        for (;;) {                                                                                \
            while (tg) {                                                                          \
                const uint32_t k_ = tgBase + (uint32_t)__builtin_ctz(tg);                         \
                tg &= tg - 1u;                                                                    \
                const float4* w_ = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(S.wprims) + mul48(k_)); \
                const Prim q_{w_[0], w_[1], w_[2]};                                               \
                const bool isS_ = __float_as_uint(q_.p2.w) != 0u;                                 \
                sTris += (uint32_t)__popcll(__ballot(!isS_));                                     \
                sSph += (uint32_t)__popcll(__ballot(isS_));                                       \
                if (sph_) wideTest<true>(q_, o, d, inv, 0.001f, closest, best, bestLo, lb_, redo_, 0u); \
                else wideTest<false>(q_, o, d, inv, 0.001f, closest, best, bestLo, lb_, redo_, 0u); \
            }                                                                                     \
            if ((ng & 0xffu) == 0u) {                                                             \
                if (sp == 0) break;                                                               \
                sp--;                                                                             \
                ng = my[sp * kWave];                                                              \
            }                                                                                     \
            const uint32_t bit_ = (uint32_t)__builtin_ctz(ng & 0xffu);                            \
            const uint32_t child_ = (ng >> 8) + (bit_ ^ (oct & 7u));                              \
            ng &= ~(1u << bit_);                                                                  \
            if (ng & 0xffu) { my[sp * kWave] = ng; sp++; }   /* sp < depth <= STACK (host check) */ \
            sVisits += (uint32_t)__popcll(__ballot(true));                                        \
            const uint32_t off_ = mul80(child_);                                                  \
            const uint4 n0_ = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off_, 0, 0)); \
            const uint4 n1_ = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off_ + 16u, 0, 0)); \
            const uint4 n2_ = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off_ + 32u, 0, 0)); \
            const uint4 n3_ = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off_ + 48u, 0, 0)); \
            const uint4 n4_ = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off_ + 64u, 0, 0)); \
            const uint32_t h_ = wideHits<PT_WIDE_MIX != 0>(n0_, n1_, n2_, n3_, n4_, o, inv, oct & 7u, 0.001f, closest); \
            ng = (n1_.x << 8) | (h_ >> 24);                                                      \
            tgBase = n1_.y;                                                                       \
            tg = h_ & 0xffffffu;                                                                  \
        }                                                                                         \
        if (redo_) oct |= 8u;   /* order-dependent candidate: SHADE repeats the query */           \
    } while (0)
    // New camera sample: main.cu:284-286 + camera::get_ray (lens sample: lensOffset; time draw skipped).
    // Sample mode: lanes with needTask take the next tasks of the wave's pool, in lane order; an
    // empty pool is refilled with the next kTaskPool tasks of the global counter (one returning
    // atomic, whose latency the wave waits out, per kTaskPool tasks instead of per SHADE step).
    // Task t = (tile slot t / 64 / nblocks in launch order, block (t / 64) % nblocks, pixel
    // t % 64 of the 8x8 tile); tasks off the frame edge are skipped.  Sets `got` for lanes
    // that received a task; lanes that find the counter exhausted stop asking.
#if PT_XCD_POOLS
    // counter x holds the groups of tile slots x, x + 8, ...: local group lg = slot / 8 * ngroups +
    // block.  A wave tries its own XCD's counter first, then the others in turn (no state kept: an
    // exhausted counter costs a wave one more atomic per refill; the host keeps the overshoot far
    // from wrapping, ntasks < 2^28); all eight empty: poolBase = ntasks
#define PT_POOL_REFILL(grab, leader)                                                                \
    do {                                                                                          \
        uint32_t gb_ = Q_.ntasks;                                                                 \
        for (uint32_t i_ = 0; i_ < 8u; i_++) {                                                    \
            const uint32_t x_ = (blockIdx.x + i_) & 7u;                                           \
            uint32_t lb_ = 0;                                                                     \
            if (lane == (leader)) lb_ = atomicAdd(Q_.taskCounter + x_, (grab));                   \
            lb_ = __builtin_amdgcn_readfirstlane((uint32_t)__shfl((int)lb_, (leader)));           \
            const uint32_t lg_ = lb_ >> 6, ng_ = (uint32_t)Q_.ngroups;                            \
            const uint32_t nt_ = (uint32_t)Q_.ntiles;                                             \
            const uint32_t nLocal_ = x_ < nt_ ? (nt_ - x_ + 7u) >> 3 : 0u;                        \
            if (lg_ < nLocal_ * ng_) {                                                            \
                const uint32_t q_ = lg_ / ng_, blk_ = lg_ - q_ * ng_;                              \
                gb_ = ((8u * q_ + x_) * ng_ + blk_) << 6;                                         \
                break;                                                                            \
            }                                                                                     \
        }                                                                                         \
        poolBase = gb_;                                                                           \
    } while (0)
#else
#define PT_POOL_REFILL(grab, leader)                                                                \
    do {                                                                                          \
        uint32_t b_ = 0;                                                                          \
        if (lane == (leader)) b_ = atomicAdd(Q_.taskCounter, (grab));                             \
        poolBase = __builtin_amdgcn_readfirstlane((uint32_t)__shfl((int)b_, (leader)));           \
    } while (0)
#endif
#define PT_TAKE_TASKS(got)                                                                          \
    do {                                                                                          \
        const auto& Q_ = *kargs();                                                                \
        for (;;) {                                                                                \
            const uint64_t m_ = __ballot(needTask);                                               \
            if (m_ == 0) break;                                                                   \
            if (poolLeft == 0u) { /* refill the wave's pool: one returning atomic per kTaskPool */ \
                const int leader_ = __ffsll((unsigned long long)m_) - 1;                          \
                /* always a full pool: = one (tile, block) group, one task per lane; smaller    \
                   grabs near the end measured slower (1/8 share: 150-158 vs 145 ms) */          \
                const uint32_t grab_ = (uint32_t)kTaskPool;                                       \
                PT_POOL_REFILL(grab_, leader_);                                                   \
                poolLeft = grab_;                                                                 \
            }                                                                                     \
            /* wave-uniform: the taken tasks span task groups (tile slot, blocks) g0 and g0 + 1 */ \
            const uint32_t base_ = poolBase;                                                      \
            const uint32_t take_ = min((uint32_t)__popcll(m_), poolLeft);                         \
            poolBase += take_;                                                                    \
            poolLeft -= take_;                                                                    \
            const uint32_t g0_ = base_ >> 6, off_ = base_ & 63u;                                  \
            const uint32_t slotA_ = Q_.nblocksShift >= 0 ? g0_ >> Q_.nblocksShift : g0_ / (uint32_t)Q_.ngroups; \
            const uint32_t blkA_ = g0_ - slotA_ * (uint32_t)Q_.ngroups;                           \
            const bool wrap_ = blkA_ + 1u == (uint32_t)Q_.ngroups;                                  \
            const uint32_t slotB_ = wrap_ ? slotA_ + 1u : slotA_, blkB_ = wrap_ ? 0u : blkA_ + 1u; \
            const uint32_t nslots_ = (uint32_t)Q_.ntiles;                                          \
            /* the slots' tiles, decoded once per launch order (tileXYKernel): no divisions here */ \
            /* (scalar loads through the constant address space: a vector load here would wait   \
               out the accumulator atomics a finishing lane has just issued -- vmcnt counts every \
               vector memory operation in issue order) */                                        \
            const uint32_t xyA_ = slotA_ < nslots_ ? ((KU32)Q_.tileXY)[__builtin_amdgcn_readfirstlane(slotA_)] : 0u; \
            const uint32_t xyB_ = slotB_ < nslots_ ? ((KU32)Q_.tileXY)[__builtin_amdgcn_readfirstlane(slotB_)] : 0u; \
            const uint32_t txA_ = xyA_ & 0xffffu, tyA_ = xyA_ >> 16;                              \
            const uint32_t txB_ = xyB_ & 0xffffu, tyB_ = xyB_ >> 16;                              \
            const uint32_t k_ = (uint32_t)__popcll(m_ & ((1ull << lane) - 1ull));                 \
            if (needTask && k_ < take_) {                                                         \
                if (base_ + k_ >= Q_.ntasks) {                                                     \
                    needTask = false;                                                             \
                } else {                                                                          \
                    const uint32_t o_ = off_ + k_, px_ = o_ & 63u;                                \
                    const bool hi_ = o_ >= 64u;                                                   \
                    const int c_ = (int)((hi_ ? txB_ : txA_) * 8u + (px_ & 7u));                  \
                    const int r_ = (int)((hi_ ? tyB_ : tyA_) * 8u + (px_ >> 3));                  \
                    if (c_ < Q_.width && r_ < Q_.nrows) {                                           \
                        needTask = false;                                                         \
                        got = true;                                                               \
                        const uint32_t s0_ = (hi_ ? blkB_ : blkA_) * (uint32_t)Q_.span;           \
                        taskState[lane] = make_uint4((uint32_t)c_ | ((uint32_t)r_ << 16), s0_,     \
                                                     min(s0_ + (uint32_t)Q_.span, (uint32_t)Q_.spp), 0u); \
                        sum = f3(0.0f, 0.0f, 0.0f);                                               \
                    }                                                                             \
                }                                                                                 \
            }                                                                                     \
        }                                                                                         \
    } while (0)
    // Compat mode, pixel queue (CQ): the lanes with needTask take the next pixels of the global queue,
    // exactly as many as ask (one returning atomic; ranked in lane order by the ballot): queue slot t
    // = pixel t % 64 of the 8x8 tile in launch slot t / 64 (longest tiles first), so a take spans at
    // most two tiles.  No pool is reserved ahead: a pixel is a long task (all its samples), and
    // slots held back by a wave would wait for that wave's lanes while other waves run dry.  A taken
    // pixel's XORWOW state comes from the film (curand_init(seed, pixel, 0) or where the last frame
    // left it).  Slots off the frame edge are skipped; lanes that find the queue exhausted stop asking.
#define PT_TAKE_PIXELS(got)                                                                         \
    do {                                                                                          \
        const auto& Q_ = *kargs();                                                                \
        for (;;) {                                                                                \
            const uint64_t m_ = __ballot(needTask);                                               \
            if (m_ == 0) break;                                                                   \
            const uint32_t n_ = (uint32_t)__popcll(m_);                                           \
            const int leader_ = __ffsll((unsigned long long)m_) - 1;                              \
            uint32_t b_ = 0;                                                                      \
            if (lane == leader_) b_ = atomicAdd(Q_.taskCounter, n_);                               \
            const uint32_t base_ = __builtin_amdgcn_readfirstlane((uint32_t)__shfl((int)b_, leader_)); \
            const uint32_t slotA_ = base_ >> 6, slotB_ = slotA_ + 1u;                             \
            const uint32_t nt_ = (uint32_t)Q_.ntiles;                                             \
            const uint32_t xyA_ = slotA_ < nt_ ? ((KU32)Q_.tileXY)[__builtin_amdgcn_readfirstlane(slotA_)] : 0u; \
            const uint32_t xyB_ = slotB_ < nt_ ? ((KU32)Q_.tileXY)[__builtin_amdgcn_readfirstlane(slotB_)] : 0u; \
            const uint32_t k_ = (uint32_t)__popcll(m_ & ((1ull << lane) - 1ull));                 \
            if (needTask) {                                                                       \
                const uint32_t t_ = base_ + k_;                                                   \
                if ((t_ >> 6) >= nt_) {                                                           \
                    needTask = false;   /* the queue is exhausted */                               \
                } else {                                                                          \
                    const bool hi_ = (t_ >> 6) != slotA_;                                         \
                    const uint32_t xy_ = hi_ ? xyB_ : xyA_, px_ = t_ & 63u;                       \
                    const uint32_t tx_ = xy_ & 0xffffu, ty_ = xy_ >> 16;                          \
                    const int c_ = (int)(tx_ * 8u + (px_ & 7u)), r_ = (int)(ty_ * 8u + (px_ >> 3)); \
                    if (c_ < Q_.width && r_ < Q_.nrows) {                                           \
                        needTask = false;                                                         \
                        got = true;                                                               \
                        const uint32_t i_ = (uint32_t)r_ * (uint32_t)Q_.width + (uint32_t)c_;     \
                        pixState[lane] = make_uint4(ty_ * (uint32_t)Q_.tiles_x + tx_, 0u, i_, 0u); \
                        fcol = (float)c_;                                                         \
                        frow = (float)globalRowFast(r_, Q_.stripe_h, Q_.stripeShift, Q_.nparts, Q_.part); \
                        g = Xorwow{Q_.sd[i_], Q_.s0[i_], Q_.s1[i_], Q_.s2[i_], Q_.s3[i_], Q_.s4[i_]}; \
                        sum = f3(0.0f, 0.0f, 0.0f);                                               \
                        sample = 0;                                                               \
                    }                                                                             \
                }                                                                                 \
            }                                                                                     \
        }                                                                                         \
    } while (0)
    // CQ: the lane's pixel has all its samples: its result and XORWOW state back to the film, its
    // ray count into its tile's cost (the longest pixel of the tile: the next launch's order), and
    // the lane asks for the next pixel.
#define PT_FINISH_PIXEL()                                                                           \
    do {                                                                                          \
        const auto& Q_ = *kargs();                                                                \
        const uint4 ps_ = pixState[lane];                                                         \
        const uint32_t i_ = ps_.z;                                                                \
        float* out_ = Q_.out + 3 * (size_t)i_;   /* (storePixel) */                               \
        if (Q_.rawOut) {                                                                          \
            out_[0] = sum.x; out_[1] = sum.y; out_[2] = sum.z;                                    \
        } else {                                                                                  \
            out_[0] = sqrtf(sum.x * Q_.invSpp); out_[1] = sqrtf(sum.y * Q_.invSpp); out_[2] = sqrtf(sum.z * Q_.invSpp); \
        }                                                                                         \
        Q_.sd[i_] = g.d; Q_.s0[i_] = g.v0; Q_.s1[i_] = g.v1; Q_.s2[i_] = g.v2; Q_.s3[i_] = g.v3; Q_.s4[i_] = g.v4; \
        if (Q_.measureCost) atomicMax(Q_.tileCost + ps_.x, ps_.y);                                \
        needTask = true;                                                                          \
    } while (0)
    // Sample mode: the lane's block (= its task; ts = the task state) is complete: its sum and ray
    // count go to the pixel's accumulator (order-free integer atomics on per-pixel addresses: no
    // contention; right here -- deferring them to a later step of the loop, where fewer registers
    // are live, measured 2.6 % slower), and the lane asks for its next task.
#define PT_FINISH_TASK(ts)                                                                          \
    do {                                                                                          \
        unsigned long long* acc_ = kargs()->pixAcc + 4 * (size_t)(((ts).x >> 16) * (uint32_t)kargs()->width + ((ts).x & 0xffffu)); \
        if constexpr (GROUPS) {   /* the task's earlier blocks wait in the lane's LDS partial */ \
            addFixed1(acc_ + 0, accPart[lane] + blockFixed(sum.x));                               \
            addFixed1(acc_ + 1, accPart[kWave + lane] + blockFixed(sum.y));                       \
            addFixed1(acc_ + 2, accPart[2 * kWave + lane] + blockFixed(sum.z));                   \
            if (kargs()->measureCost) addFixed1(acc_ + 3, (unsigned long long)((ts).w + 1u));     \
            accPart[lane] = 0ull; accPart[kWave + lane] = 0ull; accPart[2 * kWave + lane] = 0ull;   \
        } else {                                                                                  \
            addBlock(acc_, sum, (ts).w + 1u, kargs()->measureCost != 0);                          \
        }                                                                                         \
        needTask = true;                                                                          \
    } while (0)
    // Sample mode, tasks of several blocks: a block that is not the task's last one closes into the
    // lane's LDS partial (exact 64-bit additions), and the next block's sum starts from zero.
#define PT_CLOSE_BLOCK(y_)                                                                          \
    do {                                                                                          \
        const auto& Q_ = *kargs();                                                                \
        if (GROUPS && Q_.group > 1 && (Q_.blockShift >= 0 ? ((y_) & (((uint32_t)1 << Q_.blockShift) - 1u)) == 0u \
                                                 : (y_) % (uint32_t)Q_.block == 0u)) {            \
            __hip_atomic_fetch_add(&accPart[lane], blockFixed(sum.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); \
            __hip_atomic_fetch_add(&accPart[kWave + lane], blockFixed(sum.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); \
            __hip_atomic_fetch_add(&accPart[2 * kWave + lane], blockFixed(sum.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); \
            sum = f3(0.0f, 0.0f, 0.0f);                                                           \
        }                                                                                         \
    } while (0)
#define PT_NEW_PATH()                                                                               \
    do {                                                                                          \
        const auto& Q_ = *kargs();                                                                \
        if constexpr (SAMPLE) {   /* the task's pixel and next sample from LDS */                \
            const uint4 ts_ = taskState[lane];                                                    \
            fcol = (float)(ts_.x & 0xffffu);                                                      \
            const uint32_t grow_ = (uint32_t)globalRowFast((int)(ts_.x >> 16), Q_.stripe_h, Q_.stripeShift, \
                                                           Q_.nparts, Q_.part);                  \
            frow = (float)grow_;                                                                  \
            g = sampleStream(Q_.seed0, Q_.seed1, Q_.sampleBase + ts_.y,                           \
                             grow_ * (uint32_t)Q_.width + (ts_.x & 0xffffu));                      \
        }                                                                                         \
        const float u_ = (fcol + g.uniform()) * Q_.invW;                                           \
        const float v_ = (frow + g.uniform()) * Q_.invH;                                           \
        o = ld3(Q_.cam.pos);                                                                            \
        d = sub(add(add(ld3(Q_.cam.ll), scale(u_, ld3(Q_.cam.hor))), scale(v_, ld3(Q_.cam.ver))), ld3(Q_.cam.pos));       \
        if (Q_.cam.lens != 0.0f) lensOffset(ld3(Q_.cam.right), ld3(Q_.cam.up), Q_.cam.lens, g, o, d); \
        att = f3(1.0f, 1.0f, 1.0f);                                                               \
        depthLeft = Q_.max_depth;                                                                  \
    } while (0)

    bool started = false;
    if constexpr (SAMPLE) {
        // Every lane starts with needTask: the first loop iteration is a SHADE step that hands
        // out tasks.  max_depth <= 0 (no bounce: each sample is the sky colour of its camera
        // ray) is handled here, without the loop.
        if (P.max_depth <= 0) {
            for (;;) {
                bool got = false;
                PT_TAKE_TASKS(got);
                if (__ballot(got) == 0) break;
                if (got) {
                    uint4 ts = taskState[lane];
                    depthPaths += ts.z - ts.y;
                    while (ts.y < ts.z) {
                        taskState[lane].y = ts.y;
                        PT_NEW_PATH();
                        sum = add(sum, sky(d, att));
                        ts.y++;
                        if (ts.y < ts.z) PT_CLOSE_BLOCK(ts.y);
                    }
                    PT_FINISH_TASK(ts);
                }
            }
            needTask = false;
            waveReduceAdd(P.counters + 4, depthPaths);   // (paths counted per lane here)
        }
    } else if (CQ) {
        if (P.max_depth <= 0) {   // (no bounce: every sample is its camera ray's sky colour)
            for (;;) {
                bool got = false;
                PT_TAKE_PIXELS(got);
                if (__ballot(got) == 0) break;
                if (got) {
                    for (; sample < nSamples; sample++) {
                        PT_NEW_PATH();
                        sum = add(sum, sky(d, att));
                    }
                    depthPaths += (uint32_t)nSamples;
                    PT_FINISH_PIXEL();
                }
            }
            needTask = false;
            waveReduceAdd(P.counters + 4, depthPaths);
        }
    } else if (valid) {
        if (P.max_depth <= 0) {
            for (; sample < nSamples; sample++) {
                PT_NEW_PATH();
                sum = add(sum, sky(d, att));
            }
        } else if (nSamples > 0) {
            PT_NEW_PATH();
            PT_BEGIN_RAY();
            active = true;
            started = true;
        }
    }
    sRays += (uint32_t)__popcll(__ballot(started));
    sPaths += (uint32_t)__popcll(__ballot(started)) +
              (!SAMPLE && P.max_depth <= 0 ? (uint32_t)__popcll(__ballot(valid)) * (uint32_t)nSamples : 0u);

    for (;;) {
#ifdef PT_DIAG
        const unsigned long long tH0 = __builtin_amdgcn_s_memtime();
#endif
        // binary: room for both children's leaves; wide: a node (the step handles a full queue)
        // or a stack top waiting for queue space (node == -2)
        // binary: room for both children's leaves in the queue; wide: no primitives pending
        // (instanced: a lane with primitives waiting visits only siblings of its group -- the same
        // object space; it pops, and may cross an instance marker, only with none waiting)
        const bool wantNode = WIDE ? (INST ? ((tg == 0u && ((ng & 0xffu) != 0u || sp > 0)) ||
                                              (SPEC && tg != 0u && ((oct >> 4) & 3u) < (uint32_t)SPECN && (ng & 0xffu) != 0u))
                                           : ((SPEC ? (tg == 0u || ((oct >> 4) & 3u) < (uint32_t)SPECN) : tg == 0u) &&
                                              ((ng & 0xffu) != 0u || sp > 0)))
                                   : (node >= 0 && qn <= LQ - 2);
        const bool wantLeaf = WIDE ? tg != 0u : qn > 0;
        const bool wantShade = (active && (WIDE ? (tg == 0u && (ng & 0xffu) == 0u && sp == 0) : (node == -1 && qn == 0))) ||
                               needTask;
        const uint64_t mN = __ballot(wantNode), mL = __ballot(wantLeaf), mS = __ballot(wantShade);
        if ((mN | mL | mS) == 0) break;
        const int nN = __popcll(mN), nL = __popcll(mL), nS = __popcll(mS);
        int kind;   // 0 node, 1 leaf, 2 shade
        if (nN == 0) kind = nL > 0 ? 1 : 2;
        else if (nL >= P.leafBatch) kind = 1;
        else if (nS >= P.shadeBatch) kind = 2;
        else if (!SAMPLE && nN < P.nodeMin && (nL | nS)) kind = nL >= nS ? 1 : 2;
        else kind = 0;
#ifdef PT_DIAG
        const unsigned long long tK0 = __builtin_amdgcn_s_memtime();
        cycH += tK0 - tH0;
#endif

        if (kind == 0) {
            // ------------------------------------------------------------------ NODE
            sVisits += (uint32_t)nN;
            PT_DIAG_ADD(itN, 1u);
            if constexpr (WIDE) {
                PT_DIAG_ADD(sSpecN, (unsigned long long)__popcll(__ballot(tg != 0u && ((ng & 0xffu) != 0u || sp > 0))));
                PT_DIAG_ADD(sIdleN, (unsigned long long)(64 - nN));
            }
            if constexpr (INST) {
                if (wantNode) {
                    if (SPEC && tg != 0u) {   // park the waiting primitive group (a sibling follows: same space)
                        const uint32_t c = SPECN == 1 ? 0u : (oct >> 4) & 3u;
                        pend[(2u * c) * kWave + lane] = tgBase;
                        pend[(2u * c + 1u) * kWave + lane] = tg;
                        oct += 16u;
                    }
                    if constexpr (SPEC) asm volatile("" ::: "memory");
                    // pop to a group with children left; a marker returns the lane to the world
                    // (oct bit 3: the instance transformed the direction, not only the origin)
                    while ((ng & 0xffu) == 0u && sp > 0) {
                        sp--;
                        ng = my[sp * kWave];
                        if (ng == kInstMarker) {
                            o = f3(wray[0 * kWave + lane], wray[1 * kWave + lane], wray[2 * kWave + lane]);
                            if (oct & 8u) {
                                d = f3(wray[3 * kWave + lane], wray[4 * kWave + lane], wray[5 * kWave + lane]);
                                inv = f3(rcpRN(d.x), rcpRN(d.y), rcpRN(d.z));
                                oct = (inv.x < 0.0f ? 1u : 0u) | (inv.y < 0.0f ? 2u : 0u) | (inv.z < 0.0f ? 4u : 0u);
                            } else {
                                oct &= 7u;
                            }
                            ng = 0u;
                        }
                    }
                    if (ng & 0xffu) {
                        const uint32_t bit = (uint32_t)__builtin_ctz(ng & 0xffu);
                        const uint32_t child = (ng >> 8) + (bit ^ (oct & 7u));
                        ng &= ~(1u << bit);
                        if (ng & 0xffu) { my[sp * kWave] = ng; sp++; }
                        uint32_t off = mul80(child);
                        uint4 n0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off, 0, 0));
                        uint4 n1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 16u, 0, 0));
                        uint4 n2 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 32u, 0, 0));
                        uint4 n3 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 48u, 0, 0));
                        uint4 n4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 64u, 0, 0));
                        if (n0.w == kInstFlag) {   // an instance: into its object space, and its tree's root in this step
                            wray[0 * kWave + lane] = o.x; wray[1 * kWave + lane] = o.y; wray[2 * kWave + lane] = o.z;
                            uint32_t full = 0u;
                            if (n0.x == 0u) {   // (an identity instance keeps the world ray)
                                const float4 r0 = __builtin_bit_cast(float4, n2), r1 = __builtin_bit_cast(float4, n3),
                                             r2 = __builtin_bit_cast(float4, n4);
                                if (n0.y != 0u) {   // translation only: the same origin as xformPoint, the direction kept
                                    o = f3(o.x + r0.w, o.y + r1.w, o.z + r2.w);
                                } else {
                                    wray[3 * kWave + lane] = d.x; wray[4 * kWave + lane] = d.y; wray[5 * kWave + lane] = d.z;
                                    o = xformPoint(r0, r1, r2, o);
                                    d = xformDir(r0, r1, r2, d);
                                    inv = f3(rcpRN(d.x), rcpRN(d.y), rcpRN(d.z));
                                    full = 8u;
                                }
                            }
                            const uint32_t oc = (inv.x < 0.0f ? 1u : 0u) | (inv.y < 0.0f ? 2u : 0u) | (inv.z < 0.0f ? 4u : 0u);
                            my[sp * kWave] = kInstMarker;   // (depth: host check, wideStackFor)
                            sp++;
                            oct = oc | full | (n1.y << 8);   // bits 8+: the instance the lane is in
                            off = mul80(n1.x);               // the mesh tree's root
                            n0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off, 0, 0));
                            n1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 16u, 0, 0));
                            n2 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 32u, 0, 0));
                            n3 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 48u, 0, 0));
                            n4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 64u, 0, 0));
                        }
                        const uint32_t hits = wideHitsInst(n0, n1, n2, n3, n4, o, inv, oct & 7u, 0.001f, closest);
                        ng = (n1.x << 8) | (hits >> 24);
                        tgBase = n1.y;
                        tg = hits & 0xffffffu;
                        if (SPEC && tg == 0u && (oct & 48u)) {   // no new primitives: the last parked group is current again
                            oct -= 16u;
                            const uint32_t c = SPECN == 1 ? 0u : (oct >> 4) & 3u;
                            tgBase = pend[(2u * c) * kWave + lane];
                            tg = pend[(2u * c + 1u) * kWave + lane];
                        }
                    }
                }
            } else if constexpr (WIDE) {
                if (wantNode) {
                    if (SPEC && tg != 0u) {   // park the waiting primitive group, keep traversing
                        const uint32_t c = SPECN == 1 ? 0u : (oct >> 4) & 3u;
                        pend[(2u * c) * kWave + lane] = tgBase;
                        pend[(2u * c + 1u) * kWave + lane] = tg;
                        oct += 16u;
                    }
                    // (the parked values are read back from LDS, not kept in registers meanwhile)
                    if constexpr (SPEC) asm volatile("" ::: "memory");
                    if ((ng & 0xffu) == 0u) { sp--; ng = my[sp * kWave]; }   // the group below
                    const uint32_t bit = (uint32_t)__builtin_ctz(ng & 0xffu);   // nearest remaining child
                    const uint32_t child = (ng >> 8) + (bit ^ (oct & 7u));
                    ng &= ~(1u << bit);
                    if (ng & 0xffu) { my[sp * kWave] = ng; sp++; }   // sp < depth <= STACK (host check)
                    const uint32_t off = mul80(child);
                    const uint4 n0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off, 0, 0));
                    const uint4 n1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 16u, 0, 0));
                    const uint4 n2 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 32u, 0, 0));
                    const uint4 n3 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 48u, 0, 0));
                    const uint4 n4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 64u, 0, 0));
                    const uint32_t hits = wideHits<PT_WIDE_MIX != 0>(n0, n1, n2, n3, n4, o, inv, oct & 7u, 0.001f, closest);
                    ng = (n1.x << 8) | (hits >> 24);
                    tgBase = n1.y;
                    tg = hits & 0xffffffu;
#ifdef PT_DIAG
                    oct &= ~64u;   // (diagnostics: bit 6 marks a group that was parked)
#endif
                    if (SPEC && tg == 0u && (oct & 48u)) {   // no new primitives: the last parked group is current again
                        oct -= 16u;
                        const uint32_t c = SPECN == 1 ? 0u : (oct >> 4) & 3u;
                        tgBase = pend[(2u * c) * kWave + lane];
                        tg = pend[(2u * c + 1u) * kWave + lane];
#ifdef PT_DIAG
                        oct |= 64u;
#endif
                    }
                }
            } else if (wantNode) {
                // buffer loads: a 32-bit per-lane offset off a wave-uniform resource (no 64-bit
                // address arithmetic per visit); < 2^26 nodes (pt_scene_create)
                const uint32_t off = (uint32_t)node * 64u;
                const float4 a = bload4(nodeRsrc, off), b = bload4(nodeRsrc, off + 16u);
                const float4 q = bload4(nodeRsrc, off + 32u), r = bload4(nodeRsrc, off + 48u);
                const uint32_t lref = __float_as_uint(r.x), rref = __float_as_uint(r.y);
                SlabHit2 h2 = slabBoth(a, b, q, o, inv, 0.001f, closest);
                // keep the right child's packed arithmetic next to the left's (not sunk past the
                // left child's queue append, where the operand pairs are no longer at hand)
                asm volatile("" : "+v"(h2.r.lo));
                const SlabHit hl = h2.l, hr = h2.r;
                // append hit leaves in order (left, then right) with their slab entry distances
                if constexpr (LQ == 2) {
                    // a NODE step needs an empty queue (qn <= LQ - 2): the slots are fixed
                    const bool al = hl.hit && (lref & kLeafBit), ar = hr.hit && (rref & kLeafBit);
                    qref[0] = al ? lref : rref;
                    lq[0] = al ? hl.lo : hr.lo;
                    qref[1] = rref;
                    lq[1] = hr.lo;
                    qn = (al ? 1 : 0) + (ar ? 1 : 0);
                } else {
                if (hl.hit && (lref & kLeafBit)) {
#pragma unroll
                    for (int i = 0; i < LQ; i++) {
                        qref[i] = qn == i ? lref : qref[i];
                        lq[i] = qn == i ? hl.lo : lq[i];
                    }
                    qn++;
                }
                if (hr.hit && (rref & kLeafBit)) {
#pragma unroll
                    for (int i = 0; i < LQ; i++) {
                        qref[i] = qn == i ? rref : qref[i];
                        lq[i] = qn == i ? hr.lo : lq[i];
                    }
                    qn++;
                }
                }
                const bool il = hl.hit && !(lref & kLeafBit), ir = hr.hit && !(rref & kLeafBit);
                // push left then right, pop: descend straight into the child that would be popped.
                // No overflow check: an entry is pushed only for a left sibling on the current
                // path, one per level, so sp < depth <= STACK - 1 (stackFor).
                if (ir) {
                    if (il) {
                        if (LS == STACK || sp < LS) my[sp * kWave] = lref;
                        else P.stackSpill[((size_t)blockIdx.x * kWave + lane) * (STACK - LS) + (sp - LS)] = lref;
                        sp++;
                    }
                    node = (int)rref;
                } else if (il) {
                    node = (int)lref;
                } else if (sp > 0) {
                    sp--;
                    node = (LS == STACK || sp < LS)
                               ? (int)my[sp * kWave]
                               : (int)P.stackSpill[((size_t)blockIdx.x * kWave + lane) * (STACK - LS) + (sp - LS)];
                } else {
                    node = -1;
                }
            }
        }
        if (kind == 1) {
            // ------------------------------------------------------------------ LEAF
            bool tested = false, sph = false;
            PT_DIAG_ADD(itL, 1u);
            if constexpr (COOP) {
                // Wave-cooperative LEAF step: the waiting (lane, primitive) pairs are compacted
                // so that every lane of the wave tests one.  A lane offers the first `cnt` (<= CAP)
                // primitives of its group in group order; a ballot prefix sum over the lanes gives
                // each offer its queue slot (the first 64 slots are taken, the rest wait for the
                // next LEAF step); lane j tests the pair in slot j against its owner's ray (fetched
                // with ds_bpermute) and hands (t, leaf box, key) back; each owner then merges its
                // results in group order with wideMerge -- the decisions wideTest makes, in the same
                // order, so closest / best / window / redo are exactly those of the one-lane tests.
                constexpr uint32_t CAP = PT_LEAF_COOP_CAP;
                const uint32_t pc = (uint32_t)__builtin_popcount(tg);
                const uint32_t cnt = pc < CAP ? pc : CAP;
                const uint64_t c0 = __ballot(cnt & 1u), c1 = __ballot(cnt & 2u);
                const uint32_t pre = mbcnt64(c0) + 2u * mbcnt64(c1);
                const uint32_t total = (uint32_t)__popcll(c0) + 2u * (uint32_t)__popcll(c1);   // (uniform)
                const uint32_t take = pre >= (uint32_t)kWave ? 0u : min(cnt, (uint32_t)kWave - pre);
                const uint32_t own = (uint32_t)lane << 26;   // slot entry: owner << 26 | primitive (< 2^26)
                if (take > 0u) { leafQ[pre] = own | (tgBase + (uint32_t)__builtin_ctz(tg)); tg &= tg - 1u; }
                if (CAP > 1 && take > 1u) { leafQ[pre + 1u] = own | (tgBase + (uint32_t)__builtin_ctz(tg)); tg &= tg - 1u; }
                if (CAP > 2 && take > 2u) { leafQ[pre + 2u] = own | (tgBase + (uint32_t)__builtin_ctz(tg)); tg &= tg - 1u; }
                __syncthreads();   // (one wave per workgroup: orders the slot writes before the reads)
                const uint32_t nc = total < (uint32_t)kWave ? total : (uint32_t)kWave;
                PT_DIAG_ADD(sPops, nc);
                // lanes past the last pair re-test a stale (valid) entry; their results are not read
                const uint32_t e = leafQ[lane];
                const int ow = (int)(e >> 26);
                const float3 ro = f3(__shfl(o.x, ow), __shfl(o.y, ow), __shfl(o.z, ow));
                const float3 rd = f3(__shfl(d.x, ow), __shfl(d.y, ow), __shfl(d.z, ow));
                const float4* w0 = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(S.wprims) + mul48(e & 0x3ffffffu));
                const Prim q0{w0[0], w0[1], w0[2]};
                const bool lb = S.nprims > 1;
                const bool cons = (uint32_t)lane < nc;
                float rt, rlo = -__builtin_inff();
                uint32_t rkey;
                if (kargs()->S.hasSpheres) {   // (uniform)
                    const bool sph = __float_as_uint(q0.p2.w) != 0u;
                    rt = primHitAny(q0, sph, ro, rd, 0.001f);
                    if (lb) {
                        const float3 rinv = f3(__shfl(inv.x, ow), __shfl(inv.y, ow), __shfl(inv.z, ow));
                        const SlabHit b = refLeafBox(q0, sph, ro, rinv, 0.001f, __builtin_inff());
                        rlo = b.hit ? b.lo : -1.0f;   // (a hit's entry is >= tmin > 0)
                    }
                    rkey = __float_as_uint(q0.p0.w) | (sph ? kSphereBit : 0u);
                    sTris += (uint32_t)__popcll(__ballot(cons && !sph));
                    sSph += (uint32_t)__popcll(__ballot(cons && sph));
                } else {
                    rt = primHitAny(q0, false, ro, rd, 0.001f);
                    if (lb) {
                        const float3 rinv = f3(__shfl(inv.x, ow), __shfl(inv.y, ow), __shfl(inv.z, ow));
                        const SlabHit b = refLeafBox(q0, false, ro, rinv, 0.001f, __builtin_inff());
                        rlo = b.hit ? b.lo : -1.0f;
                    }
                    rkey = __float_as_uint(q0.p0.w);
                    sTris += nc;
                }
                bool redo = false;
                const bool sphScene = kargs()->S.hasSpheres != 0;
#pragma unroll
                for (uint32_t r = 0; r < CAP; r++) {
                    if (__ballot(take > r) == 0) break;
                    const int src = (int)(pre + r);
                    const float t = __shfl(rt, src);
                    const float blo = __shfl(rlo, src);
                    const uint32_t key = (uint32_t)__shfl((int)rkey, src);
                    if (take > r) {
                        if (sphScene) wideMerge<true>(t, key, blo, closest, best, bestLo, lb, redo);
                        else wideMerge<false>(t, key, blo, closest, best, bestLo, lb, redo);
                    }
                }
                if (redo) oct |= 8u;   // order-dependent candidate: repeat the query in the reference's order
                if (SPEC && tg == 0u && (oct & 48u)) {   // this group is done: the last parked one is next
                    oct -= 16u;
                    const uint32_t c = SPECN == 1 ? 0u : (oct >> 4) & 3u;
                    tgBase = pend[(2u * c) * kWave + lane];
                    tg = pend[(2u * c + 1u) * kWave + lane];
                }
            } else if constexpr (WIDE) {
                PT_DIAG_ADD(sPops, (uint32_t)nL);
                // up to two primitives of the group per step, both records loaded up front
                uint32_t k0 = 0u, k1 = 0u;
                const bool h0 = tg != 0u;
                if (h0) { k0 = tgBase + (uint32_t)__builtin_ctz(tg); tg &= tg - 1u; }
                const bool h1 = tg != 0u;
                if (h1) { k1 = tgBase + (uint32_t)__builtin_ctz(tg); tg &= tg - 1u; }
                // Every lane loads two records (lanes without a primitive read record 0): a
                // conditional load would cost a zero fill of 24 registers per step
                // 32-bit byte offsets off the uniform base (global loads with an SGPR base): no
                // 64-bit address arithmetic, no quarter-rate multiply
                const float4* w0 = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(S.wprims) + mul48(k0));
                const float4* w1 = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(S.wprims) + mul48(k1));
                const Prim q0{w0[0], w0[1], w0[2]}, q1{w1[0], w1[1], w1[2]};
                bool redo = false;
#ifdef PT_DIAG
                {   // tests the reference would skip: the primitive's exact box misses with the
                    // closest hit of this moment (its own leaf test, render_manager.h:107-123)
                    const bool a0 = h0 && !refLeafBox(q0, __float_as_uint(q0.p2.w) != 0u, o, inv, 0.001f, closest).hit;
                    const bool a1 = h1 && !refLeafBox(q1, __float_as_uint(q1.p2.w) != 0u, o, inv, 0.001f, closest).hit;
                    sAvoid += (unsigned long long)(__popcll(__ballot(a0)) + __popcll(__ballot(a1)));
                    sHalf += (unsigned long long)__popcll(__ballot(h0 && !h1));
                    const bool i0 = h0 && !refLeafBox(q0, __float_as_uint(q0.p2.w) != 0u, o, inv, 0.001f, __builtin_inff()).hit;
                    const bool i1 = h1 && !refLeafBox(q1, __float_as_uint(q1.p2.w) != 0u, o, inv, 0.001f, __builtin_inff()).hit;
                    sAvoidInf += (unsigned long long)(__popcll(__ballot(i0)) + __popcll(__ballot(i1)));
                    const bool pk = !INST && (oct & 64u) != 0u;
                    sParkT += (unsigned long long)(__popcll(__ballot(pk && h0)) + __popcll(__ballot(pk && h1)));
                    sParkA += (unsigned long long)(__popcll(__ballot(pk && a0)) + __popcll(__ballot(pk && a1)));
                }
#endif
                // (instanced: no reference leaf-box rule; the hit key carries the instance)
                const bool lb = !INST && S.nprims > 1;
                const uint32_t kh = INST ? (oct >> 8) << kargs()->S.gBits : 0u;
                if (kargs()->S.hasSpheres) {   // (uniform: read where needed)
                    if (h0) wideTest<true>(q0, o, d, inv, 0.001f, closest, best, bestLo, lb, redo, kh);
                    if (h1) wideTest<true>(q1, o, d, inv, 0.001f, closest, best, bestLo, lb, redo, kh);
                    const bool s0 = __float_as_uint(q0.p2.w) != 0u, s1 = __float_as_uint(q1.p2.w) != 0u;
                    sTris += (uint32_t)__popcll(__ballot(h0 && !s0)) + (uint32_t)__popcll(__ballot(h1 && !s1));
                    sSph += (uint32_t)__popcll(__ballot(h0 && s0)) + (uint32_t)__popcll(__ballot(h1 && s1));
                } else {
                    if (h0) wideTest<false>(q0, o, d, inv, 0.001f, closest, best, bestLo, lb, redo, kh);
                    if (h1) wideTest<false>(q1, o, d, inv, 0.001f, closest, best, bestLo, lb, redo, kh);
                    sTris += (uint32_t)__popcll(__ballot(h0)) + (uint32_t)__popcll(__ballot(h1));
                }
                if (redo) oct |= 8u;   // order-dependent candidate: repeat the query in the reference's order
                if (SPEC && tg == 0u && (oct & 48u)) {   // this group is done: the last parked one is next
                    oct -= 16u;
                    const uint32_t c = SPECN == 1 ? 0u : (oct >> 4) & 3u;
                    tgBase = pend[(2u * c) * kWave + lane];
                    tg = pend[(2u * c + 1u) * kWave + lane];
#ifdef PT_DIAG
                    oct |= 64u;
#endif
                }
            } else {
            PT_DIAG_ADD(sPops, (uint32_t)nL);
            // Every lane tests all of its queued leaves, in order, in this step (the queue then
            // is empty and the lane rejoins NODE steps; measured -4 % vs one leaf per step).
            // The first two queued primitives are loaded together up front (their addresses are
            // known; only the tests depend on `closest`): one memory round trip for two leaves.
            Prim pf0{}, pf1{};
            if (qn > 0) pf0 = loadPrim(S, qref[0] & kPrimMask);
            if (qn > 1) pf1 = loadPrim(S, qref[1] & kPrimMask);
#pragma unroll
            for (int k_ = 0; k_ < LQ; k_++) {
                const bool act = qn > 0;
                if (__ballot(act) == 0) break;
                tested = false;
                sph = false;
            if (act) {
                const uint32_t ref = qref[0];
                const float lo = lq[0];
#pragma unroll
                for (int i = 0; i + 1 < LQ; i++) { qref[i] = qref[i + 1]; lq[i] = lq[i + 1]; }
                qn--;
                const uint32_t k = ref & kPrimMask;
                sph = (ref & kSphereBit) != 0;
                // Exact re-test of the leaf box with the current closest: the box passed when it
                // was queued, with a tmax >= closest, so now it fails iff closest < lo (slabLo).
                if (!(closest < lo)) {
                    const Prim pr = k_ == 0 ? pf0 : (k_ == 1 ? pf1 : loadPrim(S, k));
                    // (wide: a leaf that waited on the stack has no entry distance, lo = -inf:
                    // exact re-test of its box from the primitive's vertices)
                    {
                        tested = true;
                        const float t = primHitT(pr, sph, o, d, 0.001f, closest);
                        if (t >= 0.0f) { closest = t; best = (int)k; }
                    }
                }
            }
            sTris += (uint32_t)__popcll(__ballot(tested && !sph));
            sSph += (uint32_t)__popcll(__ballot(tested && sph));
            }
            }
        }
        if (kind == 2) {
            // ------------------------------------------------------------------ SHADE
            if constexpr (WIDE) {
                // rare: an order-dependent query (or a far origin), repeated in the reference's
                // order.  Ranks index wshade.
                const bool redo = !INST && wantShade && !needTask && (oct & 8u);
                PT_DIAG_ADD(sRedo, (uint32_t)__popcll(__ballot(redo)));
                if (redo) {
                    const DevScene S2 = ldScene(kargs());
                    closest = __builtin_inff();
                    const int k = traceRefStackless(S2, o, d, 0.001f, closest);
                    best = k >= 0 ? (int)S2.rankOf[k] : -1;
                }
            }
            bool newRay = false, newSample = false;
            PT_DIAG_ADD(itS, 1u);
            if (wantShade && !needTask) {
                bool done = false;
                float3 contrib = f3(0.0f, 0.0f, 0.0f);
                if (best < 0) {
                    contrib = sky(d, att);
                    done = true;
                } else {
                    int objI_;
                    HitRec h = INST ? makeHitInst(ldScene(kargs()), (uint32_t)best & kPrimMask, closest, o, d, objI_)
                                    : (WIDE ? makeHitFrom(kargs()->S.wshade, best & (int)kPrimMask, closest, o, d)
                                            : makeHit(S, best, closest, o, d));
                    if (!scatterInto(h, d, att, g)) {
                        done = true;
                    } else {
                        o = h.p;
                        if (depthLeft == 0) { contrib = sky(d, att); done = true; }
                    }
                }
                if (done) {
                    sum = add(sum, contrib);
                    if constexpr (SAMPLE) {
                        uint4 ts = taskState[lane];
                        ts.y++;
                        taskState[lane].y = ts.y;
                        if (ts.y == ts.z) {
                            active = false;
                            PT_FINISH_TASK(ts);
                        } else {
                            PT_CLOSE_BLOCK(ts.y);
                            newSample = true;
                        }
                    } else {
                        ++sample;
                        if (sample == nSamples) {
                            active = false;
                            if constexpr (CQ) PT_FINISH_PIXEL();
                        } else {
                            newSample = true;
                        }
                    }
                }
                newRay = true;   // bounce, next sample (newSample) or finished (reset below)
                if (!active) newRay = false;
            }
#ifdef PT_DIAG
            const unsigned long long tS1 = __builtin_amdgcn_s_memtime();
#endif
            if constexpr (SAMPLE) {   // idle lanes take new tasks and start their first path
                bool got = false;
                PT_TAKE_TASKS(got);
                if (got) {
                    active = true;
                    newRay = newSample = true;
                }
            } else if constexpr (CQ) {   // idle lanes take new pixels and start their first sample
                bool got = false;
                PT_TAKE_PIXELS(got);
                if (got) {
                    active = true;
                    newRay = newSample = true;
                }
            }
            // one camera-ray and one ray-start site for every lane that needs them
#ifdef PT_DIAG
            const unsigned long long tS2 = __builtin_amdgcn_s_memtime();
#endif
            if (newSample) PT_NEW_PATH();
#ifdef PT_DIAG
            const unsigned long long tS3 = __builtin_amdgcn_s_memtime();
#endif
            if (newRay) PT_BEGIN_RAY();
#ifdef PT_DIAG
            const unsigned long long tS4 = __builtin_amdgcn_s_memtime();
            cycSh += tS1 - tK0; cycTk += tS2 - tS1; cycNp += tS3 - tS2; cycBr += tS4 - tS3;
#endif
            sRays += (uint32_t)__popcll(__ballot(newRay));
            sPaths += (uint32_t)__popcll(__ballot(newSample));
        }
#ifdef PT_DIAG
        {   // shader-clock cycles per step kind (the step's memory waits included)
            const unsigned long long dK = __builtin_amdgcn_s_memtime() - tK0;
            if (kind == 0) cycN += dK;
            else if (kind == 1) cycL += dK;
            else cycS += dK;
        }
#endif
    }
    if constexpr (!SAMPLE && !CQ) {   // (sample mode / CQ: every task wrote its result when it ended)
        if (valid) {
            storePixel(P, idx, sum);
            P.sd[idx] = g.d; P.s0[idx] = g.v0; P.s1[idx] = g.v1; P.s2[idx] = g.v2; P.s3[idx] = g.v3; P.s4[idx] = g.v4;
            if (CRITK && P.pixRays) P.pixRays[idx] = pxRays;   // (the next launch's critical pixels)
        }
    }
    const unsigned long long tEnd = __builtin_amdgcn_s_memrealtime();
#if PT_AB_COST_STORE
    if (!SAMPLE && !CQ && !crit && lane == 0) P.tileCost[tile] = (unsigned)min(tEnd - tStart, 0xffffffffull);
#else
    if (!SAMPLE && !CQ && !crit && lane == 0) atomicMax(P.tileCost + tile, (unsigned)min(tEnd - tStart, 0xffffffffull));   // (split tiles: several waves)
#endif
    if constexpr (SAMPLE) {   // max_depth <= 0: paths counted per lane

    }
    if (P.waveTimes && lane == 0) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        P.waveTimes[3 * (size_t)blockIdx.x + 0] = tStart;
        P.waveTimes[3 * (size_t)blockIdx.x + 1] = tEnd;
        P.waveTimes[3 * (size_t)blockIdx.x + 2] = (unsigned long long)tile | ((unsigned long long)(xcc & 0xf) << 32);
    }
    if (lane == 0) {
        atomicAdd(P.counters + 0, (unsigned long long)sRays);
        atomicAdd(P.counters + 1, (unsigned long long)sVisits);
        atomicAdd(P.counters + 2, (unsigned long long)sTris);
        atomicAdd(P.counters + 3, (unsigned long long)sSph);
        atomicAdd(P.counters + 4, (unsigned long long)sPaths);
#ifdef PT_DIAG
        atomicAdd(P.counters + 8, (unsigned long long)itN);
        atomicAdd(P.counters + 9, (unsigned long long)itL);
        atomicAdd(P.counters + 10, (unsigned long long)itS);
        atomicAdd(P.counters + 11, (unsigned long long)sPops);
        atomicAdd(P.counters + 12, cycN);
        atomicAdd(P.counters + 13, cycL);
        atomicAdd(P.counters + 14, cycS);
        atomicAdd(P.counters + 15, cycH);
        atomicAdd(P.counters + 16, cycSh);
        atomicAdd(P.counters + 17, cycTk);
        atomicAdd(P.counters + 18, cycNp);
        atomicAdd(P.counters + 19, cycBr);
        atomicAdd(P.counters + 20, (unsigned long long)sRedo);
        atomicAdd(P.counters + 21, sSpecN);
        atomicAdd(P.counters + 22, sIdleN);
        atomicAdd(P.counters + 23, sAvoid);
        atomicAdd(P.counters + 25, sHalf);
        atomicAdd(P.counters + 26, sAvoidInf);
        atomicAdd(P.counters + 27, sParkT);
        atomicAdd(P.counters + 28, sParkA);
#endif
    }
}
#undef PT_BEGIN_RAY
#undef PT_CRIT_TRACE
#undef PT_NEW_PATH
#undef PT_TAKE_TASKS
#undef PT_FINISH_TASK
#undef PT_TAKE_PIXELS
#undef PT_FINISH_PIXEL
#undef PT_CLOSE_BLOCK
#undef PT_DIAG_ADD

#ifdef PT_TU_COMPAT
}  // namespace

// pt_compat.hip compiles this file a second time with PT_TU_COMPAT: only the device code above and
// this launcher of the compat-mode wide kernels (renderKernelWF<S, false, true>), built WITHOUT the
// -mllvm --enable-post-misched=0 of the main translation unit.  That flag speeds the sample-mode
// kernels up but slows the compat kernel -- one sequential chain of samples per pixel -- by 3.5 %
// (DESIGN.md section 6), and it is a per-file option.
namespace pt {
int launchCompatWide(int stack, const void* params, hipStream_t st) {
    const RenderParams& P = *static_cast<const RenderParams*>(params);
    const int grid = PT_COMPAT_QUEUE ? P.nwaves : P.compatGrid;   // persistent waves with the pixel queue
    switch (stack) {
        case 8: renderKernelWF<8, false, true><<<grid, kWave, 0, st>>>(P); break;
        case 16: renderKernelWF<16, false, true><<<grid, kWave, 0, st>>>(P); break;
        case 24: renderKernelWF<24, false, true><<<grid, kWave, 0, st>>>(P); break;
        default: return -1;
    }
    return 0;
}
int compatWideWavesPerCU(int stack, int& n) {
    const void* k = stack == 8 ? reinterpret_cast<const void*>(&renderKernelWF<8, false, true>)
                  : stack == 16 ? reinterpret_cast<const void*>(&renderKernelWF<16, false, true>)
                  : stack == 24 ? reinterpret_cast<const void*>(&renderKernelWF<24, false, true>) : nullptr;
    if (!k || hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kWave, 0) != hipSuccess) return -1;
    return 0;
}
}  // namespace pt
#else

// Frame epilogue (one lane per pixel).  The frame's linear sum S is the raw compat sum
// (`nblocks` = 0) or, in sample mode, the block sums added in order.  Accumulating films keep
// A += S over frames (progressive rendering, the headless counterpart of the reference's
// interactive loop, main.cu:489-528) and resolve sqrt(A * (1 / samples so far)); otherwise
// sqrt(S * (1 / spp)) (main.cu:290-293).  Output: fp32 RGB, or 8-bit RGBA quantised like
// PngImage::saveColor (png_image.h:24-30: (uint8)(clamp(c, 0, 0.999) * 256), alpha 255) or like
// renderBySurface (main.cu:327-331: (unsigned)(c * 255) into an 8-bit field, alpha 255).
// Rows stay in film order (row 0 = bottom); the PNG writer flips them.
// Sample mode: the pixel's 32-B accumulator {x, y, z (32.32 fixed point), rays}; its rays are
// added to its tile's cost (the next launch's longest-first order).
__global__ __launch_bounds__(256) void resolveKernel(const float* __restrict__ src,
                                                     const unsigned long long* __restrict__ pixAcc, float* accum,
                                                     float inv, int format, void* out, int64_t npix,
                                                     unsigned* tileCost, int width, int tilesX, int costMax) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    float x, y, z;
    if (!pixAcc) {
        x = src[3 * i + 0]; y = src[3 * i + 1]; z = src[3 * i + 2];
    } else {
        const ulonglong2* a2 = reinterpret_cast<const ulonglong2*>(pixAcc + 4 * i);
        const ulonglong2 a = a2[0], b = a2[1];
        x = fixedToFloat(a.x);
        y = fixedToFloat(a.y);
        z = fixedToFloat(b.x);
        const uint32_t rays = (uint32_t)min(b.y, 0xffffffffull);
        if (tileCost) {
            const int row = (int)(i / width), col = (int)(i - (int64_t)row * width);
            unsigned* tc = tileCost + (row >> 3) * tilesX + (col >> 3);
            if (costMax) atomicMax(tc, rays);
            else atomicAdd(tc, rays);
        }
    }
    if (accum) {
        float* a = accum + 3 * i;
        x = a[0] + x; y = a[1] + y; z = a[2] + z;
        a[0] = x; a[1] = y; a[2] = z;
    }
    const float c[3] = {sqrtf(x * inv), sqrtf(y * inv), sqrtf(z * inv)};
    if (format == PT_OUT_RGB32F) {
        float* o = static_cast<float*>(out) + 3 * i;
        o[0] = c[0]; o[1] = c[1]; o[2] = c[2];
        return;
    }
    uint32_t px = 0xff000000u;
    for (int k = 0; k < 3; k++) {
        uint32_t b;
        if (format == PT_OUT_RGBA8) {
            float v = c[k];                  // utility.h:40-44 clamp(x, 0, 0.999f), then * 256
            if (v < 0.0f) v = 0.0f;
            if (v > 0.999f) v = 0.999f;
            b = (uint32_t)(v * 256.0f);
        } else {
            b = (uint32_t)(c[k] * 255.0f) & 0xffu;
        }
        px |= b << (8 * k);
    }
    static_cast<uint32_t*>(out)[i] = px;
}

// Longest-first launch order on the device: keys ~cost (ascending = cost descending) and tile ids,
// then a stable radix sort (pt_sort.hip): equal costs keep ascending tile ids.
// Sample mode: each launch slot's tile as tx | ty << 16 (`order` = the longest-first launch order,
// null = identity), so the task hand-out does no divisions per take.
__global__ __launch_bounds__(256) void tileXYKernel(const uint32_t* __restrict__ order, int n, int tilesX, uint32_t* xy) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = order ? order[i] : (uint32_t)i;
    const uint32_t ty = t / (uint32_t)tilesX;
    xy[i] = (t - ty * (uint32_t)tilesX) | (ty << 16);
}

// compat: mark the next launch's critical pixels (the first k of the pixels sorted by rays)
__global__ __launch_bounds__(256) void critFlagKernel(const uint32_t* __restrict__ sorted, int k, uint8_t* flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) flag[sorted[i]] = 1;
}

__global__ __launch_bounds__(256) void tileKeyKernel(const unsigned* __restrict__ cost, uint32_t* keys, uint32_t* ids,
                                                     int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = ~cost[i];
    ids[i] = (uint32_t)i;
}

// pt_trace_closest on the binary LBVH, in the reference order (trace<STACK>).
template <int STACK>
__global__ __launch_bounds__(kWave) void traceKernel(DevScene S, const pt_ray* rays, int64_t n, float tmin,
                                                     float tmax, pt_hit* hits, unsigned long long* counters) {
    __shared__ uint32_t stk[STACK * kWave];
    const int lane = threadIdx.x;
    Counters c{0, 0, 0, 0};
    // grid-stride over the batch: the counters are summed once per wave at the end (one global
    // atomic per counter per wave of a 64-ray block was the bottleneck of large batches)
    for (int64_t base = (int64_t)blockIdx.x * kWave; base < n; base += (int64_t)gridDim.x * kWave) {
    const int64_t i = base + lane;
    if (i < n) {
        const pt_ray r = rays[i];
        const float3 o = f3(r.o[0], r.o[1], r.o[2]), d = f3(r.d[0], r.d[1], r.d[2]);
        float closest = tmax;
        c.rays++;
        const int k = trace<STACK>(S, o, d, tmin, closest, stk + lane, c);
        pt_hit h = {};
        h.obj = -1;
        h.mat = -1;
        if (k >= 0) {
            HitRec hr = makeHit(S, k, closest, o, d);
            h.hit = 1;
            h.obj = hr.obj;
            h.mat = hr.mat;
            h.front_face = hr.front ? 1 : 0;
            h.t = closest;
            h.p[0] = hr.p.x; h.p[1] = hr.p.y; h.p[2] = hr.p.z;
            h.n[0] = hr.n.x; h.n[1] = hr.n.y; h.n[2] = hr.n.z;
        }
        hits[i] = h;
    }
    }
    waveReduceAdd(counters + 0, c.rays);
    waveReduceAdd(counters + 1, c.visits);
    waveReduceAdd(counters + 2, c.tris);
    waveReduceAdd(counters + 3, c.spheres);
}

// pt_trace_closest on the wide tree (PT_KERNEL_WIDE): the same traversal as renderKernelWF's
// WIDE steps, one lane per ray, the same hit records as traceKernel.  INST: an instanced scene's
// two-level tree (renderKernelWF<.., INST>).
template <int STACK, bool INST>
__global__ __launch_bounds__(kWave) void traceKernelWide(DevScene S, const pt_ray* rays, int64_t n, float tmin,
                                                         float tmax, pt_hit* hits, unsigned long long* counters) {
    __shared__ uint32_t stk[STACK * kWave];
    const int lane = threadIdx.x;
    uint32_t* my = stk + lane;
    const __amdgpu_buffer_rsrc_t nodeRsrc = rawRsrc(S.wnodes);
    Counters c{0, 0, 0, 0};
    for (int64_t base = (int64_t)blockIdx.x * kWave; base < n; base += (int64_t)gridDim.x * kWave) {   // grid-stride
    const int64_t i = base + lane;
    if (i < n) {
        const pt_ray r = rays[i];
        const float3 wo = f3(r.o[0], r.o[1], r.o[2]), wd = f3(r.d[0], r.d[1], r.d[2]);
        const float3 winv = f3(rcpRN(wd.x), rcpRN(wd.y), rcpRN(wd.z));
        const uint32_t woct = (winv.x < 0.0f ? 1u : 0u) | (winv.y < 0.0f ? 2u : 0u) | (winv.z < 0.0f ? 4u : 0u);
        float3 o = wo, d = wd, inv = winv;   // (inside an instance: its object space)
        uint32_t oct = woct, inst = 0u;
        // (far origin, or a direction the MIX planes cannot take: the query in the reference's order only)
        const bool far = !INST && (wideFar(S, o) || (PT_WIDE_MIX && mixUnsafe(winv, S.mixLim)));
        // instanced: a far origin moves to the ray's entry into the world (instEntry); distances
        // are then measured from there and shifted back at the end
        float3 wo2 = wo;
        const float shift = (INST && instFar(S, wo)) ? instEntry(S.cx, S.cy, S.cz, S.ext, wo2, wd, winv) : 0.0f;
        if (INST) o = wo2;
        const float tminI = tmin - shift;   // (tmin, tmax of the moved ray: t - shift)
        float closest = tmax - shift;
        int best = -1, sp = 0;
        bool redo = far;
        float bestLo = -__builtin_inff();
        uint32_t ng = S.nprims > 0 && !far ? (1u << oct) : 0u, tgBase = 0u, tg = 0u;
        c.rays++;
        for (;;) {
            while (tg) {
                const uint32_t k = tgBase + (uint32_t)__builtin_ctz(tg);
                tg &= tg - 1u;
                const float4* w = S.wprims + 3 * (size_t)k;
                const Prim q{w[0], w[1], w[2]};
                if (__float_as_uint(q.p2.w) != 0u) c.spheres++;
                else c.tris++;
                const bool lb = !INST && S.nprims > 1;
                const uint32_t kh = INST ? inst << S.gBits : 0u;
                if (S.hasSpheres) wideTest<true>(q, o, d, inv, tminI, closest, best, bestLo, lb, redo, kh);
                else wideTest<false>(q, o, d, inv, tminI, closest, best, bestLo, lb, redo, kh);
            }
            if constexpr (INST) {   // pop; a marker returns to the world ray
                while ((ng & 0xffu) == 0u && sp > 0) {
                    sp--;
                    ng = my[sp * kWave];
                    if (ng == kInstMarker) { o = wo2; d = wd; inv = winv; oct = woct; ng = 0u; }
                }
                if ((ng & 0xffu) == 0u) break;
            } else if ((ng & 0xffu) == 0u) {
                if (sp == 0) break;
                sp--;
                ng = my[sp * kWave];
            }
            const uint32_t bit = (uint32_t)__builtin_ctz(ng & 0xffu);
            const uint32_t child = (ng >> 8) + (bit ^ oct);
            ng &= ~(1u << bit);
            if (ng & 0xffu) {
                if (sp >= STACK) { atomicOr(S.err, 2u); break; }
                my[sp * kWave] = ng;
                sp++;
            }
            c.visits++;
            const uint32_t off = mul80(child);
            const uint4 n0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off, 0, 0));
            const uint4 n1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 16u, 0, 0));
            const uint4 n2 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 32u, 0, 0));
            const uint4 n3 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 48u, 0, 0));
            const uint4 n4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 64u, 0, 0));
            if (INST && n0.w == kInstFlag) {   // an instance: into its object space and bottom-level tree
                if (n0.x == 0u) {
                    const float4 r0 = __builtin_bit_cast(float4, n2), r1 = __builtin_bit_cast(float4, n3),
                                 r2 = __builtin_bit_cast(float4, n4);
                    o = xformPoint(r0, r1, r2, wo2);
                    d = xformDir(r0, r1, r2, wd);
                    inv = f3(rcpRN(d.x), rcpRN(d.y), rcpRN(d.z));
                    oct = (inv.x < 0.0f ? 1u : 0u) | (inv.y < 0.0f ? 2u : 0u) | (inv.z < 0.0f ? 4u : 0u);
                }
                if (sp >= STACK) { atomicOr(S.err, 2u); break; }
                my[sp * kWave] = kInstMarker;
                sp++;
                ng = (n1.x << 8) | (1u << oct);
                inst = n1.y;
                tg = 0u;
                continue;
            }
            const uint32_t h = INST ? wideHitsInst(n0, n1, n2, n3, n4, o, inv, oct, tminI, closest)
                                    : wideHits<PT_WIDE_MIX != 0>(n0, n1, n2, n3, n4, o, inv, oct, tminI, closest);
            ng = (n1.x << 8) | (h >> 24);
            tgBase = n1.y;
            tg = h & 0xffffffu;
        }
        if (redo) {   // an order-dependent candidate: the query in the reference's order
            closest = tmax;
            const int k = traceRefStackless(S, o, d, tmin, closest);
            best = k >= 0 ? (int)S.rankOf[k] : -1;
        }
        pt_hit hr = {};
        hr.obj = -1;
        hr.mat = -1;
        if (best >= 0) {
            int obj = 0;
            HitRec x = INST ? makeHitInst(S, (uint32_t)best & kPrimMask, closest, wo2, wd, obj)
                            : makeHitFrom(S.wshade, best & (int)kPrimMask, closest, o, d);
            hr.hit = 1;
            hr.obj = x.obj;
            hr.mat = x.mat;
            hr.front_face = x.front ? 1 : 0;
            hr.t = INST ? closest + shift : closest;
            hr.p[0] = x.p.x; hr.p[1] = x.p.y; hr.p[2] = x.p.z;
            hr.n[0] = x.n.x; hr.n[1] = x.n.y; hr.n[2] = x.n.z;
        }
        hits[i] = hr;
    }
    }
    waveReduceAdd(counters + 0, c.rays);
    waveReduceAdd(counters + 1, c.visits);
    waveReduceAdd(counters + 2, c.tris);
    waveReduceAdd(counters + 3, c.spheres);
}

// Queued closest-hit kernels (the default for pt_trace_closest; PT_TRACE_STRIDE=1 selects the
// grid-stride kernels above).  Persistent waves with a wave-level ray queue (Aila & Laine 2009,
// "persistent while-while" with dynamic fetch): a lane whose ray has finished takes the next
// ray of the batch at the top of the next loop iteration instead of idling until the wave's
// slowest ray is done.  The lanes that ask are ranked by a ballot and an mbcnt prefix count and
// served, in lane order, from the wave's pool of kTraceGrab consecutive rays (one returning
// atomic per pool on a queue word of the scene's counters).  Each loop iteration runs one
// traversal step per lane -- the reference order's node visit with its leaf tests (traceKernel),
// or the wide tree's primitive group + next node (traceKernelWide) -- with exactly those
// kernels' arithmetic, so every hit record and work counter is the same.
#ifndef PT_TRACE_GRAB
#define PT_TRACE_GRAB 256   // rays per queue grab (a wave's pool)
#endif
constexpr uint32_t kTraceGrab = PT_TRACE_GRAB;
#ifndef PT_TRACE_DIAG_REDO
#define PT_TRACE_DIAG_REDO 0   // diagnostic builds: count the queries that take the reference-order redo as sphere tests
#endif
#ifndef PT_TRACE_DIAG_VISITS
#define PT_TRACE_DIAG_VISITS 0   // diagnostic builds: each hit record's `mat` = the query's wide node visits
#endif
#ifndef PT_TRACE_WAVES
#define PT_TRACE_WAVES 1   // occupancy target of the queued trace kernels (waves per SIMD; 1 = the compiler's choice)
#endif
constexpr int kTraceQueue = 24;   // counters[24]: the ray queue (zeroed with the counters before each trace)

// Hand rays to the lanes that have none (`ray` < 0): ballot of the askers, each asker's rank among
// them (mbcnt), one pool refill by the first asker when the pool is empty.  poolBase / poolLeft /
// more are wave-uniform; `took` is set for a lane that received ray `ray` (< n).
#define PT_TRACE_REFILL(took)                                                                       \
    do {                                                                                          \
        for (;;) {                                                                                \
            const uint64_t m_ = __ballot(ray < 0 && more);                                        \
            if (m_ == 0) break;                                                                   \
            if (poolLeft == 0u) {                                                                 \
                const int leader_ = __ffsll((unsigned long long)m_) - 1;                          \
                unsigned long long b_ = 0;                                                        \
                if (lane == leader_) b_ = atomicAdd(counters + kTraceQueue, (unsigned long long)kTraceGrab); \
                const uint32_t lo_ = (uint32_t)__shfl((int)(uint32_t)b_, leader_);                \
                const uint32_t hi_ = (uint32_t)__shfl((int)(uint32_t)(b_ >> 32), leader_);         \
                poolBase = (int64_t)(((uint64_t)__builtin_amdgcn_readfirstlane(hi_) << 32) |       \
                                     __builtin_amdgcn_readfirstlane(lo_));                        \
                poolLeft = kTraceGrab;                                                            \
                if (poolBase >= n) { more = false; break; }                                       \
            }                                                                                     \
            const uint32_t take_ = min((uint32_t)__popcll(m_), poolLeft);                         \
            const uint32_t k_ = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m_ >> 32),         \
                                    __builtin_amdgcn_mbcnt_lo((uint32_t)m_, 0u));                 \
            if (ray < 0 && k_ < take_ && poolBase + (int64_t)k_ < n) {                            \
                ray = poolBase + (int64_t)k_;                                                     \
                took = true;                                                                      \
            }                                                                                     \
            poolBase += take_;                                                                    \
            poolLeft -= take_;                                                                    \
            if (poolBase >= n) more = false;                                                      \
        }                                                                                         \
    } while (0)

// traceKernel (the reference's order, render_manager.h:86-135) with the ray queue: one node visit
// (both children's slab tests and leaf tests, trace<STACK>) per lane and iteration.
template <int STACK>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(PT_TRACE_WAVES))) void traceKernelQ(DevScene S, const pt_ray* rays, int64_t n, float tmin,
                                                      float tmax, pt_hit* hits, unsigned long long* counters) {
    __shared__ uint32_t stk[STACK * kWave];
    const int lane = threadIdx.x;
    uint32_t* my = stk + lane;
    Counters c{0, 0, 0, 0};
    int64_t ray = -1, poolBase = 0;
    uint32_t poolLeft = 0u;
    bool more = true;
    float3 o = f3(0.0f, 0.0f, 0.0f), d = o, inv = o;
    float closest = 0.0f;
    int best = -1, node = 0, sp = 0, guard = 0;
    for (;;) {
        bool took = false;
        PT_TRACE_REFILL(took);
        if (__ballot(ray >= 0) == 0) break;
        if (ray < 0) continue;
        bool fin = false;
        if (took) {   // the query's start (trace<STACK>)
            const pt_ray r = rays[ray];
            o = f3(r.o[0], r.o[1], r.o[2]);
            d = f3(r.d[0], r.d[1], r.d[2]);
            closest = tmax;
            best = -1;
            c.rays++;
            if (S.nprims <= 1) {
                if (S.nprims == 1) {   // root is a leaf: tested without a box test (:92-98)
                    const uint32_t ref = kLeafBit | (__float_as_uint(S.prims[2].w) ? kSphereBit : 0u);
                    primTest(S, ref, o, d, tmin, closest, best, c);
                }
                fin = true;
            } else {
                inv = f3(rcpRN(d.x), rcpRN(d.y), rcpRN(d.z));
                node = 0;
                sp = 0;
                guard = 0;
            }
        }
        if (!fin) {   // one node visit of trace<STACK>
            if (++guard > S.nprims) { atomicOr(S.err, 1u); fin = true; }
            else {
                c.visits++;
                const float4* np = S.nodes + 4 * (size_t)node;
                const float4 a = np[0], b = np[1], q = np[2], rr = np[3];
                const uint32_t lref = __float_as_uint(rr.x), rref = __float_as_uint(rr.y);
                if (slabLeft(a, b, o, inv, tmin, closest).hit) {
                    if (lref & kLeafBit) primTest(S, lref, o, d, tmin, closest, best, c);
                    else if (sp < STACK) { my[sp * kWave] = lref; sp++; }
                    else { atomicOr(S.err, 2u); fin = true; }
                }
                if (!fin && slabRight(b, q, o, inv, tmin, closest).hit) {
                    if (rref & kLeafBit) primTest(S, rref, o, d, tmin, closest, best, c);
                    else if (sp < STACK) { my[sp * kWave] = rref; sp++; }
                    else { atomicOr(S.err, 2u); fin = true; }
                }
                if (!fin) {
                    if (sp == 0) fin = true;
                    else { sp--; node = (int)my[sp * kWave]; }
                }
            }
        }
        if (fin) {   // the hit record (traceKernel)
            pt_hit h = {};
            h.obj = -1;
            h.mat = -1;
            if (best >= 0) {
                HitRec hr = makeHit(S, best, closest, o, d);
                h.hit = 1;
                h.obj = hr.obj;
                h.mat = hr.mat;
                h.front_face = hr.front ? 1 : 0;
                h.t = closest;
                h.p[0] = hr.p.x; h.p[1] = hr.p.y; h.p[2] = hr.p.z;
                h.n[0] = hr.n.x; h.n[1] = hr.n.y; h.n[2] = hr.n.z;
            }
            hits[ray] = h;
            ray = -1;
        }
    }
    waveReduceAdd(counters + 0, c.rays);
    waveReduceAdd(counters + 1, c.visits);
    waveReduceAdd(counters + 2, c.tris);
    waveReduceAdd(counters + 3, c.spheres);
}

// traceKernelWide with the ray queue: per lane and iteration, the current primitive group's tests
// and one node (or instance entry) of the wide traversal.
template <int STACK, bool INST>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(PT_TRACE_WAVES))) void traceKernelWideQ(DevScene S, const pt_ray* rays, int64_t n, float tmin,
                                                          float tmax, pt_hit* hits, unsigned long long* counters) {
    __shared__ uint32_t stk[STACK * kWave];
    const int lane = threadIdx.x;
    uint32_t* my = stk + lane;
    const __amdgpu_buffer_rsrc_t nodeRsrc = rawRsrc(S.wnodes);
    Counters c{0, 0, 0, 0};
    int64_t ray = -1, poolBase = 0;
    uint32_t poolLeft = 0u;
    bool more = true;
    float3 wo2 = f3(0.0f, 0.0f, 0.0f), wd = wo2, winv = wo2, o = wo2, d = wo2, inv = wo2;
    uint32_t woct = 0u, oct = 0u, inst = 0u, ng = 0u, tgBase = 0u, tg = 0u;
    float shift = 0.0f, tminI = 0.0f, closest = 0.0f, bestLo = 0.0f;
    int best = -1, sp = 0;
    bool redo = false;
    uint32_t qVisits = 0u;   // (PT_TRACE_DIAG_VISITS)
    for (;;) {
        bool took = false;
        PT_TRACE_REFILL(took);
        if (__ballot(ray >= 0) == 0) break;
        if (ray < 0) continue;
        if (took) {   // the query's start (traceKernelWide)
            const pt_ray r = rays[ray];
            const float3 wo = f3(r.o[0], r.o[1], r.o[2]);
            wd = f3(r.d[0], r.d[1], r.d[2]);
            winv = f3(rcpRN(wd.x), rcpRN(wd.y), rcpRN(wd.z));
            woct = (winv.x < 0.0f ? 1u : 0u) | (winv.y < 0.0f ? 2u : 0u) | (winv.z < 0.0f ? 4u : 0u);
            o = wo; d = wd; inv = winv;
            oct = woct;
            inst = 0u;
            const bool far = !INST && (wideFar(S, o) || (PT_WIDE_MIX && mixUnsafe(winv, S.mixLim)));
            wo2 = wo;
            shift = (INST && instFar(S, wo)) ? instEntry(S.cx, S.cy, S.cz, S.ext, wo2, wd, winv) : 0.0f;
            if (INST) o = wo2;
            tminI = tmin - shift;
            closest = tmax - shift;
            best = -1;
            sp = 0;
            redo = far;
            bestLo = -__builtin_inff();
            ng = S.nprims > 0 && !far ? (1u << oct) : 0u;
            tgBase = 0u;
            tg = 0u;
            c.rays++;
            qVisits = 0u;
        }
        while (tg) {
            const uint32_t k = tgBase + (uint32_t)__builtin_ctz(tg);
            tg &= tg - 1u;
            const float4* w = S.wprims + 3 * (size_t)k;
            const Prim q{w[0], w[1], w[2]};
            if (__float_as_uint(q.p2.w) != 0u) c.spheres++;
            else c.tris++;
            const bool lb = !INST && S.nprims > 1;
            const uint32_t kh = INST ? inst << S.gBits : 0u;
            if (S.hasSpheres) wideTest<true>(q, o, d, inv, tminI, closest, best, bestLo, lb, redo, kh);
            else wideTest<false>(q, o, d, inv, tminI, closest, best, bestLo, lb, redo, kh);
        }
        bool fin = false;
        if constexpr (INST) {   // pop; a marker returns to the world ray
            while ((ng & 0xffu) == 0u && sp > 0) {
                sp--;
                ng = my[sp * kWave];
                if (ng == kInstMarker) { o = wo2; d = wd; inv = winv; oct = woct; ng = 0u; }
            }
            if ((ng & 0xffu) == 0u) fin = true;
        } else if ((ng & 0xffu) == 0u) {
            if (sp == 0) fin = true;
            else { sp--; ng = my[sp * kWave]; }
        }
        if (!fin) {
            const uint32_t bit = (uint32_t)__builtin_ctz(ng & 0xffu);
            const uint32_t child = (ng >> 8) + (bit ^ oct);
            ng &= ~(1u << bit);
            if (ng & 0xffu) {
                if (sp >= STACK) { atomicOr(S.err, 2u); fin = true; }
                else { my[sp * kWave] = ng; sp++; }
            }
            if (!fin) {
                c.visits++;
                qVisits++;
                const uint32_t off = mul80(child);
                const uint4 n0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off, 0, 0));
                const uint4 n1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 16u, 0, 0));
                const uint4 n2 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 32u, 0, 0));
                const uint4 n3 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 48u, 0, 0));
                const uint4 n4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nodeRsrc, off + 64u, 0, 0));
                if (INST && n0.w == kInstFlag) {   // an instance: into its object space and bottom-level tree
                    if (n0.x == 0u) {
                        const float4 r0 = __builtin_bit_cast(float4, n2), r1 = __builtin_bit_cast(float4, n3),
                                     r2 = __builtin_bit_cast(float4, n4);
                        o = xformPoint(r0, r1, r2, wo2);
                        d = xformDir(r0, r1, r2, wd);
                        inv = f3(rcpRN(d.x), rcpRN(d.y), rcpRN(d.z));
                        oct = (inv.x < 0.0f ? 1u : 0u) | (inv.y < 0.0f ? 2u : 0u) | (inv.z < 0.0f ? 4u : 0u);
                    }
                    if (sp >= STACK) { atomicOr(S.err, 2u); fin = true; }
                    else {
                        my[sp * kWave] = kInstMarker;
                        sp++;
                        ng = (n1.x << 8) | (1u << oct);
                        inst = n1.y;
                        tg = 0u;
                    }
                } else {
                    const uint32_t h = INST ? wideHitsInst(n0, n1, n2, n3, n4, o, inv, oct, tminI, closest)
                                            : wideHits<PT_WIDE_MIX != 0>(n0, n1, n2, n3, n4, o, inv, oct, tminI, closest);
                    ng = (n1.x << 8) | (h >> 24);
                    tgBase = n1.y;
                    tg = h & 0xffffffu;
                }
            }
        }
        if (fin) {   // the reference-order redo and the hit record (traceKernelWide)
            if (PT_TRACE_DIAG_REDO && redo) c.spheres++;
            if (redo) {
                closest = tmax;
                const int k = traceRefStackless(S, o, d, tmin, closest);
                best = k >= 0 ? (int)S.rankOf[k] : -1;
            }
            pt_hit hr = {};
            hr.obj = -1;
            hr.mat = -1;
            if (best >= 0) {
                int obj = 0;
                HitRec x = INST ? makeHitInst(S, (uint32_t)best & kPrimMask, closest, wo2, wd, obj)
                                : makeHitFrom(S.wshade, best & (int)kPrimMask, closest, o, d);
                hr.hit = 1;
                hr.obj = x.obj;
                hr.mat = x.mat;
                hr.front_face = x.front ? 1 : 0;
                hr.t = INST ? closest + shift : closest;
                hr.p[0] = x.p.x; hr.p[1] = x.p.y; hr.p[2] = x.p.z;
                hr.n[0] = x.n.x; hr.n[1] = x.n.y; hr.n[2] = x.n.z;
            }
            if (PT_TRACE_DIAG_VISITS) hr.mat = (int)qVisits;
            hits[ray] = hr;
            ray = -1;
        }
    }
    waveReduceAdd(counters + 0, c.rays);
    waveReduceAdd(counters + 1, c.visits);
    waveReduceAdd(counters + 2, c.tris);
    waveReduceAdd(counters + 3, c.spheres);
}

// initRandom (main.cu:262-269): curand_init(seed, pixel, 0).  The subsequence skip is the
// GF(2) product of jump matrices J_k = M^(2^(67+k)) for the set bits of the pixel index.
// Loops are wave-uniform (k, j); column loads are uniform, hence scalar.
__global__ __launch_bounds__(256) void rngInitKernel(uint32_t* sd, uint32_t* s0, uint32_t* s1, uint32_t* s2,
                                                     uint32_t* s3, uint32_t* s4, const uint32_t* __restrict__ jm,
                                                     uint64_t seed, int width, int nrows, int sh, int nparts,
                                                     int part) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t npix = (int64_t)width * nrows;
    if (idx >= npix) return;
    const int lrow = (int)(idx / width), col = (int)(idx % width);
    const uint64_t pixel = (uint64_t)globalRow(lrow, sh, nparts, part) * (uint64_t)width + (uint64_t)col;
    const uint32_t a = (uint32_t)seed ^ 0xaad26b49u, b = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * a, t1 = 2591861531u * b;
    uint32_t v[5] = {123456789u + t0, 362436069u ^ t0, 521288629u + t1, 88675123u ^ t1, 5783321u + t0};
    const uint32_t d = 6615241u + t1 + t0;
    for (int k = 0; k < kJumpMats; k++) {
        if (!((pixel >> k) & 1u)) continue;
        const uint32_t* m = jm + (size_t)k * 160 * 5;
        uint32_t r[5] = {0, 0, 0, 0, 0};
        for (int j = 0; j < 160; j++) {
            const uint32_t bit = (v[j >> 5] >> (j & 31)) & 1u;
            const uint32_t mask = 0u - bit;
#pragma unroll
            for (int w = 0; w < 5; w++) r[w] ^= m[j * 5 + w] & mask;
        }
#pragma unroll
        for (int w = 0; w < 5; w++) v[w] = r[w];
    }
    sd[idx] = d; s0[idx] = v[0]; s1[idx] = v[1]; s2[idx] = v[2]; s3[idx] = v[3]; s4[idx] = v[4];
}

// --- LBVH (utils/bvh.h:17-130) -----------------------------------------------------------
__device__ __forceinline__ int deltaK(const unsigned long long* k, long long n, long long i, long long j) {   // morton_code.h:47-54
    if (i < 0 || i >= n || j < 0 || j >= n) return -1;
    return __clzll(k[i] ^ k[j]);
}

// generateLBVH (bvh.h:71-115) with the node reset separated from the linking (no race):
// writes child refs of internal node i and the parent link of both children.
__global__ void karrasKernel(const unsigned long long* __restrict__ keys, int n, float4* nodes, int* iparent,
                             int* lparent, const uint32_t* __restrict__ leafSphere, int2* irange) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    // determineRange (bvh.h:17-40)
    const int ld = deltaK(keys, n, i, i - 1), rd = deltaK(keys, n, i, i + 1);
    const int dir = (rd - ld > 0) - (rd - ld < 0);
    const int dmin = min(ld, rd);
    long long maxStride = 2;
    while (deltaK(keys, n, i, i + maxStride * dir) > dmin) maxStride *= 2;
    long long l = 0;
    for (long long s = maxStride >> 1; s >= 1; s >>= 1)
        if (deltaK(keys, n, i, i + (l + s) * dir) > dmin) l += s;
    int first = i, last = (int)(i + l * dir);
    if (dir < 0) { int t = first; first = last; last = t; }
    // findSplit (bvh.h:42-69)
    const unsigned long long fc = keys[first], lc = keys[last];
    int split;
    if (first == last) {
        split = (first + last) >> 1;
    } else {
        const int common = __clzll(fc ^ lc);
        split = first;
        int step = last - first;
        do {
            step = (step + 1) >> 1;
            const int ns = split + step;
            if (ns < last && __clzll(fc ^ keys[ns]) > common) split = ns;
        } while (step > 1);
    }
    uint32_t a, b;
    if (split == first) { a = kLeafBit | (leafSphere[split] ? kSphereBit : 0u) | (uint32_t)split; lparent[split] = i; }
    else { a = (uint32_t)split; iparent[split] = i; }
    if (split + 1 == last) { b = kLeafBit | (leafSphere[split + 1] ? kSphereBit : 0u) | (uint32_t)(split + 1); lparent[split + 1] = i; }
    else { b = (uint32_t)(split + 1); iparent[split + 1] = i; }
    nodes[4 * (size_t)i + 3] = make_float4(__uint_as_float(a), __uint_as_float(b), 0.0f, 0.0f);
    irange[i] = make_int2(first, last);   // leaf range (the device wide build's ranks)
}

// growBBox (bvh.h:117-130) as a correct bottom-up refit: every leaf writes its box into its
// parent's slot, then climbs; the second thread to reach a node unions the node's two child boxes
// into the grandparent's slot.  Tight boxes.
//
// No agent-scope synchronisation (its acq_rel fence is an L2 writeback + invalidate on this
// multi-L2 chip: the all-global version spent 3.7 ms of a 5-ms C5 build in them).  Phase 1: a
// workgroup owns the 256 leaves [base, base + 256); a node whose leaf range lies inside them
// (Karras: node i is an end of its own range, so i is in the block too) is completed in LDS with
// workgroup-scope counters.  A thread reaching a node whose range crosses a block boundary
// stores its box in that node's slot and records the arrival (events).  Phase 2: one workgroup
// replays the arrivals with workgroup-scope counters in global memory -- the crossing nodes are
// the top of the tree, about 1/16 of the nodes.
constexpr int kRefitBlock = 256, kRefitTop = 1024;
__global__ __launch_bounds__(kRefitBlock) void refitKernel(float4* nodes, const int* __restrict__ iparent,
                                                           const int* __restrict__ lparent, const int2* __restrict__ irange,
                                                           const float* __restrict__ leafBoxes, unsigned int* events, int n) {
    __shared__ float sbox[kRefitBlock][2][6];   // child boxes of the block's internal nodes
    __shared__ unsigned int scnt[kRefitBlock];
    const int base = blockIdx.x * kRefitBlock, end = min(base + kRefitBlock, n);
    scnt[threadIdx.x] = 0u;
    __syncthreads();
    const int k = base + (int)threadIdx.x;
    if (k >= n) return;
    float b[6];
    for (int i = 0; i < 6; i++) b[i] = leafBoxes[6 * (size_t)k + i];
    int p = lparent[k];
    int self = k;
    bool leaf = true;
    for (int guard = 0; p >= 0 && guard < 130; guard++) {
        const float4 refs = nodes[4 * (size_t)p + 3];
        const uint32_t lref = __float_as_uint(refs.x);
        const bool isLeft = leaf ? ((lref & kLeafBit) && (int)(lref & kPrimMask) == self)
                                 : (!(lref & kLeafBit) && (int)lref == self);
        float* f = reinterpret_cast<float*>(nodes + 4 * (size_t)p);
        for (int i = 0; i < 6; i++) f[nodeBoxIdx(isLeft ? 0 : 1, i % 3, i / 3)] = b[i];
        const int2 range = irange[p];
        if (range.x < base || range.y >= end) {   // crossing: phase 2 finishes it
            events[1 + atomicAdd(events, 1u)] = (unsigned)p;
            return;
        }
        for (int i = 0; i < 6; i++) sbox[p - base][isLeft ? 0 : 1][i] = b[i];
        const unsigned int prev = __hip_atomic_fetch_add(&scnt[p - base], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (prev == 0) return;   // sibling not done yet: it will carry on
        for (int i = 0; i < 3; i++) {   // utils::unionBox (aabb.h:55-65)
            b[i] = fminf(sbox[p - base][0][i], sbox[p - base][1][i]);
            b[3 + i] = fmaxf(sbox[p - base][0][3 + i], sbox[p - base][1][3 + i]);
        }
        self = p;
        leaf = false;
        p = iparent[p];
    }
}

__global__ __launch_bounds__(kRefitTop) void refitTopKernel(float4* nodes, const int* __restrict__ iparent,
                                                            const unsigned int* __restrict__ events, unsigned int* arrivals) {
    const unsigned int count = events[0];
    for (unsigned int e = threadIdx.x; e < count; e += kRefitTop) {
        int p = (int)events[1 + e];
        for (int guard = 0; p >= 0 && guard < 130; guard++) {
            const unsigned int prev = __hip_atomic_fetch_add(arrivals + p, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (prev == 0) break;   // the other child is not done yet
            const float* f = reinterpret_cast<const float*>(nodes + 4 * (size_t)p);
            float b[6];
            for (int i = 0; i < 3; i++) {   // utils::unionBox (aabb.h:55-65)
                b[i] = fminf(f[nodeBoxIdx(0, i, 0)], f[nodeBoxIdx(1, i, 0)]);
                b[3 + i] = fmaxf(f[nodeBoxIdx(0, i, 1)], f[nodeBoxIdx(1, i, 1)]);
            }
            const int q = iparent[p];
            if (q < 0) break;
            const uint32_t lref = __float_as_uint(nodes[4 * (size_t)q + 3].x);
            const bool isLeft = !(lref & kLeafBit) && (int)lref == p;
            float* g = reinterpret_cast<float*>(nodes + 4 * (size_t)q);
            for (int i = 0; i < 6; i++) g[nodeBoxIdx(isLeft ? 0 : 1, i % 3, i / 3)] = b[i];
            p = q;
        }
    }
}

// --- Morton keys and leaf records on the device (morton_code.h:19-75, cuda_object.h:21-42) ----
// Each expression restates the host computation (pt_host.cpp mortonKeys / the leaf loop of
// pt_scene_build_bvh) in the same operation order, so keys, boxes and normals are bit-identical.

// Object box (cuda_object.h:21-42): sphere c -/+ |r|; triangle utils::unionPoints by comparisons.
__device__ __forceinline__ void objBoxDev(const pt_object& o, float mn[3], float mx[3]) {
    if (o.type == PT_SPHERE) {
        const float r = fabsf(o.v[3]);
        for (int a = 0; a < 3; a++) { mn[a] = o.v[a] - r; mx[a] = o.v[a] + r; }
        return;
    }
    for (int a = 0; a < 3; a++) {
        mn[a] = o.v[a];
        mx[a] = o.v[a];
    }
    for (int k = 1; k < 3; k++)
        for (int a = 0; a < 3; a++) {
            const float p = o.v[3 * k + a];
            if (mn[a] > p) mn[a] = p;
            if (mx[a] < p) mx[a] = p;
        }
}

// Scene box for the Morton quantisation (main.cu:122 + aabb::unionBoxInPlace, aabb.h:36-44):
// min/max are exact and order-independent, so one workgroup reduces all boxes.  The reference
// seeds the box with aabb() = the zero box (includeOrigin), or the first object's box.  Two
// launches: per-block boxes over a grid-stride range (partial[6 * block]), then their union.
constexpr int kBoxBlocks = 512;
__global__ __launch_bounds__(1024) void sceneBoxKernel(const pt_object* __restrict__ objs, int64_t n,
                                                       int includeOrigin, float* box6, float* partial) {
    __shared__ float red[6][1024];
    float b[6];
    const bool final = partial == nullptr;   // the second launch: union of the per-block boxes in box6 + 6
    if (final || includeOrigin) {
        for (int a = 0; a < 6; a++) b[a] = final ? (a < 3 ? INFINITY : -INFINITY) : 0.0f;
        if (final && includeOrigin)
            for (int a = 0; a < 6; a++) b[a] = 0.0f;
    } else {
        objBoxDev(objs[0], b, b + 3);
    }
    if (final) {
        const float* pb = box6 + 6;
        if (!includeOrigin && threadIdx.x == 0) objBoxDev(objs[0], b, b + 3);
        for (int i = threadIdx.x; i < kBoxBlocks; i += blockDim.x)
            for (int a = 0; a < 3; a++) {
                b[a] = fminf(b[a], pb[6 * i + a]);
                b[3 + a] = fmaxf(b[3 + a], pb[6 * i + 3 + a]);
            }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
            float mn[3], mx[3];
            objBoxDev(objs[i], mn, mx);
            for (int a = 0; a < 3; a++) {
                b[a] = fminf(b[a], mn[a]);
                b[3 + a] = fmaxf(b[3 + a], mx[a]);
            }
        }
    }
    for (int a = 0; a < 6; a++) red[a][threadIdx.x] = b[a];
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int a = 0; a < 3; a++) {
                red[a][threadIdx.x] = fminf(red[a][threadIdx.x], red[a][threadIdx.x + w]);
                red[3 + a][threadIdx.x] = fmaxf(red[3 + a][threadIdx.x], red[3 + a][threadIdx.x + w]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) (final ? box6 : partial + 6 * blockIdx.x)[threadIdx.x] = red[threadIdx.x][0];
}

__device__ __forceinline__ uint32_t expandBitsDev(uint32_t v) {   // morton_code.h:19-27
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

// mortonCode3D (morton_code.h:29-45): centre normalised into the scene box (an axis whose
// range is <= 1e-7 maps to 0), x1024, clamped to [0, 1023], truncated, interleaved.
__global__ __launch_bounds__(256) void mortonKernel(const pt_object* __restrict__ objs, int64_t n,
                                                    const float* __restrict__ box6, uint32_t* codes, uint32_t* ids) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float mn[3], mx[3];
    objBoxDev(objs[i], mn, mx);
    uint32_t q[3];
    for (int a = 0; a < 3; a++) {
        const float smn = box6[a], range = box6[3 + a] - box6[a];
        const float c = (mn[a] + mx[a]) * 0.5f;
        float x = 0.0f;
        if ((double)range > 1e-7) x = (c - smn) / range;
        q[a] = (uint32_t)fminf(fmaxf(x * 1024.0f, 0.0f), 1023.0f);
    }
    codes[i] = (expandBitsDev(q[0]) << 2) + (expandBitsDev(q[1]) << 1) + expandBitsDev(q[2]);
    ids[i] = (uint32_t)i;
}

// Leaf k of the sorted order: the 64-bit key (code << 32 | objID, the MORTON64 union of
// morton_code.h), the primitive record, the triangle normal (triangle.h:17-19:
// normalize(cross(v1 - v0, v2 - v0))), the exact leaf box and the sphere flag.
__global__ __launch_bounds__(256) void leafGatherKernel(const pt_object* __restrict__ objs,
                                                        const uint32_t* __restrict__ codes,
                                                        const uint32_t* __restrict__ ids, int64_t n,
                                                        unsigned long long* keys, float4* prims, float4* shade,
                                                        float* boxes, uint32_t* sphereFlag,
                                                        const float4* __restrict__ mats) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t id = ids[k];
    const pt_object o = objs[id];
    keys[k] = ((unsigned long long)codes[k] << 32) | id;
    float mn[3], mx[3];
    objBoxDev(o, mn, mx);
    for (int a = 0; a < 3; a++) { boxes[6 * k + a] = mn[a]; boxes[6 * k + 3 + a] = mx[a]; }
    if (o.type == PT_SPHERE) {
        prims[3 * k] = make_float4(o.v[0], o.v[1], o.v[2], __uint_as_float((uint32_t)o.mat));
        prims[3 * k + 1] = make_float4(o.v[3], 0.0f, 0.0f, __uint_as_float(id));
        prims[3 * k + 2] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(1u));
        shade[3 * k] = make_float4(o.v[0], o.v[1], o.v[2], o.v[3]);
        sphereFlag[k] = 1u;
    } else {
        const float3 v0 = f3(o.v[0], o.v[1], o.v[2]), v1 = f3(o.v[3], o.v[4], o.v[5]), v2 = f3(o.v[6], o.v[7], o.v[8]);
        const float3 nn = normalize3(cross3(sub(v1, v0), sub(v2, v0)));
        prims[3 * k] = make_float4(v0.x, v0.y, v0.z, __uint_as_float((uint32_t)o.mat));
        prims[3 * k + 1] = make_float4(v1.x, v1.y, v1.z, __uint_as_float(id));
        prims[3 * k + 2] = make_float4(v2.x, v2.y, v2.z, 0.0f);
        shade[3 * k] = make_float4(nn.x, nn.y, nn.z, 0.0f);
        sphereFlag[k] = 0u;
    }
    // the object's material inline: {albedo, fuzz}, {ir, type | sphere << 16, mat, obj}
    const float4 m0 = mats[2 * o.mat], m1 = mats[2 * o.mat + 1];
    shade[3 * k + 1] = m0;
    shade[3 * k + 2] = make_float4(m1.x, __uint_as_float(__float_as_uint(m1.y) | (o.type == PT_SPHERE ? 0x10000u : 0u)),
                                   __uint_as_float((uint32_t)o.mat), __uint_as_float(id));
}

// Depth of the internal hierarchy (root = 1) = the most internal ancestors of any leaf.
__global__ __launch_bounds__(256) void depthKernel(const int* __restrict__ iparent, const int* __restrict__ lparent,
                                                   int n, int* depth) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int d = 0;
    for (int p = lparent[k]; p >= 0 && d <= n; p = iparent[p]) d++;
    atomicMax(depth, d);
}

// ------------------------------------------------------------------------ host helpers
// GF(2) 160x160 jump matrices for XORWOW's xorshift part (product-side implementation).
struct Mat160 { uint32_t c[160][5]; };

void apply160(const Mat160& m, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int j = 0; j < 160; j++) {
        const uint32_t mask = 0u - ((in[j / 32] >> (j % 32)) & 1u);
        for (int w = 0; w < 5; w++) r[w] ^= m.c[j][w] & mask;
    }
    std::memcpy(out, r, sizeof(r));
}

const std::vector<uint32_t>& jumpMatrices() {
    static const std::vector<uint32_t> tables = [] {
        Mat160 m;
        for (int j = 0; j < 160; j++) {   // image of basis vector e_j under one xorshift step
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[j / 32] = 1u << (j % 32);
            const uint32_t t = v[0] ^ (v[0] >> 2);
            const uint32_t nv[5] = {v[1], v[2], v[3], v[4], (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1))};
            std::memcpy(m.c[j], nv, sizeof(nv));
        }
        auto sq = [](const Mat160& a) {
            Mat160 r;
            for (int j = 0; j < 160; j++) apply160(a, a.c[j], r.c[j]);
            return r;
        };
        for (int i = 0; i < 67; i++) m = sq(m);
        std::vector<uint32_t> out((size_t)kJumpMats * 160 * 5);
        for (int k = 0; k < kJumpMats; k++) {
            std::memcpy(&out[(size_t)k * 800], m.c, sizeof(m.c));
            m = sq(m);
        }
        return out;
    }();
    return tables;
}

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;   // bytes allocated
    ~DevBuf() { if (p) (void)hipFree(p); }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    template <class T> T* as() const { return static_cast<T*>(p); }
    void reset() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

int devAlloc(DevBuf& b, size_t bytes) {
    b.reset();
    if (bytes == 0) bytes = 16;
    HIP_TRY(hipMalloc(&b.p, bytes));
    b.cap = bytes;
    return PT_OK;
}
// Keeps the buffer when it is large enough (no hipFree / hipMalloc, which synchronise the device:
// a per-frame BVH rebuild reuses every buffer of the previous build).
int devReserve(DevBuf& b, size_t bytes) {
    if (b.p && b.cap >= std::max<size_t>(bytes, 16)) return PT_OK;
    return devAlloc(b, bytes);
}

int envInt(const char* name, int dflt) {
    const char* v = std::getenv(name);
    if (!v || !*v) return dflt;
    int x = std::atoi(v);
    if (x < 1) return dflt;   // "0": the default
    return x > 64 ? 64 : x;
}
// A count knob: any value >= 0 (0 is zero, not the default); unset or unparsable: the default.
int envCount(const char* name, int dflt) {
    const char* v = std::getenv(name);
    if (!v || !*v) return dflt;
    char* end = nullptr;
    const long x = std::strtol(v, &end, 10);
    if (end == v || x < 0) return dflt;
    return (int)std::min<long>(x, 1L << 30);
}

// Events of a synchronous device step; on an early return (ok still false) the stream's queued
// work is waited for before the caller can free or reuse what it reads.
struct StreamGuard {
    hipStream_t st;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    bool ok = false;
    explicit StreamGuard(hipStream_t s) : st(s) {}
    ~StreamGuard() {
        if (!ok) (void)hipStreamSynchronize(st);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
    }
};

int stackFor(int depth) {
    const int need = depth + 1;
#if PT_STACK24
    for (int s : {16, 24, 32, 48, 64, 80})
#else
    for (int s : {16, 32, 48, 64, 80})
#endif
        if (need <= s) return s;
    return -1;
}

}  // namespace

// ================================================================== opaque objects
struct pt_scene {
    int device = 0;
    int64_t nobj = 0, nmat = 0;
    bool hasSpheres = false;                // any sphere ever in the scene (sticky across updates)
    std::vector<pt_object> objs;            // host copy (PT_BVH_HOST_KEYS path)
    DevBuf dobjs;                           // the objects on the device (BVH build input)
    DevBuf mats, nodes, prims, shade, counters;
    DevBuf keys, iparent, lparent, leafBoxes;   // sorted 64-bit Morton keys, parent links, leaf boxes
    // build scratch, kept between builds: codes / ids (unsorted, sorted), scene box, sphere
    // flags, refit arrival counters, depth, sort temporary
    DevBuf codes, ids, codes2, ids2, box6, sph, arr, dep, sortTemp;
    DevBuf irange;                          // leaf range [first, last] per internal node
    DevBuf refitEvents;                     // refit phase 2 input: count, then crossing-node arrivals
    DevBuf wide, wprims, wshade, rankOf;    // compressed 8-wide tree, its primitive and shading records, leaf ranks (PT_KERNEL_WIDE)
    std::unique_ptr<pt::WideDevBuilder> wideDev;   // device build scratch (PT_BVH_WIDE_DEVICE), kept between builds
    bool wideReady = false;                 // the wide tree matches the current LBVH build
    bool updated = false;                   // pt_scene_update_objects was called: a dynamic scene
    int wideSource = 0;                     // 1: host binned SAH, 2: device PLOC
    int wideDepth = 0;
    int64_t wideNodes = 0;                  // node slots
    double wideBuildMs = 0.0;               // host build + upload, wall time
    int depth = 0;
    bool built = false;
    size_t deviceBytes = 0;
    double buildMs = 0.0;                   // last pt_scene_build_bvh, device time (HIP events)
    float sceneCE[4] = {0.0f, 0.0f, 0.0f, 0.0f};   // tight scene box: centre, largest extent (DevScene)
    float mixLim = -1.0f;                          // DevScene::mixLim (-1: every ray takes the reference order)
    // instanced scenes (pt_scene_create_instanced): meshes = object ranges of `objs`, instances
    bool instanced = false;
    std::vector<int64_t> meshFirst, meshCount;
    std::vector<pt_instance> inst;
    DevBuf winst;                           // per instance: world-to-object rows, {objBase, identity}
    int gBits = 0;                          // hit key = instance << gBits | shading index
};

struct pt_film {
    int device = 0;
    int width = 0, height = 0, stripe_h = 1, nparts = 1, part = 0;
    int nrows = 0;
    int64_t npix = 0;
    uint64_t seed = 0;
    DevBuf state;   // 6 x npix uint32 (SoA)
    DevBuf jumps;   // XORWOW jump matrices (for pt_film_reset)
    DevBuf tileCost, tileOrder;   // measured per-tile cost of the last launch; LPT launch order
    DevBuf tileXY, tileXYId;      // sample mode: tileOrder decoded (tileXYKernel), and the identity order decoded
    bool haveXYId = false;
    DevBuf tileKeys, tileKeys2, tileIds, sortTemp;   // the order's radix sort on the device
    bool haveOrder = false;
    int framesSinceCost = 0;      // sample mode: frames rendered since the tile costs were last measured
    DevBuf pixAcc, taskCounter;   // sample mode: per-pixel {x, y, z, rays} accumulators; task counter
    // compat mode, wide kernel: rays per pixel of the last launch, and the next launch's critical
    // pixels (the longest chains: their ids sorted by descending rays, and a flag per pixel)
    DevBuf pixRays, pixKeys, pixKeys2, pixIds, pixSorted, critFlag, critTemp;
    int critK = 0;                // critical pixels selected for the next compat launch (0: none yet)
    DevBuf stackSpill;            // sample mode on deep trees: traversal stack entries beyond LDS
    DevBuf sums;                  // compat mode: raw per-pixel sample sums of the frame (resolve input)
    DevBuf accum;                 // progressive rendering: fp32 RGB running sums of every accumulated frame
    DevBuf staging;               // device copy of a host output frame
    int64_t accumSamples = 0;     // samples per pixel in `accum`
    int cus = 0;                  // compute units of the device (persistent grid size)
    // The last render's work counters (rays, visits, tests, paths, error word), filled by its
    // kernels, and the events around its kernels: read by pt_film_stats (or by pt_render_ex when
    // it is given a pt_stats), so a render with stats == NULL never waits for the device.
    DevBuf counters;
    unsigned long long* hostCounters = nullptr;   // pinned: the counters copied back in stream order
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;   // kernels start / end, counters copied
    bool rendered = false;
    bool lastWide = false;
    ~pt_film() {
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (ev2) (void)hipEventDestroy(ev2);
        if (hostCounters) (void)hipHostFree(hostCounters);
    }
};

namespace {
// Build the compressed 8-wide tree on the host from the device's leaf-order primitive records
// and exact leaf boxes (host/pt_wide8.cpp) and upload it.
int buildWide(pt_scene* s) {
    const int64_t n = s->nobj;
    std::vector<uint32_t> prims((size_t)n * pt::kW8PrimDwords), shade((size_t)n * 12);
    std::vector<float> boxes((size_t)n * 6);
    HIP_TRY(hipMemcpy(prims.data(), s->prims.p, prims.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(shade.data(), s->shade.p, shade.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(boxes.data(), s->leafBoxes.p, boxes.size() * 4, hipMemcpyDeviceToHost));
    // the reference's leaf order over the binary LBVH (child refs are dwords 12, 13 of a node)
    std::vector<uint32_t> refs((size_t)std::max<int64_t>(1, n - 1) * 16);
    if (n > 1) HIP_TRY(hipMemcpy(refs.data(), s->nodes.p, (size_t)(n - 1) * 64, hipMemcpyDeviceToHost));
    const std::vector<uint32_t> rank = pt::referenceRanks(refs.data() + 12, refs.data() + 13, 16, n);
    std::vector<uint32_t> wshade(shade.size());
    for (int64_t k = 0; k < n; k++) std::memcpy(&wshade[(size_t)rank[k] * 12], &shade[(size_t)k * 12], 48);
    pt::Wide8 w;
    std::string err;
    if (!pt::buildWide8(prims.data(), boxes.data(), rank.data(), n, w, err)) return fail(PT_ERR_STATE, err);
    int rc;
    if ((rc = devReserve(s->wide, w.nodes.size() * 4)) || (rc = devReserve(s->wprims, w.prims.size() * 4)) ||
        (rc = devReserve(s->wshade, wshade.size() * 4)) || (rc = devReserve(s->rankOf, rank.size() * 4)))
        return rc;
    HIP_TRY(hipMemcpy(s->wide.p, w.nodes.data(), w.nodes.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->wprims.p, w.prims.data(), w.prims.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->wshade.p, wshade.data(), wshade.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->rankOf.p, rank.data(), rank.size() * 4, hipMemcpyHostToDevice));
    s->wideDepth = w.depth;
    s->wideNodes = (int64_t)(w.nodes.size() / pt::kW8NodeDwords);
    s->wideSource = 1;
    return PT_OK;
}

// The same records built on the device from the LBVH build's leaf records (csrc/pt_wide_build.hip),
// enqueued on `st` (it synchronises with the stream once per clustering pass and wide level).
int buildWideDevice(pt_scene* s, hipStream_t st) {
    const int64_t n = s->nobj;
    int rc;
    if ((rc = devReserve(s->wide, (size_t)pt::wideDevNodeSlots(n) * pt::kW8NodeDwords * 4)) ||
        (rc = devReserve(s->wprims, (size_t)n * pt::kW8PrimDwords * 4)) || (rc = devReserve(s->wshade, (size_t)n * 48)) ||
        (rc = devReserve(s->rankOf, (size_t)n * 4)))
        return rc;
    if (!s->wideDev) s->wideDev.reset(new pt::WideDevBuilder);
    pt::WideDevIn in{s->prims.as<float4>(), s->shade.as<float4>(), s->leafBoxes.as<float>(), s->nodes.as<float4>(),
                     s->iparent.as<int>(), s->lparent.as<int>(), s->irange.as<int2>(), n};
    pt::WideDevOut out{s->wide.as<uint32_t>(), s->wprims.as<uint32_t>(), s->wshade.as<float4>(), s->rankOf.as<uint32_t>()};
    std::string err;
    const hipError_t e = s->wideDev->build(in, out, st, err);
    if (e != hipSuccess) return fail(err.empty() ? PT_ERR_HIP : PT_ERR_STATE, err.empty() ? hipGetErrorString(e) : err);
    s->wideDepth = out.depth;
    s->wideNodes = out.slots;
    s->wideSource = 2;
    return PT_OK;
}

// Instanced scenes: the two-level tree, built on the host -- one 8-wide tree per mesh (binned SAH
// over the mesh's objects in object space), a top-level 8-wide tree over the instances' world boxes
// with one instance per leaf, whose leaves become instance records (pt_wide8.hpp), all in one node
// array: the top level from slot 0, then the meshes' trees.  Shading records in object space, one
// per mesh primitive (its shading index g); the hit key instance << gBits | g.
int wideStackFor(int depth);
// A top-level leaf: an instance entering its mesh's tree at `slot` (the mesh tree's own slot
// numbering: 0 = its root; relocated with the tree).
struct InstEntry {
    uint32_t inst, mesh, slot;
};
struct InstRecCtx {
    const std::vector<std::array<float, 12>>* minv;
    const std::vector<uint8_t>* ident;   // 1: identity, 2: translation only, 0: general
    const std::vector<InstEntry>* entries;
};
uint32_t instanceOfRecord(const uint32_t* rec) { return rec[7]; }
void writeInstanceRecord(uint32_t e, uint32_t* dst, void* ctx) {
    const InstRecCtx& c = *static_cast<const InstRecCtx*>(ctx);
    const InstEntry& E = (*c.entries)[e];
    std::memset(dst, 0, pt::kW8NodeDwords * 4);
    dst[0] = (*c.ident)[E.inst] == 1 ? 1u : 0u;
    dst[1] = (*c.ident)[E.inst] == 2 ? 1u : 0u;   // translation only: the kernels move the origin, keep the direction
    dst[3] = pt::kW8InstanceFlag;
    dst[4] = E.slot;   // (+ the mesh tree's base slot once the layout is known)
    dst[5] = E.inst;
    dst[6] = E.mesh;   // (layout only; cleared with the relocation)
    std::memcpy(dst + 8, (*c.minv)[E.inst].data(), 48);
}

// Partial re-braiding (Benthin et al. 2017): an instance enters its mesh tree below the root, one
// top-level leaf per internal child of the mesh root, each with its own world box, so the top
// level separates overlapping instances at the mesh's second level.  The child boxes come from the
// root's quantised planes (outward-rounded: they contain the subtrees).  Returns the mesh root's
// internal children {slot, object-space box}; empty when the root has leaf children (then the
// instance enters at the root).
struct SubRoot {
    uint32_t slot;
    double box[6];
};
std::vector<SubRoot> nodeChildren(const pt::Wide8& w, uint32_t slot) {
    std::vector<SubRoot> out;
    if (w.nodes.size() < (size_t)(slot + 1) * pt::kW8NodeDwords) return out;
    const uint32_t* R = w.nodes.data() + (size_t)slot * pt::kW8NodeDwords;
    float p[3];
    std::memcpy(p, R, 12);
    for (int j = 0; j < 8; j++) {
        const uint32_t mb = (R[6 + (j >> 2)] >> (8 * (j & 3))) & 0xffu;
        if (mb == 0u) continue;
        if ((mb & 0xf8u) != 0x38u) return {};   // a leaf child at the root
        SubRoot sr;
        sr.slot = R[4] + (mb & 7u);
        for (int a = 0; a < 3; a++) {
            const int e = (int)((R[3] >> (8 * a)) & 0xffu) - 127;
            const uint32_t ql = (R[8 + 4 * a + (j >> 2)] >> (8 * (j & 3))) & 0xffu;
            const uint32_t qh = (R[10 + 4 * a + (j >> 2)] >> (8 * (j & 3))) & 0xffu;
            sr.box[a] = (double)p[a] + std::ldexp((double)ql, e);
            sr.box[3 + a] = (double)p[a] + std::ldexp((double)qh, e);
        }
        out.push_back(sr);
    }
    return out;
}
// The entries `levels` wide levels below the root (a node with leaf children stays an entry).
void meshSubRoots(const pt::Wide8& w, uint32_t slot, const double* box, int levels, std::vector<SubRoot>& out) {
    std::vector<SubRoot> ch = levels > 0 ? nodeChildren(w, slot) : std::vector<SubRoot>{};
    if (ch.empty()) {
        SubRoot sr;
        sr.slot = slot;
        for (int k = 0; k < 6; k++) sr.box[k] = box[k];
        out.push_back(sr);
        return;
    }
    for (const SubRoot& c : ch) meshSubRoots(w, c.slot, c.box, levels - 1, out);
}

// Partial re-braiding chosen by surface area (PT_INST_ENTRIES = k > 0): start from the root's
// internal children and repeatedly open the entry of the largest surface area (a node whose children
// are all internal) while the entries stay within k per instance -- the large, overlapping boxes are
// opened, the small ones stay closed (in the spirit of Benthin et al. 2017's SAH-driven re-braiding).
void meshSubRootsBudget(const pt::Wide8& w, size_t budget, std::vector<SubRoot>& out) {
    out = nodeChildren(w, 0u);
    if (out.empty()) return;
    auto area = [](const SubRoot& r) {
        const double x = r.box[3] - r.box[0], y = r.box[4] - r.box[1], z = r.box[5] - r.box[2];
        return x * y + y * z + z * x;
    };
    std::vector<bool> closed(out.size(), false);
    for (;;) {
        int pick = -1;
        double best = -1.0;
        for (size_t i = 0; i < out.size(); i++)
            if (!closed[i] && area(out[i]) > best) { best = area(out[i]); pick = (int)i; }
        if (pick < 0) break;
        std::vector<SubRoot> ch = nodeChildren(w, out[(size_t)pick].slot);
        if (ch.empty() || out.size() - 1 + ch.size() > budget) { closed[(size_t)pick] = true; continue; }
        out.erase(out.begin() + pick);
        closed.erase(closed.begin() + pick);
        for (const SubRoot& c : ch) { out.push_back(c); closed.push_back(false); }
    }
}

float mixLimit(double m);   // (below)

int buildInstanced(pt_scene* s) {
    const auto t0 = std::chrono::steady_clock::now();
    const int nm = (int)s->meshFirst.size();
    const int64_t ni = (int64_t)s->inst.size();
    std::vector<pt::Wide8> blas((size_t)nm);
    std::vector<uint32_t> shade;   // 12 dwords per mesh primitive
    std::vector<int64_t> meshG0((size_t)nm, 0);
    int64_t gTotal = 0;
    int maxDepthB = 0;
    std::string err;
    // each mesh's primitive records, boxes and ranks; its tree is built once the instances' reach
    // into its object space is known (below)
    std::vector<std::vector<uint32_t>> meshPrims((size_t)nm), meshRank((size_t)nm);
    std::vector<std::vector<float>> meshBoxes((size_t)nm);
    for (int m = 0; m < nm; m++) {
        const int64_t n = s->meshCount[(size_t)m], first = s->meshFirst[(size_t)m];
        meshG0[(size_t)m] = gTotal;
        std::vector<uint32_t> prims((size_t)n * pt::kW8PrimDwords, 0u), rank((size_t)n);
        std::vector<float> boxes((size_t)n * 6);
        shade.resize((size_t)(gTotal + n) * 12, 0u);
        std::vector<float4> mats((size_t)std::max<int64_t>(1, 2 * s->nmat));
        HIP_TRY(hipMemcpy(mats.data(), s->mats.p, mats.size() * sizeof(float4), hipMemcpyDeviceToHost));
        for (int64_t k = 0; k < n; k++) {
            const pt_object& o = s->objs[(size_t)(first + k)];
            uint32_t* r = &prims[(size_t)k * 12];
            float* f = reinterpret_cast<float*>(r);
            float* b = &boxes[(size_t)k * 6];
            uint32_t* sh = &shade[(size_t)(gTotal + k) * 12];
            float* shf = reinterpret_cast<float*>(sh);
            r[3] = (uint32_t)o.mat;
            r[7] = (uint32_t)k;   // the object within its mesh
            if (o.type == PT_SPHERE) {
                f[0] = o.v[0]; f[1] = o.v[1]; f[2] = o.v[2]; f[4] = o.v[3]; r[11] = 1u;
                const float rr = std::fabs(o.v[3]);
                for (int a = 0; a < 3; a++) { b[a] = o.v[a] - rr; b[3 + a] = o.v[a] + rr; }
                shf[0] = o.v[0]; shf[1] = o.v[1]; shf[2] = o.v[2]; shf[3] = o.v[3];
            } else {
                for (int v = 0; v < 3; v++)
                    for (int a = 0; a < 3; a++) f[4 * v + a] = o.v[3 * v + a];
                for (int a = 0; a < 3; a++) {
                    b[a] = std::fmin(std::fmin(o.v[a], o.v[3 + a]), o.v[6 + a]);
                    b[3 + a] = std::fmax(std::fmax(o.v[a], o.v[3 + a]), o.v[6 + a]);
                }
                // triangle.h:17-19 normalize(cross(v1 - v0, v2 - v0)), the device's operation order
                const float e1[3] = {o.v[3] - o.v[0], o.v[4] - o.v[1], o.v[5] - o.v[2]};
                const float e2[3] = {o.v[6] - o.v[0], o.v[7] - o.v[1], o.v[8] - o.v[2]};
                const float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
                const float l = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
                if (l != 0.0f) {
                    const float il = 1.0f / l;
                    for (int a = 0; a < 3; a++) shf[a] = il * c[a];
                }
            }
            const float4 m0 = mats[(size_t)(2 * o.mat)], m1 = mats[(size_t)(2 * o.mat + 1)];
            shf[4] = m0.x; shf[5] = m0.y; shf[6] = m0.z; shf[7] = m0.w;
            uint32_t tp;
            std::memcpy(&tp, &m1.y, 4);
            shf[8] = m1.x;
            sh[9] = tp | (o.type == PT_SPHERE ? 0x10000u : 0u);
            sh[10] = (uint32_t)o.mat;
            sh[11] = (uint32_t)k;
            rank[(size_t)k] = (uint32_t)(gTotal + k);
        }
        meshPrims[(size_t)m] = std::move(prims);
        meshBoxes[(size_t)m] = std::move(boxes);
        meshRank[(size_t)m] = std::move(rank);
        gTotal += n;
    }
    int gBits = 1;
    while (((int64_t)1 << gBits) < gTotal) gBits++;
    if (gBits > 28 || ni > ((int64_t)1 << (30 - gBits)))
        return fail(PT_ERR_INVALID, "instanced scene: too many instances for the hit key (instance << " +
                                        std::to_string(gBits) + " | primitive)");
    // instances: world-to-object transforms, world boxes (every mesh vertex transformed, in double)
    std::vector<std::array<float, 12>> minv((size_t)ni);
    std::vector<uint8_t> ident((size_t)ni, 0);
    std::vector<std::array<double, 6>> ibox((size_t)ni);   // world box of each instance
    std::vector<uint32_t> used;
    std::vector<float> winst((size_t)std::max<int64_t>(1, ni) * 16, 0.0f);
    std::vector<std::array<double, 12>> w2o((size_t)ni);   // world-to-object, double
    double wmn[3] = {INFINITY, INFINITY, INFINITY}, wmx[3] = {-INFINITY, -INFINITY, -INFINITY};   // the world box
    uint32_t objBase = 0;
    for (int64_t i = 0; i < ni; i++) {
        const pt_instance& I = s->inst[(size_t)i];
        const double a[3][3] = {{I.m[0], I.m[1], I.m[2]}, {I.m[4], I.m[5], I.m[6]}, {I.m[8], I.m[9], I.m[10]}};
        const double t[3] = {I.m[3], I.m[7], I.m[11]};
        const double det = a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) - a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
                           a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
        if (!(std::fabs(det) > 1e-30) || !std::isfinite(det))
            return fail(PT_ERR_INVALID, "instanced scene: instance " + std::to_string(i) + " has a singular transform");
        double inv[3][3];
        inv[0][0] = (a[1][1] * a[2][2] - a[1][2] * a[2][1]) / det;
        inv[0][1] = (a[0][2] * a[2][1] - a[0][1] * a[2][2]) / det;
        inv[0][2] = (a[0][1] * a[1][2] - a[0][2] * a[1][1]) / det;
        inv[1][0] = (a[1][2] * a[2][0] - a[1][0] * a[2][2]) / det;
        inv[1][1] = (a[0][0] * a[2][2] - a[0][2] * a[2][0]) / det;
        inv[1][2] = (a[0][2] * a[1][0] - a[0][0] * a[1][2]) / det;
        inv[2][0] = (a[1][0] * a[2][1] - a[1][1] * a[2][0]) / det;
        inv[2][1] = (a[0][1] * a[2][0] - a[0][0] * a[2][1]) / det;
        inv[2][2] = (a[0][0] * a[1][1] - a[0][1] * a[1][0]) / det;
        bool id = true, lin = true;
        for (int r = 0; r < 3; r++) {
            const double it = -(inv[r][0] * t[0] + inv[r][1] * t[1] + inv[r][2] * t[2]);
            for (int c = 0; c < 3; c++) {
                minv[(size_t)i][(size_t)(4 * r + c)] = (float)inv[r][c];
                lin = lin && a[r][c] == (r == c ? 1.0 : 0.0);
            }
            minv[(size_t)i][(size_t)(4 * r + 3)] = (float)it;
            for (int c = 0; c < 3; c++) w2o[(size_t)i][(size_t)(4 * r + c)] = inv[r][c];
            w2o[(size_t)i][(size_t)(4 * r + 3)] = it;
            id = id && t[r] == 0.0;
        }
        id = id && lin;
        ident[(size_t)i] = id ? 1 : (lin ? 2 : 0);
        for (int k = 0; k < 12; k++) winst[(size_t)i * 16 + (size_t)k] = minv[(size_t)i][(size_t)k];
        uint32_t ob = objBase, idf = id ? 1u : lin ? 2u : 0u;   // identity | translation only
        std::memcpy(&winst[(size_t)i * 16 + 12], &ob, 4);
        std::memcpy(&winst[(size_t)i * 16 + 13], &idf, 4);
        objBase += (uint32_t)s->meshCount[(size_t)I.mesh];
        // world box of the instance
        const int64_t first = s->meshFirst[(size_t)I.mesh], n = s->meshCount[(size_t)I.mesh];
        if (n == 0) continue;
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        auto grow = [&](double x, double y, double z) {
            const double p[3] = {x, y, z};
            for (int r = 0; r < 3; r++) {
                const double w = a[r][0] * p[0] + a[r][1] * p[1] + a[r][2] * p[2] + t[r];
                mn[r] = std::min(mn[r], w);
                mx[r] = std::max(mx[r], w);
            }
        };
        for (int64_t k = 0; k < n; k++) {
            const pt_object& o = s->objs[(size_t)(first + k)];
            if (o.type == PT_SPHERE) {
                const double rr = std::fabs((double)o.v[3]);
                for (int c = 0; c < 8; c++)
                    grow(o.v[0] + ((c & 1) ? rr : -rr), o.v[1] + ((c & 2) ? rr : -rr), o.v[2] + ((c & 4) ? rr : -rr));
            } else {
                for (int v = 0; v < 3; v++) grow(o.v[3 * v], o.v[3 * v + 1], o.v[3 * v + 2]);
            }
        }
        for (int r = 0; r < 3; r++) { wmn[r] = std::min(wmn[r], mn[r]); wmx[r] = std::max(wmx[r], mx[r]); }
        for (int r = 0; r < 3; r++) {
            ibox[(size_t)i][(size_t)r] = mn[r];
            ibox[(size_t)i][(size_t)(3 + r)] = mx[r];
        }
        used.push_back((uint32_t)i);
    }
    if (used.empty()) return fail(PT_ERR_STATE, "instanced scene: no instance of a non-empty mesh");
    // The world box (its centre and largest extent: instFar's region, camFar), and the reach of
    // world ray origins into each mesh's object space.  Origins within kInstFarExt world extents of
    // the centre (farther camera rays are moved up to the world box first, renderKernelWF<.., INST>)
    // map into object space within `reach` of the origin; the mesh tree's plane quantum is taken
    // against that reach, not the mesh's own size, so its outward margin (wideHits) holds for
    // every ray that enters it.
    double wext = 0.0, wm = 0.0;
    for (int a = 0; a < 3; a++) {
        s->sceneCE[a] = (float)(0.5 * (wmn[a] + wmx[a]));
        wext = std::max(wext, wmx[a] - wmn[a]);
        wm = std::max({wm, std::fabs(wmn[a]), std::fabs(wmx[a]), wmx[a] - wmn[a]});
    }
    s->sceneCE[3] = std::nextafter((float)wext, INFINITY);
    s->mixLim = mixLimit(wm);
    std::vector<double> reach((size_t)nm, 0.0);
    for (int64_t i = 0; i < ni; i++) {
        const std::array<double, 12>& W = w2o[(size_t)i];
        double r = 0.0;
        for (int c = 0; c < 8; c++) {   // corners of the cube of half-size kInstFarExt world extents (+ 1 %)
            const double h = 1.01 * kInstFarExt * wext;
            const double p[3] = {0.5 * (wmn[0] + wmx[0]) + ((c & 1) ? h : -h), 0.5 * (wmn[1] + wmx[1]) + ((c & 2) ? h : -h),
                                 0.5 * (wmn[2] + wmx[2]) + ((c & 4) ? h : -h)};
            for (int a = 0; a < 3; a++)
                r = std::max(r, std::fabs(W[(size_t)(4 * a)] * p[0] + W[(size_t)(4 * a + 1)] * p[1] +
                                          W[(size_t)(4 * a + 2)] * p[2] + W[(size_t)(4 * a + 3)]));
        }
        const int m = s->inst[(size_t)i].mesh;
        reach[(size_t)m] = std::max(reach[(size_t)m], r);
    }
    for (int m = 0; m < nm; m++) {
        const int64_t n = s->meshCount[(size_t)m];
        if (n > 0 && !pt::buildWide8(meshPrims[(size_t)m].data(), meshBoxes[(size_t)m].data(), meshRank[(size_t)m].data(),
                                     n, blas[(size_t)m], err, reach[(size_t)m]))
            return fail(PT_ERR_STATE, err);
        maxDepthB = std::max(maxDepthB, blas[(size_t)m].depth);
    }
    // top-level leaves: per instance, its mesh root's internal children (re-braided; PT_INST_REBRAID=0:
    // the mesh root), each with the world box of its object-space box (8 corners in double)
    const char* rbv = std::getenv("PT_INST_REBRAID");
    const int rebraid = rbv ? std::max(0, std::min(3, std::atoi(rbv))) : 1;
    std::vector<std::vector<SubRoot>> sub((size_t)nm);
    for (int m = 0; m < nm; m++) {
        const double inf[6] = {-INFINITY, -INFINITY, -INFINITY, INFINITY, INFINITY, INFINITY};
        const int budget = envCount("PT_INST_ENTRIES", 0);   // (A/B: surface-area-chosen partial re-braiding)
        if (budget > 0) meshSubRootsBudget(blas[(size_t)m], (size_t)budget, sub[(size_t)m]);
        else if (rebraid > 0) meshSubRoots(blas[(size_t)m], 0u, inf, rebraid, sub[(size_t)m]);
        if (sub[(size_t)m].size() == 1) sub[(size_t)m].clear();   // (the root itself)
    }
    std::vector<InstEntry> entries;
    std::vector<uint32_t> iprims;
    std::vector<float> iboxes;
    auto addEntry = [&](uint32_t i, uint32_t mesh, uint32_t slot, const double* b) {
        iprims.resize(iprims.size() + pt::kW8PrimDwords, 0u);
        iprims[iprims.size() - pt::kW8PrimDwords + 7] = (uint32_t)entries.size();
        for (int r = 0; r < 3; r++) iboxes.push_back(std::nextafter((float)b[r], -INFINITY));
        for (int r = 0; r < 3; r++) iboxes.push_back(std::nextafter((float)b[3 + r], INFINITY));
        entries.push_back({i, mesh, slot});
    };
    for (uint32_t i : used) {
        const pt_instance& I = s->inst[(size_t)i];
        const std::vector<SubRoot>& sr = sub[(size_t)I.mesh];
        if (sr.empty()) {
            addEntry(i, (uint32_t)I.mesh, 0u, ibox[(size_t)i].data());
            continue;
        }
        for (const SubRoot& r : sr) {
            double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int c = 0; c < 8; c++) {
                const double q[3] = {r.box[(c & 1) ? 3 : 0], r.box[(c & 2) ? 4 : 1], r.box[(c & 4) ? 5 : 2]};
                for (int a = 0; a < 3; a++) {
                    const double w = (double)I.m[4 * a] * q[0] + (double)I.m[4 * a + 1] * q[1] + (double)I.m[4 * a + 2] * q[2] +
                                     (double)I.m[4 * a + 3];
                    mn[a] = std::min(mn[a], w);
                    mx[a] = std::max(mx[a], w);
                }
            }
            // (never beyond the instance's exact box)
            double b[6];
            for (int a = 0; a < 3; a++) {
                b[a] = std::max(mn[a], ibox[(size_t)i][(size_t)a]);
                b[3 + a] = std::min(mx[a], ibox[(size_t)i][(size_t)(3 + a)]);
            }
            addEntry(i, (uint32_t)I.mesh, r.slot, b);
        }
    }
    pt::Wide8 top;
    if (!pt::buildWide8Leaf(iprims.data(), iboxes.data(), nullptr, (int64_t)entries.size(), 1, top, err))
        return fail(PT_ERR_STATE, err);
    InstRecCtx ctx{&minv, &ident, &entries};
    if (!pt::instanceLeaves(top, instanceOfRecord, writeInstanceRecord, &ctx, err)) return fail(PT_ERR_STATE, err);
    // layout: the top level from slot 0, then each mesh's tree (child and primitive bases relocated)
    const uint32_t topSlots = (uint32_t)(top.nodes.size() / pt::kW8NodeDwords);
    std::vector<uint32_t> meshRoot((size_t)nm, 0u);
    uint32_t nodeBase = topSlots, primBase = 0;
    for (int m = 0; m < nm; m++) {
        meshRoot[(size_t)m] = nodeBase;
        pt::relocateWide8(blas[(size_t)m], nodeBase, primBase);
        nodeBase += (uint32_t)(blas[(size_t)m].nodes.size() / pt::kW8NodeDwords);
        primBase += (uint32_t)(blas[(size_t)m].prims.size() / pt::kW8PrimDwords);
    }
    if ((int64_t)nodeBase >= ((int64_t)1 << 24)) return fail(PT_ERR_STATE, "instanced BVH: more than 2^24 node slots");
    for (size_t k = 0; k < top.nodes.size(); k += pt::kW8NodeDwords)
        if (top.nodes[k + 3] == pt::kW8InstanceFlag) {
            top.nodes[k + 4] += meshRoot[top.nodes[k + 6]];
            top.nodes[k + 6] = 0u;
        }
    std::vector<uint32_t> nodes = top.nodes, prims;
    for (int m = 0; m < nm; m++) {
        nodes.insert(nodes.end(), blas[(size_t)m].nodes.begin(), blas[(size_t)m].nodes.end());
        prims.insert(prims.end(), blas[(size_t)m].prims.begin(), blas[(size_t)m].prims.end());
    }
    if (prims.empty()) prims.assign(pt::kW8PrimDwords, 0u);
    if (shade.empty()) shade.assign(12, 0u);
    int rc;
    if ((rc = devReserve(s->wide, nodes.size() * 4)) || (rc = devReserve(s->wprims, prims.size() * 4)) ||
        (rc = devReserve(s->wshade, shade.size() * 4)) || (rc = devReserve(s->winst, winst.size() * 4)))
        return rc;
    HIP_TRY(hipMemcpy(s->wide.p, nodes.data(), nodes.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->wprims.p, prims.data(), prims.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->wshade.p, shade.data(), shade.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->winst.p, winst.data(), winst.size() * 4, hipMemcpyHostToDevice));
    s->gBits = gBits;
    s->wideDepth = top.depth + 1 + maxDepthB + 1;   // stack: top levels, the marker, the mesh's levels
    s->wideNodes = (int64_t)(nodes.size() / pt::kW8NodeDwords);
    s->wideSource = 3;
    s->wideReady = true;
    s->deviceBytes = nodes.size() * 4 + prims.size() * 4 + shade.size() * 4 + winst.size() * 4 + (size_t)s->nmat * 32;
    s->wideBuildMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    s->buildMs = s->wideBuildMs;
    s->depth = 0;
    if (wideStackFor(s->wideDepth) < 0) return fail(PT_ERR_STATE, "instanced BVH too deep");
    s->built = true;
    return PT_OK;
}

// Traversal stack entries of the wide kernels (one dword per entry): >= the tree depth.
int wideStackFor(int depth) {
    for (int st : {8, 16, 24})
        if (depth <= st) return st;
    return -1;
}

int setDevice(int dev) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(PT_ERR_NODEVICE, "no HIP device visible (the library has no CPU fallback)");
    if (dev < 0 || dev >= count) return fail(PT_ERR_INVALID, "device index out of range");
    HIP_TRY(hipSetDevice(dev));
    return PT_OK;
}

template <int S>
void launchRenderWide(const RenderParams& P, hipStream_t st) {
    if (P.S.winst) {   // an instanced scene's two-level tree
        if (P.pixAcc) renderKernelWF<S, true, true, true><<<P.nwaves, kWave, 0, st>>>(P);
        else renderKernelWF<S, false, true, true><<<PT_COMPAT_QUEUE ? P.nwaves : P.compatGrid, kWave, 0, st>>>(P);
        return;
    }
    if (P.pixAcc) renderKernelWF<S, true, true><<<P.nwaves, kWave, 0, st>>>(P);
    else pt::launchCompatWide(S, &P, st);   // (its own translation unit, pt_compat.hip)
}
template <int S>
void launchRender(const RenderParams& P, hipStream_t st) {
    if (P.kernel == PT_KERNEL_WAVEFRONT && P.pixAcc)
        renderKernelWF<S, true, false><<<P.nwaves, kWave, 0, st>>>(P);
    else if (P.kernel == PT_KERNEL_WAVEFRONT)
        renderKernelWF<S, false, false><<<PT_COMPAT_QUEUE ? P.nwaves : P.compatGrid, kWave, 0, st>>>(P);
    else if (P.pixAcc) renderKernel<S, true><<<P.ntiles, kWave, 0, st>>>(P);
    else renderKernel<S, false><<<P.ntiles, kWave, 0, st>>>(P);
}
template <int S, bool WIDE, bool INST = false, bool SAMPLE = true>
int wavesPerCU(int& n) {
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&renderKernelWF<S, SAMPLE, WIDE, INST>),
                                                         kWave, 0));
    return PT_OK;
}
// Persistent waves per CU of the render kernel a launch runs (sample mode, or compat mode with the
// pixel queue): its occupancy.  The compat wide kernels live in pt_compat.hip's translation unit.
int persistentWavesPerCU(int stack, int kernel, int& n, bool inst, bool sample) {
    if (kernel == PT_KERNEL_WIDE && inst) {
        switch (stack) {
            case 8: return sample ? wavesPerCU<8, true, true>(n) : wavesPerCU<8, true, true, false>(n);
            case 16: return sample ? wavesPerCU<16, true, true>(n) : wavesPerCU<16, true, true, false>(n);
            case 24: return sample ? wavesPerCU<24, true, true>(n) : wavesPerCU<24, true, true, false>(n);
            default: return fail(PT_ERR_STATE, "unsupported instanced BVH depth");
        }
    }
    if (kernel == PT_KERNEL_WIDE) {
        if (!sample) return pt::compatWideWavesPerCU(stack, n) ? fail(PT_ERR_STATE, "unsupported wide BVH depth") : PT_OK;
        switch (stack) {
            case 8: return wavesPerCU<8, true>(n);
            case 16: return wavesPerCU<16, true>(n);
            case 24: return wavesPerCU<24, true>(n);
            default: return fail(PT_ERR_STATE, "unsupported wide BVH depth");
        }
    }
    switch (stack) {
        case 16: return sample ? wavesPerCU<16, false>(n) : wavesPerCU<16, false, false, false>(n);
#if PT_STACK24
        case 24: return sample ? wavesPerCU<24, false>(n) : wavesPerCU<24, false, false, false>(n);
#endif
        case 32: return sample ? wavesPerCU<32, false>(n) : wavesPerCU<32, false, false, false>(n);
        case 48: return sample ? wavesPerCU<48, false>(n) : wavesPerCU<48, false, false, false>(n);
        case 64: return sample ? wavesPerCU<64, false>(n) : wavesPerCU<64, false, false, false>(n);
        case 80: return sample ? wavesPerCU<80, false>(n) : wavesPerCU<80, false, false, false>(n);
        default: return fail(PT_ERR_STATE, "unsupported BVH depth");
    }
}
int dispatchRender(int stack, const RenderParams& P, hipStream_t st) {
    if (P.kernel == PT_KERNEL_WIDE) {
        switch (stack) {
            case 8: launchRenderWide<8>(P, st); break;
            case 16: launchRenderWide<16>(P, st); break;
            case 24: launchRenderWide<24>(P, st); break;
            default: return fail(PT_ERR_STATE, "unsupported wide BVH depth");
        }
        HIP_TRY(hipGetLastError());
        return PT_OK;
    }
    switch (stack) {
        case 16: launchRender<16>(P, st); break;
#if PT_STACK24
        case 24: launchRender<24>(P, st); break;
#endif
        case 32: launchRender<32>(P, st); break;
        case 48: launchRender<48>(P, st); break;
        case 64: launchRender<64>(P, st); break;
        case 80: launchRender<80>(P, st); break;
        default: return fail(PT_ERR_STATE, "unsupported BVH depth");
    }
    HIP_TRY(hipGetLastError());
    return PT_OK;
}
int dispatchTrace(int stack, bool wide, const DevScene& S, const pt_ray* r, int64_t n, float tmin, float tmax,
                  pt_hit* h, unsigned long long* cnt, hipStream_t st) {
    // a grid of at most 32 one-wave blocks per CU, striding over the batch
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + kWave - 1) / kWave, (int64_t)cus * 32);
    const char* strideEnv = std::getenv("PT_TRACE_STRIDE");   // 1: the grid-stride kernels (A/B)
    if (!(strideEnv && std::atoi(strideEnv) != 0)) {   // default: the queued kernels
        if (wide) {
            switch (stack) {
                case 8: S.winst ? traceKernelWideQ<8, true><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt)
                                : traceKernelWideQ<8, false><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
                case 16: S.winst ? traceKernelWideQ<16, true><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt)
                                 : traceKernelWideQ<16, false><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
                case 24: S.winst ? traceKernelWideQ<24, true><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt)
                                 : traceKernelWideQ<24, false><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
                default: return fail(PT_ERR_STATE, "unsupported wide BVH depth");
            }
        } else {
            switch (stack) {
                case 16: traceKernelQ<16><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
#if PT_STACK24
                case 24: traceKernelQ<24><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
#endif
                case 32: traceKernelQ<32><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
                case 48: traceKernelQ<48><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
                case 64: traceKernelQ<64><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
                case 80: traceKernelQ<80><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
                default: return fail(PT_ERR_STATE, "unsupported BVH depth");
            }
        }
        HIP_TRY(hipGetLastError());
        return PT_OK;
    }
    if (wide && S.winst) {
        switch (stack) {
            case 8: traceKernelWide<8, true><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
            case 16: traceKernelWide<16, true><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
            case 24: traceKernelWide<24, true><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
            default: return fail(PT_ERR_STATE, "unsupported instanced BVH depth");
        }
        HIP_TRY(hipGetLastError());
        return PT_OK;
    }
    if (wide) {
        switch (stack) {
            case 8: traceKernelWide<8, false><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
            case 16: traceKernelWide<16, false><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
            case 24: traceKernelWide<24, false><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
            default: return fail(PT_ERR_STATE, "unsupported wide BVH depth");
        }
        HIP_TRY(hipGetLastError());
        return PT_OK;
    }
    switch (stack) {
        case 16: traceKernel<16><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
#if PT_STACK24
        case 24: traceKernel<24><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
#endif
        case 32: traceKernel<32><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
        case 48: traceKernel<48><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
        case 64: traceKernel<64><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
        case 80: traceKernel<80><<<blocks, kWave, 0, st>>>(S, r, n, tmin, tmax, h, cnt); break;
        default: return fail(PT_ERR_STATE, "unsupported BVH depth");
    }
    HIP_TRY(hipGetLastError());
    return PT_OK;
}

// (Re)initialise every stream of the film to curand_init(seed, pixel, 0), asynchronously.
int filmInit(pt_film* f, hipStream_t st) {
    if (f->npix <= 0) return PT_OK;
    uint32_t* b = f->state.as<uint32_t>();
    const int64_t np = f->npix;
    rngInitKernel<<<(unsigned)((np + 255) / 256), 256, 0, st>>>(b, b + np, b + 2 * np, b + 3 * np, b + 4 * np, b + 5 * np,
                                                                 f->jumps.as<uint32_t>(), f->seed, f->width, f->nrows,
                                                                 f->stripe_h, f->nparts, f->part);
    HIP_TRY(hipGetLastError());
    return PT_OK;
}

// DevScene::mixLim for a scene whose coordinates and extent are at most m.  Both wide builders
// (host/pt_wide8.cpp, csrc/pt_wide_build.hip) give a node the plane quantum s = 2^e with e the
// larger of ceil(log2(m)) - 18 and ceil(log2(node extent / 251)), so s <= 2^eS with
// eS = ceil(log2(m)) + 1; then |s * 2^24 * inv| < 2^128 (finite) for |inv| <= 2^(103 - eS), and the
// exponent byte + 24 stays below 255 for eS <= 100.  Beyond that, every ray takes the reference order.
float mixLimit(double m) {
    if (!(m > 0.0) || !std::isfinite(m)) return m == 0.0 ? FLT_MAX : -1.0f;
    int ex = 0;
    const double f = std::frexp(m, &ex);   // m = f * 2^ex, f in [0.5, 1): ceil(log2(m)) = ex, or ex - 1 at f = 0.5
    const int eS = (f == 0.5 ? ex - 1 : ex) + 1;
    if (eS > 100) return -1.0f;
    if (103 - eS >= 127) return FLT_MAX;
    return std::ldexp(1.0f, 103 - eS);
}

DevScene devScene(const pt_scene* s) {
    DevScene S;
    S.nodes = s->nodes.as<float4>();
    S.prims = s->prims.as<float4>();
    S.shade = s->shade.as<float4>();
    S.mats = s->mats.as<float4>();
    S.wnodes = s->wide.as<float4>();
    S.wprims = s->wprims.as<float4>();
    S.wshade = s->wshade.as<float4>();
    S.rankOf = s->rankOf.as<uint32_t>();
    S.iparent = s->iparent.as<int>();
    S.err = reinterpret_cast<unsigned int*>(s->counters.as<unsigned long long>() + 7);
    S.nprims = (int)s->nobj;
    S.hasSpheres = s->hasSpheres ? 1 : 0;
    S.cx = s->sceneCE[0]; S.cy = s->sceneCE[1]; S.cz = s->sceneCE[2]; S.ext = s->sceneCE[3];
    S.mixLim = s->mixLim;
    S.winst = s->instanced ? s->winst.as<float4>() : nullptr;
    S.gBits = s->gBits;
    return S;
}

// Algorithmic bytes: per binary node visit both child boxes + refs (56 B), per
// wide node visit the 80-B compressed record (8 child boxes, refs, frame); 40 B per triangle
// test, 20 B per sphere test.
void fillStats(pt_stats* st, const unsigned long long c[5], double ms, bool wide = false) {
    if (!st) return;
    std::memset(st, 0, sizeof(*st));
    st->rays = c[0];
    st->node_visits = c[1];
    st->box_tests = (wide ? 8 : 2) * c[1];
    st->tri_tests = c[2];
    st->sphere_tests = c[3];
    st->paths = c[4];
    st->kernel_ms = ms;
    st->algo_bytes = (wide ? 80ull : 56ull) * c[1] + 40ull * c[2] + 20ull * c[3];
}

// Diagnostics of the wavefront scheduler (PT_ITER_STATS=1; the per-step counters need a PT_DIAG build).
void printIterStats(const unsigned long long* c, bool wide) {
    if (c[8] + c[9] + c[10] > 0)
        std::fprintf(stderr, "[pt] iterations node %llu leaf %llu shade %llu | lanes/iter node %.1f leaf %.1f "
                     "shade %.1f\n", c[8], c[9], c[10], (double)c[1] / std::max(1ull, c[8]),
                     (double)c[11] / std::max(1ull, c[9]), (double)c[0] / std::max(1ull, c[10]));
    if (c[12] + c[13] + c[14] > 0)
        std::fprintf(stderr, "[pt] cycles/iteration node %.0f leaf %.0f shade %.0f | share node %.3f leaf %.3f "
                     "shade %.3f\n", (double)c[12] / std::max(1ull, c[8]), (double)c[13] / std::max(1ull, c[9]),
                     (double)c[14] / std::max(1ull, c[10]), (double)c[12] / (double)(c[12] + c[13] + c[14]),
                     (double)c[13] / (double)(c[12] + c[13] + c[14]), (double)c[14] / (double)(c[12] + c[13] + c[14]));
    if (wide && c[8] > 0)
        std::fprintf(stderr, "[pt] wide queries repeated in the reference order: %llu (lanes x steps); NODE steps: "
                     "lanes waiting on primitives with nodes left %.1f, lanes without NODE work %.1f\n", c[20],
                     (double)c[21] / std::max(1ull, c[8]), (double)c[22] / std::max(1ull, c[8]));
    if (wide && c[9] > 0)
        std::fprintf(stderr, "[pt] LEAF: primitive tests whose exact box misses at test time %llu of %llu (%.3f); "
                     "lanes testing one primitive per step %.1f\n", c[23], c[3] + c[2], (double)c[23] / std::max(1ull, c[2] + c[3]),
                     (double)c[25] / std::max(1ull, c[9]));
    if (wide && c[9] > 0)
        std::fprintf(stderr, "[pt] LEAF: exact box misses even with tmax = inf %llu (%.3f of tests); tests in groups that "
                     "were parked %llu (%.3f), their misses %llu\n", c[26], (double)c[26] / std::max(1ull, c[2] + c[3]),
                     c[27], (double)c[27] / std::max(1ull, c[2] + c[3]), c[28]);
    if (c[15] > 0)
        std::fprintf(stderr, "[pt] loop head (choice of the step kind) cycles/iteration %.0f\n",
                     (double)c[15] / std::max(1ull, c[8] + c[9] + c[10]));
    if (c[14] > 0)
        std::fprintf(stderr, "[pt] SHADE cycles/iteration: shading %.0f tasks %.0f new-path %.0f ray-start %.0f\n",
                     (double)c[16] / std::max(1ull, c[10]), (double)c[17] / std::max(1ull, c[10]),
                     (double)c[18] / std::max(1ull, c[10]), (double)c[19] / std::max(1ull, c[10]));
}

// The film's last render -> pt_stats: waits for its counters (copied to pinned memory in stream
// order, event ev2) and takes the kernels' time from its events; reports a tripped traversal guard.
int filmStats(pt_film* f, pt_stats* stats) {
    if (!f->rendered) return fail(PT_ERR_STATE, "pt_film_stats: no render on this film yet");
    HIP_TRY(hipEventSynchronize(f->ev2));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, f->ev0, f->ev1));
    const unsigned long long* c = f->hostCounters;
    fillStats(stats, c, ms, f->lastWide);
    if (std::getenv("PT_ITER_STATS")) printIterStats(c, f->lastWide);
    if (c[7]) return fail(PT_ERR_STATE, "traversal guard tripped (corrupt BVH), flags " + std::to_string(c[7]));
    return PT_OK;
}
}  // namespace

// ================================================================== C ABI (device part)
extern "C" {

int pt_device_count(int* count) {
    if (!count) return fail(PT_ERR_INVALID, "pt_device_count: null");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return PT_OK;
}

int pt_scene_create(int device, const pt_object* objs, int64_t n, const pt_material* mats, int64_t nmat,
                    pt_scene** out) {
    if (!out || n < 0 || nmat < 0 || (n > 0 && !objs) || (nmat > 0 && !mats))
        return fail(PT_ERR_INVALID, "pt_scene_create: bad argument");
    if (n >= ((int64_t)1 << 26)) return fail(PT_ERR_INVALID, "pt_scene_create: more than 2^26 objects");
    for (int64_t i = 0; i < n; i++) {
        if (objs[i].type != PT_SPHERE && objs[i].type != PT_TRIANGLE)
            return fail(PT_ERR_INVALID, "pt_scene_create: unknown object type");
        if (objs[i].mat < 0 || objs[i].mat >= nmat) return fail(PT_ERR_INVALID, "pt_scene_create: material id out of range");
    }
    int rc = setDevice(device);
    if (rc) return rc;
    std::unique_ptr<pt_scene> s(new pt_scene);
    s->device = device;
    s->nobj = n;
    s->nmat = nmat;
    s->objs.assign(objs, objs + n);
    for (int64_t i = 0; i < n && !s->hasSpheres; i++) s->hasSpheres = objs[i].type == PT_SPHERE;
    // materials: (albedo.xyz, fuzz), (ir, type, 0, 0)
    std::vector<float4> m((size_t)std::max<int64_t>(1, 2 * nmat));
    for (int64_t i = 0; i < nmat; i++) {
        m[2 * i] = make_float4(mats[i].albedo[0], mats[i].albedo[1], mats[i].albedo[2], mats[i].fuzz);
        uint32_t t = (uint32_t)mats[i].type;
        float tf;
        std::memcpy(&tf, &t, 4);
        m[2 * i + 1] = make_float4(mats[i].ir, tf, 0.0f, 0.0f);
    }
    if ((rc = devAlloc(s->mats, m.size() * sizeof(float4)))) return rc;
    HIP_TRY(hipMemcpy(s->mats.p, m.data(), m.size() * sizeof(float4), hipMemcpyHostToDevice));
    if ((rc = devAlloc(s->counters, kNumCounters * sizeof(unsigned long long)))) return rc;
    if ((rc = devAlloc(s->dobjs, (size_t)std::max<int64_t>(1, n) * sizeof(pt_object)))) return rc;
    if (n > 0) HIP_TRY(hipMemcpy(s->dobjs.p, objs, (size_t)n * sizeof(pt_object), hipMemcpyHostToDevice));
    *out = s.release();
    return PT_OK;
}

int pt_scene_create_instanced(int device, const pt_object* objs, int64_t n, const int64_t* mesh_first,
                              const int64_t* mesh_count, int n_meshes, const pt_instance* inst, int64_t n_inst,
                              const pt_material* mats, int64_t nmat, pt_scene** out) {
    if (!out || n < 0 || n_meshes < 0 || n_inst <= 0 || (n > 0 && !objs) || (n_meshes > 0 && (!mesh_first || !mesh_count)) ||
        !inst || (nmat > 0 && !mats))
        return fail(PT_ERR_INVALID, "pt_scene_create_instanced: bad argument");
    for (int m = 0; m < n_meshes; m++)
        if (mesh_first[m] < 0 || mesh_count[m] < 0 || mesh_first[m] + mesh_count[m] > n)
            return fail(PT_ERR_INVALID, "pt_scene_create_instanced: mesh range out of bounds");
    for (int64_t i = 0; i < n_inst; i++)
        if (inst[i].mesh < 0 || inst[i].mesh >= n_meshes)
            return fail(PT_ERR_INVALID, "pt_scene_create_instanced: instance of an unknown mesh");
    pt_scene* s = nullptr;
    int rc = pt_scene_create(device, objs, n, mats, nmat, &s);
    if (rc) return rc;
    s->instanced = true;
    s->meshFirst.assign(mesh_first, mesh_first + n_meshes);
    s->meshCount.assign(mesh_count, mesh_count + n_meshes);
    s->inst.assign(inst, inst + n_inst);
    *out = s;
    return PT_OK;
}

int pt_scene_update_objects(pt_scene* s, const pt_object* objs, int64_t first, int64_t n) {
    if (!s || first < 0 || n < 0 || first > s->nobj || n > s->nobj - first || (n > 0 && !objs))
        return fail(PT_ERR_INVALID, "pt_scene_update_objects: bad argument");
    if (s->instanced) return fail(PT_ERR_INVALID, "pt_scene_update_objects: not for instanced scenes");
    for (int64_t i = 0; i < n; i++) {
        if (objs[i].type != PT_SPHERE && objs[i].type != PT_TRIANGLE)
            return fail(PT_ERR_INVALID, "pt_scene_update_objects: unknown object type");
        if (objs[i].mat < 0 || objs[i].mat >= s->nmat)
            return fail(PT_ERR_INVALID, "pt_scene_update_objects: material id out of range");
    }
    int rc = setDevice(s->device);
    if (rc) return rc;
    if (n == 0) return PT_OK;
    std::copy(objs, objs + n, s->objs.begin() + first);
    for (int64_t i = 0; i < n && !s->hasSpheres; i++) s->hasSpheres = objs[i].type == PT_SPHERE;
    HIP_TRY(hipMemcpy(s->dobjs.as<pt_object>() + first, objs, (size_t)n * sizeof(pt_object), hipMemcpyHostToDevice));
    s->built = false;   // the hierarchy no longer matches the objects: rebuild before rendering
    s->updated = true;  // from now on the wide tree is built on the device (once per rebuild)
    return PT_OK;
}

int pt_scene_build_bvh(pt_scene* s, int flags) { return pt_scene_build_bvh_ex(s, flags, nullptr); }

int pt_scene_build_bvh_ex(pt_scene* s, int flags, void* stream) {
    if (!s) return fail(PT_ERR_INVALID, "pt_scene_build_bvh: null scene");
    int rc = setDevice(s->device);
    if (rc) return rc;
    if (s->instanced) {   // the two-level tree, on the host (flags: the LBVH's, not applicable)
        s->built = false;
        return buildInstanced(s);
    }
    const int64_t n = s->nobj;
    s->built = false;
    s->wideReady = false;   // the wide buffers are kept for the next wide build
    s->wideSource = 0;
    s->wideNodes = 0;
    s->wideDepth = 0;
    // Everything on the device, on one stream: scene box -> Morton codes -> radix sort ->
    // leaf records -> Karras hierarchy -> refit -> depth.  (PT_BVH_HOST_KEYS: the keys come from
    // the host restatement of computeMortonOnHost instead; the result is identical.)
    const size_t n1 = (size_t)std::max<int64_t>(1, n), ni = (size_t)std::max<int64_t>(1, n - 1);
    if ((rc = devReserve(s->prims, n1 * 3 * sizeof(float4))) || (rc = devReserve(s->shade, n1 * 3 * sizeof(float4))) ||
        (rc = devReserve(s->nodes, ni * 4 * sizeof(float4))) || (rc = devReserve(s->keys, n1 * 8)) ||
        (rc = devReserve(s->leafBoxes, n1 * 24)) || (rc = devReserve(s->iparent, ni * 4)) ||
        (rc = devReserve(s->lparent, n1 * 4)) || (rc = devReserve(s->irange, ni * 8)) ||
        (rc = devReserve(s->refitEvents, (n1 + 2) * 4)))   // count + at most (crossing nodes + 1) <= n arrivals
        return rc;
    DevBuf &codes = s->codes, &ids = s->ids, &codes2 = s->codes2, &ids2 = s->ids2, &box6 = s->box6, &sph = s->sph,
           &arr = s->arr, &dep = s->dep, &temp = s->sortTemp;
    if ((rc = devReserve(codes, n1 * 4)) || (rc = devReserve(ids, n1 * 4)) || (rc = devReserve(codes2, n1 * 4)) ||
        (rc = devReserve(ids2, n1 * 4)) || (rc = devReserve(box6, (1 + kBoxBlocks) * 6 * sizeof(float))) || (rc = devReserve(sph, n1 * 4)) ||
        (rc = devReserve(arr, ni * 4)) || (rc = devReserve(dep, 16)))
        return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    // Every return path destroys the events and, on failure, waits for the work already queued on
    // the stream (it uses the scene's buffers).
    StreamGuard guard(st);
    HIP_TRY(hipEventCreate(&guard.e0));
    HIP_TRY(hipEventCreate(&guard.e1));
    hipEvent_t e0 = guard.e0, e1 = guard.e1;
    HIP_TRY(hipEventRecord(e0, st));
    const unsigned tb = 256, nb = (unsigned)((n1 + tb - 1) / tb), nbi = (unsigned)((ni + tb - 1) / tb);
    if (n > 0) {
        if (flags & PT_BVH_HOST_KEYS) {
            std::vector<uint64_t> hk((size_t)n);
            pt::mortonKeys(s->objs.data(), n, (flags & PT_BVH_ORIGIN_BOUNDS) != 0, hk.data());
            std::vector<uint32_t> hc((size_t)n), hi((size_t)n);
            for (int64_t k = 0; k < n; k++) { hc[k] = (uint32_t)(hk[k] >> 32); hi[k] = (uint32_t)hk[k]; }
            HIP_TRY(hipMemcpyAsync(codes2.p, hc.data(), n * 4, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(ids2.p, hi.data(), n * 4, hipMemcpyHostToDevice, st));
            HIP_TRY(hipStreamSynchronize(st));
        } else {
            const int inc = (flags & PT_BVH_ORIGIN_BOUNDS) ? 1 : 0;
            sceneBoxKernel<<<kBoxBlocks, 1024, 0, st>>>(s->dobjs.as<pt_object>(), n, inc, box6.as<float>(),
                                                        box6.as<float>() + 6);
            sceneBoxKernel<<<1, 1024, 0, st>>>(s->dobjs.as<pt_object>(), n, inc, box6.as<float>(), nullptr);
            mortonKernel<<<nb, tb, 0, st>>>(s->dobjs.as<pt_object>(), n, box6.as<float>(), codes.as<uint32_t>(),
                                            ids.as<uint32_t>());
            HIP_TRY(hipGetLastError());
            size_t tbytes = 0;
            HIP_TRY(pt::radixSortPairs(nullptr, &tbytes, codes.as<uint32_t>(), codes2.as<uint32_t>(),
                                       ids.as<uint32_t>(), ids2.as<uint32_t>(), (size_t)n, 30, st));
            if ((rc = devReserve(temp, tbytes))) return rc;
            HIP_TRY(pt::radixSortPairs(temp.p, &tbytes, codes.as<uint32_t>(), codes2.as<uint32_t>(),
                                       ids.as<uint32_t>(), ids2.as<uint32_t>(), (size_t)n, 30, st));
        }
        leafGatherKernel<<<nb, tb, 0, st>>>(s->dobjs.as<pt_object>(), codes2.as<uint32_t>(), ids2.as<uint32_t>(), n,
                                            s->keys.as<unsigned long long>(), s->prims.as<float4>(),
                                            s->shade.as<float4>(), s->leafBoxes.as<float>(), sph.as<uint32_t>(),
                                            s->mats.as<float4>());
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipMemsetAsync(s->nodes.p, 0, ni * 4 * sizeof(float4), st));
    HIP_TRY(hipMemsetAsync(s->iparent.p, 0xff, ni * 4, st));
    HIP_TRY(hipMemsetAsync(s->lparent.p, 0xff, n1 * 4, st));
    HIP_TRY(hipMemsetAsync(arr.p, 0, ni * 4, st));
    HIP_TRY(hipMemsetAsync(s->refitEvents.p, 0, 4, st));
    HIP_TRY(hipMemsetAsync(dep.p, 0, 16, st));
    if (n > 1) {
        karrasKernel<<<nbi, tb, 0, st>>>(s->keys.as<unsigned long long>(), (int)n, s->nodes.as<float4>(),
                                         s->iparent.as<int>(), s->lparent.as<int>(), sph.as<uint32_t>(),
                                         s->irange.as<int2>());
        HIP_TRY(hipGetLastError());
        refitKernel<<<(unsigned)((n + kRefitBlock - 1) / kRefitBlock), kRefitBlock, 0, st>>>(
            s->nodes.as<float4>(), s->iparent.as<int>(), s->lparent.as<int>(), s->irange.as<int2>(),
            s->leafBoxes.as<float>(), s->refitEvents.as<unsigned int>(), (int)n);
        refitTopKernel<<<1, kRefitTop, 0, st>>>(s->nodes.as<float4>(), s->iparent.as<int>(),
                                                s->refitEvents.as<unsigned int>(), arr.as<unsigned int>());
        HIP_TRY(hipGetLastError());
        depthKernel<<<nb, tb, 0, st>>>(s->iparent.as<int>(), s->lparent.as<int>(), (int)n, dep.as<int>());
        HIP_TRY(hipGetLastError());
    }
    if ((flags & PT_BVH_WIDE_DEVICE) && n > 0) {
        if ((rc = buildWideDevice(s, st))) return rc;
        s->wideReady = true;
        s->wideBuildMs = 0.0;
    }
    HIP_TRY(hipEventRecord(e1, st));
    HIP_TRY(hipEventSynchronize(e1));
    guard.ok = true;
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    s->buildMs = ms;
    int depth = 0;
    HIP_TRY(hipMemcpy(&depth, dep.p, 4, hipMemcpyDeviceToHost));
    s->depth = n > 1 ? depth : 0;
    if (n > 0) {   // the tight scene box: union of the root's child boxes (a single object: its box)
        float mn[3], mx[3];
        if (n > 1) {
            float r[12];
            HIP_TRY(hipMemcpy(r, s->nodes.p, sizeof(r), hipMemcpyDeviceToHost));
            for (int a = 0; a < 3; a++) {
                mn[a] = std::fmin(r[nodeBoxIdx(0, a, 0)], r[nodeBoxIdx(1, a, 0)]);
                mx[a] = std::fmax(r[nodeBoxIdx(0, a, 1)], r[nodeBoxIdx(1, a, 1)]);
            }
        } else {
            float b6[6];
            HIP_TRY(hipMemcpy(b6, s->leafBoxes.p, sizeof(b6), hipMemcpyDeviceToHost));
            for (int a = 0; a < 3; a++) { mn[a] = b6[a]; mx[a] = b6[3 + a]; }
        }
        float e = 0.0f;
        double m = 0.0;
        for (int a = 0; a < 3; a++) {
            s->sceneCE[a] = 0.5f * (mn[a] + mx[a]);
            e = std::fmax(e, mx[a] - mn[a]);
            m = std::max({m, std::fabs((double)mn[a]), std::fabs((double)mx[a]), (double)mx[a] - (double)mn[a]});
        }
        s->sceneCE[3] = e;
        s->mixLim = mixLimit(m);
    }
    if (n > 1 && stackFor(s->depth) < 0) return fail(PT_ERR_STATE, "BVH too deep");
    if (s->wideReady && wideStackFor(s->wideDepth) < 0) return fail(PT_ERR_STATE, "wide BVH too deep");
    s->deviceBytes = (size_t)(n > 1 ? n - 1 : 0) * 64 + (size_t)n * 96 + (size_t)s->nmat * 32;
    s->built = true;
    return PT_OK;
}

// The wide tree is only needed by PT_KERNEL_WIDE: unless pt_scene_build_bvh built it on the
// device (PT_BVH_WIDE_DEVICE), built on first use after each LBVH build -- on the device for a
// scene whose objects were updated (dynamic: a rebuild per frame) or when PT_WIDE_BUILD=device,
// else on the host (binned SAH: a few percent faster to trace, slower to build).
static int ensureWide(pt_scene* s) {
    if (s->wideReady || s->nobj <= 0) return PT_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const char* wb = std::getenv("PT_WIDE_BUILD");
    const std::string wbs = wb ? wb : "";
    const bool device = wbs == "device" || (s->updated && wbs != "host");
    int rc = device ? buildWideDevice(s, 0) : buildWide(s);
    if (!rc && s->wideSource == 2) HIP_TRY(hipStreamSynchronize(0));
    if (rc) return rc;
    s->wideReady = true;
    s->wideBuildMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (wideStackFor(s->wideDepth) < 0) return fail(PT_ERR_STATE, "wide BVH too deep");
    return PT_OK;
}

int pt_scene_wide_info(pt_scene* s, int* depth, int64_t* slots, double* ms, int* source) {
    if (!s) return fail(PT_ERR_INVALID, "pt_scene_wide_info: null scene");
    const bool ok = s->wideReady;
    if (depth) *depth = ok ? s->wideDepth : 0;
    if (slots) *slots = ok ? s->wideNodes : 0;
    if (ms) *ms = ok ? s->wideBuildMs : 0.0;
    if (source) *source = ok ? s->wideSource : 0;
    return PT_OK;
}

int pt_scene_build_time(pt_scene* s, double* ms) {
    if (!s || !ms) return fail(PT_ERR_INVALID, "pt_scene_build_time: null argument");
    if (!s->built) return fail(PT_ERR_STATE, "BVH not built");
    *ms = s->buildMs;
    return PT_OK;
}

int pt_scene_bvh_info(pt_scene* s, int* depth, int64_t* nodes, int64_t* bytes) {
    if (!s) return fail(PT_ERR_INVALID, "pt_scene_bvh_info: null scene");
    if (!s->built) return fail(PT_ERR_STATE, "BVH not built");
    if (depth) *depth = s->depth;
    if (nodes) *nodes = s->nobj > 0 ? 2 * s->nobj - 1 : 0;
    if (bytes) *bytes = (int64_t)s->deviceBytes;
    return PT_OK;
}

int pt_scene_download_bvh(pt_scene* s, pt_bvh_node* out) {
    if (!s || !out) return fail(PT_ERR_INVALID, "pt_scene_download_bvh: null argument");
    if (!s->built) return fail(PT_ERR_STATE, "BVH not built");
    if (s->instanced) return fail(PT_ERR_STATE, "pt_scene_download_bvh: an instanced scene has no LBVH");
    int rc = setDevice(s->device);
    if (rc) return rc;
    const int64_t n = s->nobj;
    if (n <= 0) return PT_OK;
    const int64_t L = n - 1;
    std::vector<float4> nodes((size_t)std::max<int64_t>(1, L) * 4);
    std::vector<uint64_t> keys((size_t)n);
    std::vector<int32_t> iparent((size_t)std::max<int64_t>(1, L)), lparent((size_t)n);
    std::vector<float> leafBoxes((size_t)n * 6);
    if (L > 0) HIP_TRY(hipMemcpy(nodes.data(), s->nodes.p, L * 4 * sizeof(float4), hipMemcpyDeviceToHost));
    if (L > 0) HIP_TRY(hipMemcpy(iparent.data(), s->iparent.p, L * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(keys.data(), s->keys.p, n * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(lparent.data(), s->lparent.p, n * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(leafBoxes.data(), s->leafBoxes.p, n * 24, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < 2 * n - 1; i++) {
        out[i].left = out[i].right = out[i].parent = out[i].objid = -1;
        for (int a = 0; a < 3; a++) out[i].bmin[a] = out[i].bmax[a] = 0.0f;
    }
    auto refIndex = [&](uint32_t r) -> int64_t { return (r & kLeafBit) ? L + (int64_t)(r & kPrimMask) : (int64_t)r; };
    for (int64_t k = 0; k < n; k++) {
        out[L + k].objid = (int32_t)(keys[k] & 0xffffffffu);
        out[L + k].parent = L > 0 ? lparent[k] : -1;
    }
    for (int64_t i = 0; i < L; i++) {
        const float* f = reinterpret_cast<const float*>(&nodes[4 * i]);
        uint32_t lr, rr;
        std::memcpy(&lr, f + 12, 4);
        std::memcpy(&rr, f + 13, 4);
        out[i].left = (int32_t)refIndex(lr);
        out[i].right = (int32_t)refIndex(rr);
        out[i].parent = i == 0 ? -1 : iparent[i];
        for (int c = 0; c < 2; c++) {   // child boxes live in this record; copy them to the child
            pt_bvh_node& ch = out[c == 0 ? out[i].left : out[i].right];
            for (int a = 0; a < 3; a++) { ch.bmin[a] = f[nodeBoxIdx(c, a, 0)]; ch.bmax[a] = f[nodeBoxIdx(c, a, 1)]; }
        }
        if (i == 0) {   // the root's own box (never tested by the traversal)
            for (int a = 0; a < 3; a++) {
                out[0].bmin[a] = std::fmin(f[nodeBoxIdx(0, a, 0)], f[nodeBoxIdx(1, a, 0)]);
                out[0].bmax[a] = std::fmax(f[nodeBoxIdx(0, a, 1)], f[nodeBoxIdx(1, a, 1)]);
            }
        }
    }
    if (L == 0) {   // single object: the root is the leaf (bvh.h:76-81 with numObjects = 1)
        for (int a = 0; a < 3; a++) { out[0].bmin[a] = leafBoxes[a]; out[0].bmax[a] = leafBoxes[3 + a]; }
    }
    return PT_OK;
}

int pt_trace_closest(pt_scene* s, const pt_ray* rays, int64_t n, float tmin, float tmax, pt_hit* hits,
                     pt_stats* stats) {
    return pt_trace_closest_ex(s, rays, n, tmin, tmax, PT_KERNEL_DEFAULT, hits, stats);
}

}  // extern "C"

namespace {
// Closest hits of n rays: rays / hits are device arrays (dr, dh), traced on `st`; the host waits
// for the end (counters and the guard word are read back).
int traceDevice(pt_scene* s, const pt_ray* dr, int64_t n, float tmin, float tmax, int kernel, pt_hit* dh,
                hipStream_t st, pt_stats* stats) {
    if (kernel != PT_KERNEL_DEFAULT && kernel != PT_KERNEL_SIMPLE && kernel != PT_KERNEL_WAVEFRONT &&
        kernel != PT_KERNEL_WIDE)
        return fail(PT_ERR_INVALID, "pt_trace_closest: unknown kernel");
    if (!s->built) return fail(PT_ERR_STATE, "BVH not built");
    int rc = setDevice(s->device);
    if (rc) return rc;
    const bool wide = kernel == PT_KERNEL_WIDE || s->instanced;
    if (s->instanced && kernel != PT_KERNEL_DEFAULT && kernel != PT_KERNEL_WIDE)
        return fail(PT_ERR_INVALID, "pt_trace_closest: instanced scenes trace with the wide kernel");
    if (wide && (rc = ensureWide(s))) return rc;
    const int stack = wide ? wideStackFor(s->wideDepth) : (s->nobj > 1 ? stackFor(s->depth) : 16);
    StreamGuard guard(st);
    HIP_TRY(hipMemsetAsync(s->counters.p, 0, kNumCounters * sizeof(unsigned long long), st));
    HIP_TRY(hipEventCreate(&guard.e0));
    HIP_TRY(hipEventCreate(&guard.e1));
    HIP_TRY(hipEventRecord(guard.e0, st));
    if (n > 0 && (rc = dispatchTrace(stack, wide, devScene(s), dr, n, tmin, tmax, dh, s->counters.as<unsigned long long>(), st)))
        return rc;
    HIP_TRY(hipEventRecord(guard.e1, st));
    HIP_TRY(hipEventSynchronize(guard.e1));
    guard.ok = true;
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, guard.e0, guard.e1));
    unsigned long long c[kNumCounters] = {0};
    HIP_TRY(hipMemcpy(c, s->counters.p, sizeof(c), hipMemcpyDeviceToHost));
    c[4] = 0;
    fillStats(stats, c, ms, wide);
    if (c[7]) return fail(PT_ERR_STATE, "traversal guard tripped (corrupt BVH), flags " + std::to_string(c[7]));
    return PT_OK;
}
}  // namespace

extern "C" {

int pt_trace_closest_ex(pt_scene* s, const pt_ray* rays, int64_t n, float tmin, float tmax, int kernel, pt_hit* hits,
                        pt_stats* stats) {
    if (!s || n < 0 || (n > 0 && (!rays || !hits))) return fail(PT_ERR_INVALID, "pt_trace_closest: bad argument");
    int rc = setDevice(s->device);
    if (rc) return rc;
    DevBuf dr, dh;
    if ((rc = devAlloc(dr, n * sizeof(pt_ray))) || (rc = devAlloc(dh, n * sizeof(pt_hit)))) return rc;
    if (n > 0) HIP_TRY(hipMemcpy(dr.p, rays, n * sizeof(pt_ray), hipMemcpyHostToDevice));
    if ((rc = traceDevice(s, dr.as<pt_ray>(), n, tmin, tmax, kernel, dh.as<pt_hit>(), 0, stats))) return rc;
    if (n > 0) HIP_TRY(hipMemcpy(hits, dh.p, n * sizeof(pt_hit), hipMemcpyDeviceToHost));
    return PT_OK;
}

int pt_trace_closest_device(pt_scene* s, const pt_ray* rays, int64_t n, float tmin, float tmax, int kernel,
                            pt_hit* hits, void* stream, pt_stats* stats) {
    if (!s || n < 0 || (n > 0 && (!rays || !hits))) return fail(PT_ERR_INVALID, "pt_trace_closest_device: bad argument");
    return traceDevice(s, rays, n, tmin, tmax, kernel, hits, static_cast<hipStream_t>(stream), stats);
}

int pt_film_create(int device, int width, int height, int sh, int nparts, int part, uint64_t seed, pt_film** out) {
    if (!out || width <= 0 || height <= 0 || sh <= 0 || nparts <= 0 || part < 0 || part >= nparts)
        return fail(PT_ERR_INVALID, "pt_film_create: bad argument");
    if ((int64_t)width * height >= (1ll << kJumpMats)) return fail(PT_ERR_INVALID, "pt_film_create: frame too large");
    int rc = setDevice(device);
    if (rc) return rc;
    std::unique_ptr<pt_film> f(new pt_film);
    f->device = device;
    f->width = width;
    f->height = height;
    f->stripe_h = sh;
    f->nparts = nparts;
    f->part = part;
    int rows = 0;
    for (int r = 0; r < height; r++)
        if ((r / sh) % nparts == part) rows++;
    f->nrows = rows;
    f->npix = (int64_t)rows * width;
    if ((rc = devAlloc(f->state, (size_t)std::max<int64_t>(1, f->npix) * 6 * 4))) return rc;
    f->seed = seed;
    const std::vector<uint32_t>& jm = jumpMatrices();
    if ((rc = devAlloc(f->jumps, jm.size() * 4))) return rc;
    HIP_TRY(hipMemcpy(f->jumps.p, jm.data(), jm.size() * 4, hipMemcpyHostToDevice));
    if ((rc = filmInit(f.get(), 0))) return rc;
    HIP_TRY(hipDeviceSynchronize());
    *out = f.release();
    return PT_OK;
}

int pt_film_reset(pt_film* f, void* stream) {
    if (!f) return fail(PT_ERR_INVALID, "pt_film_reset: null film");
    int rc = setDevice(f->device);
    if (rc) return rc;
    return filmInit(f, (hipStream_t)stream);
}

int pt_film_clear(pt_film* f, void* stream) {
    if (!f) return fail(PT_ERR_INVALID, "pt_film_clear: null film");
    int rc = setDevice(f->device);
    if (rc) return rc;
    if (f->accum.p) HIP_TRY(hipMemsetAsync(f->accum.p, 0, (size_t)std::max<int64_t>(1, f->npix) * 12, (hipStream_t)stream));
    f->accumSamples = 0;
    return PT_OK;
}

int pt_film_accumulated(pt_film* f, int64_t* samples) {
    if (!f || !samples) return fail(PT_ERR_INVALID, "pt_film_accumulated: null argument");
    *samples = f->accumSamples;
    return PT_OK;
}

int pt_film_info(pt_film* f, int* nrows, int64_t* npix) {
    if (!f) return fail(PT_ERR_INVALID, "pt_film_info: null film");
    if (nrows) *nrows = f->nrows;
    if (npix) *npix = f->npix;
    return PT_OK;
}

int pt_film_rows(pt_film* f, int32_t* rows) {
    if (!f || !rows) return fail(PT_ERR_INVALID, "pt_film_rows: null argument");
    int k = 0;
    for (int r = 0; r < f->height; r++)
        if ((r / f->stripe_h) % f->nparts == f->part) rows[k++] = r;
    return PT_OK;
}

int pt_film_get_rng(pt_film* f, uint32_t* states) {
    if (!f || !states) return fail(PT_ERR_INVALID, "pt_film_get_rng: null argument");
    int rc = setDevice(f->device);
    if (rc) return rc;
    const int64_t np = f->npix;
    std::vector<uint32_t> soa((size_t)np * 6);
    if (np) HIP_TRY(hipMemcpy(soa.data(), f->state.p, np * 24, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < np; i++)
        for (int w = 0; w < 6; w++) states[6 * i + w] = soa[(size_t)w * np + i];
    return PT_OK;
}

int pt_film_set_rng(pt_film* f, const uint32_t* states) {
    if (!f || !states) return fail(PT_ERR_INVALID, "pt_film_set_rng: null argument");
    int rc = setDevice(f->device);
    if (rc) return rc;
    const int64_t np = f->npix;
    std::vector<uint32_t> soa((size_t)np * 6);
    for (int64_t i = 0; i < np; i++)
        for (int w = 0; w < 6; w++) soa[(size_t)w * np + i] = states[6 * i + w];
    if (np) HIP_TRY(hipMemcpy(f->state.p, soa.data(), np * 24, hipMemcpyHostToDevice));
    return PT_OK;
}

int pt_render(pt_scene* s, pt_film* f, const pt_camera* cam, int spp, int max_depth, float* out, int on_dev,
              void* stream, pt_stats* stats) {
    return pt_render_ex(s, f, cam, spp, max_depth, out, on_dev, stream, nullptr, stats);
}

int pt_render_ex(pt_scene* s, pt_film* f, const pt_camera* cam, int spp, int max_depth, float* out, int on_dev,
                 void* stream, const pt_render_opts* opts, pt_stats* stats) {
    if (!s || !f || !cam || !out || spp <= 0) return fail(PT_ERR_INVALID, "pt_render: bad argument");
    if (!s->built) return fail(PT_ERR_STATE, "pt_render: BVH not built");
    if (s->device != f->device) return fail(PT_ERR_INVALID, "pt_render: scene and film on different devices");
    if (!(cam->lens_radius >= 0.0f) || !std::isfinite(cam->lens_radius))
        return fail(PT_ERR_INVALID, "pt_render: lens radius must be finite and >= 0");
    int rc = setDevice(s->device);
    if (rc) return rc;
    hipStream_t st = on_dev ? (hipStream_t)stream : 0;
    const int64_t np = f->npix;
    const int fmt = opts ? opts->out_format : PT_OUT_RGB32F;
    if (fmt != PT_OUT_RGB32F && fmt != PT_OUT_RGBA8 && fmt != PT_OUT_RGBA8_SURFACE)
        return fail(PT_ERR_INVALID, "pt_render_ex: unknown output format");
    const bool accumulate = opts && (opts->flags & PT_RENDER_ACCUMULATE);
    const size_t outBpp = fmt == PT_OUT_RGB32F ? 12 : 4;
    if (accumulate && f->accumSamples + spp >= (1ll << 24))
        return fail(PT_ERR_INVALID, "pt_render_ex: accumulated samples must stay below 2^24");
    // Kernel choice and wavefront-scheduler thresholds (lanes of 64): explicit options win, then
    // the PT_RENDER_KERNEL / PT_LEAF_BATCH / PT_SHADE_BATCH environment (tuning), then defaults.
    int kernel = opts ? opts->kernel : PT_KERNEL_DEFAULT;
    if (kernel == PT_KERNEL_DEFAULT) {
        const char* k = std::getenv("PT_RENDER_KERNEL");
        const std::string ks = k ? k : "";
        kernel = ks == "simple" ? PT_KERNEL_SIMPLE : (ks == "wavefront" ? PT_KERNEL_WAVEFRONT : PT_KERNEL_WIDE);
    }
    if (kernel != PT_KERNEL_SIMPLE && kernel != PT_KERNEL_WAVEFRONT && kernel != PT_KERNEL_WIDE)
        return fail(PT_ERR_INVALID, "pt_render_ex: unknown kernel");
    if (s->instanced && kernel != PT_KERNEL_WIDE)
        return fail(PT_ERR_INVALID, "pt_render_ex: instanced scenes render with the wide kernel (PT_KERNEL_WIDE)");
    const int rng = opts ? opts->rng : PT_RNG_COMPAT;
    if (rng != PT_RNG_COMPAT && rng != PT_RNG_SAMPLE) return fail(PT_ERR_INVALID, "pt_render_ex: unknown rng mode");
    if (kernel == PT_KERNEL_WIDE && (rc = ensureWide(s))) return rc;   // (first use: builds the tree)

    // Film resources, allocated once and reused by every later render (no hipMalloc / hipFree,
    // which synchronise the device, in the per-frame path).
    if (!f->ev0) {
        HIP_TRY(hipEventCreate(&f->ev0));
        HIP_TRY(hipEventCreate(&f->ev1));
        HIP_TRY(hipEventCreateWithFlags(&f->ev2, hipEventDisableTiming));
    }
    if (!f->counters.p && (rc = devAlloc(f->counters, kNumCounters * sizeof(unsigned long long)))) return rc;
    if (!f->hostCounters) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&f->hostCounters),
                                                kNumCounters * sizeof(unsigned long long), hipHostMallocDefault));
    void* dst = out;
    if (!on_dev) {
        if ((rc = devReserve(f->staging, (size_t)std::max<int64_t>(1, np) * outBpp))) return rc;
        dst = f->staging.p;
    }
    HIP_TRY(hipMemsetAsync(f->counters.p, 0, kNumCounters * sizeof(unsigned long long), st));
    RenderParams P;
    P.S = devScene(s);
    P.S.err = reinterpret_cast<unsigned int*>(f->counters.as<unsigned long long>() + 7);
    P.cam.pos = make_float3(cam->origin[0], cam->origin[1], cam->origin[2]);
    P.cam.ll = make_float3(cam->lower_left[0], cam->lower_left[1], cam->lower_left[2]);
    P.cam.hor = make_float3(cam->horizontal[0], cam->horizontal[1], cam->horizontal[2]);
    P.cam.ver = make_float3(cam->vertical[0], cam->vertical[1], cam->vertical[2]);
    P.cam.right = make_float3(cam->right[0], cam->right[1], cam->right[2]);
    P.cam.up = make_float3(cam->up[0], cam->up[1], cam->up[2]);
    P.cam.lens = cam->lens_radius;
    uint32_t* b = f->state.as<uint32_t>();
    P.sd = b; P.s0 = b + np; P.s1 = b + 2 * np; P.s2 = b + 3 * np; P.s3 = b + 4 * np; P.s4 = b + 5 * np;
    P.out = static_cast<float*>(dst);
    P.rawOut = 0;
    P.sampleBase = 0;
    P.counters = f->counters.as<unsigned long long>();
    P.width = f->width;
    P.nrows = f->nrows;
    P.stripe_h = f->stripe_h;
    P.stripeShift = (f->stripe_h & (f->stripe_h - 1)) == 0 ? __builtin_ctz((unsigned)f->stripe_h) : -1;
    P.nparts = f->nparts;
    P.part = f->part;
    P.tiles_x = (f->width + 7) / 8;
    P.ntiles = P.tiles_x * ((f->nrows + 7) / 8);
    P.spp = spp;
    P.max_depth = max_depth;
    P.invW = 1.0f / (float)f->width;    // main.cu:281
    P.invH = 1.0f / (float)f->height;
    P.invSpp = 1.0f / (float)spp;
    if (kernel == PT_KERNEL_WIDE && s->nobj > 0 && (!P.S.wnodes || !P.S.wprims)) return fail(PT_ERR_STATE, "wide BVH missing");
    P.kernel = kernel;
    P.nblocks = 0;
    P.block = 0;
    P.blockShift = -1;
    P.group = 1;
    P.span = 0;
    P.ngroups = 0;
    P.pixAcc = nullptr;
    P.taskCounter = nullptr;
    P.stackSpill = nullptr;
    P.ntasks = 0;
    P.nwaves = 0;
    P.seed0 = (uint32_t)f->seed;
    P.seed1 = (uint32_t)(f->seed >> 32);
    P.measureCost = 0;
    {   // wideFar (pt_device.hip) for the camera: its rays then take the reference-order path
        // (instanced scenes: start at their entry into the world, instEntry).  A lens sample moves
        // the origin by lens * (x right + y up) with x^2 + y^2 < 1, i.e. by at most
        // lens * (|right_a| + |up_a|) on axis a, whatever right / up the caller filled in.
        double m = 0.0;
        for (int a = 0; a < 3; a++)
            m = std::max(m, std::fabs((double)cam->origin[a] - (double)s->sceneCE[a]) +
                                (double)cam->lens_radius * (std::fabs((double)cam->right[a]) + std::fabs((double)cam->up[a])));
        P.camFar = !(m <= (s->wideSource == 3 ? (double)kInstFarExt : (double)kWideFarExt) * (double)s->sceneCE[3]) ? 1 : 0;
    }
    // Defaults swept on C3 (tools/ab_env.py): sample mode is throughput-bound and prefers full
    // LEAF / SHADE steps.  Compat mode on the binary tree is bound by its slowest pixels' sequential
    // chains: 20 / 12 together with nodeMin 8 (C3 1,521 -> 1,442 ms, C2 90.7 -> 80.0, C5 1,311 ->
    // 1,180 against 8 / 12).  Compat on the flattened wide tree, since round 6 (its critical chains
    // in critical-pixel waves, or short paths): the sample mode's wide thresholds with nodeMin 8 --
    // C3 @1024 (critical pixels on) 705 -> 649 ms (SHADE 28 alone 665, 20 674; LEAF 28 alone 695),
    // C5 @512 558 -> 539 (24 / 24), C2 @256 37.7 -> 37.1; nodeMin 0 740 / 617 ms, 4: 656 on C3.
    const bool sampleRng = rng == PT_RNG_SAMPLE;
    // sample mode, wide kernel (speculative traversal): LEAF at 28 waiting lanes, SHADE at 28
    // (C3 @256 spp 148.4 -> 145.0 ms vs 24 / 32; C5 @64 75.9 -> 74.5; C2 @1024 135.4 -> 134.5);
    // deep wide trees (a 16+ entry stack: C5's 1.04 M triangles) at 24 / 24 (round 3 close: C5 @64
    // 67.1 -> 65.1 ms, median of 5; C3 at 24 / 24 is 1 % slower, so shallow trees keep 28 / 28)
    const bool wideSample = sampleRng && kernel == PT_KERNEL_WIDE;
    const bool wideFlatCompat = !sampleRng && kernel == PT_KERNEL_WIDE && !s->instanced;
    const int stack = kernel == PT_KERNEL_WIDE ? wideStackFor(s->wideDepth) : (s->nobj > 1 ? stackFor(s->depth) : 16);
    const int wideBatch = stack >= 16 ? 24 : 28;
    // instanced scenes (no speculative traversal: a lane with primitives waiting cannot visit nodes)
    // take their LEAF steps earlier: LEAF 16 / SHADE 20 (round 5, C5 instanced @128 spp, interleaved
    // median of 3: 131.8 -> 128.8 ms; LEAF 12: 131.8, 8: 135.9, 32: 140.7; SHADE 28 with LEAF 16: 131.4)
    // (instanced compat takes them too: C5 instanced compat @512 618.6 -> 594.6 ms; 24 / 24: 609.8,
    // 28 / 28: 646.5)
    const bool instWide = kernel == PT_KERNEL_WIDE && s->instanced;
    P.leafBatch = (opts && opts->leaf_batch > 0) ? std::min(opts->leaf_batch, 64)
                                                 : envInt("PT_LEAF_BATCH", instWide ? 16 : (wideSample || wideFlatCompat) ? wideBatch
                                                                                                       : (sampleRng ? 24 : 20));
    // compat mode: a NODE step with fewer than nodeMin lanes yields to the larger of the waiting
    // LEAF / SHADE groups (C3 compat 1,620 -> 1,517 ms at 8; 4: 1,548, 16: 1,671, 32: 1,989)
    P.nodeMin = std::getenv("PT_NODE_MIN") ? std::atoi(std::getenv("PT_NODE_MIN")) : 8;
    P.shadeBatch = (opts && opts->shade_batch > 0) ? std::min(opts->shade_batch, 64)
                                                   : envInt("PT_SHADE_BATCH", instWide ? 20 : (wideSample || wideFlatCompat) ? wideBatch
                                                                                                           : (sampleRng ? 32 : 12));
    if (kernel == PT_KERNEL_SIMPLE) P.leafBatch = 0;
    const size_t ntl = (size_t)std::max(1, P.ntiles);
    if (!f->tileCost.p) {
        if ((rc = devAlloc(f->tileCost, ntl * 4)) || (rc = devAlloc(f->tileOrder, ntl * 4)) ||
            (rc = devAlloc(f->tileXY, ntl * 4)) || (rc = devAlloc(f->tileXYId, ntl * 4)))
            return rc;
        f->haveOrder = false;
    }
    const bool lpt = !(opts && (opts->flags & PT_RENDER_IDENTITY_ORDER));
    const bool sample = rng == PT_RNG_SAMPLE && np > 0 && P.ntiles > 0;
    // compat mode, pixel queue (renderKernelWF, PT_COMPAT_QUEUE): persistent waves take pixels
    const bool cq = PT_COMPAT_QUEUE && !sample && kernel != PT_KERNEL_SIMPLE && np > 0 && P.ntiles > 0;
    if (!f->cus) {
        if (hipDeviceGetAttribute(&f->cus, hipDeviceAttributeMultiprocessorCount, f->device) != hipSuccess)
            f->cus = 256;
        f->cus = std::max(f->cus, 1);
    }
    // persistent waves (sample mode, CQ): exactly the waves that fit at once -- the kernel's
    // occupancy per CU, which the LDS stack caps on deep trees.  Queried once per (device, kernel
    // instantiation) and process.
    auto perCUFor = [&](int& perCU) -> int {
        static std::atomic<int> cached[16][2][2][2][3];   // [device][sample][instanced][wide][stack 8, 16, 24]
        const bool small = stack <= 24 && stack % 8 == 0 && f->device >= 0 && f->device < 16;
        std::atomic<int>* c = small ? &cached[f->device][sample ? 1 : 0][s->instanced ? 1 : 0]
                                             [kernel == PT_KERNEL_WIDE ? 1 : 0][stack / 8 - 1] : nullptr;
        const int known = c ? c->load(std::memory_order_relaxed) : 0;
        if (known > 0) {
            perCU = known;
            return PT_OK;
        }
        if (int r = persistentWavesPerCU(stack, kernel, perCU, s->instanced, sample)) return r;
        if (c) c->store(perCU, std::memory_order_relaxed);
        return PT_OK;
    };
    // compat critical pixels (wide kernel, flattened scene, long paths): the previous launch's
    // PT_CRIT_PIXELS longest per-pixel chains run first, PT_CRIT_LANES pixels per wave, each lane
    // tracing its rays in one per-lane loop (a lane alone on its chain is not held back by the wave's
    // step kinds).  C3 compat @1024 (interleaved, median of 2): 773 ms without; 256 x 4 699 ms;
    // 64 x 1 710, 128 x 4 707, 512 x 4 712, 256 x 8 751 (with the split tiles as well).  The rays
    // per pixel are measured on every launch.
    P.nCrit = 0;
    P.critLanes = std::max(1, std::min(64, envCount("PT_CRIT_LANES", kCritLanes)));
    P.critWaves = 0;
    P.critList = nullptr;
    P.critFlag = nullptr;
    P.pixRays = nullptr;
    const bool critOn = lpt && critFor(sample, kernel == PT_KERNEL_WIDE, s->instanced, cq, stack) && np > 0 &&
                        max_depth > 16 && envCount("PT_CRIT_PIXELS", kCritPixels) > 0;
    if (critOn) {
        if ((rc = devReserve(f->pixRays, (size_t)np * 4))) return rc;
        P.pixRays = f->pixRays.as<uint32_t>();
        if (f->critK > 0) {
            P.nCrit = f->critK;
            P.critWaves = (P.nCrit + P.critLanes - 1) / P.critLanes;
            P.critList = f->pixSorted.as<uint32_t>();
            P.critFlag = f->critFlag.as<uint8_t>();
        }
    }
    // compat tile waves: the longest tiles of the launch order split into splitWays waves (renderKernelWF).
    // Only where a pixel's sequential chain can outlast the frame's throughput-bound part: long paths
    // (max_depth > 16; C3, depth 50: 800 -> 766 ms) on kernels without critical-pixel waves, which
    // take those chains out of the tile waves (C3 with both: 710 ms, critical pixels alone 699 ms).
    // Short-path frames are throughput-bound and the split's idle lanes cost (C5, depth 16: 548 ->
    // 553 ms; C2, depth 8: +0.9 %).
    P.splitWays = std::max(1, std::min(8, envCount("PT_SPLIT_WAYS", 2)));
    P.splitTiles = (lpt && f->haveOrder && !sample && !cq && kernel != PT_KERNEL_SIMPLE)
                       ? std::max(0, std::min(P.ntiles, envCount("PT_SPLIT_TILES", max_depth > 16 && !critOn ? 128 : 0))) : 0;
    if (P.splitWays == 1 || PT_AB_NO_SPLIT) P.splitTiles = 0;   // (a build without the split prologue: grid = tiles)
    P.compatGrid = P.critWaves + P.ntiles + P.splitTiles * (P.splitWays - 1);
    // diagnostic: only the first k waves of the launch order (the longest tiles) -- their chains'
    // latency with the machine otherwise idle; the other pixels are not rendered
    if (const int lim = envCount("PT_COMPAT_GRID_LIMIT", 0)) P.compatGrid = std::min(P.compatGrid, lim);
    if (cq) {
        P.ntasks = (uint32_t)P.ntiles * 64u;   // queue slots: tile slot x 64 pixels
        if (!f->taskCounter.p && (rc = devAlloc(f->taskCounter, 64))) return rc;
        HIP_TRY(hipMemsetAsync(f->taskCounter.p, 0, 4, st));
        P.taskCounter = f->taskCounter.as<unsigned>();
        int perCU = 0;
        if ((rc = perCUFor(perCU))) return rc;
        P.nwaves = (int)std::min<uint64_t>((uint64_t)f->cus * (uint64_t)std::max(1, perCU) * (uint64_t)envInt("PT_CQ_WAVES_MULT", 1),
                                           (uint64_t)P.ntiles);
        if (std::getenv("PT_ITER_STATS"))
            std::fprintf(stderr, "[pt] compat pixel queue: persistent waves %d (%d per CU, stack %d)\n", P.nwaves, perCU, stack);
        // tile costs (the rays of the tile's longest pixel, atomicMax per pixel) on every launch
        P.measureCost = lpt ? 1 : 0;
        if (P.measureCost) HIP_TRY(hipMemsetAsync(f->tileCost.p, 0, ntl * 4, st));
    }
    if (sample) {
        if (f->width >= 65536 || f->nrows >= 65536)
            return fail(PT_ERR_INVALID, "sample mode: frame width and rows must be < 65536");
        P.block = (opts && opts->chunk > 0) ? opts->chunk : std::max(16, (spp + 63) / 64);
        P.nblocks = (spp + P.block - 1) / P.block;
        P.blockShift = (P.block & (P.block - 1)) == 0 ? __builtin_ctz((unsigned)P.block) : -1;
        // blocks per task (the simple kernel always takes one)
        P.group = (!PT_TASK_GROUPS || kernel != PT_KERNEL_WIDE || stack > 16) ? 1   // (renderKernelWF's GROUPS)
                                                          : std::max(1, std::min(P.nblocks, envInt("PT_TASK_BLOCKS", kTaskBlocks)));
        P.span = P.group * P.block;
        P.ngroups = (spp + P.span - 1) / P.span;
        if ((rc = devReserve(f->pixAcc, (size_t)np * 32))) return rc;   // {x, y, z, rays} per pixel
        HIP_TRY(hipMemsetAsync(f->pixAcc.p, 0, (size_t)np * 32, st));
        P.pixAcc = f->pixAcc.as<unsigned long long>();
        const uint64_t ntasks = (uint64_t)P.ntiles * (uint64_t)P.ngroups * 64u;
        if (ntasks >= (1ull << 32) - 4096)
            return fail(PT_ERR_INVALID, "sample mode: too many (pixel, block) tasks; raise the block size (chunk)");
        P.ntasks = (uint32_t)ntasks;
        if (PT_XCD_POOLS && ntasks >= (1ull << 28))
            return fail(PT_ERR_INVALID, "sample mode with XCD pools: too many tasks; raise the block size (chunk)");
        if (!f->taskCounter.p && (rc = devAlloc(f->taskCounter, 64))) return rc;
#if PT_XCD_POOLS
        HIP_TRY(hipMemsetAsync(f->taskCounter.p, 0, 32, st));   // the eight XCD counters
#else
        HIP_TRY(hipMemsetAsync(f->taskCounter.p, 0, 4, st));
#endif
        P.taskCounter = f->taskCounter.as<unsigned>();
        int perCU = 0;
        if ((rc = perCUFor(perCU))) return rc;
        const uint64_t full = (uint64_t)f->cus * (uint64_t)std::max(1, perCU);
        P.nwaves = (int)std::min<uint64_t>(full, (ntasks + 63) / 64);
        if (std::getenv("PT_ITER_STATS"))
            std::fprintf(stderr, "[pt] persistent waves %d (%d per CU, stack %d)\n", P.nwaves, perCU, stack);
        // Tile costs (rays of the tile's most expensive pixel) are measured on the first frame and
        // then on one frame in eight: the order only steers the launch's tail, and counting costs
        // one more atomic per task.
        P.measureCost = (lpt && (!f->haveOrder || f->framesSinceCost >= 7)) ? 1 : 0;
        f->framesSinceCost = P.measureCost ? 0 : f->framesSinceCost + 1;
        if (P.measureCost) HIP_TRY(hipMemsetAsync(f->tileCost.p, 0, ntl * 4, st));
    }
    // Deep trees: stack entries beyond kLdsStack live in memory, per wave slot (persistent wave or
    // compat tile) and lane
    if (kernel == PT_KERNEL_WAVEFRONT && stack > PT_LDS_STACK && P.ntiles > 0) {
        const size_t slots = (sample || cq) ? (size_t)P.nwaves : (size_t)P.compatGrid;
        if ((rc = devReserve(f->stackSpill, slots * kWave * (size_t)(stack - PT_LDS_STACK) * 4))) return rc;
        P.stackSpill = f->stackSpill.as<uint32_t>();
    }
    // A resolve pass follows the render kernel in sample mode (block sums) and whenever the film
    // accumulates or the output is 8-bit; compat kernels then store raw sums into f->sums.
    const bool resolve = np > 0 && (sample || accumulate || fmt != PT_OUT_RGB32F);
    if (resolve && !sample) {
        if (!f->sums.p && (rc = devAlloc(f->sums, (size_t)np * 12))) return rc;
        P.out = f->sums.as<float>();
        P.rawOut = 1;
    }
    if (accumulate) {
        if (!f->accum.p) {
            if ((rc = devAlloc(f->accum, (size_t)std::max<int64_t>(1, np) * 12))) return rc;
            HIP_TRY(hipMemsetAsync(f->accum.p, 0, (size_t)std::max<int64_t>(1, np) * 12, st));
            f->accumSamples = 0;
        }
        if (sample) P.sampleBase = (uint32_t)f->accumSamples;   // frames continue the sample sequence
    }
    P.tileCost = f->tileCost.as<unsigned>();
    P.tileOrder = (lpt && f->haveOrder) ? f->tileOrder.as<int>() : nullptr;
    P.tileXY = nullptr;
    P.nblocksShift = -1;
    if (sample || cq) {   // the launch order decoded per slot (tileXYKernel; the ordered table follows each sort)
        if (sample) P.nblocksShift = (P.ngroups & (P.ngroups - 1)) == 0 ? __builtin_ctz((unsigned)P.ngroups) : -1;
        if (!P.tileOrder && !f->haveXYId) {
            tileXYKernel<<<(unsigned)((ntl + 255) / 256), 256, 0, st>>>(nullptr, (int)ntl, P.tiles_x, f->tileXYId.as<uint32_t>());
            HIP_TRY(hipGetLastError());
            f->haveXYId = true;
        }
        P.tileXY = P.tileOrder ? f->tileXY.as<uint32_t>() : f->tileXYId.as<uint32_t>();
    }
    P.prioTiles = (P.tileOrder && !sample && !cq) ? envCount("PT_PRIO_TILES", 1024) : 0;
    P.prioLevel = std::max(1, std::min(3, envCount("PT_PRIO_LEVEL", 2)));
    if (!sample && !cq && kernel != PT_KERNEL_SIMPLE && P.ntiles > 0)   // (tile costs: atomicMax of the tile's waves)
        HIP_TRY(hipMemsetAsync(f->tileCost.p, 0, ntl * 4, st));
    DevBuf dtimes;
    const char* timesPath = std::getenv("PT_WAVE_TIMES");   // diagnostic: per-wave timestamps
    P.waveTimes = nullptr;
    const size_t nwaves = (sample || (cq && kernel != PT_KERNEL_SIMPLE)) ? (size_t)P.nwaves
                        : (kernel != PT_KERNEL_SIMPLE ? (size_t)std::max(1, P.compatGrid) : ntl);   // = grid size
    if (timesPath && *timesPath && kernel != PT_KERNEL_SIMPLE) {
        if ((rc = devAlloc(dtimes, nwaves * 24))) return rc;
        HIP_TRY(hipMemsetAsync(dtimes.p, 0, nwaves * 24, st));
        P.waveTimes = dtimes.as<unsigned long long>();
    }
    // From here on the film describes this render (pt_film_stats reads it).
    f->rendered = false;
    f->lastWide = kernel == PT_KERNEL_WIDE;
    HIP_TRY(hipEventRecord(f->ev0, st));
    if (P.ntiles > 0 && (rc = dispatchRender(stack, P, st))) return rc;
    if (resolve) {
        const float inv = accumulate ? 1.0f / (float)(f->accumSamples + spp) : P.invSpp;
        resolveKernel<<<(unsigned)((np + 255) / 256), 256, 0, st>>>(f->sums.as<float>(), sample ? P.pixAcc : nullptr,
                                                                     accumulate ? f->accum.as<float>() : nullptr,
                                                                     inv, fmt, dst, np,
                                                                     P.measureCost ? f->tileCost.as<unsigned>() : nullptr,
                                                                     f->width, P.tiles_x, envInt("PT_TILE_KEY_MAX", 1));
        HIP_TRY(hipGetLastError());
    }
    if (accumulate) f->accumSamples += spp;
    HIP_TRY(hipEventRecord(f->ev1, st));
    // the counters to pinned host memory, in stream order (pt_film_stats waits for ev2 only)
    HIP_TRY(hipMemcpyAsync(f->hostCounters, f->counters.p, kNumCounters * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(f->ev2, st));
    f->rendered = true;
    if (lpt && P.ntiles > 0 && (!sample || P.measureCost)) {   // next launches: longest tiles first (a stable radix sort, on the device)
        const int nt = (int)ntl;
        if ((rc = devReserve(f->tileKeys, ntl * 4)) || (rc = devReserve(f->tileKeys2, ntl * 4)) ||
            (rc = devReserve(f->tileIds, ntl * 4)))
            return rc;
        size_t tbytes = 0;
        HIP_TRY(pt::radixSortPairs(nullptr, &tbytes, f->tileKeys.as<uint32_t>(), f->tileKeys2.as<uint32_t>(),
                                   f->tileIds.as<uint32_t>(), f->tileOrder.as<uint32_t>(), ntl, 32, st));
        if ((rc = devReserve(f->sortTemp, tbytes))) return rc;
        tileKeyKernel<<<(unsigned)((nt + 255) / 256), 256, 0, st>>>(f->tileCost.as<unsigned>(), f->tileKeys.as<uint32_t>(),
                                                                    f->tileIds.as<uint32_t>(), nt);
        HIP_TRY(hipGetLastError());
        HIP_TRY(pt::radixSortPairs(f->sortTemp.p, &tbytes, f->tileKeys.as<uint32_t>(), f->tileKeys2.as<uint32_t>(),
                                   f->tileIds.as<uint32_t>(), f->tileOrder.as<uint32_t>(), ntl, 32, st));
        tileXYKernel<<<(unsigned)((nt + 255) / 256), 256, 0, st>>>(f->tileOrder.as<uint32_t>(), nt, P.tiles_x,
                                                                   f->tileXY.as<uint32_t>());
        HIP_TRY(hipGetLastError());
        f->haveOrder = true;
        if (std::getenv("PT_CHECK_ORDER")) {   // diagnostic: the launch order must be a permutation of the tiles
            std::vector<uint32_t> ord(ntl), cst(ntl);
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipMemcpy(ord.data(), f->tileOrder.p, ntl * 4, hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(cst.data(), f->tileCost.p, ntl * 4, hipMemcpyDeviceToHost));
            std::vector<uint8_t> seen(ntl, 0);
            size_t dup = 0, bad = 0, unsorted = 0;
            for (size_t k = 0; k < ntl; k++) {
                if (ord[k] >= ntl) { bad++; continue; }
                if (seen[ord[k]]++) dup++;
                if (k && ord[k - 1] < ntl && cst[ord[k - 1]] < cst[ord[k]]) unsorted++;
            }
            std::fprintf(stderr, "[pt] tile order check: %zu tiles, %zu out of range, %zu duplicates, %zu unsorted pairs\n",
                         ntl, bad, dup, unsorted);
        }
    }
    if (critOn) {   // the next launch's critical pixels: the K longest chains of this one (a stable radix sort)
        const int64_t K = std::min<int64_t>(envCount("PT_CRIT_PIXELS", kCritPixels), np);
        const size_t n = (size_t)np;
        if ((rc = devReserve(f->pixKeys, n * 4)) || (rc = devReserve(f->pixKeys2, n * 4)) ||
            (rc = devReserve(f->pixIds, n * 4)) || (rc = devReserve(f->pixSorted, n * 4)) ||
            (rc = devReserve(f->critFlag, n)))
            return rc;
        size_t cbytes = 0;
        HIP_TRY(pt::radixSortPairs(nullptr, &cbytes, f->pixKeys.as<uint32_t>(), f->pixKeys2.as<uint32_t>(),
                                   f->pixIds.as<uint32_t>(), f->pixSorted.as<uint32_t>(), n, 32, st));
        if ((rc = devReserve(f->critTemp, cbytes))) return rc;
        tileKeyKernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(f->pixRays.as<unsigned>(), f->pixKeys.as<uint32_t>(),
                                                                  f->pixIds.as<uint32_t>(), (int)n);
        HIP_TRY(hipGetLastError());
        HIP_TRY(pt::radixSortPairs(f->critTemp.p, &cbytes, f->pixKeys.as<uint32_t>(), f->pixKeys2.as<uint32_t>(),
                                   f->pixIds.as<uint32_t>(), f->pixSorted.as<uint32_t>(), n, 32, st));
        HIP_TRY(hipMemsetAsync(f->critFlag.p, 0, n, st));
        critFlagKernel<<<(unsigned)((K + 255) / 256), 256, 0, st>>>(f->pixSorted.as<uint32_t>(), (int)K,
                                                                   f->critFlag.as<uint8_t>());
        HIP_TRY(hipGetLastError());
        f->critK = (int)K;
    }
    if (P.waveTimes) {
        HIP_TRY(hipStreamSynchronize(st));
        std::vector<unsigned long long> t(nwaves * 3);
        HIP_TRY(hipMemcpy(t.data(), dtimes.p, t.size() * 8, hipMemcpyDeviceToHost));
        if (FILE* fp = std::fopen(timesPath, "wb")) {
            std::fwrite(t.data(), 8, t.size(), fp);
            std::fclose(fp);
        }
    }
    if (!on_dev && np > 0) HIP_TRY(hipMemcpy(out, dst, np * outBpp, hipMemcpyDeviceToHost));
    // With stats (or a host output) the call waits for the frame; without, it returns at once.
    if (stats || !on_dev) return filmStats(f, stats);
    return PT_OK;
}

int pt_film_stats(pt_film* f, pt_stats* stats) {
    if (!f || !stats) return fail(PT_ERR_INVALID, "pt_film_stats: null argument");
    int rc = setDevice(f->device);
    if (rc) return rc;
    return filmStats(f, stats);
}

void pt_film_destroy(pt_film* f) {
    if (!f) return;
    (void)hipSetDevice(f->device);
    delete f;
}

void pt_scene_destroy(pt_scene* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    delete s;
}

}  // extern "C"
#endif  // PT_TU_COMPAT
