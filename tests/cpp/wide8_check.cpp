// CPU check of the wide-tree builder (host/pt_wide8.cpp) and of the traversal rule the wide
// kernels run (TEST INFRASTRUCTURE: compiled and run by tests/test_wide_builder.py; the product
// never uses it).  Reads objects and rays, builds the binary LBVH with the oracle (oracle/), the
// reference ranks and the wide tree exactly as libpt does, then
//   1. checks the tree: every primitive once, child boxes contain the exact primitive boxes
//      with at least the tree's smallest quantum 2^emin to spare on every side (the outward margin
//      the traversal's rounding bound needs, pt_device.hip wideHits), node/primitive encodings in
//      range;
//   2. traces every ray through a scalar restatement of renderKernelWF<.., WIDE>'s NODE / LEAF
//      steps (nearest-first slots, conservative quantised slab test, (t, tie rank) minimum,
//      the reference's leaf box test, the redo rule) and writes {leaf k or -1, t, redo} per ray.
// usage: wide8_check objects.bin rays.bin out.bin
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pt.h"
#include "pt_wide8.hpp"

extern "C" {
typedef struct { int32_t left, right, parent, objid; float bmin[3], bmax[3]; } orc_node;
int orc_morton_keys(const pt_object* objs, int64_t n, int include_origin, uint64_t* keys_out);
int orc_build_lbvh(const pt_object* objs, int64_t n, const uint64_t* keys, int tight, orc_node* nodes);
}

namespace {
float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
struct V { float x, y, z; };
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V cross(V u, V v) { return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x}; }
float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
const uint32_t* P;
const uint32_t* N;

// primHitAny (pt_device.hip): the sphere's first root >= tmin, else the second; triangles as the
// reference (cuda_object.h:44-92) without the closest-hit bound
float primT(int i, V o, V d, float tmin) {
    const uint32_t* r = P + 12 * i;
    if (r[11] != 0) {
        V c{u2f(r[0]), u2f(r[1]), u2f(r[2])};
        const float rad = u2f(r[4]);
        V oc = sub(o, c);
        const float a = dot(d, d), hb = dot(oc, d), cc = dot(oc, oc) - rad * rad, disc = hb * hb - a * cc;
        if (disc < 0) return -1;
        const float sq = std::sqrt(disc);
        float root = (-hb - sq) / a;
        if (!(root < tmin)) return root;
        root = (-hb + sq) / a;
        if (!(root < tmin)) return root;
        return -1;
    }
    V v0{u2f(r[0]), u2f(r[1]), u2f(r[2])}, v1{u2f(r[4]), u2f(r[5]), u2f(r[6])}, v2{u2f(r[8]), u2f(r[9]), u2f(r[10])};
    V e1 = sub(v1, v0), e2 = sub(v2, v0), s1 = cross(d, e2);
    const float det = dot(s1, e1);
    if (det == 0) return -1;
    V s = sub(o, v0), s2 = cross(s, e1);
    const float inv = 1.0f / det, t = dot(s2, e2) * inv, b1 = dot(s1, s) * inv, b2 = dot(s2, d) * inv;
    if (b1 >= 1 || b1 <= 0 || b2 >= 1 || b2 <= 0 || b1 + b2 <= 0 || b1 + b2 >= 1 || t <= tmin) return -1;
    return t;
}
// the reference's leaf box test (aabb.h:21-34) with tmax = +inf: {passes, entry lo}
bool leafBox(int i, V o, V inv, float tmin, float& lo) {
    const uint32_t* r = P + 12 * i;
    float mn[3], mx[3];
    if (r[11] != 0) {
        const float rr = std::fabs(u2f(r[4]));
        for (int a = 0; a < 3; a++) { mn[a] = u2f(r[a]) - rr; mx[a] = u2f(r[a]) + rr; }
    } else {
        for (int a = 0; a < 3; a++) {
            mn[a] = std::fmin(std::fmin(u2f(r[a]), u2f(r[4 + a])), u2f(r[8 + a]));
            mx[a] = std::fmax(std::fmax(u2f(r[a]), u2f(r[4 + a])), u2f(r[8 + a]));
        }
    }
    const float ov[3] = {o.x, o.y, o.z}, iv[3] = {inv.x, inv.y, inv.z};
    float l = tmin, h = INFINITY;
    for (int a = 0; a < 3; a++) {
        float t0 = (mn[a] - ov[a]) * iv[a], t1 = (mx[a] - ov[a]) * iv[a];
        if (iv[a] < 0) std::swap(t0, t1);
        l = t0 > l ? t0 : l;
        h = t1 < h ? t1 : h;
    }
    lo = l;
    return !(h < l);
}
// renderKernelWF<.., WIDE>'s traversal for one ray; returns the best rank (-1), sets redo
int traceWide(V o, V d, float tmin, float& closest, bool single, bool& redo) {
    const V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    const uint32_t oct = (inv.x < 0 ? 1u : 0u) | (inv.y < 0 ? 2u : 0u) | (inv.z < 0 ? 4u : 0u);
    uint32_t ng = 1u << oct, tgBase = 0, tg = 0, stk[64];
    int sp = 0, best = -1;
    bool bestSph = false;
    float bestLo = -INFINITY;
    closest = INFINITY;
    redo = false;
    for (;;) {
        while (tg) {
            const int i = (int)(tgBase + (uint32_t)__builtin_ctz(tg));
            tg &= tg - 1u;
            const float t = primT(i, o, d, tmin);
            if (!(t >= 0)) continue;
            const uint32_t* r = P + 12 * i;
            const int k = (int)r[3];
            const bool sph = r[11] != 0, none = best < 0;
            const bool tie = sph ? (none || !bestSph || k > best) : (!none && !bestSph && k < best);
            if (t >= closest && t < bestLo) redo = true;
            if (t < closest || (t == closest && tie)) {
                bool take = true;
                float lo2 = -INFINITY;
                if (!single) {
                    float lo;
                    const bool h = leafBox(i, o, inv, tmin, lo);
                    take = h && !(closest < lo);
                    if (h && closest < lo) redo = true;
                    if (t < lo) lo2 = lo;
                }
                if (take) { closest = t; best = k; bestSph = sph; bestLo = lo2; }
            }
        }
        if ((ng & 0xffu) == 0) {
            if (sp == 0) break;
            ng = stk[--sp];
        }
        const uint32_t bit = (uint32_t)__builtin_ctz(ng & 0xffu);
        const uint32_t child = (ng >> 8) + (bit ^ oct);
        ng &= ~(1u << bit);
        if (ng & 0xffu) stk[sp++] = ng;
        const uint32_t* R = N + 20 * child;
        float a[3], b[3];
        const float ov[3] = {o.x, o.y, o.z}, iv[3] = {inv.x, inv.y, inv.z};
        for (int ax = 0; ax < 3; ax++) {
            a[ax] = u2f(((R[3] >> (8 * ax)) & 0xffu) << 23) * iv[ax];
            b[ax] = (u2f(R[ax]) - ov[ax]) * iv[ax];
        }
        uint32_t hits = 0;
        for (int j = 0; j < 8; j++) {
            const uint32_t meta = ((j < 4 ? R[6] : R[7]) >> (8 * (j & 3))) & 0xffu;
            float lo = tmin, hi = closest;
            for (int ax = 0; ax < 3; ax++) {
                const uint32_t ql = (R[8 + 4 * ax + (j >> 2)] >> (8 * (j & 3))) & 0xffu;
                const uint32_t qh = (R[10 + 4 * ax + (j >> 2)] >> (8 * (j & 3))) & 0xffu;
                const uint32_t qn = iv[ax] < 0 ? qh : ql, qf = iv[ax] < 0 ? ql : qh;
                lo = std::fmax(lo, std::fma((float)qn, a[ax], b[ax]));
                hi = std::fmin(hi, std::fma((float)qf, a[ax], b[ax]));
            }
            if (lo <= hi && meta) {
                uint32_t bi = meta & 31u;
                if ((meta & 0x18u) == 0x18u) bi = 24u + ((bi - 24u) ^ oct);
                hits |= (meta >> 5) << bi;
            }
        }
        ng = (R[4] << 8) | (hits >> 24);
        tgBase = R[5];
        tg = hits & 0xffffffu;
    }
    return best;
}
template <class T>
std::vector<T> readAll(const char* path) {
    std::vector<T> v;
    FILE* f = std::fopen(path, "rb");
    if (!f) return v;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    v.resize((size_t)n / sizeof(T));
    if (std::fread(v.data(), 1, (size_t)n, f) != (size_t)n) v.clear();
    std::fclose(f);
    return v;
}
int failures = 0;
void check(bool ok, const std::string& what) {
    if (!ok && failures++ < 10) std::fprintf(stderr, "CHECK FAILED: %s\n", what.c_str());
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const std::vector<pt_object> objs = readAll<pt_object>(argv[1]);
    const std::vector<float> rays = readAll<float>(argv[2]);
    const int64_t n = (int64_t)objs.size(), nr = (int64_t)rays.size() / 6;
    if (n < 1) return 2;
    std::vector<uint64_t> keys((size_t)n);
    orc_morton_keys(objs.data(), n, 1, keys.data());
    std::vector<orc_node> nd((size_t)(2 * n - 1));
    orc_build_lbvh(objs.data(), n, keys.data(), 1, nd.data());
    // leaf-order primitive records and boxes, as the device's leafGatherKernel writes them
    std::vector<uint32_t> prims((size_t)n * 12, 0u);
    std::vector<float> boxes((size_t)n * 6);
    for (int64_t k = 0; k < n; k++) {
        const pt_object& o = objs[keys[k] & 0xffffffffu];
        uint32_t* r = &prims[(size_t)k * 12];
        float* f = reinterpret_cast<float*>(r);
        float* b = &boxes[(size_t)k * 6];
        r[3] = (uint32_t)o.mat;
        r[7] = (uint32_t)(keys[k] & 0xffffffffu);
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
    // reference ranks from the binary tree's child refs (leaf bit 31, leaf k in the low bits)
    std::vector<uint32_t> lref((size_t)std::max<int64_t>(1, n - 1)), rref(lref.size());
    for (int64_t i = 0; i + 1 < n; i++) {
        auto ref = [&](int32_t c) { return c >= n - 1 ? (0x80000000u | (uint32_t)(c - (n - 1))) : (uint32_t)c; };
        lref[(size_t)i] = ref(nd[(size_t)i].left);
        rref[(size_t)i] = ref(nd[(size_t)i].right);
    }
    const std::vector<uint32_t> rank = pt::referenceRanks(lref.data(), rref.data(), 1, n);
    pt::Wide8 w;
    std::string err;
    if (!pt::buildWide8(prims.data(), boxes.data(), rank.data(), n, w, err)) {
        std::fprintf(stderr, "build failed: %s\n", err.c_str());
        return 1;
    }
    P = w.prims.data();
    N = w.nodes.data();
    // 1. structure.  The smallest quantum, as the builder takes it: 2^-18 of the larger of the
    // scene's extent and coordinates (rounded up to a power of two)
    double ext = 0.0;
    {
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int64_t k = 0; k < n; k++)
            for (int a = 0; a < 3; a++) {
                mn[a] = std::fmin(mn[a], (double)boxes[(size_t)k * 6 + a]);
                mx[a] = std::fmax(mx[a], (double)boxes[(size_t)k * 6 + 3 + a]);
            }
        for (int a = 0; a < 3; a++) ext = std::fmax(ext, std::fmax(std::fmax(std::fabs(mn[a]), std::fabs(mx[a])), mx[a] - mn[a]));
    }
    const int emin = ext > 0.0 ? std::max(-100, (int)std::ceil(std::log2(ext)) - 18) : -100;
    const double minQuantum = std::ldexp(1.0, emin);
    std::vector<int> seen((size_t)n, 0);
    std::vector<int> kOfRank((size_t)n, -1);
    for (int64_t k = 0; k < n; k++) kOfRank[rank[k]] = (int)k;
    for (int64_t i = 0; i < n; i++) {
        const uint32_t rk = w.prims[(size_t)i * 12 + 3];
        check(rk < (uint32_t)n, "rank in range");
        if (rk < (uint32_t)n) seen[rk]++;
    }
    for (int64_t k = 0; k < n; k++) check(seen[k] == 1, "every primitive exactly once");
    const int64_t slots = (int64_t)(w.nodes.size() / 20);
    int64_t reached = 0;
    std::vector<int64_t> todo{0};
    while (!todo.empty()) {
        const int64_t s = todo.back();
        todo.pop_back();
        reached++;
        const uint32_t* R = &w.nodes[(size_t)s * 20];
        for (int j = 0; j < 8; j++) {
            const uint32_t meta = ((j < 4 ? R[6] : R[7]) >> (8 * (j & 3))) & 0xffu;
            if (!meta) continue;
            double lo[3], hi[3];   // exact child planes
            for (int a = 0; a < 3; a++) {
                const double sc = std::ldexp(1.0, (int)((R[3] >> (8 * a)) & 0xffu) - 127);
                const uint32_t ql = (R[8 + 4 * a + (j >> 2)] >> (8 * (j & 3))) & 0xffu;
                const uint32_t qh = (R[10 + 4 * a + (j >> 2)] >> (8 * (j & 3))) & 0xffu;
                lo[a] = (double)u2f(R[a]) + ql * sc;
                hi[a] = (double)u2f(R[a]) + qh * sc;
            }
            auto contains = [&](int64_t prim) {
                const int64_t k = kOfRank[w.prims[(size_t)prim * 12 + 3]];
                for (int a = 0; a < 3; a++)
                    if (!(lo[a] <= (double)boxes[(size_t)k * 6 + a] - minQuantum &&
                          hi[a] >= (double)boxes[(size_t)k * 6 + 3 + a] + minQuantum))
                        return false;
                return true;
            };
            if ((meta & 0x18u) == 0x18u) {
                const int64_t c = (int64_t)R[4] + (meta & 7u);
                check(c < slots && (meta & 7u) == (uint32_t)j, "child slot in range");
                if (c < slots) todo.push_back(c);
                // every primitive below the child lies strictly inside its planes
                std::vector<int64_t> sub{c};
                while (!sub.empty()) {
                    const int64_t x = sub.back();
                    sub.pop_back();
                    const uint32_t* X = &w.nodes[(size_t)x * 20];
                    for (int jj = 0; jj < 8; jj++) {
                        const uint32_t m = ((jj < 4 ? X[6] : X[7]) >> (8 * (jj & 3))) & 0xffu;
                        if (!m) continue;
                        if ((m & 0x18u) == 0x18u) sub.push_back((int64_t)X[4] + (m & 7u));
                        else
                            for (uint32_t q = 0; q < 3 && ((m >> 5) >> q & 1u); q++)
                                check(contains((int64_t)X[5] + (m & 31u) + q), "subtree primitive inside child box");
                    }
                }
            } else {
                const uint32_t cnt = (meta >> 5) == 1u ? 1u : ((meta >> 5) == 3u ? 2u : 3u);
                check((meta >> 5) == 1u || (meta >> 5) == 3u || (meta >> 5) == 7u, "unary leaf count");
                check((meta & 31u) + cnt <= 24u, "leaf offset < 24");
                for (uint32_t q = 0; q < cnt; q++) check(contains((int64_t)R[5] + (meta & 31u) + q), "leaf inside box");
            }
        }
    }
    check(reached == w.usedNodes, "every used node reachable once");
    // 2. traversal
    std::vector<float> out((size_t)nr * 3);
    for (int64_t i = 0; i < nr; i++) {
        const float* r = &rays[(size_t)i * 6];
        float t = 0;
        bool redo = false;
        const int b = traceWide(V{r[0], r[1], r[2]}, V{r[3], r[4], r[5]}, 0.001f, t, n == 1, redo);
        out[(size_t)i * 3 + 0] = (float)(b < 0 ? -1 : kOfRank[(size_t)b]);
        out[(size_t)i * 3 + 1] = t;
        out[(size_t)i * 3 + 2] = redo ? 1.0f : 0.0f;
    }
    FILE* f = std::fopen(argv[3], "wb");
    if (!f) return 2;
    std::fwrite(out.data(), 4, out.size(), f);
    std::fclose(f);
    std::printf("nodes %lld used %lld depth %d leaves %lld failures %d\n", (long long)slots, (long long)w.usedNodes,
                w.depth, (long long)w.leaves, failures);
    return failures ? 1 : 0;
}
