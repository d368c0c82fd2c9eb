// sort_check.hip — the build path's hand-written device primitives (csrc/pt_sort.hip) against
// host references (tests/test_gpu_math.py):
//   * radixSortPairs == std::stable_sort by the low `bits` bits of the key (values carried), for
//     sizes around the 1024-pair tile and the 2048 / 1024-item scan tiles, up to 2^22 pairs, with
//     heavy duplicates (Morton codes of coincident centroids), all-equal keys and 30 / 32 / 8 bits;
//   * exclusiveScanU32 / exclusiveScanU3 == the sequential exclusive sums (uint32 wrap-around),
//     including sizes that span many tiles (the decoupled look-back).
// Prints one line per case and "ok" at the end; exit status 1 on the first mismatch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#include "../../path-tracer-cuda-opengl_amd/csrc/pt_prims.hpp"

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(2);                                                               \
        }                                                                               \
    } while (0)

static bool sortCase(size_t n, int bits, int dupMode, std::mt19937& rng) {
    std::vector<uint32_t> k(n), v(n);
    const uint32_t mask = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u);
    for (size_t i = 0; i < n; i++) {
        uint32_t x = rng();
        if (dupMode == 1) x = (x % 97u) * 0x01010101u;   // many duplicates
        if (dupMode == 2) x = 0x2aaaaaau;                 // all equal
        k[i] = x;                                         // high bits beyond `bits` are ignored by the sort
        v[i] = (uint32_t)i;
    }
    std::vector<size_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return (k[a] & mask) < (k[b] & mask); });
    uint32_t *dk, *dv, *ok, *ov;
    const size_t bytes = std::max<size_t>(n, 1) * 4;
    CK(hipMalloc(&dk, bytes)); CK(hipMalloc(&dv, bytes)); CK(hipMalloc(&ok, bytes)); CK(hipMalloc(&ov, bytes));
    CK(hipMemcpy(dk, k.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, v.data(), n * 4, hipMemcpyHostToDevice));
    size_t tb = 0;
    CK(pt::radixSortPairs(nullptr, &tb, dk, ok, dv, ov, n, bits, 0));
    void* tmp;
    CK(hipMalloc(&tmp, tb));
    CK(pt::radixSortPairs(tmp, &tb, dk, ok, dv, ov, n, bits, 0));
    std::vector<uint32_t> rk(n), rv(n), ik(n);
    CK(hipMemcpy(rk.data(), ok, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rv.data(), ov, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ik.data(), dk, n * 4, hipMemcpyDeviceToHost));
    bool good = ik == k;   // inputs untouched
    for (size_t i = 0; i < n && good; i++) good = rk[i] == k[idx[i]] && rv[i] == (uint32_t)idx[i];
    std::printf("sort n=%zu bits=%d dup=%d: %s\n", n, bits, dupMode, good ? "ok" : "MISMATCH");
    CK(hipFree(dk)); CK(hipFree(dv)); CK(hipFree(ok)); CK(hipFree(ov)); CK(hipFree(tmp));
    return good;
}

static bool scanCase(size_t n, std::mt19937& rng) {
    std::vector<uint32_t> a(n);
    std::vector<uint4> b(n);
    for (size_t i = 0; i < n; i++) {
        a[i] = (i % 5 == 0) ? rng() : rng() % 4u;   // includes wrap-around
        b[i] = make_uint4(rng() % 9u, rng() % 3u, rng(), rng());
    }
    uint32_t *da, *oa;
    uint4 *db, *ob;
    const size_t na = std::max<size_t>(n, 1);
    CK(hipMalloc(&da, na * 4)); CK(hipMalloc(&oa, na * 4)); CK(hipMalloc(&db, na * 16)); CK(hipMalloc(&ob, na * 16));
    CK(hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, b.data(), n * 16, hipMemcpyHostToDevice));
    void* tmp;
    CK(hipMalloc(&tmp, std::max(pt::scanScratchBytesU32(n), pt::scanScratchBytesU3(n))));
    CK(pt::exclusiveScanU32(tmp, da, oa, n, 0));
    CK(pt::exclusiveScanU3(tmp, db, ob, n, 0));
    std::vector<uint32_t> ra(n);
    std::vector<uint4> rb(n);
    CK(hipMemcpy(ra.data(), oa, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rb.data(), ob, n * 16, hipMemcpyDeviceToHost));
    bool good = true;
    uint32_t s = 0;
    uint4 t = make_uint4(0, 0, 0, 0);
    for (size_t i = 0; i < n && good; i++) {
        good = ra[i] == s && rb[i].x == t.x && rb[i].y == t.y && rb[i].z == t.z && rb[i].w == 0u;
        s += a[i];
        t = make_uint4(t.x + b[i].x, t.y + b[i].y, t.z + b[i].z, 0u);
    }
    std::printf("scan n=%zu: %s\n", n, good ? "ok" : "MISMATCH");
    CK(hipFree(da)); CK(hipFree(oa)); CK(hipFree(db)); CK(hipFree(ob)); CK(hipFree(tmp));
    return good;
}

int main() {
    std::mt19937 rng(12345);
    bool ok = true;
    for (size_t n : {(size_t)0, (size_t)1, (size_t)2, (size_t)63, (size_t)64, (size_t)65, (size_t)1023, (size_t)1024,
                     (size_t)1025, (size_t)5000, (size_t)65553, (size_t)1043312})
        for (int dup : {0, 1}) ok = ok && sortCase(n, 30, dup, rng);
    ok = ok && sortCase(100000, 32, 0, rng) && sortCase(33000, 32, 1, rng) && sortCase(7777, 8, 0, rng) &&
         sortCase(4096 + 3, 30, 2, rng) && sortCase((size_t)1 << 22, 30, 1, rng);
    for (size_t n : {(size_t)0, (size_t)1, (size_t)255, (size_t)256, (size_t)1023, (size_t)1024, (size_t)1025,
                     (size_t)2047, (size_t)2048, (size_t)2049, (size_t)100000, (size_t)1043312, (size_t)1 << 23})
        ok = ok && scanCase(n, rng);
    if (!ok) return 1;
    std::printf("ok\n");
    return 0;
}
