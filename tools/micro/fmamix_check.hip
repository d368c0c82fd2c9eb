// Micro-check for the wide NODE step's plane distances: a quantised plane byte q
// placed in the low byte of an fp16 (0x00qq = q * 2^-24, an fp16 denormal, built by v_perm_b32
// with the zero-byte selector) and fed to v_fma_mix_f32 with the scale multiplied by 2^24 gives
// fma(q * 2^-24, a * 2^24, c) == fma((float)q, a, c) exactly whenever a * 2^24 is finite (both are
// the same exact product-sum, rounded once) -- provided the f16 input is not flushed.
//  1. exactness: every q in 0..255 against 2^22 random (a, c) pairs per q (a over all exponents
//     that keep a * 2^24 finite), mismatches counted;
//  2. throughput: independent v_fma_mix_f32 vs v_cvt_f32_ubyte + v_fma_f32 chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "pt_math.hpp"   // planePairLo / planePairHi / fmaMixLo / fmaMixHi: the kernels' own helpers

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void exact(unsigned long long* bad, uint32_t* example) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long n = 0;
    for (uint32_t it = 0; it < 64; it++) {
        const uint32_t r0 = hash(gid * 131u + it * 7u + 1u), r1 = hash(r0 ^ 0x9e3779b9u), r2 = hash(r1 + 17u);
        // a: random sign / mantissa, exponent 1..229 (a * 2^24 finite); c: any finite
        const uint32_t ea = 1u + (r1 >> 8) % 229u, ec = 1u + (r2 >> 8) % 254u;
        const float a = __uint_as_float((r1 & 0x807fffffu) | (ea << 23));
        const float c = __uint_as_float((r2 & 0x807fffffu) | (ec << 23));
        const float aS = a * 16777216.0f;   // exact: a power-of-two scale, finite by the exponent bound
        const uint32_t x = r0;              // four plane bytes
        const uint32_t p01 = planePairLo(x);   // bytes 0, 1 -> fp16 lo / hi
        const uint32_t p23 = planePairHi(x);
        const float m0 = fmaMixLo(p01, aS, c), m1 = fmaMixHi(p01, aS, c);
        const float m2 = fmaMixLo(p23, aS, c), m3 = fmaMixHi(p23, aS, c);
        const float f0 = __builtin_fmaf((float)(x & 0xffu), a, c), f1 = __builtin_fmaf((float)((x >> 8) & 0xffu), a, c);
        const float f2 = __builtin_fmaf((float)((x >> 16) & 0xffu), a, c), f3 = __builtin_fmaf((float)(x >> 24), a, c);
        const bool e = __float_as_uint(m0) != __float_as_uint(f0) || __float_as_uint(m1) != __float_as_uint(f1) ||
                       __float_as_uint(m2) != __float_as_uint(f2) || __float_as_uint(m3) != __float_as_uint(f3);
        if (e) {
            n++;
            if (atomicCAS(example, 0u, 1u) == 0u) { example[1] = x; example[2] = __float_as_uint(a); example[3] = __float_as_uint(c); }
        }
    }
    if (n) atomicAdd(bad, n);
}

// every byte value explicitly, with a few scales around the denormal / overflow edges
__global__ void everyByte(unsigned long long* bad) {
    const uint32_t q = threadIdx.x;   // 0..255
    const float as[6] = {1.0f, -3.0e-30f, 7.5e25f, 1.1754944e-38f, -0.3f, 1.0e31f};
    const float cs[4] = {0.0f, -1.0f, 3.4e38f, 1.0e-40f};
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 4; j++) {
            const uint32_t h = planePairLo(q * 0x01010101u);
            const float m0 = fmaMixLo(h, as[i] * 16777216.0f, cs[j]), m1 = fmaMixHi(h, as[i] * 16777216.0f, cs[j]);
            const float f = __builtin_fmaf((float)q, as[i], cs[j]);
            if (__float_as_uint(m0) != __float_as_uint(f) && !(m0 != m0 && f != f)) atomicAdd(bad, 1ull);
            if (__float_as_uint(m1) != __float_as_uint(f) && !(m1 != m1 && f != f)) atomicAdd(bad, 1ull);
        }
}

template <bool MIX>
__global__ void rate(const uint32_t* in, float* out, int iters) {
    uint32_t x0 = in[threadIdx.x], x1 = x0 * 3u, x2 = x0 * 5u, x3 = x0 * 7u;
    float a = __uint_as_float(0x3f800000u | (x0 & 0xfffu)), c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
    for (int i = 0; i < iters; i++) {
        if (MIX) {
            const uint32_t p0 = planePairLo(x0), p1 = planePairLo(x1), p2 = planePairLo(x2), p3 = planePairLo(x3);
            c0 = fmaMixLo(p0, a, c0); c1 = fmaMixHi(p0, a, c1); c2 = fmaMixLo(p1, a, c2); c3 = fmaMixHi(p1, a, c3);
            c4 = fmaMixLo(p2, a, c4); c5 = fmaMixHi(p2, a, c5); c6 = fmaMixLo(p3, a, c6); c7 = fmaMixHi(p3, a, c7);
        } else {
            c0 = __builtin_fmaf((float)(x0 & 0xffu), a, c0); c1 = __builtin_fmaf((float)((x0 >> 8) & 0xffu), a, c1);
            c2 = __builtin_fmaf((float)(x1 & 0xffu), a, c2); c3 = __builtin_fmaf((float)((x1 >> 8) & 0xffu), a, c3);
            c4 = __builtin_fmaf((float)(x2 & 0xffu), a, c4); c5 = __builtin_fmaf((float)((x2 >> 8) & 0xffu), a, c5);
            c6 = __builtin_fmaf((float)(x3 & 0xffu), a, c6); c7 = __builtin_fmaf((float)((x3 >> 8) & 0xffu), a, c7);
        }
        x0 = x0 * 1664525u + 1013904223u;  // (keeps the bytes changing: 1 quarter-rate op per 8 planes, both variants)
        x1 ^= x0; x2 += x0; x3 ^= x2;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

#define CK(x) (void)(x)
int main() {
    unsigned long long* bad;
    uint32_t* ex;
    CK(hipMalloc(&bad, 16));
    CK(hipMalloc(&ex, 16));
    CK(hipMemset(bad, 0, 16));
    CK(hipMemset(ex, 0, 16));
    exact<<<65536, 256>>>(bad, ex);   // 2^24 threads x 64 draws x 4 bytes
    everyByte<<<1, 256>>>(bad + 1);
    unsigned long long h[2];
    uint32_t e[4];
    CK(hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(e, ex, 16, hipMemcpyDeviceToHost));
    std::printf("{\"random_tests\": %llu, \"random_mismatches\": %llu, \"edge_mismatches\": %llu", 65536ull * 256 * 64 * 4, h[0], h[1]);
    if (h[0]) std::printf(", \"example\": [%u, %u, %u]", e[1], e[2], e[3]);
    uint32_t* in;
    float* out;
    CK(hipMalloc(&in, 4096));
    CK(hipMemset(in, 1, 4096));
    CK(hipMalloc(&out, 4u * 256 * 4 * 2048));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms[2];
    for (int v = 0; v < 2; v++) {
        for (int rep = 0; rep < 2; rep++) {
            CK(hipEventRecord(a));
            if (v) rate<true><<<256 * 4 * 8, 64>>>(in, out, 4096);
            else rate<false><<<256 * 4 * 8, 64>>>(in, out, 4096);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms[v], a, b));
        }
    }
    std::printf(", \"cvt_fma_ms\": %.3f, \"perm_fmamix_ms\": %.3f}\n", ms[0], ms[1]);
    return h[0] || h[1] ? 1 : 0;
}
