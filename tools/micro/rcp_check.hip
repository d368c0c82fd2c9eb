// Exhaustive check of the render kernels' reciprocal (csrc/pt_math.hpp) against the IEEE
// division 1.0f / x over all 2^32 fp32 bit patterns, and of the XORWOW draw mappings against
// their two-operation forms over all 2^32 draws, on the GPU, with the kernels' own compiler
// flags.  Prints one JSON line: mismatches of the bare Newton step per biased exponent of x, and
// the total mismatches of rcpRN (must be 0: the guard sends every exponent outside the fast range
// to the division).  NaN results compare equal when both are NaN.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "pt_math.hpp"

__global__ __launch_bounds__(256) void check(uint64_t base, unsigned long long* expMis, unsigned long long* rnMis) {
    __shared__ unsigned long long local[256];
    __shared__ unsigned long long localRn;
    for (int i = threadIdx.x; i < 256; i += 256) local[i] = 0ull;
    if (threadIdx.x == 0) localRn = 0ull;
    __syncthreads();
    // each thread: 16 consecutive patterns
    const uint64_t first = base + ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 16u;
    unsigned long long rn = 0ull;
    for (int k = 0; k < 16; k++) {
        const uint32_t bits = (uint32_t)(first + (uint64_t)k);
        const float x = __uint_as_float(bits);
        const float ref = 1.0f / x;
        const float a = rcpNewton(x), b = rcpRN(x);
        const bool refNan = ref != ref;
        const bool badA = refNan ? (a == a) : (__float_as_uint(a) != __float_as_uint(ref));
        const bool badB = refNan ? (b == b) : (__float_as_uint(b) != __float_as_uint(ref));
        if (badA) atomicAdd(&local[(bits >> 23) & 0xffu], 1ull);
        rn += badB ? 1ull : 0ull;
    }
    if (rn) atomicAdd(&localRn, rn);
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += 256)
        if (local[i]) atomicAdd(&expMis[i], local[i]);
    if (threadIdx.x == 0 && localRn) atomicAdd(rnMis, localRn);
}

// The XORWOW draw mappings (pt_math.hpp): uniformOf(x) == (float)x * 2^-32 + 2^-33 and
// centered2Of(u) == (u - 0.5f) * 2.0f, each against the separately rounded operations, for all
// 2^32 draws x.
// (scale = 2^-32 and two = 2.0f arrive as kernel arguments, so the compiler keeps the
// two-operation forms as written.)
__global__ __launch_bounds__(256) void checkDraws(uint64_t base, unsigned long long* mis, float scale, float two) {
    unsigned long long mu = 0ull, mc = 0ull;
    const uint64_t first = base + ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 16u;
    for (int k = 0; k < 16; k++) {
        const uint32_t x = (uint32_t)(first + (uint64_t)k);
        const float prod = (float)x * scale;
        const float u = prod + 0x1p-33f;
        const float half = u - 0.5f;
        const float c = half * two;
        const float uf = uniformOf(x), cf = centered2Of(uf);
        mu += __float_as_uint(uf) != __float_as_uint(u) ? 1ull : 0ull;
        mc += __float_as_uint(cf) != __float_as_uint(c) ? 1ull : 0ull;
    }
    if (mu) atomicAdd(&mis[0], mu);
    if (mc) atomicAdd(&mis[1], mc);
}

// The sample-mode fixed-point conversions (pt_math.hpp): blockFixedSmall(x) == blockFixed(x) for
// every fp32 x the kernels hand it (x >= 0 and x < 2^24, NaN excluded: all patterns 0 ... 0x4b7fffff
// and -0), each of those patterns once.
__global__ __launch_bounds__(256) void checkFixed(uint64_t base, unsigned long long* mis) {
    unsigned long long m = 0ull, n = 0ull;
    const uint64_t first = base + ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 16u;
    for (int k = 0; k < 16; k++) {
        const uint32_t bits = (uint32_t)(first + (uint64_t)k);
        const float x = __uint_as_float(bits);
        if (!(x >= 0.0f && x < 16777216.0f)) continue;
        m += blockFixedSmall(x) != blockFixed(x) ? 1ull : 0ull;
        n++;
    }
    if (m) atomicAdd(&mis[0], m);
    if (n) atomicAdd(&mis[1], n);
}

int main() {
    unsigned long long *dExp = nullptr, *dRn = nullptr;
    if (hipMalloc(&dExp, 256 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&dRn, sizeof(unsigned long long)) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 2;
    }
    (void)hipMemset(dExp, 0, 256 * sizeof(unsigned long long));
    (void)hipMemset(dRn, 0, sizeof(unsigned long long));
    const uint64_t perLaunch = 1ull << 28;   // 2^28 patterns: 65,536 blocks of 256 threads x 16
    for (uint64_t base = 0; base < (1ull << 32); base += perLaunch) {
        hipLaunchKernelGGL(check, dim3((unsigned)(perLaunch / (256 * 16))), dim3(256), 0, 0, base, dExp, dRn);
    }
    unsigned long long* dDraw = nullptr;
    if (hipMalloc(&dDraw, 2 * sizeof(unsigned long long)) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 2;
    }
    (void)hipMemset(dDraw, 0, 2 * sizeof(unsigned long long));
    for (uint64_t base = 0; base < (1ull << 32); base += perLaunch) {
        hipLaunchKernelGGL(checkDraws, dim3((unsigned)(perLaunch / (256 * 16))), dim3(256), 0, 0, base, dDraw, 0x1p-32f, 2.0f);
    }
    unsigned long long* dFix = nullptr;
    if (hipMalloc(&dFix, 2 * sizeof(unsigned long long)) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 2;
    }
    (void)hipMemset(dFix, 0, 2 * sizeof(unsigned long long));
    for (uint64_t base = 0; base < (1ull << 32); base += perLaunch) {
        hipLaunchKernelGGL(checkFixed, dim3((unsigned)(perLaunch / (256 * 16))), dim3(256), 0, 0, base, dFix);
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "kernel failed\n");
        return 2;
    }
    unsigned long long hExp[256], hRn = 0;
    (void)hipMemcpy(hExp, dExp, sizeof(hExp), hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hRn, dRn, sizeof(hRn), hipMemcpyDeviceToHost);
    printf("{\"inputs\": %llu, \"rcpRN_mismatches\": %llu, \"fast_range\": [%u, %u], \"newton_mismatches_by_exponent\": {",
           1ull << 32, hRn, kRcpExpLo, kRcpExpHi);
    bool first = true;
    unsigned long long inRange = 0;
    for (int e = 0; e < 256; e++) {
        if (!hExp[e]) continue;
        printf("%s\"%d\": %llu", first ? "" : ", ", e, hExp[e]);
        first = false;
        if ((uint32_t)e >= kRcpExpLo && (uint32_t)e <= kRcpExpHi) inRange += hExp[e];
    }
    unsigned long long hDraw[2] = {0ull, 0ull};
    (void)hipMemcpy(hDraw, dDraw, sizeof(hDraw), hipMemcpyDeviceToHost);
    unsigned long long hFix[2] = {0ull, 0ull};
    (void)hipMemcpy(hFix, dFix, sizeof(hFix), hipMemcpyDeviceToHost);
    printf("}, \"newton_mismatches_in_fast_range\": %llu, \"uniform_fma_mismatches\": %llu, "
           "\"centered2_fma_mismatches\": %llu, \"block_fixed_small_checked\": %llu, \"block_fixed_small_mismatches\": %llu}\n",
           inRange, hDraw[0], hDraw[1], hFix[1], hFix[0]);
    return (hRn == 0 && inRange == 0 && hDraw[0] == 0 && hDraw[1] == 0 && hFix[0] == 0 && hFix[1] == 0x4b800000ull + 1ull) ? 0 : 1;
}
