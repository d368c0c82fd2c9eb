// Exhaustive check of the render kernels' reciprocal (csrc/pt_math.hpp) against the IEEE
// division 1.0f / x over all 2^32 fp32 bit patterns, on the GPU, with the kernels' own compiler
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
    printf("}, \"newton_mismatches_in_fast_range\": %llu}\n", inRange);
    return (hRn == 0 && inRange == 0) ? 0 : 1;
}
