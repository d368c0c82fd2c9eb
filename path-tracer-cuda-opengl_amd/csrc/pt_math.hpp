// Exact fp32 helpers shared by the render kernels (pt_device.hip) and their exhaustive checker
// (tools/micro/rcp_check.hip).  Compiled with the kernels' flags: -ffp-contract=off, no fast math,
// fp32 denormals on (HIP's default for gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

// The IEEE division 1.0f / x costs eleven VALU operations on gfx950 (v_div_scale x2, v_rcp_f32,
// five FMAs / multiplies, v_div_fmas, v_div_fixup).  The reference divides by the determinant
// of every triangle test (triangle.h / cuda_object.h:73-78), by every ray direction component
// (aabb.h:24) and by every vector it normalises (vec3.h:89-91), so the render kernel spends a
// measurable share of its issue slots there.
//
// rcpNewton: v_rcp_f32 (1 ulp) refined by one Newton step with fused multiply-adds,
//   e = 1 - x * r,  y = r + e * r,
// three VALU operations.  It equals 1.0f / x bit for bit for every x whose biased exponent lies
// in [kRcpExpLo, kRcpExpHi]; tools/micro/rcp_check.hip compares the two over all 2^32 inputs on
// the GPU (tests/test_gpu_math.py) and reports the exponents where they differ (zeros,
// denormals, and magnitudes whose reciprocal is denormal).  rcpRN takes the division for those.
constexpr uint32_t kRcpExpLo = 1u;     // smallest biased exponent of the fast path
constexpr uint32_t kRcpExpHi = 252u;   // largest (|x| < 2^126: the reciprocal is a normal number)

__device__ __forceinline__ float rcpNewton(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

#ifndef PT_FAST_RCP
#define PT_FAST_RCP 1   // 0: every reciprocal is the IEEE division (A/B builds)
#endif

__device__ __forceinline__ float rcpRN(float x) {
    if constexpr (!PT_FAST_RCP) return 1.0f / x;
    const uint32_t ex = (__float_as_uint(x) >> 23) & 0xffu;
    float y;
    if (__builtin_expect(ex - kRcpExpLo > kRcpExpHi - kRcpExpLo, 0)) {
        y = 1.0f / x;   // zero, denormal, huge, inf, NaN: the IEEE division
    } else {
        y = rcpNewton(x);
    }
    return y;
}

// curand_uniform (x * 2^-32 + 2^-33, in (0, 1]) as one FMA: (float)x is 0 or >= 1, so its product
// with 2^-32 is exact and normal, and fma rounds the same exact sum the separate multiply and
// add round.  Checked against the two-operation form for all 2^32 x (tools/micro/rcp_check.hip).
__device__ __forceinline__ float uniformOf(uint32_t x) { return __builtin_fmaf((float)x, 0x1p-32f, 0x1p-33f); }

// The coordinates of random_in_unit_sphere / random_unit_vector (utility.h:51-62, 73-82):
// 2 * (u - 0.5f).  Doubling is exact and commutes with rounding for normal values and zero, so
// round(2u - 1) = 2 * round(u - 0.5): one FMA instead of a subtract and a multiply.  Checked for
// every u = uniformOf(x) (tools/micro/rcp_check.hip).
__device__ __forceinline__ float centered2Of(float u) { return __builtin_fmaf(u, 2.0f, -1.0f); }

// The wide NODE step's plane distances t = q * a + c for a quantised plane byte q.  One
// v_perm_b32 turns two plane bytes into two fp16 denormals 0x00qq = q * 2^-24 (the zero-byte
// selector 0x0c fills the high bytes), and v_fma_mix_f32 multiplies such an fp16 half (widened
// exactly) by aS = a * 2^24 and adds c with one rounding: the same exact product-sum as
// fma((float)q, a, c), so the same result bit for bit whenever aS is finite (the kernels' fp16
// denormals are on: amdhsa_float_denorm_mode_16_64 3).  Two planes per v_perm instead of one
// v_cvt_f32_ubyte each.  tools/micro/fmamix_check.hip compares the two forms on the GPU (every q,
// 2^32 random (q, a, c), denormal / overflow edges; tests/test_gpu_math.py).
__device__ __forceinline__ uint32_t planePairLo(uint32_t bytes4) { return __builtin_amdgcn_perm(0u, bytes4, 0x0c010c00u); }
__device__ __forceinline__ uint32_t planePairHi(uint32_t bytes4) { return __builtin_amdgcn_perm(0u, bytes4, 0x0c030c02u); }
// (The low half as a plain conversion the compiler folds into v_fma_mix_f32 and schedules freely;
// the high half in asm: with both halves of one register converted, the compiler would widen them
// as a pair with two v_cvt_f32_f16 instead.)
__device__ __forceinline__ float fmaMixLo(uint32_t h2, float aS, float c) {
    return __builtin_fmaf((float)__builtin_bit_cast(_Float16, (unsigned short)(h2 & 0xffffu)), aS, c);
}
__device__ __forceinline__ float fmaMixHi(uint32_t h2, float aS, float c) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h2), "v"(aS), "v"(c));
    return r;
}
// v_max3_f32 / v_min3_f32 on fmaMixHi results: an fmaxf / fminf on an asm output makes the compiler
// quiet it first (one v_max_f32 x, x, x per operand: it cannot know the value is canonical).  The
// plain instructions give the same result here (IEEE mode: a quiet NaN operand is ignored, the
// fma results are never signalling).
__device__ __forceinline__ float max3Raw(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float min3Raw(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// Sample mode: a block's fp32 sum as a 32.32 fixed-point integer (truncated toward zero; NaN -> 0,
// saturated at +-2^62), and back (oracle/pt_oracle.cpp blockFixed / fixedToFloat, same roundings).
// (Truncation done as two 32-bit halves of |p|: a * 2^-32 and a - hi * 2^32 are exact, hi has at
// most 24 significant bits; fewer registers than the generic float -> int64 conversion.)
__device__ __forceinline__ unsigned long long blockFixed(float x) {
    const float p = x * 4294967296.0f;   // exact: a power-of-two scale
    const float a = p == p ? fminf(fabsf(p), 0x1p62f) : 0.0f;
    const uint32_t hi = (uint32_t)(a * 0x1p-32f);
    const uint32_t lo = (uint32_t)__builtin_fmaf((float)hi, -0x1p32f, a);
    const unsigned long long u = ((unsigned long long)hi << 32) | lo;
    return p < 0.0f ? 0ull - u : u;
}
__device__ __forceinline__ float fixedToFloat(unsigned long long a) { return (float)((double)(long long)a * 0x1p-32); }
// blockFixed for 0 <= x < 2^24 (every block sum of a scene whose radiance is bounded, e.g. by the
// sky's <= 1 per sample): x = hi + frac with hi = trunc(x) (exact in float below 2^24) and frac = x -
// hi exact, so trunc(x * 2^32) = hi * 2^32 + trunc(frac * 2^32) -- five VALU per channel instead of
// the clamped, signed conversion's fourteen.  The same integer as blockFixed for such x (the
// oracle's (int64_t)(x * 2^32)); -0 gives 0 either way.
__device__ __forceinline__ unsigned long long blockFixedSmall(float x) {
    const uint32_t hi = __float2uint_rz(x);
    const float frac = x - (float)hi;
    const uint32_t lo = __float2uint_rz(frac * 4294967296.0f);
    return ((unsigned long long)hi << 32) | lo;
}
