// pt_sort.hip — hand-written device primitives of the build path (gfx950): a stable LSD radix sort
// of (key, value) pairs and a single-pass exclusive scan with decoupled look-back.
//
// The radix sort replaces the host std::stable_sort of morton::computeMortonOnHost
// (utils/morton_code.h:64-75): the (code, objID) pairs enter in objID order and an LSD radix sort
// is stable, so sorting the 30-bit codes with the objIDs as values gives exactly the reference's
// order (equal codes keep ascending objIDs).  It also orders the render's tiles longest first.
// The scan serves the device wide-tree build (csrc/pt_wide_build.hip: cluster compaction and the
// per-level node / primitive allocation).
//
// Radix sort, per 8-bit digit (passes over bits [0, 8), [8, 16), ... up to `bits`):
//   1. digitCountKernel: each tile of 1024 pairs counts its digits (LDS atomics) into
//      hist[digit][tile] (digit-major);
//   2. an exclusive scan of hist gives, for every (digit, tile), where that tile's pairs of that
//      digit start in the output;
//   3. digitScatterKernel: each tile ranks its pairs stably -- a wave takes 64 consecutive pairs at
//      a time, finds the lanes holding the same digit with 8 ballots (one per digit bit), ranks by
//      the lanes below it, and a per-wave digit counter in LDS carries the rank across rounds;
//      the waves' counts then give each wave's start per digit -- and writes each pair to
//      start(digit, tile) + its rank.
// Scan (Merrill & Garland 2016, single-pass prefix scan with decoupled look-back): tiles are taken
// in launch order from an atomic counter; a tile scans its items (per thread, then across the
// wave with shuffles, then across the 4 waves), publishes its aggregate, looks back over its
// predecessors' published aggregates / inclusive prefixes until it meets a prefix, and publishes
// its own inclusive prefix (flag and value in one 64-bit word, relaxed agent-scope atomics).
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "pt_prims.hpp"

namespace pt {
namespace {

constexpr int kThreads = 256;   // 4 waves
constexpr int kWaves = kThreads / 64;

// --------------------------------------------------------------------------- scan
// Per tile and component one 64-bit status word {flag << 32 | value}, written and read with relaxed
// agent-scope atomics: flag and value travel together, so no release / acquire fences (on this chip
// an L2 writeback / invalidate each) are needed.  The uint4 scan keeps three words per tile and looks
// back over each component on its own (three lanes in parallel).
struct OpU32 {
    using T = uint32_t;
    static constexpr int kItems = 8, kComps = 1;
    __device__ static T id() { return 0u; }
    __device__ static T add(T a, T b) { return a + b; }
    __device__ static T shflUp(T v, int d) { return (T)__shfl_up((int)v, d, 64); }
    __device__ static uint32_t comp(const T& v, int) { return v; }
    __device__ static void setComp(T& v, int, uint32_t x) { v = x; }
};
struct OpU3 {   // the x, y, z words summed, w = 0 (the wide build's {nodes, primitives, items} counts)
    using T = uint4;
    static constexpr int kItems = 4, kComps = 3;
    __device__ static T id() { return make_uint4(0u, 0u, 0u, 0u); }
    __device__ static T add(T a, T b) { return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, 0u); }
    __device__ static T shflUp(T v, int d) {
        return make_uint4((uint32_t)__shfl_up((int)v.x, d, 64), (uint32_t)__shfl_up((int)v.y, d, 64),
                          (uint32_t)__shfl_up((int)v.z, d, 64), 0u);
    }
    __device__ static uint32_t comp(const T& v, int c) { return c == 0 ? v.x : (c == 1 ? v.y : v.z); }
    __device__ static void setComp(T& v, int c, uint32_t x) {
        if (c == 0) v.x = x;
        else if (c == 1) v.y = x;
        else v.z = x;
    }
};

constexpr unsigned long long kFlagAggregate = 1ull << 32, kFlagPrefix = 2ull << 32;

// Scan scratch: [tile counter, padding to 256 B][status words: kComps x u64 per tile]
template <class Op>
size_t scanScratch(size_t n) {
    const size_t tile = (size_t)kThreads * Op::kItems;
    const size_t tiles = (n + tile - 1) / tile;
    return 256 + tiles * Op::kComps * 8;
}

template <class Op>
__global__ __launch_bounds__(kThreads) void scanKernel(const typename Op::T* __restrict__ in, typename Op::T* out,
                                                        size_t n, unsigned char* scratch) {
    using T = typename Op::T;
    constexpr int ITEMS = Op::kItems, C = Op::kComps;
    uint32_t* counter = reinterpret_cast<uint32_t*>(scratch);
    unsigned long long* status = reinterpret_cast<unsigned long long*>(scratch + 256);
    __shared__ uint32_t sTile;
    __shared__ T sWave[kWaves];
    __shared__ uint32_t sExcl[C];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) sTile = atomicAdd(counter, 1u);   // tiles in the order blocks start: look-back never waits on an unstarted tile
    __syncthreads();
    const size_t tile = sTile;
    const size_t base = tile * (size_t)(kThreads * ITEMS) + (size_t)tid * ITEMS;
    T v[ITEMS];
    T run = Op::id();
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const T x = base + i < n ? in[base + i] : Op::id();
        v[i] = run;
        run = Op::add(run, x);
    }
    T incl = run;   // inclusive scan of the thread totals across the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T y = Op::shflUp(incl, d);
        if (lane >= d) incl = Op::add(y, incl);
    }
    T wexcl = Op::shflUp(incl, 1);
    if (lane == 0) wexcl = Op::id();
    if (lane == 63) sWave[wave] = incl;
    __syncthreads();
    T wpre = Op::id(), agg = Op::id();
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
        if (w < wave) wpre = Op::add(wpre, sWave[w]);
        agg = Op::add(agg, sWave[w]);
    }
    if (tid < C) {   // component `tid`: publish, look back, publish the inclusive prefix
        const uint32_t a = Op::comp(agg, tid);
        unsigned long long* my = status + tile * C + tid;
        uint32_t excl = 0u;
        if (tile == 0) {
            __hip_atomic_store(my, kFlagPrefix | a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(my, kFlagAggregate | a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (size_t j = tile - 1;; j--) {   // (tile 0 always publishes a prefix: j never wraps)
                unsigned long long w;
                while (((w = __hip_atomic_load(status + j * C + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) == 0u)
                    __builtin_amdgcn_s_sleep(1);
                excl += (uint32_t)w;
                if ((w >> 32) == (kFlagPrefix >> 32)) break;
            }
            __hip_atomic_store(my, kFlagPrefix | (uint32_t)(excl + a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        sExcl[tid] = excl;
    }
    __syncthreads();
    T ex = Op::id();
#pragma unroll
    for (int c = 0; c < C; c++) Op::setComp(ex, c, sExcl[c]);
    const T pre = Op::add(ex, Op::add(wpre, wexcl));
#pragma unroll
    for (int i = 0; i < ITEMS; i++)
        if (base + i < n) out[base + i] = Op::add(pre, v[i]);
}

template <class Op>
hipError_t exclusiveScan(void* scratch, const typename Op::T* in, typename Op::T* out, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const size_t tile = (size_t)kThreads * Op::kItems;
    const size_t tiles = (n + tile - 1) / tile;
    hipError_t e = hipMemsetAsync(scratch, 0, scanScratch<Op>(n), st);
    if (e != hipSuccess) return e;
    scanKernel<Op><<<(unsigned)tiles, kThreads, 0, st>>>(in, out, n, static_cast<unsigned char*>(scratch));
    return hipGetLastError();
}

// --------------------------------------------------------------------------- radix sort
constexpr int kDigitBits = 8, kRadix = 1 << kDigitBits;
constexpr int kRounds = 4;                            // 64-pair rounds per wave
constexpr int kSortTile = kThreads * kRounds;         // 1024 pairs per tile

// (`dmask`: the digit's bits -- the last pass of a `bits`-bit sort takes fewer than 8, the keys'
// higher bits are ignored)
__global__ __launch_bounds__(kThreads) void digitCountKernel(const uint32_t* __restrict__ keys, size_t n, int shift,
                                                             uint32_t dmask, uint32_t* hist, uint32_t tiles) {
    __shared__ uint32_t cnt[kRadix];
    cnt[threadIdx.x] = 0u;   // (kThreads == kRadix)
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kSortTile;
#pragma unroll
    for (int r = 0; r < kRounds; r++) {
        const size_t i = base + (size_t)r * kThreads + threadIdx.x;
        if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & dmask], 1u);
    }
    __syncthreads();
    hist[(size_t)threadIdx.x * tiles + blockIdx.x] = cnt[threadIdx.x];
}

__global__ __launch_bounds__(kThreads) void digitScatterKernel(const uint32_t* __restrict__ kin,
                                                               const uint32_t* __restrict__ vin, uint32_t* kout,
                                                               uint32_t* vout, size_t n, int shift, uint32_t dmask,
                                                               const uint32_t* __restrict__ start, uint32_t tiles) {
    __shared__ uint32_t cnt[kWaves][kRadix];   // per wave: pairs of each digit so far, then the wave's start
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int w = 0; w < kWaves; w++) cnt[w][tid] = 0u;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kSortTile + (size_t)wave * (kRounds * 64);   // a wave's pairs are consecutive
    uint32_t key[kRounds], val[kRounds], rank[kRounds];
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < kRounds; r++) {
        const size_t i = base + (size_t)r * 64 + lane;
        const bool ok = i < n;
        key[r] = ok ? kin[i] : 0u;
        val[r] = ok ? vin[i] : 0u;
        const uint32_t d = (key[r] >> shift) & dmask;
        uint64_t same = __ballot(ok);
#pragma unroll
        for (int b = 0; b < kDigitBits; b++) {
            const uint64_t m = __ballot((d >> b) & 1u);
            same &= ((d >> b) & 1u) ? m : ~m;
        }
        const uint32_t before = (uint32_t)__popcll(same & below);
        const uint32_t c = cnt[wave][d];   // (every lane of the digit reads it before its lowest lane adds)
        rank[r] = c + before;
        __builtin_amdgcn_wave_barrier();
        if (ok && before == 0u) cnt[wave][d] = c + (uint32_t)__popcll(same);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {   // per digit: each wave's start = the tile's start of the digit + the earlier waves' counts
        uint32_t s = start[(size_t)tid * tiles + blockIdx.x];
#pragma unroll
        for (int w = 0; w < kWaves; w++) {
            const uint32_t c = cnt[w][tid];
            cnt[w][tid] = s;
            s += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; r++) {
        const size_t i = base + (size_t)r * 64 + lane;
        if (i < n) {
            const uint32_t p = cnt[wave][(key[r] >> shift) & dmask] + rank[r];
            kout[p] = key[r];
            vout[p] = val[r];
        }
    }
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

size_t scanScratchBytesU32(size_t n) { return scanScratch<OpU32>(n); }
size_t scanScratchBytesU3(size_t n) { return scanScratch<OpU3>(n); }
hipError_t exclusiveScanU32(void* scratch, const uint32_t* in, uint32_t* out, size_t n, hipStream_t st) {
    return exclusiveScan<OpU32>(scratch, in, out, n, st);
}
hipError_t exclusiveScanU3(void* scratch, const uint4* in, uint4* out, size_t n, hipStream_t st) {
    return exclusiveScan<OpU3>(scratch, in, out, n, st);
}

// Sorts n (code, id) pairs by the low `bits` bits of code, stably.  With temp == nullptr only the
// required temporary storage size is returned in *temp_bytes.  The inputs are not modified.
hipError_t radixSortPairs(void* temp, size_t* temp_bytes, const uint32_t* codes_in, uint32_t* codes_out,
                          const uint32_t* ids_in, uint32_t* ids_out, size_t n, int bits, hipStream_t stream) {
    const uint32_t tiles = (uint32_t)((n + kSortTile - 1) / kSortTile);
    const size_t histN = (size_t)kRadix * tiles;
    const size_t need = 2 * align256(n * 4) + 2 * align256(histN * 4) + align256(scanScratch<OpU32>(histN));
    if (!temp) {
        *temp_bytes = need > 0 ? need : 256;
        return hipSuccess;
    }
    if (*temp_bytes < need) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    const int passes = bits <= 0 ? 0 : (bits + kDigitBits - 1) / kDigitBits;
    if (passes == 0) {
        hipError_t e = hipMemcpyAsync(codes_out, codes_in, n * 4, hipMemcpyDeviceToDevice, stream);
        if (e != hipSuccess) return e;
        return hipMemcpyAsync(ids_out, ids_in, n * 4, hipMemcpyDeviceToDevice, stream);
    }
    unsigned char* t = static_cast<unsigned char*>(temp);
    uint32_t* kT = reinterpret_cast<uint32_t*>(t);
    uint32_t* vT = reinterpret_cast<uint32_t*>(t + align256(n * 4));
    uint32_t* hist = reinterpret_cast<uint32_t*>(t + 2 * align256(n * 4));
    uint32_t* start = reinterpret_cast<uint32_t*>(t + 2 * align256(n * 4) + align256(histN * 4));
    void* scratch = t + 2 * align256(n * 4) + 2 * align256(histN * 4);
    const uint32_t* ks = codes_in;
    const uint32_t* vs = ids_in;
    for (int p = 0; p < passes; p++) {
        // ping-pong so that the last pass writes the output
        const bool toOut = ((passes - 1 - p) & 1) == 0;
        uint32_t* kd = toOut ? codes_out : kT;
        uint32_t* vd = toOut ? ids_out : vT;
        const int shift = p * kDigitBits;
        const int db = bits - shift < kDigitBits ? bits - shift : kDigitBits;
        const uint32_t dmask = (1u << db) - 1u;
        digitCountKernel<<<tiles, kThreads, 0, stream>>>(ks, n, shift, dmask, hist, tiles);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        if ((e = exclusiveScan<OpU32>(scratch, hist, start, histN, stream)) != hipSuccess) return e;
        digitScatterKernel<<<tiles, kThreads, 0, stream>>>(ks, vs, kd, vd, n, shift, dmask, start, tiles);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        ks = kd;
        vs = vd;
    }
    return hipSuccess;
}

}  // namespace pt
