// fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE against known byte counts for the access
// shapes of the render kernel ("C5 past-L2 traffic").  Run each mode under
// `rocprofv3 --pmc FETCH_SIZE` (and TCC_EA0_RDREQ_sum / TCC_EA0_RDREQ_32B_sum / TCC_MISS_sum in
// passes of their own); every launch touches each record at most once, so every access misses L2.
//
//   fetch_calib <mode>
//   stream    : 1 GiB read once, 16 B per lane, coalesced (the guide's reference shape: FETCH_SIZE = 1/2)
//   g128      : 2^23 random 128-B records (8 x 16-B loads per lane), 128-B aligned, from a 1 GiB table
//   g64s128   : 2^23 random 64-B records at a 128-B stride (the first half of each line)
//   g80s128   : 2^23 random 80-B records at a 128-B stride (one line each)
//   g80       : 2^23 random 80-B records at an 80-B stride (the wide tree's node array: 1.5 lines each)
//   g80mall   : 2^21 random 80-B records at an 80-B stride from a 168 MB table (C5's working set fits
//               the 256 MiB Infinity Cache): one warm-up launch, then the measured one
//   g80warm   : g80 (671 MB table, larger than the Infinity Cache) with a warm-up launch first
//   g48       : 2^23 random 48-B records at a 48-B stride (primitive and shading records)
// Cold modes stream 1 GiB through the caches before the measured launch (the Infinity Cache then
// holds none of the table); every mode first launches its kernel once on a small table, so the
// timed launch does not include loading the code object.
// Prints one JSON line per measured launch: the bytes the lanes requested, the 128-B lines and
// 64-B sectors those requests cover, and the launch time.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            std::exit(2);                                                                       \
        }                                                                                       \
    } while (0)

__global__ __launch_bounds__(256) void streamKernel(const uint4* __restrict__ a, size_t n16, unsigned* out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Access k (0 <= k < nacc) reads record perm(k) = (k * odd) mod nrec (nrec a power of two): every
// record at most once per launch.  NV4 16-B loads per record, records `stride` bytes apart.
template <int NV4>
__global__ __launch_bounds__(256) void gatherKernel(const unsigned char* __restrict__ tab, uint32_t nrecMask,
                                                    uint32_t stride, uint32_t steps, unsigned* out) {
    const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t s = 0; s < steps; s++) {
        const uint32_t k = lane * steps + s;
        const uint32_t r = (k * 0x9E3779B1u) & nrecMask;
        const uint4* p = reinterpret_cast<const uint4*>(tab + (size_t)r * stride);
#pragma unroll
        for (int j = 0; j < NV4; j++) {
            const uint4 v = p[j];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "stream";
    unsigned* out;
    CK(hipMalloc(&out, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    if (mode == "stream") {
        const size_t bytes = (size_t)1 << 30;
        void* a;
        CK(hipMalloc(&a, bytes));
        CK(hipMemset(a, 1, bytes));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        streamKernel<<<256 * 16, 256>>>(static_cast<const uint4*>(a), bytes / 16, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"mode\": \"stream\", \"requested_bytes\": %zu, \"lines128\": %zu, \"sectors64\": %zu, \"ms\": %.4f}\n",
                    bytes, bytes / 128, bytes / 64, ms);
        return 0;
    }
    int nv4 = 0;
    uint32_t stride = 0, logRec = 23;
    bool warm = false;
    if (mode == "g128") { nv4 = 8; stride = 128; }
    else if (mode == "g64s128") { nv4 = 4; stride = 128; }
    else if (mode == "g80s128") { nv4 = 5; stride = 128; }
    else if (mode == "g80") { nv4 = 5; stride = 80; }
    else if (mode == "g80mall") { nv4 = 5; stride = 80; logRec = 21; warm = true; }
    else if (mode == "g80warm") { nv4 = 5; stride = 80; warm = true; }
    else if (mode == "g48") { nv4 = 3; stride = 48; }
    else { std::fprintf(stderr, "unknown mode\n"); return 2; }
    const size_t nrec = (size_t)1 << logRec;
    const size_t bytes = nrec * stride + 256;
    void* tab;
    CK(hipMalloc(&tab, bytes));
    CK(hipMemset(tab, 1, bytes));
    const uint32_t steps = 8, lanes = (uint32_t)(nrec / steps);   // nrec accesses: every record once
    const unsigned grid = lanes / 256;
    auto launchOn = [&](const void* t, uint32_t mask, unsigned g) {
        const unsigned char* tb = static_cast<const unsigned char*>(t);
        switch (nv4) {
            case 3: gatherKernel<3><<<g, 256>>>(tb, mask, stride, steps, out); break;
            case 4: gatherKernel<4><<<g, 256>>>(tb, mask, stride, steps, out); break;
            case 5: gatherKernel<5><<<g, 256>>>(tb, mask, stride, steps, out); break;
            default: gatherKernel<8><<<g, 256>>>(tb, mask, stride, steps, out); break;
        }
    };
    auto launch = [&]() { launchOn(tab, (uint32_t)(nrec - 1), grid); };
    CK(hipDeviceSynchronize());
    launchOn(tab, 255u, 1);   // code object load (a small corner of the table)
    CK(hipDeviceSynchronize());
    if (warm) {   // the measured launch then finds the table in the Infinity Cache
        launch();
        CK(hipDeviceSynchronize());
    } else {      // flush: 1 GiB streamed through L2 and the Infinity Cache
        const size_t fb = (size_t)1 << 30;
        void* f;
        CK(hipMalloc(&f, fb));
        CK(hipMemset(f, 2, fb));
        streamKernel<<<256 * 16, 256>>>(static_cast<const uint4*>(f), fb / 16, out);
        CK(hipDeviceSynchronize());
        CK(hipFree(f));
    }
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // lines / sectors covered: record r spans [r * stride, r * stride + 16 * nv4)
    size_t lines = 0, sectors = 0;
    for (size_t r = 0; r < nrec; r++) {
        const size_t lo = r * stride, hi = lo + 16 * (size_t)nv4 - 1;
        lines += hi / 128 - lo / 128 + 1;
        sectors += hi / 64 - lo / 64 + 1;
    }
    std::printf("{\"mode\": \"%s\", \"records\": %zu, \"table_bytes\": %zu, \"requested_bytes\": %zu, \"lines128\": %zu, "
                "\"sectors64\": %zu, \"warm\": %s, \"ms\": %.4f}\n",
                mode.c_str(), nrec, nrec * stride, nrec * 16 * (size_t)nv4, lines, sectors, warm ? "true" : "false", ms);
    return 0;
}
