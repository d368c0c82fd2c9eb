// Micro-benchmark: dependent random gathers of R-byte records per lane (pointer chasing through a
// table of T bytes), 4 waves/SIMD, all CUs: how the per-step time depends on the record size
// (number of dwordx4 loads per step).  Informs the BVH node size.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

template <int NV4>
__global__ __launch_bounds__(64) void chase(const float4* __restrict__ tab, unsigned nrec, int steps, unsigned* out) {
    unsigned idx = (blockIdx.x * 64u + threadIdx.x) * 2654435761u % nrec;
    float acc = 0.0f;
    for (int s = 0; s < steps; s++) {
        const float4* r = tab + (size_t)idx * NV4;
        float4 v[NV4];
#pragma unroll
        for (int k = 0; k < NV4; k++) v[k] = r[k];
        float x = 0.0f;
#pragma unroll
        for (int k = 0; k < NV4; k++) x += v[k].x + v[k].y + v[k].z;
        acc += x;
        idx = __float_as_uint(v[NV4 - 1].w);   // next record
    }
    if (acc == 12345.0f) out[0] = idx;
}

template <int NV4>
void run(size_t tableBytes, int waves, int steps) {
    const unsigned nrec = (unsigned)(tableBytes / (16 * NV4));
    std::vector<float4> h((size_t)nrec * NV4);
    srand(1);
    for (unsigned i = 0; i < nrec; i++) {
        for (int k = 0; k < NV4; k++) h[(size_t)i * NV4 + k] = make_float4(1, 2, 3, 0);
        unsigned nxt = (unsigned)(((unsigned long long)rand() * 7919ull + i) % nrec);
        float f;
        memcpy(&f, &nxt, 4);
        h[(size_t)i * NV4 + NV4 - 1].w = f;
    }
    float4* d;
    unsigned* o;
    hipMalloc(&d, h.size() * 16);
    hipMalloc(&o, 4);
    hipMemcpy(d, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    chase<NV4><<<waves, 64>>>(d, nrec, steps, o);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    chase<NV4><<<waves, 64>>>(d, nrec, steps, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("record %3d B  table %7zu KB  waves %6d  steps %d: %.3f ms, %.0f ns/step, %.1f G steps/s\n", 16 * NV4,
           tableBytes / 1024, waves, steps, ms, ms * 1e6 / steps, (double)waves * 64 * steps / (ms * 1e-3) / 1e9);
    hipFree(d);
    hipFree(o);
}

int main() {
    const int waves = 256 * 16, steps = 4000;
    for (size_t tb : {320u << 10, 64u << 20}) {
        run<1>(tb, waves, steps);
        run<2>(tb, waves, steps);
        run<4>(tb, waves, steps);
        run<8>(tb, waves, steps);
    }
    return 0;
}
