// pt_prims.hpp — the build path's device primitives (pt_sort.hip): stable LSD radix sort of
// (key, value) pairs and single-pass exclusive scans with decoupled look-back.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace pt {
// Sorts n (code, id) pairs by the low `bits` bits of code, stably (= std::stable_sort by code,
// morton_code.h:64-75).  temp == nullptr: returns the scratch size in *temp_bytes.
hipError_t radixSortPairs(void* temp, size_t* temp_bytes, const uint32_t* codes_in, uint32_t* codes_out,
                          const uint32_t* ids_in, uint32_t* ids_out, size_t n, int bits, hipStream_t stream);
// Exclusive prefix sums; `scratch` holds scanScratchBytes*(n) bytes (cleared by the call itself).
size_t scanScratchBytesU32(size_t n);
size_t scanScratchBytesU3(size_t n);
hipError_t exclusiveScanU32(void* scratch, const uint32_t* in, uint32_t* out, size_t n, hipStream_t st);
hipError_t exclusiveScanU3(void* scratch, const uint4* in, uint4* out, size_t n, hipStream_t st);   // x, y, z; w = 0
}  // namespace pt
