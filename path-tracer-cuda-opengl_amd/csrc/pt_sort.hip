// pt_sort.hip — the LBVH build's key sort on the device (replaces the host std::stable_sort of
// morton::computeMortonOnHost, utils/morton_code.h:64-75).
//
// The reference sorts (code, objID) pairs by code with a stable sort, the objects entering in
// objID order; an LSD radix sort is stable, so sorting the 30-bit codes with the objIDs as
// values gives exactly the reference's order (equal codes keep ascending objIDs).  Kept in its
// own translation unit: rocPRIM's radix sort is header-heavy and slow to compile.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstddef>
#include <cstdint>

namespace pt {

// Sorts n (code, id) pairs by the low `bits` bits of code.  With temp == nullptr only the
// required temporary storage size is returned in *temp_bytes.
hipError_t radixSortPairs(void* temp, size_t* temp_bytes, const uint32_t* codes_in, uint32_t* codes_out,
                          const uint32_t* ids_in, uint32_t* ids_out, size_t n, int bits, hipStream_t stream) {
    return rocprim::radix_sort_pairs(temp, *temp_bytes, codes_in, codes_out, ids_in, ids_out, n, 0, bits, stream);
}

}  // namespace pt
