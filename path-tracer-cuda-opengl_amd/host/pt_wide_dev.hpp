// pt_wide_dev.hpp — the compressed 8-wide tree built on the device (csrc/pt_wide_build.hip).
//
// Same node and primitive records as the host build (pt_wide8.hpp, layout in pt_wide8.cpp), a
// binary tree built in parallel: the host's binned SAH top down (default), or parallel
// locally-ordered clustering (PT_WIDE_DEVICE_BUILDER=ploc: clusters in Morton order repeatedly
// merge with their mutual nearest neighbour within a window, distance = surface area of the
// merged box), then the same top-down
// collapse to 8 children and the same outward 8-bit quantisation, one level of the wide tree per
// launch.  Milliseconds instead of the host build's tens of milliseconds to seconds: it is the
// per-frame rebuild of dynamic scenes (PT_BVH_WIDE_DEVICE).  Closest hits do not depend on the
// tree, so the images equal the host tree's.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace pt {

struct WideDevIn {
    const float4* prims;       // n x 3 float4 leaf-order primitive records (pt_device.hip DevScene::prims)
    const float4* shade;       // n x 3 float4 leaf-order shading records
    const float* leafBoxes;    // n x {min xyz, max xyz}
    const float4* lbvh;        // the binary LBVH, 4 float4 per internal node, child refs in [4i + 3].xy
    const int* iparent;        // parent of internal node i (-1 for the root)
    const int* lparent;        // parent of leaf k
    const int2* irange;        // leaf range [first, last] of internal node i
    int64_t n;
};

struct WideDevOut {
    uint32_t* nodes;           // node slots x kW8NodeDwords dwords, capacity wideDevNodeSlots(n)
    uint32_t* wprims;          // n x 12 dwords
    float4* wshade;            // n x 3 float4, shading records in reference rank order
    uint32_t* rank;            // n: leaf k -> its rank in the reference's traversal order
    int depth = 0;             // wide levels (root = 1)
    int64_t slots = 0;         // node slots written
};

// Node slots the device build may use: a node with a child block has 8 children and consumes 7
// internal nodes of the binary tree, so at most 1 + 8 * floor((n - 1) / 7) slots.
inline int64_t wideDevNodeSlots(int64_t n) { return 1 + 8 * ((n > 1 ? n - 1 : 0) / 7 + 1); }
// The traversal kernels carry a node's child base in 24 bits (ng = childBase << 8 | hit slots), so
// a child block must end at or below 2^24 slots: the build reports an error instead of writing a
// base that would be truncated (host build: pt_wide8.cpp checks the same limit).
constexpr int64_t kWideMaxSlots = (int64_t)1 << 24;
inline uint32_t wideDevSlotCap(int64_t n) {
    const int64_t s = wideDevNodeSlots(n);
    return (uint32_t)(s < kWideMaxSlots ? s : kWideMaxSlots);
}

class WideDevBuilder {
public:
    WideDevBuilder() = default;
    WideDevBuilder(const WideDevBuilder&) = delete;
    WideDevBuilder& operator=(const WideDevBuilder&) = delete;
    ~WideDevBuilder();
    // Enqueues the build on `stream`; synchronises with it once per PLOC pass and per wide level
    // (the next launch's size).  Scratch is kept between builds of up to the same n.
    hipError_t build(const WideDevIn& in, WideDevOut& out, hipStream_t stream, std::string& err);

private:
    struct Buf {
        void* p = nullptr;
        size_t cap = 0;
    };
    hipError_t reserve(Buf& b, size_t bytes);
    // step 2 by SAH (the root's id left in cid_[0][0])
    hipError_t buildSah(const WideDevIn& in, hipStream_t stream, float trav, std::string& err);
    Buf pbox_, pchild_, cid_[2], nn_, flag_, pos_, items_[2], cnt_, ofs_, scanTemp_, misc_;
    Buf sahCen_, sahRef_[2], sahLarge_[2], sahSmall_, sahSplit_, sahBins_, sahMulti_, sahBlk_, sahBlkR_, sahBlkO_, sahCnt_;
};

}  // namespace pt
