// pt_wide8.hpp — host build of the compressed 8-wide BVH traversed by the wide render kernel.
//
// The reference traverses its binary LBVH depth first (RenderManager::hitBvh,
// utils/render_manager.h:86-135).  The wide tree is an acceleration structure of this build
// only: a binned-SAH binary tree over the same primitive records, collapsed to 8 children per
// node, child boxes quantised outward to 8 bits per plane.  It changes which nodes are visited
// and in which order, never which primitive is the closest hit ("Wide tree").
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace pt {

#ifndef PT_NODE_DWORDS
#define PT_NODE_DWORDS 20   // a node slot: the 80-B record; 32 pads each slot to one 128-B cache line (A/B builds)
#endif
constexpr int kW8NodeDwords = PT_NODE_DWORDS;   // node slot in dwords: 80-B record (layout in pt_wide8.cpp) + padding
static_assert(kW8NodeDwords == 20 || kW8NodeDwords == 32, "node slots of 80 or 128 B");
constexpr int kW8PrimDwords = 12;   // 48-B primitive record

struct Wide8 {
    std::vector<uint32_t> nodes;   // kW8NodeDwords per node slot; slot 0 = root
    std::vector<uint32_t> prims;   // kW8PrimDwords per primitive, in traversal (leaf) order
    int depth = 0;                 // wide levels, root = 1 (= traversal stack entries needed)
    int64_t usedNodes = 0;         // slots holding a node (children blocks are 8 slots, sparse)
    int64_t leaves = 0;
};

// prims: n leaf-order (Morton) primitive records of kW8PrimDwords dwords (the device `prims`
// array: {v0, mat}{v1, objID}{v2, sphere flag} or {c, mat}{r, 0, 0, objID}{0, 0, 0, 1});
// boxes: n x {min xyz, max xyz}; rank: per leaf k its position in the reference's traversal
// order (referenceRanks).  The output records carry the rank in place of the material id
// ({v0, rank}...): ties between equal hit distances are decided by it, and it indexes the wide
// kernels' shading records.  Returns false with `err` set when the tree exceeds the encoding
// limits.
// scaleFloor: the plane quantum is at least 2^-18 of max(scaleFloor, the tree's extent and
// coordinates) -- the distance up to which ray origins keep the boxes' outward margin (instanced
// meshes: the world's reach in object space).
bool buildWide8(const uint32_t* prims, const float* boxes, const uint32_t* rank, int64_t n, Wide8& out,
                std::string& err, double scaleFloor = 0.0);
// buildWide8 with at most maxLeaf (1..3) primitives per leaf child (instancing's top level: one
// instance per leaf).
bool buildWide8Leaf(const uint32_t* prims, const float* boxes, const uint32_t* rank, int64_t n, int maxLeaf,
                    Wide8& out, std::string& err, double scaleFloor = 0.0);

// Instancing (two-level tree in one node array).  Record of an instance node, kW8NodeDwords:
//   [0] 1 if the transform is the identity (the ray is not transformed), [1] 1 if it only
//   translates (the origin moves, the direction stays), [2] 0,
//   [3] kW8InstanceFlag (never a valid exponent word: byte 3 of a node's exponents is 0),
//   [4] the instance's bottom-level root slot, [5] the instance id, [6..7] 0,
//   [8..19] the world-to-object transform, 3 rows of {m0, m1, m2, t} (fp32).
constexpr uint32_t kW8InstanceFlag = 0xff000000u;
// Relocate a tree built on its own into a shared node / primitive array: child bases += nodeBase,
// primitive bases += primBase.
void relocateWide8(Wide8& w, uint32_t nodeBase, uint32_t primBase);
// Turn the leaf children of a top-level tree built with buildWide8Leaf(.., 1, ..) over instance
// boxes into internal children whose slots hold instance records: instanceOf(prim record) gives
// the instance id of a leaf's primitive record, record(id, dst) writes its 20-dword record.
// Nodes without a child block get one.  Returns false with err set past the encoding limits.
bool instanceLeaves(Wide8& top, uint32_t (*instanceOf)(const uint32_t* primRecord),
                    void (*record)(uint32_t id, uint32_t* dst, void* ctx), void* ctx, std::string& err);

// The order in which RenderManager::hitBvh (render_manager.h:105-133) would test the leaves of
// the binary LBVH if every box passed: at a node, its leaf children (left, then right), then the
// right subtree, then the left one (the left child is pushed first, so the right one is popped
// first).  refs: per internal node its two child refs (bit 31 = leaf, low 30 bits = leaf k).
// Returns rank[k].
std::vector<uint32_t> referenceRanks(const uint32_t* leftRef, const uint32_t* rightRef, size_t stride, int64_t n);

}  // namespace pt
