// pt_wide8.cpp — compressed 8-wide BVH for the wide render kernel (see pt_wide8.hpp).
//
// Build: binned SAH over the primitives' exact boxes (binary, leaves of at most 3 primitives),
// then a top-down collapse to at most 8 children per node (repeatedly open the internal child
// with the largest surface area).
//
// Node record, 20 dwords = 80 B (five 16-B loads):
//   [0..2]  frame origin p (fp32 x, y, z)
//   [3]     biased exponents ex | ey << 8 | ez << 16 (plane quantum s_a = 2^(e_a - 127))
//   [4]     child base: the internal child in slot j is node (child base + j)
//   [5]     primitive base: leaf primitives are primitive (base + offset)
//   [6..7]  meta byte per slot: 0 = empty; internal 0b001_11000 | j; leaf (unary count << 5) | offset
//   [8..11] qlo_x[0..3], qlo_x[4..7], qhi_x[0..3], qhi_x[4..7]     (8-bit planes, byte j = slot j)
//   [12..15] the same for y, [16..19] for z
// A child box is [p + qlo * s, p + qhi * s] per axis, rounded OUTWARD by at least the tree's
// smallest quantum 2^emin (2^-18 of the scene's extent and coordinates) beyond the exact box, so a
// slab test on it (with any fp32 rounding of the ray arithmetic) is conservative: it never rejects
// a box the exact test accepts.
//
// Slots are ordered per ray octant: slot j holds the child nearest along the octant direction j
// (bit a of j set = negative direction on axis a).  A ray of octant o visits internal children
// in increasing (slot ^ o), i.e. its own octant's nearest child first.
#include "pt_wide8.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace pt {
namespace {

struct BBox {
    float mn[3], mx[3];
};
BBox emptyBox() {
    const float inf = INFINITY;
    return {{inf, inf, inf}, {-inf, -inf, -inf}};
}
void growBox(BBox& a, const BBox& b) {
    for (int i = 0; i < 3; i++) {
        a.mn[i] = std::min(a.mn[i], b.mn[i]);
        a.mx[i] = std::max(a.mx[i], b.mx[i]);
    }
}
double halfArea(const BBox& b) {
    double d[3];
    for (int i = 0; i < 3; i++) d[i] = std::max(0.0, (double)b.mx[i] - (double)b.mn[i]);
    return d[0] * d[1] + d[1] * d[2] + d[2] * d[0];
}

struct BNode {
    BBox box;
    int32_t left = -1, right = -1;   // internal
    int32_t first = 0, count = 0;    // leaf: idx[first, first + count)
};

constexpr int kBins = 32;
// The smallest plane quantum is 2^-PT_WIDE_EMIN_SHIFT of the scene's extent and coordinates; the
// traversal's far-origin line (pt_device.hip PT_WIDE_FAR_EXT) must match it (A/B knobs, one pair).
#ifndef PT_WIDE_EMIN_SHIFT
#define PT_WIDE_EMIN_SHIFT 18
#endif
constexpr double kPrimCost = 1.0;

// Build parameters (tuning knobs, PT_WIDE_MAX_LEAF / PT_WIDE_TRAV_COST): at most kMaxLeaf <= 3
// primitives per leaf (the meta byte's unary count); the SAH weight of a binary node visit
// relative to a primitive test.
int envLeaf() {
    const char* v = std::getenv("PT_WIDE_MAX_LEAF");
    const int x = v ? std::atoi(v) : 0;
    return x >= 1 && x <= 3 ? x : 3;
}
// Subtrees of at most this many primitives are split by an exact sweep over the centroid order on
// each axis instead of bins (PT_WIDE_SWEEP, 0 = bins everywhere; the device build's wave tasks
// sweep up to 64).  Default: 16, and the whole tree of a scene of at most 64 primitives (C2 @1024
// spp 32.1 -> 30.0 ms; C3 and C5 within +-0.2 % for thresholds 8 / 16 / 32, +0.3 % at 64).
int envSweep(int64_t n) {
    const char* v = std::getenv("PT_WIDE_SWEEP");
    const int x = v ? std::atoi(v) : (n <= 64 ? 64 : 16);
    return x < 0 ? 0 : (x > 64 ? 64 : x);
}
double envTrav() {
    const char* v = std::getenv("PT_WIDE_TRAV_COST");
    const double x = v ? std::atof(v) : 0.0;
    return x > 0.0 ? x : 1.0;
}

struct SahBuilder {
    int kMaxLeaf = 3;
    int kSweep = 64;
    double kTravCost = 1.0;
    const BBox* boxes = nullptr;
    std::vector<float> cen;           // centroids, 3 per primitive
    std::vector<int32_t> idx;
    std::vector<BNode> nodes;
    std::atomic<int32_t> next{0};
    std::atomic<int> threads{1};
    int maxThreads = 1;

    int32_t alloc() { return next.fetch_add(1); }

    // Exact sweep SAH (small subtrees): every split position of the centroid order on each axis
    // (ties by primitive index), the cheapest (cost, axis, position); a leaf of at most kMaxLeaf
    // primitives when that is not dearer.
    int32_t sweep(int32_t me, BNode& nd, int32_t first, int32_t count) {
        int32_t ord[3][64];
        double suf[64];
        double bestCost = INFINITY;
        int bestAxis = 0, bestPos = 0;
        for (int a = 0; a < 3; a++) {
            int32_t* o = ord[a];
            std::copy(idx.begin() + first, idx.begin() + first + count, o);
            std::sort(o, o + count, [&](int32_t x, int32_t y) {
                const float cx = cen[3 * x + a], cy = cen[3 * y + a];
                return cx < cy || (cx == cy && x < y);
            });
            BBox acc = emptyBox();
            for (int i = count - 1; i >= 1; i--) {
                growBox(acc, boxes[o[i]]);
                suf[i] = halfArea(acc);
            }
            acc = emptyBox();
            for (int i = 0; i < count - 1; i++) {   // left = o[0..i]
                growBox(acc, boxes[o[i]]);
                const double c = halfArea(acc) * (i + 1) + suf[i + 1] * (count - i - 1);
                if (c < bestCost) {
                    bestCost = c;
                    bestAxis = a;
                    bestPos = i;
                }
            }
        }
        const double area = halfArea(nd.box);
        if (count <= kMaxLeaf && kPrimCost * count * area <= kTravCost * area + kPrimCost * bestCost) {
            nd.first = first;
            nd.count = count;
            nodes[me] = nd;
            return me;
        }
        std::copy(ord[bestAxis], ord[bestAxis] + count, idx.begin() + first);
        const int32_t nl = bestPos + 1;
        const int32_t l = build(first, nl);
        const int32_t r = build(first + nl, count - nl);
        nd.left = l;
        nd.right = r;
        nodes[me] = nd;
        return me;
    }

    int32_t build(int32_t first, int32_t count) {
        const int32_t me = alloc();
        BNode nd;
        nd.box = emptyBox();
        float cmn[3] = {INFINITY, INFINITY, INFINITY}, cmx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int32_t i = first; i < first + count; i++) {
            const int32_t p = idx[i];
            growBox(nd.box, boxes[p]);
            for (int a = 0; a < 3; a++) {
                cmn[a] = std::min(cmn[a], cen[3 * p + a]);
                cmx[a] = std::max(cmx[a], cen[3 * p + a]);
            }
        }
        if (count == 1) {
            nd.first = first;
            nd.count = 1;
            nodes[me] = nd;
            return me;
        }
        if (count <= kSweep) return sweep(me, nd, first, count);
        double bestCost = INFINITY;
        int bestAxis = -1, bestSplit = -1;
        for (int a = 0; a < 3; a++) {
            const double lo = cmn[a], ext = (double)cmx[a] - lo;
            if (!(ext > 0.0)) continue;
            BBox bb[kBins];
            int bc[kBins] = {0};
            for (int i = 0; i < kBins; i++) bb[i] = emptyBox();
            for (int32_t i = first; i < first + count; i++) {
                const int32_t p = idx[i];
                int k = (int)(((double)cen[3 * p + a] - lo) / ext * kBins);
                k = std::min(kBins - 1, std::max(0, k));
                bc[k]++;
                growBox(bb[k], boxes[p]);
            }
            double leftArea[kBins];
            int leftCount[kBins];
            BBox acc = emptyBox();
            int cnt = 0;
            for (int i = 0; i < kBins; i++) {
                growBox(acc, bb[i]);
                cnt += bc[i];
                leftArea[i] = halfArea(acc);
                leftCount[i] = cnt;
            }
            acc = emptyBox();
            cnt = 0;
            for (int i = kBins - 1; i >= 1; i--) {
                growBox(acc, bb[i]);
                cnt += bc[i];
                if (leftCount[i - 1] == 0 || cnt == 0) continue;
                const double c = leftArea[i - 1] * leftCount[i - 1] + halfArea(acc) * cnt;
                if (c < bestCost) {
                    bestCost = c;
                    bestAxis = a;
                    bestSplit = i;
                }
            }
        }
        const double area = halfArea(nd.box);
        const double leafCost = kPrimCost * count * area;
        const double splitCost = kTravCost * area + kPrimCost * bestCost;
        int32_t mid;
        if (bestAxis < 0) {   // all centroids coincide: a leaf if small enough, else split the list
            if (count <= kMaxLeaf) {
                nd.first = first;
                nd.count = count;
                nodes[me] = nd;
                return me;
            }
            mid = first + count / 2;
        } else if (count <= kMaxLeaf && leafCost <= splitCost) {
            nd.first = first;
            nd.count = count;
            nodes[me] = nd;
            return me;
        } else {
            const double lo = cmn[bestAxis], ext = (double)cmx[bestAxis] - lo;
            auto it = std::partition(idx.begin() + first, idx.begin() + first + count, [&](int32_t p) {
                int k = (int)(((double)cen[3 * p + bestAxis] - lo) / ext * kBins);
                k = std::min(kBins - 1, std::max(0, k));
                return k < bestSplit;
            });
            mid = (int32_t)(it - idx.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        const int32_t nl = mid - first, nr = first + count - mid;
        int32_t l = -1, r = -1;
        bool spawned = false;
        if (count > (1 << 14)) {   // large subtrees: the left half on a thread of its own
            if (threads.fetch_add(1) < maxThreads) {
                std::thread t([&] { l = build(first, nl); });
                r = build(mid, nr);
                t.join();
                spawned = true;
            }
            threads.fetch_sub(1);
        }
        if (!spawned) {
            l = build(first, nl);
            r = build(mid, nr);
        }
        nd.left = l;
        nd.right = r;
        nodes[me] = nd;
        return me;
    }
};

uint32_t f2u(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

}  // namespace

std::vector<uint32_t> referenceRanks(const uint32_t* leftRef, const uint32_t* rightRef, size_t stride, int64_t n) {
    std::vector<uint32_t> rank((size_t)std::max<int64_t>(n, 0), 0u);
    if (n <= 1) return rank;
    const uint32_t leaf = 0x80000000u, mask = 0x3fffffffu;
    uint32_t next = 0;
    std::vector<uint32_t> stack{0u};
    while (!stack.empty()) {
        const uint32_t i = stack.back();
        stack.pop_back();
        const uint32_t l = leftRef[(size_t)i * stride], r = rightRef[(size_t)i * stride];
        if (l & leaf) rank[l & mask] = next++;
        if (r & leaf) rank[r & mask] = next++;
        if (!(l & leaf)) stack.push_back(l);
        if (!(r & leaf)) stack.push_back(r);
    }
    return rank;
}

bool buildWide8(const uint32_t* prims, const float* boxes, const uint32_t* rank, int64_t n, Wide8& out,
                std::string& err, double scaleFloor) {
    return buildWide8Leaf(prims, boxes, rank, n, envLeaf(), out, err, scaleFloor);
}

void relocateWide8(Wide8& w, uint32_t nodeBase, uint32_t primBase) {
    for (size_t s = 0; s < w.nodes.size(); s += kW8NodeDwords) {
        w.nodes[s + 4] += nodeBase;
        w.nodes[s + 5] += primBase;
    }
}

bool instanceLeaves(Wide8& top, uint32_t (*instanceOf)(const uint32_t* primRecord),
                    void (*record)(uint32_t id, uint32_t* dst, void* ctx), void* ctx, std::string& err) {
    const size_t nodes0 = top.nodes.size() / kW8NodeDwords;
    for (size_t s = 0; s < nodes0; s++) {
        uint32_t* R = &top.nodes[s * kW8NodeDwords];
        if (R[3] == kW8InstanceFlag) continue;
        uint8_t meta[8];
        for (int j = 0; j < 8; j++) meta[j] = (uint8_t)((j < 4 ? R[6] : R[7]) >> (8 * (j & 3)));
        bool anyInternal = false, anyLeaf = false;
        for (int j = 0; j < 8; j++) {
            if (!meta[j]) continue;
            if ((meta[j] & 0x1f) >= 24) anyInternal = true;
            else anyLeaf = true;
        }
        if (!anyLeaf) continue;
        if (!anyInternal) {   // no child block yet: one for the instance records
            R[4] = (uint32_t)(top.nodes.size() / kW8NodeDwords);
            top.nodes.resize(top.nodes.size() + 8 * (size_t)kW8NodeDwords, 0u);
            R = &top.nodes[s * kW8NodeDwords];
        }
        if ((int64_t)R[4] + 8 > ((int64_t)1 << 24)) {
            err = "instanced BVH: more than 2^24 node slots";
            return false;
        }
        for (int j = 0; j < 8; j++) {
            if (!meta[j] || (meta[j] & 0x1f) >= 24) continue;
            if ((meta[j] >> 5) != 1u) {
                err = "instanced BVH: top-level leaf with more than one instance";
                return false;
            }
            const uint32_t prim = R[5] + (meta[j] & 0x1fu);
            const uint32_t id = instanceOf(&top.prims[(size_t)prim * kW8PrimDwords]);
            record(id, &top.nodes[(size_t)(R[4] + (uint32_t)j) * kW8NodeDwords], ctx);
            meta[j] = (uint8_t)(0x20 | 24 | j);   // an internal child: its slot holds the instance
            top.usedNodes++;
        }
        R[6] = (uint32_t)meta[0] | (uint32_t)meta[1] << 8 | (uint32_t)meta[2] << 16 | (uint32_t)meta[3] << 24;
        R[7] = (uint32_t)meta[4] | (uint32_t)meta[5] << 8 | (uint32_t)meta[6] << 16 | (uint32_t)meta[7] << 24;
    }
    top.prims.clear();   // (the top level has no primitives left)
    return true;
}

bool buildWide8Leaf(const uint32_t* prims, const float* boxes, const uint32_t* rank, int64_t n, int maxLeaf,
                    Wide8& out, std::string& err, double scaleFloor) {
    out = Wide8{};
    if (n <= 0) return true;
    if (n >= (int64_t)1 << 26) {
        err = "wide BVH: more than 2^26 primitives";
        return false;
    }
    SahBuilder B;
    B.kMaxLeaf = std::max(1, std::min(3, maxLeaf));
    B.kTravCost = envTrav();
    B.kSweep = envSweep(n);
    B.boxes = reinterpret_cast<const BBox*>(boxes);
    B.cen.resize((size_t)n * 3);
    B.idx.resize((size_t)n);
    for (int64_t k = 0; k < n; k++) {
        B.idx[k] = (int32_t)k;
        for (int a = 0; a < 3; a++) B.cen[3 * k + a] = 0.5f * (boxes[6 * k + a] + boxes[6 * k + 3 + a]);
    }
    B.nodes.resize((size_t)(2 * n));
    // up to 16 host threads; PT_BUILD_THREADS caps them (several ranks on one host share its cores)
    B.maxThreads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char* bt = std::getenv("PT_BUILD_THREADS"))
        if (std::atoi(bt) > 0) B.maxThreads = std::min(B.maxThreads, std::atoi(bt));
    const int32_t root = B.build(0, (int32_t)n);
    const BBox rootBox = B.nodes[root].box;

    // Smallest plane quantum: far below any box of interest, far above the rounding of the
    // ray arithmetic (|p - o| * inv: about 2^-21.6 |p - o|, for origins within 8 scene extents of
    // the centre -- farther ones are traced in the reference's order, pt_device.hip wideFar):
    // 2^-18 of the larger of the scene's extent and coordinates -- or of `scaleFloor` when that is
    // larger: an instanced mesh's rays arrive in its object space from the whole world
    // (pt_device.hip buildInstanced), so its planes keep the margin for those origins.
    double ext = std::isfinite(scaleFloor) && scaleFloor > 0.0 ? scaleFloor : 0.0;
    for (int a = 0; a < 3; a++)
        ext = std::max({ext, std::fabs((double)rootBox.mn[a]), std::fabs((double)rootBox.mx[a]),
                        (double)rootBox.mx[a] - (double)rootBox.mn[a]});
    int emin = ext > 0.0 ? (int)std::ceil(std::log2(ext)) - PT_WIDE_EMIN_SHIFT : -100;
    emin = std::max(emin, -100);

    // outward margin of the child planes: PT_WIDE_MARGIN=0 one quantum of the node (the round-1..6
    // rule), otherwise the smallest quantum 2^emin (what the rounding bound above needs)
    const char* mg = std::getenv("PT_WIDE_MARGIN");
    const bool nodeMargin = mg && *mg == '0';
    const double minQuantum = std::ldexp(1.0, emin);
    const char* sl = std::getenv("PT_WIDE_SPLIT_LEAVES");
    const bool splitLeaves = !(sl && *sl == '0');
    struct Work { int32_t bnode; int64_t slot; int depth; };
    std::vector<Work> work{{root, 0, 1}};
    out.nodes.assign(kW8NodeDwords, 0u);
    out.usedNodes = 1;
    for (size_t wi = 0; wi < work.size(); wi++) {
        const Work w = work[wi];
        out.depth = std::max(out.depth, w.depth);
        // children: open the largest internal child until 8 (a leaf root is its own single child)
        std::vector<int32_t> ch;
        const BNode bn = B.nodes[w.bnode];
        if (bn.count > 0) ch.push_back(w.bnode);
        else ch = {bn.left, bn.right};
        while (ch.size() < 8) {
            int bi = -1;
            double ba = -1.0;
            for (int i = 0; i < (int)ch.size(); i++) {
                const BNode& c = B.nodes[ch[i]];
                if (c.count == 0 && halfArea(c.box) > ba) {
                    ba = halfArea(c.box);
                    bi = i;
                }
            }
            if (bi < 0) break;
            const BNode& c = B.nodes[ch[bi]];
            const int32_t l = c.left, r = c.right;
            ch[bi] = l;
            ch.insert(ch.begin() + bi + 1, r);
        }
        // free slots left (every internal child opened): split multi-primitive leaves, largest
        // first, so more primitives get a box of their own (the slots are tested anyway)
        while (splitLeaves && ch.size() < 8) {
            int bi = -1;
            for (int i = 0; i < (int)ch.size(); i++) {
                const BNode& c = B.nodes[ch[i]];
                if (c.count > 1 && (bi < 0 || c.count > B.nodes[ch[bi]].count)) bi = i;
            }
            if (bi < 0) break;
            const BNode c = B.nodes[ch[bi]];
            BNode a, b;
            a.first = c.first;
            a.count = 1;
            b.first = c.first + 1;
            b.count = c.count - 1;
            a.box = B.boxes[B.idx[c.first]];
            b.box = emptyBox();
            for (int32_t i = b.first; i < b.first + b.count; i++) growBox(b.box, B.boxes[B.idx[i]]);
            B.nodes.push_back(a);
            ch[bi] = (int32_t)B.nodes.size() - 1;
            B.nodes.push_back(b);
            ch.insert(ch.begin() + bi + 1, (int32_t)B.nodes.size() - 1);
        }
        BBox nb = emptyBox();
        for (int32_t c : ch) growBox(nb, B.nodes[c].box);
        // octant slots: slot j <- the child nearest along direction j (greedy on the projection
        // of the child's centre relative to the node's centre)
        int slotOf[8], childIn[8];
        for (int i = 0; i < 8; i++) slotOf[i] = childIn[i] = -1;
        {
            struct Cand { double cost; int c, s; };
            std::vector<Cand> cand;
            for (int c = 0; c < (int)ch.size(); c++) {
                const BBox& b = B.nodes[ch[c]].box;
                for (int s = 0; s < 8; s++) {
                    double cost = 0.0;
                    for (int a = 0; a < 3; a++) {
                        const double d = 0.5 * ((double)b.mn[a] + b.mx[a]) - 0.5 * ((double)nb.mn[a] + nb.mx[a]);
                        cost += ((s >> a) & 1) ? -d : d;
                    }
                    cand.push_back({cost, c, s});
                }
            }
            std::stable_sort(cand.begin(), cand.end(), [](const Cand& x, const Cand& y) { return x.cost < y.cost; });
            for (const Cand& x : cand)
                if (slotOf[x.c] < 0 && childIn[x.s] < 0) { slotOf[x.c] = x.s; childIn[x.s] = x.c; }
        }
        bool anyInternal = false;
        for (int32_t c : ch) anyInternal |= B.nodes[c].count == 0;
        int64_t childBase = 0;
        if (anyInternal) {
            childBase = (int64_t)(out.nodes.size() / kW8NodeDwords);
            out.nodes.resize(out.nodes.size() + 8 * (size_t)kW8NodeDwords, 0u);
        }
        const int64_t primBase = (int64_t)(out.prims.size() / kW8PrimDwords);
        if (childBase >= ((int64_t)1 << 24) - 8) {
            err = "wide BVH: more than 2^24 node slots";
            return false;
        }
        uint8_t meta[8] = {0};
        int offset = 0;
        for (int s = 0; s < 8; s++) {
            const int c = childIn[s];
            if (c < 0) continue;
            const BNode& cn = B.nodes[ch[c]];
            if (cn.count == 0) {
                meta[s] = (uint8_t)(0x20 | 24 | s);
                work.push_back({ch[c], childBase + s, w.depth + 1});
                out.usedNodes++;
            } else {
                meta[s] = (uint8_t)((((1u << cn.count) - 1u) << 5) | (unsigned)offset);
                for (int i = 0; i < cn.count; i++) {
                    const int32_t k = B.idx[cn.first + i];
                    const uint32_t* src = prims + (size_t)k * kW8PrimDwords;
                    const uint32_t rk = rank ? rank[k] : (uint32_t)k;
                    for (int d = 0; d < kW8PrimDwords; d++) out.prims.push_back(d == 3 ? rk : src[d]);
                }
                offset += cn.count;
                out.leaves++;
            }
        }
        // quantised planes: origin one quantum below the node box, quantum s = 2^e with the
        // node extent <= 251 s, child planes rounded outward by the margin m (the smallest quantum:
        // round 6, C3 @256 spp 134.8 -> 131.2 ms, C5 @64 65.3 -> 62.2, C2 @1024 115.9 -> 114.4, the
        // same frames; 2.1 % fewer node visits, 1.4 % fewer primitive tests)
        uint32_t* R = &out.nodes[(size_t)w.slot * kW8NodeDwords];
        uint8_t qlo[3][8], qhi[3][8];
        uint32_t exps = 0;
        for (int a = 0; a < 3; a++) {
            const double lo = nb.mn[a], hi = nb.mx[a];
            int e = emin;
            if (hi - lo > 0.0) e = std::max(e, (int)std::ceil(std::log2((hi - lo) / 251.0)));
            for (;; e++) {
                if (e > 127 - 1) {
                    err = "wide BVH: scene extent out of range";
                    return false;
                }
                const double s = std::ldexp(1.0, e);
                const double m = nodeMargin ? s : minQuantum;
                float p = (float)(lo - s);
                if ((double)p > lo - s) p = std::nextafter(p, -INFINITY);
                bool ok = true;
                for (int j = 0; j < 8; j++) {
                    const int c = childIn[j];
                    if (c < 0) { qlo[a][j] = 255; qhi[a][j] = 0; continue; }
                    const BBox& b = B.nodes[ch[c]].box;
                    const double ql = std::floor(((double)b.mn[a] - m - (double)p) / s);
                    const double qh = std::ceil(((double)b.mx[a] + m - (double)p) / s);
                    if (!(ql >= 0.0) || !(qh <= 255.0)) { ok = false; break; }
                    qlo[a][j] = (uint8_t)ql;
                    qhi[a][j] = (uint8_t)qh;
                }
                if (!ok) continue;
                R[a] = f2u(p);
                exps |= (uint32_t)(e + 127) << (8 * a);
                break;
            }
        }
        R[3] = exps;
        R[4] = (uint32_t)childBase;
        R[5] = (uint32_t)primBase;
        R[6] = (uint32_t)meta[0] | (uint32_t)meta[1] << 8 | (uint32_t)meta[2] << 16 | (uint32_t)meta[3] << 24;
        R[7] = (uint32_t)meta[4] | (uint32_t)meta[5] << 8 | (uint32_t)meta[6] << 16 | (uint32_t)meta[7] << 24;
        for (int a = 0; a < 3; a++) {
            uint32_t* Q = R + 8 + 4 * a;
            for (int h = 0; h < 2; h++) {
                Q[h] = (uint32_t)qlo[a][4 * h] | (uint32_t)qlo[a][4 * h + 1] << 8 | (uint32_t)qlo[a][4 * h + 2] << 16 |
                       (uint32_t)qlo[a][4 * h + 3] << 24;
                Q[2 + h] = (uint32_t)qhi[a][4 * h] | (uint32_t)qhi[a][4 * h + 1] << 8 |
                           (uint32_t)qhi[a][4 * h + 2] << 16 | (uint32_t)qhi[a][4 * h + 3] << 24;
            }
        }
    }
    if ((int64_t)(out.prims.size() / kW8PrimDwords) != n) {
        err = "wide BVH: primitive count mismatch";
        return false;
    }
    return true;
}

}  // namespace pt
