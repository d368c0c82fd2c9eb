// pt_wide_build.hip — the compressed 8-wide tree built on the device (see host/pt_wide_dev.hpp).
//
// 1. Ranks: leaf k's position in the order RenderManager::hitBvh (utils/render_manager.h:105-133)
//    would test the LBVH's leaves (the tie order of the closest hit), from the leaf up: at each
//    ancestor, the offset of the child's part in its parent's visit (leaf children first, left
//    then right; then the right subtree; then the left one).  = pt::referenceRanks, in parallel.
// 2. Binary tree: top-down SAH (default; "binned SAH" below), or with PT_WIDE_DEVICE_BUILDER=ploc
//    PLOC over the leaves in Morton order.  PLOC pass: every cluster finds its
//    nearest neighbour within kRadius positions (smallest merged surface area; ties by the pair's
//    positions, a strict total order, so the globally closest pair is mutual and every pass
//    merges), mutual pairs merge into a new node at the lower position, survivors are compacted.
//    Each merge also decides, bottom up, whether its subtree (at most 3 primitives) is cheaper as
//    one leaf (SAH: count x area vs traversal x area + the children's costs).
// 3. Collapse + quantisation, one wide level per launch pair: count (children, primitives, child
//    block), exclusive scan, write.  Slots and primitive records are allocated in level order,
//    parents' order, slot order -- the host build's breadth-first order -- so the output is
//    deterministic (the node ids either builder hands out never reach it).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "pt_prims.hpp"
#include "pt_wide8.hpp"
#include "pt_wide_dev.hpp"

#ifndef PT_WIDE_EMIN_SHIFT
#define PT_WIDE_EMIN_SHIFT 18   // the smallest plane quantum, as host/pt_wide8.cpp
#endif

namespace pt {
namespace {

constexpr uint32_t kRefLeaf = 0x80000000u, kRefMask = 0x3fffffffu;
constexpr uint32_t kGroupFlag = 0x80000000u;   // pbox[2 id + 1].w: subtree kept as one leaf
constexpr int kRadiusDefault = 8;              // PLOC neighbourhood (positions on each side; PT_PLOC_RADIUS 8/16/32/64)
constexpr int kTile = 256;
constexpr int kMaxGroup = 3;                   // primitives per leaf (the meta byte's unary count)
constexpr int kMaxLevels = 24;                 // the wide kernels' deepest traversal stack
// device scalars: node counter, cluster count (two slots: a pass reads one, writes the other),
// a level's totals and the error flags (read by the host in one copy)
enum { kMiscNodes = 0, kMiscM = 1, kMiscTotA = 3, kMiscTotB = 4, kMiscTotC = 5, kMiscErr = 6, kMiscWords = 8 };
constexpr int kPassesPerSync = 4;              // PLOC passes enqueued per host read of the cluster count

__device__ __forceinline__ float areaOf(float4 lo, float4 hi) {
    const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
    return dx * dy + dy * dz + dz * dx;
}
__device__ __forceinline__ float4 minBox(float4 a, float4 b) { return make_float4(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z), 0.0f); }
__device__ __forceinline__ float4 maxBox(float4 a, float4 b) { return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), 0.0f); }

// ceil(log2(x)) for x > 0, exactly (frexp is exact; log2 may round across an integer)
__device__ __forceinline__ int ceilLog2(double x) {
    int e = 0;
    const double m = frexp(x, &e);
    return m == 0.5 ? e - 1 : e;
}

// ---------------------------------------------------------------------------------- ranks
__global__ void rankKernel(const float4* __restrict__ lbvh, const int* __restrict__ iparent,
                           const int* __restrict__ lparent, const int2* __restrict__ irange, int n, uint32_t* rank) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint32_t r = 0;
    int child = k, p = lparent[k];
    bool leaf = true;
    for (int guard = 0; p >= 0 && guard < 130; guard++) {
        const float4 refs = lbvh[4 * (size_t)p + 3];
        const uint32_t lref = __float_as_uint(refs.x), rref = __float_as_uint(refs.y);
        const bool lLeaf = lref & kRefLeaf, rLeaf = rref & kRefLeaf;
        const bool isLeft = leaf ? (lLeaf && (int)(lref & kRefMask) == child) : (!lLeaf && (int)lref == child);
        const uint32_t nl = (lLeaf ? 1u : 0u) + (rLeaf ? 1u : 0u);
        if (leaf) r += (!isLeft && lLeaf) ? 1u : 0u;
        else if (!isLeft) r += nl;
        else r += nl + (rLeaf ? 0u : (uint32_t)(irange[rref].y - irange[rref].x + 1));
        child = p;
        leaf = false;
        p = iparent[p];
    }
    rank[k] = r;
}

__global__ void shadeByRankKernel(const float4* __restrict__ shade, const uint32_t* __restrict__ rank, int n, float4* wshade) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const size_t r = rank[k];
    wshade[3 * r] = shade[3 * (size_t)k];
    wshade[3 * r + 1] = shade[3 * (size_t)k + 1];
    wshade[3 * r + 2] = shade[3 * (size_t)k + 2];
}

// ---------------------------------------------------------------------------------- PLOC
// Node ids: leaf k = k, internal = n + j.  pbox[2 id] = {min xyz, SAH cost}, pbox[2 id + 1] =
// {max xyz, primitive count | kGroupFlag}; pchild[j] = the two child ids of internal node n + j.
__global__ void plocInitKernel(const float* __restrict__ leafBoxes, int n, float4* pbox, uint32_t* cid) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float* b = leafBoxes + 6 * (size_t)k;
    const float4 lo = make_float4(b[0], b[1], b[2], 0.0f), hi = make_float4(b[3], b[4], b[5], 0.0f);
    pbox[2 * (size_t)k] = make_float4(lo.x, lo.y, lo.z, areaOf(lo, hi));
    pbox[2 * (size_t)k + 1] = make_float4(hi.x, hi.y, hi.z, __uint_as_float(1u));
    cid[k] = (uint32_t)k;
}

// The PLOC kernels read the cluster count m from the device (several passes run between two
// host reads; the grid covers the count the host last read, an upper bound).
template <int kRadius>
__global__ __launch_bounds__(kTile) void plocNearestKernel(const uint32_t* __restrict__ cid, const float4* __restrict__ pbox,
                                                           const uint32_t* __restrict__ mDev, int* nn) {
    const int m = (int)*mDev;
    __shared__ float4 tlo[kTile + 2 * kRadius], thi[kTile + 2 * kRadius];
    const int base = blockIdx.x * kTile - kRadius;
    for (int t = threadIdx.x; t < kTile + 2 * kRadius; t += kTile) {
        const int j = base + t;
        if (j >= 0 && j < m) {
            const size_t id = cid[j];
            tlo[t] = pbox[2 * id];
            thi[t] = pbox[2 * id + 1];
        }
    }
    __syncthreads();
    const int i = blockIdx.x * kTile + threadIdx.x;
    if (i >= m) return;
    const int ti = threadIdx.x + kRadius;
    const float4 lo = tlo[ti], hi = thi[ti];
    // pairs ordered by (area, |i - j|, min(i, j) odd, min(i, j)): a strict total order on pairs,
    // the same seen from either end, so the globally first pair is mutual; among equal areas
    // adjacent pairs starting at an even position come first, so equal boxes pair off (0,1),
    // (2,3), ... and a pass halves them
    int best = -1;
    float bestA = INFINITY;
    uint64_t bestKey = ~0ull;
    for (int o = -kRadius; o <= kRadius; o++) {
        const int j = i + o;
        if (o == 0 || j < 0 || j >= m) continue;
        const float a = areaOf(minBox(lo, tlo[ti + o]), maxBox(hi, thi[ti + o]));
        const int mn = o < 0 ? j : i;
        const uint64_t key = ((uint64_t)(o < 0 ? -o : o) << 27) | ((uint64_t)(mn & 1) << 26) | (uint64_t)mn;
        if (a < bestA || (a == bestA && key < bestKey)) {
            bestA = a;
            bestKey = key;
            best = j;
        }
    }
    nn[i] = best;
}

// The merged node of the clusters at positions i < j (ids a, b): box, primitive count, SAH cost
// and the leaf decision (count x area vs traversal x area + the children's costs).
__device__ __forceinline__ void makeNode(float4* pbox, uint2* pchild, uint32_t n, uint32_t id, uint32_t a, uint32_t b,
                                         float kTravCost) {
    const float4 la = pbox[2 * (size_t)a], ha = pbox[2 * (size_t)a + 1];
    const float4 lb = pbox[2 * (size_t)b], hb = pbox[2 * (size_t)b + 1];
    const float4 lo = minBox(la, lb), hi = maxBox(ha, hb);
    const float area = areaOf(lo, hi);
    const uint32_t count = (__float_as_uint(ha.w) & ~kGroupFlag) + (__float_as_uint(hb.w) & ~kGroupFlag);
    const float split = kTravCost * area + la.w + lb.w;
    const float asLeaf = count <= (uint32_t)kMaxGroup ? (float)count * area : INFINITY;
    const bool group = asLeaf <= split;
    pbox[2 * (size_t)id] = make_float4(lo.x, lo.y, lo.z, group ? asLeaf : split);
    pbox[2 * (size_t)id + 1] = make_float4(hi.x, hi.y, hi.z, __uint_as_float(count | (group ? kGroupFlag : 0u)));
    pchild[id - n] = make_uint2(a, b);
}

__global__ void plocMergeKernel(uint32_t* cid, float4* pbox, uint2* pchild, const int* __restrict__ nn,
                                const uint32_t* __restrict__ mDev, int mGrid, int n, float kTravCost, uint32_t* flag,
                                uint32_t* misc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = (int)*mDev;
    const int j = i < m ? nn[i] : -1;
    const bool mutual = j >= 0 && nn[j] == i;
    const bool merge = mutual && i < j;
    // node ids: one counter add per wave
    const uint64_t mask = __ballot(merge);
    uint32_t base = 0;
    if (mask) {
        const int leader = __builtin_ctzll(mask);
        if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(misc + kMiscNodes, (uint32_t)__popcll(mask));
        base = __shfl(base, leader);
    }
    if (i >= mGrid) return;
    // flags: 1 = the position survives (0 beyond m: the scan runs over the grid's range)
    flag[i] = (i < m && !(mutual && i > j)) ? 1u : 0u;
    if (!merge) return;
    const uint32_t id = (uint32_t)n + base + (uint32_t)__popcll(mask & ((1ull << (threadIdx.x & 63)) - 1ull));
    makeNode(pbox, pchild, (uint32_t)n, id, cid[i], cid[j], kTravCost);
    cid[i] = id;
}

// The last passes (m <= kTailMax clusters) in one workgroup: no launches or host reads per pass.
constexpr int kTailThreads = 1024, kTailMax = 16384;
template <int kRadius>
__global__ __launch_bounds__(kTailThreads) void plocTailKernel(uint32_t* cidA, uint32_t* cidB, float4* pbox, uint2* pchild,
                                                               int* nn, uint32_t* flag, const uint32_t* __restrict__ mDev,
                                                               uint32_t* misc, int n, float kTravCost) {
    __shared__ uint32_t sNodes, sM, sums[kTailThreads];
    const int t = threadIdx.x;
    if (t == 0) {
        sNodes = misc[kMiscNodes];
        sM = *mDev;
    }
    __syncthreads();
    uint32_t* cur = cidA;
    uint32_t* nxt = cidB;
    int m = (int)sM;
    while (m > 1) {
        for (int i = t; i < m; i += kTailThreads) {   // nearest neighbour (the same rule as plocNearestKernel)
            const uint32_t ci = cur[i];
            const float4 lo = pbox[2 * (size_t)ci], hi = pbox[2 * (size_t)ci + 1];
            int best = -1;
            float bestA = INFINITY;
            uint64_t bestKey = ~0ull;
            for (int o = -kRadius; o <= kRadius; o++) {
                const int j = i + o;
                if (o == 0 || j < 0 || j >= m) continue;
                const uint32_t cj = cur[j];
                const float a = areaOf(minBox(lo, pbox[2 * (size_t)cj]), maxBox(hi, pbox[2 * (size_t)cj + 1]));
                const int mn = o < 0 ? j : i;
                const uint64_t key = ((uint64_t)(o < 0 ? -o : o) << 27) | ((uint64_t)(mn & 1) << 26) | (uint64_t)mn;
                if (a < bestA || (a == bestA && key < bestKey)) {
                    bestA = a;
                    bestKey = key;
                    best = j;
                }
            }
            nn[i] = best;
        }
        __syncthreads();
        for (int i = t; i < m; i += kTailThreads) {   // merges
            const int j = nn[i];
            const bool mutual = j >= 0 && nn[j] == i;
            flag[i] = (mutual && i > j) ? 0u : 1u;
            if (mutual && i < j) {
                const uint32_t id = (uint32_t)n + atomicAdd(&sNodes, 1u);
                makeNode(pbox, pchild, (uint32_t)n, id, cur[i], cur[j], kTravCost);
                cur[i] = id;
            }
        }
        __syncthreads();
        // compaction in order: thread t owns the contiguous chunk [t * c, (t + 1) * c)
        const int c = (m + kTailThreads - 1) / kTailThreads;
        const int lo = min(m, t * c), hi = min(m, lo + c);
        uint32_t cnt = 0;
        for (int i = lo; i < hi; i++) cnt += flag[i];
        sums[t] = cnt;
        __syncthreads();
        for (int off = 1; off < kTailThreads; off <<= 1) {   // inclusive scan of the chunk counts
            const uint32_t v = t >= off ? sums[t - off] : 0u;
            __syncthreads();
            sums[t] += v;
            __syncthreads();
        }
        uint32_t pos = sums[t] - cnt;
        for (int i = lo; i < hi; i++)
            if (flag[i]) nxt[pos++] = cur[i];
        const int mNext = (int)sums[kTailThreads - 1];
        __syncthreads();
        uint32_t* tmp = cur;
        cur = nxt;
        nxt = tmp;
        m = mNext;
    }
    if (t == 0) {   // the root, wherever the host expects the final clusters
        cidA[0] = cur[0];
        cidB[0] = cur[0];
        misc[kMiscNodes] = sNodes;
    }
}

__global__ void plocCompactKernel(const uint32_t* __restrict__ cid, const uint32_t* __restrict__ flag,
                                  const uint32_t* __restrict__ pos, const uint32_t* __restrict__ mDev, uint32_t* out,
                                  uint32_t* mNext) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = (int)*mDev;
    if (i >= m) return;
    if (flag[i]) out[pos[i]] = cid[i];
    if (i == m - 1) *mNext = pos[i] + flag[i];
}

// ---------------------------------------------------------------------------------- collapse
struct Tree {
    const float4* pbox;
    const uint2* pchild;
    uint32_t n;
    __device__ bool group(uint32_t id) const { return id < n || (__float_as_uint(pbox[2 * (size_t)id + 1].w) & kGroupFlag); }
    __device__ uint32_t count(uint32_t id) const { return id < n ? 1u : (__float_as_uint(pbox[2 * (size_t)id + 1].w) & ~kGroupFlag); }
    __device__ float area(uint32_t id) const { return areaOf(pbox[2 * (size_t)id], pbox[2 * (size_t)id + 1]); }
};

// The children of the wide node over binary node `root` (the host build's rule,
// pt_wide8.cpp): open the internal child of largest area until 8; with slots still free, open
// multi-primitive leaves (their parts stay leaves).  Returns the child count; grp[i] = leaf.
__device__ int collapse(const Tree& T, uint32_t root, uint32_t ch[8], bool grp[8]) {
    int c;
    if (T.group(root)) {
        ch[0] = root;
        grp[0] = true;
        c = 1;
    } else {
        const uint2 k = T.pchild[root - T.n];
        ch[0] = k.x;
        ch[1] = k.y;
        grp[0] = T.group(k.x);
        grp[1] = T.group(k.y);
        c = 2;
    }
    for (int phase = 0; phase < 2; phase++) {
        while (c < 8) {
            int bi = -1;
            float ba = -1.0f;
            uint32_t bc = 0;
            for (int i = 0; i < c; i++) {
                const bool open = phase == 0 ? !grp[i] : (grp[i] && ch[i] >= T.n);
                if (!open) continue;
                // largest area; among equal areas the most primitives (equal boxes open breadth first)
                const float a = T.area(ch[i]);
                const uint32_t cn = T.count(ch[i]);
                if (a > ba || (a == ba && cn > bc)) {
                    ba = a;
                    bc = cn;
                    bi = i;
                }
            }
            if (bi < 0) break;
            const uint2 k = T.pchild[ch[bi] - T.n];
            const bool inGroup = grp[bi];
            for (int i = c; i > bi + 1; i--) {
                ch[i] = ch[i - 1];
                grp[i] = grp[i - 1];
            }
            ch[bi] = k.x;
            ch[bi + 1] = k.y;
            grp[bi] = inGroup || T.group(k.x);
            grp[bi + 1] = inGroup || T.group(k.y);
            c++;
        }
    }
    return c;
}

__global__ void setRootKernel(const uint32_t* __restrict__ cid, uint2* items) { items[0] = make_uint2(cid[0], 0u); }

__global__ void wideCountKernel(Tree T, const uint2* __restrict__ items, int m, uint4* cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint32_t ch[8];
    bool grp[8];
    const int c = collapse(T, items[i].x, ch, grp);
    uint32_t prims = 0, internal = 0;
    for (int j = 0; j < c; j++) {
        if (grp[j]) prims += T.count(ch[j]);
        else internal++;
    }
    cnt[i] = make_uint4(internal ? 8u : 0u, prims, internal, 0u);
}

__global__ void wideWriteKernel(Tree T, const uint2* __restrict__ items, int m, const uint4* __restrict__ cnt,
                                const uint4* __restrict__ ofs, uint32_t nodeBase, uint32_t primBase, uint32_t slotCap,
                                const uint32_t* __restrict__ rootCid, const float4* __restrict__ prims,
                                const uint32_t* __restrict__ rank, uint32_t* nodes, uint4* wprims, uint2* next,
                                uint32_t* misc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint4 o = ofs[i];
    if (i == m - 1) {
        const uint4 c = cnt[i];
        misc[kMiscTotA] = o.x + c.x;
        misc[kMiscTotB] = o.y + c.y;
        misc[kMiscTotC] = o.z + c.z;
    }
    uint32_t ch[8];
    bool grp[8];
    const uint2 item = items[i];
    const int c = collapse(T, item.x, ch, grp);
    const uint32_t childBase = nodeBase + o.x, myPrims = primBase + o.y;
    bool anyInternal = false;
    for (int j = 0; j < c; j++) anyInternal |= !grp[j];
    if (item.y >= slotCap || (anyInternal && childBase + 8u > slotCap)) {
        atomicOr(misc + kMiscErr, 1u);
        return;
    }
    // smallest plane quantum: 2^-18 of the scene extent (the host build's rule, pt_wide8.cpp)
    const uint32_t root = *rootCid;
    const float4 rlo = T.pbox[2 * (size_t)root], rhi = T.pbox[2 * (size_t)root + 1];
    double ext = 0.0;
    {
        const float l[3] = {rlo.x, rlo.y, rlo.z}, h[3] = {rhi.x, rhi.y, rhi.z};
        for (int a = 0; a < 3; a++)
            ext = fmax(ext, fmax(fabs((double)l[a]), fmax(fabs((double)h[a]), (double)h[a] - (double)l[a])));
    }
    int emin = ext > 0.0 ? ceilLog2(ext) - PT_WIDE_EMIN_SHIFT : -100;
    emin = emin < -100 ? -100 : emin;
    const double minQuantum = ldexp(1.0, emin);

    float cmn[8][3], cmx[8][3];
    float nmn[3] = {INFINITY, INFINITY, INFINITY}, nmx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int j = 0; j < c; j++) {
        const float4 lo = T.pbox[2 * (size_t)ch[j]], hi = T.pbox[2 * (size_t)ch[j] + 1];
        cmn[j][0] = lo.x; cmn[j][1] = lo.y; cmn[j][2] = lo.z;
        cmx[j][0] = hi.x; cmx[j][1] = hi.y; cmx[j][2] = hi.z;
        for (int a = 0; a < 3; a++) {
            nmn[a] = fminf(nmn[a], cmn[j][a]);
            nmx[a] = fmaxf(nmx[a], cmx[j][a]);
        }
    }
    // octant slots: greedy on the projection of the child's centre (the host build's rule:
    // candidates in increasing cost, ties in (child, slot) order)
    int slotOf[8], childIn[8];
    for (int j = 0; j < 8; j++) slotOf[j] = childIn[j] = -1;
    for (int round = 0; round < c; round++) {
        double bc = INFINITY;
        int bj = -1, bs = -1;
        for (int j = 0; j < c; j++) {
            if (slotOf[j] >= 0) continue;
            for (int s = 0; s < 8; s++) {
                if (childIn[s] >= 0) continue;
                double cost = 0.0;
                for (int a = 0; a < 3; a++) {
                    const double d = 0.5 * ((double)cmn[j][a] + cmx[j][a]) - 0.5 * ((double)nmn[a] + nmx[a]);
                    cost += ((s >> a) & 1) ? -d : d;
                }
                if (cost < bc) {
                    bc = cost;
                    bj = j;
                    bs = s;
                }
            }
        }
        slotOf[bj] = bs;
        childIn[bs] = bj;
    }
    uint32_t meta[2] = {0u, 0u};
    uint32_t offset = 0, nextPos = o.z;
    for (int s = 0; s < 8; s++) {
        const int j = childIn[s];
        if (j < 0) continue;
        uint32_t mb;
        if (!grp[j]) {
            mb = 0x20u | 24u | (uint32_t)s;
            next[nextPos++] = make_uint2(ch[j], childBase + (uint32_t)s);
        } else {
            const uint32_t cntj = T.count(ch[j]);
            mb = (((1u << cntj) - 1u) << 5) | offset;
            // the group's primitives, left to right
            uint32_t st[4];
            int sp = 0;
            st[sp++] = ch[j];
            while (sp > 0) {
                const uint32_t x = st[--sp];
                if (x < T.n) {
                    const float4* src = prims + 3 * (size_t)x;
                    uint4* dst = wprims + 3 * (size_t)(myPrims + offset);
                    const float4 p0 = src[0], p1 = src[1], p2 = src[2];
                    dst[0] = make_uint4(__float_as_uint(p0.x), __float_as_uint(p0.y), __float_as_uint(p0.z), rank[x]);
                    dst[1] = make_uint4(__float_as_uint(p1.x), __float_as_uint(p1.y), __float_as_uint(p1.z), __float_as_uint(p1.w));
                    dst[2] = make_uint4(__float_as_uint(p2.x), __float_as_uint(p2.y), __float_as_uint(p2.z), __float_as_uint(p2.w));
                    offset++;
                } else if (sp <= 2) {
                    const uint2 k = T.pchild[x - T.n];
                    st[sp++] = k.y;
                    st[sp++] = k.x;
                } else {
                    atomicOr(misc + kMiscErr, 2u);
                    break;
                }
            }
        }
        meta[s >> 2] |= mb << (8 * (s & 3));
    }
    // quantised planes (pt_wide8.cpp): origin below the node box, quantum 2^e with the node
    // extent <= 251 quanta, child planes rounded outward by the smallest quantum 2^emin (the margin the
    // traversal's rounding bound needs; pt_wide8.cpp)
    uint32_t R[20];
    uint32_t exps = 0;
    for (int a = 0; a < 3; a++) {
        const double lo = nmn[a], hi = nmx[a];
        int e = emin;
        if (hi - lo > 0.0) e = max(e, ceilLog2((hi - lo) / 251.0));
        uint32_t ql[2] = {0u, 0u}, qh[2] = {0u, 0u};
        for (;; e++) {
            if (e > 126) {
                atomicOr(misc + kMiscErr, 4u);
                return;
            }
            const double s = ldexp(1.0, e);
            float p = (float)(lo - s);
            if ((double)p > lo - s) p = nextafterf(p, -INFINITY);
            bool ok = true;
            ql[0] = ql[1] = qh[0] = qh[1] = 0u;
            for (int sl = 0; sl < 8; sl++) {
                const int j = childIn[sl];
                uint32_t l8 = 255u, h8 = 0u;
                if (j >= 0) {
                    const double qlo = floor(((double)cmn[j][a] - minQuantum - (double)p) / s);
                    const double qhi = ceil(((double)cmx[j][a] + minQuantum - (double)p) / s);
                    if (!(qlo >= 0.0) || !(qhi <= 255.0)) {
                        ok = false;
                        break;
                    }
                    l8 = (uint32_t)qlo;
                    h8 = (uint32_t)qhi;
                }
                ql[sl >> 2] |= l8 << (8 * (sl & 3));
                qh[sl >> 2] |= h8 << (8 * (sl & 3));
            }
            if (!ok) continue;
            R[a] = __float_as_uint(p);
            exps |= (uint32_t)(e + 127) << (8 * a);
            R[8 + 4 * a] = ql[0];
            R[9 + 4 * a] = ql[1];
            R[10 + 4 * a] = qh[0];
            R[11 + 4 * a] = qh[1];
            break;
        }
    }
    R[3] = exps;
    R[4] = anyInternal ? childBase : 0u;
    R[5] = myPrims;
    R[6] = meta[0];
    R[7] = meta[1];
    uint4* dst = reinterpret_cast<uint4*>(nodes + (size_t)pt::kW8NodeDwords * (size_t)item.y);
    for (int q = 0; q < 5; q++) dst[q] = make_uint4(R[4 * q], R[4 * q + 1], R[4 * q + 2], R[4 * q + 3]);
}

// ---------------------------------------------------------------------------------- binned SAH
// Step 2 by top-down SAH instead of PLOC (PT_WIDE_DEVICE_BUILDER=sah, the default): the host
// build's rule (pt_wide8.cpp: centroid bins per axis -- 32 here, 64 there --, the split minimising count x area summed
// over the two sides, subtrees of at most 3 primitives kept as one leaf group when that is
// cheaper) run on the device.  Tasks -- a node and its primitives, contiguous in `ref` -- of more
// than kWaveTask primitives are split level by level: one block per kChunk primitives bins its part
// in LDS (a task of one block then picks its split itself; bigger tasks merge their blocks' bins
// with atomics on order-preserving integers and pick it in one more launch), and a stable partition
// from per-block counts and a scan.  A task of at most kWaveTask primitives is finished by one
// wave, a primitive per lane, every node of a level at once: sweep SAH over the centroid order on
// each axis (a bitonic sort across the lanes, segmented prefix / suffix box scans) -- an exact
// sweep, not bins, at this size.  Node ids come from an atomic counter and never reach the output
// (the collapse walks the tree by structure), so the wide tree is deterministic.
constexpr int kBins = 32;
constexpr int kWaveTask = 64;           // tasks a wave finishes
constexpr int kChunk = 2048;            // primitives per block of a large task (256 threads x 8)
constexpr int kPerThread = kChunk / 256;
constexpr int kBinWords = 16;           // per bin: count, box lo / hi, centroid lo / hi (ordered), pad
constexpr uint32_t kNoSlot = 0xffffffffu;
// device counters: nodes allocated, next level's large tasks, wave tasks, error flag, final node
// count, this level's blocks and tasks of several blocks
enum { kSahNodes = 0, kSahLarge = 1, kSahSmall = 2, kSahErr = 3, kSahTotal = 4, kSahBlocks = 5, kSahMulti = 6, kSahWords = 8 };
struct SahTask {                        // 80 B
    uint32_t begin, count, node, firstBlock;
    float lo[3], hi[3], clo[3], chi[3];
    uint32_t binSlot, pad[3];           // global bins of a task of several blocks (kNoSlot: one block)
};
struct SahSplit {                       // the split and the two children's box / centroid box
    uint32_t axis, bin, left, median;
    float child[2][12];                 // lo xyz, hi xyz, centroid lo xyz, centroid hi xyz
};

// floats as unsigned integers of the same order (atomic min / max on boxes)
__device__ __forceinline__ uint32_t ordF(float f) {
    const uint32_t u = __float_as_uint(f);
    return u ^ ((u >> 31) ? 0xffffffffu : 0x80000000u);
}
__device__ __forceinline__ float unordF(uint32_t u) { return __uint_as_float(u ^ ((u >> 31) ? 0x80000000u : 0xffffffffu)); }

__device__ __forceinline__ int binOf(float c, float lo, float hi) {
    const float ext = hi - lo;
    if (!(ext > 0.0f)) return 0;
    const int b = (int)((c - lo) * ((float)kBins / ext));
    return b < 0 ? 0 : (b >= kBins ? kBins - 1 : b);
}
__device__ __forceinline__ float halfArea3(const float* lo, const float* hi) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return dx * dy + dy * dz + dz * dx;
}

// bins (u32 words): [axis][bin][kBinWords] = count, lo xyz, hi xyz, clo xyz, chi xyz (ordered floats)
__device__ __forceinline__ bool binMinWord(int w) { return (w >= 1 && w <= 3) || (w >= 7 && w <= 9); }
__device__ __forceinline__ void binInit(uint32_t* b) {
    for (int w = 0; w < 13; w++) b[w] = binMinWord(w) ? 0xffffffffu : 0u;
}

// The best split of a task from its bins (LDS or global), by the first 96 threads of a block: thread
// = (axis, bin); inclusive prefix (bins 0..b) and suffix (bins b..31) of the count and of the box
// and centroid bounds within each axis's 32 lanes; cost of a split after bin b = left count x
// area + right count x area, the minimum over (cost, axis, bin) -- the host build's rule and tie
// order.  Empty bins hold NaN bounds (the min / max identities), which fminf / fmaxf skip.
struct SweepLds {
    uint64_t key[3];
    float child[2][12];
    uint32_t left;
};
__device__ void sweepSplit(const uint32_t* B, const SahTask& t, SahSplit* out, SweepLds& sl) {
    const int tid = (int)threadIdx.x, axis = tid >> 5, b = tid & 31;
    const bool on = tid < 3 * kBins;
    uint32_t pc = 0, sc = 0;
    float pv[12], sv[12];
    const uint32_t* x = B + (on ? (axis * kBins + b) * kBinWords : 0);
    pc = sc = on ? x[0] : 0u;
    for (int w = 0; w < 12; w++) pv[w] = sv[w] = unordF(on ? x[1 + w] : 0u);
    for (int off = 1; off < kBins; off <<= 1) {
        const uint32_t ac = __shfl_up(pc, off, kBins), bc = __shfl_down(sc, off, kBins);
        const bool inL = b >= off, inR = b + off < kBins;
        if (inL) pc += ac;
        if (inR) sc += bc;
        for (int w = 0; w < 12; w++) {
            const float av = __shfl_up(pv[w], off, kBins), bv = __shfl_down(sv[w], off, kBins);
            const bool mn = binMinWord(1 + w);
            if (inL) pv[w] = mn ? fminf(pv[w], av) : fmaxf(pv[w], av);
            if (inR) sv[w] = mn ? fminf(sv[w], bv) : fmaxf(sv[w], bv);
        }
    }
    // the right side of a split after bin b: the suffix from b + 1
    const uint32_t rc = __shfl_down(sc, 1, kBins);
    float rv[12];
    for (int w = 0; w < 12; w++) rv[w] = __shfl_down(sv[w], 1, kBins);
    uint64_t key = ~0ull;
    if (on && b < kBins - 1 && pc > 0 && rc > 0) {
        const float cost = (float)pc * halfArea3(pv, pv + 3) + (float)rc * halfArea3(rv, rv + 3);
        key = ((uint64_t)ordF(cost) << 32) | ((uint64_t)axis << 8) | (uint64_t)b;
    }
    for (int off = 1; off < kBins; off <<= 1) {
        const uint64_t o = __shfl_xor(key, off, kBins);
        key = o < key ? o : key;
    }
    if (on && b == 0) sl.key[axis] = key;
    __syncthreads();
    uint64_t best = sl.key[0];
    best = sl.key[1] < best ? sl.key[1] : best;
    best = sl.key[2] < best ? sl.key[2] : best;
    if (best != ~0ull && on && axis == (int)((best >> 8) & 3u) && b == (int)(best & 31u)) {
        for (int w = 0; w < 12; w++) {
            sl.child[0][w] = pv[w];
            sl.child[1][w] = rv[w];
        }
        sl.left = pc;
    }
    __syncthreads();
    if (tid != 0) return;
    SahSplit& s = *out;
    if (best == ~0ull) {   // every centroid in one bin on every axis (coincident centroids): split at the middle
        s.axis = 0; s.bin = 0; s.left = t.count / 2; s.median = 1;
        for (int side = 0; side < 2; side++)
            for (int a = 0; a < 3; a++) {   // the parent's boxes bound either half
                s.child[side][a] = t.lo[a]; s.child[side][3 + a] = t.hi[a];
                s.child[side][6 + a] = t.clo[a]; s.child[side][9 + a] = t.chi[a];
            }
        return;
    }
    s.axis = (uint32_t)((best >> 8) & 3u); s.bin = (uint32_t)(best & 31u); s.left = sl.left; s.median = 0;
    for (int w = 0; w < 12; w++) {
        s.child[0][w] = sl.child[0][w];
        s.child[1][w] = sl.child[1][w];
    }
}

__device__ __forceinline__ void writeNodeBox(float4* pbox, uint32_t id, const float* lo, const float* hi, uint32_t count,
                                             bool group) {
    pbox[2 * (size_t)id] = make_float4(lo[0], lo[1], lo[2], 0.0f);
    pbox[2 * (size_t)id + 1] = make_float4(hi[0], hi[1], hi[2], __uint_as_float(count | (group ? kGroupFlag : 0u)));
}

// centroids, the identity order, the leaves' boxes, and the scene's box and centroid box (block
// reduction + atomics)
__global__ __launch_bounds__(256) void sahInitKernel(const float* __restrict__ leafBoxes, int n, float4* cen, uint32_t* ref,
                                                     float4* pbox, uint32_t* rootAcc) {
    __shared__ uint32_t acc[12];
    if (threadIdx.x < 12) acc[threadIdx.x] = (threadIdx.x % 6) < 3 ? 0xffffffffu : 0u;
    __syncthreads();
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v[12];
    for (int w = 0; w < 12; w++) v[w] = (w % 6) < 3 ? 0xffffffffu : 0u;
    if (k < n) {
        const float* b = leafBoxes + 6 * (size_t)k;
        const float c[3] = {0.5f * (b[0] + b[3]), 0.5f * (b[1] + b[4]), 0.5f * (b[2] + b[5])};
        cen[k] = make_float4(c[0], c[1], c[2], 0.0f);
        ref[k] = (uint32_t)k;
        writeNodeBox(pbox, (uint32_t)k, b, b + 3, 1u, false);
        for (int a = 0; a < 3; a++) {
            v[a] = ordF(b[a]);
            v[3 + a] = ordF(b[3 + a]);
            v[6 + a] = v[9 + a] = ordF(c[a]);
        }
    }
    for (int w = 0; w < 12; w++) {   // wave reduction, one LDS atomic per wave
        uint32_t x = v[w];
        for (int off = 32; off > 0; off >>= 1) {
            const uint32_t y = __shfl_xor(x, off);
            x = (w % 6) < 3 ? min(x, y) : max(x, y);
        }
        if ((threadIdx.x & 63) == 0) {
            if ((w % 6) < 3) atomicMin(&acc[w], x);
            else atomicMax(&acc[w], x);
        }
    }
    __syncthreads();
    if (threadIdx.x < 12) {
        if ((threadIdx.x % 6) < 3) atomicMin(rootAcc + threadIdx.x, acc[threadIdx.x]);
        else atomicMax(rootAcc + threadIdx.x, acc[threadIdx.x]);
    }
}

__global__ void sahRootKernel(const uint32_t* __restrict__ rootAcc, int n, float4* pbox, SahTask* large, SahTask* small,
                              uint32_t* cnt, uint32_t* rootCid) {
    SahTask t;
    t.begin = 0;
    t.count = (uint32_t)n;
    t.node = (uint32_t)n;
    t.firstBlock = 0;
    t.binSlot = kNoSlot;
    t.pad[0] = t.pad[1] = t.pad[2] = 0u;
    for (int a = 0; a < 3; a++) {
        t.lo[a] = unordF(rootAcc[a]);
        t.hi[a] = unordF(rootAcc[3 + a]);
        t.clo[a] = unordF(rootAcc[6 + a]);
        t.chi[a] = unordF(rootAcc[9 + a]);
    }
    writeNodeBox(pbox, t.node, t.lo, t.hi, (uint32_t)n, false);
    *rootCid = t.node;
    cnt[kSahNodes] = 1u;
    if (n > kWaveTask) {
        large[0] = t;
        cnt[kSahLarge] = 1u;
        cnt[kSahSmall] = 0u;
    } else {
        small[0] = t;
        cnt[kSahLarge] = 0u;
        cnt[kSahSmall] = 1u;
    }
}

// A level's block map on the device: blocks per task (kChunk primitives each) and whether the task
// needs global bins, an exclusive scan of both, then each task writes its blocks and bin slot.
__global__ void sahMapCountKernel(const SahTask* __restrict__ tasks, int ntask, uint4* need) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ntask) return;
    const uint32_t c = tasks[i].count;
    need[i] = make_uint4((c + kChunk - 1) / kChunk, c > (uint32_t)kChunk ? 1u : 0u, 0u, 0u);
}
__global__ void sahMapWriteKernel(SahTask* tasks, int ntask, const uint4* __restrict__ need, const uint4* __restrict__ ofs,
                                  uint2* blockTask, uint32_t* multiTask, uint32_t* cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ntask) return;
    const uint4 nd = need[i], o = ofs[i];
    SahTask& t = tasks[i];
    t.firstBlock = o.x;
    t.binSlot = nd.y ? o.y : kNoSlot;
    if (nd.y) multiTask[o.y] = (uint32_t)i;
    for (uint32_t b = 0; b < nd.x; b++) blockTask[o.x + b] = make_uint2((uint32_t)i, t.begin + b * (uint32_t)kChunk);
    if (i == ntask - 1) {
        cnt[kSahBlocks] = o.x + nd.x;
        cnt[kSahMulti] = o.y + nd.y;
    }
}

// (grids sized by the host's upper bound; the device counts say how much of them is work)
__global__ void sahZeroBinsKernel(uint32_t* bins, const uint32_t* __restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (int)cnt[kSahMulti] * 3 * kBins) binInit(bins + (size_t)i * kBinWords);
}

// One block per (task, chunk of kChunk primitives): LDS bins.  A thread takes kPerThread
// consecutive primitives and adds a run of primitives in the same bin to the LDS bin once
// (neighbours in `ref` are neighbours in space: their Morton order, stably partitioned).  A task of
// one block then picks its split here; a bigger task's bins go to its global bins.
__global__ __launch_bounds__(256) void sahBinKernel(const SahTask* __restrict__ tasks, const uint2* __restrict__ blockTask,
                                                    const uint32_t* __restrict__ ref, const float4* __restrict__ cen,
                                                    const float* __restrict__ leafBoxes, uint32_t* bins, SahSplit* splits,
                                                    const uint32_t* __restrict__ cnt) {
    __shared__ uint32_t lb[3 * kBins * kBinWords];
    __shared__ SweepLds sl;
    if (blockIdx.x >= cnt[kSahBlocks]) return;
    for (int i = threadIdx.x; i < 3 * kBins; i += 256) binInit(lb + i * kBinWords);
    __syncthreads();
    const uint2 bt = blockTask[blockIdx.x];
    const SahTask& t = tasks[bt.x];
    const uint32_t end = min(t.begin + t.count, bt.y + (uint32_t)kChunk);
    const uint32_t i0 = bt.y + threadIdx.x * kPerThread;
    const int here = end > i0 ? min(kPerThread, (int)(end - i0)) : 0;
    // this thread's primitives, every load issued before the first use
    uint32_t kk[kPerThread];
    float4 c4[kPerThread];
    float2 bx[kPerThread][3];
#pragma unroll
    for (int r = 0; r < kPerThread; r++) kk[r] = r < here ? ref[i0 + r] : 0u;
#pragma unroll
    for (int r = 0; r < kPerThread; r++) {
        if (r < here) {
            const float2* b2 = reinterpret_cast<const float2*>(leafBoxes + 6 * (size_t)kk[r]);
            c4[r] = cen[kk[r]];
            bx[r][0] = b2[0]; bx[r][1] = b2[1]; bx[r][2] = b2[2];
        }
    }
    for (int a = 0; a < 3; a++) {
        int run = -1;
        uint32_t rc = 0, acc[12];
#pragma unroll
        for (int r = 0; r < kPerThread; r++) {
            if (r >= here) continue;
            const float c = a == 0 ? c4[r].x : (a == 1 ? c4[r].y : c4[r].z);
            const int b = binOf(c, t.clo[a], t.chi[a]);
            const uint32_t v[12] = {ordF(bx[r][0].x), ordF(bx[r][0].y), ordF(bx[r][1].x), ordF(bx[r][1].y),
                                    ordF(bx[r][2].x), ordF(bx[r][2].y), ordF(c4[r].x),   ordF(c4[r].y),
                                    ordF(c4[r].z),   ordF(c4[r].x),   ordF(c4[r].y),   ordF(c4[r].z)};
            if (b != run) {
                if (run >= 0) {
                    uint32_t* y = lb + (a * kBins + run) * kBinWords;
                    atomicAdd(y, rc);
                    for (int w = 0; w < 12; w++) {
                        if (binMinWord(1 + w)) atomicMin(y + 1 + w, acc[w]);
                        else atomicMax(y + 1 + w, acc[w]);
                    }
                }
                run = b;
                rc = 0;
                for (int w = 0; w < 12; w++) acc[w] = v[w];
            }
            rc++;
            for (int w = 0; w < 12; w++) acc[w] = binMinWord(1 + w) ? min(acc[w], v[w]) : max(acc[w], v[w]);
        }
        if (run >= 0) {
            uint32_t* y = lb + (a * kBins + run) * kBinWords;
            atomicAdd(y, rc);
            for (int w = 0; w < 12; w++) {
                if (binMinWord(1 + w)) atomicMin(y + 1 + w, acc[w]);
                else atomicMax(y + 1 + w, acc[w]);
            }
        }
    }
    __syncthreads();
    if (t.binSlot == kNoSlot) {   // the whole task: pick the split
        sweepSplit(lb, t, splits + bt.x, sl);
        return;
    }
    uint32_t* g = bins + (size_t)t.binSlot * 3 * kBins * kBinWords;
    for (int i = threadIdx.x; i < 3 * kBins; i += 256) {
        const uint32_t* x = lb + i * kBinWords;
        if (!x[0]) continue;
        uint32_t* y = g + i * kBinWords;
        atomicAdd(y, x[0]);
        for (int w = 1; w < 13; w++) {
            if (binMinWord(w)) atomicMin(y + w, x[w]);
            else atomicMax(y + w, x[w]);
        }
    }
}

// one block per task of several blocks (multiTask: task indices): the split from the merged bins
__global__ __launch_bounds__(128) void sahSplitKernel(const SahTask* __restrict__ tasks, const uint32_t* __restrict__ multiTask,
                                                      const uint32_t* __restrict__ bins, SahSplit* splits,
                                                      const uint32_t* __restrict__ cnt) {
    __shared__ SweepLds sl;
    if (blockIdx.x >= cnt[kSahMulti]) return;
    const uint32_t ti = multiTask[blockIdx.x];
    const SahTask& t = tasks[ti];
    sweepSplit(bins + (size_t)t.binSlot * 3 * kBins * kBinWords, t, splits + ti, sl);
}

__device__ __forceinline__ bool goesRight(const SahTask& t, const SahSplit& s, uint32_t pos, const float4* cen, uint32_t k) {
    if (s.median) return pos - t.begin >= s.left;
    const float4 c4 = cen[k];
    const float c = s.axis == 0 ? c4.x : (s.axis == 1 ? c4.y : c4.z);
    return (uint32_t)binOf(c, t.clo[s.axis], t.chi[s.axis]) > s.bin;
}

__global__ __launch_bounds__(256) void sahPartCountKernel(const SahTask* __restrict__ tasks, const SahSplit* __restrict__ splits,
                                                          const uint2* __restrict__ blockTask, const uint32_t* __restrict__ ref,
                                                          const float4* __restrict__ cen, uint32_t* blockRight,
                                                          const uint32_t* __restrict__ cnt) {
    __shared__ uint32_t waveSum[4];
    if (blockIdx.x >= cnt[kSahBlocks]) {   // no work: a zero in the scan
        if (threadIdx.x == 0) blockRight[blockIdx.x] = 0u;
        return;
    }
    const uint2 bt = blockTask[blockIdx.x];
    const SahTask& t = tasks[bt.x];
    const SahSplit* sp = splits + bt.x;
    const uint32_t end = min(t.begin + t.count, bt.y + (uint32_t)kChunk);
    uint32_t c = 0;
    for (uint32_t i = bt.y + threadIdx.x; i < end; i += 256) c += goesRight(t, *sp, i, cen, ref[i]) ? 1u : 0u;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0) waveSum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) blockRight[blockIdx.x] = waveSum[0] + waveSum[1] + waveSum[2] + waveSum[3];
}

// stable partition: a block's primitives in order, 256 at a time, ranked by a block scan of the flags
__global__ __launch_bounds__(256) void sahPartScatterKernel(const SahTask* __restrict__ tasks, const SahSplit* __restrict__ splits,
                                                            const uint2* __restrict__ blockTask, const uint32_t* __restrict__ ref,
                                                            const float4* __restrict__ cen, const uint32_t* __restrict__ rightOfs,
                                                            uint32_t* refOut, const uint32_t* __restrict__ cnt) {
    __shared__ uint32_t waveCnt[4];
    if (blockIdx.x >= cnt[kSahBlocks]) return;
    const uint2 bt = blockTask[blockIdx.x];
    const SahTask& t = tasks[bt.x];
    const SahSplit* sp = splits + bt.x;
    const uint32_t end = min(t.begin + t.count, bt.y + (uint32_t)kChunk);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // rights before this block within the task, then before each element
    uint32_t rightsBefore = rightOfs[blockIdx.x] - rightOfs[t.firstBlock];
    const uint32_t leftCount = sp->left;
    for (uint32_t base = bt.y; base < end; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const bool ok = i < end;
        const uint32_t k = ok ? ref[i] : 0u;
        const bool r = ok && goesRight(t, *sp, i, cen, k);
        const uint64_t m = __ballot(r);
        const uint32_t inWave = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) waveCnt[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (uint32_t w = 0; w < 4; w++) {
            if (w < wave) before += waveCnt[w];
            total += waveCnt[w];
        }
        if (ok) {
            const uint32_t rb = rightsBefore + before + inWave;   // rights before element i in the task
            refOut[r ? t.begin + leftCount + rb : i - rb] = k;
        }
        rightsBefore += total;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void sahCopyKernel(const SahTask* __restrict__ tasks, const uint2* __restrict__ blockTask,
                                                     const uint32_t* __restrict__ refOut, uint32_t* ref,
                                                     const uint32_t* __restrict__ cnt) {
    if (blockIdx.x >= cnt[kSahBlocks]) return;
    const uint2 bt = blockTask[blockIdx.x];
    const SahTask& t = tasks[bt.x];
    const uint32_t end = min(t.begin + t.count, bt.y + (uint32_t)kChunk);
    for (uint32_t i = bt.y + threadIdx.x; i < end; i += 256) ref[i] = refOut[i];
}

// One atomic add per wave: lane's slot in a counter for `want` lanes (whole waves call it).
__device__ __forceinline__ uint32_t waveAlloc(uint32_t* counter, bool want) {
    const uint64_t m = __ballot(want);
    if (!m) return 0u;
    const int lane = (int)(threadIdx.x & 63), leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// children of the split large tasks: a primitive id (one primitive) or a new node; tasks for the
// next level or for the wave kernel
__global__ __launch_bounds__(64) void sahEmitKernel(const SahTask* __restrict__ tasks, const SahSplit* __restrict__ splits,
                                                    int ntask, const uint32_t* __restrict__ ref, uint32_t n, float4* pbox,
                                                    uint2* pchild, SahTask* nextLarge, SahTask* small, uint32_t* cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool on = i < ntask;
    const SahTask& t = tasks[on ? i : 0];
    const SahSplit& s = splits[on ? i : 0];
    uint32_t ids[2];
    for (int side = 0; side < 2; side++) {
        SahTask c;
        c.begin = side ? t.begin + s.left : t.begin;
        c.count = side ? t.count - s.left : s.left;
        c.firstBlock = 0;
        c.binSlot = kNoSlot;
        c.pad[0] = c.pad[1] = c.pad[2] = 0u;
        for (int a = 0; a < 3; a++) {
            c.lo[a] = s.child[side][a];
            c.hi[a] = s.child[side][3 + a];
            c.clo[a] = s.child[side][6 + a];
            c.chi[a] = s.child[side][9 + a];
        }
        const bool node = on && c.count >= 2, large = node && c.count > (uint32_t)kWaveTask;
        c.node = n + waveAlloc(cnt + kSahNodes, node);
        const uint32_t qL = waveAlloc(cnt + kSahLarge, large), qS = waveAlloc(cnt + kSahSmall, node && !large);
        if (!on) continue;
        if (!node) {
            ids[side] = ref[c.begin];
            continue;
        }
        ids[side] = c.node;
        writeNodeBox(pbox, c.node, c.lo, c.hi, c.count, false);
        if (large) nextLarge[qL] = c;
        else small[qS] = c;
    }
    if (on) pchild[t.node - n] = make_uint2(ids[0], ids[1]);
}

// node ids of the wave tasks: a task of c primitives adds c - 2 nodes below its root
__global__ void sahWaveCountKernel(const SahTask* __restrict__ tasks, int ntask, uint32_t* need) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < ntask) need[i] = tasks[i].count - 2u;
}

// Segmented scans for the wave kernel (min / max only: a lane may combine its own value again).
// Hillis-Steele within each row of 16 lanes by DPP row shifts (a lane whose source is outside its
// row keeps its own value), then across rows in two ds_bpermute steps: from the neighbouring
// row's end lane, then from the end lane two rows away (which by then covers two rows).
template <int CTRL>
__device__ __forceinline__ float dppF(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dppU(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
// step s (0..5): lanes 1, 2, 4, 8 back within the row, then the previous row's last lane, then the
// last lane two rows back; `src` = the source lane of steps 4 and 5
__device__ __forceinline__ int prefixSrc(int lane, int s) { return s == 4 ? (lane & ~15) - 1 : (lane & ~15) - 17; }
__device__ __forceinline__ int suffixSrc(int lane, int s) { return s == 4 ? (lane | 15) + 1 : (lane | 15) + 17; }

template <int S>
__device__ __forceinline__ float prefixGet(float v, int lane) {
    if constexpr (S < 4) return dppF<0x110 + (1 << S)>(v);   // row_shr
    else return __shfl(v, prefixSrc(lane, S) & 63);
}
template <int S>
__device__ __forceinline__ float suffixGet(float v, int lane) {
    if constexpr (S < 4) return dppF<0x100 + (1 << S)>(v);   // row_shl
    else return __shfl(v, suffixSrc(lane, S) & 63);
}
template <int S>
__device__ __forceinline__ bool prefixIn(int lane, int sb) { return S < 4 ? lane - (1 << S) >= sb : prefixSrc(lane, S) >= sb; }
template <int S>
__device__ __forceinline__ bool suffixIn(int lane, int se) {
    return S < 4 ? lane + (1 << S) < se : (suffixSrc(lane, S) < se && suffixSrc(lane, S) < 64);
}

// one step of the boxes' prefix over [sb, lane] and suffix over [lane, se)
template <int S>
__device__ __forceinline__ void scanStep(int lane, int sb, int se, float* plo, float* phi, float* slo, float* shi) {
    const bool inL = prefixIn<S>(lane, sb), inR = suffixIn<S>(lane, se);
    for (int x = 0; x < 3; x++) {
        const float al = prefixGet<S>(plo[x], lane), ah = prefixGet<S>(phi[x], lane);
        const float bl = suffixGet<S>(slo[x], lane), bh = suffixGet<S>(shi[x], lane);
        if (inL) { plo[x] = fminf(plo[x], al); phi[x] = fmaxf(phi[x], ah); }
        if (inR) { slo[x] = fminf(slo[x], bl); shi[x] = fmaxf(shi[x], bh); }
    }
}
template <int S>
__device__ __forceinline__ void prefixStep(int lane, int sb, float* plo, float* phi) {
    const bool inL = prefixIn<S>(lane, sb);
    for (int x = 0; x < 3; x++) {
        const float al = prefixGet<S>(plo[x], lane), ah = prefixGet<S>(phi[x], lane);
        if (inL) { plo[x] = fminf(plo[x], al); phi[x] = fmaxf(phi[x], ah); }
    }
}
template <int S>
__device__ __forceinline__ void minStep(int lane, int sb, uint64_t& best) {
    uint64_t o;
    if constexpr (S < 4) {
        const uint32_t lo = dppU<0x110 + (1 << S)>((uint32_t)best), hi = dppU<0x110 + (1 << S)>((uint32_t)(best >> 32));
        o = ((uint64_t)hi << 32) | lo;
    } else {
        o = __shfl(best, prefixSrc(lane, S) & 63);
    }
    if (prefixIn<S>(lane, sb) && o < best) best = o;
}
template <int S>
__device__ __forceinline__ void boxScans(int lane, int sb, int se, float* plo, float* phi, float* slo, float* shi) {
    scanStep<S>(lane, sb, se, plo, phi, slo, shi);
    if constexpr (S < 5) boxScans<S + 1>(lane, sb, se, plo, phi, slo, shi);
}
template <int S>
__device__ __forceinline__ void boxPrefix(int lane, int sb, float* plo, float* phi) {
    prefixStep<S>(lane, sb, plo, phi);
    if constexpr (S < 5) boxPrefix<S + 1>(lane, sb, plo, phi);
}
template <int S>
__device__ __forceinline__ void segMin(int lane, int sb, uint64_t& best) {
    minStep<S>(lane, sb, best);
    if constexpr (S < 5) segMin<S + 1>(lane, sb, best);
}

struct WaveLds {   // one wave's task: primitives by local index, the axis orders' exchange slots
    float box[kWaveTask][6];
    uint32_t prim[kWaveTask];
    uint32_t left[kWaveTask];
    uint32_t slot[3][kWaveTask];
};

// One wave finishes a task of at most kWaveTask primitives, every node of a level at once.  The
// primitives stay in LDS by local index; each lane is a position in three orders of them (by
// centroid along x, y, z: one bitonic sort each at the start), and a node is a segment
// [sb, sb + sc) of positions holding the same primitives in all three orders.  Per level and
// axis, segmented scans of the boxes in that order give every split position's cost; the
// cheapest over the axes wins (a segment of at most 3 primitives becomes a leaf group when that
// is cheaper); then every order is stably partitioned by the winning side (ballot counts), so the
// children are again segments in all three orders.
__global__ __launch_bounds__(256) void sahWaveKernel(const SahTask* __restrict__ tasks, int ntask, const uint32_t* __restrict__ idBase,
                                                     const uint32_t* __restrict__ ref, const float4* __restrict__ cen,
                                                     const float* __restrict__ leafBoxes, uint32_t n, float trav, float4* pbox,
                                                     uint2* pchild, uint32_t* cnt) {
    __shared__ WaveLds lds[4];
    const int lane = (int)(threadIdx.x & 63);
    const int ti = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (ti >= ntask) return;   // whole waves
    WaveLds& L = lds[threadIdx.x >> 6];
    const SahTask& t = tasks[ti];
    const int c = (int)t.count;
    const bool real = lane < c;
    float ce[3] = {0.0f, 0.0f, 0.0f};
    if (real) {
        const uint32_t k = ref[t.begin + lane];
        const float* b = leafBoxes + 6 * (size_t)k;
        const float4 c4 = cen[k];
        for (int w = 0; w < 6; w++) L.box[lane][w] = b[w];
        L.prim[lane] = k;
        ce[0] = c4.x; ce[1] = c4.y; ce[2] = c4.z;
    }
    int idx[3];
    for (int a = 0; a < 3; a++) {   // positions past c keep their own index (the sort keeps them last)
        uint64_t key = real ? (((uint64_t)ordF(ce[a]) << 6) | (uint64_t)lane) : ((0xffffffffull << 6) | (uint64_t)lane);
        for (int kk = 2; kk <= 64; kk <<= 1)
            for (int j = kk >> 1; j > 0; j >>= 1) {
                const uint64_t o = __shfl_xor(key, j);
                const bool takeMin = ((lane & j) == 0) == ((lane & kk) == 0);
                key = takeMin ? (o < key ? o : key) : (o > key ? o : key);
            }
        idx[a] = (int)(key & 63u);
    }
    __builtin_amdgcn_wave_barrier();
    int sb = real ? 0 : lane, sc = real ? c : 1;
    uint32_t node = t.node;
    bool active = real && c >= 2;
    // this task's node ids: a block after the large levels' nodes (no atomics: c - 2 of them)
    uint32_t nextId = n + cnt[kSahNodes] + idBase[ti];
    if (ti == ntask - 1 && lane == 0) cnt[kSahTotal] = cnt[kSahNodes] + idBase[ti] + (uint32_t)(c - 2);
    if (c < 2 || c > kWaveTask || nextId + (uint32_t)(c - 2) > 2 * n - 1) {   // (ids past the node arrays: never written)
        if (lane == 0) atomicOr(cnt + kSahErr, 2u);
        return;
    }
    while (__ballot(active)) {
        const int se = sb + sc;   // segment end (exclusive)
        uint64_t best = ~0ull;
        float segArea = 0.0f, segHi[3] = {0.0f, 0.0f, 0.0f};
        for (int a = 0; a < 3; a++) {
            float plo[3], phi[3], slo[3], shi[3];
            for (int x = 0; x < 3; x++) {
                plo[x] = slo[x] = L.box[idx[a]][x];
                phi[x] = shi[x] = L.box[idx[a]][3 + x];
            }
            boxScans<0>(lane, sb, se, plo, phi, slo, shi);
            const float pa = halfArea3(plo, phi), sa = halfArea3(slo, shi);
            const float saNext = __shfl_down(sa, 1);
            if (a == 0) {
                segArea = __shfl(pa, se - 1);
                for (int x = 0; x < 3; x++) segHi[x] = __shfl(phi[x], se - 1);
            }
            if (active && lane < se - 1) {
                const int lc = lane - sb + 1;
                const float cst = (float)lc * pa + (float)(sc - lc) * saNext;
                const uint64_t kk = ((uint64_t)ordF(cst) << 32) | ((uint64_t)a << 8) | (uint64_t)(lane - sb);
                best = kk < best ? kk : best;
            }
        }
        segMin<0>(lane, sb, best);   // segment minimum, at the segment's last position
        best = __shfl(best, se - 1);
        const float bestCost = unordF((uint32_t)(best >> 32));
        int axis = (int)((best >> 8) & 3u), lc = (int)(best & 63u) + 1;
        if (axis > 2 || lc >= sc) {   // (no candidate: cannot happen for sc >= 2; split in the middle)
            axis = 0;
            lc = sc / 2;
        }
        const bool leaf = active && sc <= kMaxGroup && (float)sc * segArea <= trav * segArea + bestCost;
        // a leaf group: node over two primitives, or node(p0, inner(p1, p2))
        const int j1 = __shfl(idx[0], (sb + 1) & 63), j2 = __shfl(idx[0], (sb + 2) & 63);
        const uint64_t m3 = __ballot(leaf && lane == sb && sc == 3);
        const uint32_t inner = nextId + (uint32_t)__popcll(m3 & ((1ull << lane) - 1ull));
        nextId += (uint32_t)__popcll(m3);
        if (leaf && lane == sb) {
            const uint32_t k0 = L.prim[idx[0]], k1 = L.prim[j1];
            pbox[2 * (size_t)node + 1] = make_float4(segHi[0], segHi[1], segHi[2], __uint_as_float((uint32_t)sc | kGroupFlag));
            if (sc == 2) {
                pchild[node - n] = make_uint2(k0, k1);
            } else {
                const uint32_t k2 = L.prim[j2];
                float ilo[3], ihi[3];
                for (int x = 0; x < 3; x++) {
                    ilo[x] = fminf(L.box[j1][x], L.box[j2][x]);
                    ihi[x] = fmaxf(L.box[j1][3 + x], L.box[j2][3 + x]);
                }
                writeNodeBox(pbox, inner, ilo, ihi, 2u, true);
                pchild[inner - n] = make_uint2(k1, k2);
                pchild[node - n] = make_uint2(k0, inner);
            }
        }
        // a split: the winning order says each primitive's side; every order partitions stably
        const bool split = active && !leaf;
        if (split) L.left[axis == 0 ? idx[0] : (axis == 1 ? idx[1] : idx[2])] = lane < sb + lc ? 1u : 0u;
        __builtin_amdgcn_wave_barrier();
        const uint64_t below = ((1ull << lane) - 1ull) & ~((1ull << sb) - 1ull);   // positions [sb, lane)
        for (int a = 0; a < 3; a++) {
            const bool goL = split && L.left[idx[a]] != 0u;
            const uint64_t mL = __ballot(goL), mR = __ballot(split && !goL);
            const int np = !split ? lane
                                  : (goL ? sb + __popcll(mL & below) : sb + lc + __popcll(mR & below));
            L.slot[a][np] = (uint32_t)idx[a];
        }
        __builtin_amdgcn_wave_barrier();
        for (int a = 0; a < 3; a++) idx[a] = (int)L.slot[a][lane];
        __builtin_amdgcn_wave_barrier();
        int nsb = sb, nsc = sc;
        if (split) {
            if (lane < sb + lc) nsc = lc;
            else { nsb = sb + lc; nsc = sc - lc; }
        }
        const bool needNode = split && lane == nsb && nsc >= 2;
        const uint64_t m = __ballot(needNode);
        uint32_t myId = needNode ? nextId + (uint32_t)__popcll(m & ((1ull << lane) - 1ull)) : L.prim[idx[0]];
        nextId += (uint32_t)__popcll(m);
        myId = __shfl(myId, nsb);                            // the id of the child holding this position
        const uint32_t rightId = __shfl(myId, (nsb + nsc) & 63);
        if (split && lane == sb) pchild[node - n] = make_uint2(myId, rightId);
        float blo[3], bhi[3];
        for (int x = 0; x < 3; x++) { blo[x] = L.box[idx[0]][x]; bhi[x] = L.box[idx[0]][3 + x]; }
        boxPrefix<0>(lane, nsb, blo, bhi);   // the children's boxes, at their last positions
        if (split && nsc >= 2 && lane == nsb + nsc - 1) writeNodeBox(pbox, myId, blo, bhi, (uint32_t)nsc, false);
        if (split) {
            sb = nsb;
            sc = nsc;
            node = myId;
        }
        active = split && nsc >= 2;
    }
}

// Before the collapse reads it: every child id of the SAH build's nodes in range (a bad tree is
// reported, never walked).
__global__ void sahCheckKernel(const uint2* __restrict__ pchild, uint32_t* cnt, uint32_t n) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x, nodes = cnt[kSahTotal];
    if (j == 0 && nodes != n - 1) atomicOr(cnt + kSahErr, 1u);   // a binary tree over n leaves
    if (j >= nodes || j >= n) return;
    const uint2 c = pchild[j];
    if (c.x >= n + nodes || c.y >= n + nodes) atomicOr(cnt + kSahErr, 1u);
}

unsigned blocks(int64_t n, unsigned tb) { return (unsigned)((n + tb - 1) / tb); }

}  // namespace

WideDevBuilder::~WideDevBuilder() {
    for (Buf* b : {&pbox_, &pchild_, &cid_[0], &cid_[1], &nn_, &flag_, &pos_, &items_[0], &items_[1], &cnt_, &ofs_,
                   &scanTemp_, &misc_, &sahCen_, &sahRef_[0], &sahRef_[1], &sahLarge_[0], &sahLarge_[1], &sahSmall_,
                   &sahSplit_, &sahBins_, &sahMulti_, &sahBlk_, &sahBlkR_, &sahBlkO_, &sahCnt_})
        if (b->p) (void)hipFree(b->p);
}

hipError_t WideDevBuilder::reserve(Buf& b, size_t bytes) {
    bytes = bytes < 16 ? 16 : bytes;
    if (b.p && b.cap >= bytes) return hipSuccess;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e == hipSuccess) b.cap = bytes;
    return e;
}

#define WB_TRY(x)                          \
    do {                                   \
        const hipError_t e_ = (x);         \
        if (e_ != hipSuccess) return e_;   \
    } while (0)

// Step 2 by SAH: large tasks level by level (one host read per level: the task list, to map
// blocks to tasks), then every wave-sized task in one launch.
hipError_t WideDevBuilder::buildSah(const WideDevIn& in, hipStream_t st, float trav, std::string& err) {
    const int64_t n = in.n;
    const size_t nn = (size_t)n;
    const size_t largeCap = nn / (kWaveTask + 1) + 2, smallCap = nn / 2 + 2, multiCap = nn / kChunk + 2;
    const size_t blockCap = nn / kChunk + largeCap + 1;
    WB_TRY(reserve(sahCen_, nn * 16));
    WB_TRY(reserve(sahRef_[0], nn * 4));
    WB_TRY(reserve(sahRef_[1], nn * 4));
    WB_TRY(reserve(sahLarge_[0], largeCap * sizeof(SahTask)));
    WB_TRY(reserve(sahLarge_[1], largeCap * sizeof(SahTask)));
    WB_TRY(reserve(sahSmall_, smallCap * sizeof(SahTask)));
    WB_TRY(reserve(sahSplit_, largeCap * sizeof(SahSplit)));
    WB_TRY(reserve(sahBins_, multiCap * 3 * kBins * kBinWords * 4));
    WB_TRY(reserve(sahMulti_, multiCap * 4));
    WB_TRY(reserve(sahBlk_, blockCap * 8));
    WB_TRY(reserve(sahBlkR_, (blockCap > smallCap ? blockCap : smallCap) * 4));   // block counts, then wave-task node counts
    WB_TRY(reserve(sahBlkO_, (blockCap > smallCap ? blockCap : smallCap) * 4));
    WB_TRY(reserve(sahCnt_, (kSahWords + 12) * 4));
    float4* pbox = static_cast<float4*>(pbox_.p);
    uint2* pchild = static_cast<uint2*>(pchild_.p);
    float4* cen = static_cast<float4*>(sahCen_.p);
    uint32_t* ref = static_cast<uint32_t*>(sahRef_[0].p);
    uint32_t* ref2 = static_cast<uint32_t*>(sahRef_[1].p);
    uint32_t* cnt = static_cast<uint32_t*>(sahCnt_.p);
    uint32_t* rootAcc = cnt + kSahWords;   // 12 words
    uint32_t* rootCid = static_cast<uint32_t*>(cid_[0].p);
    SahTask* small = static_cast<SahTask*>(sahSmall_.p);
    SahSplit* splits = static_cast<SahSplit*>(sahSplit_.p);
    uint32_t* bins = static_cast<uint32_t*>(sahBins_.p);
    uint32_t* multi = static_cast<uint32_t*>(sahMulti_.p);
    uint2* blk = static_cast<uint2*>(sahBlk_.p);
    uint32_t* blkR = static_cast<uint32_t*>(sahBlkR_.p);
    uint32_t* blkO = static_cast<uint32_t*>(sahBlkO_.p);
    const unsigned tb = 256;
    // PT_SAH_SYNC=1: synchronise after every launch and name the kernel of a failure (debugging)
    const bool dbgSync = std::getenv("PT_SAH_SYNC") != nullptr;
    auto check = [&](const char* what) -> hipError_t {
        hipError_t e = hipGetLastError();
        if (e == hipSuccess && dbgSync) e = hipStreamSynchronize(st);
        if (e != hipSuccess) err = std::string("wide BVH (device): ") + what + ": " + hipGetErrorString(e);
        return e;
    };

    {
        uint32_t init[kSahWords + 12] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        for (int w = 0; w < 12; w++) init[kSahWords + w] = (w % 6) < 3 ? 0xffffffffu : 0u;
        WB_TRY(hipMemcpyAsync(cnt, init, sizeof(init), hipMemcpyHostToDevice, st));
    }
    sahInitKernel<<<blocks(n, tb), tb, 0, st>>>(in.leafBoxes, (int)n, cen, ref, pbox, rootAcc);
    WB_TRY(check("init"));
    if (n == 1) {
        const uint32_t zero = 0u;
        WB_TRY(hipMemcpyAsync(rootCid, &zero, 4, hipMemcpyHostToDevice, st));
        return hipStreamSynchronize(st);
    }
    int cur = 0;
    sahRootKernel<<<1, 1, 0, st>>>(rootAcc, (int)n, pbox, static_cast<SahTask*>(sahLarge_[0].p), small, cnt, rootCid);
    WB_TRY(check("root"));
    uint4* need = static_cast<uint4*>(cnt_.p);
    uint4* needOfs = static_cast<uint4*>(ofs_.p);
    uint32_t c[kSahWords];
    for (int level = 0;; level++) {
        WB_TRY(hipMemcpyAsync(c, cnt, sizeof(c), hipMemcpyDeviceToHost, st));
        WB_TRY(hipStreamSynchronize(st));
        const uint32_t nLarge = c[kSahLarge];
        if (nLarge == 0) break;
        if (level > 64 || nLarge > largeCap || c[kSahSmall] > smallCap) {
            err = "wide BVH (device): SAH build does not converge";
            return hipErrorUnknown;
        }
        // upper bounds of this level's blocks and multi-block tasks (the exact counts stay on the device)
        const unsigned nb = (unsigned)(nLarge + nn / kChunk + 1);
        const unsigned nm = (unsigned)(nLarge < nn / kChunk + 1 ? nLarge : nn / kChunk + 1);
        if (nb > blockCap || nm > multiCap) {
            err = "wide BVH (device): SAH block map overflow";
            return hipErrorUnknown;
        }
        SahTask* large = static_cast<SahTask*>(sahLarge_[cur].p);
        sahMapCountKernel<<<blocks(nLarge, tb), tb, 0, st>>>(large, (int)nLarge, need);
        WB_TRY(check("block counts"));
        WB_TRY(exclusiveScanU3(scanTemp_.p, need, needOfs, (size_t)nLarge, st));
        sahMapWriteKernel<<<blocks(nLarge, tb), tb, 0, st>>>(large, (int)nLarge, need, needOfs, blk, multi, cnt);
        WB_TRY(check("block map"));
        sahZeroBinsKernel<<<blocks((int64_t)nm * 3 * kBins, tb), tb, 0, st>>>(bins, cnt);
        WB_TRY(check("zero bins"));
        sahBinKernel<<<nb, 256, 0, st>>>(large, blk, ref, cen, in.leafBoxes, bins, splits, cnt);
        WB_TRY(check("bins"));
        sahSplitKernel<<<nm, 128, 0, st>>>(large, multi, bins, splits, cnt);
        WB_TRY(check("split"));
        sahPartCountKernel<<<nb, 256, 0, st>>>(large, splits, blk, ref, cen, blkR, cnt);
        WB_TRY(check("partition count"));
        WB_TRY(exclusiveScanU32(scanTemp_.p, blkR, blkO, (size_t)nb, st));
        sahPartScatterKernel<<<nb, 256, 0, st>>>(large, splits, blk, ref, cen, blkO, ref2, cnt);
        WB_TRY(check("partition"));
        sahCopyKernel<<<nb, 256, 0, st>>>(large, blk, ref2, ref, cnt);
        WB_TRY(check("copy"));
        WB_TRY(hipMemsetAsync(cnt + kSahLarge, 0, 4, st));
        sahEmitKernel<<<blocks(nLarge, 64), 64, 0, st>>>(large, splits, (int)nLarge, ref, (uint32_t)n, pbox, pchild,
                                                         static_cast<SahTask*>(sahLarge_[cur ^ 1].p), small, cnt);
        WB_TRY(check("emit"));
        cur ^= 1;
    }
    if (c[kSahSmall] > smallCap) {
        err = "wide BVH (device): SAH small-task overflow";
        return hipErrorUnknown;
    }
    if (c[kSahSmall]) {
        const int ns = (int)c[kSahSmall];
        sahWaveCountKernel<<<blocks(ns, tb), tb, 0, st>>>(small, ns, blkR);
        WB_TRY(check("wave counts"));
        WB_TRY(exclusiveScanU32(scanTemp_.p, blkR, blkO, (size_t)ns, st));
        sahWaveKernel<<<blocks(ns, 4), 256, 0, st>>>(small, ns, blkO, ref, cen, in.leafBoxes, (uint32_t)n, trav, pbox, pchild,
                                                     cnt);
        WB_TRY(check("wave tasks"));
    }
    if (!c[kSahSmall]) WB_TRY(hipMemcpyAsync(cnt + kSahTotal, cnt + kSahNodes, 4, hipMemcpyDeviceToDevice, st));
    sahCheckKernel<<<blocks(n, tb), tb, 0, st>>>(pchild, cnt, (uint32_t)n);
    WB_TRY(check("check"));
    WB_TRY(hipMemcpyAsync(c, cnt, sizeof(c), hipMemcpyDeviceToHost, st));
    WB_TRY(hipStreamSynchronize(st));
    if (c[kSahErr]) {
        err = "wide BVH (device): SAH build produced a malformed tree";
        return hipErrorUnknown;
    }
    return hipSuccess;
}

hipError_t WideDevBuilder::build(const WideDevIn& in, WideDevOut& out, hipStream_t st, std::string& err) {
    const int64_t n = in.n;
    out.depth = 0;
    out.slots = 0;
    if (n <= 0) return hipSuccess;
    if (n >= ((int64_t)1 << 26)) {
        err = "wide BVH (device): more than 2^26 primitives";
        return hipErrorInvalidValue;
    }
    const size_t nn = (size_t)n, nodesAll = 2 * nn;
    WB_TRY(reserve(pbox_, nodesAll * 32));
    WB_TRY(reserve(pchild_, nn * 8));
    WB_TRY(reserve(cid_[0], nn * 4));
    WB_TRY(reserve(cid_[1], nn * 4));
    WB_TRY(reserve(nn_, nn * 4));
    WB_TRY(reserve(flag_, nn * 4));
    WB_TRY(reserve(pos_, nn * 4));
    WB_TRY(reserve(items_[0], nn * 8));
    WB_TRY(reserve(items_[1], nn * 8));
    WB_TRY(reserve(cnt_, nn * 16));
    WB_TRY(reserve(ofs_, nn * 16));
    WB_TRY(reserve(misc_, kMiscWords * 4));
    const size_t tb1 = scanScratchBytesU32(nn), tb2 = scanScratchBytesU3(nn);
    WB_TRY(reserve(scanTemp_, tb1 > tb2 ? tb1 : tb2));
    uint32_t* misc = static_cast<uint32_t*>(misc_.p);
    float4* pbox = static_cast<float4*>(pbox_.p);
    uint2* pchild = static_cast<uint2*>(pchild_.p);
    uint32_t* flag = static_cast<uint32_t*>(flag_.p);
    uint32_t* pos = static_cast<uint32_t*>(pos_.p);
    int* nearest = static_cast<int*>(nn_.p);
    const unsigned tb = 256;
    // tuning knobs: the binary builder, PLOC radius, the SAH weight of a node visit relative to
    // a primitive test (defaults: the host build's 1 for binned SAH, 0.5 for PLOC's bottom-up rule)
    const char* bv = std::getenv("PT_WIDE_DEVICE_BUILDER");
    const bool ploc = bv && std::strcmp(bv, "ploc") == 0;
    const char* rv = std::getenv("PT_PLOC_RADIUS");
    const int radius = rv ? std::atoi(rv) : kRadiusDefault;
    const char* tv = std::getenv("PT_WIDE_TRAV_COST");
    const float trav = tv && std::atof(tv) > 0.0 ? (float)std::atof(tv) : (ploc ? 0.5f : 1.0f);

    // 1. ranks, shading records in rank order
    rankKernel<<<blocks(n, tb), tb, 0, st>>>(in.lbvh, in.iparent, in.lparent, in.irange, (int)n, out.rank);
    shadeByRankKernel<<<blocks(n, tb), tb, 0, st>>>(in.shade, out.rank, (int)n, out.wshade);
    WB_TRY(hipGetLastError());

    // 2. the binary tree
    WB_TRY(hipMemsetAsync(misc, 0, kMiscWords * 4, st));
    int cur = 0;
    if (!ploc) {
        WB_TRY(buildSah(in, st, trav, err));
    } else {
        plocInitKernel<<<blocks(n, tb), tb, 0, st>>>(in.leafBoxes, (int)n, pbox, static_cast<uint32_t*>(cid_[0].p));
        WB_TRY(hipGetLastError());
        int64_t m = n;
        {
            const uint32_t m0 = (uint32_t)n;
            WB_TRY(hipMemcpyAsync(misc + kMiscM, &m0, 4, hipMemcpyHostToDevice, st));
        }
        int pass = 0;
        while (m > kTailMax) {
            if (pass > 4 * 64 + 64) {
                err = "wide BVH (device): clustering does not converge";
                return hipErrorUnknown;
            }
            for (int b = 0; b < kPassesPerSync; b++, pass++) {
                uint32_t* cid = static_cast<uint32_t*>(cid_[cur].p);
                const uint32_t* mIn = misc + kMiscM + (pass & 1);
                switch (radius) {
                    case 8: plocNearestKernel<8><<<blocks(m, kTile), kTile, 0, st>>>(cid, pbox, mIn, nearest); break;
                    case 32: plocNearestKernel<32><<<blocks(m, kTile), kTile, 0, st>>>(cid, pbox, mIn, nearest); break;
                    case 64: plocNearestKernel<64><<<blocks(m, kTile), kTile, 0, st>>>(cid, pbox, mIn, nearest); break;
                    default: plocNearestKernel<16><<<blocks(m, kTile), kTile, 0, st>>>(cid, pbox, mIn, nearest); break;
                }
                plocMergeKernel<<<blocks(m, tb), tb, 0, st>>>(cid, pbox, pchild, nearest, mIn, (int)m, (int)n, trav, flag, misc);
                WB_TRY(hipGetLastError());
                WB_TRY(exclusiveScanU32(scanTemp_.p, flag, pos, (size_t)m, st));
                plocCompactKernel<<<blocks(m, tb), tb, 0, st>>>(cid, flag, pos, mIn, static_cast<uint32_t*>(cid_[cur ^ 1].p),
                                                                misc + kMiscM + ((pass + 1) & 1));
                WB_TRY(hipGetLastError());
                cur ^= 1;
            }
            uint32_t mNext = 0;
            WB_TRY(hipMemcpyAsync(&mNext, misc + kMiscM + (pass & 1), 4, hipMemcpyDeviceToHost, st));
            WB_TRY(hipStreamSynchronize(st));
            if ((int64_t)mNext >= m) {
                err = "wide BVH (device): clustering passes merged nothing";
                return hipErrorUnknown;
            }
            m = mNext;
        }
        if (m > 1) {
            uint32_t* a0 = static_cast<uint32_t*>(cid_[cur].p);
            uint32_t* a1 = static_cast<uint32_t*>(cid_[cur ^ 1].p);
            const uint32_t* mIn = misc + kMiscM + (pass & 1);
            switch (radius) {
                case 8: plocTailKernel<8><<<1, kTailThreads, 0, st>>>(a0, a1, pbox, pchild, nearest, flag, mIn, misc, (int)n, trav); break;
                case 32: plocTailKernel<32><<<1, kTailThreads, 0, st>>>(a0, a1, pbox, pchild, nearest, flag, mIn, misc, (int)n, trav); break;
                case 64: plocTailKernel<64><<<1, kTailThreads, 0, st>>>(a0, a1, pbox, pchild, nearest, flag, mIn, misc, (int)n, trav); break;
                default: plocTailKernel<16><<<1, kTailThreads, 0, st>>>(a0, a1, pbox, pchild, nearest, flag, mIn, misc, (int)n, trav); break;
            }
            WB_TRY(hipGetLastError());
        }
    }
    const uint32_t* rootCid = static_cast<const uint32_t*>(cid_[cur].p);

    // 3. collapse + quantisation, level by level
    const Tree T{pbox, pchild, (uint32_t)n};
    const uint32_t slotCap = wideDevSlotCap(n);   // <= 2^24: child bases fit the kernels' 24-bit field
    setRootKernel<<<1, 1, 0, st>>>(rootCid, static_cast<uint2*>(items_[0].p));
    WB_TRY(hipGetLastError());
    int it = 0;
    int64_t items = 1;
    uint32_t nodeBase = 1, primBase = 0;
    int level = 0;
    while (items > 0) {
        if (++level > kMaxLevels) {
            err = "wide BVH (device): deeper than the traversal stack";
            return hipErrorUnknown;
        }
        const uint2* cur2 = static_cast<const uint2*>(items_[it].p);
        uint4* cnt = static_cast<uint4*>(cnt_.p);
        uint4* ofs = static_cast<uint4*>(ofs_.p);
        wideCountKernel<<<blocks(items, tb), tb, 0, st>>>(T, cur2, (int)items, cnt);
        WB_TRY(hipGetLastError());
        WB_TRY(exclusiveScanU3(scanTemp_.p, cnt, ofs, (size_t)items, st));
        wideWriteKernel<<<blocks(items, tb), tb, 0, st>>>(T, cur2, (int)items, cnt, ofs, nodeBase, primBase, slotCap, rootCid,
                                                          in.prims, out.rank, out.nodes, reinterpret_cast<uint4*>(out.wprims),
                                                          static_cast<uint2*>(items_[it ^ 1].p), misc);
        WB_TRY(hipGetLastError());
        uint32_t tot[4] = {0, 0, 0, 0};
        WB_TRY(hipMemcpyAsync(tot, misc + kMiscTotA, 16, hipMemcpyDeviceToHost, st));
        WB_TRY(hipStreamSynchronize(st));
        if (tot[3]) {   // kMiscErr follows the totals
            err = "wide BVH (device): encoding limits exceeded";
            return hipErrorUnknown;
        }
        nodeBase += tot[0];
        primBase += tot[1];
        items = tot[2];
        it ^= 1;
    }
    if ((int64_t)primBase != n) {
        err = "wide BVH (device): primitive count mismatch";
        return hipErrorUnknown;
    }
    out.depth = level;
    out.slots = nodeBase;
    return hipSuccess;
}

}  // namespace pt
