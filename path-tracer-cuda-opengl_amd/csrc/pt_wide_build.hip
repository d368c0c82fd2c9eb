// pt_wide_build.hip — the compressed 8-wide tree built on the device (see host/pt_wide_dev.hpp).
//
// 1. Ranks: leaf k's position in the order RenderManager::hitBvh (utils/render_manager.h:105-133)
//    would test the LBVH's leaves (the tie order of the closest hit), from the leaf up: at each
//    ancestor, the offset of the child's part in its parent's visit (leaf children first, left
//    then right; then the right subtree; then the left one).  = pt::referenceRanks, in parallel.
// 2. Binary tree: PLOC over the leaves in Morton order.  Each pass: every cluster finds its
//    nearest neighbour within kRadius positions (smallest merged surface area; ties by the pair's
//    positions, a strict total order, so the globally closest pair is mutual and every pass
//    merges), mutual pairs merge into a new node at the lower position, survivors are compacted.
//    Each merge also decides, bottom up, whether its subtree (at most 3 primitives) is cheaper as
//    one leaf (SAH: count x area vs traversal x area + the children's costs).
// 3. Collapse + quantisation, one wide level per launch pair: count (children, primitives, child
//    block), exclusive scan, write.  Slots and primitive records are allocated in level order,
//    parents' order, slot order -- the host build's breadth-first order -- so the output is
//    deterministic (the node ids PLOC hands out by atomic counter never reach it).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "pt_prims.hpp"
#include "pt_wide_dev.hpp"

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
    int emin = ext > 0.0 ? ceilLog2(ext) - 18 : -100;
    emin = emin < -100 ? -100 : emin;

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
    // extent <= 251 quanta, child planes rounded outward by one more quantum
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
                    const double qlo = floor(((double)cmn[j][a] - (double)p) / s) - 1.0;
                    const double qhi = ceil(((double)cmx[j][a] - (double)p) / s) + 1.0;
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
    uint4* dst = reinterpret_cast<uint4*>(nodes + 20 * (size_t)item.y);
    for (int q = 0; q < 5; q++) dst[q] = make_uint4(R[4 * q], R[4 * q + 1], R[4 * q + 2], R[4 * q + 3]);
}

unsigned blocks(int64_t n, unsigned tb) { return (unsigned)((n + tb - 1) / tb); }

}  // namespace

WideDevBuilder::~WideDevBuilder() {
    for (Buf* b : {&pbox_, &pchild_, &cid_[0], &cid_[1], &nn_, &flag_, &pos_, &items_[0], &items_[1], &cnt_, &ofs_,
                   &scanTemp_, &misc_})
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
    // tuning knobs: PLOC radius, the SAH weight of a node visit relative to a primitive test
    const char* rv = std::getenv("PT_PLOC_RADIUS");
    const int radius = rv ? std::atoi(rv) : kRadiusDefault;
    const char* tv = std::getenv("PT_WIDE_TRAV_COST");
    const float trav = tv && std::atof(tv) > 0.0 ? (float)std::atof(tv) : 0.5f;

    // 1. ranks, shading records in rank order
    rankKernel<<<blocks(n, tb), tb, 0, st>>>(in.lbvh, in.iparent, in.lparent, in.irange, (int)n, out.rank);
    shadeByRankKernel<<<blocks(n, tb), tb, 0, st>>>(in.shade, out.rank, (int)n, out.wshade);
    WB_TRY(hipGetLastError());

    // 2. PLOC
    WB_TRY(hipMemsetAsync(misc, 0, kMiscWords * 4, st));
    plocInitKernel<<<blocks(n, tb), tb, 0, st>>>(in.leafBoxes, (int)n, pbox, static_cast<uint32_t*>(cid_[0].p));
    WB_TRY(hipGetLastError());
    int cur = 0;
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
