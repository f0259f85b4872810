// pbr_bvh_build.hip — BVHAccel's bucketed-SAH build (Accelerator/BVHAccel.cpp:97-283) on the device.
//
// The output is the host builder's (pbr_scene.cpp SahBuilder), i.e. the reference's as g++ compiles it:
// the same LinearBVHNode array (flattenBVHTree's depth-first preorder, BVHAccel.cpp:262-283) and the
// same orderedPrims.  The F8 tie rule makes that topology observable, so every step reproduces the
// sequential build exactly:
//   * box / centroid unions (Bounds3 Union = std::min / std::max, first operand kept on ties) are a
//     min over (value, position) keys with +-0 collapsed — the first minimal element in the range's
//     current order wins, as in the left-to-right loop (BVHAccel.cpp:104-105, 120-121, 184-191);
//   * the 12 bucket counts and boxes are the same keyed reductions per bucket; costs, the split
//     bucket and the leaf test are evaluated per node in the reference's operation order (:194-225);
//   * libstdc++'s bidirectional std::partition (:228-235) swaps the r-th element failing the
//     predicate from the front with the r-th passing one from the back: a ballot/popcount rank per
//     element gives both lists, then the swaps are independent;
//   * std::nth_element on two elements (:165-171) is insertion sort: swap iff c[1] < c[0].
// Nodes are built level by level (one wave per node's range).  Preorder positions need no
// bottom-up pass: a node at depth d whose root path has rc right-child steps and whose range starts
// at s has preorder index d + 2 * (leaves ending at or before s) - rc (every leaf left of it lies in
// one of the rc left-sibling subtrees, each of 2L - 1 nodes).  recursiveBuild builds the second child
// first (InitInterior's arguments are evaluated right to left, :250-254), so a leaf [s, e) holds
// orderedPrims[N - e, N - s).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "pbr_scene.h"

namespace pbr {

namespace {

constexpr int kNB = 12;       // BVHAccel.cpp:176 nBuckets
constexpr int kWave = 64;

struct SegRec { int start, end, depth, rc; };
struct NodeRec { int start, end, mid, depth, rc, axis; float box[6]; };   // mid < 0: leaf

__device__ inline uint32_t fkey(float x) {   // monotone float -> uint, +-0 collapsed (ties go by position)
    uint32_t u = __float_as_uint(x == 0.f ? 0.f : x);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline unsigned long long key_lo(float x, uint32_t pos) { return (unsigned long long)fkey(x) << 32 | pos; }
__device__ inline unsigned long long key_hi(float x, uint32_t pos) { return (unsigned long long)(~fkey(x)) << 32 | pos; }
__device__ inline unsigned long long umin64(unsigned long long a, unsigned long long b) { return b < a ? b : a; }
__device__ inline unsigned long long wave_min(unsigned long long v) {
    for (int o = kWave / 2; o > 0; o >>= 1) {
        uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
        v = umin64(v, (unsigned long long)hi << 32 | lo);
    }
    return v;
}
__device__ inline float comp(const float4& v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
// BVHPrimitiveInfo::centroid = .5f * pMin + .5f * pMax (BVHAccel.cpp:27-29)
__device__ inline float centroid(const float4& lo, const float4& hi, int a) { return .5f * comp(lo, a) + .5f * comp(hi, a); }
__device__ inline float mnf(float a, float b) { return (b < a) ? b : a; }   // std::min
__device__ inline float mxf(float a, float b) { return (a < b) ? b : a; }   // std::max
__device__ inline float area6(const float* b) {   // Bounds3::SurfaceArea
    float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    return 2 * (dx * dy + dx * dz + dy * dz);
}
// Bounds3::Offset(p)[dim] scaled to a bucket (BVHAccel.cpp:185-187)
__device__ inline int bucket_of(float c, float lo, float hi) {
    float o = c - lo;
    if (hi > lo) o /= hi - lo;
    int b = kNB * o;
    return b == kNB ? kNB - 1 : b;
}

// Children go to one of three lists by size.  A range above kBig is split by blocks of kBigBS threads, one
// per kChunk elements (k_big_*: keyed reductions through device-scope atomics into its BigAcc, counts per
// chunk for the partition ranks); a range above kSmall by one wave (k_bvh_level); a range of at most
// kSmall elements is finished — its whole subtree — by one thread running the sequential algorithm
// on a copy in LDS (k_bvh_small).
constexpr int kBig = 1024, kSmall = 8, kChunk = 2048, kBigBS = 256;
enum { LIST_BIG, LIST_MID, LIST_SMALL, CNT_CHUNKS, CNT_RECS, kCounters };   // the first four restart per level

struct BigAcc {
    unsigned long long key[12];        // box lo, box hi (key_hi), centroid lo, centroid hi
    unsigned long long bkey[kNB][6];
    int bcnt[kNB];
    int chunkBase, nChunks;
    int leaf, dim, split, P;           // the split decision (chunk 0 of k_big_count)
    float B[6];
};
struct ChunkRec { int seg, c; };

struct Lists {
    SegRec* l[3];
    BigAcc* acc;       // per LIST_BIG entry
    ChunkRec* chunks;  // the big ranges' chunks
};

__device__ inline void push_child(const Lists& nx, int* counters, SegRec r) {
    const int n = r.end - r.start;
    const int which = n > kBig ? LIST_BIG : (n > kSmall ? LIST_MID : LIST_SMALL);
    const int q = atomicAdd(&counters[which], 1);
    nx.l[which][q] = r;
    if (which != LIST_BIG) return;
    BigAcc& A = nx.acc[q];
    for (int i = 0; i < 12; ++i) A.key[i] = ~0ull;
    for (int k = 0; k < kNB; ++k) {
        A.bcnt[k] = 0;
        for (int i = 0; i < 6; ++i) A.bkey[k][i] = ~0ull;
    }
    const int nCh = (n + kChunk - 1) / kChunk, base = atomicAdd(&counters[CNT_CHUNKS], nCh);
    A.chunkBase = base;
    A.nChunks = nCh;
    for (int c = 0; c < nCh; ++c) nx.chunks[base + c] = ChunkRec{q, c};
}

__device__ inline void emit_node(NodeRec* recs, int* counters, int s, int e, int mid, int depth, int rc, int axis,
                                 const float* B) {
    NodeRec R;
    R.start = s; R.end = e; R.mid = mid; R.depth = depth; R.rc = rc; R.axis = axis;
    for (int a = 0; a < 6; ++a) R.box[a] = B[a];
    recs[atomicAdd(&counters[CNT_RECS], 1)] = R;
}

template <int BS>
__device__ inline unsigned long long block_min(unsigned long long v, unsigned long long* sh) {
    v = wave_min(v);
    if (BS == kWave) return v;
    const int w = threadIdx.x / kWave;
    __syncthreads();
    if ((threadIdx.x & (kWave - 1)) == 0) sh[w] = v;
    __syncthreads();
    unsigned long long r = sh[0];
    for (int i = 1; i < BS / kWave; ++i) r = umin64(r, sh[i]);
    return r;
}

// One block per range [start, end): decide leaf / split exactly as recursiveBuild, partition in place.
template <int BS>
__global__ __launch_bounds__(BS) void k_bvh_level(float4* __restrict__ items, int N, const SegRec* __restrict__ segs,
                                                 int nSegs, Lists nx, int* __restrict__ counters, NodeRec* __restrict__ recs,
                                                 int* __restrict__ leafMark, int32_t* __restrict__ primIds,
                                                 int* __restrict__ scratch, int maxPrims) {
    constexpr int NW = BS / kWave;
    __shared__ unsigned long long bkey[kNB][6];
    __shared__ int bcnt[kNB];
    __shared__ float bbox[kNB][6];
    __shared__ float cost[kNB];
    __shared__ unsigned long long red[NW];
    __shared__ int wcnt[2][NW];
    if ((int)blockIdx.x >= nSegs) return;
    const SegRec sg = segs[blockIdx.x];
    const int s = sg.start, e = sg.end, n = e - s, tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    const float4* it = items + 2 * (size_t)s;
    // 1. bounds and centroid bounds of the range (:104-105, :120-121)
    unsigned long long kb[6], kc[6];
    for (int a = 0; a < 6; ++a) kb[a] = kc[a] = ~0ull;
    for (int j = tid; j < n; j += BS) {
        const float4 lo = it[2 * j], hi = it[2 * j + 1];
        for (int a = 0; a < 3; ++a) {
            kb[a] = umin64(kb[a], key_lo(comp(lo, a), j));
            kb[a + 3] = umin64(kb[a + 3], key_hi(comp(hi, a), j));
            const float c = centroid(lo, hi, a);
            kc[a] = umin64(kc[a], key_lo(c, j));
            kc[a + 3] = umin64(kc[a + 3], key_hi(c, j));
        }
    }
    float B[6], C[6];
    for (int a = 0; a < 6; ++a) {
        const uint32_t pb = (uint32_t)block_min<BS>(kb[a], red), pc = (uint32_t)block_min<BS>(kc[a], red);
        const int ax = a % 3, hiSide = a / 3;
        B[a] = comp(it[2 * pb + hiSide], ax);
        C[a] = centroid(it[2 * pc], it[2 * pc + 1], ax);
    }
    bool leaf = false;
    int mid = 0, dim = 0;
    if (n == 1) {
        leaf = true;
    } else {
        const float dx = C[3] - C[0], dy = C[4] - C[1], dz = C[5] - C[2];   // Bounds3::MaximumExtent
        dim = (dx > dy && dx > dz) ? 0 : (dy > dz ? 1 : 2);
        const float clo = C[dim], chi = C[3 + dim];
        if (chi == clo) {
            leaf = true;
        } else if (n <= 2) {   // std::nth_element(start, mid, end) on two elements: insertion sort
            mid = s + 1;
            if (tid == 0) {
                const float4 l0 = it[0], h0 = it[1], l1 = it[2], h1 = it[3];
                if (centroid(l1, h1, dim) < centroid(l0, h0, dim)) {
                    items[2 * (size_t)s] = l1; items[2 * (size_t)s + 1] = h1;
                    items[2 * (size_t)s + 2] = l0; items[2 * (size_t)s + 3] = h0;
                }
            }
        } else {
            // 2. buckets (:179-192): keyed LDS minima per element
            for (int i = tid; i < kNB * 6; i += BS) bkey[i / 6][i % 6] = ~0ull;
            if (tid < kNB) bcnt[tid] = 0;
            __syncthreads();
            for (int j = tid; j < n; j += BS) {
                const float4 lo = it[2 * j], hi = it[2 * j + 1];
                const int k = bucket_of(centroid(lo, hi, dim), clo, chi);
                atomicAdd(&bcnt[k], 1);
                for (int a = 0; a < 3; ++a) {
                    atomicMin(&bkey[k][a], key_lo(comp(lo, a), j));
                    atomicMin(&bkey[k][a + 3], key_hi(comp(hi, a), j));
                }
            }
            __syncthreads();
            for (int i = tid; i < kNB * 6; i += BS) {   // decode; an empty bucket keeps Bounds3f()
                const int k = i / 6, a = i % 6;
                float v = a < 3 ? 3.40282347e+38f : -3.40282347e+38f;
                if (bcnt[k]) { const uint32_t p = (uint32_t)bkey[k][a]; v = comp(it[2 * p + a / 3], a % 3); }
                bbox[k][a] = v;
            }
            __syncthreads();
            // 3. split costs (:194-210), one per thread, in the reference's operation order
            if (tid < kNB - 1) {
                float b0[6] = {3.40282347e+38f, 3.40282347e+38f, 3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f};
                float b1[6] = {3.40282347e+38f, 3.40282347e+38f, 3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f};
                int c0 = 0, c1 = 0;
                for (int j = 0; j <= tid; ++j) {
                    for (int a = 0; a < 3; ++a) { b0[a] = mnf(b0[a], bbox[j][a]); b0[a + 3] = mxf(b0[a + 3], bbox[j][a + 3]); }
                    c0 += bcnt[j];
                }
                for (int j = tid + 1; j < kNB; ++j) {
                    for (int a = 0; a < 3; ++a) { b1[a] = mnf(b1[a], bbox[j][a]); b1[a + 3] = mxf(b1[a + 3], bbox[j][a + 3]); }
                    c1 += bcnt[j];
                }
                cost[tid] = 1 + (c0 * area6(b0) + c1 * area6(b1)) / area6(B);
            }
            __syncthreads();
            float minCost = cost[0];   // :213-219
            int split = 0;
            for (int i = 1; i < kNB - 1; ++i)
                if (cost[i] < minCost) { minCost = cost[i]; split = i; }
            const float leafCost = n;
            if (!(n > maxPrims || minCost < leafCost)) {
                leaf = true;
            } else {
                // 4. std::partition (:228-235): pair the r-th front failure with the r-th back success
                int P = 0;
                for (int k = 0; k <= split; ++k) P += bcnt[k];
                int rf = 0, rb = 0;
                const unsigned long long below = (1ull << lane) - 1;
                for (int base = 0; base < n; base += BS) {
                    const int j = base + tid;
                    bool pred = false;
                    if (j < n) pred = bucket_of(centroid(it[2 * j], it[2 * j + 1], dim), clo, chi) <= split;
                    const bool ff = j < n && j < P && !pred, bp = j < n && j >= P && pred;
                    const unsigned long long mf = __ballot(ff), mb = __ballot(bp);
                    int offF = 0, offB = 0, totF = __popcll(mf), totB = __popcll(mb);
                    if (NW > 1) {
                        if (lane == 0) { wcnt[0][w] = totF; wcnt[1][w] = totB; }
                        __syncthreads();
                        totF = totB = 0;
                        for (int i = 0; i < NW; ++i) {
                            if (i < w) { offF += wcnt[0][i]; offB += wcnt[1][i]; }
                            totF += wcnt[0][i];
                            totB += wcnt[1][i];
                        }
                        __syncthreads();
                    }
                    if (ff) scratch[s + rf + offF + __popcll(mf & below)] = j;
                    if (bp) scratch[s + P + rb + offB + __popcll(mb & below)] = j;
                    rf += totF;
                    rb += totB;
                }
                __threadfence_block();
                __syncthreads();
                const int m = rf;   // == rb
                for (int r = tid; r < m; r += BS) {
                    const size_t a = s + scratch[s + r], c = s + scratch[s + P + m - 1 - r];
                    const float4 la = items[2 * a], ha = items[2 * a + 1], lc = items[2 * c], hc = items[2 * c + 1];
                    items[2 * a] = lc; items[2 * a + 1] = hc;
                    items[2 * c] = la; items[2 * c + 1] = ha;
                }
                mid = s + P;
            }
        }
    }
    if (tid == 0) {
        emit_node(recs, counters, s, e, leaf ? -1 : mid, sg.depth, sg.rc, leaf ? 0 : dim, B);
        if (leaf) {
            leafMark[s] = 1;
        } else {
            push_child(nx, counters, SegRec{s, mid, sg.depth + 1, sg.rc});
            push_child(nx, counters, SegRec{mid, e, sg.depth + 1, sg.rc + 1});
        }
    }
    if (leaf)   // orderedPrims (:107-112): a leaf's range is final
        for (int j = tid; j < n; j += BS) primIds[N - e + j] = __float_as_int(it[2 * j].w);
}

// The range's bounds and centroid bounds from its 12 keyed minima (positions of the first extreme).
__device__ inline void decode_bounds(const float4* it, const unsigned long long* key, float* B, float* C) {
    for (int a = 0; a < 6; ++a) {
        const uint32_t pb = (uint32_t)key[a], pc = (uint32_t)key[6 + a];
        B[a] = comp(it[2 * pb + a / 3], a % 3);
        C[a] = centroid(it[2 * pc], it[2 * pc + 1], a % 3);
    }
}
__device__ inline int max_extent(const float* C) {   // Bounds3::MaximumExtent
    const float dx = C[3] - C[0], dy = C[4] - C[1], dz = C[5] - C[2];
    return (dx > dy && dx > dz) ? 0 : (dy > dz ? 1 : 2);
}

// k_big_*: one block per kChunk-element chunk of a big range.
__global__ __launch_bounds__(kBigBS) void k_big_bounds(const float4* __restrict__ items, Lists in) {
    __shared__ unsigned long long red[kBigBS / kWave];
    const ChunkRec ch = in.chunks[blockIdx.x];
    const SegRec sg = in.l[LIST_BIG][ch.seg];
    const int n = sg.end - sg.start, j0 = ch.c * kChunk, j1 = min(n, j0 + kChunk);
    const float4* it = items + 2 * (size_t)sg.start;
    unsigned long long k[12];
    for (int a = 0; a < 12; ++a) k[a] = ~0ull;
    for (int j = j0 + threadIdx.x; j < j1; j += kBigBS) {
        const float4 lo = it[2 * j], hi = it[2 * j + 1];
        for (int a = 0; a < 3; ++a) {
            k[a] = umin64(k[a], key_lo(comp(lo, a), j));
            k[a + 3] = umin64(k[a + 3], key_hi(comp(hi, a), j));
            const float c = centroid(lo, hi, a);
            k[6 + a] = umin64(k[6 + a], key_lo(c, j));
            k[9 + a] = umin64(k[9 + a], key_hi(c, j));
        }
    }
    for (int a = 0; a < 12; ++a) {
        const unsigned long long v = block_min<kBigBS>(k[a], red);
        if (threadIdx.x == 0) atomicMin(&in.acc[ch.seg].key[a], v);
    }
}

__global__ __launch_bounds__(kBigBS) void k_big_buckets(const float4* __restrict__ items, Lists in) {
    __shared__ unsigned long long bkey[kNB][6];
    __shared__ int bcnt[kNB];
    const ChunkRec ch = in.chunks[blockIdx.x];
    const SegRec sg = in.l[LIST_BIG][ch.seg];
    BigAcc& A = in.acc[ch.seg];
    const int n = sg.end - sg.start, j0 = ch.c * kChunk, j1 = min(n, j0 + kChunk), tid = threadIdx.x,
              lane = tid & (kWave - 1);
    const float4* it = items + 2 * (size_t)sg.start;
    float B[6], C[6];
    decode_bounds(it, A.key, B, C);
    const int dim = max_extent(C);
    const float clo = C[dim], chi = C[3 + dim];
    if (chi == clo) return;   // a leaf (k_big_count records it)
    for (int i = tid; i < kNB * 6; i += kBigBS) bkey[i / 6][i % 6] = ~0ull;
    if (tid < kNB) bcnt[tid] = 0;
    __syncthreads();
    for (int base = j0; base < j1; base += kBigBS) {
        const int j = base + tid;
        float4 lo = make_float4(0, 0, 0, 0), hi = lo;
        int k = -1;
        if (j < j1) { lo = it[2 * j]; hi = it[2 * j + 1]; k = bucket_of(centroid(lo, hi, dim), clo, chi); }
        bool pending = j < j1;
        unsigned long long pm = __ballot(pending);
        while (pm) {
            const int lead = __ffsll((unsigned long long)pm) - 1;
            const int kk = __shfl(k, lead);
            const bool mine = pending && k == kk;
            const unsigned long long cm = __ballot(mine);
            unsigned long long key[6];
            for (int a = 0; a < 3; ++a) {
                key[a] = wave_min(mine ? key_lo(comp(lo, a), j) : ~0ull);
                key[a + 3] = wave_min(mine ? key_hi(comp(hi, a), j) : ~0ull);
            }
            if (lane == lead) {
                atomicAdd(&bcnt[kk], __popcll(cm));
                for (int a = 0; a < 6; ++a) atomicMin(&bkey[kk][a], key[a]);
            }
            pending = pending && !mine;
            pm &= ~cm;
        }
    }
    __syncthreads();
    if (tid < kNB * 6 && bcnt[tid / 6]) atomicMin(&A.bkey[tid / 6][tid % 6], bkey[tid / 6][tid % 6]);
    if (tid < kNB && bcnt[tid]) atomicAdd(&A.bcnt[tid], bcnt[tid]);
}

// SAH split choice (BVHAccel.cpp:194-225) from decoded bucket boxes in LDS; every thread gets the answer.
__device__ inline void sah_choose(const float (*bbox)[6], const int* bcnt, const float* B, float* cost, int nThreads,
                                  int* split, float* minCost) {
    const int tid = threadIdx.x;
    if (tid < kNB - 1) {
        float b0[6] = {3.40282347e+38f, 3.40282347e+38f, 3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f};
        float b1[6] = {3.40282347e+38f, 3.40282347e+38f, 3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f};
        int c0 = 0, c1 = 0;
        for (int j = 0; j <= tid; ++j) {
            for (int a = 0; a < 3; ++a) { b0[a] = mnf(b0[a], bbox[j][a]); b0[a + 3] = mxf(b0[a + 3], bbox[j][a + 3]); }
            c0 += bcnt[j];
        }
        for (int j = tid + 1; j < kNB; ++j) {
            for (int a = 0; a < 3; ++a) { b1[a] = mnf(b1[a], bbox[j][a]); b1[a + 3] = mxf(b1[a + 3], bbox[j][a + 3]); }
            c1 += bcnt[j];
        }
        cost[tid] = 1 + (c0 * area6(b0) + c1 * area6(b1)) / area6(B);
    }
    __syncthreads();
    float m = cost[0];
    int sp = 0;
    for (int i = 1; i < kNB - 1; ++i)
        if (cost[i] < m) { m = cost[i]; sp = i; }
    *split = sp;
    *minCost = m;
}

__global__ __launch_bounds__(kBigBS) void k_big_count(const float4* __restrict__ items, Lists in, int2* __restrict__ chunkCnt,
                                                      int maxPrims) {
    __shared__ float bbox[kNB][6];
    __shared__ int bcnt[kNB];
    __shared__ float cost[kNB];
    __shared__ int tot[2];
    const ChunkRec ch = in.chunks[blockIdx.x];
    const SegRec sg = in.l[LIST_BIG][ch.seg];
    BigAcc& A = in.acc[ch.seg];
    const int n = sg.end - sg.start, j0 = ch.c * kChunk, j1 = min(n, j0 + kChunk), tid = threadIdx.x;
    const float4* it = items + 2 * (size_t)sg.start;
    float B[6], C[6];
    decode_bounds(it, A.key, B, C);
    const int dim = max_extent(C);
    const float clo = C[dim], chi = C[3 + dim];
    if (ch.c == 0 && tid == 0) {
        for (int a = 0; a < 6; ++a) A.B[a] = B[a];
        A.dim = dim;
        A.leaf = 1;
    }
    if (chi == clo) return;
    for (int i = tid; i < kNB * 6; i += kBigBS) {
        const int k = i / 6, a = i % 6;
        float v = a < 3 ? 3.40282347e+38f : -3.40282347e+38f;
        if (A.bcnt[k]) { const uint32_t p = (uint32_t)A.bkey[k][a]; v = comp(it[2 * p + a / 3], a % 3); }
        bbox[k][a] = v;
    }
    if (tid < kNB) bcnt[tid] = A.bcnt[tid];
    if (tid < 2) tot[tid] = 0;
    __syncthreads();
    int split;
    float minCost;
    sah_choose(bbox, bcnt, B, cost, kBigBS, &split, &minCost);
    const float leafCost = n;
    if (!(n > maxPrims || minCost < leafCost)) return;
    int P = 0;
    for (int k = 0; k <= split; ++k) P += bcnt[k];
    int ff = 0, bp = 0;
    for (int j = j0 + tid; j < j1; j += kBigBS) {
        const bool pred = bucket_of(centroid(it[2 * j], it[2 * j + 1], dim), clo, chi) <= split;
        ff += (j < P && !pred);
        bp += (j >= P && pred);
    }
    atomicAdd(&tot[0], ff);
    atomicAdd(&tot[1], bp);
    __syncthreads();
    if (tid == 0) {
        chunkCnt[A.chunkBase + ch.c] = make_int2(tot[0], tot[1]);
        if (ch.c == 0) { A.split = split; A.P = P; A.leaf = 0; }
    }
}

// Front failures and back successes in position order: ranks across chunks from the chunk counts.
__global__ __launch_bounds__(kBigBS) void k_big_lists(const float4* __restrict__ items, Lists in,
                                                      const int2* __restrict__ chunkCnt, int* __restrict__ scratch) {
    constexpr int NW = kBigBS / kWave;
    __shared__ int wcnt[2][NW];
    const ChunkRec ch = in.chunks[blockIdx.x];
    const SegRec sg = in.l[LIST_BIG][ch.seg];
    const BigAcc& A = in.acc[ch.seg];
    if (A.leaf) return;
    const int s = sg.start, n = sg.end - s, j0 = ch.c * kChunk, j1 = min(n, j0 + kChunk), tid = threadIdx.x,
              lane = tid & (kWave - 1), w = tid / kWave;
    const float4* it = items + 2 * (size_t)s;
    float C[6];
    for (int a = 0; a < 6; ++a) { const uint32_t pc = (uint32_t)A.key[6 + a]; C[a] = centroid(it[2 * pc], it[2 * pc + 1], a % 3); }
    const int dim = A.dim, split = A.split, P = A.P;
    const float clo = C[dim], chi = C[3 + dim];
    int rf = 0, rb = 0;
    for (int c = 0; c < ch.c; ++c) { const int2 t = chunkCnt[A.chunkBase + c]; rf += t.x; rb += t.y; }
    const unsigned long long below = (1ull << lane) - 1;
    for (int base = j0; base < j1; base += kBigBS) {
        const int j = base + tid;
        bool pred = false;
        if (j < j1) pred = bucket_of(centroid(it[2 * j], it[2 * j + 1], dim), clo, chi) <= split;
        const bool ff = j < j1 && j < P && !pred, bp = j < j1 && j >= P && pred;
        const unsigned long long mf = __ballot(ff), mb = __ballot(bp);
        if (lane == 0) { wcnt[0][w] = __popcll(mf); wcnt[1][w] = __popcll(mb); }
        __syncthreads();
        int offF = 0, offB = 0, totF = 0, totB = 0;
        for (int i = 0; i < NW; ++i) {
            if (i < w) { offF += wcnt[0][i]; offB += wcnt[1][i]; }
            totF += wcnt[0][i];
            totB += wcnt[1][i];
        }
        __syncthreads();
        if (ff) scratch[s + rf + offF + __popcll(mf & below)] = j;
        if (bp) scratch[s + P + rb + offB + __popcll(mb & below)] = j;
        rf += totF;
        rb += totB;
    }
}

__global__ __launch_bounds__(kBigBS) void k_big_swap(float4* __restrict__ items, Lists in, const int2* __restrict__ chunkCnt,
                                                     const int* __restrict__ scratch) {
    const ChunkRec ch = in.chunks[blockIdx.x];
    const SegRec sg = in.l[LIST_BIG][ch.seg];
    const BigAcc& A = in.acc[ch.seg];
    if (A.leaf) return;
    const int s = sg.start, P = A.P;
    int m = 0;
    for (int c = 0; c < A.nChunks; ++c) m += chunkCnt[A.chunkBase + c].x;
    const int r1 = min(m, (ch.c + 1) * kChunk);
    for (int r = ch.c * kChunk + threadIdx.x; r < r1; r += kBigBS) {
        const size_t a = s + scratch[s + r], c = s + scratch[s + P + m - 1 - r];
        const float4 la = items[2 * a], ha = items[2 * a + 1], lc = items[2 * c], hc = items[2 * c + 1];
        items[2 * a] = lc; items[2 * a + 1] = hc;
        items[2 * c] = la; items[2 * c + 1] = ha;
    }
}

// One wave per big range: the node record, its children or (a leaf) its primitives.
__global__ __launch_bounds__(kWave) void k_big_emit(const float4* __restrict__ items, int N, Lists in, int nSegs, Lists nx,
                                                    int* __restrict__ counters, NodeRec* __restrict__ recs,
                                                    int* __restrict__ leafMark, int32_t* __restrict__ primIds) {
    if ((int)blockIdx.x >= nSegs) return;
    const SegRec sg = in.l[LIST_BIG][blockIdx.x];
    const BigAcc& A = in.acc[blockIdx.x];
    const int s = sg.start, e = sg.end, n = e - s;
    const bool leaf = A.leaf != 0;
    const int mid = s + A.P;
    if (threadIdx.x == 0) {
        emit_node(recs, counters, s, e, leaf ? -1 : mid, sg.depth, sg.rc, leaf ? 0 : A.dim, A.B);
        if (leaf) {
            leafMark[s] = 1;
        } else {
            push_child(nx, counters, SegRec{s, mid, sg.depth + 1, sg.rc});
            push_child(nx, counters, SegRec{mid, e, sg.depth + 1, sg.rc + 1});
        }
    }
    if (leaf)
        for (int j = threadIdx.x; j < n; j += kWave) primIds[N - e + j] = __float_as_int(items[2 * ((size_t)s + j)].w);
}

// A small range's whole subtree, one thread, the sequential algorithm itself (first-wins unions in
// range order, libstdc++'s partition loop) on a private copy of the range in LDS ([slot][thread]).
constexpr int kSmallBS = 64;
__global__ __launch_bounds__(kSmallBS) void k_bvh_small(const float4* __restrict__ items, int N, const SegRec* __restrict__ segs,
                                                        int nSegs, int* __restrict__ counters, NodeRec* __restrict__ recs,
                                                        int* __restrict__ leafMark, int32_t* __restrict__ primIds, int maxPrims) {
    __shared__ float4 sIt[2 * kSmall][kSmallBS];
    __shared__ float sBB[kNB * 6][kSmallBS];
    __shared__ int sCnt[kNB][kSmallBS];
    __shared__ int4 sStack[kSmall + 1][kSmallBS];
    const int t = threadIdx.x, g = blockIdx.x * kSmallBS + t;
    if (g >= nSegs) return;
    const SegRec root = segs[g];
    const int base = root.start;
    for (int j = 0; j < 2 * (root.end - base); ++j) sIt[j][t] = items[2 * (size_t)base + j];
#define IT(j, h) sIt[2 * (j) + (h)][t]
    int sp = 0;
    sStack[sp++][t] = make_int4(root.start, root.end, root.depth, root.rc);
    const float BIG = 3.40282347e+38f;
    while (sp > 0) {
        const int4 sv = sStack[--sp][t];
        const int s = sv.x, e = sv.y, n = e - s, o = s - base;
        float B[6] = {BIG, BIG, BIG, -BIG, -BIG, -BIG}, C[6] = {BIG, BIG, BIG, -BIG, -BIG, -BIG};
        for (int j = o; j < o + n; ++j) {
            const float4 lo = IT(j, 0), hi = IT(j, 1);
            B[0] = mnf(B[0], lo.x); B[1] = mnf(B[1], lo.y); B[2] = mnf(B[2], lo.z);
            B[3] = mxf(B[3], hi.x); B[4] = mxf(B[4], hi.y); B[5] = mxf(B[5], hi.z);
        }
        bool leaf = n == 1;
        int mid = 0, dim = 0;
        if (!leaf) {
            for (int j = o; j < o + n; ++j) {
                const float4 lo = IT(j, 0), hi = IT(j, 1);
                for (int a = 0; a < 3; ++a) {
                    const float c = centroid(lo, hi, a);
                    C[a] = mnf(C[a], c);
                    C[a + 3] = mxf(C[a + 3], c);
                }
            }
            dim = max_extent(C);
            const float clo = C[dim], chi = C[3 + dim];
            if (chi == clo) {
                leaf = true;
            } else if (n <= 2) {
                mid = s + 1;
                const float4 l0 = IT(o, 0), h0 = IT(o, 1), l1 = IT(o + 1, 0), h1 = IT(o + 1, 1);
                if (centroid(l1, h1, dim) < centroid(l0, h0, dim)) { IT(o, 0) = l1; IT(o, 1) = h1; IT(o + 1, 0) = l0; IT(o + 1, 1) = h0; }
            } else {
                for (int k = 0; k < kNB; ++k) {
                    sCnt[k][t] = 0;
                    for (int a = 0; a < 3; ++a) { sBB[6 * k + a][t] = BIG; sBB[6 * k + a + 3][t] = -BIG; }
                }
                for (int j = o; j < o + n; ++j) {
                    const float4 lo = IT(j, 0), hi = IT(j, 1);
                    const int k = bucket_of(centroid(lo, hi, dim), clo, chi);
                    sCnt[k][t]++;
                    sBB[6 * k + 0][t] = mnf(sBB[6 * k + 0][t], lo.x);
                    sBB[6 * k + 1][t] = mnf(sBB[6 * k + 1][t], lo.y);
                    sBB[6 * k + 2][t] = mnf(sBB[6 * k + 2][t], lo.z);
                    sBB[6 * k + 3][t] = mxf(sBB[6 * k + 3][t], hi.x);
                    sBB[6 * k + 4][t] = mxf(sBB[6 * k + 4][t], hi.y);
                    sBB[6 * k + 5][t] = mxf(sBB[6 * k + 5][t], hi.z);
                }
                float minCost = 0;
                int split = 0;
                const float A = area6(B);
                for (int i = 0; i < kNB - 1; ++i) {
                    float b0[6] = {BIG, BIG, BIG, -BIG, -BIG, -BIG}, b1[6] = {BIG, BIG, BIG, -BIG, -BIG, -BIG};
                    int c0 = 0, c1 = 0;
                    for (int j = 0; j < kNB; ++j) {
                        float* bx = j <= i ? b0 : b1;
                        for (int a = 0; a < 3; ++a) { bx[a] = mnf(bx[a], sBB[6 * j + a][t]); bx[a + 3] = mxf(bx[a + 3], sBB[6 * j + a + 3][t]); }
                        if (j <= i) c0 += sCnt[j][t];
                        else c1 += sCnt[j][t];
                    }
                    const float c = 1 + (c0 * area6(b0) + c1 * area6(b1)) / A;
                    if (i == 0 || c < minCost) { minCost = c; split = i; }
                }
                const float leafCost = n;
                if (!(n > maxPrims || minCost < leafCost)) {
                    leaf = true;
                } else {   // libstdc++ std::__partition, bidirectional
                    int f = o, l = o + n;
                    for (;;) {
                        for (;;) {
                            if (f == l) goto done;
                            if (bucket_of(centroid(IT(f, 0), IT(f, 1), dim), clo, chi) <= split) ++f;
                            else break;
                        }
                        --l;
                        for (;;) {
                            if (f == l) goto done;
                            if (!(bucket_of(centroid(IT(l, 0), IT(l, 1), dim), clo, chi) <= split)) --l;
                            else break;
                        }
                        {
                            const float4 la = IT(f, 0), ha = IT(f, 1);
                            IT(f, 0) = IT(l, 0); IT(f, 1) = IT(l, 1);
                            IT(l, 0) = la; IT(l, 1) = ha;
                        }
                        ++f;
                    }
                done:
                    mid = base + f;
                }
            }
        }
        emit_node(recs, counters, s, e, leaf ? -1 : mid, sv.z, sv.w, leaf ? 0 : dim, B);
        if (leaf) {
            leafMark[s] = 1;
            for (int j = 0; j < n; ++j) primIds[N - e + j] = __float_as_int(IT(o + j, 0).w);
        } else {
            sStack[sp++][t] = make_int4(mid, e, sv.z + 1, sv.w + 1);
            sStack[sp++][t] = make_int4(s, mid, sv.z + 1, sv.w);
        }
    }
#undef IT
}

// Exclusive prefix sum of n ints (leaf marks): block sums, one block over the sums, add back.
constexpr int kScanBlock = 1024;
__device__ inline int block_incl_scan(int v, int* sh) {
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    for (int o = 1; o < kWave; o <<= 1) {
        const int t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    if (lane == kWave - 1) sh[w] = v;
    __syncthreads();
    if (w == 0) {
        int x = lane < (int)(blockDim.x / kWave) ? sh[lane] : 0;
        for (int o = 1; o < kWave; o <<= 1) {
            const int t = __shfl_up(x, o);
            if (lane >= o) x += t;
        }
        sh[lane] = x;
    }
    __syncthreads();
    return v + (w > 0 ? sh[w - 1] : 0);
}
__global__ __launch_bounds__(kScanBlock) void k_scan_local(const int* __restrict__ in, int* __restrict__ out, int n, int* __restrict__ sums) {
    __shared__ int sh[kWave];
    const int i = blockIdx.x * kScanBlock + threadIdx.x;
    const int v = i < n ? in[i] : 0;
    const int incl = block_incl_scan(v, sh);
    if (i < n) out[i] = incl - v;
    if (threadIdx.x == kScanBlock - 1) sums[blockIdx.x] = incl;
}
__global__ __launch_bounds__(kScanBlock) void k_scan_sums(int* __restrict__ sums, int nb) {
    __shared__ int sh[kWave];
    int carry = 0;
    for (int base = 0; base < nb; base += kScanBlock) {
        const int i = base + threadIdx.x;
        const int v = i < nb ? sums[i] : 0;
        const int incl = block_incl_scan(v, sh);
        const int total = sh[kScanBlock / kWave - 1];
        __syncthreads();
        if (i < nb) sums[i] = carry + incl - v;
        carry += total;
    }
}
__global__ __launch_bounds__(256) void k_scan_add(int* __restrict__ out, int n, const int* __restrict__ sums) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] += sums[i / kScanBlock];
}

// flattenBVHTree (:262-283): every node record to its preorder slot.
__global__ __launch_bounds__(256) void k_bvh_emit(const NodeRec* __restrict__ recs, int nRecs, const int* __restrict__ lb,
                                                  int N, LinearBVHNode* __restrict__ nodes) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nRecs) return;
    const NodeRec R = recs[i];
    const int pre = R.depth + 2 * lb[R.start] - R.rc;
    LinearBVHNode o;
    for (int a = 0; a < 3; ++a) { o.pMin[a] = R.box[a]; o.pMax[a] = R.box[a + 3]; }
    o.pad = 0;
    o.axis = (uint8_t)R.axis;
    if (R.mid < 0) {
        o.offset = N - R.end;
        o.nPrimitives = (uint16_t)(R.end - R.start);
    } else {
        o.offset = R.depth + 2 * lb[R.mid] - R.rc;   // the second child: depth + 1, one more right step
        o.nPrimitives = 0;
    }
    nodes[pre] = o;
}

__global__ void k_bvh_root(Lists l, int* counters, int N) { push_child(l, counters, SegRec{0, N, 0, 0}); }

struct Mem {
    std::vector<void*> ps;
    ~Mem() { for (void* p : ps) (void)hipFree(p); }
    template <class T> hipError_t get(T** p, size_t count) {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, count ? count * sizeof(T) : 16);
        if (e == hipSuccess) ps.push_back(q);
        *p = (T*)q;
        return e;
    }
};

}  // namespace

void device_build_bvh(void* stream_, const std::vector<float>& primBounds, int maxPrims, std::vector<LinearBVHNode>* nodes,
                      std::vector<int32_t>* primIds, double* kernelMs) {
    hipStream_t st = (hipStream_t)stream_;
    const size_t nn = primBounds.size() / 6;
    if (nn >= (size_t)1 << 30) throw std::invalid_argument("too many primitives for the device BVH build");
    const int N = (int)nn;
    nodes->clear();
    primIds->clear();
    if (kernelMs) *kernelMs = 0;
    if (N == 0) return;
    maxPrims = std::min(255, std::max(1, maxPrims));
#define BVH_TRY(x)                                                                                 \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)
    // BVHPrimitiveInfo array in prims order: float4 pMin (w = primitive number), float4 pMax
    std::vector<float> packed((size_t)N * 8);
    for (int i = 0; i < N; ++i) {
        const float* b = &primBounds[(size_t)i * 6];
        float* p = &packed[(size_t)i * 8];
        p[0] = b[0]; p[1] = b[1]; p[2] = b[2];
        std::memcpy(&p[3], &i, 4);
        p[4] = b[3]; p[5] = b[4]; p[6] = b[5]; p[7] = 0.f;
    }
    Mem mem;
    float4* dItems; NodeRec* dRecs; int *dMark, *dLB, *dScratch, *dCnt, *dSums; int32_t* dIds; int2* dChunkCnt;
    LinearBVHNode* dNodes;
    Lists lists[2];
    const int nb = (N + kScanBlock - 1) / kScanBlock;
    const int maxBig = N / kBig + 2, maxChunks = N / kChunk + maxBig;
    BVH_TRY(mem.get(&dItems, (size_t)N * 2));
    for (int b = 0; b < 2; ++b) {
        for (int l = 0; l < 3; ++l) BVH_TRY(mem.get(&lists[b].l[l], N));
        BVH_TRY(mem.get(&lists[b].acc, maxBig));
        BVH_TRY(mem.get(&lists[b].chunks, maxChunks));
    }
    BVH_TRY(mem.get(&dChunkCnt, maxChunks));
    BVH_TRY(mem.get(&dRecs, (size_t)2 * N));
    BVH_TRY(mem.get(&dMark, N));
    BVH_TRY(mem.get(&dLB, N));
    BVH_TRY(mem.get(&dScratch, N));
    BVH_TRY(mem.get(&dCnt, kCounters));
    BVH_TRY(mem.get(&dSums, nb));
    BVH_TRY(mem.get(&dIds, N));
    BVH_TRY(mem.get(&dNodes, (size_t)2 * N));
    int* hCnt = nullptr;
    BVH_TRY(hipHostMalloc((void**)&hCnt, kCounters * sizeof(int), hipHostMallocDefault));
    struct PinFree { int* p; ~PinFree() { if (p) (void)hipHostFree(p); } } pinGuard{hCnt};
    hipEvent_t ev0, ev1;
    BVH_TRY(hipEventCreate(&ev0));
    BVH_TRY(hipEventCreate(&ev1));
    struct EvFree { hipEvent_t a, b; ~EvFree() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); } } evGuard{ev0, ev1};
    BVH_TRY(hipMemcpyAsync(dItems, packed.data(), packed.size() * 4, hipMemcpyHostToDevice, st));
    BVH_TRY(hipMemsetAsync(dMark, 0, (size_t)N * 4, st));
    BVH_TRY(hipMemsetAsync(dCnt, 0, kCounters * 4, st));
    BVH_TRY(hipEventRecord(ev0, st));
    hipLaunchKernelGGL(k_bvh_root, dim3(1), dim3(1), 0, st, lists[0], dCnt, N);
    BVH_TRY(hipGetLastError());
    BVH_TRY(hipMemcpyAsync(hCnt, dCnt, kCounters * sizeof(int), hipMemcpyDeviceToHost, st));
    BVH_TRY(hipStreamSynchronize(st));
    int nIn[4] = {hCnt[0], hCnt[1], hCnt[2], hCnt[3]};
    for (int level = 0, cur = 0; nIn[0] + nIn[1] + nIn[2] > 0; ++level, cur ^= 1) {
        if (level > 1 << 20) throw std::runtime_error("device BVH build: runaway level count");
        const Lists& in = lists[cur];
        const Lists& out = lists[cur ^ 1];
        BVH_TRY(hipMemsetAsync(dCnt, 0, 4 * sizeof(int), st));   // the output lists' counts (CNT_RECS runs on)
        if (nIn[LIST_BIG]) {
            const dim3 g(nIn[CNT_CHUNKS]), b(kBigBS);
            hipLaunchKernelGGL(k_big_bounds, g, b, 0, st, dItems, in);
            hipLaunchKernelGGL(k_big_buckets, g, b, 0, st, dItems, in);
            hipLaunchKernelGGL(k_big_count, g, b, 0, st, dItems, in, dChunkCnt, maxPrims);
            hipLaunchKernelGGL(k_big_lists, g, b, 0, st, dItems, in, dChunkCnt, dScratch);
            hipLaunchKernelGGL(k_big_swap, g, b, 0, st, dItems, in, dChunkCnt, dScratch);
            hipLaunchKernelGGL(k_big_emit, dim3(nIn[LIST_BIG]), dim3(kWave), 0, st, dItems, N, in, nIn[LIST_BIG], out, dCnt,
                               dRecs, dMark, dIds);
        }
        if (nIn[LIST_MID])
            hipLaunchKernelGGL(k_bvh_level<kWave>, dim3(nIn[LIST_MID]), dim3(kWave), 0, st, dItems, N, in.l[LIST_MID],
                               nIn[LIST_MID], out, dCnt, dRecs, dMark, dIds, dScratch, maxPrims);
        if (nIn[LIST_SMALL])
            hipLaunchKernelGGL(k_bvh_small, dim3((nIn[LIST_SMALL] + kSmallBS - 1) / kSmallBS), dim3(kSmallBS), 0, st, dItems,
                               N, in.l[LIST_SMALL], nIn[LIST_SMALL], dCnt, dRecs, dMark, dIds, maxPrims);
        BVH_TRY(hipGetLastError());
        BVH_TRY(hipMemcpyAsync(hCnt, dCnt, kCounters * sizeof(int), hipMemcpyDeviceToHost, st));
        BVH_TRY(hipStreamSynchronize(st));
        for (int l = 0; l < 4; ++l) {
            nIn[l] = hCnt[l];
            if (nIn[l] < 0 || nIn[l] > N || (l == LIST_BIG && nIn[l] > maxBig) || (l == CNT_CHUNKS && nIn[l] > maxChunks))
                throw std::runtime_error("device BVH build: bad range count");
        }
    }
    const int nRecs = hCnt[CNT_RECS];
    if (nRecs < 1 || nRecs > 2 * N - 1) throw std::runtime_error("device BVH build: bad node count");
    hipLaunchKernelGGL(k_scan_local, dim3(nb), dim3(kScanBlock), 0, st, dMark, dLB, N, dSums);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kScanBlock), 0, st, dSums, nb);
    hipLaunchKernelGGL(k_scan_add, dim3((N + 255) / 256), dim3(256), 0, st, dLB, N, dSums);
    hipLaunchKernelGGL(k_bvh_emit, dim3((nRecs + 255) / 256), dim3(256), 0, st, dRecs, nRecs, dLB, N, dNodes);
    BVH_TRY(hipGetLastError());
    BVH_TRY(hipEventRecord(ev1, st));
    nodes->resize(nRecs);
    primIds->resize(N);
    BVH_TRY(hipMemcpyAsync(nodes->data(), dNodes, (size_t)nRecs * sizeof(LinearBVHNode), hipMemcpyDeviceToHost, st));
    BVH_TRY(hipMemcpyAsync(primIds->data(), dIds, (size_t)N * 4, hipMemcpyDeviceToHost, st));
    BVH_TRY(hipStreamSynchronize(st));
    interior_bounds_from_children(nodes);   // InitInterior's Union(c0, c1): the sign of a zero (pbr_scene.cpp)
    float ms = 0;
    BVH_TRY(hipEventElapsedTime(&ms, ev0, ev1));
    if (kernelMs) *kernelMs = ms;
#undef BVH_TRY
}

}  // namespace pbr
