// pbr_wavefront.h — wavefront schedule for WhittedIntegrator::Li (WhittedIntegrator.cpp:11-65).
// Included by pbr_kernels.hip inside its anonymous namespace (uses KParams, the sampler, film_out).
//
// The megakernel keeps a whole recursion's state live while it traverses the BVH, which caps it at
// 2 waves/SIMD.  Here each stage is its own small kernel, so the latency-bound traversals run at
// high occupancy:
//
//   k_wf_camera_extend   sampler dims 0-4 → camera ray → closest hit          (level 0, 1 lane/sample)
//   k_wf_shade           SI + BSDF; light sample → shadow queue; SpecularReflect → next ray queue
//   k_wf_shadow          any-hit; visible → rec[depth].A += contribution   (one light → no ordering issue)
//   k_wf_extend          closest hit for the continuation queue
//   k_wf_finish          fold L_k = A_k + ((F_k·L_{k+1})·c_k)/pdf_k deepest-first, per-pixel in-order sum, film
//
// Queues are SoA in HBM.  The shade kernel runs kWfBlocks workgroups and workgroup b appends to
// segment b ([b·segCap, b·segCap + count[b])) of the queues it writes, through an LDS counter
// (ballot + popcount per wave) — no device-scope atomic: one counter hit by every wave of the grid
// serialised the level-0 shade (1015 µs → 274 µs per 2^23-sample launch without it).  Consumers
// read a segmented queue densely: each workgroup scans the kWfBlocks counts into LDS and maps its
// grid-stride index to (segment, offset) by binary search, so the traversal kernels stay load
// balanced (reading segment b in workgroup b was measured 16% slower overall).  Records are indexed
// by sample, so the fold reproduces the recursive evaluation bit for bit in any queue order.
#pragma once

constexpr int kWfMaxDepth = 16;   // Whitted levels of the wavefront schedule (deeper: the megakernel)
#ifndef PBR_WF_BLOCKS
#define PBR_WF_BLOCKS 2048
#endif
constexpr int kWfBlocks = PBR_WF_BLOCKS;   // workgroups of the queue kernels = segments of a queue
static_assert(kWfBlocks % 256 == 0, "the segment scan reads kWfBlocks / 256 counts per thread");

// Per-kernel profile (pbr_hip_set_profiling): kernel families and their work counters
// [kind * kProfFields + field].  Field 0 counts the units a family processed, fields 1..4 the
// entries it pushed (or, for the any-hit kernels, the rays that got through), field 5 the units
// read from a segmented queue (beyond level 0: one more 4-B id each).
enum ProfKind {
    KP_WF_CAMERA, KP_WF_SHADE, KP_WF_SHADOW, KP_WF_EXTEND, KP_WF_FINISH,
    KP_WFP_CAMERA, KP_WFP_SHADE, KP_WFP_SHADOW, KP_WFP_PROBE, KP_WFP_RESOLVE, KP_WFP_FINISH,
    KP_WFV_SHADE, KP_WFV_TR, KP_WFV_RESOLVE, KP_MEGA,
    KP_WF_SHADE0,   // k_wf_shade's fused level-0 launches (camera rays traced in the shade): own family
    KP_COUNT
};
constexpr int kProfFields = 8;
// wave-aggregated count of the lanes for which pred holds (every active lane must call it)
__device__ __forceinline__ void prof_count(unsigned long long* ctr, bool pred) {
    const unsigned long long m = __ballot(pred), act = __ballot(1);
    if (m && (int)__lane_id() == __ffsll((long long)act) - 1) atomicAdd(ctr, (unsigned long long)__popcll(m));
}
// a per-lane count added once per wave (every active lane must call it): the lane-refill kernels count
// in a register while they trace and add at the end, so a profiled launch runs the same loop as an
// unprofiled one (a per-completion atomic had slowed the counting window's any-hit launches 2-8x)
__device__ __forceinline__ void prof_add(unsigned long long* ctr, unsigned v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const unsigned long long act = __ballot(1);
    if (v && (int)__lane_id() == __ffsll((long long)act) - 1) atomicAdd(ctr, (unsigned long long)v);
}

struct WfQueue {
    float4* o;      // origin.xyz, tMax (the hit distance once a closest-hit kernel has traced the ray)
    float4* d;      // dir.xyz, packed (dim | depth << 16) as int bits
    int* id;        // sample index within the chunk
    float4* hit;    // slot (int bits, -1 = miss), b0, b1, b2
    float4* s0;     // Path/VolPath state carried with the ray: L.rgb, beta.r
    float4* s1;     //   beta.g, beta.b, etaScale, the sample's global index (bits)
    int* segCount;  // [kWfBlocks]; null for the dense level-0 queue
};
struct WfParams {
    KParams P;
    long long chunkPix0;   // first packed pixel of the chunk
    int chunkPix;          // pixels in the chunk
    int nSamples;          // chunkPix * spp
    int segCap;            // capacity of one queue segment
    WfQueue cur, next;
    // shadow queue (segmented like the ray queues)
    float4* so; float4* sd; float4* sc; int* sid; int* shadowSeg;
    // SkyBox light (single-light schedule): the sampled direction wi of each shadow entry; the sky's
    // radiance is looked up in k_wf_shadow, for visible rays only (skyDeferred)
    float4* sw;
    int skyDeferred;
    // per-sample records, [depth * cap + sample]
    float4* recA;          // A.rgb, flags (bit0: add +0 at the end)
    float4* recF;          // F.rgb, cos term
    float* recP;           // pdf
    int* depthOf;          // deepest level of each sample
    uint32_t* sampleIndex; // Halton global index of each sample (GlobalSampler::SetSampleNumber)
    int cap;               // record stride (>= nSamples)
    int initRecords;       // some primitive has no material (Whitted's pass-through branch)
    int shadowSegCap;      // capacity of one shadow-queue segment (segCap × lights per shade)
    // multi-light Whitted (k_wf_shade_ml): per (level, light, sample) the light's contribution and
    // whether its shadow ray got through, [(depth * nLightsML + light) * cap + id]
    float4* recC;
    uint8_t* recV;
    int nLightsML;         // 0: the single-light schedule
    unsigned long long* prof;   // profile counters (ProfKind rows) while profiling, else null
};

// XCD-aware workgroup order: the dispatcher deals workgroup b to XCD b % 8, each XCD with its own
// L2.  Kernels whose grid is a whole number of rounds of 8 runs of K = PBR_XCD_RUN workgroups (the
// camera kernels, the kWfBlocks-wide shade kernels, resolve) work on a logical workgroup such
// that K consecutive logical workgroups — consecutive queue entries, so neighbouring pixels — run on
// one XCD, the runs dealt round-robin over the XCDs; that XCD's L2 then holds the part of the BVH,
// mesh and sky the run touches.  Queue segments are numbered by the logical workgroup, so queue
// order is unchanged, and records are indexed by sample, so frames are bit-identical either way.
// Measured (profiles/r2_xcd_ab.log): K = 128 C2 -1.2..-1.6%, C3 -3.0..-3.9%, C5 ±0.3%; one
// contiguous band per XCD C2 +5.6% (unbalanced); runs of 32 in the resident-size traversal grids
// (1792 = 7 × 256 workgroups, not a multiple of 8 × 128, so left in dispatch order here) C2 +1%.
#ifndef PBR_XCD_RUN
#define PBR_XCD_RUN 128
#endif
constexpr int kXcds = 8;
__device__ __forceinline__ int wf_block() {
    const int G = (int)gridDim.x, b = (int)blockIdx.x;
    constexpr int K = PBR_XCD_RUN;
    if constexpr (K == 0) return b;
    else {
        if (G % (kXcds * K) != 0) return b;
        const int x = b % kXcds, k = b / kXcds;   // the k-th workgroup dealt to XCD x
        return ((k / K) * kXcds + x) * K + k % K;
    }
}

// The same remap for the resident-size lane-refill traversal grids (5-7 workgroups per CU, so
// G = 1280-1792): runs of PBR_XCD_TRAV_RUN workgroups per XCD (-1: one contiguous band per XCD,
// 0: dispatch order).
#ifndef PBR_XCD_TRAV_RUN
#define PBR_XCD_TRAV_RUN 0
#endif
__device__ __forceinline__ int trav_block() {
    const int G = (int)gridDim.x, b = (int)blockIdx.x;
    constexpr int K = PBR_XCD_TRAV_RUN;
    if constexpr (K == 0) return b;
    else {
        if (G % kXcds != 0) return b;
        const int per = G / kXcds, run = K < 0 ? per : K;
        if (per % run != 0) return b;
        const int x = b % kXcds, k = b / kXcds;
        return ((k / run) * kXcds + x) * run + k % run;
    }
}

// LDS counter; the wave's lanes must be converged
__device__ __forceinline__ int wave_push(int* counter, bool pred) {
    unsigned long long m = __ballot(pred);
    int lane = (int)__lane_id();
    int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (m != 0ull && lane == leader) base = atomicAdd(counter, (int)__popcll(m));
    base = __shfl(base, leader < 0 ? 0 : leader);
    return pred ? base + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}
__device__ __forceinline__ int pack_dd(int dim, int depth) { return (dim & 0xffff) | (depth << 16); }

// Exclusive prefix of the kWfBlocks segment counts into s_off[0..kWfBlocks] (whole workgroup of
// 256); returns the total.
__shared__ int s_seg_off[kWfBlocks + 1];
constexpr int kSegCoarse = kWfBlocks / 64;     // segments per coarse bucket of seg_pos_wave
static_assert(kSegCoarse >= 1 && kSegCoarse <= 32, "seg_pos_wave: a 64-way then a 32-way ballot");
__shared__ int s_seg_coarse[64];                // s_seg_off[k * kSegCoarse]: conflict-free for 64 lanes
__device__ int seg_scan(const int* counts) {
    constexpr int per = kWfBlocks / 256;
    __shared__ int s_wave[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int local[per], sum = 0;
    for (int i = 0; i < per; ++i) { local[i] = counts[t * per + i]; sum += local[i]; }
    int incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) s_wave[w] = incl;
    __syncthreads();
    int excl = incl - sum;
    for (int k = 0; k < w; ++k) excl += s_wave[k];
    for (int i = 0; i < per; ++i) {
        const int g = t * per + i;
        s_seg_off[g] = excl;
        if (g % kSegCoarse == 0) s_seg_coarse[g / kSegCoarse] = excl;
        excl += local[i];
    }
    if (t == 255) s_seg_off[kWfBlocks] = excl;
    __syncthreads();
    return s_seg_off[kWfBlocks];
}
// dense index q < total → queue position: the last segment whose offset is <= q holds it
__device__ __forceinline__ int seg_pos(int segCap, int q) {
    int lo = 0, hi = kWfBlocks;
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (s_seg_off[mid] <= q) lo = mid; else hi = mid;
    }
    return lo * segCap + (q - s_seg_off[lo]);
}
// seg_pos for a wave whose lanes look up dense indices in [lo, hi] (wave-uniform, 0 <= lo <= hi):
// the same position, from two LDS round trips instead of seg_pos's 11 dependent ones.  A 64-way
// ballot over the coarse offsets and a 32-way one over the chosen bucket's offsets (lanes 0-31 for
// lo, 32-63 for hi) find the last segments whose offsets are <= lo and <= hi — the offsets are
// nondecreasing, so each ballot is a prefix of lanes — and each lane bisects between the two, which
// bracket its answer (usually one segment: no step).  Every lane of the wave must call it (full
// exec); lanes whose q lies outside [lo, hi] get a position inside the queue that they must not use.
#ifndef PBR_SEG_WAVE
#define PBR_SEG_WAVE 1
#endif
__device__ __forceinline__ int seg_pos_wave(int segCap, int q, int lo, int hi) {
    if constexpr (!PBR_SEG_WAVE) return seg_pos(segCap, q);
    // (the lane's LDS addresses are formed here, not hoisted out of the caller's loop, where they
    // would hold VGPRs across a shade kernel's whole body)
    int lane = (int)__lane_id();
    asm volatile("" : "+v"(lane));
    const int cv = s_seg_coarse[lane];
    const int cLo = __popcll(__ballot(cv <= lo)) - 1, cHi = __popcll(__ballot(cv <= hi)) - 1;   // >= 0: offset 0 is 0
    const int k = lane & 31;
    const int c = lane < 32 ? cLo : cHi, tgt = lane < 32 ? lo : hi;
    const unsigned long long m = __ballot(k < kSegCoarse && s_seg_off[c * kSegCoarse + min(k, kSegCoarse - 1)] <= tgt);
    int a = cLo * kSegCoarse + __popc((unsigned)m) - 1;             // last segment with offset <= lo
    int b = cHi * kSegCoarse + __popc((unsigned)(m >> 32));         // one past the last with offset <= hi
    while (b - a > 1) {                                             // offset[a] <= q < offset[b] (or b = end)
        const int mid = (a + b) >> 1;
        if (s_seg_off[mid] <= q) a = mid; else b = mid;
    }
    return a * segCap + (q - s_seg_off[a]);
}
// The position of dense index i in a wave-uniform loop over n entries whose wave holds 64 consecutive
// indices (i = the wave's first + lane; every lane calls it).  Lanes with i >= n get an unusable
// position; a wave wholly past n skips the search.
__device__ __forceinline__ int seg_pos_dense(int segCap, int i, int n) {
    const int w0 = __builtin_amdgcn_readfirstlane(i - (int)__lane_id());
    if (w0 >= n) return 0;
    return seg_pos_wave(segCap, min(i, n - 1), w0, min(w0 + 63, n - 1));
}

// Queue traversal with lane refill (Aila & Laine's "replace terminated rays").  Incoherent rays
// (Path/VolPath continuations, shadow and probe rays) need very different numbers of traversal steps,
// and a wave that traces 64 of them at a time runs until its slowest lane is done: measured SIMD
// utilisation of the traversal loop 0.27 (C3 continuations, 9.25 steps per ray), 0.29 (C3 shadow),
// 0.33 (probe), against 0.96 for the coherent camera rays (tools/trav_diag.py).  Here every lane of a
// wave keeps its own ray state, the loop runs one traversal step (a quad node, or a leaf and the pops
// after it) per iteration, and once at least PBR_REFILL lanes are idle they take the wave's next rays.
// The wave's rays are those the grid-stride loop would give it (batches of 64 consecutive queue
// entries, `stride` apart), so the load balance over waves is unchanged.  Each ray's traversal — node
// order, primitive order, ray.tMax updates — is exactly traverse_quad's, so results are identical.
#ifndef PBR_REFILL
#define PBR_REFILL 16
#endif
// Workgroups per CU the lane-refill traversal kernels are compiled for.  Keeping 64 lanes busy
// needs more registers per lane (at 7 the closest-hit loop spilled 19 VGPRs).  Measured (C3 / C5
// ms per frame of the family, bit-identical): closest hit (extend) 7: 175 / 610, 6: 163 / 587,
// 5: 155 / 584; any hit (shadow) 7: 107, 6: 126, 5: 122; transmittance (C5) 7: 546, 6: 518, 5: 582.
// Round 5, built without the SLP vectorizer (62 VGPRs): any hit 8 — C4-material shadow 99.9 → 82.3
// ms, C3 quarter 19.2 → 15.5 (profiles/r5_slp_ab.log); closest hit 6 with the 8-entry LDS stack
// (kRefillShort).
#ifndef PBR_REFILL_OCC
#define PBR_REFILL_OCC 6
#endif
#ifndef PBR_REFILL_OCC_ANY
#define PBR_REFILL_OCC_ANY 8
#endif
#ifndef PBR_REFILL_OCC_TR
#define PBR_REFILL_OCC_TR 6
#endif
constexpr int kRefill = PBR_REFILL;

static_assert(kRefill >= 1 && kRefill <= 64, "refill threshold: idle lanes of a 64-wide wave");
// LDS short-stack entries of the camera kernels.  They have no segment scan, so 7 workgroups per CU
// would fit 10 entries (20 KB): C2's camera kernel then took 8.95 → 8.02 ms/frame, but the other
// lane's extend, sharing the CUs, 5.28 → 6.75 and the frame 17.7 → 18.0 ms — kept at 6.
#ifndef PBR_CAMERA_SHORT
#define PBR_CAMERA_SHORT PBR_SHORT_STACK_DEPTH
#endif
constexpr int kCameraShort = PBR_CAMERA_SHORT;

// The queue holds n rays in segments of segCap (seg_scan has run); load(q, &key) → the ray at queue
// position q (key: what store needs, e.g. q); store(key, hit, ray, h) → the ray's result (closest
// hit: ray.tMax and h; any hit: hit only).
template <bool ANY, int SHORT, bool NF = true, class Load, class Store>
__device__ void traverse_stream(const DeviceScene& S, int n, int segCap, Load load, Store store,
                                unsigned long long* diag = nullptr, int diagKind = 0) {
    const int lane = (int)__lane_id();
    const int stride = (int)(gridDim.x * blockDim.x);
    const int wbase = trav_block() * (int)blockDim.x + ((int)threadIdx.x & ~63);
    auto rayOf = [&](int j) { return (j >> 6) * stride + wbase + (j & 63); };   // increasing in j
    const unsigned long long below = (1ull << lane) - 1ull;
    int* lref;
    float* lt;
    trav_lds<SHORT>(&lref, &lt);
    constexpr int PRIV = kTraversalStack - SHORT;
    int stackRef[PRIV];
    float stackT[PRIV];
    int cursor = 0;              // wave-uniform: the next ray of the wave's sequence
    bool have = false;           // the lane holds a ray in flight
    int key = 0, cur = 0, sp = 0;
    bool found = false;
    Ray r;
    f3 inv = mk(0, 0, 0);
    bool n0 = false, n1 = false, n2 = false;
    HitRec h;
    h.slot = -1; h.b0 = h.b1 = h.b2 = 0.f;
    unsigned long long laneSteps = 0, waveSteps = 0;
    (void)laneSteps; (void)waveSteps;
    int maxSp = 0;   // PBR_STACK_DIAG: the ray's deepest stack
    (void)maxSp;
    // the binary root's box, read once (scalar): a refilled ray's first test waits on no fetch
    float4 rootA = make_float4(0.f, 0.f, 0.f, 0.f), rootB = rootA;
    if (S.nNodes > 0) {
        const ScalarF4Ptr w = scalar_f4(S.nodes);
        rootA = as_f4(w[0]); rootB = as_f4(w[1]);
    }
    while (true) {
        const unsigned long long idle = __ballot(!have);
        const int nIdle = __popcll(idle);
        if (nIdle >= kRefill && rayOf(cursor) < n) {   // wave-uniform (every lane is here)
            const int i = rayOf(cursor + __popcll(idle & below));   // this lane's ray if it is idle
            const int iHi = min(rayOf(cursor + nIdle - 1), n - 1);   // the idle lanes' rays: rayOf(cursor) ..
            const int qi = seg_pos_wave(segCap, min(i, iHi), rayOf(cursor), iHi);
            if (!have) {
                if (i < n) {
                    r = load(qi, &key);
                    found = false;
                    h.slot = -1; h.b0 = h.b1 = h.b2 = 0.f;
                    // traverse(): the root is visited first (the binary root box)
                    bool ok = S.nNodes > 0;
                    if (ok) {
                        inv = ANY ? mk(1.f / r.d.x, 1.f / r.d.y, 1.f / r.d.z) : mk(1 / r.d.x, 1 / r.d.y, 1 / r.d.z);
                        n0 = inv.x < 0; n1 = inv.y < 0; n2 = inv.z < 0;
                        ok = node_hit(rootA, rootB, r, inv, n0, n1, n2);
                    }
                    if (ok) {
                        cur = S.quadRootRef;
                        sp = 0;
                        maxSp = 0;
                        have = true;
                    } else {
                        store(key, false, r, h);
                    }
                }
            }
            cursor += nIdle;
        }
        if (__ballot(have) == 0ull) {
            if (rayOf(cursor) >= n) break;
            continue;
        }
        if constexpr (PBR_TRAV_DIAG) { waveSteps += 64; laneSteps += have ? 1 : 0; }
        if (!have) continue;
        bool done = false;
        bool descend = false;
        if (cur < 0) {   // leaf: its slots run up to the one flagged PRIM_LEAF_END
            int slot = cur & 0x7fffffff;
            while (true) {
                float4 v0, v1, v2;
                const int uslot = __builtin_amdgcn_readfirstlane(slot);
                if (kScalarLoads && __builtin_amdgcn_ballot_w64(slot != uslot) == 0ull) {
                    const ScalarF4Ptr tv = scalar_f4(S.triVerts + 3 * (size_t)uslot);
                    v0 = as_f4(tv[0]); v1 = as_f4(tv[1]); v2 = as_f4(tv[2]);
                } else {
                    const float4* tv = S.triVerts + 3 * (size_t)slot;
                    v0 = tv[0]; v1 = tv[1]; v2 = tv[2];
                }
                const int flags = __float_as_int(v0.w);
                float t, b0 = 0, b1 = 0, b2 = 0;
                const bool hit = (flags & PRIM_SPHERE)
                                     ? sphere_test(S.spheres[__float_as_int(v0.x)], r, &t)
                                     : tri_test(mk(v0.x, v0.y, v0.z), mk(v1.x, v1.y, v1.z), mk(v2.x, v2.y, v2.z), r, &t, &b0, &b1, &b2);
                if (hit) {
                    found = true;
                    if (ANY) { done = true; break; }
                    r.tMax = t;   // GeometricPrimitive::Intersect (Primitive.cpp:26)
                    h.slot = slot; h.b0 = b0; h.b1 = b1; h.b2 = b2;
                }
                if (flags & PRIM_LEAF_END) break;
                ++slot;
            }
        } else {
            QuadSlots q;
            quad_slots<ANY, NF>(S, cur, r, inv, n0, n1, n2, &q);
            const float tM = r.tMax;
            const bool p0 = q.k[0] && q.t[0] < tM, p1 = q.k[1] && q.t[1] < tM, p2 = q.k[2] && q.t[2] < tM,
                       p3 = q.k[3] && q.t[3] < tM;
            if ((p0 | p1 | p2 | p3) && sp > kQuadStackLimit) {   // unreachable (upload check): end the walk
                atomicOr(S.guard, kGuardStack);
                done = true;
            } else if (p0 | p1 | p2 | p3) {
                const int first = p0 ? 0 : (p1 ? 1 : (p2 ? 2 : 3));
                auto push = [&](int ref, float t) {
                    if (SHORT && sp < SHORT) { lref[sp * 256] = ref; if (!ANY) lt[sp * 256] = t; }
                    else { stackRef[sp - SHORT] = ref; if (!ANY) stackT[sp - SHORT] = t; }
                    ++sp;
                };
                if (p3 && first < 3) push(q.ref[3], q.t[3]);
                if (p2 && first < 2) push(q.ref[2], q.t[2]);
                if (p1 && first < 1) push(q.ref[1], q.t[1]);
                if constexpr (PBR_STACK_DIAG) maxSp = max(maxSp, sp);
                cur = first == 0 ? q.ref[0] : (first == 1 ? q.ref[1] : (first == 2 ? q.ref[2] : q.ref[3]));
                descend = true;
            }
        }
        if (!done && !descend) {   // pop until an entry passes its box test against the current tMax
            bool more = false;
            while (sp > 0) {
                --sp;
                if (ANY) { cur = (SHORT && sp < SHORT) ? lref[sp * 256] : stackRef[sp - SHORT]; more = true; break; }
                int rr;
                float tt;
                if (SHORT && sp < SHORT) { rr = lref[sp * 256]; tt = lt[sp * 256]; }
                else { rr = stackRef[sp - SHORT]; tt = stackT[sp - SHORT]; }
                if (tt < r.tMax) { cur = rr; more = true; break; }
            }
            done = !more;
        }
        if (done) {
            if constexpr (PBR_STACK_DIAG) {   // rays whose stack went past 6 / 10 / 16 / 24 entries
                if (diag) {
                    prof_count(diag + diagKind * kProfFields + 2, maxSp > 6);
                    prof_count(diag + diagKind * kProfFields + 3, maxSp > 10);
                    prof_count(diag + diagKind * kProfFields + 4, maxSp > 16);
                    prof_count(diag + diagKind * kProfFields + 5, maxSp > 24);
                }
            }
            store(key, found, r, h);
            have = false;
        }
    }
#if PBR_TRAV_DIAG
    if (diag) {
        unsigned long long sum = laneSteps;
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
        if (lane == 0) {
            atomicAdd(diag + diagKind * 8 + 6, sum);
            atomicAdd(diag + diagKind * 8 + 7, waveSteps);
        }
    }
#endif
}

template <int SHORT>
__global__ __launch_bounds__(256, PBR_TRAV_OCC) void k_wf_camera_extend(WfParams W) {
    const KParams& P = W.P;
    int q = wf_block() * blockDim.x + threadIdx.x;
    if (q >= W.nSamples) return;
    int lp = q / P.spp, s = q - lp * P.spp;
    int x, y;
    pixel_xy(P, W.chunkPix0 + lp, &x, &y);
    SState st;
    st.index = sample_index(P.smp, x, y, s).lo;
    st.sid = s;
    st.dim = 0;
    st.px = x;
    st.py = y;
    Ray r = camera_sample_ray(P, st, x, y);
    HitRec h;
    Counters c;
    bool hit;
    if constexpr (kPacket && kQuadTraversal) {   // a wave holds one pixel's samples: coherent
        h.slot = -1; h.b0 = h.b1 = h.b2 = 0.f;
        hit = traverse_wave<false>(P.S, r, &h, true);
    } else {
        hit = traverse<false, false, SHORT>(P.S, r, &h, &c);
    }
    trav_diag(W.prof, KP_WF_CAMERA, h);
    W.cur.o[q] = make_float4(r.o.x, r.o.y, r.o.z, r.tMax);
    W.cur.d[q] = make_float4(r.d.x, r.d.y, r.d.z, __int_as_float(pack_dd(st.dim, 0)));
    W.sampleIndex[q] = st.index;   // the level-0 queue is dense: queue slot == sample id
    if (W.initRecords) {           // only pass-through levels can leave a sample without records
        W.depthOf[q] = 0;          // a sample dropped by the level cap reads black
        W.recA[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    W.cur.hit[q] = make_float4(__int_as_float(hit ? h.slot : -1), h.b0, h.b1, h.b2);
}

// REFILL: the lane-refill traversal (Path/VolPath continuations: C3 204 → 179 ms/frame of extend,
// C5 760 → 617).  Whitted's mirror continuations are coherent (SIMD utilisation 0.90 without
// refill) and keep the plain loop: with refill C2's extend took 5.4 → 8.6 ms.
template <int SHORT, bool REFILL = false>
__global__ __launch_bounds__(256, REFILL ? PBR_REFILL_OCC : PBR_TRAV_OCC) void k_wf_extend(WfParams W) {
    const int n = seg_scan(W.cur.segCount);
    if constexpr (REFILL && kRefill > 0 && SHORT > 0 && kQuadTraversal) {
        traverse_stream<false, kRefillShort>(
            W.P.S, n, W.segCap,
            [&](int q, int* key) {
                *key = q;
                const float4 o = W.cur.o[q], d = W.cur.d[q];
                return mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
            },
            [&](int q, bool hit, const Ray& r, const HitRec& h) {
                W.cur.o[q] = make_float4(r.o.x, r.o.y, r.o.z, r.tMax);
                W.cur.hit[q] = make_float4(__int_as_float(hit ? h.slot : -1), h.b0, h.b1, h.b2);
            },
            W.prof, KP_WF_EXTEND);
        return;
    }
    // (per-lane seg_pos: the wave-cooperative lookup made this 63-VGPR packet walk spill 2)
    for (int i = wf_block() * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int q = seg_pos(W.segCap, i);
        float4 o = W.cur.o[q], d = W.cur.d[q];
        Ray r = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
        HitRec h;
        Counters c;
        bool hit;
        if constexpr (kPacket && PBR_PACKET_EXTEND && kQuadTraversal) {   // Whitted's mirror continuations stay coherent
            h.slot = -1; h.b0 = h.b1 = h.b2 = 0.f;
            hit = traverse_wave<false>(W.P.S, r, &h, true);
        } else {
            hit = traverse<false, false, SHORT>(W.P.S, r, &h, &c);
        }
        trav_diag(W.prof, KP_WF_EXTEND, h);
        // the whole 16-B origin record is rewritten with the hit distance: full-line stores.  Measured
        // (bit-identical; C3 / C5 / C2 frame ms): o.w alone 325 / 1642 / 17.66, the whole record
        // 321 / 1646 / 17.73, a separate dense t[] array 349 / 1736 / 18.94 (the traversal loop's
        // register allocation got worse: 13 scratch reloads instead of 9)
        W.cur.o[q] = make_float4(r.o.x, r.o.y, r.o.z, r.tMax);
        W.cur.hit[q] = make_float4(__int_as_float(hit ? h.slot : -1), h.b0, h.b1, h.b2);
    }
}

// One level of WhittedIntegrator::Li for every queued ray (single-light scenes).  LOBES: the lobe
// kinds present in the scene (kSimpleLobes drops the microfacet code and its registers).
constexpr int kSimpleLobes = (1 << L_LAMBERT) | (1 << L_OREN) | (1 << L_SPEC_R) | (1 << L_SPEC_T) | (1 << L_FRESNEL_SPEC);
// Lambert and rough (microfacet) reflection / transmission only — matte, plastic, metal and rough
// glass: the Path/VolPath shading kernels for C4 and C5 without the specular and Oren-Nayar code
constexpr int kMicroLobes = (1 << L_LAMBERT) | (1 << L_MF_R) | (1 << L_MF_T);
// Lambert and perfect mirror reflection only — matte (σ = 0) and mirror materials: C2's dragon and
// floor, C3's scene
constexpr int kMatteMirrorLobes = (1 << L_LAMBERT) | (1 << L_SPEC_R);
// MATS_LDS: the material templates fit kLdsMats and are read from an LDS copy (the BSDF code walks
// them with dependent loads).
constexpr int kLdsMats = 32;
__shared__ MatTemplate s_mats[kLdsMats];

// Waves per SIMD of the Whitted shade kernel for the simple lobe set (C2).  Measured (C2 ms):
// round 1 4: 19.97, 3: 20.16, 5: 20.11; round 3 4: 17.91-18.02, 3: 18.64, 5: 18.55.
#ifndef PBR_WF_SHADE_OCC
#define PBR_WF_SHADE_OCC 4
#endif
#ifndef PBR_WF_SHADE_OCC_MM
#define PBR_WF_SHADE_OCC_MM PBR_WF_SHADE_OCC
#endif
// Round 5: with the per-ray body as a lambda the fused level-0 SkyBox shade needs 96 VGPRs (112
// before), so 5 workgroups per CU fit in registers; they fit in LDS once its material templates are
// read from global memory instead of an LDS copy (30.4 KB instead of 37.8).  C2 14.58 → 14.15 ms
// (profiles/r5_fused_occ_ab.log; the LDS copy alone at 4: 14.63).
#ifndef PBR_WF_FUSED_OCC
#define PBR_WF_FUSED_OCC 5
#endif
#ifndef PBR_WF_FUSED_MATS_LDS
#define PBR_WF_FUSED_MATS_LDS 0
#endif
// k_wf_camera_extend's work for queue position q inside the level-0 shade (CAMERA): the camera
// sample's ray and its closest hit, as the queue entry the shade would have read.  Every lane of
// the wave calls it (the packet walk is wave-wide); `active` lanes hold a sample.
template <bool PINHOLE = false, int KIND = -1>
__device__ __forceinline__ void camera_trace(const WfParams& W, bool active, int q, float4* o, float4* d, float4* hr,
                                             uint32_t* index) {
    const KParams& P = W.P;
    Ray r;
    r.o = mk(0, 0, 0); r.d = mk(0, 0, 1); r.tMax = 0; r.medium = -1;
    int dim = 0;
    if (active) {
        const int lp = q / P.spp, s = q - lp * P.spp;
        int x, y;
        pixel_xy(P, W.chunkPix0 + lp, &x, &y);
        SState st;
        st.index = sample_index<KIND>(P.smp, x, y, s).lo;
        st.sid = s;
        st.dim = 0;
        st.px = x;
        st.py = y;
        r = camera_sample_ray<PINHOLE, KIND>(P, st, x, y);
        dim = st.dim;
        *index = st.index;
        W.sampleIndex[q] = st.index;   // later levels read it by sample id
        if (W.initRecords) {
            W.depthOf[q] = 0;
            W.recA[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    HitRec h;
    h.slot = -1; h.b0 = h.b1 = h.b2 = 0.f;
    const bool hit = traverse_wave<false>(P.S, r, &h, active);
    *o = make_float4(r.o.x, r.o.y, r.o.z, r.tMax);
    *d = make_float4(r.d.x, r.d.y, r.d.z, __int_as_float(pack_dd(dim, 0)));
    *hr = make_float4(__int_as_float(hit ? h.slot : -1), h.b0, h.b1, h.b2);
}

// CAMERA (level 0 only): the shade generates and traces its camera rays itself — the camera
// kernel's 52-B queue entry is neither written nor read back, and the chunk has one launch fewer.
// The walk is the camera kernel's wave packet.  Measured (bit-identical, C2 frame ms): 17.33-17.39
// → 17.18 (profiles/r3_fused_ab.log).  Tracing the continuations inside the later shades as well
// (no extend launch) was slower: 17.46.
//
// SKY (untextured lobes, the scene's one light is a SkyBox, a pinhole camera — C2): the kernel
// holds only the SkyBox branches and no lens sampling, and the light sample's direction wi = UniformSampleSphere(u) is computed before the hit's
// geometry, where few values are live across its out-of-line sin/cos call (the calls clobber every
// caller-saved VGPR; around the late call the shade spilled its whole shading state).  The draw is
// the light loop's own (same dimensions, same sample index), made under the same condition: a
// material make_bsdf accepts, with a non-specular lobe.
template <int LOBES, bool MATS_LDS,
          int OCC = (LOBES & ~kSimpleLobes) ? 2 : (LOBES == kMatteMirrorLobes ? PBR_WF_SHADE_OCC_MM : PBR_WF_SHADE_OCC),
          bool CAMERA = false, bool SKY = false>
__global__ __launch_bounds__(256, OCC) void k_wf_shade(WfParams W, int level0) {
    static_assert(!SKY || (LOBES & kTexturedLobes) == 0, "the SkyBox variant is untextured");
    constexpr int kSmp = SKY ? PBR_SAMPLER_HALTON : -1;   // the SkyBox variants run Halton frames only
    const KParams& P = W.P;
    const DeviceScene& S = P.S;
    stage_halton_lds(P.smp);
    const MatTemplate* mats = S.materials;
    if constexpr (MATS_LDS) {
        constexpr int words = (int)(sizeof(MatTemplate) / 4);
        const int n = 2 * S.nMaterials * words;
        const uint32_t* src = (const uint32_t*)S.materials;
        uint32_t* dst = (uint32_t*)s_mats;
        for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
        mats = s_mats;
    }
    __shared__ int s_push[2];   // shadow, next
    if (threadIdx.x < 2) s_push[threadIdx.x] = 0;
    __syncthreads();
    const int n = level0 ? W.nSamples : seg_scan(W.cur.segCount);
    const int stride = gridDim.x * blockDim.x;
    const int nIter = (n + stride - 1) / stride;   // <= segCap / 256: a segment holds all pushes
    const int base = wf_block() * W.segCap, sbase = wf_block() * W.shadowSegCap;
    // one queued ray (a lambda: its registers are allocated apart from the loop's, as k_wfp_shade's)
    auto shade = [&](const bool active, const int q) {
        bool pushShadow = false, pushNext = false;
        int id = 0, depth = 0, dim = 0, emitDepth = 0;
        Ray ray, shadow, cont;
        rgb contrib = sp(0.f);
        float skyCos = 0.f;
        f3 skyWi = mk(0, 0, 0);
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f), d = o, hr = o;
        uint32_t camIndex = 0;
        if constexpr (CAMERA) camera_trace<SKY, kSmp>(W, active, q, &o, &d, &hr, &camIndex);   // level 0 only
        else if (active) { o = W.cur.o[q]; d = W.cur.d[q]; hr = W.cur.hit[q]; }
        if (active) {
            id = level0 ? q : W.cur.id[q];
            int dd = __float_as_int(d.w);
            dim = dd & 0xffff;
            depth = dd >> 16;
            emitDepth = depth;
            ray = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
            int slot = __float_as_int(hr.x);
            size_t ri = (size_t)depth * W.cap + id;
            if (slot < 0) {   // miss: Σ over all lights of Le (F4)
                rgb L = sp(0.f);
                if constexpr (SKY) {   // light_Le's SkyBox branch
                    const DLight& light = S.lights[0];
                    float u, v;
                    sphere_uv(normalize(ray.d), &u, &v);
                    L = L + (light.envW > 0 ? sky_value(S, light, u, v) : sp(0.f));
                }
                else for (int i = 0; i < S.nLights; ++i) L = L + light_Le(S, S.lights[i], ray);
                W.recA[ri] = make_float4(L.r, L.g, L.b, 0.f);
                W.depthOf[id] = depth;
            } else {
                f3 skyDir = mk(0, 0, 0);
                if constexpr (SKY) {
                    const int mat = S.primInfo[slot].y;
                    if (mat >= 0 && mats[2 * mat].valid && num_components(mats[2 * mat], BSDF_ALL & ~BSDF_SPECULAR) > 0) {
                        SState t;
                        t.index = CAMERA ? camIndex : W.sampleIndex[id];
                        t.sid = id; t.dim = dim; t.px = t.py = 0;
                        float a, b;
                        get2d<true, kSmp>(P.smp, t, &a, &b);
                        skyDir = uniform_sphere(a, b);
                    }
                }
                Isect isect;
                int flags = __float_as_int(S.triVerts[3 * (size_t)slot].w);
                if (flags & PRIM_SPHERE) sphere_si(S.spheres[__float_as_int(S.triVerts[3 * (size_t)slot].x)], ray, ray.tMax, &isect);
                else triangle_si(S, slot, ray, hr.y, hr.z, hr.w, flags, &isect);
                isect.slot = slot;
                isect.medIn = isect.medOut = -1;
                BSDF bsdf;
                MatTemplate texLocal;   // a textured material's per-hit lobes (make_bsdf)
                if (!make_bsdf<(LOBES & kTexturedLobes) != 0>(S, mats, isect, false, &bsdf, &texLocal)) {
                    cont = spawn_ray(isect, ray.d);        // Li(isect.SpawnRay(ray.d), depth)
                    pushNext = true;
                } else {
                    f3 n = isect.sn, wo = isect.wo;
                    rgb L = sp(0.f);
                    L = L + si_Le(S, isect, wo);
                    SState st;
                    st.index = CAMERA ? camIndex : W.sampleIndex[id];
                    st.sid = id;   // ≡ the sample number mod spp (pixel-major ids)
                    st.dim = dim;
                    st.px = st.py = 0;   // dims >= 2 only past the camera
                    {   // the single light (WhittedIntegrator.cpp:39-54)
                        float a, b;
                        get2d<true, kSmp>(P.smp, st, &a, &b);
                        // Reordered but equivalent: f(wo, wi) does not depend on Li, and nothing is
                        // added when f is black — so the light's radiance (for the SkyBox: atan2,
                        // asin and an env gather) is only evaluated when f is not black, and a
                        // purely specular BSDF (f ≡ 0) skips the light sample altogether.
                        if (num_components(bsdf, BSDF_ALL & ~BSDF_SPECULAR) > 0) {
                            f3 wi;
                            float pdf;
                            VisPt vis;
                            const DLight& light = S.lights[0];
                            rgb Li;
                            if (SKY || light.type == LT_SKY) {
                                // The sky's radiance Li(wi) (atan2, asin and a texel gather) moves to the
                                // shadow kernel, evaluated for the rays that get through: the term is
                                // f·Li·|wi·n|/pdf added when Li is not black and the ray is unoccluded,
                                // and neither test has side effects, so the order does not matter.  The
                                // entry carries f, |wi·n| and wi (W.sw); the sum is formed there in the
                                // same operation order.
                                wi = SKY ? skyDir : uniform_sphere(a, b);   // SKY: drawn above, same (a, b)
                                vis.p = isect.p + wi * (2 * light.worldRadius); vis.pError = mk(0, 0, 0); vis.n = mk(0, 0, 0);
                                rgb f = bsdf_f<LOBES>(bsdf, wo, wi, BSDF_ALL);
                                if (!black(f) && light.envW > 0) {
                                    contrib = f;
                                    skyCos = absdot(wi, n);
                                    skyWi = wi;
                                    shadow = spawn_ray_to(isect, vis.p, vis.pError, vis.n);
                                    pushShadow = true;
                                }
                            } else if constexpr (!SKY) {
                                Li = sample_li(S, light, isect, a, b, &wi, &pdf, &vis);
                                if (!(black(Li) || pdf == 0)) {
                                    rgb f = bsdf_f<LOBES>(bsdf, wo, wi, BSDF_ALL);
                                    if (!black(f)) {
                                        contrib = f * Li * absdot(wi, n) / pdf;
                                        shadow = spawn_ray_to(isect, vis.p, vis.pError, vis.n);
                                        pushShadow = true;
                                    }
                                }
                            }
                        }
                    }
                    float flagsA = 0.f;
                    bool final_ = true;
                    // SpecularReflect (Integrator.cpp:179-222).  A BSDF without a specular reflection lobe
                    // returns black from Sample_f whatever the sample (Reflection.cpp:113-114), and the
                    // path ends here, so the two sampler dimensions are not drawn (C2's matte dragon)
                    if (depth + 1 < P.maxDepth && num_components(bsdf, BSDF_REFLECTION | BSDF_SPECULAR) == 0) {
                        flagsA = 1.f;   // L += Spectrum(0) from a failed SpecularReflect
                    } else if (depth + 1 < P.maxDepth) {
                        f3 wi = mk(0, 0, 0);
                        float pdf = 0;
                        int stype = 0;
                        float a, b;
                        get2d<true, kSmp>(P.smp, st, &a, &b);
                        // only L_SPEC_R lobes match BSDF_REFLECTION | BSDF_SPECULAR
                        rgb f = bsdf_sample<(1 << L_SPEC_R)>(bsdf, wo, &wi, a, b, &pdf, BSDF_REFLECTION | BSDF_SPECULAR, &stype);
                        if (!black(f) && pdf > 0.f && absdot(wi, isect.sn) != 0.f && depth + 1 < kWfMaxDepth) {
                            W.recF[ri] = make_float4(f.r, f.g, f.b, absdot(wi, isect.sn));
                            W.recP[ri] = pdf;
                            cont = spawn_ray(isect, wi);
                            pushNext = true;
                            final_ = false;
                            depth += 1;
                        } else {
                            flagsA = 1.f;   // L += Spectrum(0) from a failed SpecularReflect
                        }
                    }
                    W.recA[ri] = make_float4(L.r, L.g, L.b, flagsA);
                    if (final_) W.depthOf[id] = depth;
                    dim = st.dim;
                }
            }
        }
        int si = sbase + wave_push(&s_push[0], pushShadow);
        if (pushShadow) {   // the visibility result lands in the level that emitted the ray
            W.so[si] = make_float4(shadow.o.x, shadow.o.y, shadow.o.z, shadow.tMax);
            W.sd[si] = make_float4(shadow.d.x, shadow.d.y, shadow.d.z, __int_as_float(emitDepth));
            W.sc[si] = make_float4(contrib.r, contrib.g, contrib.b, skyCos);
            W.sid[si] = id;
            if (W.skyDeferred) W.sw[si] = make_float4(skyWi.x, skyWi.y, skyWi.z, 0.f);
        }
        int ni = base + wave_push(&s_push[1], pushNext);
        if (pushNext) {
            W.next.o[ni] = make_float4(cont.o.x, cont.o.y, cont.o.z, cont.tMax);
            W.next.d[ni] = make_float4(cont.d.x, cont.d.y, cont.d.z, __int_as_float(pack_dd(dim, depth)));
            W.next.id[ni] = id;
        }
    };
    for (int it = 0; it < nIter; ++it) {   // uniform trip count: wave_push needs convergent lanes
        const int i = it * stride + wf_block() * blockDim.x + threadIdx.x;
        const bool active = i < n;
        const int q = level0 ? i : seg_pos_dense(W.segCap, i, n);
        shade(active, active ? q : 0);
    }
    __syncthreads();
    if (threadIdx.x == 0) { W.shadowSeg[wf_block()] = s_push[0]; W.next.segCount[wf_block()] = s_push[1]; }
}

// any-hit for the shadow queue; a visible light adds its contribution to the emitting level.
// Per-lane walks: C2's shadow rays leave one pixel's surface patch in uniform sphere directions, and
// wave-packet walks of them (build order) took the frame 17.2 → 22.4 ms (profiles/r3_post.log).
template <int SHORT>
__global__ __launch_bounds__(256, PBR_TRAV_OCC) void k_wf_shadow(WfParams W) {
    const int n = seg_scan(W.shadowSeg);
    // Whitted's shadow rays keep the plain loop: lane refill (traverse_stream) measured 5.45 → 5.90
    // ms/frame on C2 (refill 16), 5.40 (refill 32)
    for (int i0 = wf_block() * blockDim.x + ((int)threadIdx.x & ~63); i0 < n; i0 += gridDim.x * blockDim.x) {   // per wave
        const int i = i0 + (int)__lane_id();
        const int q = seg_pos_dense(W.shadowSegCap, i, n);
        if (i >= n) continue;
        float4 o = W.so[q], d = W.sd[q];
        Ray r = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
        HitRec h;
        Counters c;
        const bool visible = !traverse<true, false, SHORT>(W.P.S, r, &h, &c);
        trav_diag(W.prof, KP_WF_SHADOW, h);
        if (W.prof) prof_count(W.prof + KP_WF_SHADOW * kProfFields + 1, visible);
        if (W.prof && W.skyDeferred) prof_count(W.prof + KP_WF_SHADOW * kProfFields + 2, visible);
        if (visible) {
            int id = W.sid[q];
            float4 cc = W.sc[q];
            if (W.skyDeferred) {   // SkyBox light: cc = (f, |wi·n|), the term f·Li·|wi·n|/pdf (k_wf_shade)
                const DLight& light = W.P.S.lights[0];
                const float4 w4 = W.sw[q];
                float ul, vl;
                sphere_uv(normalize(mk(w4.x, w4.y, w4.z)), &ul, &vl);
                const rgb Li = sky_value(W.P.S, light, ul, vl);
                if (black(Li)) continue;
                const rgb c = sp3(cc.x, cc.y, cc.z) * Li * cc.w / (1.f / (4 * kPi));
                cc = make_float4(c.r, c.g, c.b, 0.f);
            }
            size_t ri = (size_t)__float_as_int(d.w) * W.cap + id;
            float4 A = W.recA[ri];
            A.x = A.x + cc.x; A.y = A.y + cc.y; A.z = A.z + cc.z;
            W.recA[ri] = A;
        }
    }
}

// Fold the recursion and run the film.  A workgroup takes finishPixels() whole pixels (<= 2048
// samples): one thread per sample folds L_k = A_k + ((F_k·L_{k+1})·c_k)/pdf_k deepest-first
// (coalesced record reads) into LDS laid out [pixel][channel][sample] with a pitch of spp + 1
// (conflict-free), then one thread per (pixel, channel) adds that pixel's samples in sample order
// — the reference's colObj += Li order; Spectrum addition is per channel — and one thread per
// pixel runs the film.
// One level of WhittedIntegrator::Li for scenes with 2..kWfMaxLightsML lights.  The light loop
// (WhittedIntegrator.cpp:39-54) runs for every lane of the wave — lanes with nothing to shade just
// consume no sampler dimensions — so each light's shadow rays are pushed with one ballot; a light
// whose shadow ray is pushed leaves its contribution in recC and recV = 0, which k_wf_shadow_ml
// turns to 1 when the ray gets through.  Everything else is k_wf_shade.
constexpr int kWfMaxLightsML = 8;
template <int LOBES, bool MATS_LDS, int OCC = (LOBES & ~kSimpleLobes) ? 2 : 3>
__global__ __launch_bounds__(256, OCC) void k_wf_shade_ml(WfParams W, int level0) {
    const KParams& P = W.P;
    const DeviceScene& S = P.S;
    stage_halton_lds(P.smp);
    const MatTemplate* mats = S.materials;
    if constexpr (MATS_LDS) {
        constexpr int words = (int)(sizeof(MatTemplate) / 4);
        const int n = 2 * S.nMaterials * words;
        const uint32_t* src = (const uint32_t*)S.materials;
        uint32_t* dst = (uint32_t*)s_mats;
        for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
        mats = s_mats;
    }
    __shared__ int s_push[2];   // shadow, next
    if (threadIdx.x < 2) s_push[threadIdx.x] = 0;
    __syncthreads();
    const int n = level0 ? W.nSamples : seg_scan(W.cur.segCount);
    const int stride = gridDim.x * blockDim.x;
    const int nIter = (n + stride - 1) / stride;
    const int base = wf_block() * W.segCap, sbase = wf_block() * W.shadowSegCap;
    const int nL = W.nLightsML;
    for (int it = 0; it < nIter; ++it) {
        const int i = it * stride + wf_block() * blockDim.x + threadIdx.x;
        const bool active = i < n;
        const int qd = level0 ? i : seg_pos_dense(W.segCap, i, n);
        const int q = active ? qd : 0;
        bool pushNext = false, shading = false, nonSpecular = false;
        int id = 0, depth = 0, dim = 0;
        Ray ray, cont;
        Isect isect;
        BSDF bsdf;
        MatTemplate texLocal;   // a textured material's per-hit lobes (make_bsdf)
        rgb L = sp(0.f);
        SState st;
        st.index = 0; st.dim = 0; st.px = st.py = 0; st.sid = 0;
        if (active) {
            float4 o = W.cur.o[q], d = W.cur.d[q], hr = W.cur.hit[q];
            id = level0 ? q : W.cur.id[q];
            int dd = __float_as_int(d.w);
            dim = dd & 0xffff;
            depth = dd >> 16;
            ray = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
            int slot = __float_as_int(hr.x);
            if (slot < 0) {   // miss: Σ over all lights of Le (F4); no direct light at this level
                for (int k = 0; k < S.nLights; ++k) L = L + light_Le(S, S.lights[k], ray);
                W.recA[(size_t)depth * W.cap + id] = make_float4(L.r, L.g, L.b, 0.f);
                for (int k = 0; k < nL; ++k) W.recV[((size_t)depth * nL + k) * W.cap + id] = 0;
                W.depthOf[id] = depth;
            } else {
                int flags = __float_as_int(S.triVerts[3 * (size_t)slot].w);
                if (flags & PRIM_SPHERE) sphere_si(S.spheres[__float_as_int(S.triVerts[3 * (size_t)slot].x)], ray, ray.tMax, &isect);
                else triangle_si(S, slot, ray, hr.y, hr.z, hr.w, flags, &isect);
                isect.slot = slot;
                isect.medIn = isect.medOut = -1;
                if (!make_bsdf<(LOBES & kTexturedLobes) != 0>(S, mats, isect, false, &bsdf, &texLocal)) {
                    cont = spawn_ray(isect, ray.d);        // Li(isect.SpawnRay(ray.d), depth)
                    pushNext = true;
                } else {
                    shading = true;
                    L = sp(0.f) + si_Le(S, isect, isect.wo);
                    st.index = W.sampleIndex[id];
                    st.sid = id;   // ≡ the sample number mod spp (pixel-major ids)
                    st.dim = dim;
                    nonSpecular = num_components(bsdf, BSDF_ALL & ~BSDF_SPECULAR) > 0;
                }
            }
        }
        for (int k = 0; k < nL; ++k) {   // uniform trip count: one ballot per light
            bool push = false;
            Ray shadow;
            if (shading) {
                float a, b;
                get2d<true>(P.smp, st, &a, &b);
                const size_t ci = ((size_t)depth * nL + k) * W.cap + id;
                W.recV[ci] = 0;
                if (nonSpecular) {   // f ≡ 0 for a purely specular BSDF: nothing would be added
                    f3 wi;
                    float pdf;
                    VisPt vis;
                    rgb Li = sample_li(S, S.lights[k], isect, a, b, &wi, &pdf, &vis);
                    if (!(black(Li) || pdf == 0)) {
                        rgb f = bsdf_f<LOBES>(bsdf, isect.wo, wi, BSDF_ALL);
                        if (!black(f)) {
                            rgb c = f * Li * absdot(wi, isect.sn) / pdf;
                            W.recC[ci] = make_float4(c.r, c.g, c.b, 0.f);
                            shadow = spawn_ray_to(isect, vis.p, vis.pError, vis.n);
                            push = true;
                        }
                    }
                }
            }
            const int si = sbase + wave_push(&s_push[0], push);
            if (push) {
                W.so[si] = make_float4(shadow.o.x, shadow.o.y, shadow.o.z, shadow.tMax);
                W.sd[si] = make_float4(shadow.d.x, shadow.d.y, shadow.d.z, __int_as_float(depth | (k << 8)));
                W.sid[si] = id;
            }
        }
        if (shading) {
            const size_t ri = (size_t)depth * W.cap + id;
            float flagsA = 0.f;
            bool final_ = true;
            // SpecularReflect (Integrator.cpp:179-222); no specular reflection lobe: black, the path
            // ends, no sampler dimensions drawn (as k_wf_shade)
            if (depth + 1 < P.maxDepth && num_components(bsdf, BSDF_REFLECTION | BSDF_SPECULAR) == 0) {
                flagsA = 1.f;   // L += Spectrum(0) from a failed SpecularReflect
            } else if (depth + 1 < P.maxDepth) {
                f3 wi = mk(0, 0, 0);
                float pdf = 0;
                int stype = 0;
                float a, b;
                get2d<true>(P.smp, st, &a, &b);
                rgb f = bsdf_sample<(1 << L_SPEC_R)>(bsdf, isect.wo, &wi, a, b, &pdf, BSDF_REFLECTION | BSDF_SPECULAR, &stype);
                if (!black(f) && pdf > 0.f && absdot(wi, isect.sn) != 0.f && depth + 1 < kWfMaxDepth) {
                    W.recF[ri] = make_float4(f.r, f.g, f.b, absdot(wi, isect.sn));
                    W.recP[ri] = pdf;
                    cont = spawn_ray(isect, wi);
                    pushNext = true;
                    final_ = false;
                    depth += 1;
                } else {
                    flagsA = 1.f;   // L += Spectrum(0) from a failed SpecularReflect
                }
            }
            W.recA[ri] = make_float4(L.r, L.g, L.b, flagsA);
            if (final_) W.depthOf[id] = depth;
            dim = st.dim;
        }
        const int ni = base + wave_push(&s_push[1], pushNext);
        if (pushNext) {
            W.next.o[ni] = make_float4(cont.o.x, cont.o.y, cont.o.z, cont.tMax);
            W.next.d[ni] = make_float4(cont.d.x, cont.d.y, cont.d.z, __int_as_float(pack_dd(dim, depth)));
            W.next.id[ni] = id;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) { W.shadowSeg[wf_block()] = s_push[0]; W.next.segCount[wf_block()] = s_push[1]; }
}

// any-hit for the multi-light shadow queue: the ray's (level, light) record turns visible
template <int SHORT>
__global__ __launch_bounds__(256, PBR_TRAV_OCC) void k_wf_shadow_ml(WfParams W) {
    const int n = seg_scan(W.shadowSeg);
    for (int i0 = wf_block() * blockDim.x + ((int)threadIdx.x & ~63); i0 < n; i0 += gridDim.x * blockDim.x) {   // per wave
        const int i = i0 + (int)__lane_id();
        const int q = seg_pos_dense(W.shadowSegCap, i, n);
        if (i >= n) continue;
        float4 o = W.so[q], d = W.sd[q];
        Ray r = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
        HitRec h;
        Counters c;
        const bool visible = !traverse<true, false, SHORT>(W.P.S, r, &h, &c);
        trav_diag(W.prof, KP_WF_SHADOW, h);
        if (W.prof) prof_count(W.prof + KP_WF_SHADOW * kProfFields + 1, visible);
        if (visible) {
            const int code = __float_as_int(d.w);
            W.recV[((size_t)(code & 0xff) * W.nLightsML + (code >> 8)) * W.cap + W.sid[q]] = 1;
        }
    }
}

// Le plus the direct light of one level: single-light records already hold the sum (k_wf_shadow
// adds it); multi-light ones add each light's contribution whose shadow ray got through, in the
// order of WhittedIntegrator's light loop (WhittedIntegrator.cpp:39-54).
__device__ __forceinline__ rgb level_direct(const WfParams& W, int lv, int id, float4 A) {
    rgb L = sp3(A.x, A.y, A.z);
    for (int k = 0; k < W.nLightsML; ++k) {
        const size_t ci = ((size_t)lv * W.nLightsML + k) * W.cap + id;
        if (W.recV[ci]) {
            const float4 c = W.recC[ci];
            L = L + sp3(c.x, c.y, c.z);
        }
    }
    return L;
}

constexpr int kFinishSamples = 2048;
__host__ __device__ inline int finish_pixels(int spp) {
    int pb = kFinishSamples / spp;
    return pb < 1 ? 1 : (pb > 64 ? 64 : pb);
}
template <int DUMMY>
__global__ __launch_bounds__(256) void k_wf_finish(WfParams W) {
    __shared__ float lds[3 * (kFinishSamples + 64)];
    __shared__ float sum[64 * 3];
    const KParams& P = W.P;
    const int spp = P.spp, pitch = min(spp, kFinishSamples) + 1;
    const int pb = finish_pixels(spp);
    const int lp0 = blockIdx.x * pb;   // dispatch order: the XCD-run order made finish 28% slower
    const int npx = min(pb, W.chunkPix - lp0);
    // spp > kFinishSamples: one pixel per block, folded and summed in slices of kFinishSamples
    const int slice = min(spp, kFinishSamples);
    float acc = 0.f;   // thread t < 3·npx: channel t%3 of pixel t/3
    for (int s0 = 0; s0 < spp; s0 += slice) {
        const int ns = npx * min(slice, spp - s0);
        for (int t = threadIdx.x; t < ns; t += blockDim.x) {
            const int p = spp <= kFinishSamples ? t / spp : 0, k = spp <= kFinishSamples ? t - p * spp : s0 + t;
            const int id = (lp0 + p) * spp + k;
            const int dpt = W.depthOf[id];
            float4 a = W.recA[(size_t)dpt * W.cap + id];
            rgb L = level_direct(W, dpt, id, a);
            if (a.w != 0.f) L = L + sp(0.f);
            for (int lv = dpt - 1; lv >= 0; --lv) {
                size_t ri = (size_t)lv * W.cap + id;
                float4 A = W.recA[ri], F = W.recF[ri];
                float pdf = W.recP[ri];
                L = level_direct(W, lv, id, A) + sp3(F.x, F.y, F.z) * L * F.w / pdf;
            }
            const int kk = k - s0;
            lds[(p * 3 + 0) * pitch + kk] = L.r;
            lds[(p * 3 + 1) * pitch + kk] = L.g;
            lds[(p * 3 + 2) * pitch + kk] = L.b;
        }
        __syncthreads();
        if ((int)threadIdx.x < 3 * npx) {
            const int n = min(slice, spp - s0);
            const float* row = lds + threadIdx.x * pitch;
            for (int k = 0; k < n; ++k) acc = acc + row[k];
        }
        __syncthreads();
    }
    if ((int)threadIdx.x < 3 * npx) sum[threadIdx.x] = acc;
    __syncthreads();
    if ((int)threadIdx.x < npx)
        film_out(P, W.chunkPix0 + lp0 + threadIdx.x, sp3(sum[3 * threadIdx.x], sum[3 * threadIdx.x + 1], sum[3 * threadIdx.x + 2]));
}
