// pbr_device.h — device-side geometry, BVH traversal, BSDFs, lights and media for gfx950.
// Everything here runs per lane on 64-wide waves; data comes from the flattened HBM layout in
// pbr_layout.h.  The float op order of each routine follows the reference function cited next
// to it (see pbr_math.h for the numerics contract).
#pragma once
#include "pbr_layout.h"
#include "pbr_material.h"
#include "pbr_math.h"

namespace pbr {

struct Ray { f3 o, d; float tMax; int medium; };
PBR_HD Ray mkray(f3 o, f3 d, float tMax, int medium) { Ray r; r.o = o; r.d = d; r.tMax = tMax; r.medium = medium; return r; }

struct Counters { uint32_t rays, nodes, prims, shading; };

// Interaction / SurfaceInteraction / MediumInteraction collapsed to the fields the path uses.
struct Isect {
    f3 p, pError, wo, n;       // n == 0 → medium interaction
    f3 sn, dpdu;               // shading normal and shading dpdu (surfaces)
    int slot;                  // BVH-ordered primitive slot (surfaces)
    int medIn, medOut;
    float u, v;                // SurfaceInteraction::uv (Triangle.cpp:170), read by image textures
};
PBR_HD int get_medium(const Isect& it, f3 w) { return dot(w, it.n) > 0 ? it.medOut : it.medIn; }   // Interaction.h:48-50
PBR_HD Ray spawn_ray(const Isect& it, f3 d) {   // Interaction.h:28-31
    f3 o = offset_ray_origin(it.p, it.pError, it.n, d);
    return mkray(o, d, PBR_INF, get_medium(it, d));
}
PBR_HD Ray spawn_ray_to(const Isect& a, f3 bp, f3 bErr, f3 bn) {   // Interaction.h:38-44
    f3 origin = offset_ray_origin(a.p, a.pError, a.n, bp - a.p);
    f3 target = offset_ray_origin(bp, bErr, bn, origin - bp);
    f3 d = target - origin;
    return mkray(origin, d, 1 - kShadowEpsilon, get_medium(a, d));
}

// ---------------------------------------------------------------- BVH node test (Geometry.h:1438-1468)
__device__ __forceinline__ bool node_hit(float4 a, float4 b, const Ray& r, f3 inv, bool n0, bool n1, bool n2) {
    // pMin = (a.x, a.y, a.z), pMax = (a.w, b.x, b.y)
    float tMin = ((n0 ? a.w : a.x) - r.o.x) * inv.x;
    float tMax = ((n0 ? a.x : a.w) - r.o.x) * inv.x;
    float tyMin = ((n1 ? b.x : a.y) - r.o.y) * inv.y;
    float tyMax = ((n1 ? a.y : b.x) - r.o.y) * inv.y;
    if (tMin > tyMax || tyMin > tMax) return false;
    if (tyMin > tMin) tMin = tyMin;
    if (tyMax < tMax) tMax = tyMax;
    float tzMin = ((n2 ? b.y : a.z) - r.o.z) * inv.z;
    float tzMax = ((n2 ? a.z : b.y) - r.o.z) * inv.z;
    if (tMin > tzMax || tzMin > tMax) return false;
    if (tzMin > tMin) tMin = tzMin;
    if (tzMax < tMax) tMax = tzMax;
    return (tMin < r.tMax) && (tMax > 0);
}

// ---------------------------------------------------------------- watertight triangle (Triangle.cpp:62-206)
__device__ __forceinline__ bool tri_test(f3 p0, f3 p1, f3 p2, const Ray& ray, float* tOut, float* b0o, float* b1o, float* b2o) {
    f3 p0t = p0 - ray.o, p1t = p1 - ray.o, p2t = p2 - ray.o;
    int kz = maxdim(vabs(ray.d));
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    f3 d = permute(ray.d, kx, ky, kz);
    p0t = permute(p0t, kx, ky, kz); p1t = permute(p1t, kx, ky, kz); p2t = permute(p2t, kx, ky, kz);
    float Sx = -d.x / d.z, Sy = -d.y / d.z, Sz = 1.f / d.z;
    p0t.x += Sx * p0t.z; p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z; p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z; p2t.y += Sy * p2t.z;
    float e0 = p1t.x * p2t.y - p1t.y * p2t.x;
    float e1 = p2t.x * p0t.y - p2t.y * p0t.x;
    float e2 = p0t.x * p1t.y - p0t.y * p1t.x;
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {
        double a = (double)p2t.x * (double)p1t.y, b = (double)p2t.y * (double)p1t.x;
        e0 = (float)(b - a);
        a = (double)p0t.x * (double)p2t.y; b = (double)p0t.y * (double)p2t.x;
        e1 = (float)(b - a);
        a = (double)p1t.x * (double)p0t.y; b = (double)p1t.y * (double)p0t.x;
        e2 = (float)(b - a);
    }
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0t.z *= Sz; p1t.z *= Sz; p2t.z *= Sz;
    float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    if (det < 0 && (tScaled >= 0 || tScaled < ray.tMax * det)) return false;
    else if (det > 0 && (tScaled <= 0 || tScaled > ray.tMax * det)) return false;
    float invDet = 1 / det;
    float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    float t = tScaled * invDet;
    float maxZt = maxcomp(vabs(mk(p0t.z, p1t.z, p2t.z)));
    float deltaZ = gamma_n(3) * maxZt;
    float maxXt = maxcomp(vabs(mk(p0t.x, p1t.x, p2t.x)));
    float maxYt = maxcomp(vabs(mk(p0t.y, p1t.y, p2t.y)));
    float deltaX = gamma_n(5) * (maxXt + maxZt);
    float deltaY = gamma_n(5) * (maxYt + maxZt);
    float deltaE = 2 * (gamma_n(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    float maxE = maxcomp(vabs(mk(e0, e1, e2)));
    float deltaT = 3 * (gamma_n(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * fabsf(invDet);
    if (t <= deltaT) return false;
    *tOut = t; *b0o = b0; *b1o = b1; *b2o = b2;
    return true;
}

// ---------------------------------------------------------------- sphere (reference stub F2; pbrt-v3 form)
__device__ __forceinline__ bool sphere_test(const SphereRec& s, const Ray& r, float* tOut) {
    f3 o = xf_point(s.w2o, r.o), d = xf_vector(s.w2o, r.d);
    double ox = o.x, oy = o.y, oz = o.z, dx = d.x, dy = d.y, dz = d.z, rad = s.radius;
    double a = dx * dx + dy * dy + dz * dz;
    double b = 2 * (dx * ox + dy * oy + dz * oz);
    double c = ox * ox + oy * oy + oz * oz - rad * rad;
    double disc = b * b - 4 * a * c;
    if (disc < 0) return false;
    double rd = sqrt(disc);
    double q = (b < 0) ? -0.5 * (b - rd) : -0.5 * (b + rd);
    double t0 = q / a, t1 = c / q;
    if (t0 > t1) { double tt = t0; t0 = t1; t1 = tt; }
    float f0 = (float)t0, f1 = (float)t1;
    if (f0 > r.tMax || f1 <= 0) return false;
    float t = f0;
    if (t <= 0) { t = f1; if (t > r.tMax) return false; }
    *tOut = t;
    return true;
}

// PBR_TRAV_DIAG (diagnostic builds only): traversal loop steps per ray, reduced per wave by the queue
// kernels into profile fields 6 (lane steps) and 7 (wave steps x 64): their ratio is the SIMD
// utilisation of the traversal loop.
#ifndef PBR_TRAV_DIAG
#define PBR_TRAV_DIAG 0
#endif
#if PBR_TRAV_DIAG
struct HitRec { int slot; float b0, b1, b2; int steps = 0; };
#else
struct HitRec { int slot; float b0, b1, b2; };
#endif
__device__ __forceinline__ void trav_diag(unsigned long long* prof, int kind, const HitRec& h) {
#if PBR_TRAV_DIAG
    if (!prof) return;
    int sum = h.steps, mxs = h.steps;
    for (int o = 32; o > 0; o >>= 1) { sum += __shfl_xor(sum, o); mxs = max(mxs, __shfl_xor(mxs, o)); }
    const unsigned long long act = __ballot(1);
    if ((int)__lane_id() == __ffsll((long long)act) - 1) {
        atomicAdd(prof + kind * 8 + 6, (unsigned long long)sum);
        atomicAdd(prof + kind * 8 + 7, (unsigned long long)mxs * 64ull);
    }
#endif
}

// Triangle::Intersect's SurfaceInteraction (Triangle.cpp:148-246), no shading normals
// Hit-record and light-sampling helpers are inlined into the kernels: as calls, every live register
// of the shading kernels was saved to scratch around them (C5 1757 -> 1701 ms, bit-identical).
#ifndef PBR_HELPER
#define PBR_HELPER __device__ __forceinline__
#endif
PBR_HELPER void triangle_si(const DeviceScene& S, int slot, const Ray& ray, float b0, float b1, float b2, int flags, Isect* si) {
    const float4* tv = S.triVerts + 3 * (size_t)slot;
    float4 v0 = tv[0], v1 = tv[1], v2 = tv[2];
    f3 p0 = mk(v0.x, v0.y, v0.z), p1 = mk(v1.x, v1.y, v1.z), p2 = mk(v2.x, v2.y, v2.z);
    float u0x = 0, u0y = 0, u1x = 1, u1y = 0, u2x = 1, u2y = 1;
    if (flags & PRIM_HAS_UV) {
        const float2* uv = S.triUV + 3 * (size_t)slot;
        u0x = uv[0].x; u0y = uv[0].y; u1x = uv[1].x; u1y = uv[1].y; u2x = uv[2].x; u2y = uv[2].y;
    }
    float d02x = u0x - u2x, d02y = u0y - u2y, d12x = u1x - u2x, d12y = u1y - u2y;
    f3 dp02 = p0 - p2, dp12 = p1 - p2;
    float determinant = d02x * d12y - d02y * d12x;
    bool degenerate = (double)fabsf(determinant) < 1e-8;
    f3 dpdu = mk(0, 0, 0);
    if (!degenerate) {
        float invdet = 1 / determinant;
        dpdu = (d12y * dp02 - d02y * dp12) * invdet;
    }
    float xs = (fabsf(b0 * p0.x) + fabsf(b1 * p1.x) + fabsf(b2 * p2.x));
    float ys = (fabsf(b0 * p0.y) + fabsf(b1 * p1.y) + fabsf(b2 * p2.y));
    float zs = (fabsf(b0 * p0.z) + fabsf(b1 * p1.z) + fabsf(b2 * p2.z));
    si->pError = gamma_n(7) * mk(xs, ys, zs);
    si->p = b0 * p0 + b1 * p1 + b2 * p2;
    si->wo = normalize(-ray.d);
    f3 n = normalize(cross(dp02, dp12));
    if (flags & PRIM_FLIP) n = -n;
    si->n = n;
    si->sn = n;
    si->dpdu = dpdu;
    si->u = b0 * u0x + b1 * u1x + b2 * u2x;   // uvHit = b0 * uv[0] + b1 * uv[1] + b2 * uv[2]
    si->v = b0 * u0y + b1 * u1y + b2 * u2y;
}
PBR_HELPER void sphere_si(const SphereRec& s, const Ray& r, float t, Isect* si) {
    f3 o = xf_point(s.w2o, r.o), d = xf_vector(s.w2o, r.d);
    f3 pHit = o + d * t;
    pHit = pHit * (s.radius / len(pHit));
    if (pHit.x == 0 && pHit.y == 0) pHit.x = 1e-5f * s.radius;
    const float phiMax = 2 * kPi;
    float zRadius = sqrtf(pHit.x * pHit.x + pHit.y * pHit.y);
    float invZRadius = 1 / zRadius;
    float cosPhi = pHit.x * invZRadius, sinPhi = pHit.y * invZRadius;
    float cosTheta = clampf(pHit.z / s.radius, -1, 1);
    float sinTheta = sqrtf(mx((float)0, 1 - cosTheta * cosTheta));
    f3 dpdu = mk(-phiMax * pHit.y, phiMax * pHit.x, 0);
    f3 dpdv = (-kPi) * mk(pHit.z * cosPhi, pHit.z * sinPhi, -s.radius * sinTheta);
    f3 pw = xf_point(s.o2w, pHit);
    f3 pErrObj = gamma_n(5) * vabs(pHit);
    si->pError = gamma_n(6) * (vabs(pw) + pErrObj);
    si->p = pw;
    si->wo = normalize(-r.d);
    f3 du = xf_vector(s.o2w, dpdu), dv = xf_vector(s.o2w, dpdv);
    f3 n = normalize(cross(du, dv));
    if (s.flip) n = -n;
    si->n = n;
    si->sn = n;
    si->dpdu = du;
    si->u = si->v = 0.f;   // image textures are refused on spheres at upload
}

__device__ __forceinline__ bool prim_hit(const DeviceScene& S, int slot, const Ray& r, float* t, float* b0, float* b1, float* b2) {
    const float4* tv = S.triVerts + 3 * (size_t)slot;
    float4 v0 = tv[0], v1 = tv[1], v2 = tv[2];   // one 48-B record; issue all loads before the branch
    int flags = __float_as_int(v0.w);
    if (flags & PRIM_SPHERE) return sphere_test(S.spheres[__float_as_int(v0.x)], r, t);
    return tri_test(mk(v0.x, v0.y, v0.z), mk(v1.x, v1.y, v1.z), mk(v2.x, v2.y, v2.z), r, t, b0, b1, b2);
}

// BVHAccel::Intersect / IntersectP (BVHAccel.cpp:285-366): the same near-first order (dirIsNeg of
// the node's split axis) so ties between primitives resolve exactly as on the CPU (F8).
// The slab part of node_hit: everything but the final (tMin < ray.tMax), which is the only term
// that depends on ray.tMax.  Returns false where node_hit would whatever ray.tMax is.
// node_slab on the box's near and far planes, already picked by the direction signs (nr = the
// planes the ray enters through: hi on a negative axis, lo on a positive one; fr the others).
// PBR_SLAB_BRANCHLESS: the same comparisons and selects as straight-line code (every lane computes
// all three axes; the early exits become a mask), so a quad node's four tests are one block with no
// exec-mask branches.  tEnter is only read where the test passes, and there it is the same value.
#ifndef PBR_SLAB_BRANCHLESS
#define PBR_SLAB_BRANCHLESS 1
#endif
__device__ __forceinline__ bool slab_nf(f3 nr, f3 fr, const Ray& r, f3 inv, float* tEnter) {
    if constexpr (PBR_SLAB_BRANCHLESS) {
        float tMin = (nr.x - r.o.x) * inv.x;
        float tMax = (fr.x - r.o.x) * inv.x;
        const float tyMin = (nr.y - r.o.y) * inv.y;
        const float tyMax = (fr.y - r.o.y) * inv.y;
        const float tzMin = (nr.z - r.o.z) * inv.z;
        const float tzMax = (fr.z - r.o.z) * inv.z;
        const bool okY = !(tMin > tyMax) & !(tyMin > tMax);
        tMin = tyMin > tMin ? tyMin : tMin;
        tMax = tyMax < tMax ? tyMax : tMax;
        const bool okZ = !(tMin > tzMax) & !(tzMin > tMax);
        tMin = tzMin > tMin ? tzMin : tMin;
        tMax = tzMax < tMax ? tzMax : tMax;
        *tEnter = tMin;
        return okY & okZ & (tMax > 0);
    }
    float tMin = (nr.x - r.o.x) * inv.x;
    float tMax = (fr.x - r.o.x) * inv.x;
    float tyMin = (nr.y - r.o.y) * inv.y;
    float tyMax = (fr.y - r.o.y) * inv.y;
    if (tMin > tyMax || tyMin > tMax) return false;
    if (tyMin > tMin) tMin = tyMin;
    if (tyMax < tMax) tMax = tyMax;
    float tzMin = (nr.z - r.o.z) * inv.z;
    float tzMax = (fr.z - r.o.z) * inv.z;
    if (tMin > tzMax || tzMin > tMax) return false;
    if (tzMin > tMin) tMin = tzMin;
    if (tzMax < tMax) tMax = tzMax;
    *tEnter = tMin;
    return tMax > 0;
}
__device__ __forceinline__ bool node_slab(f3 lo, f3 hi, const Ray& r, f3 inv, bool n0, bool n1, bool n2, float* tEnter) {
    return slab_nf(mk(n0 ? hi.x : lo.x, n1 ? hi.y : lo.y, n2 ? hi.z : lo.z),
                   mk(n0 ? lo.x : hi.x, n1 ? lo.y : hi.y, n2 ? lo.z : hi.z), r, inv, tEnter);
}

// Short traversal stack in LDS for the 256-lane wavefront kernels: entries [0, SHORT) live in LDS
// ([entry][lane], conflict-free), deeper ones in the private (scratch) array.  Only where entries
// are kept changes; the visit order does not.
// LDS entries of the traversal short stack and the minimum 256-lane workgroups per CU the
// traversal kernels are compiled for: 6 entries (12 KB) + the 8-KB segment scan fit 7 workgroups
// per CU in LDS, and 7 × 4 waves per CU leave each lane 72 VGPRs.  Measured on C2: 8/1 25.71 ms,
// 8/6 25.30, 6/7 25.22, 5/8 25.63, 4/8 25.65 (the deeper entries live in scratch).
#ifndef PBR_SHORT_STACK_DEPTH
#define PBR_SHORT_STACK_DEPTH 6
#endif
// Round 5, built without the SLP vectorizer (59-63 VGPRs): 8 — C2 shadow 3.5 → 3.0 ms per frame,
// the frame 14.78 → 14.73 (profiles/r5_trav_occ_ab.log).
#ifndef PBR_TRAV_OCC
#define PBR_TRAV_OCC 8
#endif
constexpr int kShortStack = PBR_SHORT_STACK_DEPTH;
__shared__ int s_trav_ref[kShortStack * 256];
__shared__ float s_trav_t[kShortStack * 256];
// A deeper LDS short stack for the kernels with LDS to spare: the closest-hit lane-refill kernels
// (5 workgroups per CU) and the camera kernels (no segment scan).  C3 / C5 frame ms with the refill
// kernels at 6 entries 276.6 / 1416, 10: 271.6 / 1386, 14 (4 workgroups per CU fit): 285.5 / 1403.
// Round 5 (no SLP: 77 VGPRs, so 6 workgroups per CU fit in registers): 8 entries let 6 fit in LDS
// too — C4-material extend 118.5 → 112.8 ms, C5 quarter 39.6 → 37.7 (profiles/r5_refill_short_ab.log).
#ifndef PBR_REFILL_SHORT
#define PBR_REFILL_SHORT 8
#endif
constexpr int kRefillShort = PBR_REFILL_SHORT;
__shared__ int s_trav_ref_r[kRefillShort * 256];
__shared__ float s_trav_t_r[kRefillShort * 256];
// The Path shadow kernel's any-hit walk keeps no entry distances, so a deeper LDS stack costs it 4 B
// per entry and lane: it walks with kRefillShort entries (a stack diagnostic found 12% of C4-material
// shadow rays deeper than 6 entries, 0.6% deeper than 10).  C4-material shadow 82.2 → 78.7 ms, frame
// 339.4 → 336.3 (profiles/r5_any_short_ab.log).  VolPath's transmittance kernel keeps 6: its other
// walk stores distances, and both stacks in LDS would cost it a workgroup per CU.
#ifndef PBR_ANY_SHORT
#define PBR_ANY_SHORT 1
#endif
constexpr int kAnyShort = PBR_ANY_SHORT ? kRefillShort : kShortStack;
// the LDS short stack of depth SHORT ([entry][lane]) for this thread
template <int SHORT>
__device__ __forceinline__ void trav_lds(int** ref, float** t) {
    static_assert(SHORT == kShortStack || SHORT == kRefillShort, "short stack depth");
    if constexpr (SHORT == kShortStack) { *ref = s_trav_ref + threadIdx.x; *t = s_trav_t + threadIdx.x; }
    else { *ref = s_trav_ref_r + threadIdx.x; *t = s_trav_t_r + threadIdx.x; }
}

// The binary traversal below over the quad layout of build_quad_nodes: one node fetch covers two
// binary levels, halving the chain of dependent node loads per ray.  Visit order stays BVHAccel's:
// at binary node N with near child A (dirIsNeg[axN] order) the reference visits A's near and far
// children, then B's, each gated by its box test against the tMax current at that point.  The four
// slots are ordered the same way from the direction signs of (axN, axA, axB); the first one whose
// slab passes with tEnter < tMax is visited now (the reference visits it after A's test, which
// the nested boxes make pass — a slot box lies inside its parent's, and the slab test is monotone
// in the box) and the passing slots after it are pushed far-last, each re-tested against tMax
// when popped — the moment the reference would test it.  Slots that fail now would fail later
// (tMax only shrinks), so primitive tests run in exactly the reference's order (F8 ties).
// Wave-uniform reads through the scalar cache: a pointer into the constant address space built
// from a readfirstlane'd index is loaded with s_load (the BVH and the mesh are read-only for the
// whole render), so a node every active lane visits costs one scalar fetch instead of 64 lanes of
// vector-L1 traffic.  Switch: PBR_SCALAR_LOADS (results are identical either way).
#ifndef PBR_SCALAR_LOADS
#define PBR_SCALAR_LOADS 1
#endif
constexpr bool kScalarLoads = PBR_SCALAR_LOADS != 0;
typedef float ScalarF4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) ScalarF4* ScalarF4Ptr;
__device__ __forceinline__ ScalarF4Ptr scalar_f4(const float4* p) { return (ScalarF4Ptr)(size_t)p; }
__device__ __forceinline__ float4 as_f4(ScalarF4 v) { return make_float4(v.x, v.y, v.z, v.w); }

#ifndef PBR_QUAD_TRAVERSAL
#define PBR_QUAD_TRAVERSAL 1
#endif
constexpr bool kQuadTraversal = PBR_QUAD_TRAVERSAL != 0;
struct QuadSlots {   // one quad node's four slots in visit order
    float t[4];
    int ref[4];
    bool k[4];       // slab passes (box valid)
};
// A quad node's four slots from its fetched 128 B (LX..HZ: SoA boxes, R: child refs, meta: axes,
// valid mask).
template <bool ANY>
__device__ __forceinline__ void quad_slots_nf(float4 NX, float4 NY, float4 NZ, float4 FX, float4 FY, float4 FZ, float4 R,
                                              int meta, const Ray& r, f3 inv, bool n0, bool n1, bool n2, QuadSlots* q);
// PBR_NF_ROWS: the near and far planes of a quad node are fetched as rows picked by the direction
// signs (a lane walking alone: per-lane row addresses; a packet: the wave's common signs, scalar
// addresses) instead of fetching lo and hi and picking each value with a select — the same floats
// reach the same operations, so the results are the same bits, with 24 VALU selects fewer per node
// (4 slots × 3 axes × near/far).  Per-lane row addresses take more VGPRs: the lane-refill walks
// (NF = true) have the room; the plain per-lane walk (traverse_quad: Whitted's shadow rays at 8
// waves per SIMD, 60 VGPRs) spilled with them (6 VGPRs) and keeps the selects.
#ifndef PBR_NF_ROWS
#define PBR_NF_ROWS 1
#endif
template <bool ANY>
__device__ __forceinline__ void quad_slots_lohi(float4 LX, float4 LY, float4 LZ, float4 HX, float4 HY, float4 HZ, float4 R,
                                                int meta, const Ray& r, f3 inv, bool n0, bool n1, bool n2, QuadSlots* q);
template <bool ANY, bool NF = false>
__device__ __forceinline__ void quad_slots(const DeviceScene& S, int cur, const Ray& r, f3 inv, bool n0, bool n1, bool n2,
                                           QuadSlots* q) {
    if constexpr (!NF || !PBR_NF_ROWS) {   // lo and hi fetched, each plane picked per slot (node_slab)
        float4 LX, LY, LZ, HX, HY, HZ, R;
        int meta;
        const int ucur = __builtin_amdgcn_readfirstlane(cur);
        if (kScalarLoads && __builtin_amdgcn_ballot_w64(cur != ucur) == 0ull) {
            const ScalarF4Ptr w = scalar_f4(S.quad + 8 * (size_t)ucur);
            LX = as_f4(w[0]); LY = as_f4(w[1]); LZ = as_f4(w[2]); HX = as_f4(w[3]); HY = as_f4(w[4]);
            HZ = as_f4(w[5]); R = as_f4(w[6]);
            meta = __float_as_int(w[7].x);
        } else {
            const float4* w = S.quad + 8 * (size_t)cur;
            LX = w[0]; LY = w[1]; LZ = w[2]; HX = w[3]; HY = w[4]; HZ = w[5]; R = w[6];
            meta = __float_as_int(w[7].x);
        }
        quad_slots_lohi<ANY>(LX, LY, LZ, HX, HY, HZ, R, meta, r, inv, n0, n1, n2, q);
        return;
    }
    float4 NX, NY, NZ, FX, FY, FZ, R;
    int meta;
    // Coherent waves (a pixel's samples share a wave) often have every active lane at the
    // same node: then it is fetched once through the scalar cache.
    const int ucur = __builtin_amdgcn_readfirstlane(cur);
    if (kScalarLoads && __builtin_amdgcn_ballot_w64(cur != ucur) == 0ull) {
        const ScalarF4Ptr w = scalar_f4(S.quad + 8 * (size_t)ucur);
        const float4 LX = as_f4(w[0]), LY = as_f4(w[1]), LZ = as_f4(w[2]), HX = as_f4(w[3]), HY = as_f4(w[4]),
                     HZ = as_f4(w[5]);
        NX = n0 ? HX : LX; FX = n0 ? LX : HX;
        NY = n1 ? HY : LY; FY = n1 ? LY : HY;
        NZ = n2 ? HZ : LZ; FZ = n2 ? LZ : HZ;
        R = as_f4(w[6]);
        meta = __float_as_int(w[7].x);
    } else {
        const float4* w = S.quad + 8 * (size_t)cur;
        // rows 0-2: lo.x/y/z, 3-5: hi.x/y/z of the four slots
        NX = w[n0 ? 3 : 0]; FX = w[n0 ? 0 : 3];
        NY = w[n1 ? 4 : 1]; FY = w[n1 ? 1 : 4];
        NZ = w[n2 ? 5 : 2]; FZ = w[n2 ? 2 : 5];
        R = w[6];
        meta = __float_as_int(w[7].x);
    }
    quad_slots_nf<ANY>(NX, NY, NZ, FX, FY, FZ, R, meta, r, inv, n0, n1, n2, q);
}
template <bool ANY>
__device__ __forceinline__ void quad_order(bool k0, bool k1, bool k2, bool k3, float t0, float t1, float t2, float t3,
                                           float4 R, int meta, bool n0, bool n1, bool n2, QuadSlots* q);
template <bool ANY>
__device__ __forceinline__ void quad_slots_lohi(float4 LX, float4 LY, float4 LZ, float4 HX, float4 HY, float4 HZ, float4 R,
                                                int meta, const Ray& r, f3 inv, bool n0, bool n1, bool n2, QuadSlots* q) {
    float t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    bool k0 = node_slab(mk(LX.x, LY.x, LZ.x), mk(HX.x, HY.x, HZ.x), r, inv, n0, n1, n2, &t0) & ((meta >> 8) & 1);
    bool k1 = node_slab(mk(LX.y, LY.y, LZ.y), mk(HX.y, HY.y, HZ.y), r, inv, n0, n1, n2, &t1) & ((meta >> 9) & 1);
    bool k2 = node_slab(mk(LX.z, LY.z, LZ.z), mk(HX.z, HY.z, HZ.z), r, inv, n0, n1, n2, &t2) & ((meta >> 10) & 1);
    bool k3 = node_slab(mk(LX.w, LY.w, LZ.w), mk(HX.w, HY.w, HZ.w), r, inv, n0, n1, n2, &t3) & ((meta >> 11) & 1);
    quad_order<ANY>(k0, k1, k2, k3, t0, t1, t2, t3, R, meta, n0, n1, n2, q);
}
template <bool ANY>
__device__ __forceinline__ void quad_slots_nf(float4 NX, float4 NY, float4 NZ, float4 FX, float4 FY, float4 FZ, float4 R,
                                              int meta, const Ray& r, f3 inv, bool n0, bool n1, bool n2, QuadSlots* q) {
    // (The two-slot pairs written as packed fp32 — v_pk_add/v_pk_mul — measured slower: 8-9 more
    // VGPRs, C4-material extend 119.5 → 129.0 ms; profiles/r5_slp_ab.log.)
    float t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    bool k0 = slab_nf(mk(NX.x, NY.x, NZ.x), mk(FX.x, FY.x, FZ.x), r, inv, &t0) & ((meta >> 8) & 1);
    bool k1 = slab_nf(mk(NX.y, NY.y, NZ.y), mk(FX.y, FY.y, FZ.y), r, inv, &t1) & ((meta >> 9) & 1);
    bool k2 = slab_nf(mk(NX.z, NY.z, NZ.z), mk(FX.z, FY.z, FZ.z), r, inv, &t2) & ((meta >> 10) & 1);
    bool k3 = slab_nf(mk(NX.w, NY.w, NZ.w), mk(FX.w, FY.w, FZ.w), r, inv, &t3) & ((meta >> 11) & 1);
    quad_order<ANY>(k0, k1, k2, k3, t0, t1, t2, t3, R, meta, n0, n1, n2, q);
}
// the four slots in visit order (closest hit) or build order (any hit)
template <bool ANY>
__device__ __forceinline__ void quad_order(bool k0, bool k1, bool k2, bool k3, float t0, float t1, float t2, float t3,
                                           float4 R, int meta, bool n0, bool n1, bool n2, QuadSlots* q) {
    int r0 = __float_as_int(R.x), r1 = __float_as_int(R.y), r2 = __float_as_int(R.z), r3 = __float_as_int(R.w);
    auto swp = [](bool c, auto& a, auto& b) { auto x = c ? b : a; b = c ? a : b; a = x; };
    auto neg = [&](int axis) { return axis == 0 ? n0 : (axis == 1 ? n1 : n2); };
    // Any-hit (IntersectP) keeps the slots in build order instead.  Its answer does not
    // depend on the visit order: ray.tMax never shrinks, so every box test and the set of
    // reachable leaves are order-free, and the result is whether any primitive there is
    // hit.  Build order reaches occluders of C2's shadow rays sooner (C2 19.95 → 18.55 ms).
    if constexpr (!ANY) {
        const bool sA = neg((meta >> 2) & 3), sB = neg((meta >> 4) & 3), sN = neg(meta & 3);
        swp(sA, k0, k1); swp(sA, t0, t1); swp(sA, r0, r1);
        swp(sB, k2, k3); swp(sB, t2, t3); swp(sB, r2, r3);
        swp(sN, k0, k2); swp(sN, t0, t2); swp(sN, r0, r2);
        swp(sN, k1, k3); swp(sN, t1, t3); swp(sN, r1, r3);
    }
    q->t[0] = t0; q->t[1] = t1; q->t[2] = t2; q->t[3] = t3;
    q->ref[0] = r0; q->ref[1] = r1; q->ref[2] = r2; q->ref[3] = r3;
    q->k[0] = k0; q->k[1] = k1; q->k[2] = k2; q->k[3] = k3;
}

template <bool ANY, int SHORT>
__device__ bool traverse_quad(const DeviceScene& S, Ray& r, HitRec* h, f3 inv, bool n0, bool n1, bool n2) {
    constexpr int PRIV = kTraversalStack - SHORT;
    int stackRef[PRIV];
    float stackT[PRIV];
    int* lref = nullptr;
    float* lt = nullptr;
    if constexpr (SHORT > 0) trav_lds<SHORT>(&lref, &lt);
    int sp = 0;
    // any-hit: ray.tMax never shrinks, so a pushed slot (tEnter < tMax) always passes its re-test
    // on the way out and only the reference is kept
    auto push = [&](int ref, float t) {
        if (SHORT && sp < SHORT) { lref[sp * 256] = ref; if (!ANY) lt[sp * 256] = t; }
        else { stackRef[sp - SHORT] = ref; if (!ANY) stackT[sp - SHORT] = t; }
        ++sp;
    };
    int cur = S.quadRootRef;
    bool found = false;
    while (true) {
#if PBR_TRAV_DIAG
        h->steps++;
#endif
        if (cur < 0) {   // leaf: its slots run up to the one flagged PRIM_LEAF_END
            int slot = cur & 0x7fffffff;
            while (true) {
                float4 v0, v1, v2;
                const int uslot = __builtin_amdgcn_readfirstlane(slot);
                if (kScalarLoads && __builtin_amdgcn_ballot_w64(slot != uslot) == 0ull) {   // one primitive for the wave
                    const ScalarF4Ptr tv = scalar_f4(S.triVerts + 3 * (size_t)uslot);
                    v0 = as_f4(tv[0]); v1 = as_f4(tv[1]); v2 = as_f4(tv[2]);
                } else {
                    const float4* tv = S.triVerts + 3 * (size_t)slot;
                    v0 = tv[0]; v1 = tv[1]; v2 = tv[2];
                }
                int flags = __float_as_int(v0.w);
                float t, b0 = 0, b1 = 0, b2 = 0;
                bool hit = (flags & PRIM_SPHERE)
                               ? sphere_test(S.spheres[__float_as_int(v0.x)], r, &t)
                               : tri_test(mk(v0.x, v0.y, v0.z), mk(v1.x, v1.y, v1.z), mk(v2.x, v2.y, v2.z), r, &t, &b0, &b1, &b2);
                if (hit) {
                    if (ANY) return true;
                    r.tMax = t;   // GeometricPrimitive::Intersect (Primitive.cpp:26)
                    h->slot = slot; h->b0 = b0; h->b1 = b1; h->b2 = b2;
                    found = true;
                }
                if (flags & PRIM_LEAF_END) break;
                ++slot;
            }
        } else {
            QuadSlots q;
            quad_slots<ANY>(S, cur, r, inv, n0, n1, n2, &q);
            const float tM = r.tMax;
            const bool p0 = q.k[0] && q.t[0] < tM, p1 = q.k[1] && q.t[1] < tM, p2 = q.k[2] && q.t[2] < tM,
                       p3 = q.k[3] && q.t[3] < tM;
            if (p0 | p1 | p2 | p3) {
                // unreachable: the upload refuses trees whose quad walk can need more (kQuadStackLimit)
                if (sp > kQuadStackLimit) { atomicOr(S.guard, kGuardStack); break; }
                const int first = p0 ? 0 : (p1 ? 1 : (p2 ? 2 : 3));
                if (p3 && first < 3) push(q.ref[3], q.t[3]);
                if (p2 && first < 2) push(q.ref[2], q.t[2]);
                if (p1 && first < 1) push(q.ref[1], q.t[1]);
                cur = first == 0 ? q.ref[0] : (first == 1 ? q.ref[1] : (first == 2 ? q.ref[2] : q.ref[3]));
                continue;
            }
        }
        bool more = false;   // pop until an entry passes its box test against the current tMax
        while (sp > 0) {
            --sp;
            int rr;
            float tt;
            if (ANY) { cur = (SHORT && sp < SHORT) ? lref[sp * 256] : stackRef[sp - SHORT]; more = true; break; }
            if (SHORT && sp < SHORT) { rr = lref[sp * 256]; tt = lt[sp * 256]; }
            else { rr = stackRef[sp - SHORT]; tt = stackT[sp - SHORT]; }
            if (tt < r.tMax) { cur = rr; more = true; break; }
        }
        if (!more) break;
    }
    return found;
}

// Wave-packet traversal of the quad layout for coherent waves (a camera wave holds one pixel's
// sub-pixel rays; a flat mirror keeps them together).  The wave walks ONE node at a time with a
// wave-uniform stack in LDS; each lane tests the node's four slots against its own ray, and the
// wave enters the first slot (in visit order) that any lane passes, pushing the later ones that
// some lane passes.  Per lane this is traverse_quad exactly:
//   * the visit order of a quad node's slots depends only on the ray's direction signs on the
//     node's split axes; the caller takes this path only when every live lane has the same three
//     signs (closest hit — any hit keeps build order, which depends on nothing), so the order is
//     wave-uniform;
//   * a lane is `active` at the wave's current node iff its own traversal would enter it: it passed
//     that slot's test (entered now, or on a pop) — inactive lanes test nothing there;
//   * a stack entry is (parent node, slot column) plus the ballot of the lanes that pushed it; on a
//     pop each of those lanes re-derives the slot's slab (the same float operations on the same
//     box, so the same tEnter) and tests it against its current tMax — what traverse_quad's pop
//     test computes from the stored tEnter.
// So every lane runs its own primitive tests in BVHAccel's order with its own tMax (F8 ties
// unchanged), while node and triangle fetches are scalar (one per wave), the stack costs no
// per-lane memory and control flow is wave-uniform.  The stack is 64 entries per wave, like the
// per-lane one.
constexpr int kPacketStack = kTraversalStack;
__shared__ int s_pk_ref[4][kPacketStack];                  // parent quad node << 2 | slot column
__shared__ unsigned long long s_pk_mask[4][kPacketStack];  // lanes that pushed the entry
#ifndef PBR_PACKET
#define PBR_PACKET 1
#endif
constexpr bool kPacket = PBR_PACKET != 0;
#ifndef PBR_PACKET_EXTEND
#define PBR_PACKET_EXTEND 1
#endif
template <bool ANY>
__device__ bool traverse_packet(const DeviceScene& S, Ray& r, HitRec* h, f3 inv, bool n0, bool n1, bool n2, bool alive,
                                int u0, int u1, int u2) {
    const int wv = (int)(threadIdx.x >> 6);
    int* sref = s_pk_ref[wv];
    unsigned long long* smask = s_pk_mask[wv];
    const unsigned long long lanebit = 1ull << __lane_id();
    int sp = 0;
    bool found = false;
    int cur = S.quadRootRef;
    bool active = alive;
    // closest hit: the live lanes' common signs, wave-uniform, so the near/far plane selects of the
    // slab tests are scalar (any hit: each lane's own signs)
    if constexpr (!ANY) { n0 = u0 != 0; n1 = u1 != 0; n2 = u2 != 0; }
    while (true) {
        if (cur < 0) {   // leaf: the active lanes test its primitives in slot order
            if (active) {
                int slot = cur & 0x7fffffff;
                while (true) {
                    const ScalarF4Ptr tv = scalar_f4(S.triVerts + 3 * (size_t)slot);
                    const float4 v0 = as_f4(tv[0]), v1 = as_f4(tv[1]), v2 = as_f4(tv[2]);
                    const int flags = __float_as_int(v0.w);
                    float t, b0 = 0, b1 = 0, b2 = 0;
                    const bool hit = (flags & PRIM_SPHERE)
                                         ? sphere_test(S.spheres[__float_as_int(v0.x)], r, &t)
                                         : tri_test(mk(v0.x, v0.y, v0.z), mk(v1.x, v1.y, v1.z), mk(v2.x, v2.y, v2.z), r, &t, &b0, &b1, &b2);
                    if (hit) {
                        found = true;
                        if (ANY) { alive = false; active = false; break; }
                        r.tMax = t;   // GeometricPrimitive::Intersect (Primitive.cpp:26)
                        h->slot = slot; h->b0 = b0; h->b1 = b1; h->b2 = b2;
                    }
                    if (flags & PRIM_LEAF_END) break;
                    ++slot;
                }
            }
            if (ANY && __builtin_amdgcn_ballot_w64(alive) == 0ull) break;
        } else {
            const ScalarF4Ptr w = scalar_f4(S.quad + 8 * (size_t)cur);
            // near / far plane rows (PBR_NF_ROWS): closest hit picks them by the wave's common signs
            // with scalar addresses — no selects; any hit keeps each lane's own signs
            float4 NX, NY, NZ, FX, FY, FZ;
            if constexpr (!ANY && PBR_NF_ROWS) {
                NX = as_f4(w[u0 ? 3 : 0]); FX = as_f4(w[u0 ? 0 : 3]);
                NY = as_f4(w[u1 ? 4 : 1]); FY = as_f4(w[u1 ? 1 : 4]);
                NZ = as_f4(w[u2 ? 5 : 2]); FZ = as_f4(w[u2 ? 2 : 5]);
            } else {
                const float4 LX = as_f4(w[0]), LY = as_f4(w[1]), LZ = as_f4(w[2]), HX = as_f4(w[3]), HY = as_f4(w[4]),
                             HZ = as_f4(w[5]);
                NX = n0 ? HX : LX; FX = n0 ? LX : HX;
                NY = n1 ? HY : LY; FY = n1 ? LY : HY;
                NZ = n2 ? HZ : LZ; FZ = n2 ? LZ : HZ;
            }
            const float4 R = as_f4(w[6]);
            const int meta = __float_as_int(w[7].x);
            float t[4] = {0.f, 0.f, 0.f, 0.f};
            bool p[4];
            if constexpr (PBR_SLAB_BRANCHLESS) {   // (the lane and valid masks applied after the tests)
                p[0] = slab_nf(mk(NX.x, NY.x, NZ.x), mk(FX.x, FY.x, FZ.x), r, inv, &t[0]) & (t[0] < r.tMax);
                p[1] = slab_nf(mk(NX.y, NY.y, NZ.y), mk(FX.y, FY.y, FZ.y), r, inv, &t[1]) & (t[1] < r.tMax);
                p[2] = slab_nf(mk(NX.z, NY.z, NZ.z), mk(FX.z, FY.z, FZ.z), r, inv, &t[2]) & (t[2] < r.tMax);
                p[3] = slab_nf(mk(NX.w, NY.w, NZ.w), mk(FX.w, FY.w, FZ.w), r, inv, &t[3]) & (t[3] < r.tMax);
                p[0] = p[0] & active & (((meta >> 8) & 1) != 0);
                p[1] = p[1] & active & (((meta >> 9) & 1) != 0);
                p[2] = p[2] & active & (((meta >> 10) & 1) != 0);
                p[3] = p[3] & active & (((meta >> 11) & 1) != 0);
            } else {
            p[0] = active && slab_nf(mk(NX.x, NY.x, NZ.x), mk(FX.x, FY.x, FZ.x), r, inv, &t[0]) && ((meta >> 8) & 1) && t[0] < r.tMax;
            p[1] = active && slab_nf(mk(NX.y, NY.y, NZ.y), mk(FX.y, FY.y, FZ.y), r, inv, &t[1]) && ((meta >> 9) & 1) && t[1] < r.tMax;
            p[2] = active && slab_nf(mk(NX.z, NY.z, NZ.z), mk(FX.z, FY.z, FZ.z), r, inv, &t[2]) && ((meta >> 10) & 1) && t[2] < r.tMax;
            p[3] = active && slab_nf(mk(NX.w, NY.w, NZ.w), mk(FX.w, FY.w, FZ.w), r, inv, &t[3]) && ((meta >> 11) & 1) && t[3] < r.tMax;
            }
            const unsigned long long bm[4] = {__builtin_amdgcn_ballot_w64(p[0]), __builtin_amdgcn_ballot_w64(p[1]),
                                              __builtin_amdgcn_ballot_w64(p[2]), __builtin_amdgcn_ballot_w64(p[3])};
            // visit position → slot column (quad_slots' swaps; any hit: build order)
            int col[4] = {0, 1, 2, 3};
            if constexpr (!ANY) {
                // the live lanes' common direction signs (u0, u1, u2) on the three split axes
                const int aN = meta & 3, aA = (meta >> 2) & 3, aB = (meta >> 4) & 3;
                const int sN = aN == 0 ? u0 : (aN == 1 ? u1 : u2);
                const int sA = aA == 0 ? u0 : (aA == 1 ? u1 : u2);
                const int sB = aB == 0 ? u0 : (aB == 1 ? u1 : u2);
                for (int pos = 0; pos < 4; ++pos) {
                    const int hi = (pos >> 1) ^ sN;
                    col[pos] = hi * 2 + ((pos & 1) ^ (hi == 0 ? sA : sB));
                }
            }
            int first = -1;
            for (int pos = 0; pos < 4; ++pos)
                if (first < 0 && bm[col[pos]] != 0ull) first = pos;
            // unreachable: the upload refuses trees whose quad walk can need more (kQuadStackLimit)
            if (first >= 0 && sp > kQuadStackLimit) {
                atomicOr(S.guard, kGuardStack);
                break;
            }
            if (first >= 0) {
                for (int pos = 3; pos > first; --pos)
                    if (bm[col[pos]] != 0ull) {
                        sref[sp] = (cur << 2) | col[pos];   // every lane stores the same values
                        smask[sp] = bm[col[pos]];
                        ++sp;
                    }
                const int c = col[first];
                active = c == 0 ? p[0] : (c == 1 ? p[1] : (c == 2 ? p[2] : p[3]));
                cur = __float_as_int(c == 0 ? R.x : (c == 1 ? R.y : (c == 2 ? R.z : R.w)));
                cur = __builtin_amdgcn_readfirstlane(cur);
                continue;
            }
        }
        // pop until some lane that pushed an entry passes its re-derived test against its tMax
        bool more = false;
        while (sp > 0) {
            --sp;
            const int e = __builtin_amdgcn_readfirstlane(sref[sp]);
            const unsigned long long m = smask[sp];   // a uniform LDS address: the same value in every lane
            const int parent = e >> 2, c = e & 3;
            const ScalarF4Ptr w = scalar_f4(S.quad + 8 * (size_t)parent);
            // the slot's one box: its six floats are scalars, column c of each row (PBR_NF_ROWS:
            // the rows picked by the wave's common signs, scalar addresses, as above)
            const float* wf = (const float*)(S.quad + 8 * (size_t)parent);
            f3 nr, fr;
            if constexpr (!ANY && PBR_NF_ROWS) {
                const __attribute__((address_space(4))) float* sf = (const __attribute__((address_space(4))) float*)(size_t)wf;
                nr = mk(sf[(u0 ? 12 : 0) + c], sf[(u1 ? 16 : 4) + c], sf[(u2 ? 20 : 8) + c]);
                fr = mk(sf[(u0 ? 0 : 12) + c], sf[(u1 ? 4 : 16) + c], sf[(u2 ? 8 : 20) + c]);
            } else {
                auto pick = [c](float4 v) { return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)); };
                const f3 lo = mk(pick(as_f4(w[0])), pick(as_f4(w[1])), pick(as_f4(w[2])));
                const f3 hi = mk(pick(as_f4(w[3])), pick(as_f4(w[4])), pick(as_f4(w[5])));
                nr = mk(n0 ? hi.x : lo.x, n1 ? hi.y : lo.y, n2 ? hi.z : lo.z);
                fr = mk(n0 ? lo.x : hi.x, n1 ? lo.y : hi.y, n2 ? lo.z : hi.z);
            }
            const __attribute__((address_space(4))) float* rf = (const __attribute__((address_space(4))) float*)(size_t)(wf + 24);
            float tt = 0.f;
            bool a = (m & lanebit) != 0ull && (!ANY || alive);
            if constexpr (PBR_SLAB_BRANCHLESS) a = a & slab_nf(nr, fr, r, inv, &tt) & (tt < r.tMax);
            else a = a && slab_nf(nr, fr, r, inv, &tt) && tt < r.tMax;
            if (__builtin_amdgcn_ballot_w64(a) != 0ull) {
                active = a;
                cur = __builtin_amdgcn_readfirstlane(__float_as_int(rf[c]));
                more = true;
                break;
            }
        }
        if (!more) break;
    }
    return found;
}

// traverse() for a whole wave as packet walks.  Closest hit: one walk per direction-sign class
// (octant) present among the live lanes — a camera wave inside one pixel nearly always holds one;
// each lane takes part in its own class's walk only, so its result is its own traversal's.  Any
// hit: one walk (build order).  Every lane of the wave that is still running must call it (`live`
// = the lane has a ray).  No per-lane stack: the kernels that use it need no scratch for one.
template <bool ANY>
__device__ bool traverse_wave(const DeviceScene& S, Ray& r, HitRec* h, bool live) {
    f3 inv = ANY ? mk(1.f / r.d.x, 1.f / r.d.y, 1.f / r.d.z) : mk(1 / r.d.x, 1 / r.d.y, 1 / r.d.z);
    bool n0 = inv.x < 0, n1 = inv.y < 0, n2 = inv.z < 0;
    const bool ok = live && S.nNodes > 0 && node_hit(S.nodes[0], S.nodes[1], r, inv, n0, n1, n2);   // the root first
    unsigned long long left = __builtin_amdgcn_ballot_w64(ok);
    if constexpr (ANY) return left ? traverse_packet<true>(S, r, h, inv, n0, n1, n2, ok, 0, 0, 0) : false;
    const int cls = (int)n0 | ((int)n1 << 1) | ((int)n2 << 2);
    bool found = false;
    while (left) {
        const int c = __builtin_amdgcn_readlane(cls, __ffsll((long long)left) - 1);
        const bool mine = ok && cls == c;
        left &= ~__builtin_amdgcn_ballot_w64(mine);
        const bool f = traverse_packet<false>(S, r, h, inv, n0, n1, n2, mine, c & 1, (c >> 1) & 1, (c >> 2) & 1);
        if (mine) found = f;
    }
    return found;
}

// BVHAccel::Intersect / IntersectP (BVHAccel.cpp:285-366) over the wide layout of
// build_wide_nodes.  The reference pops a node and tests its box against the current ray.tMax;
// since only the last comparison of that test reads ray.tMax (Geometry.h:1438-1468), the slab part
// is evaluated once, from the parent, for both children, and the stack keeps (child, tEnter):
//   * near child (dirIsNeg[axis] order) visited next iff slab && tEnter < tMax — what the
//     reference's immediate visit of it computes, tMax being unchanged in between;
//   * far child: the reference pushes it before descending; here it is pushed only if its slab
//     passes (a failing one is a no-op pop there), and tested against the then-current tMax when
//     popped; if the near child failed, the reference's next pop is this far child, tested now.
// Primitive tests therefore run in exactly the reference's order, so ties resolve the same (F8).
// STATS counts node tests as the reference performs them (root, every visited child, every pop):
// there a far child whose slab fails is still pushed (with a NaN key, so its pop test fails).
template <bool ANY, bool STATS, int SHORT = 0>
__device__ bool traverse(const DeviceScene& S, Ray& r, HitRec* h, Counters* c) {
    static_assert(SHORT == 0 || SHORT == kShortStack || SHORT == kRefillShort, "short stack depth");
    if (STATS) c->rays++;
    if (S.nNodes == 0) return false;
    f3 inv = ANY ? mk(1.f / r.d.x, 1.f / r.d.y, 1.f / r.d.z) : mk(1 / r.d.x, 1 / r.d.y, 1 / r.d.z);
    bool n0 = inv.x < 0, n1 = inv.y < 0, n2 = inv.z < 0;
    {   // the root is visited first
        float4 a = S.nodes[0], b = S.nodes[1];
        if (STATS) c->nodes++;
        if (!node_hit(a, b, r, inv, n0, n1, n2)) return false;
    }
    // The quad walk, except in a tree whose quad walk could need more stack than it has
    // (S.binaryWalk, see pbr_hip_upload_scene): those run the megakernel (SHORT == 0) over the
    // binary layout, whose one-entry-per-level stack holds BVHAccel's 64 levels.  Same primitive
    // tests in the same order either way.
    if constexpr (!STATS && kQuadTraversal) {
        if (SHORT > 0 || !S.binaryWalk) return traverse_quad<ANY, SHORT>(S, r, h, inv, n0, n1, n2);
    }
    int stackRef[kTraversalStack - SHORT];
    float stackT[kTraversalStack - SHORT];
    int* lref = nullptr;
    float* lt = nullptr;
    if constexpr (SHORT > 0) trav_lds<SHORT>(&lref, &lt);
    int cur = S.rootRef, sp = 0;
    bool found = false;
    while (true) {
#if PBR_TRAV_DIAG
        h->steps++;
#endif
        if (cur < 0) {   // leaf: its slots run up to the one flagged PRIM_LEAF_END
            int slot = cur & 0x7fffffff;
            while (true) {
                const float4* tv = S.triVerts + 3 * (size_t)slot;
                float4 v0 = tv[0], v1 = tv[1], v2 = tv[2];
                int flags = __float_as_int(v0.w);
                float t, b0 = 0, b1 = 0, b2 = 0;
                if (STATS) c->prims++;
                bool hit = (flags & PRIM_SPHERE)
                               ? sphere_test(S.spheres[__float_as_int(v0.x)], r, &t)
                               : tri_test(mk(v0.x, v0.y, v0.z), mk(v1.x, v1.y, v1.z), mk(v2.x, v2.y, v2.z), r, &t, &b0, &b1, &b2);
                if (hit) {
                    if (ANY) return true;
                    r.tMax = t;   // GeometricPrimitive::Intersect (Primitive.cpp:26)
                    h->slot = slot; h->b0 = b0; h->b1 = b1; h->b2 = b2;
                    found = true;
                }
                if (flags & PRIM_LEAF_END) break;
                ++slot;
            }
        } else {
            const float4* w = S.wide + 4 * (size_t)cur;
            float4 A = w[0], B = w[1], C = w[2], D = w[3];
            float t0 = 0, t1 = 0;
            bool ok0 = node_slab(mk(A.x, A.y, A.z), mk(A.w, B.x, B.y), r, inv, n0, n1, n2, &t0);
            bool ok1 = node_slab(mk(B.z, B.w, C.x), mk(C.y, C.z, C.w), r, inv, n0, n1, n2, &t1);
            int axis = __float_as_int(D.z);
            bool neg = axis == 0 ? n0 : (axis == 1 ? n1 : n2);
            int nearRef = __float_as_int(neg ? D.y : D.x), farRef = __float_as_int(neg ? D.x : D.y);
            bool okN = neg ? ok1 : ok0, okF = neg ? ok0 : ok1;
            float tN = neg ? t1 : t0, tF = neg ? t0 : t1;
            if (STATS) c->nodes++;   // the near child's visit
            if (okN && tN < r.tMax) {
                if (STATS && !okF) tF = __int_as_float(0x7fc00000);
                if (okF || STATS) {
                    // unreachable: the upload refuses trees deeper than BVHAccel's 64-entry stack
                    if (sp >= kTraversalStack) { atomicOr(S.guard, kGuardStack); break; }
                    if (SHORT && sp < SHORT) { lref[sp * 256] = farRef; lt[sp * 256] = tF; }
                    else { stackRef[sp - SHORT] = farRef; stackT[sp - SHORT] = tF; }
                    ++sp;
                }
                cur = nearRef;
                continue;
            }
            if (STATS) c->nodes++;   // the far child, popped straight back
            if (okF && tF < r.tMax) { cur = farRef; continue; }
        }
        bool more = false;   // pop until an entry passes its box test against the current tMax
        while (sp > 0) {
            --sp;
            int rr;
            float tt;
            if (SHORT && sp < SHORT) { rr = lref[sp * 256]; tt = lt[sp * 256]; }
            else { rr = stackRef[sp - SHORT]; tt = stackT[sp - SHORT]; }
            if (STATS) c->nodes++;
            if (tt < r.tMax) { cur = rr; more = true; break; }
        }
        if (!more) break;
    }
    return found;
}

// Scene::Intersect + SurfaceInteraction construction for the surviving primitive.
template <bool STATS>
__device__ bool intersect(const DeviceScene& S, Ray& r, Isect* si, Counters* c) {
    HitRec h;
    if (!traverse<false, STATS>(S, r, &h, c)) return false;
    int flags = __float_as_int(S.triVerts[3 * (size_t)h.slot].w);
    if (flags & PRIM_SPHERE) sphere_si(S.spheres[__float_as_int(S.triVerts[3 * (size_t)h.slot].x)], r, r.tMax, si);
    else triangle_si(S, h.slot, r, h.b0, h.b1, h.b2, flags, si);
    si->slot = h.slot;
    int4 info = S.primInfo[h.slot];
    int mi = (int)(short)(info.w & 0xffff), mo = (int)(short)((info.w >> 16) & 0xffff);
    if (mi != mo) { si->medIn = mi; si->medOut = mo; }     // Primitive.cpp:30-34
    else { si->medIn = r.medium; si->medOut = r.medium; }
    return true;
}

// ---------------------------------------------------------------- BSDF (Material/Reflection.*)
PBR_HD float cos_t(f3 w) { return w.z; }
PBR_HD float cos2_t(f3 w) { return w.z * w.z; }
PBR_HD float abscos_t(f3 w) { return fabsf(w.z); }
PBR_HD float sin2_t(f3 w) { return mx((float)0, (float)1 - cos2_t(w)); }
PBR_HD float sin_t(f3 w) { return sqrtf(sin2_t(w)); }
PBR_HD float tan_t(f3 w) { return sin_t(w) / cos_t(w); }
PBR_HD float tan2_t(f3 w) { return sin2_t(w) / cos2_t(w); }
PBR_HD float cos_phi(f3 w) { float s = sin_t(w); return (s == 0) ? 1 : clampf(w.x / s, -1, 1); }
PBR_HD float sin_phi(f3 w) { float s = sin_t(w); return (s == 0) ? 0 : clampf(w.y / s, -1, 1); }
PBR_HD float cos2_phi(f3 w) { return cos_phi(w) * cos_phi(w); }
PBR_HD float sin2_phi(f3 w) { return sin_phi(w) * sin_phi(w); }
PBR_HD f3 reflect_(f3 wo, f3 n) { return -wo + 2 * dot(wo, n) * n; }
PBR_HD bool refract_(f3 wi, f3 n, float eta, f3* wt) {
    float cosI = dot(n, wi);
    float sin2I = mx(float(0), float(1 - cosI * cosI));
    float sin2T = eta * eta * sin2I;
    if (sin2T >= 1) return false;
    float cosT = sqrtf(1 - sin2T);
    *wt = eta * -wi + (eta * cosI - cosT) * n;
    return true;
}
PBR_HD bool same_hemi(f3 w, f3 wp) { return w.z * wp.z > 0; }

PBR_HD float fr_dielectric(float cosThetaI, float etaI, float etaT) {   // Fresnel.cpp:7-28
    cosThetaI = clampf(cosThetaI, -1, 1);
    bool entering = cosThetaI > 0.f;
    if (!entering) { float t = etaI; etaI = etaT; etaT = t; cosThetaI = fabsf(cosThetaI); }
    float sinThetaI = sqrtf(mx((float)0, 1 - cosThetaI * cosThetaI));
    float sinThetaT = etaI / etaT * sinThetaI;
    if (sinThetaT >= 1) return 1;
    float cosThetaT = sqrtf(mx((float)0, 1 - sinThetaT * sinThetaT));
    float Rparl = ((etaT * cosThetaI) - (etaI * cosThetaT)) / ((etaT * cosThetaI) + (etaI * cosThetaT));
    float Rperp = ((etaI * cosThetaI) - (etaT * cosThetaT)) / ((etaI * cosThetaI) + (etaT * cosThetaT));
    return (Rparl * Rparl + Rperp * Rperp) / 2;
}
PBR_HD rgb fr_conductor(float cosThetaI, rgb etai, rgb etat, rgb k) {   // Fresnel.cpp:31-54
    cosThetaI = clampf(cosThetaI, -1, 1);
    rgb eta = etat / etai, etak = k / etai;
    float c2 = cosThetaI * cosThetaI;
    float s2 = (float)(1. - (double)c2);
    rgb eta2 = eta * eta, etak2 = etak * etak;
    rgb t0 = eta2 - etak2 - sp(s2);
    rgb a2plusb2 = sqrt_s(t0 * t0 + 4.f * eta2 * etak2);
    rgb t1 = a2plusb2 + sp(c2);
    rgb a = sqrt_s(0.5f * (a2plusb2 + t0));
    rgb t2 = (float)2 * cosThetaI * a;
    rgb Rs = (t1 - t2) / (t1 + t2);
    rgb t3 = c2 * a2plusb2 + sp(s2 * s2);
    rgb t4 = t2 * s2;
    rgb Rp = Rs * (t3 - t4) / (t3 + t4);
    return 0.5f * (Rp + Rs);
}
PBR_HD rgb ld3(const float* v) { return sp3(v[0], v[1], v[2]); }
PBR_HD rgb fresnel_eval(const Lobe& l, float cosI) {
    if (l.fresnel == FR_NOOP) return sp(1.f);
    if (l.fresnel == FR_DIEL) return sp(fr_dielectric(cosI, l.fEtaI, l.fEtaT));
    return fr_conductor(fabsf(cosI), ld3(l.cEtaI), ld3(l.cEtaT), ld3(l.cK));
}
// Trowbridge-Reitz (Microfacet.cpp:116-292), sampleVisibleArea = true
PBR_HD float tr_D(const Lobe& l, f3 wh) {
    float t2 = tan2_t(wh);
    if (is_inf(t2)) return 0.;
    const float c4 = cos2_t(wh) * cos2_t(wh);
    float e = (cos2_phi(wh) / (l.ax * l.ax) + sin2_phi(wh) / (l.ay * l.ay)) * t2;
    return 1 / (kPi * l.ax * l.ay * c4 * (1 + e) * (1 + e));
}
PBR_HD float tr_lambda(const Lobe& l, f3 w) {
    float at = fabsf(tan_t(w));
    if (is_inf(at)) return 0.;
    float alpha = sqrtf(cos2_phi(w) * l.ax * l.ax + sin2_phi(w) * l.ay * l.ay);
    float a2t2 = (alpha * at) * (alpha * at);
    return (-1 + sqrtf(1.f + a2t2)) / 2;
}
PBR_HD float tr_G1(const Lobe& l, f3 w) { return 1 / (1 + tr_lambda(l, w)); }
PBR_HD float tr_G(const Lobe& l, f3 wo, f3 wi) { return 1 / (1 + tr_lambda(l, wo) + tr_lambda(l, wi)); }
// Lambda(wo) handed down by a caller that evaluated it once for a shading event (lamWo: NaN = not
// given).  A material's microfacet lobes share (ax, ay) — one lobe, or a rough dielectric's reflection
// and transmission built from the same roughness — and wo is fixed for the event, so the light
// sample's f and pdf, the BSDF sample's pdf and the sum of f over the lobes all read one value, the
// same bits each would compute (C4/C5: 2-6 evaluations of Lambda(wo) per event before).
constexpr float kNoLambda = __builtin_nanf("");
PBR_HD float lam_or(const Lobe& l, f3 wo, float lamWo) { return lamWo == lamWo ? lamWo : tr_lambda(l, wo); }
PBR_HD void tr_sample11(float cosTheta, float U1, float U2, float* sx, float* sy) {
    if ((double)cosTheta > .9999) {   // the reference's unqualified sqrt/cos/sin resolve to double
        float r = (float)sqrt((double)(U1 / (1 - U1)));
        float phi = (float)(6.28318530718 * (double)U2);
        *sx = (float)((double)r * cos((double)phi));
        *sy = (float)((double)r * sin((double)phi));
        return;
    }
    float sinTheta = sqrtf(mx((float)0, (float)1 - cosTheta * cosTheta));
    float tanTheta = sinTheta / cosTheta;
    float a = 1 / tanTheta;
    float G1 = 2 / (1 + sqrtf(1.f + 1.f / (a * a)));
    float A = 2 * U1 / G1 - 1;
    float tmp = 1.f / (A * A - 1.f);
    if ((double)tmp > 1e10) tmp = 1e10f;
    float B = tanTheta;
    float D = sqrtf(mx(float(B * B * tmp * tmp - (A * A - B * B) * tmp), float(0)));
    float s1 = B * tmp - D, s2 = B * tmp + D;
    *sx = (A < 0 || s2 > 1.f / tanTheta) ? s1 : s2;
    float S;
    if (U2 > 0.5f) { S = 1.f; U2 = 2.f * (U2 - .5f); }
    else { S = -1.f; U2 = 2.f * (.5f - U2); }
    float z = (U2 * (U2 * (U2 * 0.27385f - 0.73369f) + 0.46341f)) /
              (U2 * (U2 * (U2 * 0.093073f + 0.309420f) - 1.000000f) + 0.597999f);
    *sy = S * z * sqrtf(1.f + *sx * *sx);
}
PBR_HD f3 tr_sample_wh(const Lobe& l, f3 wo, float u0, float u1) {
    bool flip = wo.z < 0;
    f3 wi = flip ? -wo : wo;
    f3 ws = normalize(mk(l.ax * wi.x, l.ay * wi.y, wi.z));
    float sx, sy;
    tr_sample11(cos_t(ws), u0, u1, &sx, &sy);
    float tmp = cos_phi(ws) * sx - sin_phi(ws) * sy;
    sy = sin_phi(ws) * sx + cos_phi(ws) * sy;
    sx = tmp;
    sx = l.ax * sx;
    sy = l.ay * sy;
    f3 wh = normalize(mk(-sx, -sy, 1.f));
    if (flip) wh = -wh;
    return wh;
}
PBR_HD float tr_pdf(const Lobe& l, f3 wo, f3 wh, float lamWo = kNoLambda) {
    return tr_D(l, wh) * (1 / (1 + lam_or(l, wo, lamWo))) * absdot(wo, wh) / abscos_t(wo);   // tr_G1(wo)
}

// K: bit mask of the LobeKinds the caller can meet (the scene's materials, or what a type filter
// admits); kinds outside it compile out, which keeps the microfacet code out of simple kernels.
constexpr int kAllLobes = 0x7f;
constexpr int kTexturedLobes = 0x80;   // LOBES flag of the shading kernels: some material has image textures
#define PBR_HAS(K, kind) (((K) >> (kind)) & 1)
template <int K = kAllLobes>
PBR_HD rgb lobe_f(const Lobe& l, f3 wo, f3 wi, float lamWo = kNoLambda) {
    switch (l.kind) {
    case L_LAMBERT: if constexpr (PBR_HAS(K, L_LAMBERT)) return ld3(l.R) * kInvPi; break;
    case L_OREN: if constexpr (PBR_HAS(K, L_OREN)) {
        float sI = sin_t(wi), sO = sin_t(wo);
        float maxCos = 0;
        if ((double)sI > 1e-4 && (double)sO > 1e-4) {
            float dCos = cos_phi(wi) * cos_phi(wo) + sin_phi(wi) * sin_phi(wo);
            maxCos = mx((float)0, dCos);
        }
        float sinAlpha, tanBeta;
        if (abscos_t(wi) > abscos_t(wo)) { sinAlpha = sO; tanBeta = sI / abscos_t(wi); }
        else { sinAlpha = sI; tanBeta = sO / abscos_t(wo); }
        return ld3(l.R) * kInvPi * (l.A + l.B * maxCos * sinAlpha * tanBeta);
    } break;
    case L_MF_R: if constexpr (PBR_HAS(K, L_MF_R)) {
        float cO = abscos_t(wo), cI = abscos_t(wi);
        f3 wh = wi + wo;
        if (cI == 0 || cO == 0) return sp(0.f);
        if (wh.x == 0 && wh.y == 0 && wh.z == 0) return sp(0.f);
        wh = normalize(wh);
        rgb F = fresnel_eval(l, dot(wi, faceforward(wh, mk(0, 0, 1))));
        return ld3(l.R) * tr_D(l, wh) * (1 / (1 + lam_or(l, wo, lamWo) + tr_lambda(l, wi))) * F / (4 * cI * cO);   // tr_G
    } break;
    case L_MF_T: if constexpr (PBR_HAS(K, L_MF_T)) {
        if (same_hemi(wo, wi)) return sp(0.f);
        float cO = cos_t(wo), cI = cos_t(wi);
        if (cI == 0 || cO == 0) return sp(0.f);
        float eta = cos_t(wo) > 0 ? (l.etaB / l.etaA) : (l.etaA / l.etaB);
        f3 wh = normalize(wo + wi * eta);
        if (wh.z < 0) wh = -wh;
        if (dot(wo, wh) * dot(wi, wh) > 0) return sp(0.f);
        rgb F = sp(fr_dielectric(dot(wo, wh), l.etaA, l.etaB));
        float sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
        float factor = 1 / eta;
        return (sp(1.f) - F) * ld3(l.T) *
               fabsf(tr_D(l, wh) * (1 / (1 + lam_or(l, wo, lamWo) + tr_lambda(l, wi))) * eta * eta * absdot(wi, wh) *
                     absdot(wo, wh) * factor * factor /
                     (cI * cO * sqrtDenom * sqrtDenom));
    } break;
    default: break;
    }
    return sp(0.f);
}
template <int K = kAllLobes>
PBR_HD float lobe_pdf(const Lobe& l, f3 wo, f3 wi, float lamWo = kNoLambda) {
    switch (l.kind) {
    case L_LAMBERT: case L_OREN:
        if constexpr (PBR_HAS(K, L_LAMBERT) || PBR_HAS(K, L_OREN)) return same_hemi(wo, wi) ? abscos_t(wi) * kInvPi : 0;
        break;
    case L_MF_R: if constexpr (PBR_HAS(K, L_MF_R)) {
        if (!same_hemi(wo, wi)) return 0;
        f3 wh = normalize(wo + wi);
        return tr_pdf(l, wo, wh, lamWo) / (4 * dot(wo, wh));
    } break;
    case L_MF_T: if constexpr (PBR_HAS(K, L_MF_T)) {
        if (same_hemi(wo, wi)) return 0;
        float eta = cos_t(wo) > 0 ? (l.etaB / l.etaA) : (l.etaA / l.etaB);
        f3 wh = normalize(wo + wi * eta);
        if (dot(wo, wh) * dot(wi, wh) > 0) return 0;
        float sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
        float dwh = fabsf((eta * eta * dot(wi, wh)) / (sqrtDenom * sqrtDenom));
        return tr_pdf(l, wo, wh, lamWo) * dwh;
    } break;
    default: break;
    }
    return 0;
}
// lobe_f and lobe_pdf for one (wo, wi) in one pass (bsdf_f_pdf): the microfacet kinds evaluate the
// half vector, D(wh) and Lambda(wo) once for both.  Every value is the separate functions' own:
// the sums wi + wo and wo + wi are the same floats, and for transmission f's half vector is pdf's
// turned to +z, where D — a function of wh.z², |wh.x / sinθ| and |wh.y / sinθ| — is the same and
// the two dot products change sign together.  wantF: the caller adds f (BSDF::f's reflect /
// transmit filter); f is then exactly what lobe_f returns, black where it returns black.
template <int K = kAllLobes>
PBR_HD void lobe_f_pdf(const Lobe& l, f3 wo, f3 wi, bool wantF, rgb* fOut, float* pdfOut, float lamWo = kNoLambda) {
    rgb f = sp(0.f);
    float pdf = 0.f;
    switch (l.kind) {
    case L_MF_R: if constexpr (PBR_HAS(K, L_MF_R)) {
        const float cO = abscos_t(wo), cI = abscos_t(wi);
        const f3 whRaw = wi + wo;
        const bool sh = same_hemi(wo, wi);
        const bool fLive = wantF && !(cI == 0 || cO == 0) && !(whRaw.x == 0 && whRaw.y == 0 && whRaw.z == 0);
        if (fLive || sh) {
            const f3 wh = normalize(whRaw);
            const float D = tr_D(l, wh), lo = lam_or(l, wo, lamWo);
            if (fLive) {
                const rgb F = fresnel_eval(l, dot(wi, faceforward(wh, mk(0, 0, 1))));
                const float G = 1 / (1 + lo + tr_lambda(l, wi));   // tr_G
                f = ld3(l.R) * D * G * F / (4 * cI * cO);
            }
            if (sh) pdf = D * (1 / (1 + lo)) * absdot(wo, wh) / abscos_t(wo) / (4 * dot(wo, wh));   // tr_pdf / (4 wo·wh)
        }
        break;
    } break;
    case L_MF_T: if constexpr (PBR_HAS(K, L_MF_T)) {
        if (same_hemi(wo, wi)) break;
        const float eta = cos_t(wo) > 0 ? (l.etaB / l.etaA) : (l.etaA / l.etaB);
        const f3 whp = normalize(wo + wi * eta);   // lobe_pdf's half vector
        if (dot(wo, whp) * dot(wi, whp) > 0) break;
        const float D = tr_D(l, whp), lo = lam_or(l, wo, lamWo);
        const float cO = cos_t(wo), cI = cos_t(wi);
        if (wantF && !(cI == 0 || cO == 0)) {
            const f3 wh = whp.z < 0 ? -whp : whp;   // lobe_f's
            const rgb F = sp(fr_dielectric(dot(wo, wh), l.etaA, l.etaB));
            const float sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
            const float factor = 1 / eta;
            const float G = 1 / (1 + lo + tr_lambda(l, wi));   // tr_G
            f = (sp(1.f) - F) * ld3(l.T) *
                fabsf(D * G * eta * eta * absdot(wi, wh) * absdot(wo, wh) * factor * factor / (cI * cO * sqrtDenom * sqrtDenom));
        }
        const float sqrtDenom = dot(wo, whp) + eta * dot(wi, whp);
        const float dwh = fabsf((eta * eta * dot(wi, whp)) / (sqrtDenom * sqrtDenom));
        pdf = D * (1 / (1 + lo)) * absdot(wo, whp) / abscos_t(wo) * dwh;   // tr_pdf · dwh
        break;
    } break;
    default:
        if (wantF) f = lobe_f<K>(l, wo, wi, lamWo);
        pdf = lobe_pdf<K>(l, wo, wi, lamWo);
        break;
    }
    *fOut = f;
    *pdfOut = pdf;
}
// Sampling.cpp:74-92, Sampling.h:57-61
PBR_HD void concentric_disk(float u0, float u1, float* dx, float* dy) {
    float ox = 2.f * u0 - 1, oy = 2.f * u1 - 1;
    if (ox == 0 && oy == 0) { *dx = 0; *dy = 0; return; }
    float theta, r;
    if (fabsf(ox) > fabsf(oy)) { r = ox; theta = kPiOver4 * (oy / ox); }
    else { r = oy; theta = kPiOver2 - kPiOver4 * (ox / oy); }
    *dx = r * t_cos(theta);
    *dy = r * t_sin(theta);
}
PBR_HD f3 cosine_hemisphere(float u0, float u1) {
    float dx, dy;
    concentric_disk(u0, u1, &dx, &dy);
    float z = sqrtf(mx((float)0, 1 - dx * dx - dy * dy));
    return mk(dx, dy, z);
}
// BxDF::Sample_f.  The value it returns is only used for specular lobes: BSDF::Sample_f replaces a
// non-specular lobe's f by the sum of f over the matching lobes (Reflection.cpp:150-160), so for
// the diffuse and microfacet kinds the lobe's own f(wo, wi) — which the reference evaluates and
// then drops — is not computed here (black is returned; wi and pdf are the reference's).
template <int K = kAllLobes>
PBR_HD rgb lobe_sample(const Lobe& l, f3 wo, f3* wi, float u0, float u1, float* pdf, int* st, float lamWo = kNoLambda) {
    switch (l.kind) {
    case L_LAMBERT: case L_OREN: if constexpr (PBR_HAS(K, L_LAMBERT) || PBR_HAS(K, L_OREN)) {
        *wi = cosine_hemisphere(u0, u1);
        if (wo.z < 0) wi->z *= -1;
        *pdf = lobe_pdf<K>(l, wo, *wi);
        return sp(0.f);   // (f: dropped by bsdf_sample)
    } break;
    case L_SPEC_R: if constexpr (PBR_HAS(K, L_SPEC_R)) {
        *wi = mk(-wo.x, -wo.y, wo.z);
        *pdf = 1;
        return fresnel_eval(l, cos_t(*wi)) * ld3(l.R) / abscos_t(*wi);
    } break;
    case L_SPEC_T: if constexpr (PBR_HAS(K, L_SPEC_T)) {
        bool entering = cos_t(wo) > 0;
        float etaI = entering ? l.etaA : l.etaB, etaT = entering ? l.etaB : l.etaA;
        if (!refract_(wo, faceforward(mk(0, 0, 1), wo), etaI / etaT, wi)) return sp(0.f);
        *pdf = 1;
        rgb ft = ld3(l.T) * (sp(1.f) - sp(fr_dielectric(cos_t(*wi), l.etaA, l.etaB)));
        ft = ft * ((etaI * etaI) / (etaT * etaT));
        return ft / abscos_t(*wi);
    } break;
    case L_FRESNEL_SPEC: if constexpr (PBR_HAS(K, L_FRESNEL_SPEC)) {
        float F = fr_dielectric(cos_t(wo), l.etaA, l.etaB);
        if (u0 < F) {
            *wi = mk(-wo.x, -wo.y, wo.z);
            *st = BSDF_SPECULAR | BSDF_REFLECTION;
            *pdf = F;
            return F * ld3(l.R) / abscos_t(*wi);
        }
        bool entering = cos_t(wo) > 0;
        float etaI = entering ? l.etaA : l.etaB, etaT = entering ? l.etaB : l.etaA;
        if (!refract_(wo, faceforward(mk(0, 0, 1), wo), etaI / etaT, wi)) return sp(0.f);
        rgb ft = ld3(l.T) * (1 - F);
        ft = ft * ((etaI * etaI) / (etaT * etaT));
        *st = BSDF_SPECULAR | BSDF_TRANSMISSION;
        *pdf = 1 - F;
        return ft / abscos_t(*wi);
    } break;
    case L_MF_R: if constexpr (PBR_HAS(K, L_MF_R)) {
        if (wo.z == 0) return sp(0.f);
        f3 wh = tr_sample_wh(l, wo, u0, u1);
        if (dot(wo, wh) < 0) return sp(0.f);
        *wi = reflect_(wo, wh);
        if (!same_hemi(wo, *wi)) return sp(0.f);
        *pdf = tr_pdf(l, wo, wh, lamWo) / (4 * dot(wo, wh));
        return sp(0.f);   // (f: dropped by bsdf_sample)
    } break;
    case L_MF_T: if constexpr (PBR_HAS(K, L_MF_T)) {
        if (wo.z == 0) return sp(0.f);
        f3 wh = tr_sample_wh(l, wo, u0, u1);
        if (dot(wo, wh) < 0) return sp(0.f);
        float eta = cos_t(wo) > 0 ? (l.etaA / l.etaB) : (l.etaB / l.etaA);
        if (!refract_(wo, wh, eta, wi)) return sp(0.f);
        *pdf = lobe_pdf<K>(l, wo, *wi, lamWo);
        return sp(0.f);   // (f: dropped by bsdf_sample)
    } break;
    default: break;
    }
    return sp(0.f);
}

struct BSDF {                    // Reflection.h:101-149: frame + the material's lobe template
    f3 ns, ng, ss, ts;
    const MatTemplate* mt;
    PBR_HD f3 to_local(f3 v) const { return mk(dot(v, ss), dot(v, ts), dot(v, ns)); }
    PBR_HD f3 to_world(f3 v) const {
        return mk(ss.x * v.x + ts.x * v.y + ns.x * v.z, ss.y * v.x + ts.y * v.y + ns.y * v.z, ss.z * v.x + ts.z * v.y + ns.z * v.z);
    }
};
PBR_HD bool matches(const Lobe& l, int t) { return (l.type & t) == l.type; }
PBR_HD int num_components(const MatTemplate& mt, int flags) {
    int k = 0;
    for (int i = 0; i < mt.nLobes; ++i) if (matches(mt.lobes[i], flags)) ++k;
    return k;
}
PBR_HD int num_components(const BSDF& b, int flags) { return num_components(*b.mt, flags); }
// Lambda(wo) of the BSDF's microfacet lobes for a local wo, evaluated once (kNoLambda when it has
// none, or — never for the reference's materials — lobes of different alphas, which then evaluate
// their own)
template <int K = kAllLobes>
PBR_HD float mf_lambda(const BSDF& b, f3 wo) {
    if constexpr (!(PBR_HAS(K, L_MF_R) || PBR_HAS(K, L_MF_T))) {
        return kNoLambda;
    } else {
        const MatTemplate& m = *b.mt;
        const bool mf0 = m.nLobes > 0 && (m.lobes[0].kind == L_MF_R || m.lobes[0].kind == L_MF_T);
        const bool mf1 = m.nLobes > 1 && (m.lobes[1].kind == L_MF_R || m.lobes[1].kind == L_MF_T);
        if (!mf0 && !mf1) return kNoLambda;
        if (mf0 && mf1 && !(m.lobes[0].ax == m.lobes[1].ax && m.lobes[0].ay == m.lobes[1].ay)) return kNoLambda;
        return tr_lambda(m.lobes[mf0 ? 0 : 1], wo);
    }
}
template <int K = kAllLobes>
PBR_HD rgb bsdf_f(const BSDF& b, f3 woW, f3 wiW, int flags) {   // Reflection.cpp:56-71
    f3 wi = b.to_local(wiW), wo = b.to_local(woW);
    if (wo.z == 0) return sp(0.f);
    bool reflect = dot(wiW, b.ng) * dot(woW, b.ng) > 0;
    rgb f = sp(0.f);
    for (int i = 0; i < b.mt->nLobes; ++i) {
        const Lobe& l = b.mt->lobes[i];
        if (matches(l, flags) && ((reflect && (l.type & BSDF_REFLECTION)) || (!reflect && (l.type & BSDF_TRANSMISSION))))
            f = f + lobe_f<K>(l, wo, wi);
    }
    return f;
}
// BSDF::f (Reflection.cpp:56-71) and BSDF::Pdf (:92-106) of one direction in one pass: the same
// per-lobe values and the same sums in the same order, each lobe's shared terms evaluated once
// (lobe_f_pdf).  Returns f; *pdf as bsdf_pdf.
template <int K = kAllLobes>
PBR_HD rgb bsdf_f_pdf(const BSDF& b, f3 woW, f3 wiW, int flags, float* pdfOut, float lamWo = kNoLambda) {
    const f3 wi = b.to_local(wiW), wo = b.to_local(woW);
    if (wo.z == 0) { *pdfOut = 0.f; return sp(0.f); }   // both return 0 there (BSDF::Pdf also with no lobes)
    const bool reflect = dot(wiW, b.ng) * dot(woW, b.ng) > 0;
    rgb f = sp(0.f);
    float pdf = 0.f;
    int m = 0;
    for (int i = 0; i < b.mt->nLobes; ++i) {
        const Lobe& l = b.mt->lobes[i];
        if (!matches(l, flags)) continue;
        ++m;
        const bool wantF = (reflect && (l.type & BSDF_REFLECTION)) || (!reflect && (l.type & BSDF_TRANSMISSION));
        rgb fl;
        float pl;
        lobe_f_pdf<K>(l, wo, wi, wantF, &fl, &pl, lamWo);
        if (wantF) f = f + fl;
        pdf += pl;
    }
    *pdfOut = m > 0 ? pdf / m : 0.f;
    return f;
}
template <int K = kAllLobes>
PBR_HD float bsdf_pdf(const BSDF& b, f3 woW, f3 wiW, int flags) {   // Reflection.cpp:92-106
    if (b.mt->nLobes == 0) return 0.f;
    f3 wo = b.to_local(woW), wi = b.to_local(wiW);
    if (wo.z == 0) return 0.f;
    float pdf = 0.f;
    int m = 0;
    for (int i = 0; i < b.mt->nLobes; ++i)
        if (matches(b.mt->lobes[i], flags)) { ++m; pdf += lobe_pdf<K>(b.mt->lobes[i], wo, wi); }
    return m > 0 ? pdf / m : 0.f;
}
// BSDF::Sample_f (Reflection.cpp:108-164) in two steps.  bsdf_sample_dir picks the lobe, samples
// its direction and forms the pdf; bsdf_sample_sum forms the value — a specular lobe's own f, else
// the sum of f over the matching lobes.  Both are pure, so a caller that needs the value only in some
// cases (EstimateDirect's BSDF sample: only when the sampled direction can reach the light) asks for
// it only then; bsdf_sample is the two in sequence.  dir returns false where the reference returns
// black before the sum (no matching lobe, wo.z == 0 — *pdf and *sampledType left as they were —
// or a zero pdf).
struct BsdfDraw {
    f3 wi;          // the sampled direction, local
    rgb fSpec;      // a specular lobe's own value
    bool specular;  // the chosen lobe is specular
    float lamWo;    // Lambda(wo) of the microfacet lobes (mf_lambda), for the sum
};
template <int K = kAllLobes>
PBR_HD bool bsdf_sample_dir(const BSDF& b, f3 woW, f3* wiW, float u0, float u1, float* pdf, int type, int* sampledType,
                            BsdfDraw* d, float lamWo = kNoLambda) {
    int m = num_components(b, type);
    if (m == 0) { *pdf = 0; *sampledType = 0; return false; }
    int comp = (int)floorf(u0 * m);
    if (comp > m - 1) comp = m - 1;
    int chosen = -1, count = comp;
    for (int i = 0; i < b.mt->nLobes; ++i)
        if (matches(b.mt->lobes[i], type) && count-- == 0) { chosen = i; break; }
    const Lobe& bx = b.mt->lobes[chosen];
    float ur0 = mn(u0 * m - comp, kOneMinusEpsilon);
    f3 wi, wo = b.to_local(woW);
    if (wo.z == 0) return false;
    *pdf = 0;
    int st = bx.type;
    const bool mfChosen = bx.kind == L_MF_R || bx.kind == L_MF_T;
    if (lamWo != lamWo && (mfChosen || m > 1)) lamWo = mf_lambda<K>(b, wo);   // (not given: evaluated once here)
    d->lamWo = lamWo;
    d->fSpec = lobe_sample<K>(bx, wo, &wi, ur0, u1, pdf, &st, lamWo);
    *sampledType = st;
    if (*pdf == 0) { *sampledType = 0; return false; }
    *wiW = b.to_world(wi);
    d->wi = wi;
    d->specular = (bx.type & BSDF_SPECULAR) != 0;
    if (!d->specular && m > 1)
        for (int i = 0; i < b.mt->nLobes; ++i)
            if (i != chosen && matches(b.mt->lobes[i], type)) *pdf += lobe_pdf<K>(b.mt->lobes[i], wo, wi, lamWo);
    if (m > 1) *pdf /= m;
    return true;
}
template <int K = kAllLobes>
PBR_HD rgb bsdf_sample_sum(const BSDF& b, f3 woW, f3 wiW, int type, const BsdfDraw& d) {
    if (d.specular) return d.fSpec;
    const f3 wo = b.to_local(woW);   // the same operations as bsdf_sample_dir's: the same bits
    bool reflect = dot(wiW, b.ng) * dot(woW, b.ng) > 0;
    rgb f = sp(0.f);
    for (int i = 0; i < b.mt->nLobes; ++i) {
        const Lobe& l = b.mt->lobes[i];
        if (matches(l, type) && ((reflect && (l.type & BSDF_REFLECTION)) || (!reflect && (l.type & BSDF_TRANSMISSION))))
            f = f + lobe_f<K>(l, wo, d.wi, d.lamWo);
    }
    return f;
}
template <int K = kAllLobes>
PBR_HD rgb bsdf_sample(const BSDF& b, f3 woW, f3* wiW, float u0, float u1, float* pdf, int type, int* sampledType) {
    BsdfDraw d;
    if (!bsdf_sample_dir<K>(b, woW, wiW, u0, u1, pdf, type, sampledType, &d)) return sp(0.f);
    return bsdf_sample_sum<K>(b, woW, *wiW, type, d);
}
// ImageTexture::Evaluate (ImageTexture.h:52-60) with zero differentials: MIPMap::triangle(0, st)
// (MIPMap.h:240-252) on the level-0 texels, Texel's wrap modes (:166-190).
__device__ __forceinline__ float4 tex_texel(const float4* texels, const TexDev& t, int s, int u) {
    if (t.wrap == 0) { s = s % t.w; if (s < 0) s += t.w; u = u % t.h; if (u < 0) u += t.h; }
    else if (t.wrap == 2) { s = clampi(s, 0, t.w - 1); u = clampi(u, 0, t.h - 1); }
    else if (s < 0 || s >= t.w || u < 0 || u >= t.h) return make_float4(0.f, 0.f, 0.f, 0.f);
    return texels[t.offset + (size_t)u * t.w + s];
}
__device__ __forceinline__ float4 tex_lookup(const float4* texels, const TexDev& t, float su, float sv) {
    const float s = su * t.w - 0.5f, u = sv * t.h - 0.5f;
    const int s0 = (int)floorf(s), u0 = (int)floorf(u);
    const float ds = s - s0, du = u - u0;
    const float w00 = (1 - ds) * (1 - du), w01 = (1 - ds) * du, w10 = ds * (1 - du), w11 = ds * du;
    const float4 a = tex_texel(texels, t, s0, u0), b = tex_texel(texels, t, s0, u0 + 1), c = tex_texel(texels, t, s0 + 1, u0),
                 d = tex_texel(texels, t, s0 + 1, u0 + 1);
    return make_float4(w00 * a.x + w01 * b.x + w10 * c.x + w11 * d.x, w00 * a.y + w01 * b.y + w10 * c.y + w11 * d.y,
                       w00 * a.z + w01 * b.z + w10 * c.z + w11 * d.z, 0.f);
}
// A textured material's lobes at one hit: its textures evaluated through their UVMapping2D
// (Texture.cpp:8-14), then the material's ComputeScatteringFunctions (pbr_material.h).  Out of line:
// the untextured scenes' shading kernels pay no registers for it.  It takes the three arrays by value:
// a reference to the kernel's DeviceScene parameter would make the compiler copy the whole parameter
// block into per-lane scratch and read every parameter from there.
__device__ __noinline__ void textured_template(const TexMat* texMats, const TexDev* textures, const float4* texels, int mat,
                                               float u, float v, bool multiLobe, MatTemplate* out) {
    const TexMat& tm = texMats[mat];
    MatParams p = tm.p;
    for (int k = 0; k < 6; ++k) {
        const int ti = tm.tex[k];
        if (ti < 0) continue;
        const TexDev& t = textures[ti];
        const float4 val = tex_lookup(texels, t, t.su * u + t.du, t.sv * v + t.dv);
        float* dst = k == 0 ? p.Kd : (k == 1 ? p.Ks : (k == 2 ? p.Kr : p.Kt));
        if (k == 4) p.sigma = val.x;
        else if (k == 5) p.roughness = val.x;
        else { dst[0] = val.x; dst[1] = val.y; dst[2] = val.z; }
    }
    material_template(p, multiLobe, out);
}

// SurfaceInteraction::ComputeScatteringFunctions → BSDF(si, eta) frame (Reflection.h:105-110)
// mats: S.materials, or a kernel's LDS copy of it; texLocal: where a textured material's per-hit
// lobes go (the BSDF points at it)
// TEX = false (scenes without image textures) keeps every template read on its known address space.
template <bool TEX>
__device__ __forceinline__ bool make_bsdf(const DeviceScene& S, const MatTemplate* mats, const Isect& si, bool multiLobe, BSDF* b,
                                          MatTemplate* texLocal) {
    int mat = S.primInfo[si.slot].y;
    if (mat < 0) return false;
    const MatTemplate* mt = mats + 2 * mat + (multiLobe ? 1 : 0);
    if (!mt->valid) return false;
    if constexpr (TEX) {
        if (mt->textured) {
            textured_template(S.texMats, S.textures, S.texels, mat, si.u, si.v, multiLobe, texLocal);
            mt = texLocal;
        }
    }
    b->mt = mt;
    b->ns = si.sn;
    b->ng = si.n;
    b->ss = normalize(si.dpdu);
    b->ts = cross(b->ns, b->ss);
    return true;
}

// ---------------------------------------------------------------- lights (Light/*.cpp)
PBR_HD rgb area_L(const DLight& l, f3 n, f3 w) { return (l.twoSided || dot(n, w) > 0) ? ld3(l.L) : sp(0.f); }
PBR_HD void sphere_uv(f3 p, float* u, float* v) {   // SkyBoxLight.cpp:12-17
    const Atan2Asin a = t_atan2_asin(p.z, p.x, p.y);
    float phi = a.phi;
    float theta = a.theta;
    *u = 1 - (phi + kPi) * kInv2Pi;
    *v = (theta + kPiOver2) * kInvPi;
}
__device__ __forceinline__ rgb sky_value(const DeviceScene& S, const DLight& l, float u, float v) {   // SkyBoxLight.cpp:27-40
    u = clampf(u, 0.f, 1.f);
    v = clampf(v, 0.f, 1.f);
    int w = u * l.envW, h = v * l.envH;
    w = clampi(w, 0, l.envW - 1);
    h = clampi(h, 0, l.envH - 1);
    float4 t = S.env[w + h * l.envW];   // HDRtoLDR already applied at upload
    return sp3(t.x, t.y, t.z);
}
// ---- InfiniteAreaLight (Light/InfiniteAreaLight.cpp:63-110) over the tables of pbr_infinite.cpp
// MIPMap::Lookup(st, 0) = triangle(0, st): bilinear on level 0, ImageWrap::Repeat (MIPMap.h:240-252)
__device__ __forceinline__ rgb inf_lookup(const InfDev& E, float s0f, float t0f) {
    float s = s0f * E.w - 0.5f, t = t0f * E.h - 0.5f;
    float fs = floorf(s), ft = floorf(t);
    int s0 = (int)fs, t0 = (int)ft;
    float ds = s - s0, dt = t - t0;
    auto wrap = [](int a, int b) { int r = a - (a / b) * b; return r < 0 ? r + b : r; };   // Mod (PBR.h:194-197)
    int sa = wrap(s0, E.w), sb = wrap(s0 + 1, E.w), ta = wrap(t0, E.h), tb = wrap(t0 + 1, E.h);
    float4 a = E.tex[(size_t)ta * E.w + sa], b = E.tex[(size_t)tb * E.w + sa];
    float4 c = E.tex[(size_t)ta * E.w + sb], d = E.tex[(size_t)tb * E.w + sb];
    return ((1 - ds) * (1 - dt)) * sp3(a.x, a.y, a.z) + ((1 - ds) * dt) * sp3(b.x, b.y, b.z) +
           (ds * (1 - dt)) * sp3(c.x, c.y, c.z) + (ds * dt) * sp3(d.x, d.y, d.z);
}
PBR_HD float spherical_theta(f3 v) { return t_acos(clampf(v.z, -1, 1)); }   // Geometry.h:1517-1519
PBR_HD float spherical_phi(f3 v) {                                           // Geometry.h:1521-1524
    float p = t_atan2(v.y, v.x);
    return (p < 0) ? (p + 2 * kPi) : p;
}
// FindInterval (PBR.h:168-181) over a cdf of `size` entries
__device__ __forceinline__ int find_interval(const float* cdf, int size, float u) {
    int first = 0, len_ = size;
    while (len_ > 0) {
        int half = len_ >> 1, middle = first + half;
        if (cdf[middle] <= u) { first = middle + 1; len_ -= half + 1; }
        else len_ = half;
    }
    return clampi(first - 1, 0, size - 2);
}
// Distribution1D::SampleContinuous (Sampling.h:117-131)
__device__ __forceinline__ float sample_continuous(const float* func, const float* cdf, int n, float funcInt, float u,
                                                   float* pdf, int* off) {
    int offset = find_interval(cdf, n + 1, u);
    *off = offset;
    float du = u - cdf[offset];
    if ((cdf[offset + 1] - cdf[offset]) > 0) du /= (cdf[offset + 1] - cdf[offset]);
    *pdf = (funcInt > 0) ? func[offset] / funcInt : 0;
    return (offset + du) / n;
}
// The InfiniteAreaLight functions are out of line and read the light's record from device memory,
// so scenes without one pay neither registers nor kernel-argument SGPRs for them.
__device__ __noinline__ rgb inf_Le(const InfDev* E, f3 d) {   // InfiniteAreaLight.cpp:70-75
    f3 w = normalize(xf_vector(E->w2l, d));
    return inf_lookup(*E, spherical_phi(w) * kInv2Pi, spherical_theta(w) * kInvPi);
}
// Pdf_Li (InfiniteAreaLight.cpp:103-110) with Distribution2D::Pdf (Sampling.h:159-166)
__device__ __noinline__ float inf_pdf_li(const InfDev* Ep, f3 w) {
    const InfDev& E = *Ep;
    f3 wi = xf_vector(E.w2l, w);
    float theta = spherical_theta(wi), phi = spherical_phi(wi);
    float sinTheta = t_sin(theta);
    if (sinTheta == 0) return 0;
    float p0 = phi * kInv2Pi, p1 = theta * kInvPi;
    int iu = clampi((int)(p0 * E.w), 0, E.w - 1);
    int iv = clampi((int)(p1 * E.h), 0, E.h - 1);
    return E.condFunc[(size_t)iv * E.w + iu] / E.margInt / (2 * kPi * kPi * sinTheta);
}

__device__ __forceinline__ rgb light_Le(const DeviceScene& S, const DLight& l, const Ray& r) {
    if (l.type == LT_INF) return inf_Le(S.inf, r.d);
    if (l.type == LT_SKY) {
        f3 dn = normalize(r.d);
        float u, v;
        sphere_uv(dn, &u, &v);
        if (l.envW > 0) return sky_value(S, l, u, v);
        return sp(0.f);
    }
    return sp(0.8f);   // Light::Le default (Light.h:58, F4)
}
PBR_HD f3 uniform_sphere(float u0, float u1) {   // Sampling.cpp:59-64
    float z = 1 - 2 * u0;
    float r = sqrtf(mx((float)0, (float)1 - z * z));
    float phi = 2 * kPi * u1;
    const SinCos sc = t_sincos(phi);
    return mk(r * sc.c, r * sc.s, z);
}
struct VisPt { f3 p, pError, n; int medIn, medOut; };
__device__ __forceinline__ void tri_verts(const DeviceScene& S, int slot, f3* p0, f3* p1, f3* p2) {
    const float4* tv = S.triVerts + 3 * (size_t)slot;
    float4 a = tv[0], b = tv[1], c = tv[2];
    *p0 = mk(a.x, a.y, a.z); *p1 = mk(b.x, b.y, b.z); *p2 = mk(c.x, c.y, c.z);
}
// InfiniteAreaLight::Sample_Li (InfiniteAreaLight.cpp:78-100) with Distribution2D::SampleContinuous
// (Sampling.h:146-156)
// Out of line, returning by value: pointer out-parameters of a call make the caller keep its
// (wi, pdf, vis) variables in private memory, so every shading kernel would store them to scratch
// on every light sample, whichever light type it samples.
struct InfLiSample { rgb L; f3 wi; float pdf; bool mapped; };   // mapped: mapPdf != 0 (wi set)
__device__ __noinline__ InfLiSample inf_sample_li(const InfDev* Ep, float u0, float u1) {
    const InfDev& E = *Ep;
    InfLiSample o;
    o.L = sp(0.f);
    o.wi = mk(0, 0, 0);
    o.mapped = false;
    float pdf0, pdf1;
    int row, col;
    float d1 = sample_continuous(E.margFunc, E.margCdf, E.h, E.margInt, u1, &pdf1, &row);
    float d0 = sample_continuous(E.condFunc + (size_t)row * E.w, E.condCdf + (size_t)row * (E.w + 1), E.w,
                                 E.margFunc[row], u0, &pdf0, &col);
    float mapPdf = pdf0 * pdf1;
    if (mapPdf == 0) { o.pdf = 0; return o; }
    o.mapped = true;
    float theta = d1 * kPi, phi = d0 * 2 * kPi;
    float cosTheta = t_cos(theta), sinTheta = t_sin(theta);
    float sinPhi = t_sin(phi), cosPhi = t_cos(phi);
    o.wi = xf_vector(E.l2w, mk(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta));
    o.pdf = mapPdf / (2 * kPi * kPi * sinTheta);
    if (sinTheta == 0) o.pdf = 0;
    o.L = inf_lookup(E, d0, d1);
    return o;
}
PBR_HELPER rgb sample_li(const DeviceScene& S, const DLight& l, const Isect& ref, float u0, float u1, f3* wi, float* pdf, VisPt* v) {
    if (l.type == LT_POINT) {   // PointLight.cpp:5-15
        f3 pl = mk(l.p[0], l.p[1], l.p[2]);
        *wi = normalize(pl - ref.p);
        *pdf = 1.f;
        v->p = pl; v->pError = mk(0, 0, 0); v->n = mk(0, 0, 0); v->medIn = l.medIn; v->medOut = l.medOut;
        f3 dd = pl - ref.p;
        return ld3(l.L) / len2(dd);
    }
    if (l.type == LT_AREA) {    // DiffuseLight.cpp:25-40, Shape.cpp:18-30, Triangle.cpp:360-387
        f3 p0, p1, p2;
        tri_verts(S, l.primSlot, &p0, &p1, &p2);
        float su0 = sqrtf(u0);
        float b0 = 1 - su0, b1 = u1 * su0;
        f3 ip = b0 * p0 + b1 * p1 + (1 - b0 - b1) * p2;
        f3 in = normalize(cross(p1 - p0, p2 - p0));
        int flags = __float_as_int(S.triVerts[3 * (size_t)l.primSlot].w);
        if (flags & PRIM_FLIP) in = in * -1.f;
        f3 pAbs = vabs(b0 * p0) + vabs(b1 * p1) + vabs((1 - b0 - b1) * p2);
        f3 ipErr = gamma_n(6) * pAbs;
        float area = (float)(0.5 * (double)len(cross(p1 - p0, p2 - p0)));
        *pdf = 1 / area;
        f3 w = ip - ref.p;
        if (len2(w) == 0) *pdf = 0;
        else {
            w = normalize(w);
            *pdf *= len2(ref.p - ip) / absdot(in, -w);
            if (is_inf(*pdf)) *pdf = 0.f;
        }
        if (*pdf == 0 || len2(ip - ref.p) == 0) { *pdf = 0; return sp(0.f); }
        *wi = normalize(ip - ref.p);
        v->p = ip; v->pError = ipErr; v->n = in; v->medIn = -1; v->medOut = -1;
        return area_L(l, in, -*wi);
    }
    if (l.type == LT_INF) {   // InfiniteAreaLight::Sample_Li (InfiniteAreaLight.cpp:78-100)
        const InfLiSample o = inf_sample_li(S.inf, u0, u1);
        *pdf = o.pdf;
        if (!o.mapped) return o.L;   // (wi and vis untouched, as the reference leaves them)
        *wi = o.wi;
        v->p = ref.p + o.wi * (2 * l.worldRadius); v->pError = mk(0, 0, 0); v->n = mk(0, 0, 0); v->medIn = -1; v->medOut = -1;
        return o.L;
    }
    // SkyBoxLight::Sample_Li (SkyBoxLight.cpp:43-56)
    *wi = uniform_sphere(u0, u1);
    *pdf = 1.f / (4 * kPi);
    v->p = ref.p + *wi * (2 * l.worldRadius); v->pError = mk(0, 0, 0); v->n = mk(0, 0, 0); v->medIn = -1; v->medOut = -1;
    float ul, vl;
    sphere_uv(normalize(*wi), &ul, &vl);
    if (l.envW <= 0) return sp(0.f);
    return sky_value(S, l, ul, vl);
}
// Shape::Pdf through the light's own triangle (Shape.cpp:31-42); 0 for point and skybox lights
PBR_HELPER float pdf_li(const DeviceScene& S, const DLight& l, const Isect& ref, f3 wi) {
    if (l.type == LT_INF) return inf_pdf_li(S.inf, wi);
    if (l.type != LT_AREA) return 0;
    Ray ray = spawn_ray(ref, wi);
    f3 p0, p1, p2;
    tri_verts(S, l.primSlot, &p0, &p1, &p2);
    float t, b0, b1, b2;
    if (!tri_test(p0, p1, p2, ray, &t, &b0, &b1, &b2)) return 0;
    Isect li;
    int flags = __float_as_int(S.triVerts[3 * (size_t)l.primSlot].w);
    triangle_si(S, l.primSlot, ray, b0, b1, b2, flags, &li);
    float area = (float)(0.5 * (double)len(cross(p1 - p0, p2 - p0)));
    float pdf = len2(ref.p - li.p) / (absdot(li.n, -wi) * area);
    if (is_inf(pdf)) pdf = 0.f;
    return pdf;
}
__device__ __forceinline__ rgb si_Le(const DeviceScene& S, const Isect& si, f3 w) {   // Interaction.cpp:116-119
    int al = S.primInfo[si.slot].z;
    return al >= 0 ? area_L(S.lights[al], si.n, w) : sp(0.f);
}

// ---------------------------------------------------------------- media (Media/*.cpp)
PBR_HD float phase_hg(float cosTheta, float g) {   // Medium.h:24-27
    float denom = 1 + g * g + 2 * g * cosTheta;
    return kInv4Pi * (1 - g * g) / (denom * sqrtf(denom));
}
PBR_HD float hg_sample(float g, f3 wo, f3* wi, float u0, float u1) {   // Medium.cpp:9-26
    float cosTheta;
    if ((double)fabsf(g) < 1e-3) cosTheta = 1 - 2 * u0;
    else {
        float sq = (1 - g * g) / (1 + g - 2 * g * u0);
        cosTheta = -(1 + g * g - sq * sq) / (2 * g);
    }
    float sinTheta = sqrtf(mx((float)0, 1 - cosTheta * cosTheta));
    float phi = 2 * kPi * u1;
    f3 v1, v2;
    coordinate_system(wo, &v1, &v2);
    *wi = spherical_direction(sinTheta, cosTheta, phi, v1, v2, wo);
    return phase_hg(cosTheta, g);
}
__device__ __forceinline__ rgb medium_tr(const DeviceScene& S, int m, const Ray& ray) {   // HomogeneousMedium.cpp:10-12
    const float* md = S.media + 10 * m;
    return exp_s(sp3(-md[6], -md[7], -md[8]) * mn(ray.tMax * len(ray.d), kMaxFloat));
}

}  // namespace pbr
