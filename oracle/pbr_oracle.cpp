// pbr_oracle.cpp — TEST INFRASTRUCTURE ONLY (the parity checker; never linked by the product).
// CPU restatement of the reference's per-pixel integrator loop. Each function cites the reference
// file:line it follows. See pbr_oracle.h for the pinning story and the documented deviations.
#include "pbr_oracle.h"
#include "orc_core.h"
#include "orc_envmap.h"

#include <chrono>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

std::vector<int> first_primes(int n) {
    std::vector<int> p;
    for (int c = 2; (int)p.size() < n; ++c) {
        bool ok = true;
        for (int q : p) { if (q * q > c) break; if (c % q == 0) { ok = false; break; } }
        if (ok) p.push_back(c);
    }
    return p;
}

// BxDFType (Material/Reflection.h:60-68)
enum { BSDF_REFLECTION = 1, BSDF_TRANSMISSION = 2, BSDF_DIFFUSE = 4, BSDF_GLOSSY = 8, BSDF_SPECULAR = 16, BSDF_ALL = 31 };

// per-thread instrumentation for the roofline bytes model
struct Counters { uint64_t rays = 0, nodes = 0, prims = 0, shading = 0; };
static thread_local Counters* tl_counters = nullptr;

// ---------------------------------------------------------------- scene
struct Mesh {
    std::vector<V3> p;          // world space (Shape/Triangle.cpp:26-28)
    std::vector<int> idx;
    std::vector<P2> uv;
    bool hasUV = false;
    bool reverse = false, swaps = false;
};
struct SphereS {
    Xform o2w, w2o;
    float radius;
    bool reverse = false, swaps = false;
};
struct Prim {
    int shape, tri;             // tri < 0 → sphere
    int material, areaLight;
    int medIn, medOut;
};
struct Light {
    int type;
    Spec I, Lemit;
    V3 pLight;
    int prim;                   // area light shape primitive
    bool twoSided;
    float area;
    // skybox
    V3 worldCenter;
    float worldRadius;
    int w = 0, h = 0, comps = 0;
    std::vector<float> data;
    int medIn = -1, medOut = -1;
    // InfiniteAreaLight (Light/InfiniteAreaLight.h:11-45); built by Preprocess once the BVH exists
    Xform l2w, w2l;
    std::shared_ptr<MIPMapS> Lmap;
    std::shared_ptr<Distribution2D> distribution;
};
struct Medium { Spec sigma_a, sigma_s, sigma_t; float g; };
struct MaterialO { pbr_material_desc d; float ua, va, ra; };   // pre-remapped roughness
// ImageTexture<RGBSpectrum, Spectrum> / <float, float> with its UVMapping2D (Texture/ImageTexture.h)
struct TextureO {
    bool isFloat = false, trilinear = false;
    float su = 1, sv = 1, du = 0, dv = 0;
    std::shared_ptr<MIPMapT<Spec>> ms;
    std::shared_ptr<MIPMapT<float>> mf;
};

}  // namespace orc

// keep LinearBVHNode byte-identical to the reference layout
struct OrcLinearBVHNode {
    float pMin[3], pMax[3];
    int32_t offset;             // primitivesOffset | secondChildOffset
    uint16_t nPrimitives;
    uint8_t axis;
    uint8_t pad[1];
};
static_assert(sizeof(OrcLinearBVHNode) == 32, "LinearBVHNode must be 32 bytes");

namespace orc {

struct Scene {
    std::vector<Mesh> meshes;       // indexed by shape id (empty for spheres)
    std::vector<SphereS> spheres;   // indexed by shape id
    std::vector<int> shapeType;
    std::vector<Prim> prims;        // BVH-ordered after build
    std::vector<int> primIds;       // original prims-vector index per ordered slot
    std::vector<OrcLinearBVHNode> nodes;
    std::vector<MaterialO> materials;
    std::vector<TextureO> textures;
    std::vector<Light> lights;
    std::vector<int> infinite;
    std::vector<Medium> media;
    std::vector<int> primOfOriginal; // original index → ordered slot
};

// ---------------------------------------------------------------- bounds of a primitive
static Bounds3 PrimBound(const Scene& s, const Prim& pr) {
    if (pr.tri >= 0) {   // Shape/Triangle.cpp:55-62
        const Mesh& m = s.meshes[pr.shape];
        V3 p0 = m.p[m.idx[3 * pr.tri]], p1 = m.p[m.idx[3 * pr.tri + 1]], p2 = m.p[m.idx[3 * pr.tri + 2]];
        return Union(Bounds3(p0, p1), p2);
    }
    // Shape::WorldBound (Shape/Shape.cpp:14) → Transform::operator()(Bounds3f) (Transform.cpp:241-252)
    const SphereS& sp = s.spheres[pr.shape];
    float r = sp.radius;
    V3 lo(-r, -r, -r), hi(r, r, r);
    const Xform& M = sp.o2w;
    Bounds3 ret;
    ret.pMin = ret.pMax = M.point(V3(lo.x, lo.y, lo.z));
    ret = Union(ret, M.point(V3(hi.x, lo.y, lo.z)));
    ret = Union(ret, M.point(V3(lo.x, hi.y, lo.z)));
    ret = Union(ret, M.point(V3(lo.x, lo.y, hi.z)));
    ret = Union(ret, M.point(V3(lo.x, hi.y, hi.z)));
    ret = Union(ret, M.point(V3(hi.x, hi.y, lo.z)));
    ret = Union(ret, M.point(V3(hi.x, lo.y, hi.z)));
    ret = Union(ret, M.point(V3(hi.x, hi.y, hi.z)));
    return ret;
}

// ---------------------------------------------------------------- BVH build (BVHAccel.cpp:57-283)
struct PrimInfo {
    size_t primitiveNumber;
    Bounds3 bounds;
    V3 centroid;
};
struct BuildNode {
    Bounds3 bounds;
    BuildNode* children[2] = {nullptr, nullptr};
    int splitAxis = 0, firstPrimOffset = 0, nPrimitives = 0;
};
struct BucketInfo { int count = 0; Bounds3 bounds; };

struct Builder {
    const std::vector<Prim>& in;
    int maxPrimsInNode;
    int splitMethod;                 // BVHAccel::SplitMethod (BVHAccel.h:18)
    std::vector<std::unique_ptr<BuildNode>> pool;
    std::vector<int> ordered;
    Builder(const std::vector<Prim>& p, int m, int split) : in(p), maxPrimsInNode(std::min(255, m)), splitMethod(split) {}

    BuildNode* leaf(BuildNode* node, std::vector<PrimInfo>& pi, int start, int end, const Bounds3& bounds) {
        int first = (int)ordered.size();
        for (int i = start; i < end; ++i) ordered.push_back((int)pi[i].primitiveNumber);
        node->firstPrimOffset = first;
        node->nPrimitives = end - start;
        node->bounds = bounds;
        return node;
    }
    BuildNode* build(std::vector<PrimInfo>& pi, int start, int end, int* totalNodes) {
        pool.emplace_back(new BuildNode);
        BuildNode* node = pool.back().get();
        (*totalNodes)++;
        Bounds3 bounds;
        for (int i = start; i < end; ++i) bounds = Union(bounds, pi[i].bounds);
        int nPrimitives = end - start;
        if (nPrimitives == 1) return leaf(node, pi, start, end, bounds);
        Bounds3 centroidBounds;
        for (int i = start; i < end; ++i) centroidBounds = Union(centroidBounds, pi[i].centroid);
        int dim = centroidBounds.MaximumExtent();
        int mid = (start + end) / 2;
        if (centroidBounds.pMax[dim] == centroidBounds.pMin[dim]) return leaf(node, pi, start, end, bounds);
        auto cmp = [dim](const PrimInfo& a, const PrimInfo& b) { return a.centroid[dim] < b.centroid[dim]; };
        bool done = false;
        if (splitMethod == PBR_SPLIT_MIDDLE) {   // BVHAccel.cpp:136-148
            float pmid = (centroidBounds.pMin[dim] + centroidBounds.pMax[dim]) / 2;
            PrimInfo* midPtr = std::partition(&pi[start], &pi[end - 1] + 1, [dim, pmid](const PrimInfo& p) { return p.centroid[dim] < pmid; });
            mid = midPtr - &pi[0];
            done = mid != start && mid != end;
        }
        if (!done && (splitMethod == PBR_SPLIT_MIDDLE || splitMethod == PBR_SPLIT_EQUAL_COUNTS)) {   // :149-158
            mid = (start + end) / 2;
            std::nth_element(&pi[start], &pi[mid], &pi[end - 1] + 1, cmp);
            done = true;
        }
        if (done) {
        } else if (nPrimitives <= 2) {
            mid = (start + end) / 2;
            std::nth_element(&pi[start], &pi[mid], &pi[end - 1] + 1,
                             [dim](const PrimInfo& a, const PrimInfo& b) { return a.centroid[dim] < b.centroid[dim]; });
        } else {
            constexpr int nBuckets = 12;
            BucketInfo buckets[nBuckets];
            for (int i = start; i < end; ++i) {
                int b = nBuckets * centroidBounds.Offset(pi[i].centroid)[dim];
                if (b == nBuckets) b = nBuckets - 1;
                buckets[b].count++;
                buckets[b].bounds = Union(buckets[b].bounds, pi[i].bounds);
            }
            float cost[nBuckets - 1];
            for (int i = 0; i < nBuckets - 1; ++i) {
                Bounds3 b0, b1;
                int count0 = 0, count1 = 0;
                for (int j = 0; j <= i; ++j) { b0 = Union(b0, buckets[j].bounds); count0 += buckets[j].count; }
                for (int j = i + 1; j < nBuckets; ++j) { b1 = Union(b1, buckets[j].bounds); count1 += buckets[j].count; }
                cost[i] = 1 + (count0 * b0.SurfaceArea() + count1 * b1.SurfaceArea()) / bounds.SurfaceArea();
            }
            float minCost = cost[0];
            int minCostSplitBucket = 0;
            for (int i = 1; i < nBuckets - 1; ++i)
                if (cost[i] < minCost) { minCost = cost[i]; minCostSplitBucket = i; }
            float leafCost = nPrimitives;
            if (nPrimitives > maxPrimsInNode || minCost < leafCost) {
                Bounds3 cb = centroidBounds;
                PrimInfo* pmid = std::partition(&pi[start], &pi[end - 1] + 1, [=](const PrimInfo& p) {
                    int b = nBuckets * cb.Offset(p.centroid)[dim];
                    if (b == nBuckets) b = nBuckets - 1;
                    return b <= minCostSplitBucket;
                });
                mid = pmid - &pi[0];
            } else {
                return leaf(node, pi, start, end, bounds);
            }
        }
        // InitInterior(dim, recursiveBuild(start, mid), recursiveBuild(mid, end)) (BVHAccel.cpp:250-254):
        // C++ leaves the order of the two argument evaluations open; GCC (and MSVC) evaluate them
        // right to left, so the SECOND child's subtree is built — and its primitives appended to
        // orderedPrims — first.  Pinned by the reference-built node array (ref_fixtures.json).
        BuildNode* c1 = build(pi, mid, end, totalNodes);
        BuildNode* c0 = build(pi, start, mid, totalNodes);
        node->children[0] = c0;
        node->children[1] = c1;
        node->bounds = Union(c0->bounds, c1->bounds);
        node->splitAxis = dim;
        node->nPrimitives = 0;
        return node;
    }
    int flatten(BuildNode* node, int* offset, std::vector<OrcLinearBVHNode>& nodes) {   // BVHAccel.cpp:261-283
        OrcLinearBVHNode* ln = &nodes[*offset];
        std::memset(ln, 0, sizeof(*ln));
        ln->pMin[0] = node->bounds.pMin.x; ln->pMin[1] = node->bounds.pMin.y; ln->pMin[2] = node->bounds.pMin.z;
        ln->pMax[0] = node->bounds.pMax.x; ln->pMax[1] = node->bounds.pMax.y; ln->pMax[2] = node->bounds.pMax.z;
        int myOffset = (*offset)++;
        if (node->nPrimitives > 0) {
            ln->offset = node->firstPrimOffset;
            ln->nPrimitives = (uint16_t)node->nPrimitives;
        } else {
            ln->axis = (uint8_t)node->splitAxis;
            ln->nPrimitives = 0;
            flatten(node->children[0], offset, nodes);
            int second = flatten(node->children[1], offset, nodes);
            nodes[myOffset].offset = second;
        }
        return myOffset;
    }
};

static void BuildBVH(Scene& s, std::vector<Prim>& prims, int maxPrimsInNode, int splitMethod) {
    if (prims.empty()) return;
    std::vector<PrimInfo> pi(prims.size());
    for (size_t i = 0; i < prims.size(); ++i) {
        Bounds3 b = PrimBound(s, prims[i]);
        pi[i].primitiveNumber = i;
        pi[i].bounds = b;
        pi[i].centroid = .5f * b.pMin + .5f * b.pMax;
    }
    Builder bld(prims, maxPrimsInNode, splitMethod);
    int total = 0;
    BuildNode* root = bld.build(pi, 0, (int)prims.size(), &total);
    s.nodes.assign(total, OrcLinearBVHNode());
    int off = 0;
    bld.flatten(root, &off, s.nodes);
    s.primIds = bld.ordered;
    s.prims.resize(prims.size());
    s.primOfOriginal.assign(prims.size(), -1);
    for (size_t i = 0; i < bld.ordered.size(); ++i) {
        s.prims[i] = prims[bld.ordered[i]];
        s.primOfOriginal[bld.ordered[i]] = (int)i;
    }
}

// ---------------------------------------------------------------- surface interaction
struct Interaction {
    V3 p, pError, wo, n;
    int medIn = -1, medOut = -1;
    bool IsSurface() const { return !IsZero(n); }   // Core/Interaction.h:25
    int GetMedium(V3 w) const { return Dot(w, n) > 0 ? medOut : medIn; }   // Interaction.h:48-50
    Ray SpawnRay(V3 d) const {   // Interaction.h:28-31
        V3 o = OffsetRayOrigin(p, pError, n, d);
        return Ray(o, d, Infinity, GetMedium(d));
    }
    Ray SpawnRayTo(const Interaction& it) const {   // Interaction.h:38-44
        V3 origin = OffsetRayOrigin(p, pError, n, it.p - p);
        V3 target = OffsetRayOrigin(it.p, it.pError, it.n, origin - it.p);
        V3 d = target - origin;
        return Ray(origin, d, 1 - ShadowEpsilon, GetMedium(d));
    }
};
struct SurfaceInteraction : Interaction {
    int prim = -1;          // ordered primitive slot
    P2 uv;                  // Triangle.cpp:170 uvHit
    V3 dpdu;                // shading.dpdu (== dpdu without shading normals)
    V3 sn;                  // shading.n
};
struct MediumInteraction : Interaction { int medium = -1; float g = 0; bool valid = false; };

// ---------------------------------------------------------------- shapes
// Shape/Triangle.cpp:62-260 (intersection part); returns b0,b1,b2,t on hit
static bool TriangleTest(V3 p0, V3 p1, V3 p2, const Ray& ray, float* tOut, float* b0o, float* b1o, float* b2o) {
    V3 p0t = p0 - ray.o, p1t = p1 - ray.o, p2t = p2 - ray.o;
    int kz = MaxDimension(Abs(ray.d));
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    V3 d = Permute(ray.d, kx, ky, kz);
    p0t = Permute(p0t, kx, ky, kz); p1t = Permute(p1t, kx, ky, kz); p2t = Permute(p2t, kx, ky, kz);
    float Sx = -d.x / d.z, Sy = -d.y / d.z, Sz = 1.f / d.z;
    p0t.x += Sx * p0t.z; p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z; p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z; p2t.y += Sy * p2t.z;
    float e0 = p1t.x * p2t.y - p1t.y * p2t.x;
    float e1 = p2t.x * p0t.y - p2t.y * p0t.x;
    float e2 = p0t.x * p1t.y - p0t.y * p1t.x;
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {   // double fallback (Triangle.cpp:98-109)
        double p2txp1ty = (double)p2t.x * (double)p1t.y, p2typ1tx = (double)p2t.y * (double)p1t.x;
        e0 = (float)(p2typ1tx - p2txp1ty);
        double p0txp2ty = (double)p0t.x * (double)p2t.y, p0typ2tx = (double)p0t.y * (double)p2t.x;
        e1 = (float)(p0typ2tx - p0txp2ty);
        double p1txp0ty = (double)p1t.x * (double)p0t.y, p1typ0tx = (double)p1t.y * (double)p0t.x;
        e2 = (float)(p1typ0tx - p1txp0ty);
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
    float maxZt = MaxComponent(Abs(V3(p0t.z, p1t.z, p2t.z)));
    float deltaZ = gamma(3) * maxZt;
    float maxXt = MaxComponent(Abs(V3(p0t.x, p1t.x, p2t.x)));
    float maxYt = MaxComponent(Abs(V3(p0t.y, p1t.y, p2t.y)));
    float deltaX = gamma(5) * (maxXt + maxZt);
    float deltaY = gamma(5) * (maxYt + maxZt);
    float deltaE = 2 * (gamma(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    float maxE = MaxComponent(Abs(V3(e0, e1, e2)));
    float deltaT = 3 * (gamma(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * std::abs(invDet);
    if (t <= deltaT) return false;
    *tOut = t; *b0o = b0; *b1o = b1; *b2o = b2;
    return true;
}

// Triangle::Intersect SI construction (Triangle.cpp:148-246); no shading normals
static void TriangleSI(const Mesh& m, int tri, const Ray& ray, float b0, float b1, float b2, SurfaceInteraction* si) {
    V3 p0 = m.p[m.idx[3 * tri]], p1 = m.p[m.idx[3 * tri + 1]], p2 = m.p[m.idx[3 * tri + 2]];
    P2 uv[3];
    if (m.hasUV) { uv[0] = m.uv[m.idx[3 * tri]]; uv[1] = m.uv[m.idx[3 * tri + 1]]; uv[2] = m.uv[m.idx[3 * tri + 2]]; }
    else { uv[0] = P2(0, 0); uv[1] = P2(1, 0); uv[2] = P2(1, 1); }
    P2 duv02(uv[0].x - uv[2].x, uv[0].y - uv[2].y), duv12(uv[1].x - uv[2].x, uv[1].y - uv[2].y);
    V3 dp02 = p0 - p2, dp12 = p1 - p2;
    float determinant = duv02.x * duv12.y - duv02.y * duv12.x;
    bool degenerateUV = std::abs(determinant) < 1e-8;
    V3 dpdu(0, 0, 0);
    if (!degenerateUV) {
        float invdet = 1 / determinant;
        dpdu = (duv12.y * dp02 - duv02.y * dp12) * invdet;
    }
    float xAbsSum = (std::abs(b0 * p0.x) + std::abs(b1 * p1.x) + std::abs(b2 * p2.x));
    float yAbsSum = (std::abs(b0 * p0.y) + std::abs(b1 * p1.y) + std::abs(b2 * p2.y));
    float zAbsSum = (std::abs(b0 * p0.z) + std::abs(b1 * p1.z) + std::abs(b2 * p2.z));
    si->pError = gamma(7) * V3(xAbsSum, yAbsSum, zAbsSum);
    si->p = b0 * p0 + b1 * p1 + b2 * p2;
    si->wo = Normalize(-ray.d);                              // Interaction ctor normalizes wo (Interaction.h:15-19)
    V3 n = Normalize(Cross(dp02, dp12));
    if (m.reverse ^ m.swaps) n = -n;
    si->n = n; si->sn = n;
    si->dpdu = dpdu;
    si->uv = P2(b0 * uv[0].x + b1 * uv[1].x + b2 * uv[2].x, b0 * uv[0].y + b1 * uv[1].y + b2 * uv[2].y);   // b0*uv0 + b1*uv1 + b2*uv2
}

// Sphere: the reference's is a stub (F2). This is the pbrt-v3 full-sphere algorithm with the
// quadratic solved in double; parity for spheres is between this restatement and the device only.
static bool SphereTest(const SphereS& sp, const Ray& r, float* tOut) {
    V3 o = sp.w2o.point(r.o), d = sp.w2o.vector(r.d);
    double ox = o.x, oy = o.y, oz = o.z, dx = d.x, dy = d.y, dz = d.z, rad = sp.radius;
    double a = dx * dx + dy * dy + dz * dz;
    double b = 2 * (dx * ox + dy * oy + dz * oz);
    double c = ox * ox + oy * oy + oz * oz - rad * rad;
    double disc = b * b - 4 * a * c;
    if (disc < 0) return false;
    double rd = std::sqrt(disc);
    double q = (b < 0) ? -0.5 * (b - rd) : -0.5 * (b + rd);
    double t0 = q / a, t1 = c / q;
    if (t0 > t1) std::swap(t0, t1);
    float f0 = (float)t0, f1 = (float)t1;
    if (f0 > r.tMax || f1 <= 0) return false;
    float t = f0;
    if (t <= 0) { t = f1; if (t > r.tMax) return false; }
    *tOut = t;
    return true;
}
static void SphereSI(const SphereS& sp, const Ray& r, float t, SurfaceInteraction* si) {
    V3 o = sp.w2o.point(r.o), d = sp.w2o.vector(r.d);
    V3 pHit = o + d * t;
    pHit = pHit * (sp.radius / Length(pHit));
    if (pHit.x == 0 && pHit.y == 0) pHit.x = 1e-5f * sp.radius;
    float phi = t_atan2(pHit.y, pHit.x);
    if (phi < 0) phi += 2 * Pi;
    const float phiMax = 2 * Pi;
    float zRadius = std::sqrt(pHit.x * pHit.x + pHit.y * pHit.y);
    float invZRadius = 1 / zRadius;
    float cosPhi = pHit.x * invZRadius, sinPhi = pHit.y * invZRadius;
    float cosTheta = Clampf(pHit.z / sp.radius, -1, 1);
    float sinTheta = std::sqrt(fmax_((float)0, 1 - cosTheta * cosTheta));
    V3 dpdu(-phiMax * pHit.y, phiMax * pHit.x, 0);
    V3 dpdv = (-Pi) * V3(pHit.z * cosPhi, pHit.z * sinPhi, -sp.radius * sinTheta);
    V3 pw = sp.o2w.point(pHit);
    V3 pErrObj = gamma(5) * Abs(pHit);
    si->pError = gamma(6) * (Abs(pw) + pErrObj);
    si->p = pw;
    si->wo = Normalize(-r.d);
    V3 dpduW = sp.o2w.vector(dpdu), dpdvW = sp.o2w.vector(dpdv);
    V3 n = Normalize(Cross(dpduW, dpdvW));
    if (sp.reverse ^ sp.swaps) n = -n;
    si->n = n; si->sn = n;
    si->dpdu = dpduW;
}

// ---------------------------------------------------------------- traversal (BVHAccel.cpp:285-366)
static bool PrimIntersect(const Scene& s, int slot, const Ray& ray, SurfaceInteraction* si, bool* hitRecorded,
                          float* bb) {
    const Prim& pr = s.prims[slot];
    if (tl_counters) tl_counters->prims++;
    float t;
    if (pr.tri >= 0) {
        const Mesh& m = s.meshes[pr.shape];
        float b0, b1, b2;
        if (!TriangleTest(m.p[m.idx[3 * pr.tri]], m.p[m.idx[3 * pr.tri + 1]], m.p[m.idx[3 * pr.tri + 2]], ray, &t, &b0, &b1, &b2))
            return false;
        bb[0] = b0; bb[1] = b1; bb[2] = b2;
    } else {
        if (!SphereTest(s.spheres[pr.shape], ray, &t)) return false;
    }
    ray.tMax = t;                                       // GeometricPrimitive::Intersect (Primitive.cpp:24-26)
    si->prim = slot;
    *hitRecorded = true;
    return true;
}

static bool Intersect(const Scene& s, const Ray& ray, SurfaceInteraction* isect) {
    if (tl_counters) tl_counters->rays++;
    if (s.nodes.empty()) return false;
    bool hit = false;
    V3 invDir(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
    int dirIsNeg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    int toVisitOffset = 0, currentNodeIndex = 0;
    int nodesToVisit[64];
    int lastSlot = -1;
    float lastB[3] = {0, 0, 0};
    Ray rayAtHit;
    while (true) {
        const OrcLinearBVHNode* node = &s.nodes[currentNodeIndex];
        if (tl_counters) tl_counters->nodes++;
        Bounds3 b;
        b.pMin = V3(node->pMin[0], node->pMin[1], node->pMin[2]);
        b.pMax = V3(node->pMax[0], node->pMax[1], node->pMax[2]);
        if (BoundsIntersectP(b, ray, invDir, dirIsNeg)) {
            if (node->nPrimitives > 0) {
                for (int i = 0; i < node->nPrimitives; ++i) {
                    bool rec = false;
                    float bb[3];
                    if (PrimIntersect(s, node->offset + i, ray, isect, &rec, bb)) {
                        hit = true;
                        lastSlot = node->offset + i;
                        lastB[0] = bb[0]; lastB[1] = bb[1]; lastB[2] = bb[2];
                    }
                }
                if (toVisitOffset == 0) break;
                currentNodeIndex = nodesToVisit[--toVisitOffset];
            } else {
                if (dirIsNeg[node->axis]) {
                    nodesToVisit[toVisitOffset++] = currentNodeIndex + 1;
                    currentNodeIndex = node->offset;
                } else {
                    nodesToVisit[toVisitOffset++] = node->offset;
                    currentNodeIndex = currentNodeIndex + 1;
                }
            }
        } else {
            if (toVisitOffset == 0) break;
            currentNodeIndex = nodesToVisit[--toVisitOffset];
        }
    }
    if (hit) {
        // The reference builds the SurfaceInteraction inside every accepted test; only the last
        // accepted primitive's survives, so building it once here is equivalent.
        const Prim& pr = s.prims[lastSlot];
        if (pr.tri >= 0) TriangleSI(s.meshes[pr.shape], pr.tri, ray, lastB[0], lastB[1], lastB[2], isect);
        else SphereSI(s.spheres[pr.shape], ray, ray.tMax, isect);
        isect->prim = lastSlot;
        // MediumInterface (Primitive.cpp:30-34)
        if (pr.medIn != pr.medOut) { isect->medIn = pr.medIn; isect->medOut = pr.medOut; }
        else { isect->medIn = ray.medium; isect->medOut = ray.medium; }
    }
    return hit;
}

static bool IntersectP(const Scene& s, const Ray& ray) {
    if (tl_counters) tl_counters->rays++;
    if (s.nodes.empty()) return false;
    V3 invDir(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
    int dirIsNeg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    int nodesToVisit[64];
    int toVisitOffset = 0, currentNodeIndex = 0;
    while (true) {
        const OrcLinearBVHNode* node = &s.nodes[currentNodeIndex];
        if (tl_counters) tl_counters->nodes++;
        Bounds3 b;
        b.pMin = V3(node->pMin[0], node->pMin[1], node->pMin[2]);
        b.pMax = V3(node->pMax[0], node->pMax[1], node->pMax[2]);
        if (BoundsIntersectP(b, ray, invDir, dirIsNeg)) {
            if (node->nPrimitives > 0) {
                for (int i = 0; i < node->nPrimitives; ++i) {
                    const Prim& pr = s.prims[node->offset + i];
                    if (tl_counters) tl_counters->prims++;
                    float t, b0, b1, b2;
                    bool h;
                    if (pr.tri >= 0) {
                        const Mesh& m = s.meshes[pr.shape];
                        h = TriangleTest(m.p[m.idx[3 * pr.tri]], m.p[m.idx[3 * pr.tri + 1]], m.p[m.idx[3 * pr.tri + 2]], ray, &t, &b0, &b1, &b2);
                    } else {
                        h = SphereTest(s.spheres[pr.shape], ray, &t);
                    }
                    if (h) return true;
                }
                if (toVisitOffset == 0) break;
                currentNodeIndex = nodesToVisit[--toVisitOffset];
            } else {
                if (dirIsNeg[node->axis]) {
                    nodesToVisit[toVisitOffset++] = currentNodeIndex + 1;
                    currentNodeIndex = node->offset;
                } else {
                    nodesToVisit[toVisitOffset++] = node->offset;
                    currentNodeIndex = currentNodeIndex + 1;
                }
            }
        } else {
            if (toVisitOffset == 0) break;
            currentNodeIndex = nodesToVisit[--toVisitOffset];
        }
    }
    return false;
}

// ---------------------------------------------------------------- BSDF (Material/Reflection.*)
inline float CosTheta(V3 w) { return w.z; }
inline float Cos2Theta(V3 w) { return w.z * w.z; }
inline float AbsCosTheta(V3 w) { return std::abs(w.z); }
inline float Sin2Theta(V3 w) { return fmax_((float)0, (float)1 - Cos2Theta(w)); }
inline float SinTheta(V3 w) { return std::sqrt(Sin2Theta(w)); }
inline float TanTheta(V3 w) { return SinTheta(w) / CosTheta(w); }
inline float Tan2Theta(V3 w) { return Sin2Theta(w) / Cos2Theta(w); }
inline float CosPhi(V3 w) { float s = SinTheta(w); return (s == 0) ? 1 : Clampf(w.x / s, -1, 1); }
inline float SinPhi(V3 w) { float s = SinTheta(w); return (s == 0) ? 0 : Clampf(w.y / s, -1, 1); }
inline float Cos2Phi(V3 w) { return CosPhi(w) * CosPhi(w); }
inline float Sin2Phi(V3 w) { return SinPhi(w) * SinPhi(w); }
inline V3 Reflect(V3 wo, V3 n) { return -wo + 2 * Dot(wo, n) * n; }   // Reflection.h:43
inline bool Refract(V3 wi, V3 n, float eta, V3* wt) {   // Reflection.h:44-53
    float cosThetaI = Dot(n, wi);
    float sin2ThetaI = fmax_(float(0), float(1 - cosThetaI * cosThetaI));
    float sin2ThetaT = eta * eta * sin2ThetaI;
    if (sin2ThetaT >= 1) return false;
    float cosThetaT = std::sqrt(1 - sin2ThetaT);
    *wt = eta * -wi + (eta * cosThetaI - cosThetaT) * n;
    return true;
}
inline bool SameHemisphere(V3 w, V3 wp) { return w.z * wp.z > 0; }

// Fresnel.cpp:7-28
static float FrDielectric(float cosThetaI, float etaI, float etaT) {
    cosThetaI = Clampf(cosThetaI, -1, 1);
    bool entering = cosThetaI > 0.f;
    if (!entering) { std::swap(etaI, etaT); cosThetaI = std::abs(cosThetaI); }
    float sinThetaI = std::sqrt(fmax_((float)0, 1 - cosThetaI * cosThetaI));
    float sinThetaT = etaI / etaT * sinThetaI;
    if (sinThetaT >= 1) return 1;
    float cosThetaT = std::sqrt(fmax_((float)0, 1 - sinThetaT * sinThetaT));
    float Rparl = ((etaT * cosThetaI) - (etaI * cosThetaT)) / ((etaT * cosThetaI) + (etaI * cosThetaT));
    float Rperp = ((etaI * cosThetaI) - (etaT * cosThetaT)) / ((etaI * cosThetaI) + (etaT * cosThetaT));
    return (Rparl * Rparl + Rperp * Rperp) / 2;
}
// Fresnel.cpp:31-54
static Spec FrConductor(float cosThetaI, Spec etai, Spec etat, Spec k) {
    cosThetaI = Clampf(cosThetaI, -1, 1);
    Spec eta = etat / etai;
    Spec etak = k / etai;
    float cosThetaI2 = cosThetaI * cosThetaI;
    float sinThetaI2 = (float)(1. - (double)cosThetaI2);
    Spec eta2 = eta * eta;
    Spec etak2 = etak * etak;
    Spec t0 = eta2 - etak2 - Spec(sinThetaI2);
    Spec a2plusb2 = SqrtS(t0 * t0 + 4.f * eta2 * etak2);
    Spec t1 = a2plusb2 + Spec(cosThetaI2);
    Spec a = SqrtS(0.5f * (a2plusb2 + t0));
    Spec t2 = (float)2 * cosThetaI * a;
    Spec Rs = (t1 - t2) / (t1 + t2);
    Spec t3 = cosThetaI2 * a2plusb2 + Spec(sinThetaI2 * sinThetaI2);
    Spec t4 = t2 * sinThetaI2;
    Spec Rp = Rs * (t3 - t4) / (t3 + t4);
    return 0.5f * (Rp + Rs);   // the double 0.5 converts to the float overload
}

enum LobeKind { L_LAMBERT, L_OREN, L_SPEC_R, L_SPEC_T, L_FRESNEL_SPEC, L_MF_R, L_MF_T };
enum FresnelKind { FR_NOOP, FR_DIEL, FR_COND };
struct Lobe {
    int kind = 0, type = 0;
    Spec R, T;
    float A = 0, B = 0;               // Oren-Nayar
    float etaA = 1, etaB = 1;         // transmission / FresnelSpecular
    float ax = 0, ay = 0;             // Trowbridge-Reitz
    int fresnel = FR_NOOP;
    float fEtaI = 1, fEtaT = 1;       // FresnelDielectric
    Spec cEtaI, cEtaT, cK;            // FresnelConductor
};
static Spec FresnelEval(const Lobe& l, float cosI) {
    if (l.fresnel == FR_NOOP) return Spec(1.);
    if (l.fresnel == FR_DIEL) return Spec(FrDielectric(cosI, l.fEtaI, l.fEtaT));
    return FrConductor(std::abs(cosI), l.cEtaI, l.cEtaT, l.cK);
}
// Trowbridge-Reitz (Microfacet.cpp:116-292)
static float TR_D(const Lobe& l, V3 wh) {
    float tan2Theta = Tan2Theta(wh);
    if (std::isinf(tan2Theta)) return 0.;
    const float cos4Theta = Cos2Theta(wh) * Cos2Theta(wh);
    float e = (Cos2Phi(wh) / (l.ax * l.ax) + Sin2Phi(wh) / (l.ay * l.ay)) * tan2Theta;
    return 1 / (Pi * l.ax * l.ay * cos4Theta * (1 + e) * (1 + e));
}
static float TR_Lambda(const Lobe& l, V3 w) {
    float absTanTheta = std::abs(TanTheta(w));
    if (std::isinf(absTanTheta)) return 0.;
    float alpha = std::sqrt(Cos2Phi(w) * l.ax * l.ax + Sin2Phi(w) * l.ay * l.ay);
    float alpha2Tan2Theta = (alpha * absTanTheta) * (alpha * absTanTheta);
    return (-1 + std::sqrt(1.f + alpha2Tan2Theta)) / 2;
}
static float TR_G1(const Lobe& l, V3 w) { return 1 / (1 + TR_Lambda(l, w)); }
static float TR_G(const Lobe& l, V3 wo, V3 wi) { return 1 / (1 + TR_Lambda(l, wo) + TR_Lambda(l, wi)); }
static void TRSample11(float cosTheta, float U1, float U2, float* slope_x, float* slope_y) {
    if ((double)cosTheta > .9999) {
        // unqualified sqrt/cos/sin on floats resolve to the C double functions (Microfacet.cpp:193-196)
        float r = (float)std::sqrt((double)(U1 / (1 - U1)));
        float phi = (float)(6.28318530718 * (double)U2);
        *slope_x = (float)((double)r * std::cos((double)phi));
        *slope_y = (float)((double)r * std::sin((double)phi));
        return;
    }
    float sinTheta = std::sqrt(fmax_((float)0, (float)1 - cosTheta * cosTheta));
    float tanTheta = sinTheta / cosTheta;
    float a = 1 / tanTheta;
    float G1 = 2 / (1 + std::sqrt(1.f + 1.f / (a * a)));
    float A = 2 * U1 / G1 - 1;
    float tmp = 1.f / (A * A - 1.f);
    if (tmp > 1e10) tmp = 1e10;
    float B = tanTheta;
    float D = std::sqrt(fmax_(float(B * B * tmp * tmp - (A * A - B * B) * tmp), float(0)));
    float slope_x_1 = B * tmp - D;
    float slope_x_2 = B * tmp + D;
    *slope_x = (A < 0 || slope_x_2 > 1.f / tanTheta) ? slope_x_1 : slope_x_2;
    float S;
    if (U2 > 0.5f) { S = 1.f; U2 = 2.f * (U2 - .5f); }
    else { S = -1.f; U2 = 2.f * (.5f - U2); }
    float z = (U2 * (U2 * (U2 * 0.27385f - 0.73369f) + 0.46341f)) /
              (U2 * (U2 * (U2 * 0.093073f + 0.309420f) - 1.000000f) + 0.597999f);
    *slope_y = S * z * std::sqrt(1.f + *slope_x * *slope_x);
}
static V3 TRSample(V3 wi, float ax, float ay, float U1, float U2) {
    V3 wiStretched = Normalize(V3(ax * wi.x, ay * wi.y, wi.z));
    float slope_x, slope_y;
    TRSample11(CosTheta(wiStretched), U1, U2, &slope_x, &slope_y);
    float tmp = CosPhi(wiStretched) * slope_x - SinPhi(wiStretched) * slope_y;
    slope_y = SinPhi(wiStretched) * slope_x + CosPhi(wiStretched) * slope_y;
    slope_x = tmp;
    slope_x = ax * slope_x;
    slope_y = ay * slope_y;
    return Normalize(V3(-slope_x, -slope_y, 1.));
}
static V3 TR_Sample_wh(const Lobe& l, V3 wo, P2 u) {   // sampleVisibleArea = true (Microfacet.h:55-59)
    bool flip = wo.z < 0;
    V3 wh = TRSample(flip ? -wo : wo, l.ax, l.ay, u.x, u.y);
    if (flip) wh = -wh;
    return wh;
}
static float TR_Pdf(const Lobe& l, V3 wo, V3 wh) { return TR_D(l, wh) * TR_G1(l, wo) * AbsDot(wo, wh) / AbsCosTheta(wo); }

static Spec LobeF(const Lobe& l, V3 wo, V3 wi) {
    switch (l.kind) {
    case L_LAMBERT: return l.R * InvPi;   // Reflection.cpp:171-173
    case L_OREN: {                        // Reflection.cpp:176-199
        float sinThetaI = SinTheta(wi), sinThetaO = SinTheta(wo);
        float maxCos = 0;
        if ((double)sinThetaI > 1e-4 && (double)sinThetaO > 1e-4) {
            float sinPhiI = SinPhi(wi), cosPhiI = CosPhi(wi);
            float sinPhiO = SinPhi(wo), cosPhiO = CosPhi(wo);
            float dCos = cosPhiI * cosPhiO + sinPhiI * sinPhiO;
            maxCos = fmax_((float)0, dCos);
        }
        float sinAlpha, tanBeta;
        if (AbsCosTheta(wi) > AbsCosTheta(wo)) { sinAlpha = sinThetaO; tanBeta = sinThetaI / AbsCosTheta(wi); }
        else { sinAlpha = sinThetaI; tanBeta = sinThetaO / AbsCosTheta(wo); }
        return l.R * InvPi * (l.A + l.B * maxCos * sinAlpha * tanBeta);
    }
    case L_MF_R: {                        // Reflection.cpp:259-268
        float cosThetaO = AbsCosTheta(wo), cosThetaI = AbsCosTheta(wi);
        V3 wh = wi + wo;
        if (cosThetaI == 0 || cosThetaO == 0) return Spec(0.);
        if (wh.x == 0 && wh.y == 0 && wh.z == 0) return Spec(0.);
        wh = Normalize(wh);
        Spec F = FresnelEval(l, Dot(wi, Faceforward(wh, V3(0, 0, 1))));
        return l.R * TR_D(l, wh) * TR_G(l, wo, wi) * F / (4 * cosThetaI * cosThetaO);
    }
    case L_MF_T: {                        // Reflection.cpp:294-322
        if (SameHemisphere(wo, wi)) return Spec(0);
        float cosThetaO = CosTheta(wo), cosThetaI = CosTheta(wi);
        if (cosThetaI == 0 || cosThetaO == 0) return Spec(0);
        float eta = CosTheta(wo) > 0 ? (l.etaB / l.etaA) : (l.etaA / l.etaB);
        V3 wh = Normalize(wo + wi * eta);
        if (wh.z < 0) wh = -wh;
        if (Dot(wo, wh) * Dot(wi, wh) > 0) return Spec(0);
        Spec F(FrDielectric(Dot(wo, wh), l.etaA, l.etaB));
        float sqrtDenom = Dot(wo, wh) + eta * Dot(wi, wh);
        float factor = 1 / eta;                       // TransportMode::Radiance
        return (Spec(1.f) - F) * l.T *
               std::abs(TR_D(l, wh) * TR_G(l, wo, wi) * eta * eta * AbsDot(wi, wh) * AbsDot(wo, wh) * factor *
                        factor / (cosThetaI * cosThetaO * sqrtDenom * sqrtDenom));
    }
    default: return Spec(0.f);            // specular lobes have zero f
    }
}
static float LobePdf(const Lobe& l, V3 wo, V3 wi) {
    switch (l.kind) {
    case L_LAMBERT: case L_OREN:          // Reflection.cpp:50-53
        return SameHemisphere(wo, wi) ? AbsCosTheta(wi) * InvPi : 0;
    case L_MF_R: {                        // Reflection.cpp:285-291
        if (!SameHemisphere(wo, wi)) return 0;
        V3 wh = Normalize(wo + wi);
        return TR_Pdf(l, wo, wh) / (4 * Dot(wo, wh));
    }
    case L_MF_T: {                        // Reflection.cpp:337-347
        if (SameHemisphere(wo, wi)) return 0;
        float eta = CosTheta(wo) > 0 ? (l.etaB / l.etaA) : (l.etaA / l.etaB);
        V3 wh = Normalize(wo + wi * eta);
        if (Dot(wo, wh) * Dot(wi, wh) > 0) return 0;
        float sqrtDenom = Dot(wo, wh) + eta * Dot(wi, wh);
        float dwh_dwi = std::abs((eta * eta * Dot(wi, wh)) / (sqrtDenom * sqrtDenom));
        return TR_Pdf(l, wo, wh) * dwh_dwi;
    }
    default: return 0;
    }
}
// returns f; sets *wi, *pdf, may set *sampledType
static Spec LobeSample(const Lobe& l, V3 wo, V3* wi, P2 u, float* pdf, int* sampledType) {
    switch (l.kind) {
    case L_LAMBERT: case L_OREN: {        // BxDF::Sample_f (Reflection.cpp:7-13)
        *wi = CosineSampleHemisphere(u);
        if (wo.z < 0) wi->z *= -1;
        *pdf = LobePdf(l, wo, *wi);
        return LobeF(l, wo, *wi);
    }
    case L_SPEC_R: {                      // Reflection.cpp:204-209
        *wi = V3(-wo.x, -wo.y, wo.z);
        *pdf = 1;
        return FresnelEval(l, CosTheta(*wi)) * l.R / AbsCosTheta(*wi);
    }
    case L_SPEC_T: {                      // Reflection.cpp:212-229
        bool entering = CosTheta(wo) > 0;
        float etaI = entering ? l.etaA : l.etaB, etaT = entering ? l.etaB : l.etaA;
        if (!Refract(wo, Faceforward(V3(0, 0, 1), wo), etaI / etaT, wi)) return Spec(0);
        *pdf = 1;
        Spec ft = l.T * (Spec(1.) - Spec(FrDielectric(CosTheta(*wi), l.etaA, l.etaB)));
        ft *= (etaI * etaI) / (etaT * etaT);
        return ft / AbsCosTheta(*wi);
    }
    case L_FRESNEL_SPEC: {                // Reflection.cpp:232-256
        float F = FrDielectric(CosTheta(wo), l.etaA, l.etaB);
        if (u.x < F) {
            *wi = V3(-wo.x, -wo.y, wo.z);
            *sampledType = BSDF_SPECULAR | BSDF_REFLECTION;
            *pdf = F;
            return F * l.R / AbsCosTheta(*wi);
        } else {
            bool entering = CosTheta(wo) > 0;
            float etaI = entering ? l.etaA : l.etaB, etaT = entering ? l.etaB : l.etaA;
            if (!Refract(wo, Faceforward(V3(0, 0, 1), wo), etaI / etaT, wi)) return Spec(0);
            Spec ft = l.T * (1 - F);
            ft *= (etaI * etaI) / (etaT * etaT);
            *sampledType = BSDF_SPECULAR | BSDF_TRANSMISSION;
            *pdf = 1 - F;
            return ft / AbsCosTheta(*wi);
        }
    }
    case L_MF_R: {                        // Reflection.cpp:270-283
        if (wo.z == 0) return Spec(0.);
        V3 wh = TR_Sample_wh(l, wo, u);
        if (Dot(wo, wh) < 0) return Spec(0.);
        *wi = Reflect(wo, wh);
        if (!SameHemisphere(wo, *wi)) return Spec(0.f);
        *pdf = TR_Pdf(l, wo, wh) / (4 * Dot(wo, wh));
        return LobeF(l, wo, *wi);
    }
    case L_MF_T: {                        // Reflection.cpp:324-335
        if (wo.z == 0) return Spec(0.);
        V3 wh = TR_Sample_wh(l, wo, u);
        if (Dot(wo, wh) < 0) return Spec(0.);
        float eta = CosTheta(wo) > 0 ? (l.etaA / l.etaB) : (l.etaB / l.etaA);
        if (!Refract(wo, wh, eta, wi)) return Spec(0);
        *pdf = LobePdf(l, wo, *wi);
        return LobeF(l, wo, *wi);
    }
    }
    return Spec(0);
}

struct BSDF {   // Reflection.h:101-149
    float eta = 1;
    V3 ns, ng, ss, ts;
    int n = 0;
    Lobe lobes[2];
    bool valid = false;
    void Add(const Lobe& l) { lobes[n++] = l; }
    V3 WorldToLocal(V3 v) const { return V3(Dot(v, ss), Dot(v, ts), Dot(v, ns)); }
    V3 LocalToWorld(V3 v) const {
        return V3(ss.x * v.x + ts.x * v.y + ns.x * v.z, ss.y * v.x + ts.y * v.y + ns.y * v.z,
                  ss.z * v.x + ts.z * v.y + ns.z * v.z);
    }
    static bool Matches(const Lobe& l, int t) { return (l.type & t) == l.type; }
    int NumComponents(int flags) const { int k = 0; for (int i = 0; i < n; ++i) if (Matches(lobes[i], flags)) ++k; return k; }
    Spec f(V3 woW, V3 wiW, int flags = BSDF_ALL) const {   // Reflection.cpp:56-71
        V3 wi = WorldToLocal(wiW), wo = WorldToLocal(woW);
        if (wo.z == 0) return Spec(0.);
        bool reflect = Dot(wiW, ng) * Dot(woW, ng) > 0;
        Spec r(0.f);
        for (int i = 0; i < n; ++i)
            if (Matches(lobes[i], flags) && ((reflect && (lobes[i].type & BSDF_REFLECTION)) ||
                                            (!reflect && (lobes[i].type & BSDF_TRANSMISSION))))
                r += LobeF(lobes[i], wo, wi);
        return r;
    }
    float Pdf(V3 woW, V3 wiW, int flags = BSDF_ALL) const {   // Reflection.cpp:92-106
        if (n == 0) return 0.f;
        V3 wo = WorldToLocal(woW), wi = WorldToLocal(wiW);
        if (wo.z == 0) return 0.;
        float pdf = 0.f;
        int matching = 0;
        for (int i = 0; i < n; ++i)
            if (Matches(lobes[i], flags)) { ++matching; pdf += LobePdf(lobes[i], wo, wi); }
        return matching > 0 ? pdf / matching : 0.f;
    }
    // Reflection.cpp:108-164. *pdf is left untouched on the wo.z == 0 early-out, as in the reference.
    Spec Sample_f(V3 woW, V3* wiW, P2 u, float* pdf, int type, int* sampledType) const {
        int matchingComps = NumComponents(type);
        if (matchingComps == 0) { *pdf = 0; if (sampledType) *sampledType = 0; return Spec(0); }
        int comp = std::min((int)std::floor(u.x * matchingComps), matchingComps - 1);
        int chosen = -1, count = comp;
        for (int i = 0; i < n; ++i)
            if (Matches(lobes[i], type) && count-- == 0) { chosen = i; break; }
        const Lobe& bx = lobes[chosen];
        P2 uRemapped(fmin_(u.x * matchingComps - comp, OneMinusEpsilon), u.y);
        V3 wi, wo = WorldToLocal(woW);
        if (wo.z == 0) return Spec(0.);
        *pdf = 0;
        int st = bx.type;
        Spec f = LobeSample(bx, wo, &wi, uRemapped, pdf, &st);
        if (sampledType) *sampledType = st;
        if (*pdf == 0) { if (sampledType) *sampledType = 0; return Spec(0); }
        *wiW = LocalToWorld(wi);
        if (!(bx.type & BSDF_SPECULAR) && matchingComps > 1)
            for (int i = 0; i < n; ++i)
                if (i != chosen && Matches(lobes[i], type)) *pdf += LobePdf(lobes[i], wo, wi);
        if (matchingComps > 1) *pdf /= matchingComps;
        if (!(bx.type & BSDF_SPECULAR)) {
            bool reflect = Dot(*wiW, ng) * Dot(woW, ng) > 0;
            f = Spec(0.);
            for (int i = 0; i < n; ++i)
                if (Matches(lobes[i], type) && ((reflect && (lobes[i].type & BSDF_REFLECTION)) ||
                                               (!reflect && (lobes[i].type & BSDF_TRANSMISSION))))
                    f += LobeF(lobes[i], wo, wi);
        }
        return f;
    }
};

static float RoughnessToAlpha(float roughness) {   // Microfacet.h:78-83
    roughness = fmax_(roughness, (float)1e-3);
    float x = t_log(roughness);
    return 1.62142f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x + 0.000640711f * x * x * x * x;
}
static Lobe MakeTR(Lobe l, float ax, float ay) {   // TrowbridgeReitzDistribution ctor (Microfacet.h:62-66)
    l.ax = fmax_(float(0.001), ax);
    l.ay = fmax_(float(0.001), ay);
    return l;
}
static Spec S3(const float* v) { return Spec(v[0], v[1], v[2]); }

// Texture<Spectrum/float>::Evaluate of a material slot: ConstantTexture (the descriptor's value) or
// ImageTexture::Evaluate (ImageTexture.h:52-60): UVMapping2D::Map (Texture.cpp:8-14), then the MIPMap
// lookup with the zero differentials every hit carries (F5).
static const TextureO* SlotTex(const Scene& s, const pbr_material_desc& m, int slot) {
    return m.tex[slot] ? &s.textures[m.tex[slot] - 1] : nullptr;
}
static Spec EvalSpec(const Scene& s, const pbr_material_desc& m, int slot, const float* constant, const SurfaceInteraction& si) {
    const TextureO* t = SlotTex(s, m, slot);
    if (!t) return S3(constant);
    P2 st(t->su * si.uv.x + t->du, t->sv * si.uv.y + t->dv);
    return t->ms->LookupZeroDifferentials(st, t->trilinear);
}
static float EvalFloat(const Scene& s, const pbr_material_desc& m, int slot, float constant, const SurfaceInteraction& si) {
    const TextureO* t = SlotTex(s, m, slot);
    if (!t) return constant;
    P2 st(t->su * si.uv.x + t->du, t->sv * si.uv.y + t->dv);
    return t->mf->LookupZeroDifferentials(st, t->trilinear);
}

// Material::ComputeScatteringFunctions for each material (Material/*.cpp)
static void ComputeBSDF(const Scene& s, const SurfaceInteraction& si, bool allowMultipleLobes, BSDF* bsdf) {
    const Prim& pr = s.prims[si.prim];
    bsdf->valid = false;
    bsdf->n = 0;
    if (pr.material < 0) return;                       // no material → no bsdf (Primitive.cpp:39-46)
    const MaterialO& mo = s.materials[pr.material];
    const pbr_material_desc& m = mo.d;
    bsdf->valid = true;
    bsdf->eta = 1;
    if (m.type == PBR_MAT_GLASS) bsdf->eta = m.eta;
    bsdf->ns = si.sn; bsdf->ng = si.n;
    bsdf->ss = Normalize(si.dpdu);
    bsdf->ts = Cross(bsdf->ns, bsdf->ss);
    switch (m.type) {
    case PBR_MAT_MATTE: {                               // MatteMaterial.cpp:13-28
        Spec r = EvalSpec(s, m, PBR_TEX_KD, m.Kd, si).Clamp();
        float sig = Clampf(EvalFloat(s, m, PBR_TEX_SIGMA, m.sigma, si), 0, 90);
        if (!r.IsBlack()) {
            Lobe l; l.R = r; l.type = BSDF_REFLECTION | BSDF_DIFFUSE;
            if (sig == 0) l.kind = L_LAMBERT;
            else {
                l.kind = L_OREN;
                float sg = Radians(sig);
                float sigma2 = sg * sg;
                l.A = 1.f - (sigma2 / (2.f * (sigma2 + 0.33f)));
                l.B = 0.45f * sigma2 / (sigma2 + 0.09f);
            }
            bsdf->Add(l);
        }
        break;
    }
    case PBR_MAT_MIRROR: {                              // Mirror.cpp:5-15
        Spec R = EvalSpec(s, m, PBR_TEX_KR, m.Kr, si).Clamp();
        if (!R.IsBlack()) { Lobe l; l.kind = L_SPEC_R; l.type = BSDF_REFLECTION | BSDF_SPECULAR; l.R = R; l.fresnel = FR_NOOP; bsdf->Add(l); }
        break;
    }
    case PBR_MAT_GLASS: {                               // GlassMaterial.cpp:9-57
        float eta = m.eta, urough = m.uroughness, vrough = m.vroughness;
        Spec R = EvalSpec(s, m, PBR_TEX_KR, m.Kr, si).Clamp(), T = EvalSpec(s, m, PBR_TEX_KT, m.Kt, si).Clamp();
        if (R.IsBlack() && T.IsBlack()) break;
        bool isSpecular = urough == 0 && vrough == 0;
        if (isSpecular && allowMultipleLobes) {
            Lobe l; l.kind = L_FRESNEL_SPEC; l.type = BSDF_REFLECTION | BSDF_TRANSMISSION | BSDF_SPECULAR;
            l.R = R; l.T = T; l.etaA = 1.f; l.etaB = eta; bsdf->Add(l);
        } else {
            if (m.remap_roughness) { urough = mo.ua; vrough = mo.va; }
            if (!R.IsBlack()) {
                Lobe l; l.R = R; l.fresnel = FR_DIEL; l.fEtaI = 1.f; l.fEtaT = eta;
                if (isSpecular) { l.kind = L_SPEC_R; l.type = BSDF_REFLECTION | BSDF_SPECULAR; }
                else { l.kind = L_MF_R; l.type = BSDF_REFLECTION | BSDF_GLOSSY; l = MakeTR(l, urough, vrough); }
                bsdf->Add(l);
            }
            if (!T.IsBlack()) {
                Lobe l; l.T = T; l.etaA = 1.f; l.etaB = eta;
                if (isSpecular) { l.kind = L_SPEC_T; l.type = BSDF_TRANSMISSION | BSDF_SPECULAR; }
                else { l.kind = L_MF_T; l.type = BSDF_TRANSMISSION | BSDF_GLOSSY; l = MakeTR(l, urough, vrough); }
                bsdf->Add(l);
            }
        }
        break;
    }
    case PBR_MAT_METAL: {                               // MetalMaterial.cpp:25-43
        float uR = m.has_uv_roughness ? m.uroughness : m.roughness;
        float vR = m.has_uv_roughness ? m.vroughness : m.roughness;
        if (m.remap_roughness) { uR = mo.ua; vR = mo.va; }
        Lobe l; l.kind = L_MF_R; l.type = BSDF_REFLECTION | BSDF_GLOSSY; l.R = Spec(1.);
        l.fresnel = FR_COND; l.cEtaI = Spec(1.); l.cEtaT = S3(m.metal_eta); l.cK = S3(m.metal_k);
        bsdf->Add(MakeTR(l, uR, vR));
        break;
    }
    case PBR_MAT_PLASTIC: {                             // PlasticMaterial.cpp:8-30
        Spec kd = EvalSpec(s, m, PBR_TEX_KD, m.Kd, si).Clamp();
        if (!kd.IsBlack()) { Lobe l; l.kind = L_LAMBERT; l.type = BSDF_REFLECTION | BSDF_DIFFUSE; l.R = kd; bsdf->Add(l); }
        Spec ks = EvalSpec(s, m, PBR_TEX_KS, m.Ks, si).Clamp();
        if (!ks.IsBlack()) {
            float rough = EvalFloat(s, m, PBR_TEX_ROUGHNESS, m.roughness, si);
            if (m.remap_roughness) rough = m.tex[PBR_TEX_ROUGHNESS] ? RoughnessToAlpha(rough) : mo.ra;
            Lobe l; l.kind = L_MF_R; l.type = BSDF_REFLECTION | BSDF_GLOSSY; l.R = ks;
            l.fresnel = FR_DIEL; l.fEtaI = 1.5f; l.fEtaT = 1.f;
            bsdf->Add(MakeTR(l, rough, rough));
        }
        break;
    }
    default: break;
    }
}

// ---------------------------------------------------------------- lights (Light/*.cpp)
enum { LF_DELTA_POS = 1, LF_AREA = 4, LF_INFINITE = 8 };
static int LightFlags(const Light& l) { return l.type == PBR_LIGHT_POINT ? LF_DELTA_POS : (l.type == PBR_LIGHT_DIFFUSE_AREA ? LF_AREA : LF_INFINITE); }
static bool IsDelta(const Light& l) { return LightFlags(l) & LF_DELTA_POS; }

struct Vis { Interaction p0, p1; };

static Spec AreaL(const Light& l, const Interaction& intr, V3 w) {   // DiffuseLight.h:17-19
    return (l.twoSided || Dot(intr.n, w) > 0) ? l.Lemit : Spec(0.f);
}
static void SphereUV(V3 p, float& u, float& v) {   // SkyBoxLight.cpp:12-17
    float phi = t_atan2(p.z, p.x);
    float theta = t_asin(p.y);
    u = 1 - (phi + Pi) * Inv2Pi;
    v = (theta + PiOver2) * InvPi;
}
static Spec SkyValue(const Light& l, float u, float v) {   // SkyBoxLight.cpp:27-40
    u = Clampf(u, 0.f, 1.f);
    v = Clampf(v, 0.f, 1.f);
    int w = u * l.w, h = v * l.h;
    w = Clampi(w, 0, l.w - 1);
    h = Clampi(h, 0, l.h - 1);
    int offset = (w + h * l.w) * l.comps;
    Spec Lv(l.data[offset + 0], l.data[offset + 1], l.data[offset + 2]);
    return HDRtoLDR(Lv, 0.3f);
}
// InfiniteAreaLight (Light/InfiniteAreaLight.cpp)
static float SphericalTheta(V3 v) { return t_acos(Clampf(v.z, -1, 1)); }   // Geometry.h:1517-1519
static float SphericalPhi(V3 v) {                                           // Geometry.h:1521-1524
    float p = t_atan2(v.y, v.x);
    return (p < 0) ? (p + 2 * Pi) : p;
}
static Spec InfiniteLe(const Light& l, const Ray& ray) {   // InfiniteAreaLight.cpp:70-75
    V3 w = Normalize(l.w2l.vector(ray.d));
    P2 st(SphericalPhi(w) * Inv2Pi, SphericalTheta(w) * InvPi);
    return l.Lmap->Lookup(st, 0.f);
}
static Spec LightLe(const Light& l, const Ray& ray) {
    if (l.type == PBR_LIGHT_INFINITE_AREA) return InfiniteLe(l, ray);
    if (l.type == PBR_LIGHT_SKYBOX) {   // SkyBoxLight.cpp:59-77
        V3 dn = Normalize(ray.d);
        float u, v;
        SphereUV(dn, u, v);
        if (!l.data.empty()) return SkyValue(l, u, v);
        return Spec(0.f);
    }
    return Spec(0.8f);                  // Light::Le default (Light.h:58, F4)
}
static Interaction TriangleSample(const Scene& s, const Prim& pr, P2 u, float* pdf, float* area) {   // Triangle.cpp:360-387
    const Mesh& m = s.meshes[pr.shape];
    V3 p0 = m.p[m.idx[3 * pr.tri]], p1 = m.p[m.idx[3 * pr.tri + 1]], p2 = m.p[m.idx[3 * pr.tri + 2]];
    P2 b = UniformSampleTriangle(u);
    Interaction it;
    it.p = b.x * p0 + b.y * p1 + (1 - b.x - b.y) * p2;
    it.n = Normalize(Cross(p1 - p0, p2 - p0));
    if (m.reverse ^ m.swaps) it.n = it.n * -1;
    V3 pAbsSum = Abs(b.x * p0) + Abs(b.y * p1) + Abs((1 - b.x - b.y) * p2);
    it.pError = gamma(6) * pAbsSum;
    float A = (float)(0.5 * (double)Length(Cross(p1 - p0, p2 - p0)));
    if (area) *area = A;
    *pdf = 1 / A;
    return it;
}
static float TriangleArea(const Scene& s, const Prim& pr) {   // Triangle.cpp:352-358
    const Mesh& m = s.meshes[pr.shape];
    V3 p0 = m.p[m.idx[3 * pr.tri]], p1 = m.p[m.idx[3 * pr.tri + 1]], p2 = m.p[m.idx[3 * pr.tri + 2]];
    return (float)(0.5 * (double)Length(Cross(p1 - p0, p2 - p0)));
}
static Spec SampleLi(const Scene& s, const Light& l, const Interaction& ref, P2 u, V3* wi, float* pdf, Vis* vis) {
    if (l.type == PBR_LIGHT_POINT) {   // PointLight.cpp:5-15
        *wi = Normalize(l.pLight - ref.p);
        *pdf = 1.f;
        vis->p0 = ref; vis->p1 = Interaction(); vis->p1.p = l.pLight; vis->p1.medIn = l.medIn; vis->p1.medOut = l.medOut;
        return l.I / DistanceSquared(l.pLight, ref.p);
    }
    if (l.type == PBR_LIGHT_DIFFUSE_AREA) {   // DiffuseLight.cpp:25-40 + Shape.cpp:18-30
        const Prim& pr = s.prims[s.primOfOriginal[l.prim]];
        Interaction intr = TriangleSample(s, pr, u, pdf, nullptr);
        V3 w = intr.p - ref.p;
        if (LengthSquared(w) == 0) *pdf = 0;
        else {
            w = Normalize(w);
            *pdf *= DistanceSquared(ref.p, intr.p) / AbsDot(intr.n, -w);
            if (std::isinf(*pdf)) *pdf = 0.f;
        }
        if (*pdf == 0 || LengthSquared(intr.p - ref.p) == 0) { *pdf = 0; return Spec(0.f); }
        *wi = Normalize(intr.p - ref.p);
        vis->p0 = ref; vis->p1 = intr;
        return AreaL(l, intr, -*wi);
    }
    if (l.type == PBR_LIGHT_INFINITE_AREA) {   // InfiniteAreaLight.cpp:78-100
        float mapPdf;
        P2 uv = l.distribution->SampleContinuous2(u, &mapPdf);
        if (mapPdf == 0) { *pdf = 0; return Spec(0.f); }
        float theta = uv.y * Pi, phi = uv.x * 2 * Pi;
        float cosTheta = t_cos(theta), sinTheta = t_sin(theta);
        float sinPhi = t_sin(phi), cosPhi = t_cos(phi);
        *wi = l.l2w.vector(V3(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta));
        *pdf = mapPdf / (2 * Pi * Pi * sinTheta);
        if (sinTheta == 0) *pdf = 0;
        vis->p0 = ref; vis->p1 = Interaction(); vis->p1.p = ref.p + *wi * (2 * l.worldRadius);
        return l.Lmap->Lookup(uv, 0.f);
    }
    // SkyBoxLight::Sample_Li (SkyBoxLight.cpp:43-56)
    *wi = UniformSampleSphere(u);
    *pdf = 1.f / (4 * Pi);
    vis->p0 = ref; vis->p1 = Interaction(); vis->p1.p = ref.p + *wi * (2 * l.worldRadius);
    float ul, vl;
    SphereUV(Normalize(*wi), ul, vl);
    if (l.data.empty()) return Spec(0.f);
    return SkyValue(l, ul, vl);
}
static float PdfLi(const Scene& s, const Light& l, const Interaction& ref, V3 wi) {
    if (l.type == PBR_LIGHT_INFINITE_AREA) {   // InfiniteAreaLight.cpp:103-110
        V3 w = l.w2l.vector(wi);
        float theta = SphericalTheta(w), phi = SphericalPhi(w);
        float sinTheta = t_sin(theta);
        if (sinTheta == 0) return 0;
        return l.distribution->Pdf(P2(phi * Inv2Pi, theta * InvPi)) / (2 * Pi * Pi * sinTheta);
    }
    if (l.type != PBR_LIGHT_DIFFUSE_AREA) return 0;   // point: 0; skybox: 0 (SkyBoxLight.h:29)
    // Shape::Pdf (Shape.cpp:31-42): intersect the light's own shape only
    const Prim& pr = s.prims[s.primOfOriginal[l.prim]];
    Ray ray = ref.SpawnRay(wi);
    const Mesh& m = s.meshes[pr.shape];
    float t, b0, b1, b2;
    if (!TriangleTest(m.p[m.idx[3 * pr.tri]], m.p[m.idx[3 * pr.tri + 1]], m.p[m.idx[3 * pr.tri + 2]], ray, &t, &b0, &b1, &b2))
        return 0;
    SurfaceInteraction isectLight;
    TriangleSI(m, pr.tri, ray, b0, b1, b2, &isectLight);
    float pdf = DistanceSquared(ref.p, isectLight.p) / (AbsDot(isectLight.n, -wi) * TriangleArea(s, pr));
    if (std::isinf(pdf)) pdf = 0.f;
    return pdf;
}
static bool Unoccluded(const Scene& s, const Vis& v) { return !IntersectP(s, v.p0.SpawnRayTo(v.p1)); }   // Light.cpp:19-22

static Spec MediumTr(const Medium& m, const Ray& ray) {   // HomogeneousMedium.cpp:10-12
    return ExpS(Spec(-m.sigma_t[0], -m.sigma_t[1], -m.sigma_t[2]) * fmin_(ray.tMax * Length(ray.d), MaxFloat));
}
static Spec VisTr(const Scene& s, const Vis& v) {   // Light.cpp:31-47
    Ray ray(v.p0.SpawnRayTo(v.p1));
    Spec Tr(1.f);
    while (true) {
        SurfaceInteraction isect;
        bool hitSurface = Intersect(s, ray, &isect);
        if (hitSurface && s.prims[isect.prim].material >= 0) return Spec(0.0f);
        if (ray.medium >= 0) Tr *= MediumTr(s.media[ray.medium], ray);
        if (!hitSurface) break;
        ray = isect.SpawnRayTo(v.p1);
    }
    return Tr;
}
static Spec SILe(const Scene& s, const SurfaceInteraction& si, V3 w) {   // Interaction.cpp:116-119
    int al = s.prims[si.prim].areaLight;
    return al >= 0 ? AreaL(s.lights[al], si, w) : Spec(0.f);
}

inline float PhaseHG(float cosTheta, float g) {   // Medium.h:24-27
    float denom = 1 + g * g + 2 * g * cosTheta;
    return Inv4Pi * (1 - g * g) / (denom * std::sqrt(denom));
}
static float HGSample(float g, V3 wo, V3* wi, P2 u) {   // Medium.cpp:9-26
    float cosTheta;
    if ((double)std::abs(g) < 1e-3) cosTheta = 1 - 2 * u.x;
    else {
        float sqrTerm = (1 - g * g) / (1 + g - 2 * g * u.x);
        cosTheta = -(1 + g * g - sqrTerm * sqrTerm) / (2 * g);
    }
    float sinTheta = std::sqrt(fmax_((float)0, 1 - cosTheta * cosTheta));
    float phi = 2 * Pi * u.y;
    V3 v1, v2;
    CoordinateSystem(wo, &v1, &v2);
    *wi = SphericalDirection(sinTheta, cosTheta, phi, v1, v2, wo);
    return PhaseHG(cosTheta, g);
}

// ---------------------------------------------------------------- integrators
struct Ctx {
    const Scene* s;
    int integrator, maxDepth;
    float rrThreshold;
    Distribution1D lightDistrib;
};

// Integrator.cpp:71-177
static Spec EstimateDirect(const Ctx& c, const Interaction& it, const BSDF* bsdf, float phaseG, P2 uScattering,
                           int lightIdx, P2 uLight, Halton& sampler, bool handleMedia) {
    const Scene& s = *c.s;
    const Light& light = s.lights[lightIdx];
    int bsdfFlags = BSDF_ALL & ~BSDF_SPECULAR;
    Spec Ld(0.f);
    V3 wi;
    float lightPdf = 0, scatteringPdf = 0;
    Vis vis;
    Spec Li = SampleLi(s, light, it, uLight, &wi, &lightPdf, &vis);
    if (lightPdf > 0 && !Li.IsBlack()) {
        Spec f;
        if (it.IsSurface()) {
            const SurfaceInteraction& isect = (const SurfaceInteraction&)it;
            f = bsdf->f(isect.wo, wi, bsdfFlags) * AbsDot(wi, isect.sn);
            scatteringPdf = bsdf->Pdf(isect.wo, wi, bsdfFlags);
        } else {
            f = Spec(PhaseHG(Dot(it.wo, wi), phaseG));
        }
        if (!f.IsBlack()) {
            if (handleMedia) Li *= VisTr(s, vis);
            else if (!Unoccluded(s, vis)) Li = Spec(0.f);
            if (!Li.IsBlack()) {
                if (IsDelta(light)) Ld += f * Li / lightPdf;
                else {
                    float weight = PowerHeuristic(1, lightPdf, 1, scatteringPdf);
                    Ld += f * Li * weight / lightPdf;
                }
            }
        }
    }
    if (!IsDelta(light)) {
        Spec f;
        bool sampledSpecular = false;
        if (it.IsSurface()) {
            const SurfaceInteraction& isect = (const SurfaceInteraction&)it;
            int sampledType = 0;
            f = bsdf->Sample_f(isect.wo, &wi, uScattering, &scatteringPdf, bsdfFlags, &sampledType);
            f *= AbsDot(wi, isect.sn);
            sampledSpecular = (sampledType & BSDF_SPECULAR) != 0;
        } else {
            float p = HGSample(phaseG, it.wo, &wi, uScattering);
            f = Spec(p);
            scatteringPdf = p;
        }
        if (!f.IsBlack() && scatteringPdf > 0) {
            float weight = 1;
            if (!sampledSpecular) {
                lightPdf = PdfLi(s, light, it, wi);
                if (lightPdf == 0) return Ld;
                weight = PowerHeuristic(1, scatteringPdf, 1, lightPdf);
            }
            SurfaceInteraction lightIsect;
            Ray ray = it.SpawnRay(wi);
            bool found = Intersect(s, ray, &lightIsect);
            Spec Li2(0.f);
            if (found) {
                if (s.prims[lightIsect.prim].areaLight == lightIdx) Li2 = SILe(s, lightIsect, -wi);
            } else
                Li2 = LightLe(light, ray);
            if (!Li2.IsBlack()) Ld += f * Li2 * weight / scatteringPdf;
        }
    }
    return Ld;
}

// Integrator.cpp:46-69 (a light distribution is always passed by Path/VolPath)
static Spec UniformSampleOneLight(const Ctx& c, const Interaction& it, const BSDF* bsdf, float phaseG, Halton& sampler,
                                  bool handleMedia) {
    int nLights = (int)c.s->lights.size();
    if (nLights == 0) return Spec(0.f);
    float lightPdf;
    int lightNum = c.lightDistrib.SampleDiscrete(sampler.Get1D(), &lightPdf);
    if (lightPdf == 0) return Spec(0.f);
    P2 uLight = sampler.Get2D();
    P2 uScattering = sampler.Get2D();
    return EstimateDirect(c, it, bsdf, phaseG, uScattering, lightNum, uLight, sampler, handleMedia) / lightPdf;
}

// WhittedIntegrator.cpp:11-65 + SpecularReflect (Integrator.cpp:179-222)
static Spec WhittedLi(const Ctx& c, const Ray& ray, Halton& sampler, int depth) {
    const Scene& s = *c.s;
    Spec L(0.);
    SurfaceInteraction isect;
    if (!Intersect(s, ray, &isect)) {
        for (const Light& l : s.lights) L += LightLe(l, ray);
        return L;
    }
    if (tl_counters) tl_counters->shading++;
    V3 n = isect.sn;
    V3 wo = isect.wo;
    BSDF bsdf;
    ComputeBSDF(s, isect, false, &bsdf);
    if (!bsdf.valid) return WhittedLi(c, isect.SpawnRay(ray.d), sampler, depth);
    L += SILe(s, isect, wo);
    for (const Light& l : s.lights) {
        V3 wi;
        float pdf;
        Vis vis;
        Spec Li = SampleLi(s, l, isect, sampler.Get2D(), &wi, &pdf, &vis);
        if (Li.IsBlack() || pdf == 0) continue;
        Spec f = bsdf.f(wo, wi);
        if (!f.IsBlack() && Unoccluded(s, vis)) L += f * Li * AbsDot(wi, n) / pdf;
    }
    if (depth + 1 < c.maxDepth) {
        V3 wi;
        float pdf = 0;
        P2 u = sampler.Get2D();
        Spec f = bsdf.Sample_f(wo, &wi, u, &pdf, BSDF_REFLECTION | BSDF_SPECULAR, nullptr);
        V3 ns = isect.sn;
        Spec add(0.f);
        if (!f.IsBlack() && pdf > 0.f && AbsDot(wi, ns) != 0.f) {
            Ray rd = isect.SpawnRay(wi);
            add = f * WhittedLi(c, rd, sampler, depth + 1) * AbsDot(wi, ns) / pdf;
        }
        L += add;
    }
    return L;
}

// PathIntegrator.cpp:32-110
static Spec PathLi(const Ctx& c, Ray ray, Halton& sampler) {
    const Scene& s = *c.s;
    Spec L(0.f), beta(1.f);
    bool specularBounce = false;
    int bounces;
    float etaScale = 1;
    for (bounces = 0;; ++bounces) {
        SurfaceInteraction isect;
        bool found = Intersect(s, ray, &isect);
        if (bounces == 0 || specularBounce) {
            if (found) L += beta * SILe(s, isect, -ray.d);
            else for (int li : s.infinite) L += beta * LightLe(s.lights[li], ray);
        }
        if (!found || bounces >= c.maxDepth) break;
        if (tl_counters) tl_counters->shading++;
        BSDF bsdf;
        ComputeBSDF(s, isect, true, &bsdf);
        if (!bsdf.valid) { ray = isect.SpawnRay(ray.d); bounces--; continue; }
        if (bsdf.NumComponents(BSDF_ALL & ~BSDF_SPECULAR) > 0) {
            Spec Ld = beta * UniformSampleOneLight(c, isect, &bsdf, 0, sampler, false);
            L += Ld;
        }
        V3 wo = -ray.d, wi;
        float pdf = 0;
        int flags = 0;
        Spec f = bsdf.Sample_f(wo, &wi, sampler.Get2D(), &pdf, BSDF_ALL, &flags);
        if (f.IsBlack() || pdf == 0.f) break;
        beta *= f * AbsDot(wi, isect.sn) / pdf;
        specularBounce = (flags & BSDF_SPECULAR) != 0;
        if ((flags & BSDF_SPECULAR) && (flags & BSDF_TRANSMISSION)) {
            float eta = bsdf.eta;
            etaScale *= (Dot(wo, isect.n) > 0) ? (eta * eta) : 1 / (eta * eta);
        }
        ray = isect.SpawnRay(wi);
        Spec rrBeta = beta * etaScale;
        if (rrBeta.MaxComponentValue() < c.rrThreshold && bounces > 3) {
            float q = fmax_((float).05, 1 - rrBeta.MaxComponentValue());
            if (sampler.Get1D() < q) break;
            beta /= 1 - q;
        }
    }
    return L;
}

// HomogeneousMedium::Sample (HomogeneousMedium.cpp:15-45)
static Spec MediumSample(const Medium& m, int mediumIdx, const Ray& ray, Halton& sampler, MediumInteraction* mi) {
    int channel = std::min((int)(sampler.Get1D() * 3), 3 - 1);
    float dist = -t_log(1 - sampler.Get1D()) / m.sigma_t[channel];
    float t = fmin_(dist / Length(ray.d), ray.tMax);
    bool sampledMedium = t < ray.tMax;
    if (sampledMedium) {
        mi->p = ray.at(t); mi->wo = -ray.d; mi->n = V3(0, 0, 0); mi->pError = V3(0, 0, 0);
        mi->medIn = mi->medOut = mediumIdx; mi->medium = mediumIdx; mi->g = m.g; mi->valid = true;
    }
    Spec Tr = ExpS(Spec(-m.sigma_t[0], -m.sigma_t[1], -m.sigma_t[2]) * fmin_(t, MaxFloat) * Length(ray.d));
    Spec density = sampledMedium ? (m.sigma_t * Tr) : Tr;
    float pdf = 0;
    for (int i = 0; i < 3; ++i) pdf += density[i];
    pdf *= 1 / (float)3;
    if (pdf == 0) pdf = 1;
    return sampledMedium ? (Tr * m.sigma_s / pdf) : (Tr / pdf);
}

// VolPathIntegrator.cpp:21-107
static Spec VolPathLi(const Ctx& c, Ray ray, Halton& sampler) {
    const Scene& s = *c.s;
    Spec L(0.f), beta(1.f);
    bool specularBounce = false;
    int bounces;
    float etaScale = 1;
    for (bounces = 0;; ++bounces) {
        SurfaceInteraction isect;
        bool found = Intersect(s, ray, &isect);
        MediumInteraction mi;
        if (ray.medium >= 0) beta *= MediumSample(s.media[ray.medium], ray.medium, ray, sampler, &mi);
        if (beta.IsBlack()) break;
        if (mi.valid) {
            if (bounces >= c.maxDepth) break;
            if (tl_counters) tl_counters->shading++;
            L += beta * UniformSampleOneLight(c, mi, nullptr, mi.g, sampler, true);
            V3 wo = -ray.d, wi;
            HGSample(mi.g, wo, &wi, sampler.Get2D());
            ray = mi.SpawnRay(wi);
            specularBounce = false;
        } else {
            if (bounces == 0 || specularBounce) {
                if (found) L += beta * SILe(s, isect, -ray.d);
                else for (int li : s.infinite) L += beta * LightLe(s.lights[li], ray);
            }
            if (!found || bounces >= c.maxDepth) break;
            if (tl_counters) tl_counters->shading++;
            BSDF bsdf;
            ComputeBSDF(s, isect, true, &bsdf);
            if (!bsdf.valid) { ray = isect.SpawnRay(ray.d); bounces--; continue; }
            L += beta * UniformSampleOneLight(c, isect, &bsdf, 0, sampler, true);
            V3 wo = -ray.d, wi;
            float pdf = 0;
            int flags = 0;
            Spec f = bsdf.Sample_f(wo, &wi, sampler.Get2D(), &pdf, BSDF_ALL, &flags);
            if (f.IsBlack() || pdf == 0.f) break;
            beta *= f * AbsDot(wi, isect.sn) / pdf;
            specularBounce = (flags & BSDF_SPECULAR) != 0;
            if ((flags & BSDF_SPECULAR) && (flags & BSDF_TRANSMISSION)) {
                float eta = bsdf.eta;
                etaScale *= (Dot(wo, isect.n) > 0) ? (eta * eta) : 1 / (eta * eta);
            }
            ray = isect.SpawnRay(wi);
        }
        Spec rrBeta = beta * etaScale;
        if (rrBeta.MaxComponentValue() < c.rrThreshold && bounces > 3) {
            float q = fmax_((float).05, 1 - rrBeta.MaxComponentValue());
            if (sampler.Get1D() < q) break;
            beta /= 1 - q;
        }
    }
    return L;
}

// ---------------------------------------------------------------- camera (Camera/*.cpp)
struct Camera {
    Xform cameraToWorld, rasterToCamera;
    float lensRadius = 0, focalDistance = 0;
    int medium = -1;
    void init(const pbr_camera_desc& d) {
        if (d.use_look_at) {
            Xform lookat = LookAt(V3(d.eye[0], d.eye[1], d.eye[2]), V3(d.look[0], d.look[1], d.look[2]),
                                  V3(d.up[0], d.up[1], d.up[2]));
            cameraToWorld = InverseX(lookat);
        } else {
            cameraToWorld = Xform(M4::rows(d.camera_to_world.m), M4::rows(d.camera_to_world.m_inv));
        }
        // CreatePerspectiveCamera (Perspective.cpp:84-104)
        float frame = (float)d.width / (float)d.height;
        float sMinX, sMaxX, sMinY, sMaxY;
        if (frame > 1.f) { sMinX = -frame; sMaxX = frame; sMinY = -1.f; sMaxY = 1.f; }
        else { sMinX = -1.f; sMaxX = 1.f; sMinY = -1.f / frame; sMaxY = 1.f / frame; }
        // ProjectiveCamera ctor (Camera.h:36-53), PerspectiveCamera (Perspective.cpp:5-11)
        Xform cameraToScreen = Perspective(d.fov, 1e-2f, 1000.f);
        Xform screenToRaster = Scale((float)d.width, (float)d.height, 1) *
                               Scale(1 / (sMaxX - sMinX), 1 / (sMinY - sMaxY), 1) *
                               Translate(V3(-sMinX, -sMaxY, 0));
        Xform rasterToScreen = InverseX(screenToRaster);
        rasterToCamera = InverseX(cameraToScreen) * rasterToScreen;
        // pbr_camera_desc::use_raster_to_camera: the camera's own RasterToCamera, any fov / screen window
        if (d.use_raster_to_camera)
            rasterToCamera = Xform(M4::rows(d.raster_to_camera.m), M4::rows(d.raster_to_camera.m_inv));
        lensRadius = d.lens_radius;
        focalDistance = d.focal_distance;
        medium = d.medium;
    }
    // PerspectiveCamera::GenerateRayDifferential (Perspective.cpp:44-80); differentials are dead
    Ray generate(P2 pFilmXY, P2 pLensU) const {
        V3 pFilm(pFilmXY.x, pFilmXY.y, 0);
        V3 pCamera = rasterToCamera.point(pFilm);
        V3 dir = Normalize(V3(pCamera.x, pCamera.y, pCamera.z));
        Ray r(V3(0, 0, 0), dir);
        if (lensRadius > 0) {
            P2 pl = ConcentricSampleDisk(pLensU);
            P2 pLens(lensRadius * pl.x, lensRadius * pl.y);
            float ft = focalDistance / r.d.z;
            V3 pFocus = r.at(ft);
            r.o = V3(pLens.x, pLens.y, 0);
            r.d = Normalize(pFocus - r.o);
        }
        // CameraToWorld(RayDifferential) drops the medium (Transform.h:165-180, F12)
        return Ray(cameraToWorld.point(r.o), cameraToWorld.vector(r.d), r.tMax, -1);
    }
};

// ---------------------------------------------------------------- scene assembly from the C desc
// InfiniteAreaLight constructor (InfiniteAreaLight.cpp:7-61) and Preprocess (InfiniteAreaLight.h:15-17)
static void InfinitePreprocess(const Scene& s, Light* l) {
    int w = 1, h = 1;
    std::vector<Spec> texels;
    if (!l->data.empty()) {
        w = l->w; h = l->h;
        texels.resize((size_t)w * h);
        for (int j = 0; j < h; j++)
            for (int i = 0; i < w; i++) {
                Spec r;
                for (int k = 0; k < 3; ++k) {
                    r[k] = l->data[((size_t)i + (size_t)j * w) * l->comps + k];
                    r[k] = l->Lemit[k] * r[k];
                }
                texels[i + (size_t)j * w] = r;
            }
    } else {
        texels.assign(1, l->Lemit);   // no texmap: the 1x1 map of L (the reference frees an uninitialised pointer first)
    }
    l->Lmap = std::make_shared<MIPMapS>(w, h, texels.data());
    int width = l->Lmap->Width(), height = l->Lmap->Height();
    std::vector<float> img((size_t)width * height);
    for (int v = 0; v < height; v++) {
        float vp = (v + .5f) / (float)height;
        float sinTheta = t_sin(Pi * (v + .5f) / height);
        for (int u = 0; u < width; ++u) {
            float up = (u + .5f) / (float)width;
            img[u + (size_t)v * width] = l->Lmap->Lookup(P2(up, vp), 0.f).y();
            img[u + (size_t)v * width] *= sinTheta;
        }
    }
    l->distribution = std::make_shared<Distribution2D>(img.data(), width, height);
    // scene.WorldBound().BoundingSphere(&worldCenter, &worldRadius) (Geometry.h:1250-1254)
    Bounds3 wb;
    if (!s.nodes.empty()) {
        wb.pMin = V3(s.nodes[0].pMin[0], s.nodes[0].pMin[1], s.nodes[0].pMin[2]);
        wb.pMax = V3(s.nodes[0].pMax[0], s.nodes[0].pMax[1], s.nodes[0].pMax[2]);
    }
    V3 c = (wb.pMin + wb.pMax) * 0.5f;   // Point3::operator/(2): multiply by the reciprocal
    bool inside = c.x >= wb.pMin.x && c.x <= wb.pMax.x && c.y >= wb.pMin.y && c.y <= wb.pMax.y && c.z >= wb.pMin.z &&
                  c.z <= wb.pMax.z;
    l->worldCenter = c;
    l->worldRadius = inside ? Length(c - wb.pMax) : 0;
}

// material index of a primitive: a PBR_MAT_NONE material means material == nullptr (-1)
static int mat_index(const pbr_scene_desc* d, int m) {
    return (m >= 0 && m < d->n_materials && d->materials[m].type == PBR_MAT_NONE) ? -1 : m;
}

static std::unique_ptr<Scene> BuildScene(const pbr_scene_desc* d) {
    if (!d || d->abi_version != PBR_HIP_ABI_VERSION) throw std::runtime_error("bad scene desc");
    // A caller-built tree (pbr_scene_desc::bvh_nodes: the reference's own BVHAccel, primitives given
    // in its leaf order) is adopted as is, as the product's upload adopts it; else BVHAccel is built.
    if (d->bvh_nodes && d->n_bvh_nodes <= 0) throw std::runtime_error("bvh_nodes without n_bvh_nodes");
    std::unique_ptr<Scene> s(new Scene);
    std::vector<Prim> prims;
    int ns = d->n_shapes;
    s->meshes.resize(ns);
    s->spheres.resize(ns);
    s->shapeType.resize(ns);
    for (int i = 0; i < ns; ++i) {
        const pbr_shape_desc& sd = d->shapes[i];
        s->shapeType[i] = sd.type;
        Xform o2w(M4::rows(sd.object_to_world.m), M4::rows(sd.object_to_world.m_inv));
        if (sd.type == PBR_SHAPE_TRIANGLE_MESH) {
            if (sd.N) throw std::runtime_error("per-vertex normals are not supported");
            Mesh& m = s->meshes[i];
            m.p.resize(sd.n_vertices);
            for (int v = 0; v < sd.n_vertices; ++v) m.p[v] = o2w.point(V3(sd.P[3 * v], sd.P[3 * v + 1], sd.P[3 * v + 2]));
            m.idx.assign(sd.indices, sd.indices + 3 * sd.n_triangles);
            if (sd.UV) {
                m.hasUV = true;
                m.uv.resize(sd.n_vertices);
                for (int v = 0; v < sd.n_vertices; ++v) m.uv[v] = P2(sd.UV[2 * v], sd.UV[2 * v + 1]);
            }
            m.reverse = sd.reverse_orientation != 0;
            m.swaps = o2w.SwapsHandedness();
            for (int t = 0; t < sd.n_triangles; ++t)
                prims.push_back(Prim{i, t, mat_index(d, sd.material), sd.area_light_first >= 0 ? sd.area_light_first + t : -1,
                                     sd.medium_inside, sd.medium_outside});
        } else {
            SphereS& sp = s->spheres[i];
            sp.o2w = o2w;
            sp.w2o = InverseX(o2w);
            sp.radius = sd.radius;
            sp.reverse = sd.reverse_orientation != 0;
            sp.swaps = o2w.SwapsHandedness();
            if (sd.area_light_first >= 0) throw std::runtime_error("sphere area lights are not supported");
            prims.push_back(Prim{i, -1, mat_index(d, sd.material), -1, sd.medium_inside, sd.medium_outside});
        }
    }
    for (int i = 0; i < d->n_materials; ++i) {
        MaterialO mo;
        mo.d = d->materials[i];
        mo.ua = RoughnessToAlpha(mo.d.uroughness);
        mo.va = RoughnessToAlpha(mo.d.vroughness);
        mo.ra = RoughnessToAlpha(mo.d.roughness);
        if (mo.d.type == PBR_MAT_METAL && !mo.d.has_uv_roughness) { mo.ua = mo.va = mo.ra; }
        s->materials.push_back(mo);
    }
    // ImageTexture::GetTexture (ImageTexture.cpp:46-92): loadImage's texels (or a 0.5 grey 1x1
    // image), convertIn (ImageTexture.h:69-78), MIPMap(res, texels, doTrilinear, maxAniso, wrap)
    for (int i = 0; i < d->n_textures; ++i) {
        const pbr_texture_desc& td = d->textures[i];
        TextureO t;
        t.isFloat = td.is_float != 0;
        t.trilinear = td.trilinear != 0;
        t.su = td.su; t.sv = td.sv; t.du = td.du; t.dv = td.dv;
        int w = 1, h = 1;
        std::vector<Spec> texels;
        const ImageWrapO wrap0 = (ImageWrapO)td.wrap;
        if (td.level0) {   // pbr_texture_desc::level0: a built texture's MIPMap level 0, used as is
            if (!td.data || td.width <= 0 || td.height <= 0 || (td.width & (td.width - 1)) || (td.height & (td.height - 1)) ||
                td.components != (t.isFloat ? 1 : 3))
                throw std::invalid_argument("bad level-0 texture");
            const size_t n = (size_t)td.width * td.height;
            if (t.isFloat) {
                t.mf = std::make_shared<MIPMapT<float>>(td.width, td.height, td.data, wrap0);
            } else {
                std::vector<Spec> l0(n);
                for (size_t j = 0; j < n; ++j) l0[j] = Spec(td.data[3 * j], td.data[3 * j + 1], td.data[3 * j + 2]);
                t.ms = std::make_shared<MIPMapT<Spec>>(td.width, td.height, l0.data(), wrap0);
            }
            s->textures.push_back(t);
            continue;
        }
        if (td.data && td.width > 0 && td.height > 0) {
            w = td.width; h = td.height;
            for (int j = 0; j < w * h; ++j)
                texels.push_back(Spec(td.data[(size_t)j * td.components], td.data[(size_t)j * td.components + 1], td.data[(size_t)j * td.components + 2]));
        } else {
            texels.push_back(Spec(0.5f));
        }
        auto igc = [](float v) { return v <= 0.04045f ? v * 1.f / 12.92f : t_pow((v + 0.055f) * 1.f / 1.055f, (float)2.4f); };
        const ImageWrapO wrap = (ImageWrapO)td.wrap;
        if (t.isFloat) {
            std::vector<float> conv(texels.size());
            for (size_t j = 0; j < texels.size(); ++j) conv[j] = td.scale * (td.gamma ? igc(texels[j].y()) : texels[j].y());
            t.mf = std::make_shared<MIPMapT<float>>(w, h, conv.data(), wrap);
        } else {
            std::vector<Spec> conv(texels.size());
            for (size_t j = 0; j < texels.size(); ++j)
                for (int k = 0; k < 3; ++k) conv[j].c[k] = td.scale * (td.gamma ? igc(texels[j].c[k]) : texels[j].c[k]);
            t.ms = std::make_shared<MIPMapT<Spec>>(w, h, conv.data(), wrap);
        }
        s->textures.push_back(t);
    }
    for (int i = 0; i < d->n_media; ++i) {
        const pbr_medium_desc& md = d->media[i];
        Medium m;
        m.sigma_a = S3(md.sigma_a); m.sigma_s = S3(md.sigma_s);
        m.sigma_t = m.sigma_s + m.sigma_a;
        m.g = md.g;
        s->media.push_back(m);
    }
    // original prim index of each area-light triangle
    std::vector<int> firstPrimOfShape(ns, 0);
    {
        int acc = 0;
        for (int i = 0; i < ns; ++i) { firstPrimOfShape[i] = acc; acc += d->shapes[i].type == PBR_SHAPE_TRIANGLE_MESH ? d->shapes[i].n_triangles : 1; }
    }
    for (int i = 0; i < d->n_lights; ++i) {
        const pbr_light_desc& ld = d->lights[i];
        Light l;
        l.type = ld.type;
        l.medIn = ld.medium_inside; l.medOut = ld.medium_outside;
        Xform l2w(M4::rows(ld.light_to_world.m), M4::rows(ld.light_to_world.m_inv));
        if (ld.type == PBR_LIGHT_POINT) {
            l.pLight = l2w.point(V3(0, 0, 0));
            l.I = S3(ld.I);
        } else if (ld.type == PBR_LIGHT_DIFFUSE_AREA) {
            l.Lemit = S3(ld.Le);
            l.twoSided = ld.two_sided != 0;
            l.prim = firstPrimOfShape[ld.shape] + ld.triangle;
        } else if (ld.type == PBR_LIGHT_INFINITE_AREA) {
            l.l2w = l2w;
            l.w2l = Xform(l2w.mInv, l2w.m);   // Inverse(LightToWorld) swaps m and mInv
            l.Lemit = S3(ld.Le);              // the constructor's `power` scale
            if (ld.env_data && ld.env_width > 0 && ld.env_height > 0) {
                l.w = ld.env_width; l.h = ld.env_height; l.comps = ld.env_components;
                l.data.assign(ld.env_data, ld.env_data + (size_t)l.w * l.h * l.comps);
            }
            s->infinite.push_back(i);
        } else {
            l.worldCenter = V3(ld.world_center[0], ld.world_center[1], ld.world_center[2]);
            l.worldRadius = ld.world_radius;
            if (ld.env_data) {
                l.w = ld.env_width; l.h = ld.env_height; l.comps = ld.env_components;
                l.data.assign(ld.env_data, ld.env_data + (size_t)l.w * l.h * l.comps);
            }
            s->infinite.push_back(i);
        }
        s->lights.push_back(std::move(l));
    }
    if (d->bvh_nodes) {
        s->nodes.resize(d->n_bvh_nodes);
        std::memcpy(s->nodes.data(), d->bvh_nodes, sizeof(OrcLinearBVHNode) * (size_t)d->n_bvh_nodes);
        s->prims = prims;
        s->primIds.resize(prims.size());
        s->primOfOriginal.resize(prims.size());
        for (size_t i = 0; i < prims.size(); ++i) s->primIds[i] = s->primOfOriginal[i] = (int)i;
    } else {
        BuildBVH(*s, prims, d->max_prims_in_node > 0 ? d->max_prims_in_node : 1, d->split_method);
    }
    for (Light& l : s->lights)
        if (l.type == PBR_LIGHT_DIFFUSE_AREA) l.area = TriangleArea(*s, s->prims[s->primOfOriginal[l.prim]]);
    for (Light& l : s->lights)
        if (l.type == PBR_LIGHT_INFINITE_AREA) InfinitePreprocess(*s, &l);
    return s;
}

static Distribution1D MakeLightDistrib(const Scene& s, int strategy) {   // LightDistrib.cpp:8-48
    size_t n = s.lights.size();
    if (n == 0) return Distribution1D();
    std::vector<float> f(n, 1.f);
    if (strategy == PBR_LIGHTS_POWER && n != 1) {
        for (size_t i = 0; i < n; ++i) {
            const Light& l = s.lights[i];
            Spec P(0.f);
            if (l.type == PBR_LIGHT_POINT) P = 4 * Pi * l.I;
            else if (l.type == PBR_LIGHT_INFINITE_AREA)   // InfiniteAreaLight.cpp:63-67
                P = (4 * Pi) * Pi * l.worldRadius * l.worldRadius * l.Lmap->Lookup(P2(.5f, .5f), .5f);
            else if (l.type == PBR_LIGHT_DIFFUSE_AREA) P = (float)(l.twoSided ? 2 : 1) * l.Lemit * l.area * Pi;
            f[i] = P.y();
        }
    }
    return Distribution1D(f.data(), (int)n);
}

static int DimsNeeded(const pbr_render_desc*) { return 1000; }   // PrimeTableSize (LowDiscrepancy.h:11)

// output transform (Integrator.cpp:313-344)
static void FilmOut(Spec colObj, int spp, float* rgb, uint8_t* rgba) {
    colObj /= (float)spp;
    rgb[0] = colObj[0]; rgb[1] = colObj[1]; rgb[2] = colObj[2];
    float xyz[3], out[3];
    xyz[0] = 0.412453f * colObj[0] + 0.357580f * colObj[1] + 0.180423f * colObj[2];
    xyz[1] = 0.212671f * colObj[0] + 0.715160f * colObj[1] + 0.072169f * colObj[2];
    xyz[2] = 0.019334f * colObj[0] + 0.119193f * colObj[1] + 0.950227f * colObj[2];
    out[0] = 3.240479f * xyz[0] - 1.537150f * xyz[1] - 0.498535f * xyz[2];
    out[1] = -0.969256f * xyz[0] + 1.875991f * xyz[1] + 0.041556f * xyz[2];
    out[2] = 0.055648f * xyz[0] - 0.204043f * xyz[1] + 1.057311f * xyz[2];
    for (int k = 0; k < 3; ++k) {
        float v = out[k];
        float g = (v <= 0.0031308f) ? 12.92f * v : 1.055f * t_pow(v, (1.f / 2.4f)) - 0.055f;
        float b = Clampf(255.f * g + 0.5f, 0.f, 255.f);
        rgba[k] = (uint8_t)(int)b;
    }
    rgba[3] = 255;
}

static Spec SampleLi(const Ctx& c, const Camera& cam, Halton& sampler, int x, int y) {
    P2 u01 = sampler.Get2D();                     // GetCameraSample (Sampler.cpp:10-21)
    P2 pFilm((float)x + u01.x, (float)y + u01.y);
    sampler.Get1D();                              // time
    P2 pLens = sampler.Get2D();
    Ray r = cam.generate(pFilm, pLens);
    if (c.integrator == PBR_INTEGRATOR_WHITTED) return WhittedLi(c, r, sampler, 0);
    if (c.integrator == PBR_INTEGRATOR_PATH) return PathLi(c, r, sampler);
    return VolPathLi(c, r, sampler);
}

struct RenderSetup {
    std::unique_ptr<Scene> scene;
    HaltonTables tab;
    SobolO sob;
    bool sobol = false;
    int spp = 0;          // GlobalSampler samplesPerPixel (Sobol: RoundUpPow2)
    Camera cam;
    Ctx ctx;
    std::vector<pbr_tile> tiles;
    std::vector<size_t> tileBase;
    size_t nPixels = 0;
};
static void Setup(RenderSetup& rs, const pbr_scene_desc* sd, const pbr_render_desc* rd) {
    if (rd->sampler != PBR_SAMPLER_HALTON && rd->sampler != PBR_SAMPLER_SOBOL) throw std::runtime_error("oracle: unknown sampler");
    rs.sobol = rd->sampler == PBR_SAMPLER_SOBOL;
    rs.spp = rd->spp;
    if (rs.sobol) {
        int p2 = 1;
        while (p2 < rs.spp) p2 <<= 1;
        rs.spp = p2;                                  // SobolSampler: GlobalSampler(RoundUpPow2(spp))
        rs.sob.init(rd->sobol_matrices, rd->sobol_dims, rd->camera.width, rd->camera.height);
    }
    rs.scene = BuildScene(sd);
    rs.tab.init(DimsNeeded(rd));
    rs.cam.init(rd->camera);
    rs.ctx.s = rs.scene.get();
    rs.ctx.integrator = rd->integrator;
    rs.ctx.maxDepth = rd->max_depth;
    rs.ctx.rrThreshold = rd->rr_threshold;
    rs.ctx.lightDistrib = MakeLightDistrib(*rs.scene, rd->light_strategy);
    if (rd->n_tiles > 0) rs.tiles.assign(rd->tiles, rd->tiles + rd->n_tiles);
    else rs.tiles.push_back(pbr_tile{0, 0, rd->camera.width, rd->camera.height});
    for (const pbr_tile& t : rs.tiles) { rs.tileBase.push_back(rs.nPixels); rs.nPixels += (size_t)(t.x1 - t.x0) * (t.y1 - t.y0); }
}

}  // namespace orc

using namespace orc;

extern "C" {

int oracle_sizeof_linear_bvh_node(void) { return (int)sizeof(OrcLinearBVHNode); }

static int RenderImpl(const pbr_scene_desc* sd, const pbr_render_desc* rd, float* rgb, uint8_t* rgba, int threads,
                      double* seconds, uint64_t* counters) {
    try {
        RenderSetup rs;
        Setup(rs, sd, rd);
        auto t0 = std::chrono::steady_clock::now();
        int spp = rs.spp;
        // flat list of pixels
        std::vector<std::pair<int, int>> px;
        px.reserve(rs.nPixels);
        for (const pbr_tile& t : rs.tiles)
            for (int y = t.y0; y < t.y1; ++y)
                for (int x = t.x0; x < t.x1; ++x) px.emplace_back(x, y);
        Counters total;
#ifdef _OPENMP
        if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
        {
            Counters local;
            if (counters) tl_counters = &local;
            Halton sampler;
            sampler.init(&rs.tab, spp, rd->camera.width, rd->camera.height);
            if (rs.sobol) sampler.sob = &rs.sob;
#pragma omp for schedule(dynamic, 16)
            for (long i = 0; i < (long)px.size(); ++i) {
                int x = px[i].first, y = px[i].second;
                sampler.StartPixel(x, y);
                Spec colObj(0.0f);
                do {
                    colObj += SampleLi(rs.ctx, rs.cam, sampler, x, y);
                } while (sampler.StartNextSample());
                float tmp[3];
                uint8_t tmp8[4];
                FilmOut(colObj, spp, tmp, tmp8);
                if (rgb) { rgb[3 * i] = tmp[0]; rgb[3 * i + 1] = tmp[1]; rgb[3 * i + 2] = tmp[2]; }
                if (rgba) { for (int k = 0; k < 4; ++k) rgba[4 * i + k] = tmp8[k]; }
            }
            tl_counters = nullptr;
#pragma omp critical
            {
                total.rays += local.rays; total.nodes += local.nodes; total.prims += local.prims; total.shading += local.shading;
            }
        }
        auto t1 = std::chrono::steady_clock::now();
        if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
        if (counters) { counters[0] = total.rays; counters[1] = total.nodes; counters[2] = total.prims; counters[3] = total.shading; }
        return 0;
    } catch (const std::exception&) {
        return PBR_E_INVALID;
    }
}

int oracle_render(const pbr_scene_desc* sd, const pbr_render_desc* rd, float* rgb, uint8_t* rgba, int threads,
                  double* seconds) {
    return RenderImpl(sd, rd, rgb, rgba, threads, seconds, nullptr);
}

int oracle_render_stats(const pbr_scene_desc* sd, const pbr_render_desc* rd, int threads, uint64_t* counters) {
    return RenderImpl(sd, rd, nullptr, nullptr, threads, nullptr, counters);
}

int oracle_li_pixel(const pbr_scene_desc* sd, const pbr_render_desc* rd, int x, int y, int sample, float* rgb) {
    try {
        RenderSetup rs;
        Setup(rs, sd, rd);
        Halton sampler;
        sampler.init(&rs.tab, rs.spp, rd->camera.width, rd->camera.height);
        if (rs.sobol) sampler.sob = &rs.sob;
        sampler.StartPixel(x, y);
        sampler.SetSampleNumber(sample);
        Spec L = SampleLi(rs.ctx, rs.cam, sampler, x, y);
        rgb[0] = L[0]; rgb[1] = L[1]; rgb[2] = L[2];
        return 0;
    } catch (const std::exception&) {
        return PBR_E_INVALID;
    }
}

int oracle_halton(int width, int height, int spp, int n, const int32_t* q, float* out) {
    int maxDim = 0;
    for (int i = 0; i < n; ++i) maxDim = std::max(maxDim, q[4 * i + 3]);
    if (maxDim >= 1000) return PBR_E_INVALID;
    HaltonTables tab;
    tab.init(std::max(maxDim + 1, 2));
    Halton h;
    h.init(&tab, spp, width, height);
    for (int i = 0; i < n; ++i) {
        int64_t idx = h.GetIndexForSample(q[4 * i], q[4 * i + 1], q[4 * i + 2]);
        out[i] = h.SampleDimension(idx, q[4 * i + 3]);
    }
    return 0;
}

int oracle_sobol(int width, int height, int n, const int32_t* q, const uint32_t* matrices, int dims, float* out,
                 int64_t* index_out) {
    try {
        SobolO s;
        s.init(matrices, dims, width, height);
        for (int i = 0; i < n; ++i) {
            int64_t idx = s.GetIndexForSample(q[4 * i], q[4 * i + 1], q[4 * i + 2]);
            if (index_out) index_out[i] = idx;
            out[i] = s.SampleDimension(idx, q[4 * i + 3], q[4 * i], q[4 * i + 1]);
        }
        return 0;
    } catch (const std::exception&) {
        return PBR_E_INVALID;
    }
}

int oracle_sobol_matrices(int dims, uint32_t* out) {
    std::vector<uint32_t> m;
    SobolO::builtin(dims, &m);
    std::memcpy(out, m.data(), m.size() * 4);
    return 0;
}

int oracle_halton_perms(int n_primes, uint16_t* out, int* n_out) {
    std::vector<uint16_t> p = RadicalInversePerms(n_primes);
    if (n_out) *n_out = (int)p.size();
    if (out) std::memcpy(out, p.data(), p.size() * 2);
    return 0;
}

int oracle_camera_rays(const pbr_camera_desc* cd, int n, const float* pfilm, float* out) {
    Camera cam;
    cam.init(*cd);
    for (int i = 0; i < n; ++i) {
        Ray r = cam.generate(P2(pfilm[2 * i], pfilm[2 * i + 1]), P2(0.5f, 0.5f));
        out[6 * i] = r.o.x; out[6 * i + 1] = r.o.y; out[6 * i + 2] = r.o.z;
        out[6 * i + 3] = r.d.x; out[6 * i + 4] = r.d.y; out[6 * i + 5] = r.d.z;
    }
    return 0;
}

int oracle_build_bvh(const pbr_scene_desc* sd, void* nodes_out, int* n_nodes, int32_t* prim_ids_out, int* n_prims) {
    try {
        std::unique_ptr<Scene> s = BuildScene(sd);
        if (n_nodes) *n_nodes = (int)s->nodes.size();
        if (n_prims) *n_prims = (int)s->primIds.size();
        if (nodes_out) std::memcpy(nodes_out, s->nodes.data(), s->nodes.size() * sizeof(OrcLinearBVHNode));
        if (prim_ids_out) for (size_t i = 0; i < s->primIds.size(); ++i) prim_ids_out[i] = s->primIds[i];
        return 0;
    } catch (const std::exception&) {
        return PBR_E_INVALID;
    }
}

int oracle_intersect(const pbr_scene_desc* sd, int n, const float* rays, float* out, int any_hit) {
    try {
        std::unique_ptr<Scene> s = BuildScene(sd);
        for (int i = 0; i < n; ++i) {
            const float* r = rays + 7 * i;
            Ray ray(V3(r[0], r[1], r[2]), V3(r[3], r[4], r[5]), r[6]);
            float* o = out + 5 * i;
            if (any_hit) {
                o[0] = IntersectP(*s, ray) ? 1.f : 0.f;
                o[1] = o[2] = o[3] = o[4] = 0;
            } else {
                // closest hit with barycentrics of the surviving primitive
                SurfaceInteraction si;
                bool hit = false;
                // replicate Intersect but keep the barycentrics
                V3 invDir(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
                int dirIsNeg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
                int stack[64], sp = 0, cur = 0, last = -1;
                float lb[3] = {0, 0, 0};
                while (true) {
                    const OrcLinearBVHNode* nd = &s->nodes[cur];
                    Bounds3 b;
                    b.pMin = V3(nd->pMin[0], nd->pMin[1], nd->pMin[2]);
                    b.pMax = V3(nd->pMax[0], nd->pMax[1], nd->pMax[2]);
                    if (BoundsIntersectP(b, ray, invDir, dirIsNeg)) {
                        if (nd->nPrimitives > 0) {
                            for (int k = 0; k < nd->nPrimitives; ++k) {
                                bool rec = false;
                                float bb[3];
                                if (PrimIntersect(*s, nd->offset + k, ray, &si, &rec, bb)) {
                                    hit = true; last = nd->offset + k; lb[0] = bb[0]; lb[1] = bb[1]; lb[2] = bb[2];
                                }
                            }
                            if (sp == 0) break;
                            cur = stack[--sp];
                        } else if (dirIsNeg[nd->axis]) { stack[sp++] = cur + 1; cur = nd->offset; }
                        else { stack[sp++] = nd->offset; cur = cur + 1; }
                    } else {
                        if (sp == 0) break;
                        cur = stack[--sp];
                    }
                }
                o[0] = hit ? 1.f : 0.f;
                o[1] = hit ? ray.tMax : 0.f;
                o[2] = hit ? (float)s->primIds[last] : -1.f;
                o[3] = hit ? lb[1] : 0.f;
                o[4] = hit ? lb[2] : 0.f;
            }
        }
        return 0;
    } catch (const std::exception&) {
        return PBR_E_INVALID;
    }
}

int oracle_triangle_test(const float* tri, const float* r, float* out) {
    Ray ray(V3(r[0], r[1], r[2]), V3(r[3], r[4], r[5]), r[6]);
    float t = 0, b0 = 0, b1 = 0, b2 = 0;
    bool h = TriangleTest(V3(tri[0], tri[1], tri[2]), V3(tri[3], tri[4], tri[5]), V3(tri[6], tri[7], tri[8]), ray, &t, &b0, &b1, &b2);
    out[0] = h ? 1.f : 0.f; out[1] = t; out[2] = b0; out[3] = b1; out[4] = b2;
    return 0;
}

}  // extern "C"
