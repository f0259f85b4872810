// pbr_scene.cpp — host half of pbr_hip_upload_scene: turns the reference-shaped scene descriptor
// into the flattened HBM layout (pbr_layout.h).
//
// The BVH must come out node-for-node identical to BVHAccel (Accelerator/BVHAccel.cpp:57-283):
// the F8 tie rule (later primitive wins on t == tMax) makes the traversal order — and so the
// topology — observable in the image.  The builder below is iterative and writes nodes directly
// in depth-first preorder (the reference's flatten order), but performs the same bucket SAH,
// the same std::partition / std::nth_element calls on the same element order, so the layout is
// identical.
#include "pbr_scene.h"
#include "pbr_material.h"
#include "pbr_sobol_jk.h"
#include "pbr_xform.h"

#include <algorithm>
#include <cstring>
#include <limits>

namespace pbr {

namespace {

using namespace xform;

struct Box {
    f3 lo, hi;
    Box() {
        float big = std::numeric_limits<float>::max(), low = std::numeric_limits<float>::lowest();
        lo = mk(big, big, big);
        hi = mk(low, low, low);
    }
    void add(f3 p) { lo = vmin(lo, p); hi = vmax(hi, p); }
    void add(const Box& b) { lo = vmin(lo, b.lo); hi = vmax(hi, b.hi); }
    float area() const { f3 d = hi - lo; return 2 * (d.x * d.y + d.x * d.z + d.y * d.z); }
    int longest() const {
        f3 d = hi - lo;
        if (d.x > d.y && d.x > d.z) return 0;
        if (d.y > d.z) return 1;
        return 2;
    }
    float rel(f3 p, int axis) const {   // Bounds3::Offset(p)[axis]
        float o = get(p, axis) - get(lo, axis);
        float ext_hi = get(hi, axis), ext_lo = get(lo, axis);
        if (ext_hi > ext_lo) o /= ext_hi - ext_lo;
        return o;
    }
};

struct Item {                 // BVHPrimitiveInfo
    size_t id;
    Box box;
    f3 c;
};

struct PrimRef { int shape, tri; };

void fail(const std::string& why) { throw std::invalid_argument(why); }

// The same tree collapsed two levels at a time for the closest/any-hit traversal (pbr_device.h
// traverse_quad): a quad node stands for binary interior node N and holds the boxes of N's
// grandchildren — or of a child itself where that child is a leaf — in the slots
// [A.near-side, A.far-side, B.near-side, B.far-side] (A = N's first child, B = its second), plus
// the split axes of N, A and B, so the traversal recovers BVHAccel's near-first order from the
// ray's direction signs.  Layout, 8 float4 (128 B, one L2 line) per node:
//   [0..5] lo.x, lo.y, lo.z, hi.x, hi.y, hi.z of the four slots (SoA)
//   [6]    slot references: quad-node index, or kLeafRef | first primitive slot
//   [7]    .x = axN | axA << 2 | axB << 4 | validMask << 8 (slot 1 / 3 is empty when A / B is a leaf)
// The child boxes are nested inside their parent's, so a slot that passes its slab test implies
// the skipped parent test passes too; primitive tests keep the reference's order (see traverse_quad).
template <class Ref>
void build_quad_nodes(HostScene* S, Ref&& binRef) {
    const std::vector<LinearBVHNode>& L = S->nodes;
    S->quad.clear();
    S->quadRootRef = binRef(0);
    S->quadStackNeed = 0;
    if (L.empty() || L[0].nPrimitives > 0) return;
    std::vector<int32_t> qid(L.size(), -1);
    int nQuad = 0;
    // quad nodes exist for the root and every interior grandchild of a quad node (preorder)
    std::vector<int> todo{0};
    std::vector<int> order;
    while (!todo.empty()) {
        int i = todo.back();
        todo.pop_back();
        qid[i] = nQuad++;
        order.push_back(i);
        int kids[2] = {i + 1, L[i].offset};
        for (int k = 1; k >= 0; --k) {
            int c = kids[k];
            if (L[c].nPrimitives > 0) continue;
            int g[2] = {c + 1, L[c].offset};
            for (int m = 1; m >= 0; --m)
                if (L[g[m]].nPrimitives == 0) todo.push_back(g[m]);
        }
    }
    auto ref = [&](int i) -> int32_t { return L[i].nPrimitives > 0 ? binRef(i) : qid[i]; };
    S->quad.assign((size_t)nQuad * 32, 0.f);
    for (int i : order) {
        float* w = &S->quad[(size_t)qid[i] * 32];
        int kids[2] = {i + 1, L[i].offset};
        int32_t refs[4] = {0, 0, 0, 0};
        int axes[2] = {0, 0}, mask = 0;
        for (int k = 0; k < 2; ++k) {
            int c = kids[k];
            int slots[2] = {-1, -1};
            if (L[c].nPrimitives > 0) slots[0] = c;
            else { slots[0] = c + 1; slots[1] = L[c].offset; axes[k] = L[c].axis; }
            for (int m = 0; m < 2; ++m) {
                int s = 2 * k + m, n = slots[m];
                if (n < 0) {   // empty slot: an inverted box, never tested (validMask)
                    for (int a = 0; a < 3; ++a) { w[4 * a + s] = 1.f; w[12 + 4 * a + s] = -1.f; }
                    continue;
                }
                for (int a = 0; a < 3; ++a) { w[4 * a + s] = L[n].pMin[a]; w[12 + 4 * a + s] = L[n].pMax[a]; }
                refs[s] = ref(n);
                mask |= 1 << s;
            }
        }
        std::memcpy(&w[24], refs, 16);
        int32_t meta = (int32_t)L[i].axis | axes[0] << 2 | axes[1] << 4 | mask << 8;
        std::memcpy(&w[28], &meta, 4);
    }
    // Stack need of the quad walk: entering one slot of node Q pushes at most the other valid
    // slots, which stay on the stack while any of Q's subtrees is walked, so need(Q) = (valid
    // slots − 1) + max need of its quad children.  Children follow their parent in preorder.
    std::vector<int> need(nQuad, 0);
    for (size_t k = order.size(); k-- > 0;) {
        const int i = order[k];
        const float* w = &S->quad[(size_t)qid[i] * 32];
        int32_t refs[4], meta;
        std::memcpy(refs, &w[24], 16);
        std::memcpy(&meta, &w[28], 4);
        int valid = 0, deeper = 0;
        for (int s = 0; s < 4; ++s) {
            if (!((meta >> (8 + s)) & 1)) continue;
            ++valid;
            if (refs[s] >= 0) deeper = std::max(deeper, need[refs[s]]);
        }
        need[qid[i]] = valid - 1 + deeper;
    }
    S->quadStackNeed = need[qid[0]];
    S->quadRootRef = qid[0];
}

// The same tree re-laid out for traversal: each interior node carries both children's boxes (so a
// child is box-tested from its parent, before its own record is fetched) and child references
// (interior rank, or kLeafRef | first primitive slot).  The last primitive of every leaf gets
// PRIM_LEAF_END in its v0.w flags.  Visit order is unchanged (pbr_device.h traverse).
void build_wide_nodes(HostScene* S) {
    const std::vector<LinearBVHNode>& L = S->nodes;
    S->wide.clear();
    S->rootRef = 0;
    S->binaryStackNeed = 0;
    if (L.empty()) return;
    {   // interior levels on the deepest root-to-leaf path (the binary walk pushes one far child per level)
        std::vector<int> depth(L.size(), 0);
        for (size_t i = 0; i < L.size(); ++i) {   // preorder: a parent precedes its children
            if (L[i].nPrimitives > 0) continue;
            depth[i + 1] = depth[L[i].offset] = depth[i] + 1;
            S->binaryStackNeed = std::max(S->binaryStackNeed, depth[i] + 1);
        }
    }
    std::vector<int> rank(L.size(), -1);
    int nInterior = 0;
    for (size_t i = 0; i < L.size(); ++i)
        if (L[i].nPrimitives == 0) rank[i] = nInterior++;
    auto ref = [&](int i) -> int32_t {
        if (L[i].nPrimitives > 0) return (int32_t)(kLeafRef | (uint32_t)L[i].offset);
        return rank[i];
    };
    for (size_t i = 0; i < L.size(); ++i) {
        if (L[i].nPrimitives == 0) continue;
        // every leaf ends at its last slot; slots are contiguous per leaf
        int last = L[i].offset + L[i].nPrimitives - 1;
        uint32_t f;
        std::memcpy(&f, &S->triVerts[(size_t)last * 12 + 3], 4);
        f |= PRIM_LEAF_END;
        std::memcpy(&S->triVerts[(size_t)last * 12 + 3], &f, 4);
    }
    if ((uint32_t)S->primIds.size() >= kLeafRef) fail("too many primitives for the traversal layout");
    S->wide.assign((size_t)nInterior * 16, 0.f);
    for (size_t i = 0; i < L.size(); ++i) {
        if (L[i].nPrimitives > 0) continue;
        const LinearBVHNode& c0 = L[i + 1];
        const LinearBVHNode& c1 = L[L[i].offset];
        float* w = &S->wide[(size_t)rank[i] * 16];
        w[0] = c0.pMin[0]; w[1] = c0.pMin[1]; w[2] = c0.pMin[2]; w[3] = c0.pMax[0];
        w[4] = c0.pMax[1]; w[5] = c0.pMax[2]; w[6] = c1.pMin[0]; w[7] = c1.pMin[1];
        w[8] = c1.pMin[2]; w[9] = c1.pMax[0]; w[10] = c1.pMax[1]; w[11] = c1.pMax[2];
        int32_t r0 = ref((int)i + 1), r1 = ref(L[i].offset), ax = L[i].axis;
        std::memcpy(&w[12], &r0, 4);
        std::memcpy(&w[13], &r1, 4);
        std::memcpy(&w[14], &ax, 4);
    }
    S->rootRef = ref(0);
    build_quad_nodes(S, ref);
}

// Bucketed SAH builder writing LinearBVHNodes in depth-first preorder.
class SahBuilder {
  public:
    SahBuilder(std::vector<Item>& items, int maxPrims, int splitMethod, std::vector<LinearBVHNode>* nodes, std::vector<int32_t>* order)
        : it_(items), maxPrims_(std::min(255, maxPrims)), split_(splitMethod), nodes_(nodes), order_(order) {}

    void run() {
        nodes_->clear();
        order_->clear();
        leaves_.clear();
        if (it_.empty()) return;
        // explicit DFS: each task is (start, end, parentIndexToPatch or -1)
        struct Task { int start, end, patch; };
        std::vector<Task> todo;
        todo.push_back({0, (int)it_.size(), -1});
        while (!todo.empty()) {
            Task t = todo.back();
            todo.pop_back();
            int me = (int)nodes_->size();
            nodes_->push_back(LinearBVHNode());
            if (t.patch >= 0) (*nodes_)[t.patch].offset = me;   // secondChildOffset
            int mid, axis;
            Box box;
            if (!split(t.start, t.end, &mid, &axis, &box)) {
                emit_leaf(me, t.start, t.end, box);
                continue;
            }
            LinearBVHNode& n = (*nodes_)[me];
            put_box(n, box);
            n.axis = (uint8_t)axis;
            n.nPrimitives = 0;
            // right child is visited after the whole left subtree: push it first
            todo.push_back({mid, t.end, me});
            todo.push_back({t.start, mid, -1});
        }
        // Primitive order.  BVHAccel::recursiveBuild appends a leaf's primitives to orderedPrims
        // when the leaf is built, and builds an interior node's children inside one call,
        // InitInterior(dim, recursiveBuild(start, mid), recursiveBuild(mid, end))
        // (BVHAccel.cpp:250-254), whose arguments GCC and MSVC evaluate right to left: the second
        // child's subtree comes first.  Over the whole tree that is the leaves in reverse of the
        // left-first order collected above, each leaf's primitives in range order.  (The
        // partitions are per disjoint range, so the build order changes nothing else.)
        for (size_t k = leaves_.size(); k-- > 0;) {
            const Leaf& l = leaves_[k];
            (*nodes_)[l.node].offset = (int32_t)order_->size();
            for (int i = l.start; i < l.end; ++i) order_->push_back((int32_t)it_[i].id);
        }
    }

  private:
    static void put_box(LinearBVHNode& n, const Box& b) {
        n.pMin[0] = b.lo.x; n.pMin[1] = b.lo.y; n.pMin[2] = b.lo.z;
        n.pMax[0] = b.hi.x; n.pMax[1] = b.hi.y; n.pMax[2] = b.hi.z;
    }
    void emit_leaf(int me, int s, int e, const Box& box) {
        LinearBVHNode& n = (*nodes_)[me];
        put_box(n, box);
        n.nPrimitives = (uint16_t)(e - s);
        leaves_.push_back({me, s, e});   // primitivesOffset: assigned in build order (run())
    }
    // Decide leaf vs interior for [s,e); on interior, partitions it_ and returns the split.
    bool split(int s, int e, int* mid, int* axis, Box* box) {
        Box b;
        for (int i = s; i < e; ++i) b.add(it_[i].box);
        *box = b;
        int n = e - s;
        if (n == 1) return false;
        Box cb;
        for (int i = s; i < e; ++i) cb.add(it_[i].c);
        int dim = cb.longest();
        *axis = dim;
        if (get(cb.hi, dim) == get(cb.lo, dim)) return false;
        Item* first = it_.data() + s;
        Item* last = it_.data() + e;
        auto byCentroid = [dim](const Item& a, const Item& c) { return get(a.c, dim) < get(c.c, dim); };
        if (split_ == PBR_SPLIT_MIDDLE) {   // BVHAccel.cpp:136-148, falling through to EqualCounts
            float pmid = (get(cb.lo, dim) + get(cb.hi, dim)) / 2;
            Item* pm = std::partition(first, last, [dim, pmid](const Item& p) { return get(p.c, dim) < pmid; });
            *mid = (int)(pm - it_.data());
            if (*mid != s && *mid != e) return true;
        }
        if (split_ == PBR_SPLIT_MIDDLE || split_ == PBR_SPLIT_EQUAL_COUNTS) {   // :149-158
            *mid = (s + e) / 2;
            std::nth_element(first, it_.data() + *mid, last, byCentroid);
            return true;
        }
        if (n <= 2) {
            *mid = (s + e) / 2;
            std::nth_element(first, it_.data() + *mid, last,
                             [dim](const Item& a, const Item& c) { return get(a.c, dim) < get(c.c, dim); });
            return true;
        }
        const int NB = 12;
        int cnt[NB] = {0};
        Box bb[NB];
        for (int i = s; i < e; ++i) {
            int k = NB * cb.rel(it_[i].c, dim);
            if (k == NB) k = NB - 1;
            cnt[k]++;
            bb[k].add(it_[i].box);
        }
        float cost[NB - 1];
        for (int i = 0; i < NB - 1; ++i) {
            Box b0, b1;
            int c0 = 0, c1 = 0;
            for (int j = 0; j <= i; ++j) { b0.add(bb[j]); c0 += cnt[j]; }
            for (int j = i + 1; j < NB; ++j) { b1.add(bb[j]); c1 += cnt[j]; }
            cost[i] = 1 + (c0 * b0.area() + c1 * b1.area()) / b.area();
        }
        float best = cost[0];
        int bestK = 0;
        for (int i = 1; i < NB - 1; ++i)
            if (cost[i] < best) { best = cost[i]; bestK = i; }
        float leafCost = n;
        if (!(n > maxPrims_ || best < leafCost)) return false;
        Item* pm = std::partition(first, last, [=](const Item& p) {
            int k = NB * cb.rel(p.c, dim);
            if (k == NB) k = NB - 1;
            return k <= bestK;
        });
        *mid = (int)(pm - it_.data());
        return true;
    }

    struct Leaf { int node, start, end; };
    std::vector<Leaf> leaves_;
    std::vector<Item>& it_;
    int maxPrims_;
    int split_;
    std::vector<LinearBVHNode>* nodes_;
    std::vector<int32_t>* order_;
};

// A material's constant parameters (ConstantTexture values, Material/*.cpp constructors).
MatParams mat_params(const pbr_material_desc& m) {
    MatParams p;
    std::memset(&p, 0, sizeof(p));
    p.type = m.type;
    for (int i = 0; i < 3; ++i) {
        p.Kd[i] = m.Kd[i]; p.Kr[i] = m.Kr[i]; p.Kt[i] = m.Kt[i]; p.Ks[i] = m.Ks[i];
        p.metal_eta[i] = m.metal_eta[i]; p.metal_k[i] = m.metal_k[i];
    }
    p.sigma = m.sigma; p.eta = m.eta;
    p.roughness = m.roughness; p.uroughness = m.uroughness; p.vroughness = m.vroughness;
    p.has_uv_roughness = m.has_uv_roughness; p.remap_roughness = m.remap_roughness;
    return p;
}

// Material::ComputeScatteringFunctions with constant textures folded (Material/*.cpp)
MatTemplate material_template(const pbr_material_desc& m, bool multi) {
    MatTemplate t;
    if (!pbr::material_template(mat_params(m), multi, &t)) fail("unknown material type");
    return t;
}

// Distribution1D construction (Sampling.h:77-90)
void distribution1d(const std::vector<float>& f, std::vector<float>* cdf, float* funcInt) {
    int n = (int)f.size();
    cdf->assign(n + 1, 0.f);
    (*cdf)[0] = 0;
    for (int i = 1; i < n + 1; ++i) (*cdf)[i] = (*cdf)[i - 1] + f[i - 1] / n;
    *funcInt = (*cdf)[n];
    if (*funcInt == 0) for (int i = 1; i < n + 1; ++i) (*cdf)[i] = float(i) / float(n);
    else for (int i = 1; i < n + 1; ++i) (*cdf)[i] /= *funcInt;
}

}  // namespace

// InitInterior (BVHAccel.cpp:33-38) overwrites an interior node's box with Union(c0->bounds,
// c1->bounds).  The builders reduce the range before partitioning it, which gives the same values;
// only the sign of a zero can differ (Union keeps its first operand on ties, -0 == +0), so the
// boxes are rebuilt from the children, children first (reverse preorder).
void interior_bounds_from_children(std::vector<LinearBVHNode>* nodes) {
    std::vector<LinearBVHNode>& L = *nodes;
    for (size_t i = L.size(); i-- > 0;) {
        if (L[i].nPrimitives > 0) continue;
        const LinearBVHNode& c0 = L[i + 1];
        const LinearBVHNode& c1 = L[L[i].offset];
        for (int a = 0; a < 3; ++a) {
            L[i].pMin[a] = mn(c0.pMin[a], c1.pMin[a]);
            L[i].pMax[a] = mx(c0.pMax[a], c1.pMax[a]);
        }
    }
}

void host_build_bvh(const std::vector<float>& primBounds, int maxPrims, std::vector<LinearBVHNode>* nodes,
                    std::vector<int32_t>* primIds, int splitMethod) {
    const size_t np = primBounds.size() / 6;
    std::vector<Item> items(np);
    for (size_t i = 0; i < np; ++i) {   // BVHPrimitiveInfo (BVHAccel.cpp:24-31)
        const float* p = &primBounds[i * 6];
        items[i].id = i;
        items[i].box.lo = mk(p[0], p[1], p[2]);
        items[i].box.hi = mk(p[3], p[4], p[5]);
        items[i].c = .5f * items[i].box.lo + .5f * items[i].box.hi;
    }
    SahBuilder(items, maxPrims, splitMethod, nodes, primIds).run();
    interior_bounds_from_children(nodes);
}

// A caller-built BVHAccel (pbr_scene_desc::bvh_nodes): the reference's flattened tree over the
// primitives in the given (orderedPrims) order.  Checked before use: a preorder tree (first child
// right after its parent, the second at `offset`), every node reached once, the leaves' primitive
// ranges tiling 0..n-1 (recursiveBuild's arguments are evaluated right to left, so preorder leaves
// need not be in offset order), each leaf box bit-equal to the union of its primitives' bounds
// (BVHAccel.cpp:189-196 computes it with the same Union as Triangle::WorldBound here, so a flattening
// that moved a vertex fails).  Interior boxes are kept as given.
void adopt_bvh(const pbr_scene_desc* d, const std::vector<float>& primBounds, std::vector<LinearBVHNode>* nodes,
               std::vector<int32_t>* primIds) {
    const size_t np = primBounds.size() / 6;
    if (d->n_bvh_nodes <= 0 || (size_t)d->n_bvh_nodes > 2 * np + 1) fail("bvh_nodes: bad node count");
    const LinearBVHNode* in = static_cast<const LinearBVHNode*>(d->bvh_nodes);
    nodes->assign(in, in + d->n_bvh_nodes);
    const std::vector<LinearBVHNode>& L = *nodes;
    std::vector<unsigned char> covered(np, 0);
    size_t nCovered = 0;
    int visited = 0;
    std::vector<int> stack{0};
    while (!stack.empty()) {
        const int i = stack.back();
        stack.pop_back();
        if (i < 0 || i >= d->n_bvh_nodes || visited++ >= d->n_bvh_nodes) fail("bvh_nodes: not a tree");
        const LinearBVHNode& n = L[i];
        if (n.nPrimitives > 0) {
            if (n.offset < 0 || (size_t)n.offset + n.nPrimitives > np) fail("bvh_nodes: a leaf indexes past the primitives");
            Box b;
            for (int k = 0; k < n.nPrimitives; ++k) {
                const size_t p = (size_t)n.offset + k;
                if (covered[p]++) fail("bvh_nodes: a primitive in two leaves");
                ++nCovered;
                const float* pb = &primBounds[p * 6];
                Box e;
                e.lo = mk(pb[0], pb[1], pb[2]);
                e.hi = mk(pb[3], pb[4], pb[5]);
                if (k == 0) b = e;
                else b.add(e);
            }
            const float box[6] = {b.lo.x, b.lo.y, b.lo.z, b.hi.x, b.hi.y, b.hi.z};
            if (std::memcmp(box, n.pMin, 12) != 0 || std::memcmp(box + 3, n.pMax, 12) != 0)
                fail("bvh_nodes: a leaf box is not its primitives' bounds");
        } else {
            if (n.offset <= i + 1 || n.axis > 2) fail("bvh_nodes: bad interior node");
            stack.push_back(n.offset);   // second child after the first one's subtree (preorder)
            stack.push_back(i + 1);
        }
    }
    if (visited != d->n_bvh_nodes || nCovered != np) fail("bvh_nodes: the tree does not cover every node and primitive");
    primIds->resize(np);
    for (size_t i = 0; i < np; ++i) (*primIds)[i] = (int32_t)i;
}

void build_host_scene(const pbr_scene_desc* d, HostScene* S, const BvhBuildFn* bvh) {
    if (!d) fail("null scene");
    if (d->abi_version != PBR_HIP_ABI_VERSION) fail("abi_version mismatch");
    if (d->n_shapes < 0 || (d->n_shapes > 0 && !d->shapes)) fail("bad shapes");
    *S = HostScene();
    const int ns = d->n_shapes;
    // 1. world-space vertex bake (TriangleMesh ctor, Triangle.cpp:12-44) + primitive list
    std::vector<std::vector<f3>> world(ns);
    std::vector<PrimRef> prims;
    std::vector<int> firstPrim(ns, 0);
    std::vector<int> flip(ns, 0);
    S->spheres.clear();
    std::vector<int> sphereIndex(ns, -1);
    for (int i = 0; i < ns; ++i) {
        const pbr_shape_desc& sd = d->shapes[i];
        Mat o2w = from_rows(sd.object_to_world.m);
        flip[i] = (sd.reverse_orientation != 0) ^ swaps_handedness(o2w);
        firstPrim[i] = (int)prims.size();
        if (sd.material >= d->n_materials) fail("material index out of range");
        if (sd.type == PBR_SHAPE_TRIANGLE_MESH) {
            if (sd.N) fail("per-vertex normals are not supported");
            if (sd.n_triangles < 0 || sd.n_vertices < 0 || (sd.n_triangles && (!sd.indices || !sd.P))) fail("bad mesh");
            world[i].resize(sd.n_vertices);
            for (int v = 0; v < sd.n_vertices; ++v)
                world[i][v] = xf_point(&o2w.a[0][0], mk(sd.P[3 * v], sd.P[3 * v + 1], sd.P[3 * v + 2]));
            for (int t = 0; t < sd.n_triangles; ++t) {
                for (int k = 0; k < 3; ++k) {
                    int vi = sd.indices[3 * t + k];
                    if (vi < 0 || vi >= sd.n_vertices) fail("vertex index out of range");
                }
                prims.push_back({i, t});
            }
        } else if (sd.type == PBR_SHAPE_SPHERE) {
            if (sd.area_light_first >= 0) fail("sphere area lights are not supported");
            SphereRec r;
            std::memset(&r, 0, sizeof(r));
            std::memcpy(r.o2w, sd.object_to_world.m, 64);
            std::memcpy(r.w2o, sd.object_to_world.m_inv, 64);
            r.radius = sd.radius;
            r.flip = flip[i];
            sphereIndex[i] = (int)S->spheres.size();
            S->spheres.push_back(r);
            prims.push_back({i, -1});
        } else {
            fail("unknown shape type");
        }
    }
    const int np = (int)prims.size();
    auto vert = [&](const PrimRef& p, int k) {
        const pbr_shape_desc& sd = d->shapes[p.shape];
        return world[p.shape][sd.indices[3 * p.tri + k]];
    };
    // 2. SAH BVH over primitive world bounds
    S->primBounds.clear();
    S->primBounds.reserve((size_t)np * 6);
    for (int i = 0; i < np; ++i) {
        Box b;
        if (prims[i].tri >= 0) {   // Triangle::WorldBound (Triangle.cpp:55-62)
            f3 p0 = vert(prims[i], 0), p1 = vert(prims[i], 1), p2 = vert(prims[i], 2);
            b.lo = vmin(p0, p1); b.hi = vmax(p0, p1);
            b.add(p2);
        } else {                   // Shape::WorldBound → Transform(Bounds3f)
            const SphereRec& r = S->spheres[sphereIndex[prims[i].shape]];
            float rad = r.radius;
            f3 lo = mk(-rad, -rad, -rad), hi = mk(rad, rad, rad);
            f3 corners[8] = {mk(lo.x, lo.y, lo.z), mk(hi.x, lo.y, lo.z), mk(lo.x, hi.y, lo.z), mk(lo.x, lo.y, hi.z),
                             mk(lo.x, hi.y, hi.z), mk(hi.x, hi.y, lo.z), mk(hi.x, lo.y, hi.z), mk(hi.x, hi.y, hi.z)};
            f3 c0 = xf_point(r.o2w, corners[0]);
            b.lo = c0; b.hi = c0;
            for (int k = 1; k < 8; ++k) b.add(xf_point(r.o2w, corners[k]));
        }
        S->primBounds.insert(S->primBounds.end(), {b.lo.x, b.lo.y, b.lo.z, b.hi.x, b.hi.y, b.hi.z});
    }
    const int maxPrims = d->max_prims_in_node > 0 ? d->max_prims_in_node : 1;
    if (d->split_method < PBR_SPLIT_SAH || d->split_method > PBR_SPLIT_EQUAL_COUNTS) fail("unknown split method");
    // the device builder is the SAH one (HLBVH is SAH in the reference); Middle / EqualCounts build here
    const bool sah = d->split_method == PBR_SPLIT_SAH || d->split_method == PBR_SPLIT_HLBVH;
    if (d->bvh_nodes) adopt_bvh(d, S->primBounds, &S->nodes, &S->primIds);
    else if (bvh && sah) (*bvh)(S->primBounds, maxPrims, &S->nodes, &S->primIds);
    else host_build_bvh(S->primBounds, maxPrims, &S->nodes, &S->primIds, d->split_method);
    if (S->primIds.size() != (size_t)np) fail("BVH build returned a wrong primitive count");
    // 3. primitive payloads in BVH order
    std::vector<int>& slotOf = S->slotOf;
    slotOf.assign(np, -1);
    bool anyUV = false;
    for (int i = 0; i < ns; ++i) if (d->shapes[i].type == PBR_SHAPE_TRIANGLE_MESH && d->shapes[i].UV) anyUV = true;
    S->triVerts.assign((size_t)np * 12, 0.f);
    S->primInfo.assign((size_t)np * 4, 0);
    if (anyUV) S->triUV.assign((size_t)np * 6, 0.f);
    for (int slot = 0; slot < np; ++slot) {
        const PrimRef& p = prims[S->primIds[slot]];
        slotOf[S->primIds[slot]] = slot;
        const pbr_shape_desc& sd = d->shapes[p.shape];
        int flags = flip[p.shape] ? PRIM_FLIP : 0;
        float* tv = &S->triVerts[(size_t)slot * 12];
        if (p.tri >= 0) {
            for (int k = 0; k < 3; ++k) {
                f3 v = vert(p, k);
                tv[4 * k] = v.x; tv[4 * k + 1] = v.y; tv[4 * k + 2] = v.z; tv[4 * k + 3] = 0.f;
            }
            if (sd.UV) {
                flags |= PRIM_HAS_UV;
                for (int k = 0; k < 3; ++k) {
                    int vi = sd.indices[3 * p.tri + k];
                    S->triUV[(size_t)slot * 6 + 2 * k] = sd.UV[2 * vi];
                    S->triUV[(size_t)slot * 6 + 2 * k + 1] = sd.UV[2 * vi + 1];
                }
            }
        } else {
            flags |= PRIM_SPHERE;
            tv[0] = bitsf((uint32_t)sphereIndex[p.shape]);
        }
        tv[3] = bitsf((uint32_t)flags);   // the traversal reads the primitive flags from v0.w
        int32_t* pi = &S->primInfo[(size_t)slot * 4];
        pi[0] = flags;
        // a PBR_MAT_NONE material is material == nullptr (a medium boundary): stored as -1 like no index
        pi[1] = (sd.material >= 0 && sd.material < d->n_materials && d->materials[sd.material].type == PBR_MAT_NONE) ? -1 : sd.material;
        pi[2] = (p.tri >= 0 && sd.area_light_first >= 0) ? sd.area_light_first + p.tri : -1;
        if (sd.medium_inside >= d->n_media || sd.medium_outside >= d->n_media) fail("medium index out of range");
        pi[3] = (int32_t)(((uint32_t)(sd.medium_inside & 0xffff)) | ((uint32_t)(sd.medium_outside & 0xffff) << 16));
    }
    build_wide_nodes(S);
    for (int slot = 0; slot < np; ++slot) {
        int m = S->primInfo[(size_t)slot * 4 + 1];
        if (m < 0 || d->materials[m].type == PBR_MAT_NONE) S->anyNoMaterial = true;
    }
    // 4. materials → lobe templates for allowMultipleLobes = false / true
    S->materials.clear();
    for (int m = 0; m < d->n_materials; ++m) {
        S->materials.push_back(material_template(d->materials[m], false));
        S->materials.push_back(material_template(d->materials[m], true));
    }
    // 4b. image textures (ImageTexture, Texture/ImageTexture.cpp) and the materials that read them:
    //     those get their lobes per hit (pbr_device.h textured_template)
    if (d->n_textures < 0 || (d->n_textures > 0 && !d->textures)) fail("bad textures");
    S->textures.assign(d->n_textures, TexDev());
    S->texTexels.clear();
    for (int i = 0; i < d->n_textures; ++i) build_image_texture(d->textures[i], &S->textures[i], &S->texTexels);
    S->texMats.clear();
    bool anyTex = false;
    for (int m = 0; m < d->n_materials; ++m)
        for (int k = 0; k < PBR_TEX_SLOTS; ++k) anyTex |= d->materials[m].tex[k] != 0;
    if (anyTex) {
        // which slots each material type reads (Material/*.cpp ComputeScatteringFunctions)
        static const int reads[6][PBR_TEX_SLOTS] = {
            {0, 0, 0, 0, 0, 0}, {1, 0, 0, 0, 1, 0}, {0, 0, 1, 0, 0, 0}, {0, 0, 1, 1, 0, 0}, {0, 0, 0, 0, 0, 0}, {1, 1, 0, 0, 0, 1}};
        static const int isFloatSlot[PBR_TEX_SLOTS] = {0, 0, 0, 0, 1, 1};
        S->texMats.resize(d->n_materials);
        for (int m = 0; m < d->n_materials; ++m) {
            const pbr_material_desc& md = d->materials[m];
            TexMat& tm = S->texMats[m];
            tm.p = mat_params(md);
            bool textured = false;
            for (int k = 0; k < PBR_TEX_SLOTS; ++k) {
                tm.tex[k] = -1;
                if (!md.tex[k]) continue;
                const int ti = md.tex[k] - 1;
                if (ti < 0 || ti >= d->n_textures) fail("texture index out of range");
                if (md.type < 0 || md.type > PBR_MAT_PLASTIC || !reads[md.type][k])
                    fail("this material type has no such texture slot");
                if ((d->textures[ti].is_float != 0) != (isFloatSlot[k] != 0))
                    fail("texture slot needs a " + std::string(isFloatSlot[k] ? "float" : "RGB") + " texture");
                tm.tex[k] = ti;
                textured = true;
            }
            S->materials[2 * m].textured = S->materials[2 * m + 1].textured = textured ? 1 : 0;
            if (!textured) continue;
            for (int i = 0; i < ns; ++i)
                if (d->shapes[i].material == m && d->shapes[i].type != PBR_SHAPE_TRIANGLE_MESH)
                    fail("image textures are supported on triangle meshes only (the reference's sphere is a stub)");
        }
    }
    // 5. media (HomogeneousMedium.h: sigma_t = sigma_s + sigma_a)
    for (int m = 0; m < d->n_media; ++m) {
        const pbr_medium_desc& md = d->media[m];
        for (int k = 0; k < 3; ++k) S->media.push_back(md.sigma_a[k]);
        for (int k = 0; k < 3; ++k) S->media.push_back(md.sigma_s[k]);
        for (int k = 0; k < 3; ++k) S->media.push_back(md.sigma_s[k] + md.sigma_a[k]);
        S->media.push_back(md.g);
    }
    // 6. lights
    for (int li = 0; li < d->n_lights; ++li) {
        const pbr_light_desc& ld = d->lights[li];
        DLight L;
        std::memset(&L, 0, sizeof(L));
        L.type = ld.type;
        L.medIn = ld.medium_inside;
        L.medOut = ld.medium_outside;
        L.primSlot = -1;
        if (ld.type == PBR_LIGHT_POINT) {
            f3 p = xf_point(ld.light_to_world.m, mk(0, 0, 0));
            L.p[0] = p.x; L.p[1] = p.y; L.p[2] = p.z;
            mt_put3(L.L, ld.I);
            float P[3];
            for (int k = 0; k < 3; ++k) P[k] = (4 * kPi) * ld.I[k];   // PointLight::Power
            S->lightPower.push_back(0.212671f * P[0] + 0.715160f * P[1] + 0.072169f * P[2]);
        } else if (ld.type == PBR_LIGHT_DIFFUSE_AREA) {
            if (ld.shape < 0 || ld.shape >= ns || d->shapes[ld.shape].type != PBR_SHAPE_TRIANGLE_MESH ||
                ld.triangle < 0 || ld.triangle >= d->shapes[ld.shape].n_triangles)
                fail("area light shape out of range");
            int orig = firstPrim[ld.shape] + ld.triangle;
            L.primSlot = slotOf[orig];
            L.twoSided = ld.two_sided;
            mt_put3(L.L, ld.Le);
            f3 p0 = vert(prims[orig], 0), p1 = vert(prims[orig], 1), p2 = vert(prims[orig], 2);
            L.area = (float)(0.5 * (double)len(cross(p1 - p0, p2 - p0)));   // Triangle::Area
            float P[3];
            for (int k = 0; k < 3; ++k) P[k] = (float)(ld.two_sided ? 2 : 1) * ld.Le[k] * L.area * kPi;
            S->lightPower.push_back(0.212671f * P[0] + 0.715160f * P[1] + 0.072169f * P[2]);
        } else if (ld.type == PBR_LIGHT_SKYBOX) {
            if (S->envLight >= 0) fail("only one SkyBoxLight is supported");
            L.worldRadius = ld.world_radius;
            if (ld.env_data && ld.env_width > 0 && ld.env_height > 0) {
                if (ld.env_components < 3) fail("SkyBox env needs >= 3 components");
                L.envW = ld.env_width;
                L.envH = ld.env_height;
                // HDRtoLDR(texel, 0.3) once per texel (Spectrum.h:219-226, SkyBoxLight.cpp:37)
                float invExposure = (float)(1.0 / (1.0 - (double)0.3f));
                size_t nt = (size_t)L.envW * L.envH;
                S->env.resize(nt * 4);
                for (size_t t = 0; t < nt; ++t) {
                    for (int k = 0; k < 3; ++k) {
                        float c = ld.env_data[t * ld.env_components + k];
                        S->env[4 * t + k] = (float)(1.0 - (double)t_exp(-c * invExposure));
                    }
                    S->env[4 * t + 3] = 0.f;
                }
            }
            S->envLight = li;
            S->infinite.push_back(li);
            S->lightPower.push_back(0.f);
        } else if (ld.type == PBR_LIGHT_INFINITE_AREA) {
            if (S->inf.light >= 0) fail("only one InfiniteAreaLight is supported");
            // Preprocess sees scene.WorldBound() = the BVH root's bounds (empty Bounds3f → radius 0)
            const float big = std::numeric_limits<float>::max(), low = std::numeric_limits<float>::lowest();
            float lo[3] = {big, big, big}, hi[3] = {low, low, low};
            if (!S->nodes.empty())
                for (int k = 0; k < 3; ++k) { lo[k] = S->nodes[0].pMin[k]; hi[k] = S->nodes[0].pMax[k]; }
            float P[3];
            build_infinite_light(ld, lo, hi, &S->inf, P);
            S->inf.light = li;
            L.worldRadius = S->inf.worldRadius;
            S->infinite.push_back(li);
            S->lightPower.push_back(0.212671f * P[0] + 0.715160f * P[1] + 0.072169f * P[2]);
        } else {
            fail("unknown light type");
        }
        S->lights.push_back(L);
    }
    for (size_t slot = 0; slot < (size_t)np; ++slot) {
        int al = S->primInfo[slot * 4 + 2];
        if (al >= d->n_lights) fail("area light index out of range");
    }
    if (S->infinite.size() > 4) fail("at most 4 infinite lights");
    light_distribution(*S, PBR_LIGHTS_UNIFORM, &S->lightCdf, &S->lightFunc, &S->lightFuncInt);
}

void light_distribution(const HostScene& s, int strategy, std::vector<float>* cdf, std::vector<float>* func,
                        float* funcInt) {
    size_t n = s.lights.size();
    func->assign(n, 1.f);
    // CreateLightSampleDistribution: "uniform" or a single light → uniform (LightDistrib.cpp:10-12)
    if (strategy == PBR_LIGHTS_POWER && n != 1) *func = s.lightPower;
    if (n == 0) { cdf->assign(1, 0.f); *funcInt = 0; return; }
    distribution1d(*func, cdf, funcInt);
}

void build_camera(const pbr_camera_desc* c, DeviceCamera* out) {
    if (c->width <= 0 || c->height <= 0) fail("bad raster size");
    Xf camToWorld;
    if (c->use_look_at) {
        camToWorld = inverse(look_at(mk(c->eye[0], c->eye[1], c->eye[2]), mk(c->look[0], c->look[1], c->look[2]),
                                     mk(c->up[0], c->up[1], c->up[2])));
    } else {
        camToWorld = Xf{from_rows(c->camera_to_world.m), from_rows(c->camera_to_world.m_inv)};
    }
    // CreatePerspectiveCamera screen window (Perspective.cpp:84-104)
    float frame = (float)c->width / (float)c->height;
    float x0, x1, y0, y1;
    if (frame > 1.f) { x0 = -frame; x1 = frame; y0 = -1.f; y1 = 1.f; }
    else { x0 = -1.f; x1 = 1.f; y0 = -1.f / frame; y1 = 1.f / frame; }
    // ProjectiveCamera (Camera.h:36-53)
    Xf camToScreen = perspective(c->fov, 1e-2f, 1000.f);
    Xf screenToRaster = compose(compose(scale((float)c->width, (float)c->height, 1), scale(1 / (x1 - x0), 1 / (y0 - y1), 1)),
                                translate(mk(-x0, -y1, 0)));
    Xf rasterToCamera = compose(inverse(camToScreen), inverse(screenToRaster));
    // a camera's own RasterToCamera (any fov / screen window): used as given
    if (c->use_raster_to_camera) rasterToCamera = Xf{from_rows(c->raster_to_camera.m), from_rows(c->raster_to_camera.m_inv)};
    std::memcpy(out->rasterToCamera, &rasterToCamera.m.a[0][0], 64);
    std::memcpy(out->cameraToWorld, &camToWorld.m.a[0][0], 64);
    out->lensRadius = c->lens_radius;
    out->focalDistance = c->focal_distance;
    out->width = c->width;
    out->height = c->height;
}

void build_halton_tables(int nPrimes, HaltonTables* t) {
    t->primes.clear();
    for (uint32_t c = 2; (int)t->primes.size() < nPrimes; ++c) {
        bool prime = true;
        for (uint32_t q : t->primes) { if (q * q > c) break; if (c % q == 0) { prime = false; break; } }
        if (prime) t->primes.push_back(c);
    }
    t->recips.resize(nPrimes);
    t->primeSums.resize(nPrimes);
    uint32_t acc = 0;
    for (int i = 0; i < nPrimes; ++i) {
        t->recips[i] = (uint32_t)((((uint64_t)1) << 32) / t->primes[i]);
        t->primeSums[i] = acc;
        acc += t->primes[i];
    }
    // ComputeRadicalInversePermutations (LowDiscrepancy.cpp:2284-2298) with PCG32 defaults
    t->perms.resize(acc);
    uint64_t state = 0x853c49e6748fea9bULL;
    const uint64_t inc = 0xda3e39cb94b95bdbULL;
    auto next = [&]() -> uint32_t {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31));
    };
    auto bounded = [&](uint32_t b) -> uint32_t {
        uint32_t threshold = (~b + 1u) % b;
        for (;;) { uint32_t r = next(); if (r >= threshold) return r % b; }
    };
    uint16_t* p = t->perms.data();
    for (int i = 0; i < nPrimes; ++i) {
        uint32_t n = t->primes[i];
        for (uint32_t j = 0; j < n; ++j) p[j] = (uint16_t)j;
        for (uint32_t j = 0; j < n; ++j) {           // Shuffle (Sampling.h:47-54)
            uint32_t other = j + bounded(n - j);
            std::swap(p[j], p[other]);
        }
        p += n;
    }
}

void halton_params(int resX, int resY, DeviceSampler* s) {   // HaltonSampler ctor (Halton.cpp:30-58)
    int res[2] = {resX, resY}, scale[2], expo[2];
    for (int i = 0; i < 2; ++i) {
        int base = i == 0 ? 2 : 3, sc = 1, e = 0;
        while (sc < std::min(res[i], 128)) { sc *= base; ++e; }
        scale[i] = sc;
        expo[i] = e;
    }
    auto inv_mod = [](int64_t a, int64_t n) -> int64_t {   // multiplicativeInverse via extended GCD
        int64_t r0 = n, r1 = a % n, s0 = 0, s1 = 1;
        while (r1 != 0) {
            int64_t q = r0 / r1, t = r0 - q * r1;
            r0 = r1; r1 = t;
            t = s0 - q * s1; s0 = s1; s1 = t;
        }
        int64_t x = s0 % n;
        return x < 0 ? x + n : x;
    };
    s->baseExp0 = expo[0];
    s->baseExp1 = expo[1];
    s->baseScale1 = scale[1];
    s->stride = scale[0] * scale[1];
    s->mult0 = scale[0] > 1 ? (int)inv_mod(scale[1], scale[0]) : 0;
    s->mult1 = scale[1] > 1 ? (int)inv_mod(scale[0], scale[1]) : 0;
    s->ratio0 = s->stride / scale[0];
    s->ratio1 = s->stride / scale[1];
}

// ---------------------------------------------------------------- Sobol (pbrt-v3 SobolSampler)
// pbrt-v3's SobolMatrices32 (the reference's Sampler/SobolMatrices.cpp:69), regenerated from the
// Joe-Kuo direction numbers it was built from (pbr_sobol_jk.h): dimension 0 is van der Corput,
// dimension d >= 1 runs the Bratley-Fox recurrence over its primitive polynomial (degree s, inner
// coefficients a) from m_1..m_s; column c holds v_{c+1} = m_{c+1} / 2^{c+1} as 32 bits (index bits
// >= 32 keep v's top 32 bits).  tests/test_oracle_golden.py hash-matches all 1024 × 52 words.
void build_sobol_matrices(int nDims, std::vector<uint32_t>* out) {
    if (nDims > kSobolJKDims) fail("Sobol: at most 1024 dimensions");
    out->assign((size_t)nDims * kSobolMatrixSize, 0u);
    uint32_t* M = out->data();
    for (int c = 0; c < 32 && nDims > 0; ++c) M[c] = 0x80000000u >> c;
    const uint16_t* jk = kSobolJK;
    for (int d = 1; d < nDims; ++d) {
        const int deg = jk[0] & 15;
        const uint32_t a = jk[0] >> 4;
        uint64_t m[kSobolMatrixSize + 1];
        for (int k = 1; k <= kSobolMatrixSize; ++k) {
            if (k <= deg) { m[k] = jk[k]; continue; }
            uint64_t v = m[k - deg] ^ (m[k - deg] << deg);
            for (int i = 1; i < deg; ++i)
                if ((a >> (deg - 1 - i)) & 1u) v ^= m[k - i] << i;
            m[k] = v;
        }
        for (int c = 0; c < kSobolMatrixSize; ++c)
            M[(size_t)d * kSobolMatrixSize + c] = (uint32_t)(c < 32 ? m[c + 1] << (31 - c) : m[c + 1] >> (c - 31));
        jk += 1 + deg;
    }
}

// SobolIntervalToIndex at resolution 2^m, restated as a GF(2) solve: the top m bits of
// dimensions 0 and 1 of sample index i are T·i; with i = (frame << 2m) | j (up to 52 bits) the low block of T is
// invertible (the first two dimensions form a (0,2)-sequence), so j = T_low^-1 (p ^ T_high·frame)
// with p = (px << m) | py.  out = T_low^-1 columns [2m], then T_high columns [52 - 2m].
void sobol_pixel_tables(const uint32_t* mats, int m, std::vector<uint32_t>* out) {
    out->clear();
    if (m <= 0) return;
    if (2 * m > 32) fail("Sobol resolution too large");
    const int n = 2 * m;
    auto col = [&](int c) -> uint32_t {   // the 2m-bit image of index bit c
        uint32_t x = mats[c] >> (32 - m), y = mats[kSobolMatrixSize + c] >> (32 - m);
        return (x << m) | y;
    };
    // Gauss-Jordan on [T_low | I] by columns: rows are bit positions
    std::vector<uint32_t> A(n), inv(n);
    for (int c = 0; c < n; ++c) { A[c] = col(c); inv[c] = 1u << c; }   // column c of T_low and of I
    // solve via column operations: reduce A's columns to the unit vectors
    for (int r = 0; r < n; ++r) {
        int piv = -1;
        for (int c = r; c < n; ++c)
            if ((A[c] >> r) & 1u) { piv = c; break; }
        if (piv < 0) fail("Sobol dimensions 0/1 are not a (0,2)-sequence");
        std::swap(A[r], A[piv]);
        std::swap(inv[r], inv[piv]);
        for (int c = 0; c < n; ++c)
            if (c != r && ((A[c] >> r) & 1u)) { A[c] ^= A[r]; inv[c] ^= inv[r]; }
    }
    // now T_low · inv[r] (as a combination of index bits) = unit vector e_r: inv[r] is the index
    // bit pattern that produces pixel bit r
    out->resize(kSobolMatrixSize);   // frame bits reach index bit 51 (64-bit pbrt-v3 indices)
    for (int r = 0; r < n; ++r) (*out)[r] = inv[r];
    for (int k = 0; k < kSobolMatrixSize - n; ++k) (*out)[n + k] = col(n + k);
}

}  // namespace pbr
