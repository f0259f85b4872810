// pbr_hip_integrator.cpp — reference-side binding (see pbr_hip_integrator.h): flatten a reference
// PBR::Scene into the C-ABI's pbr_scene_desc and render it on the MI355X.
//
// Built against the reference's unmodified headers.  The members read below are private in the
// reference; inside the reference tree each class would befriend pbrhip::SceneFlattener, here they
// are opened for this translation unit only.  The standard headers come first so the override
// touches only the reference's classes.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#define private public
#define protected public
#include "Accelerator\BVHAccel.h"
#include "Camera\Perspective.h"
#include "Core\FrameBuffer.h"
#include "Core\Primitive.h"
#include "Core\Scene.h"
#include "Core\Spectrum.h"
#include "Core\Transform.h"
#include "Light\DiffuseLight.h"
#include "Light\InfiniteAreaLight.h"
#include "Light\PointLight.h"
#include "Light\SkyBoxLight.h"
#include "Material\GlassMaterial.h"
#include "Material\MatteMaterial.h"
#include "Material\MetalMaterial.h"
#include "Material\Mirror.h"
#include "Material\PlasticMaterial.h"
#include "Media\HomogeneousMedium.h"
#include "Sampler\Halton.h"
#include "Shape\Triangle.h"
#include "Texture\ConstantTexture.h"
#include "Texture\ImageTexture.h"
#include "Texture\MIPMap.h"
#undef protected
#undef private

#include "pbr_hip_integrator.h"

using namespace PBR;

namespace pbrhip {
namespace {

void need(bool ok, const char* what) {
    if (!ok) throw std::invalid_argument(std::string("pbr_hip binding: ") + what);
}
void put3(float* dst, const Spectrum& s) { dst[0] = s[0]; dst[1] = s[1]; dst[2] = s[2]; }
void put_transform(const Transform& t, pbr_transform* out) {   // Transform.h:49-60: m and mInv, row-major
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            out->m[4 * r + c] = t.m.m[r][c];
            out->m_inv[4 * r + c] = t.mInv.m[r][c];
        }
}
pbr_transform identity() {
    pbr_transform t;
    std::memset(&t, 0, sizeof(t));
    for (int i = 0; i < 4; ++i) t.m[5 * i] = t.m_inv[5 * i] = 1.f;
    return t;
}
// A material parameter: a ConstantTexture's value (Texture/ConstantTexture.h), or an ImageTexture
// (Texture/ImageTexture.h:43-91) handed over as what the built texture holds — its MIPMap's level 0
// (MIPMap.h:150-153: the image after convertIn and the power-of-two resample) and its UVMapping2D
// (Texture.h:16-27) — with pbr_texture_desc::level0.  The reference's ray differentials are zero
// (F5), so level 0 is all its lookups ever read (pbr_hip.h, pbr_texture_desc).
template <class Tm, class Tr>
int image_texture(FlatScene* F, const ImageTexture<Tm, Tr>* it) {
    auto found = F->textureOf.find(it);
    if (found != F->textureOf.end()) return found->second;
    auto* uv = dynamic_cast<const UVMapping2D*>(it->mapping.get());
    need(uv != nullptr, "an ImageTexture's mapping must be a UVMapping2D");
    const MIPMap<Tm>& mm = *it->mipmap;
    constexpr bool isFloat = std::is_same<Tm, float>::value;
    const int W = mm.Width(), H = mm.Height(), nc = isFloat ? 1 : 3;
    std::vector<float> t0((size_t)W * H * nc);
    for (int t = 0; t < H; ++t)
        for (int s = 0; s < W; ++s) {
            const Tm& v = (*mm.pyramid[0])(s, t);
            float* o = &t0[((size_t)t * W + s) * nc];
            if constexpr (isFloat) o[0] = v;
            else { o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; }
        }
    pbr_texture_desc d;
    std::memset(&d, 0, sizeof(d));
    d.is_float = isFloat ? 1 : 0;
    d.width = W;
    d.height = H;
    d.components = nc;
    d.level0 = 1;
    d.scale = 1.f;
    d.wrap = mm.wrapMode == ImageWrap::Repeat ? PBR_WRAP_REPEAT : (mm.wrapMode == ImageWrap::Black ? PBR_WRAP_BLACK : PBR_WRAP_CLAMP);
    d.trilinear = mm.doTrilinear;
    d.max_aniso = mm.maxAnisotropy;
    d.su = uv->su; d.sv = uv->sv; d.du = uv->du; d.dv = uv->dv;
    F->texels.push_back(std::move(t0));
    d.data = F->texels.back().data();   // a moved vector keeps its buffer: stable as texels grows
    F->textures.push_back(d);
    const int k = (int)F->textures.size() - 1;
    F->textureOf[it] = k;
    return k;
}
// slot: pbr_texture_slot, or -1 where the device takes constants only
void slotS(FlatScene* F, pbr_material_desc* d, int slot, const std::shared_ptr<Texture<Spectrum>>& t, float* out, const char* what) {
    if (auto* c = dynamic_cast<const ConstantTexture<Spectrum>*>(t.get())) { put3(out, c->value); return; }
    auto* it = dynamic_cast<const ImageTexture<RGBSpectrum, Spectrum>*>(t.get());
    need(it != nullptr && slot >= 0, what);
    d->tex[slot] = image_texture(F, it) + 1;
}
float slotF(FlatScene* F, pbr_material_desc* d, int slot, const std::shared_ptr<Texture<float>>& t, const char* what) {
    if (auto* c = dynamic_cast<const ConstantTexture<float>*>(t.get())) return c->value;
    auto* it = dynamic_cast<const ImageTexture<float, float>*>(t.get());
    need(it != nullptr && slot >= 0, what);
    d->tex[slot] = image_texture(F, it) + 1;
    return 0.f;
}

// Material/*.h → pbr_material_desc (the fields pbr_hip.h documents per type).  Bump maps are not
// read: the reference's ComputeScatteringFunctions never applies them.
pbr_material_desc material_desc(FlatScene* F, const Material* m) {
    pbr_material_desc d;
    std::memset(&d, 0, sizeof(d));
    if (auto* x = dynamic_cast<const MatteMaterial*>(m)) {
        d.type = PBR_MAT_MATTE;
        slotS(F, &d, PBR_TEX_KD, x->Kd, d.Kd, "MatteMaterial Kd must be a Constant or ImageTexture");
        d.sigma = slotF(F, &d, PBR_TEX_SIGMA, x->sigma, "MatteMaterial sigma must be a Constant or ImageTexture");
    } else if (auto* x = dynamic_cast<const MirrorMaterial*>(m)) {
        d.type = PBR_MAT_MIRROR;
        slotS(F, &d, PBR_TEX_KR, x->Kr, d.Kr, "MirrorMaterial Kr must be a Constant or ImageTexture");
    } else if (auto* x = dynamic_cast<const GlassMaterial*>(m)) {
        d.type = PBR_MAT_GLASS;
        slotS(F, &d, PBR_TEX_KR, x->Kr, d.Kr, "GlassMaterial Kr must be a Constant or ImageTexture");
        slotS(F, &d, PBR_TEX_KT, x->Kt, d.Kt, "GlassMaterial Kt must be a Constant or ImageTexture");
        d.uroughness = slotF(F, &d, -1, x->uRoughness, "GlassMaterial uRoughness must be a ConstantTexture");
        d.vroughness = slotF(F, &d, -1, x->vRoughness, "GlassMaterial vRoughness must be a ConstantTexture");
        d.eta = slotF(F, &d, -1, x->index, "GlassMaterial index must be a ConstantTexture");
        d.remap_roughness = x->remapRoughness;
    } else if (auto* x = dynamic_cast<const MetalMaterial*>(m)) {
        d.type = PBR_MAT_METAL;
        slotS(F, &d, -1, x->eta, d.metal_eta, "MetalMaterial eta must be a ConstantTexture");
        slotS(F, &d, -1, x->k, d.metal_k, "MetalMaterial k must be a ConstantTexture");
        d.roughness = slotF(F, &d, -1, x->roughness, "MetalMaterial roughness must be a ConstantTexture");
        d.has_uv_roughness = x->uRoughness != nullptr;   // MetalMaterial.cpp: u/v textures when present
        if (x->uRoughness) d.uroughness = slotF(F, &d, -1, x->uRoughness, "MetalMaterial uRoughness must be a ConstantTexture");
        if (x->vRoughness) d.vroughness = slotF(F, &d, -1, x->vRoughness, "MetalMaterial vRoughness must be a ConstantTexture");
        d.remap_roughness = x->remapRoughness;
    } else if (auto* x = dynamic_cast<const PlasticMaterial*>(m)) {
        d.type = PBR_MAT_PLASTIC;
        slotS(F, &d, PBR_TEX_KD, x->Kd, d.Kd, "PlasticMaterial Kd must be a Constant or ImageTexture");
        slotS(F, &d, PBR_TEX_KS, x->Ks, d.Ks, "PlasticMaterial Ks must be a Constant or ImageTexture");
        d.roughness = slotF(F, &d, PBR_TEX_ROUGHNESS, x->roughness, "PlasticMaterial roughness must be a Constant or ImageTexture");
        d.remap_roughness = x->remapRoughness;
    } else {
        need(false, "material type not on the GPU path");
    }
    return d;
}

}  // namespace

int SceneFlattener::MediumIndex(const FlatScene& f, const void* medium) {
    if (!medium) return -1;
    auto it = std::find(f.mediumOf.begin(), f.mediumOf.end(), medium);
    need(it != f.mediumOf.end(), "medium not part of the scene");
    return (int)(it - f.mediumOf.begin());
}

std::shared_ptr<FlatScene> SceneFlattener::Flatten(const Scene& scene) {
    auto F = std::make_shared<FlatScene>();
    auto* bvh = dynamic_cast<const BVHAccel*>(scene.aggregate.get());
    need(bvh != nullptr, "the Scene's aggregate must be a BVHAccel");
    // BVHAccel's constructor swapped `primitives` into leaf order (BVHAccel.cpp:75-80): the order
    // its LinearBVHNode leaves index, handed over with the nodes themselves
    const std::vector<std::shared_ptr<Primitive>>& prims = bvh->primitives;
    std::vector<const GeometricPrimitive*> gps;
    gps.reserve(prims.size());
    auto addMedium = [&](const Medium* m) {
        if (!m || std::find(F->mediumOf.begin(), F->mediumOf.end(), (const void*)m) != F->mediumOf.end()) return;
        auto* h = dynamic_cast<const HomogeneousMedium*>(m);
        need(h != nullptr, "only HomogeneousMedium is on the GPU path");
        pbr_medium_desc d;
        put3(d.sigma_a, h->sigma_a);
        put3(d.sigma_s, h->sigma_s);
        d.g = h->g;
        F->mediumOf.push_back(m);
        F->media.push_back(d);
    };
    for (const auto& p : prims) {
        auto* gp = dynamic_cast<const GeometricPrimitive*>(p.get());
        need(gp != nullptr, "BVHAccel primitives must be GeometricPrimitives");
        gps.push_back(gp);
        addMedium(gp->mediumInterface.inside);
        addMedium(gp->mediumInterface.outside);
    }
    for (const auto& l : scene.lights) {
        addMedium(l->mediumInterface.inside);
        addMedium(l->mediumInterface.outside);
    }
    std::map<const Material*, int> matIndex;
    for (auto* gp : gps) {
        const Material* m = gp->material.get();
        if (!m || matIndex.count(m)) continue;
        matIndex[m] = (int)F->materials.size();
        F->materials.push_back(material_desc(F.get(), m));
    }
    std::unordered_map<const Light*, int> lightIndex;
    for (size_t i = 0; i < scene.lights.size(); ++i) lightIndex[scene.lights[i].get()] = (int)i;
    F->lights.resize(scene.lights.size());
    std::vector<bool> boundArea(scene.lights.size(), false);
    // Vertices: TriangleMesh::p is already in world space (Triangle.cpp:12-44), so meshes go over
    // with an identity transform; one point array per mesh.
    std::map<const TriangleMesh*, int> meshIndex;
    auto meshOf = [&](const TriangleMesh* mesh) {
        auto it = meshIndex.find(mesh);
        if (it != meshIndex.end()) return it->second;
        need(!mesh->n, "per-vertex shading normals are not on the GPU path");
        std::vector<float> P((size_t)mesh->nVertices * 3);
        for (int v = 0; v < mesh->nVertices; ++v) {
            P[3 * v] = mesh->p[v].x; P[3 * v + 1] = mesh->p[v].y; P[3 * v + 2] = mesh->p[v].z;
        }
        F->points.push_back(std::move(P));
        std::vector<float> UV;
        if (mesh->uv) {
            UV.resize((size_t)mesh->nVertices * 2);
            for (int v = 0; v < mesh->nVertices; ++v) { UV[2 * v] = mesh->uv[v].x; UV[2 * v + 1] = mesh->uv[v].y; }
        }
        F->uvs.push_back(std::move(UV));
        const int k = (int)F->points.size() - 1;
        meshIndex[mesh] = k;
        return k;
    };
    auto lightOf = [&](const GeometricPrimitive* g) -> int {
        if (!g->areaLight) return -1;
        auto it = lightIndex.find(g->areaLight.get());
        need(it != lightIndex.end(), "an area light is not in Scene::lights");
        return it->second;
    };
    // Shapes: maximal runs of consecutive (leaf-order) triangles sharing mesh, orientation,
    // material, medium interface and consecutively numbered area lights.  A triangle's orientation
    // flip is reverseOrientation ^ transformSwapsHandedness (Triangle.cpp:197-206) of its own
    // transform; the identity transform here swaps nothing, so the flip travels as the flag.
    size_t i = 0;
    while (i < gps.size()) {
        const GeometricPrimitive* gp = gps[i];
        auto* tri = dynamic_cast<const Triangle*>(gp->shape.get());
        need(tri != nullptr, "only triangle meshes are on the GPU path (the reference's Sphere is a stub)");
        const bool flip = tri->reverseOrientation ^ tri->transformSwapsHandedness;
        const int firstLight = lightOf(gp);
        const int shapeIdx = (int)F->shapes.size();
        const int mk = meshOf(tri->mesh.get());
        std::vector<int32_t> idx;
        size_t j = i;
        while (j < gps.size()) {
            const GeometricPrimitive* g = gps[j];
            auto* t = dynamic_cast<const Triangle*>(g->shape.get());
            if (!t || t->mesh != tri->mesh || (t->reverseOrientation ^ t->transformSwapsHandedness) != flip ||
                g->material != gp->material || g->mediumInterface.inside != gp->mediumInterface.inside ||
                g->mediumInterface.outside != gp->mediumInterface.outside)
                break;
            const int li = lightOf(g), k = (int)(j - i);
            if ((firstLight < 0) != (li < 0) || (firstLight >= 0 && li != firstLight + k)) break;
            if (li >= 0) {   // DiffuseAreaLight (Light/DiffuseLight.h:13-34) bound to this triangle
                auto* dl = dynamic_cast<const DiffuseAreaLight*>(g->areaLight.get());
                need(dl != nullptr && dl->shape.get() == g->shape.get(), "area light / shape mismatch");
                pbr_light_desc& L = F->lights[li];
                std::memset(&L, 0, sizeof(L));
                L.type = PBR_LIGHT_DIFFUSE_AREA;
                put_transform(dl->LightToWorld, &L.light_to_world);
                put3(L.Le, dl->Lemit);
                L.shape = shapeIdx;
                L.triangle = k;
                L.two_sided = dl->twoSided;
                L.n_samples = dl->nSamples;
                L.medium_inside = MediumIndex(*F, dl->mediumInterface.inside);
                L.medium_outside = MediumIndex(*F, dl->mediumInterface.outside);
                boundArea[li] = true;
            }
            idx.insert(idx.end(), t->v, t->v + 3);
            ++j;
        }
        pbr_shape_desc sd;
        std::memset(&sd, 0, sizeof(sd));
        sd.type = PBR_SHAPE_TRIANGLE_MESH;
        sd.object_to_world = identity();
        sd.reverse_orientation = flip;
        sd.n_triangles = (int)(j - i);
        sd.n_vertices = tri->mesh->nVertices;
        sd.material = gp->material ? matIndex[gp->material.get()] : -1;
        sd.area_light_first = firstLight;
        sd.medium_inside = MediumIndex(*F, gp->mediumInterface.inside);
        sd.medium_outside = MediumIndex(*F, gp->mediumInterface.outside);
        sd.P = F->points[mk].data();
        sd.UV = F->uvs[mk].empty() ? nullptr : F->uvs[mk].data();
        F->indexRuns.push_back(std::move(idx));
        F->shapes.push_back(sd);
        i = j;
    }
    for (size_t s = 0; s < F->shapes.size(); ++s) F->shapes[s].indices = F->indexRuns[s].data();
    for (size_t li = 0; li < scene.lights.size(); ++li) {
        const Light* l = scene.lights[li].get();
        pbr_light_desc& L = F->lights[li];
        if (auto* pl = dynamic_cast<const PointLight*>(l)) {   // Light/PointLight.h:13-34
            std::memset(&L, 0, sizeof(L));
            L.type = PBR_LIGHT_POINT;
            put_transform(pl->LightToWorld, &L.light_to_world);
            put3(L.I, pl->I);
            L.n_samples = pl->nSamples;
            L.medium_inside = MediumIndex(*F, pl->mediumInterface.inside);
            L.medium_outside = MediumIndex(*F, pl->mediumInterface.outside);
        } else if (auto* sk = dynamic_cast<const SkyBoxLight*>(l)) {   // Light/SkyBoxLight.h: the loaded image
            std::memset(&L, 0, sizeof(L));
            L.type = PBR_LIGHT_SKYBOX;
            put_transform(sk->LightToWorld, &L.light_to_world);
            L.world_center[0] = sk->worldCenter.x; L.world_center[1] = sk->worldCenter.y; L.world_center[2] = sk->worldCenter.z;
            L.world_radius = sk->worldRadius;
            L.env_width = sk->imageWidth;
            L.env_height = sk->imageHeight;
            L.env_components = sk->nrComponents;
            L.env_data = sk->data;
            L.n_samples = sk->nSamples;
            L.medium_inside = L.medium_outside = -1;
        } else if (dynamic_cast<const DiffuseAreaLight*>(l)) {
            need(boundArea[li], "a DiffuseAreaLight whose shape is not a scene triangle");
        } else if (auto* il = dynamic_cast<const InfiniteAreaLight*>(l)) {
            // InfiniteAreaLight keeps its map as the MIPMap Lmap (InfiniteAreaLight.h:33): level 0 is
            // the image times L after the power-of-two resample.  It goes over with Le = 1 (pbr_hip.h):
            // the upload rebuilds the same pyramid, Distribution2D and Power() from it.
            const MIPMap<RGBSpectrum>& mm = *il->Lmap;
            const int W = mm.Width(), H = mm.Height();
            std::vector<float> t0((size_t)W * H * 3);
            for (int t = 0; t < H; ++t)
                for (int s = 0; s < W; ++s) {
                    const RGBSpectrum& v = (*mm.pyramid[0])(s, t);
                    float* o = &t0[((size_t)t * W + s) * 3];
                    o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
                }
            F->texels.push_back(std::move(t0));
            std::memset(&L, 0, sizeof(L));
            L.type = PBR_LIGHT_INFINITE_AREA;
            put_transform(il->LightToWorld, &L.light_to_world);
            L.Le[0] = L.Le[1] = L.Le[2] = 1.f;
            L.n_samples = il->nSamples;
            L.env_width = W;
            L.env_height = H;
            L.env_components = 3;
            L.env_data = F->texels.back().data();
            L.medium_inside = L.medium_outside = -1;
        } else {
            need(false, "light type not on the GPU path of the binding");
        }
    }
    // the reference's own tree: LinearBVHNode records (BVHAccel.cpp:46-55), counted by a preorder walk
    struct Node { float b[6]; int offset; uint16_t nPrims; uint8_t axis, pad; };
    static_assert(sizeof(Node) == 32, "LinearBVHNode layout");
    const Node* nd = reinterpret_cast<const Node*>(bvh->nodes);
    int total = 0;
    if (nd && !prims.empty()) {
        std::vector<int> stack{0};
        while (!stack.empty()) {
            const int k = stack.back();
            stack.pop_back();
            ++total;
            if (nd[k].nPrims == 0) { stack.push_back(nd[k].offset); stack.push_back(k + 1); }
        }
        F->nodes.assign(reinterpret_cast<const unsigned char*>(nd), reinterpret_cast<const unsigned char*>(nd + total));
    }
    pbr_scene_desc& d = F->desc;
    d.abi_version = PBR_HIP_ABI_VERSION;
    d.n_shapes = (int)F->shapes.size();
    d.shapes = F->shapes.data();
    d.n_materials = (int)F->materials.size();
    d.materials = F->materials.data();
    d.n_lights = (int)F->lights.size();
    d.lights = F->lights.data();
    d.n_media = (int)F->media.size();
    d.media = F->media.data();
    d.max_prims_in_node = bvh->maxPrimsInNode;
    d.split_method = (int)bvh->splitMethod;
    d.bvh_nodes = F->nodes.empty() ? nullptr : F->nodes.data();
    d.n_bvh_nodes = total;
    d.n_textures = (int)F->textures.size();
    d.textures = F->textures.empty() ? nullptr : F->textures.data();
    return F;
}

HipSamplerIntegrator::HipSamplerIntegrator(int integrator, int maxDepth, std::shared_ptr<const Camera> camera,
                                           std::shared_ptr<Sampler> sampler, const Bounds2i& pixelBounds, float rrThreshold,
                                           const std::string& lightSampleStrategy, FrameBuffer* frameBuffer)
    : SamplerIntegrator(camera, sampler, pixelBounds, frameBuffer),
      integrator_(integrator),
      maxDepth_(maxDepth),
      rrThreshold_(rrThreshold),
      strategy_(lightSampleStrategy),
      sampler_(sampler),
      bounds_(pixelBounds),
      fb_(frameBuffer) {}

HipSamplerIntegrator::~HipSamplerIntegrator() {
    if (ctx_) pbr_hip_destroy(ctx_);
}

void HipSamplerIntegrator::Render(const Scene& scene, double& timeConsume) {
    const auto t0 = std::chrono::steady_clock::now();
    auto check = [&](int rc, const char* what) {
        if (rc != PBR_OK)
            throw std::runtime_error(std::string("pbr_hip ") + what + ": " + (ctx_ ? pbr_hip_last_error(ctx_) : "no device"));
    };
    if (!ctx_) check(pbr_hip_create(device_, &ctx_), "create");
    if (uploaded_ != &scene) {   // SamplerIntegrator::Preprocess's place: once per Scene
        flat_ = SceneFlattener::Flatten(scene);
        check(pbr_hip_upload_scene(ctx_, &flat_->desc), "upload_scene");
        uploaded_ = &scene;
    }
    // the camera: its CameraToWorld, lens and its own RasterToCamera (ProjectiveCamera, Camera.h:36-53)
    // — whatever fov and screen window it was constructed with (Perspective.cpp:6-9) — go over as they
    // are (pbr_camera_desc::use_raster_to_camera)
    auto* pc = dynamic_cast<const PerspectiveCamera*>(camera.get());
    need(pc != nullptr, "the camera must be a PerspectiveCamera");
    auto* halton = dynamic_cast<const HaltonSampler*>(sampler_.get());
    need(halton != nullptr, "the sampler must be a HaltonSampler");
    const int W = bounds_.pMax.x, H = bounds_.pMax.y;
    need(bounds_.pMin.x == 0 && bounds_.pMin.y == 0 && W > 0 && H > 0, "pixel bounds must start at (0, 0)");
    // the device derives the Halton base scales from the raster (Halton.cpp:39-51): the sampler's
    // sampleBounds must be these pixel bounds
    for (int i = 0; i < 2; ++i) {
        const int base = i == 0 ? 2 : 3, res = i == 0 ? W : H;
        int scale = 1;
        while (scale < std::min(res, 128)) scale *= base;
        need(halton->baseScales[i] == scale, "the HaltonSampler's sample bounds must be the integrator's pixel bounds");
    }
    pbr_render_desc rd;
    std::memset(&rd, 0, sizeof(rd));
    rd.integrator = integrator_;
    rd.max_depth = maxDepth_;
    rd.rr_threshold = rrThreshold_;
    // LightDistrib.cpp:10-21: "power" builds the power distribution; anything else is uniform
    rd.light_strategy = strategy_ == "power" ? PBR_LIGHTS_POWER : PBR_LIGHTS_UNIFORM;
    rd.sampler = PBR_SAMPLER_HALTON;
    rd.spp = (int)halton->samplesPerPixel;
    rd.camera.width = W;
    rd.camera.height = H;
    put_transform(pc->CameraToWorld, &rd.camera.camera_to_world);
    rd.camera.fov = 90.f;
    rd.camera.use_raster_to_camera = 1;
    put_transform(pc->RasterToCamera, &rd.camera.raster_to_camera);
    rd.camera.lens_radius = pc->lensRadius;
    rd.camera.focal_distance = pc->focalDistance;
    rd.camera.medium = SceneFlattener::MediumIndex(*flat_, pc->medium);
    std::vector<uint8_t> rgba((size_t)W * H * 4);
    std::vector<float> rgb((size_t)W * H * 3);
    check(pbr_hip_render(ctx_, &rd, rgb.data(), rgba.data(), nullptr), "render");
    lastDesc_ = rd;
    // Integrator.cpp:327-344: pixel (x, y) → set_uc(x, height - 1 - y); the device produced the same
    // bytes (ToXYZ, XYZToRGB, GammaCorrect, +0.5, clamp) with alpha 255.  The FrameBuffer's float
    // buffer, which the reference allocates but never writes, is left as the caller had it
    // unless SetWriteFloatBuffer(true) asked for colObj / spp (linear RGB, alpha 1) there, at the same
    // place, through its own set_fc.
    if (fb_) {
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                for (int c = 0; c < 4; ++c) fb_->set_uc(x, H - y - 1, c, rgba[((size_t)y * W + x) * 4 + c]);
                if (!writeFloat_) continue;
                for (int c = 0; c < 3; ++c) fb_->set_fc(x, H - y - 1, c, rgb[((size_t)y * W + x) * 3 + c]);
                fb_->set_fc(x, H - y - 1, 3, 1.f);
            }
    }
    timeConsume = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace pbrhip
