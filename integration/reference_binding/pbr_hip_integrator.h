// pbr_hip_integrator.h — the reference-side drop-in for the MI355X render path.
//
// This file is written against the reference's OWN headers (G0T-cha/PysicalBasedRaytracer: the
// `PBR` namespace, Core/Scene.h, Integrator/Integrator.h, ...): it is what a maintainer adds to the
// reference tree.  In Main/main.cpp (:384-413) the integrator line
//
//     auto integ = std::make_shared<WhittedIntegrator>(maxDepth, camera, sampler, pixelBounds, &fb);
//
// becomes
//
//     auto integ = std::make_shared<pbrhip::HipWhittedIntegrator>(maxDepth, camera, sampler, pixelBounds, &fb);
//
// with the same arguments (likewise HipPathIntegrator / HipVolPathIntegrator for PathIntegrator /
// VolPathIntegrator, Integrator/PathIntegrator.h:14-18, VolPathIntegrator.h:13-17).  Everything else
// stays: the scene is assembled from the reference's GeometricPrimitives, its BVHAccel, lights and
// camera exactly as before, and Render (Integrator/Integrator.h:14) fills the same FrameBuffer.
//
// Underneath, Render flattens the reference Scene into the plain-data pbr_scene_desc of the C-ABI
// (include/pbr_hip.h) — SceneFlattener below — and renders through pbr_hip_upload_scene /
// pbr_hip_render.  The flattening hands over the reference's own BVHAccel: its primitives in leaf
// order and its LinearBVHNode array (pbr_scene_desc::bvh_nodes), so the device walks the reference's
// tree, not a rebuilt one.
//
// Reading the scene needs the reference classes' private members (GeometricPrimitive's shape /
// material / light, BVHAccel's nodes, the materials' textures, the lights' parameters).  Added to
// the reference tree, each of those classes would declare `friend class pbrhip::SceneFlattener;`;
// compiled beside an unmodified tree (oracle/ref/Makefile builds it that way for the tests), the
// implementation file opens them with `#define private public` instead.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "Integrator\Integrator.h"
#include "Core\Scene.h"
#include "Core\FrameBuffer.h"

#include "../../include/pbr_hip.h"

namespace pbrhip {

// A reference Scene as the C-ABI takes it: the descriptor plus every array it points into.
struct FlatScene {
    pbr_scene_desc desc{};
    std::vector<pbr_shape_desc> shapes;
    std::vector<pbr_material_desc> materials;
    std::vector<pbr_light_desc> lights;
    std::vector<pbr_medium_desc> media;
    std::vector<std::vector<int32_t>> indexRuns;   // per shape: the triangles' vertex indices, leaf order
    std::vector<std::vector<float>> points;        // per mesh: the world-space vertices (TriangleMesh::p)
    std::vector<std::vector<float>> uvs;           // per mesh: TriangleMesh::uv, if any
    std::vector<unsigned char> nodes;              // the BVHAccel's LinearBVHNode array (32 B each)
    std::vector<const void*> mediumOf;             // media in index order (PBR::Medium*)
    std::vector<pbr_texture_desc> textures;        // ImageTextures (their MIPMap level 0), in index order
    std::map<const void*, int> textureOf;          // ImageTexture object → its index
    std::vector<std::vector<float>> texels;        // level-0 texels of the textures and InfiniteAreaLights
};

class SceneFlattener {
  public:
    // Throws std::invalid_argument for what the device path does not hold: an aggregate that is not
    // a BVHAccel, non-triangle shapes (the reference's Sphere is a stub), image textures on metal or
    // on glass roughness / index, texture mappings other than UVMapping2D, bump maps, per-vertex
    // shading normals, media other than HomogeneousMedium.  ImageTextures and InfiniteAreaLights go
    // over as the MIPMap level 0 they hold (pbr_texture_desc::level0, pbr_hip.h).
    static std::shared_ptr<FlatScene> Flatten(const PBR::Scene& scene);
    // index of a medium of the flattened scene (-1 for nullptr)
    static int MediumIndex(const FlatScene& f, const void* medium);
};

// SamplerIntegrator::Render (Integrator/Integrator.cpp:280-356) on an MI355X: every pixel × sample
// of the pixel bounds through the device's integrator, then the reference's FrameBuffer writes
// (ToXYZ → XYZToRGB → GammaCorrect → 8 bit at set_uc(x, height - 1 - y), alpha 255).  The
// reference's Render renders min(w, h)² pixels with swapped loop axes; this one renders
// every pixel of the bounds, so square rasters match the reference's frame byte for byte.
class HipSamplerIntegrator : public PBR::SamplerIntegrator {
  public:
    HipSamplerIntegrator(int integrator, int maxDepth, std::shared_ptr<const PBR::Camera> camera,
                         std::shared_ptr<PBR::Sampler> sampler, const PBR::Bounds2i& pixelBounds, float rrThreshold,
                         const std::string& lightSampleStrategy, ::FrameBuffer* frameBuffer);
    ~HipSamplerIntegrator();
    void Render(const PBR::Scene& scene, double& timeConsume);
    void SetDevice(int device) { device_ = device; }
    // Off by default, as in the reference's Render, which never writes the FrameBuffer's float buffer
    // (Integrator.cpp:341-344 writes only set_uc): on, Render also stores colObj / spp (linear RGB,
    // alpha 1) there through set_fc — the parity harness reads the device's floats that way.
    void SetWriteFloatBuffer(bool on) { writeFloat_ = on; }
    // the device context (after the first Render): parity tests read the uploaded BVH through it
    pbr_hip_ctx* Context() const { return ctx_; }
    const FlatScene* Flat() const { return flat_.get(); }
    // the render descriptor of the last Render (whole raster, host outputs): with Flat()->desc, what a
    // parity harness hands a CPU restatement to render the same frame
    const pbr_render_desc& LastRenderDesc() const { return lastDesc_; }

  private:
    const int integrator_, maxDepth_;
    const float rrThreshold_;
    const std::string strategy_;
    std::shared_ptr<PBR::Sampler> sampler_;
    const PBR::Bounds2i bounds_;
    ::FrameBuffer* fb_;
    int device_ = 0;
    bool writeFloat_ = false;
    pbr_render_desc lastDesc_{};
    pbr_hip_ctx* ctx_ = nullptr;
    const PBR::Scene* uploaded_ = nullptr;
    std::shared_ptr<FlatScene> flat_;
};

class HipWhittedIntegrator : public HipSamplerIntegrator {   // WhittedIntegrator.h:10-13
  public:
    HipWhittedIntegrator(int maxDepth, std::shared_ptr<const PBR::Camera> camera, std::shared_ptr<PBR::Sampler> sampler,
                         const PBR::Bounds2i& pixelBounds, ::FrameBuffer* frameBuffer)
        : HipSamplerIntegrator(PBR_INTEGRATOR_WHITTED, maxDepth, camera, sampler, pixelBounds, 1.f, "uniform", frameBuffer) {}
};
class HipPathIntegrator : public HipSamplerIntegrator {      // PathIntegrator.h:14-18
  public:
    HipPathIntegrator(int maxDepth, std::shared_ptr<const PBR::Camera> camera, std::shared_ptr<PBR::Sampler> sampler,
                      const PBR::Bounds2i& pixelBounds, float rrThreshold = 1, const std::string& lightSampleStrategy = "spatial",
                      ::FrameBuffer* frameBuffer = nullptr)
        : HipSamplerIntegrator(PBR_INTEGRATOR_PATH, maxDepth, camera, sampler, pixelBounds, rrThreshold, lightSampleStrategy,
                               frameBuffer) {}
};
class HipVolPathIntegrator : public HipSamplerIntegrator {   // VolPathIntegrator.h:13-17
  public:
    HipVolPathIntegrator(int maxDepth, std::shared_ptr<const PBR::Camera> camera, std::shared_ptr<PBR::Sampler> sampler,
                         const PBR::Bounds2i& pixelBounds, float rrThreshold = 1,
                         const std::string& lightSampleStrategy = "spatial", ::FrameBuffer* frameBuffer = nullptr)
        : HipSamplerIntegrator(PBR_INTEGRATOR_VOLPATH, maxDepth, camera, sampler, pixelBounds, rrThreshold,
                               lightSampleStrategy, frameBuffer) {}
};

}  // namespace pbrhip
