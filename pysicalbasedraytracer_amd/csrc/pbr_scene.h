// pbr_scene.h — host-side flattening of a pbr_scene_desc into the HBM layout of pbr_layout.h.
#pragma once
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/pbr_hip.h"
#include "pbr_layout.h"
#include "pbr_material.h"
#include "pbr_math.h"

namespace pbr {

struct LinearBVHNode {            // BVHAccel.cpp:46-55, 32 bytes
    float pMin[3], pMax[3];
    int32_t offset;               // primitivesOffset | secondChildOffset
    uint16_t nPrimitives;
    uint8_t axis;
    uint8_t pad;
};
static_assert(sizeof(LinearBVHNode) == 32, "LinearBVHNode is 32 bytes");

struct InfiniteHost {
    int light = -1;                         // index in lights, -1 = none
    int w = 0, h = 0;                       // level-0 resolution (powers of two)
    std::vector<float> tex;                 // 4 floats per texel, RGB + pad
    std::vector<float> condFunc, condCdf;   // h rows of w / w + 1
    std::vector<float> margFunc, margCdf;   // h / h + 1
    float margInt = 0;
    float l2w[16], w2l[16];
    float worldRadius = 0;
};

struct HostScene {
    std::vector<LinearBVHNode> nodes;
    std::vector<int32_t> primIds;           // ordered slot → index in the prims vector
    std::vector<float> triVerts;            // 12 floats per ordered prim
    std::vector<int32_t> primInfo;          // 4 ints per ordered prim
    std::vector<float> triUV;               // 6 floats per ordered prim (if any UVs)
    std::vector<SphereRec> spheres;
    std::vector<MatTemplate> materials;     // 2 per material
    std::vector<DLight> lights;
    std::vector<float> env;                 // 4 floats per texel
    int envLight = -1;
    std::vector<int> infinite;
    std::vector<float> lightCdf, lightFunc; // uniform distribution (power built per render)
    float lightFuncInt = 0;
    std::vector<float> lightPower;          // Power().y() per light (LightDistrib.cpp:36-41)
    std::vector<float> media;               // 10 floats per medium
    bool anyNoMaterial = false;             // some primitive has material == nullptr
    std::vector<float> wide;                // 16 floats per interior node (build_wide_nodes)
    int32_t rootRef = 0;
    std::vector<float> quad;                // 32 floats per quad node (build_quad_nodes)
    int32_t quadRootRef = 0;
    std::vector<float> primBounds;          // 6 floats (lo, hi) per primitive in prims order: GeometricPrimitive::WorldBound
    std::vector<int32_t> slotOf;            // prims index → BVH slot
    // traversal stack entries the tree can need at most (pbr_layout.h kTraversalStack): the binary
    // walk's (one per interior level on the deepest root-to-leaf path) and the quad walk's (per quad
    // node on a path, its valid slots minus the one entered)
    int binaryStackNeed = 0, quadStackNeed = 0;
    InfiniteHost inf;                       // the InfiniteAreaLight, if any (pbr_infinite.cpp)
    std::vector<TexDev> textures;           // ImageTextures (level 0 + mapping)
    std::vector<float> texTexels;           // their texels, 4 floats each
    std::vector<TexMat> texMats;            // per material, only when some material is textured
};

// InfiniteAreaLight tables (Light/InfiniteAreaLight.cpp:7-61): the level-0 MIPMap image (resampled
// to powers of two as Texture/MIPMap.h:86-150 does) and the Distribution2D over its luminance.
void build_infinite_light(const pbr_light_desc& ld, const float worldMin[3], const float worldMax[3],
                          InfiniteHost* out, float power[3]);
// BVHAccel's SAH build (BVHAccel.cpp:57-283) over primitive world bounds (6 floats per primitive in
// prims order): LinearBVHNode array in flatten order + orderedPrims ids.  The host builder
// (pbr_scene.cpp) and the device builder (pbr_bvh_build.hip, on `stream`; device time in kernelMs;
// throws std::runtime_error on a HIP failure) produce identical arrays.
void host_build_bvh(const std::vector<float>& primBounds, int maxPrims, std::vector<LinearBVHNode>* nodes,
                    std::vector<int32_t>* primIds, int splitMethod = PBR_SPLIT_SAH);
void device_build_bvh(void* stream, const std::vector<float>& primBounds, int maxPrims, std::vector<LinearBVHNode>* nodes,
                      std::vector<int32_t>* primIds, double* kernelMs);
// Interior boxes as InitInterior sets them: Union(first child, second child) (both builders end with it).
void interior_bounds_from_children(std::vector<LinearBVHNode>* nodes);
using BvhBuildFn = std::function<void(const std::vector<float>& primBounds, int maxPrims, std::vector<LinearBVHNode>* nodes,
                                      std::vector<int32_t>* primIds)>;

// ImageTexture's MIPMap level 0 (pbr_infinite.cpp): appends the texels, fills the record.
void build_image_texture(const pbr_texture_desc& td, TexDev* out, std::vector<float>* texels);

// Throws std::invalid_argument on a malformed descriptor.  `bvh` replaces the host SAH build.
void build_host_scene(const pbr_scene_desc* desc, HostScene* out, const BvhBuildFn* bvh = nullptr);

// Light sampling distribution (Distribution1D over lights): uniform or power.
void light_distribution(const HostScene& s, int strategy, std::vector<float>* cdf, std::vector<float>* func,
                        float* funcInt);

// Camera: RasterToCamera and CameraToWorld matrices exactly as CreatePerspectiveCamera builds them.
void build_camera(const pbr_camera_desc* cam, DeviceCamera* out);

// Halton: digit permutations for the first n primes (RNG default state), plus per-dim tables.
struct HaltonTables {
    std::vector<uint32_t> primes, recips, primeSums;
    std::vector<uint16_t> perms;
};
void build_halton_tables(int nPrimes, HaltonTables* t);
void halton_params(int resX, int resY, DeviceSampler* s);

// Sobol (pbrt-v3 SobolSampler): built-in generator matrices [nDims][kSobolMatrixSize] and the
// pixel → sample-index tables for resolution 2^m (see pbr_scene.cpp).
constexpr int kSobolMatrixSize = 52;
constexpr int kSobolMaxDims = 1024;   // SobolMatrices32 rows (NumSobolDimensions, SobolMatrices.h)
void build_sobol_matrices(int nDims, std::vector<uint32_t>* out);
void sobol_pixel_tables(const uint32_t* mats, int m, std::vector<uint32_t>* out);

}  // namespace pbr
