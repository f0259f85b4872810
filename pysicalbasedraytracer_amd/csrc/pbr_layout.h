// pbr_layout.h — HBM layout of a flattened scene on the MI355X (written by the host build in
// pbr_scene.cpp, read by the kernels in pbr_kernels.hip).
//
//  nodes     : float4[2*nNodes]   LinearBVHNode, 32 B, BVHAccel.cpp:46-55 order and semantics:
//              [0] = pMin.xyz, pMax.x   [1] = pMax.yz, offset (int bits), nPrims | axis<<16
//  triVerts  : float4[3*nPrims]   world-space vertices of the BVH-ordered primitive, 48 B/prim
//              (spheres: [0].x holds the sphere index)
//  primInfo  : int4[nPrims]       {flags, material, areaLight, mediumIn | mediumOut<<16}
//  triUV     : float2[3*nPrims]   only when some mesh carries UVs
//  materials : MatTemplate[2*nMaterials]  BSDF lobe templates for allowMultipleLobes = {false,true}
//  lights    : DLight[nLights]
//  env       : float4[w*h]        SkyBox texels with HDRtoLDR(·,0.3) applied once at upload
//  halton    : primes/reciprocals/prime sums + u16 digit permutations (1000 dims)
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>   // float4/int4/float2 vector types

namespace pbr {

enum PrimFlags { PRIM_SPHERE = 1, PRIM_FLIP = 2, PRIM_HAS_UV = 4, PRIM_LEAF_END = 8 };
constexpr uint32_t kLeafRef = 0x80000000u;   // traversal child reference: leaf | first slot
enum LobeKind { L_LAMBERT = 0, L_OREN = 1, L_SPEC_R = 2, L_SPEC_T = 3, L_FRESNEL_SPEC = 4, L_MF_R = 5, L_MF_T = 6 };
enum FresnelKind { FR_NOOP = 0, FR_DIEL = 1, FR_COND = 2 };
enum BxDFType { BSDF_REFLECTION = 1, BSDF_TRANSMISSION = 2, BSDF_DIFFUSE = 4, BSDF_GLOSSY = 8, BSDF_SPECULAR = 16, BSDF_ALL = 31 };

struct Lobe {                     // one BxDF with constant-texture parameters folded in (112 B)
    int kind, type, fresnel, pad;
    float R[3], T[3];
    float A, B;                   // Oren-Nayar
    float etaA, etaB;             // transmission / FresnelSpecular
    float ax, ay;                 // Trowbridge-Reitz alphas (already clamped/remapped)
    float fEtaI, fEtaT;           // FresnelDielectric
    float cEtaI[3], cEtaT[3], cK[3];  // FresnelConductor
};
struct MatTemplate {              // what Material::ComputeScatteringFunctions adds, minus the frame
    int valid;                    // 0: material == nullptr → no BSDF
    int nLobes;
    float eta;                    // BSDF::eta (glass index, else 1)
    int textured;                 // 1: some parameter is an image texture — the lobes are built per hit
    Lobe lobes[2];
};

enum LightType { LT_POINT = 0, LT_AREA = 1, LT_SKY = 2, LT_INF = 3 };
struct DLight {
    int type;
    int primSlot;                 // area light: BVH-ordered primitive slot of its triangle
    int twoSided;
    int medIn, medOut;
    int envW, envH;
    int pad;
    float L[3];                   // point I / area Lemit
    float p[3];                   // point position
    float area;                   // area light triangle area
    float worldRadius;            // skybox
};

// ImageTexture level 0 (pbr_infinite.cpp build_image_texture) + its UVMapping2D
struct TexDev {
    int offset;                   // first texel in DeviceScene::texels (float4; float textures use .x)
    int w, h, wrap, isFloat;
    float su, sv, du, dv;
    int pad[3];
};

struct SphereRec { float o2w[16]; float w2o[16]; float radius; int flip; int pad[2]; };

// InfiniteAreaLight (Light/InfiniteAreaLight.cpp): level-0 MIPMap texels and its Distribution2D
struct InfDev {
    const float4* tex;             // w*h texels (RGB), powers of two
    const float* condFunc;         // h rows of w
    const float* condCdf;          // h rows of w + 1
    const float* margFunc;         // h (= each row's funcInt)
    const float* margCdf;          // h + 1
    float margInt;
    int w, h;
    float l2w[12], w2l[12];        // LightToWorld / WorldToLight, top three rows
};

struct DeviceScene {
    const float4* nodes;
    const float4* wide;            // 4 float4 per interior node: child boxes, child refs, axis
    int rootRef;
    const float4* quad;            // 8 float4 per quad node (two binary levels, pbr_scene.cpp build_quad_nodes)
    int quadRootRef;
    int binaryWalk;                // 1: the quad walk's stack could overflow in this tree (megakernel, binary walk)
    const float4* triVerts;
    const int4* primInfo;
    const float2* triUV;
    const SphereRec* spheres;
    const MatTemplate* materials;  // [2*m + multiLobe]
    const DLight* lights;
    const float4* env;             // texels of the (single) skybox, or null
    int nNodes, nPrims, nLights, nMaterials;
    int envLight;                  // index of the skybox light or -1
    int nInfinite;
    int infinite[4];
    // light distribution (Distribution1D over lights, LightDistrib.cpp)
    const float* lightCdf;         // n+1
    const float* lightFunc;        // n
    float lightFuncInt;
    // media
    const float* media;            // per medium: sigma_a[3] sigma_s[3] sigma_t[3] g → 10 floats
    int nMedia;
    const InfDev* inf;             // the InfiniteAreaLight's tables (device memory), or null
    int* guard;                    // set (kGuard*) when a walk stops at a safety bound; the render then fails
    // image textures (only scenes with textured materials)
    const float4* texels;
    const TexDev* textures;
    const struct TexMat* texMats;  // per material (pbr_material.h)
};
// Safety bounds of walks the reference runs without limit; reaching one fails the render
// (PBR_E_UNSUPPORTED) instead of returning a silently truncated result.
constexpr int kGuardWhittedPassThrough = 1;   // > kMaxPassThrough material-less crossings in one Whitted Li
constexpr int kGuardTransmittance = 2;        // > kMaxTrCrossings interfaces on one VisibilityTester::Tr walk
constexpr int kGuardStack = 4;                // a traversal stack was full (never, given the upload check below)
constexpr int kGuardSampleTable = 8;          // a path asked a PBR_SAMPLER_TABLE sampler for a dimension it lacks
constexpr int kMaxPassThrough = 1024;
constexpr int kMaxTrCrossings = 256;
// Traversal stacks (pbr_device.h): BVHAccel's 64 entries (BVHAccel.cpp:293).  The binary walk pushes
// at most one entry per interior level; a quad node (two binary levels) pushes up to three.  The
// upload measures both needs on the built tree (HostScene::binaryStackNeed / quadStackNeed): a tree
// the quad walk could overflow renders with the megakernel over the binary layout
// (DeviceScene::binaryWalk), and one deeper than the reference's own 64-entry stack is refused, so
// no walk is ever truncated.
constexpr int kTraversalStack = 64;
constexpr int kQuadStackLimit = kTraversalStack - 3;   // a quad walk pushes only while sp <= 61

struct DeviceSampler {
    int type;                      // pbr_sampler_type
    int spp;
    int baseExp0, baseExp1, baseScale1, stride, mult0, mult1, ratio0, ratio1;
    const uint32_t* primes;        // [1000]
    const uint32_t* recips;        // floor(2^32/p)
    const uint32_t* primeSums;     // [1000]
    const uint16_t* perms;         // digit permutations
    const uint32_t* sobol;         // Sobol nibble tables of matrix columns 0..31 (dims × 128), or null
    int nSobolDims;
    int sobolLog2Res;              // log2 of the power-of-two resolution
    int sobolRes;
    const uint32_t* sobolPix;      // sobol_pixel_tables: T_low^-1 columns [2m], T_high columns [52 - 2m]
    const uint32_t* sobolHi;       // nibble tables of matrix columns 32..51 (index bits >= 32)
    int wideIndex;                 // some sample index of this render needs bits >= 32
    int hiShift;                   // 32 - 2m: sample number >> hiShift = the index's bits >= 32
    int ldsDims;                   // Halton dimensions a kernel may stage in LDS (<= 64)
    // PBR_SAMPLER_TABLE: the caller's values, [((y * tableW + x) * spp + s) * tableDims + dim]
    const float* table;
    int tableDims, tableW;
    int* guard;                    // DeviceScene::guard: a dimension beyond the table fails the frame
};

struct DeviceCamera {
    float rasterToCamera[16];
    float cameraToWorld[16];
    float lensRadius, focalDistance;
    int width, height;
};

}  // namespace pbr
