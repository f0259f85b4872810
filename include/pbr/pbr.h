// pbr/pbr.h — C++ host API of the MI355X render path, mirroring the reference's classes.
//
// A program written against G0T-cha/PysicalBasedRaytracer's scene API (Main/main.cpp builds a
// scene from these classes and calls Integrator::Render) compiles against this header with the
// same class names, constructor arguments and call sequence; Render then runs on the GPU through
// the C-ABI of include/pbr_hip.h.  Only what the render path consumes is kept: shapes, materials
// with constant textures, lights, media, the BVH aggregate, the perspective camera, the Halton
// sampler, the frame buffer and the three sampler integrators.
//
// Differences from the reference, all deliberate:
//  * no CPU ray tracing: Primitive/Scene/BVHAccel hold the scene for flattening; intersection
//    queries run on the device (pbr_hip_intersect) — BVHAccel is built on upload, node for node
//    identical to the reference's (Accelerator/BVHAccel.cpp:57-283);
//  * Render fails loudly (std::runtime_error) instead of silently: no device, bad scene, etc.;
//  * Render writes the whole W×H frame (the reference's loop renders min(W,H)², finding F1) and
//    also fills the float buffer (getFCbuffer, F7).
#pragma once
#include <algorithm>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../pbr_hip.h"   // pbr_sampler_type (Sampler::DeviceSampler)

struct pbr_hip_ctx;
struct pbr_scene_desc;

// ---------------------------------------------------------------------------- FrameBuffer
// Core/FrameBuffer.h (global namespace, as in the reference)
class FrameBuffer {
  public:
    FrameBuffer() = default;
    ~FrameBuffer() = default;
    FrameBuffer(const FrameBuffer&) = delete;
    FrameBuffer& operator=(const FrameBuffer&) = delete;
    void InitBuffer(int width = 800, int height = 600, int channals = 4);
    void FreeBuffer();
    bool bufferResize(int width = 800, int height = 600);
    bool set_uc(int w, int h, int shifting, const unsigned char& dat);
    bool set_fc(int w, int h, int shifting, const float& dat);
    // progressive running average (FrameBuffer.h:112-126): f = dat/n + (1 - 1/n)·f, u8 = f·255
    bool update_f_u_c(int w, int h, int shifting, int renderCount, const float& dat);
    unsigned char* getUCbuffer() { return ubuffer.data(); }
    float* getFCbuffer() { return fbuffer.data(); }   // linear RGB(A) colObj/spp (not in the reference, F7)
    int width = 0, height = 0, channals = 4;

  private:
    std::vector<unsigned char> ubuffer;
    std::vector<float> fbuffer;
};

// The two stb_image_write calls main.cpp makes to save the FrameBuffer (main.cpp:419-429), so it
// compiles unchanged.  The PNG (8-bit grey / grey+alpha / RGB / RGBA for comp 1-4) is written with
// stored deflate blocks: any PNG reader decodes the same pixels as from stb's compressed file.
// Returns 1 on success, 0 on failure, like stb.
void stbi_flip_vertically_on_write(int flag);
int stbi_write_png(char const* filename, int w, int h, int comp, const void* data, int stride_in_bytes);

namespace PBR {

// ---------------------------------------------------------------------------- Core/Geometry.h
struct Vector3f {
    float x = 0, y = 0, z = 0;
    Vector3f() = default;
    Vector3f(float x, float y, float z) : x(x), y(y), z(z) {}
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
struct Point3f : Vector3f {
    using Vector3f::Vector3f;
    Point3f() = default;
};
struct Normal3f : Vector3f {
    using Vector3f::Vector3f;
    Normal3f() = default;
};
struct Point2f {
    float x = 0, y = 0;
    Point2f() = default;
    Point2f(float x, float y) : x(x), y(y) {}
};
struct Point2i {
    int x = 0, y = 0;
    Point2i() = default;
    Point2i(int x, int y) : x(x), y(y) {}
};
struct Bounds2i {
    Point2i pMin, pMax;
    Bounds2i() = default;
    Bounds2i(const Point2i& a, const Point2i& b) : pMin(a), pMax(b) {}
};
struct Bounds2f {
    Point2f pMin, pMax;
    Bounds2f() = default;
    Bounds2f(const Point2f& a, const Point2f& b) : pMin(a), pMax(b) {}
};

struct Bounds3f {   // Core/Geometry.h: an empty box is (+max, -max)
    Point3f pMin, pMax;
    Bounds3f();
    Bounds3f(const Point3f& a, const Point3f& b) : pMin(a), pMax(b) {}
};
struct Vector2f {
    float x = 0, y = 0;
};
class Medium;
// Core/Geometry.h Ray: tMax is mutable (Intersect shortens it)
struct Ray {
    Ray() = default;
    Ray(const Point3f& o, const Vector3f& d, float tMax = 3.40282347e+38f * 2.f, float time = 0.f,
        const Medium* medium = nullptr)
        : o(o), d(d), tMax(tMax), time(time), medium(medium) {}
    Point3f operator()(float t) const { return Point3f(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t); }
    Point3f o;
    Vector3f d;
    mutable float tMax = 3.40282347e+38f * 2.f;   // Infinity
    float time = 0.f;
    const Medium* medium = nullptr;
};
struct RayDifferential : Ray {   // the differentials are never read on the render path (F5)
    using Ray::Ray;
    RayDifferential() = default;
    RayDifferential(const Ray& r) : Ray(r) {}
    void ScaleDifferentials(float) {}
    bool hasDifferentials = false;
};

// ---------------------------------------------------------------------------- Core/Spectrum.h
class Spectrum {   // RGBSpectrum
  public:
    explicit Spectrum(float v = 0.f) : c{v, v, v} {}
    static Spectrum FromRGB(const float rgb[3]) { Spectrum s; s.c[0] = rgb[0]; s.c[1] = rgb[1]; s.c[2] = rgb[2]; return s; }
    float operator[](int i) const { return c[i]; }
    float& operator[](int i) { return c[i]; }

  private:
    float c[3];
};

// ---------------------------------------------------------------------------- Core/Transform.h
struct Matrix4x4 {
    float m[4][4];
    Matrix4x4();   // identity
    explicit Matrix4x4(const float mat[4][4]);
    Matrix4x4(float t00, float t01, float t02, float t03, float t10, float t11, float t12, float t13,
              float t20, float t21, float t22, float t23, float t30, float t31, float t32, float t33);
};
Matrix4x4 Inverse(const Matrix4x4& m);   // Gauss-Jordan with full pivoting, as the reference
Matrix4x4 Mul(const Matrix4x4& a, const Matrix4x4& b);

class Transform {
  public:
    Transform() = default;
    explicit Transform(const float mat[4][4]);
    explicit Transform(const Matrix4x4& m);
    Transform(const Matrix4x4& m, const Matrix4x4& mInv) : m(m), mInv(mInv) {}
    friend Transform Inverse(const Transform& t) { return Transform(t.mInv, t.m); }
    Transform operator*(const Transform& t2) const;
    const Matrix4x4& GetMatrix() const { return m; }
    const Matrix4x4& GetInverseMatrix() const { return mInv; }

  private:
    Matrix4x4 m, mInv;
};
Transform Translate(const Vector3f& delta);
Transform Scale(float x, float y, float z);
Transform RotateX(float theta);   // degrees
Transform RotateY(float theta);
Transform RotateZ(float theta);
Transform LookAt(const Point3f& pos, const Point3f& look, const Vector3f& up);

// ---------------------------------------------------------------------------- Texture/
template <typename T>
class Texture {
  public:
    virtual ~Texture() = default;
    // The render path only evaluates constant textures (every material in main.cpp uses them).
    virtual bool IsConstant() const { return false; }
    virtual T ConstantValue() const { throw std::invalid_argument("only constant textures reach the GPU path"); }
};
template <typename T>
class ConstantTexture : public Texture<T> {
  public:
    explicit ConstantTexture(const T& value) : value(value) {}
    bool IsConstant() const override { return true; }
    T ConstantValue() const override { return value; }

  private:
    T value;
};

using RGBSpectrum = Spectrum;

// Texture/Texture.h:9-27, Texture/MIPMap.h:21, Texture/ImageTexture.h:43-91
enum class ImageWrap { Repeat, Black, Clamp };
class TextureMapping2D {
  public:
    virtual ~TextureMapping2D() = default;
};
class UVMapping2D : public TextureMapping2D {
  public:
    UVMapping2D(float su = 1, float sv = 1, float du = 0, float dv = 0) : su(su), sv(sv), du(du), dv(dv) {}
    const float su, sv, du, dv;
};
// The image of an ImageTexture, as its loadImage (stbi_loadf with flip-on-load) hands it over.
struct ImageTextureData {
    const UVMapping2D* mapping = nullptr;   // nullptr: a mapping other than UVMapping2D (refused by the GPU path)
    int width = 0, height = 0, components = 0;
    std::vector<float> data;                // empty → GetTexture's 0.5 grey image
    bool doTrilinear = false, gamma = false, isFloat = false;
    float maxAniso = 8.f, scale = 1.f;
    ImageWrap wrapMode = ImageWrap::Repeat;
};
template <typename Tmemory, typename Treturn>
class ImageTexture : public Texture<Treturn> {
  public:
    // Loads `filename` as loadImage does: a Radiance .hdr read the way stbi_loadf reads it, rows
    // flipped (stbi_set_flip_vertically_on_load(true), ImageTexture.cpp:19); a missing or unreadable
    // file gives the 0.5 grey image (ImageTexture.cpp:60-66).
    ImageTexture(std::unique_ptr<TextureMapping2D> mapping, const std::string& filename, bool doTrilinear, float maxAniso,
                 ImageWrap wrapMode, float scale, bool gamma);
    // In-memory variant: data = width*height*components floats in stbi_loadf's (flipped) row order.
    ImageTexture(std::unique_ptr<TextureMapping2D> mapping, int width, int height, int components, std::vector<float> data,
                 bool doTrilinear, float maxAniso, ImageWrap wrapMode, float scale, bool gamma);
    const ImageTextureData& Image() const { return img; }

  private:
    std::unique_ptr<TextureMapping2D> mapping;
    ImageTextureData img;
};

// ---------------------------------------------------------------------------- Media/
class Medium {
  public:
    virtual ~Medium() = default;
};
class HomogeneousMedium : public Medium {   // Media/HomogeneousMedium.h
  public:
    HomogeneousMedium(const Spectrum& sigma_a, const Spectrum& sigma_s, float g) : sigma_a(sigma_a), sigma_s(sigma_s), g(g) {}
    const Spectrum sigma_a, sigma_s;
    const float g;
};
struct MediumInterface {   // Media/Medium.h:55-60
    MediumInterface() : inside(nullptr), outside(nullptr) {}
    MediumInterface(const Medium* medium) : inside(medium), outside(medium) {}
    MediumInterface(const Medium* inside, const Medium* outside) : inside(inside), outside(outside) {}
    bool IsMediumTransition() const { return inside != outside; }
    const Medium *inside, *outside;
};

// ---------------------------------------------------------------------------- Shape/
class Shape {
  public:
    Shape(const Transform* ObjectToWorld, const Transform* WorldToObject, bool reverseOrientation)
        : ObjectToWorld(ObjectToWorld), WorldToObject(WorldToObject), reverseOrientation(reverseOrientation) {}
    virtual ~Shape() = default;
    const Transform *ObjectToWorld, *WorldToObject;   // not owned (as in the reference, Shape.h:35)
    const bool reverseOrientation;
};
struct TriangleMesh {   // Shape/Triangle.h:11-24; vertices kept in object space, baked on upload
    TriangleMesh(const Transform& ObjectToWorld, int nTriangles, const int* vertexIndices, int nVertices, const Point3f* P,
                 const Vector3f* S, const Normal3f* N, const Point2f* uv, const int* faceIndices);
    const int nTriangles, nVertices;
    Transform objectToWorld;
    std::vector<int> vertexIndices;
    std::vector<float> p;    // 3 per vertex
    std::vector<float> n;    // 3 per vertex or empty
    std::vector<float> uv;   // 2 per vertex or empty
};
class Triangle : public Shape {
  public:
    Triangle(const Transform* ObjectToWorld, const Transform* WorldToObject, bool reverseOrientation,
             const std::shared_ptr<TriangleMesh>& mesh, int triNumber)
        : Shape(ObjectToWorld, WorldToObject, reverseOrientation), mesh(mesh), triNumber(triNumber) {}
    const std::shared_ptr<TriangleMesh> mesh;
    const int triNumber;
};
std::vector<std::shared_ptr<Shape>> CreateTriangleMesh(const Transform* ObjectToWorld, const Transform* WorldToObject,
                                                       bool reverseOrientation, int nTriangles, const int* vertexIndices,
                                                       int nVertices, const Point3f* p, const Vector3f* s,
                                                       const Normal3f* n, const Point2f* uv, const int* faceIndices = nullptr);
class Sphere : public Shape {
  public:
    Sphere(const Transform* ObjectToWorld, const Transform* WorldToObject, bool reverseOrientation, float radius)
        : Shape(ObjectToWorld, WorldToObject, reverseOrientation), radius(radius) {}
    const float radius;
};
// Shape/plyRead.h: the reference's ".3d" text format ("vertex N face M", vertices ×20)
class plyInfo {
  public:
    explicit plyInfo(const std::string& filePath);
    int nVertices = 0, nTriangles = 0;
    std::vector<Point3f> vertexArray;
    std::vector<int> vertexIndices;
};
// Standard PLY (ascii / binary_little_endian; x y z vertices, triangle or quad faces) for the real
// Stanford Dragon.  Vertices are not scaled.
struct PlyMesh {
    std::vector<Point3f> vertices;
    std::vector<int> indices;
};
PlyMesh LoadPLY(const std::string& path);

// ---------------------------------------------------------------------------- Material/
class Material {
  public:
    virtual ~Material() = default;
};
using SpectrumTexture = std::shared_ptr<Texture<Spectrum>>;
using FloatTexture = std::shared_ptr<Texture<float>>;
class MatteMaterial : public Material {   // Material/MatteMaterial.h
  public:
    MatteMaterial(const SpectrumTexture& Kd, const FloatTexture& sigma, const FloatTexture& bumpMap)
        : Kd(Kd), sigma(sigma), bumpMap(bumpMap) {}
    SpectrumTexture Kd;
    FloatTexture sigma, bumpMap;
};
class MirrorMaterial : public Material {   // Material/Mirror.h
  public:
    MirrorMaterial(const SpectrumTexture& r, const FloatTexture& bump) : Kr(r), bumpMap(bump) {}
    SpectrumTexture Kr;
    FloatTexture bumpMap;
};
class GlassMaterial : public Material {   // Material/GlassMaterial.h
  public:
    GlassMaterial(const SpectrumTexture& Kr, const SpectrumTexture& Kt, const FloatTexture& uRoughness,
                  const FloatTexture& vRoughness, const FloatTexture& index, const FloatTexture& bumpMap, bool remapRoughness)
        : Kr(Kr), Kt(Kt), uRoughness(uRoughness), vRoughness(vRoughness), index(index), bumpMap(bumpMap), remapRoughness(remapRoughness) {}
    SpectrumTexture Kr, Kt;
    FloatTexture uRoughness, vRoughness, index, bumpMap;
    bool remapRoughness;
};
class MetalMaterial : public Material {   // Material/MetalMaterial.h
  public:
    MetalMaterial(const SpectrumTexture& eta, const SpectrumTexture& k, const FloatTexture& rough, const FloatTexture& urough,
                  const FloatTexture& vrough, const FloatTexture& bump, bool remapRoughness)
        : eta(eta), k(k), roughness(rough), uRoughness(urough), vRoughness(vrough), bumpMap(bump), remapRoughness(remapRoughness) {}
    SpectrumTexture eta, k;
    FloatTexture roughness, uRoughness, vRoughness, bumpMap;
    bool remapRoughness;
};
class PlasticMaterial : public Material {   // Material/PlasticMaterial.h
  public:
    PlasticMaterial(const SpectrumTexture& Kd, const SpectrumTexture& Ks, const FloatTexture& roughness,
                    const FloatTexture& bumpMap, bool remapRoughness)
        : Kd(Kd), Ks(Ks), roughness(roughness), bumpMap(bumpMap), remapRoughness(remapRoughness) {}
    SpectrumTexture Kd, Ks;
    FloatTexture roughness, bumpMap;
    bool remapRoughness;
};

// ---------------------------------------------------------------------------- Light/
class Light {
  public:
    Light(const Transform& LightToWorld, const MediumInterface& mediumInterface, int nSamples = 1)
        : nSamples(nSamples > 1 ? nSamples : 1), mediumInterface(mediumInterface), LightToWorld(LightToWorld) {}
    virtual ~Light() = default;
    virtual bool IsInfinite() const { return false; }
    const int nSamples;
    const MediumInterface mediumInterface;
    const Transform LightToWorld;
};
class PointLight : public Light {   // Light/PointLight.h
  public:
    PointLight(const Transform& LightToWorld, const MediumInterface& mediumInterface, const Spectrum& I)
        : Light(LightToWorld, mediumInterface), I(I) {}
    const Spectrum I;
};
class AreaLight : public Light {
  public:
    using Light::Light;
};
class DiffuseAreaLight : public AreaLight {   // Light/DiffuseLight.h
  public:
    DiffuseAreaLight(const Transform& LightToWorld, const MediumInterface& mediumInterface, const Spectrum& Le, int nSamples,
                     const std::shared_ptr<Shape>& shape, bool twoSided = false)
        : AreaLight(LightToWorld, mediumInterface, nSamples), Lemit(Le), shape(shape), twoSided(twoSided) {}
    const Spectrum Lemit;
    const std::shared_ptr<Shape> shape;
    const bool twoSided;
};
class SkyBoxLight : public Light {   // Light/SkyBoxLight.h
  public:
    // Loads a Radiance .hdr the way stbi_loadf does (vertically flipped, 3 components).
    SkyBoxLight(const Transform& LightToWorld, const Point3f& worldCenter, float worldRadius, const char* file, int nSamples);
    // In-memory variant: data = width*height*components floats, already in stbi_loadf's row order.
    SkyBoxLight(const Transform& LightToWorld, const Point3f& worldCenter, float worldRadius, int width, int height,
                int components, std::vector<float> data, int nSamples);
    bool IsInfinite() const override { return true; }
    bool loadImage(const char* imageFile);
    const Point3f worldCenter;
    const float worldRadius;
    int imageWidth = 0, imageHeight = 0, nrComponents = 0;
    std::vector<float> data;
};

class InfiniteAreaLight : public Light {   // Light/InfiniteAreaLight.h
  public:
    // Loads texmap the way stbi_loadf does: rows flipped only if a SkyBoxLight has already set
    // stb's global stbi_set_flip_vertically_on_load(true) (SkyBoxLight.cpp:20); "" → constant power.
    InfiniteAreaLight(const Transform& LightToWorld, const Spectrum& power, int nSamples, const std::string& texmap);
    // In-memory variant: data = width*height*components floats in stbi_loadf's row order (empty → constant).
    InfiniteAreaLight(const Transform& LightToWorld, const Spectrum& power, int nSamples, int width, int height,
                      int components, std::vector<float> data);
    bool IsInfinite() const override { return true; }
    const Spectrum L;
    int imageWidth = 0, imageHeight = 0, nrComponents = 0;
    std::vector<float> data;
};

// ---------------------------------------------------------------------------- Core/Interaction.h
class Primitive;
enum class TransportMode { Radiance, Importance };   // Material/Material.h
// SurfaceInteraction (Core/Interaction.h:56-105) as Scene::Intersect fills it: the hit's fields come
// from the device (pbr_hip_query); the BSDF itself is built and evaluated on the device by the
// integrators, so ComputeScatteringFunctions records the scattering material and mode only.
class SurfaceInteraction {
  public:
    Point3f p;
    Vector3f pError;
    Vector3f wo;
    Normal3f n;
    float time = 0;
    MediumInterface mediumInterface;
    Point2f uv;
    Vector3f dpdu;
    struct {
        Normal3f n;
        Vector3f dpdu;
    } shading;
    const Primitive* primitive = nullptr;
    // set by ComputeScatteringFunctions (Primitive.cpp:46-53): the material the device scatters with
    const Material* bsdfMaterial = nullptr;
    TransportMode mode = TransportMode::Radiance;
    bool allowMultipleLobes = false;
    // not in the reference: the watertight test's barycentrics and the primitive's index in the
    // BVHAccel's primitive vector
    float b0 = 0, b1 = 0, b2 = 0;
    int primIndex = -1;
    const Medium* GetMedium(const Vector3f& w) const;   // Interaction.h:48-50
};

// ---------------------------------------------------------------------------- Core/Primitive.h
class Scene;
class Primitive {   // Core/Primitive.h:11-22
  public:
    virtual ~Primitive() = default;
    virtual Bounds3f WorldBound() const = 0;
    virtual bool Intersect(const Ray& r, SurfaceInteraction*) const = 0;
    virtual bool IntersectP(const Ray& r) const = 0;
    virtual const AreaLight* GetAreaLight() const = 0;
    virtual const Material* GetMaterial() const = 0;
    virtual void ComputeScatteringFunctions(SurfaceInteraction* isect, TransportMode mode, bool allowMultipleLobes) const = 0;
};
// Intersection queries run on the device of the Scene that holds the primitive (a primitive that
// belongs to no Scene throws std::logic_error): one query per call, or batched through
// Scene::Intersect(const std::vector<Ray>&, ...).
class GeometricPrimitive : public Primitive {   // Core/Primitive.h:24-45, Core/Primitive.cpp
  public:
    GeometricPrimitive(const std::shared_ptr<Shape>& shape, const std::shared_ptr<Material>& material,
                       const std::shared_ptr<AreaLight>& areaLight, const MediumInterface& mediumInterface)
        : material(material), areaLight(areaLight), shape(shape), mediumInterface(mediumInterface) {}
    Bounds3f WorldBound() const override;
    bool Intersect(const Ray& r, SurfaceInteraction* isect) const override;
    bool IntersectP(const Ray& r) const override;
    const AreaLight* GetAreaLight() const override { return areaLight.get(); }
    const Material* GetMaterial() const override { return material.get(); }
    void ComputeScatteringFunctions(SurfaceInteraction* isect, TransportMode mode, bool allowMultipleLobes) const override;
    std::shared_ptr<Material> material;
    std::shared_ptr<AreaLight> areaLight;
    std::shared_ptr<Shape> shape;
    MediumInterface mediumInterface;
    // the Scene (and index in its BVHAccel) whose device answers this primitive's queries
    mutable const Scene* owner = nullptr;
    mutable int ownerIndex = -1;
};
class Aggregate : public Primitive {   // Core/Primitive.h:47-55
  public:
    const AreaLight* GetAreaLight() const override { return nullptr; }
    const Material* GetMaterial() const override { return nullptr; }
    void ComputeScatteringFunctions(SurfaceInteraction*, TransportMode, bool) const override {}
};
class BVHAccel : public Aggregate {   // Accelerator/BVHAccel.h:16-21; built on the device at upload
  public:
    // SAH is the reference's builder; HLBVH falls through to SAH there (BVHAccel.cpp:131-160, no
    // HLBVH code path) and here.  SAH/HLBVH build on the device; Middle and EqualCounts run the host
    // builder (std::partition / std::nth_element as BVHAccel.cpp:136-158 calls them) at upload.
    enum class SplitMethod { SAH, HLBVH, Middle, EqualCounts };
    BVHAccel(std::vector<std::shared_ptr<Primitive>> p, int maxPrimsInNode = 1, SplitMethod splitMethod = SplitMethod::SAH);
    const std::vector<std::shared_ptr<Primitive>>& Primitives() const { return primitives; }
    Bounds3f WorldBound() const override;
    bool Intersect(const Ray& r, SurfaceInteraction* isect) const override;
    bool IntersectP(const Ray& r) const override;
    const int maxPrimsInNode;
    const SplitMethod splitMethod;
    mutable const Scene* owner = nullptr;

  private:
    std::vector<std::shared_ptr<Primitive>> primitives;
};

// ---------------------------------------------------------------------------- Core/Scene.h
struct SceneDevice;
class Scene {   // Core/Scene.h:13-29
  public:
    Scene(std::shared_ptr<Primitive> aggregate, const std::vector<std::shared_ptr<Light>>& lights);
    ~Scene();
    Scene(const Scene&) = delete;
    Scene& operator=(const Scene&) = delete;
    const Bounds3f& WorldBound() const;   // the BVH root box
    bool Intersect(const Ray& ray, SurfaceInteraction* isect) const;
    bool IntersectP(const Ray& ray) const;
    // batched queries (one device launch): hit[i] = whether rays[i] hit; rays' tMax are updated
    void Intersect(const std::vector<Ray>& rays, std::vector<SurfaceInteraction>* isects, std::vector<char>* hit) const;
    void IntersectP(const std::vector<Ray>& rays, std::vector<char>* hit) const;
    // one primitive of the BVHAccel (GeometricPrimitive::Intersect / IntersectP on the device)
    bool IntersectPrimitive(int index, const Ray& ray, SurfaceInteraction* isect) const;
    bool IntersectPPrimitive(int index, const Ray& ray) const;
    Bounds3f PrimitiveBound(int index) const;
    std::vector<std::shared_ptr<Light>> lights;
    std::vector<std::shared_ptr<Light>> infiniteLights;
    const std::shared_ptr<Primitive>& GetAggregate() const { return aggregate; }
    uint64_t Id() const { return id; }   // identifies the scene for upload caching
    void SetQueryDevice(int device) { queryDevice = device; }   // the GPU that answers the queries (default 0)

  private:
    SceneDevice& device() const;
    std::shared_ptr<Primitive> aggregate;
    uint64_t id;
    int queryDevice = 0;
    mutable std::unique_ptr<SceneDevice> dev;
};

// ---------------------------------------------------------------------------- Camera/
struct CameraSample {   // Camera/Camera.h
    Point2f pFilm, pLens;
    float time = 0;
};
// Camera rays, sampler values and SamplerIntegrator::Li below are computed on a GPU (device 0 for the
// camera and sampler helpers, the integrator's device for Li): the reference's per-sample loop
// (Integrator.cpp:286-313) can be written against these classes and gives the frame Render gives.
class Camera {
  public:
    virtual ~Camera() = default;
    virtual float GenerateRay(const CameraSample& sample, Ray* ray) const = 0;
    virtual float GenerateRayDifferential(const CameraSample& sample, RayDifferential* rd) const {
        return GenerateRay(sample, rd);   // differentials are dead on the render path (F5)
    }
};
class PerspectiveCamera : public Camera {   // Camera/Perspective.h
  public:
    PerspectiveCamera(int RasterWidth, int RasterHeight, const Transform& CameraToWorld, const Bounds2f& screenWindow,
                      float lensRadius, float focalDistance, float fov, const Medium* medium);
    // Perspective.cpp:44-62 on the device (pbr_hip_camera_rays); pinhole cameras only
    float GenerateRay(const CameraSample& sample, Ray* ray) const override;
    const int RasterWidth, RasterHeight;
    const Transform CameraToWorld;
    const Bounds2f screenWindow;
    const float lensRadius, focalDistance, fov;
    const Medium* medium;
};
PerspectiveCamera* CreatePerspectiveCamera(int RasterWidth, int RasterHeight, const Transform& cam2world, Medium* media);

// ---------------------------------------------------------------------------- Sampler/
// PCG32 (Sampler/RNG.h): pbrt's RNG, the fallback of PixelSampler beyond its sampled dimensions.
class RNG {
  public:
    RNG() : state(0x853c49e6748fea9bULL), inc(0xda3e39cb94b95bdbULL) {}
    explicit RNG(uint64_t sequenceIndex) { SetSequence(sequenceIndex); }
    void SetSequence(uint64_t initseq) {
        state = 0u;
        inc = (initseq << 1u) | 1u;
        UniformUInt32();
        state += 0x853c49e6748fea9bULL;
        UniformUInt32();
    }
    uint32_t UniformUInt32() {
        const uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        const uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        const uint32_t rot = (uint32_t)(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
    }
    float UniformFloat() { return std::min(0.99999994f, float(UniformUInt32() * 2.3283064365386963e-10f)); }

  private:
    uint64_t state, inc;
};

// Sampler (Sampler/Sampler.h:13-43) with the reference's interface — Get1D/Get2D/Clone pure
// virtual, GetCameraSample from them (Sampler.cpp:10-21), the 1D/2D sample arrays — plus
// PixelSampler (Sampler.h:46-60) and GlobalSampler (Sampler.h:62-82) with its pure
// GetIndexForSample / SampleDimension, so a sampler subclass written against the reference compiles
// here.  HaltonSampler and SobolSampler compute their values on the device
// (pbr_hip_sample_index / pbr_hip_sample_dimensions, batched per block of dimensions); any other
// GlobalSampler subclass renders too: Render tabulates its SampleDimension values for the frame
// (PBR_SAMPLER_TABLE) and the device reads them.
class Sampler {
  public:
    explicit Sampler(int64_t samplesPerPixel) : samplesPerPixel(samplesPerPixel) {}
    virtual ~Sampler() = default;
    virtual void StartPixel(const Point2i& p);
    virtual float Get1D() = 0;
    virtual Point2f Get2D() = 0;
    CameraSample GetCameraSample(const Point2i& pRaster);   // pFilm = pRaster + Get2D(), time = Get1D(), pLens = Get2D()
    void Request1DArray(int n);
    void Request2DArray(int n);
    virtual int RoundCount(int n) const { return n; }
    const float* Get1DArray(int n);
    const Point2f* Get2DArray(int n);
    virtual bool StartNextSample();
    virtual std::unique_ptr<Sampler> Clone(int seed) = 0;
    virtual bool SetSampleNumber(int64_t sampleNum);
    int64_t CurrentSampleNumber() const { return currentPixelSampleIndex; }
    const int64_t samplesPerPixel;
    // Extensions, with defaults for samplers written against the reference's interface: where the
    // sampler stands (SamplerIntegrator::Li continues the sample on the device from pixel, sample
    // number and next dimension; -1: not tracked), which device sampler serves it
    // (PBR_SAMPLER_TABLE: none — Render tabulates a GlobalSampler's values), and the raster its
    // sample indices are defined on ((0, 0): the camera's).
    const Point2i& CurrentPixel() const { return currentPixel; }
    virtual int CurrentDimension() const { return -1; }
    virtual int DeviceSampler() const { return PBR_SAMPLER_TABLE; }
    virtual Point2i SampleRaster() const { return Point2i(0, 0); }

  protected:
    Point2i currentPixel;
    int64_t currentPixelSampleIndex = 0;
    std::vector<int> samples1DArraySizes, samples2DArraySizes;
    std::vector<std::vector<float>> sampleArray1D;
    std::vector<std::vector<Point2f>> sampleArray2D;

  private:
    size_t array1DOffset = 0, array2DOffset = 0;
};
// PixelSampler (Sampler.h:46-60, Sampler.cpp:67-95): a subclass fills samples1D / samples2D in its
// StartPixel; dimensions beyond them come from rng.  Its 1D and 2D values are separate streams,
// which the device's single dimension counter cannot reproduce: Render refuses it (per-pixel API only).
class PixelSampler : public Sampler {
  public:
    PixelSampler(int64_t samplesPerPixel, int nSampledDimensions);
    bool StartNextSample() override;
    bool SetSampleNumber(int64_t) override;
    float Get1D() override;
    Point2f Get2D() override;

  protected:
    std::vector<std::vector<float>> samples1D;
    std::vector<std::vector<Point2f>> samples2D;
    int current1DDimension = 0, current2DDimension = 0;
    RNG rng;
};
class GlobalSampler : public Sampler {
  public:
    explicit GlobalSampler(int64_t samplesPerPixel) : Sampler(samplesPerPixel) {}
    bool StartNextSample() override;
    void StartPixel(const Point2i& p) override;
    bool SetSampleNumber(int64_t sampleNum) override;
    float Get1D() override;
    Point2f Get2D() override;
    // Sampler.h:69-70: the global index of the current pixel's sample `sampleNum`, and that index's
    // value in `dimension`
    virtual int64_t GetIndexForSample(int64_t sampleNum) const = 0;
    virtual float SampleDimension(int64_t index, int dimension) const = 0;
    // Extensions: batched forms (defaults: one call each; the device samplers answer a whole batch
    // with one query), the current interval sample index, the number of dimensions the sampler has
    int CurrentDimension() const override { return dimension; }
    int64_t CurrentIndex() const;
    virtual void SampleDimensions(int64_t index, int firstDim, int n, float* out) const;
    virtual void GetIndicesForSamples(int64_t firstSample, int n, int64_t* out) const;
    // dimensions [firstDim, firstDim + n) of `count` indices, index-major (default: SampleDimensions
    // per index; the device samplers answer it with one query)
    virtual void SampleDimensionsOf(const int64_t* index, int count, int firstDim, int n, float* out) const;
    virtual int MaxDimensions() const { return 1 << 30; }
    // the value of dimension `dim` for sample `sampleNum` of the current pixel, and a batch of them
    float SampleValue(int64_t sampleNum, int dim) const;
    void SampleValues(const std::vector<int64_t>& sampleNums, const std::vector<int>& dims, float* out) const;
    static constexpr int kValueBlock = 32;

  private:
    float value(int dim);
    int64_t indexOf(int64_t sampleNum) const;   // the pixel's indices, fetched once in StartPixel
    std::vector<int64_t> pixelIndex;
    int64_t intervalSample = 0;                 // the current sample number; its index on first use
    mutable int64_t intervalSampleIndex = 0;
    mutable bool intervalKnown = false;
    int dimension = 0;
    static const int arrayStartDim = 5;
    int arrayEndDim = 5;
    int cacheBase = -1;                 // first dimension held in cache (-1: nothing cached)
    float cache[kValueBlock];
};
class HaltonSampler : public GlobalSampler {   // Sampler/Halton.h
  public:
    HaltonSampler(int nsamp, const Bounds2i& sampleBounds, bool sampleAtCenter = false);
    std::unique_ptr<Sampler> Clone(int seed) override;   // Halton.cpp: a copy (the sequence has no seed)
    int64_t GetIndexForSample(int64_t sampleNum) const override;   // Halton.cpp:61-81, on the device
    float SampleDimension(int64_t index, int dimension) const override;   // Halton.cpp:83-92, on the device
    void SampleDimensions(int64_t index, int firstDim, int n, float* out) const override;
    void GetIndicesForSamples(int64_t firstSample, int n, int64_t* out) const override;
    void SampleDimensionsOf(const int64_t* index, int count, int firstDim, int n, float* out) const override;
    int DeviceSampler() const override;
    Point2i SampleRaster() const override;
    int MaxDimensions() const override { return 1000; }   // PrimeTableSize
    const Bounds2i sampleBounds;
};
HaltonSampler* CreateHaltonSampler(const Bounds2i& sampleBounds);   // 16 spp, as Halton.cpp:98-104
// pbrt-v3's SobolSampler (sobol.h/.cpp) over the reference's SobolMatrices32
// (Sampler/SobolMatrices.cpp:69; F3 — the reference ships the tables, not the sampler): spp rounded
// up to a power of two, resolution RoundUpPow2(max(width, height)) of the sample bounds.
class SobolSampler : public GlobalSampler {
  public:
    SobolSampler(int64_t samplesPerPixel, const Bounds2i& sampleBounds);
    std::unique_ptr<Sampler> Clone(int seed) override;
    int64_t GetIndexForSample(int64_t sampleNum) const override;   // SobolIntervalToIndex, on the device
    float SampleDimension(int64_t index, int dimension) const override;   // pbrt-v3 sobol.cpp, on the device
    void SampleDimensions(int64_t index, int firstDim, int n, float* out) const override;
    void GetIndicesForSamples(int64_t firstSample, int n, int64_t* out) const override;
    void SampleDimensionsOf(const int64_t* index, int count, int firstDim, int n, float* out) const override;
    int DeviceSampler() const override;
    Point2i SampleRaster() const override;
    int MaxDimensions() const override { return 1024; }   // NumSobolDimensions
    const Bounds2i sampleBounds;
};

// ---------------------------------------------------------------------------- Integrator/
struct RenderStats {   // what the last Render measured (pbr_render_stats)
    double seconds = 0, kernel_ms = 0;
    uint64_t samples = 0;
};
class Integrator {
  public:
    virtual ~Integrator() = default;
    virtual void Render(const Scene& scene, double& timeConsume) = 0;
    float IntegratorRenderTime = 0;
};
class SamplerIntegrator : public Integrator {
  public:
    SamplerIntegrator(std::shared_ptr<const Camera> camera, std::shared_ptr<Sampler> sampler, const Bounds2i& pixelBounds,
                      FrameBuffer* m_FrameBuffer);
    ~SamplerIntegrator() override;
    // SamplerIntegrator::Render (Integrator.cpp:280-356) on the GPU: uploads the scene (once per
    // Scene), renders every pixel × sample, fills m_FrameBuffer's 8-bit buffer exactly as the
    // reference (XYZ round trip, gamma, vertical flip) and its float buffer.
    void Render(const Scene& scene, double& timeConsume) override;
    // Uploads the scene to the integrator's device (BVHAccel build, lights, media); Render and Li
    // do it on first use.  The reference's SamplerIntegrator::Preprocess is a no-op hook.
    virtual void Preprocess(const Scene& scene, Sampler& sampler);
    // SamplerIntegrator::Li (Integrator.h:44) on the device for one ray, the sampler positioned at
    // its current pixel / sample / dimension (after GetCameraSample: dimension 5)
    virtual Spectrum Li(const RayDifferential& ray, const Scene& scene, Sampler& sampler, int depth = 0) const;
    // batched: ray i with the sampler at (pixels[i], samples[i], dimension)
    std::vector<Spectrum> Li(const std::vector<Ray>& rays, const std::vector<Point2i>& pixels,
                             const std::vector<int64_t>& samples, int dimension, const Scene& scene, int depth = 0) const;
    // Extensions: device ordinal; restrict to tiles (multi-GPU sharding); last stats.
    void SetDevice(int device) { this->device = device; }
    // Multi-GPU Render: the frame's 32×32 tiles are dealt round-robin over these
    // devices (one context each, frames rendered concurrently), and the per-rank RGBA8 and float
    // FrameBuffer spans are gathered to the first device with one RCCL ncclGather each (distinct
    // devices), then scattered into m_FrameBuffer.  A device listed twice gets two contexts and its
    // spans are copied instead (RCCL needs distinct devices).  Empty: the single-device Render.
    void SetDevices(const std::vector<int>& devices) { this->devices = devices; }
    void SetTiles(const std::vector<Bounds2i>& tiles) { this->tiles = tiles; }
    const RenderStats& LastStats() const { return stats; }

  protected:
    virtual int IntegratorType() const = 0;
    virtual int MaxDepth() const = 0;
    virtual float RRThreshold() const { return 1.f; }
    virtual int LightStrategy() const { return 0; }
    std::shared_ptr<const Camera> camera;

  private:
    void ensure_scene(const Scene& scene) const;   // context + upload (once per Scene)
    std::vector<Spectrum> LiWith(const Sampler& s, const std::vector<Ray>& rays, const std::vector<Point2i>& pixels,
                                 const std::vector<int64_t>& samples, int dimension, const Scene& scene, int depth) const;
    std::shared_ptr<Sampler> sampler;
    const Bounds2i pixelBounds;
    FrameBuffer* m_FrameBuffer;
    int device = 0;
    std::vector<Bounds2i> tiles;
    RenderStats stats;
    mutable pbr_hip_ctx* ctx = nullptr;
    mutable uint64_t uploadedScene = 0;
    mutable const Medium* uploadedCameraMedium = nullptr;
    std::vector<int> devices;
    struct MultiGPU;
    std::shared_ptr<MultiGPU> multi;
    void RenderMulti(const Scene& scene, double& timeConsume);
};
class WhittedIntegrator : public SamplerIntegrator {   // Integrator/WhittedIntegrator.h
  public:
    WhittedIntegrator(int maxDepth, std::shared_ptr<const Camera> camera, std::shared_ptr<Sampler> sampler,
                      const Bounds2i& pixelBounds, FrameBuffer* m_FrameBuffer)
        : SamplerIntegrator(camera, sampler, pixelBounds, m_FrameBuffer), maxDepth(maxDepth) {}

  protected:
    int IntegratorType() const override;
    int MaxDepth() const override { return maxDepth; }

  private:
    const int maxDepth;
};
class PathIntegrator : public SamplerIntegrator {   // Integrator/PathIntegrator.h
  public:
    PathIntegrator(int maxDepth, std::shared_ptr<const Camera> camera, std::shared_ptr<Sampler> sampler,
                   const Bounds2i& pixelBounds, float rrThreshold = 1, const std::string& lightSampleStrategy = "spatial",
                   FrameBuffer* framebuffer = nullptr)
        : SamplerIntegrator(camera, sampler, pixelBounds, framebuffer), maxDepth(maxDepth), rrThreshold(rrThreshold),
          lightSampleStrategy(lightSampleStrategy) {}

  protected:
    int IntegratorType() const override;
    int MaxDepth() const override { return maxDepth; }
    float RRThreshold() const override { return rrThreshold; }
    int LightStrategy() const override;

  private:
    const int maxDepth;
    const float rrThreshold;
    const std::string lightSampleStrategy;
};
class VolPathIntegrator : public PathIntegrator {   // Integrator/VolPathIntegrator.h
  public:
    using PathIntegrator::PathIntegrator;

  protected:
    int IntegratorType() const override;
};
using HipWhittedIntegrator = WhittedIntegrator;
using HipPathIntegrator = PathIntegrator;
using HipVolPathIntegrator = VolPathIntegrator;

// ---------------------------------------------------------------------------- multi-GPU tiles
// The partition the multi-GPU Render (and bench.py's ranks) use: TILE×TILE tiles in row-major order,
// tile i owned by rank i mod world (so the dragon's expensive tiles spread over the GPUs).
constexpr int kTile = 32;
std::vector<Bounds2i> TileGrid(int width, int height, int tile = kTile);
std::vector<Bounds2i> TilesForRank(int width, int height, int rank, int world, int tile = kTile);
// Scatter a rank's packed span (its tiles in order, each row-major, `channels` values per pixel)
// into a row-major width-wide frame.
void AssembleTiles(const std::vector<Bounds2i>& tiles, const uint8_t* packed, int channels, int width, uint8_t* frame);
void AssembleTiles(const std::vector<Bounds2i>& tiles, const float* packed, int channels, int width, float* frame);

// ---------------------------------------------------------------------------- flattening
// The scene as the C-ABI takes it (pbr_scene_desc + owned arrays); exposed for tests and for
// callers that drive the C-ABI themselves.
struct FlatScene;
std::shared_ptr<FlatScene> FlattenScene(const Scene& scene, const Medium* cameraMedium = nullptr);
const ::pbr_scene_desc* SceneDesc(const FlatScene& f);
int MediumIndex(const FlatScene& f, const Medium* m);

}  // namespace PBR
