// ref_harness.cpp — TEST INFRASTRUCTURE ONLY.  Linked with the reference's own translation units
// (compiled unmodified where they lie under /root/reference, oracle/ref/Makefile) into
// oracle/_ref/libpbr_ref.so: the real reference, driven through the same plain-data scene and render
// descriptors (include/pbr_hip.h) the product and the CPU restatement take, so fixtures and the CPU
// baseline can come from the reference itself.
//
// What it does with the reference's classes (no reference code is restated here):
//   * builds TriangleMesh/Triangle/GeometricPrimitive, the Matte/Mirror/Glass/Metal/Plastic
//     materials over ConstantTextures, Point/DiffuseArea/SkyBox/InfiniteArea lights,
//     HomogeneousMedium, BVHAccel(SAH), Scene, CreatePerspectiveCamera, HaltonSampler and the
//     Whitted/Path/VolPath integrators from the descriptors (the objects Main/main.cpp:186-413 builds);
//   * ref_render: SamplerIntegrator::Render's per-pixel body (Integrator/Integrator.cpp:286-344) —
//     Clone, StartPixel, GetCameraSample, GenerateRayDifferential, ScaleDifferentials, Li, colObj/spp
//     and the ToXYZ → XYZToRGB → GammaCorrect → u8 transform — over the descriptor's tiles, calling
//     the reference's own functions for each step, without the F1 axis swap (any raster);
//   * ref_render_frame: the reference's real Integrator::Render into its FrameBuffer (square rasters);
//   * ref_build_bvh / ref_intersect / ref_camera_rays: BVHAccel's node array and primitive order,
//     Scene::Intersect/IntersectP records, PerspectiveCamera rays.
//
// Memory: ~SurfaceInteraction destroys its shared_ptr-owned BSDF explicitly (Core/Interaction.cpp:
// 34-37), so every BSDF is destroyed twice; under glibc's allocator the second destroy
// touches freed memory and the process crashes.  While a render runs, this harness serves the
// render threads' operator new from a per-thread bump arena that operator delete never returns to
// the heap, so the double destroy reads memory that is still intact; the arena is rewound between
// pixels (ref_render) or is simply large (ref_render_frame).  Allocation does not change any value
// the reference computes.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include <omp.h>
#include <unistd.h>

#define private public       // BVHAccel's node array and primitive order (introspection only)
#include "Accelerator\BVHAccel.h"
#undef private
#include "Camera\Perspective.h"
#include "Core\FrameBuffer.h"
#include "Core\Interaction.h"
#include "Core\Primitive.h"
#include "Core\Scene.h"
#include "Core\Spectrum.h"
#include "Core\Transform.h"
#include "Integrator\PathIntegrator.h"
#include "Integrator\VolPathIntegrator.h"
#include "Integrator\WhittedIntegrator.h"
#include "Light\DiffuseLight.h"
#include "Sampler\Sampling.h"   // Distribution2D, before InfiniteAreaLight.h holds one
#include "Light\InfiniteAreaLight.h"
#include "Light\PointLight.h"
#include "Light\SkyBoxLight.h"
#include "Material\GlassMaterial.h"
#include "Material\MatteMaterial.h"
#include "Material\MetalMaterial.h"
#include "Material\Mirror.h"
#include "Material\PlasticMaterial.h"
#include "Texture\ImageTexture.h"
#include "Media\HomogeneousMedium.h"
#include "Sampler\Halton.h"
#include "Shape\Triangle.h"
#include "Shape\plyRead.h"
#include "Texture\ConstantTexture.h"

#include "../../include/pbr_hip.h"

// stb's HDR writer (the reference vendors stb; its implementation is compiled only in Main/main.cpp,
// which this build leaves out): environment maps reach SkyBoxLight / InfiniteAreaLight as files.
#define STB_IMAGE_WRITE_IMPLEMENTATION
#include "stb_image_write.h"   // $(REF)/include
extern "C" void stbi_set_flip_vertically_on_load(int flag_true_if_should_flip);

// ---------------------------------------------------------------- render-time arena (F6, above)
namespace {
thread_local char* tl_base = nullptr;
thread_local size_t tl_cap = 0, tl_off = 0;
thread_local bool tl_on = false;
std::atomic<bool> g_frameArena{false};   // ref_render_frame: every thread allocates from its arena

void arena_on(size_t cap) {
    if (!tl_base || tl_cap < cap) {
        std::free(tl_base);
        tl_base = (char*)std::malloc(cap);
        if (!tl_base) throw std::bad_alloc();
        tl_cap = cap;
    }
    tl_off = 0;
    tl_on = true;
}
void arena_rewind() { tl_off = 0; }
void arena_off() { tl_on = false; }
bool in_arena(void* p) { return tl_base && (char*)p >= tl_base && (char*)p < tl_base + tl_cap; }
}  // namespace

thread_local bool tl_frame = false;   // this thread's arena was opened by ref_render_frame

void* operator new(size_t n) {
    if (g_frameArena.load(std::memory_order_relaxed)) {
        if (!tl_on && omp_in_parallel()) { arena_on((size_t)1 << 31); tl_frame = true; }
    } else if (tl_frame) {
        tl_on = tl_frame = false;
    }
    if (tl_on) {
        size_t a = (tl_off + 15) & ~(size_t)15;
        if (a + n <= tl_cap) {
            tl_off = a + n;
            return tl_base + a;
        }
    }
    void* p = std::malloc(n ? n : 1);
    if (!p) throw std::bad_alloc();
    return p;
}
void* operator new[](size_t n) { return operator new(n); }
void operator delete(void* p) noexcept {
    if (!p || in_arena(p)) return;
    // Pointers of other threads' arenas are never freed either: they are not from malloc.  A heap
    // block freed twice by the F6 double destroy can only come from outside a render.
    if (g_frameArena.load(std::memory_order_relaxed)) return;
    std::free(p);
}
void operator delete[](void* p) noexcept { operator delete(p); }
void operator delete(void* p, size_t) noexcept { operator delete(p); }
void operator delete[](void* p, size_t) noexcept { operator delete(p); }

using namespace PBR;

namespace {

Transform xf(const pbr_transform& t) {
    float m[4][4], mi[4][4];
    for (int i = 0; i < 16; ++i) { m[i / 4][i % 4] = t.m[i]; mi[i / 4][i % 4] = t.m_inv[i]; }
    return Transform(Matrix4x4(m), Matrix4x4(mi));
}
Spectrum spec(const float* v) {
    Spectrum s;
    s[0] = v[0]; s[1] = v[1]; s[2] = v[2];
    return s;
}
std::shared_ptr<Texture<Spectrum>> cs(const float* v) { return std::make_shared<ConstantTexture<Spectrum>>(spec(v)); }
std::shared_ptr<Texture<float>> cf(float v) { return std::make_shared<ConstantTexture<float>>(v); }

// An .hdr file whose stbi_loadf (with the given flip state) returns exactly `data` (RGBE-exact
// values round-trip through stbi_write_hdr unchanged).
std::string write_env(const float* data, int w, int h, int comps, bool flippedOnLoad) {
    static std::atomic<int> seq{0};
    char path[256];
    std::snprintf(path, sizeof path, "/tmp/pbr_ref_env_%d_%d.hdr", (int)getpid(), seq++);
    std::vector<float> rows((size_t)w * h * comps);
    for (int y = 0; y < h; ++y) {
        const int src = flippedOnLoad ? h - 1 - y : y;
        std::memcpy(&rows[(size_t)y * w * comps], &data[(size_t)src * w * comps], (size_t)w * comps * sizeof(float));
    }
    stbi_flip_vertically_on_write(0);
    if (!stbi_write_hdr(path, w, h, comps, rows.data())) throw std::runtime_error("stbi_write_hdr failed");
    return path;
}

// The reference scene built from a descriptor; owns everything the reference's raw pointers need.
struct RefScene {
    std::vector<std::unique_ptr<Transform>> xforms;
    std::vector<std::unique_ptr<HomogeneousMedium>> media;
    std::vector<std::shared_ptr<Material>> materials;
    std::vector<std::shared_ptr<Primitive>> prims;
    std::unordered_map<const Primitive*, int> primIndex;
    std::vector<std::shared_ptr<Light>> lights;
    std::shared_ptr<BVHAccel> bvh;
    std::unique_ptr<Scene> scene;
    std::vector<std::string> tmpFiles;
    ~RefScene() {
        for (auto& f : tmpFiles) std::remove(f.c_str());
    }
    const Transform* keep(const Transform& t) {
        xforms.emplace_back(new Transform(t));
        return xforms.back().get();
    }
    const Medium* medium(int i) const { return i >= 0 && i < (int)media.size() ? media[i].get() : nullptr; }
};

std::unique_ptr<RefScene> build(const pbr_scene_desc* d) {
    if (!d || d->abi_version != PBR_HIP_ABI_VERSION) throw std::runtime_error("bad scene desc");
    std::unique_ptr<RefScene> r(new RefScene);
    for (int i = 0; i < d->n_media; ++i)
        r->media.emplace_back(new HomogeneousMedium(spec(d->media[i].sigma_a), spec(d->media[i].sigma_s), d->media[i].g));
    // ImageTextures as main.cpp / ModelLoad.cpp make them (main.cpp:63-78, ModelLoad.cpp:95-160): the
    // image goes through a file that the texture's own loadImage (stbi_loadf, flip-on-load set,
    // ImageTexture.cpp:13-37) reads back as exactly the descriptor's floats
    auto image = [&](const pbr_texture_desc& td) {
        if (td.level0) throw std::runtime_error("a level-0 texture: build the reference ImageTexture itself");
        std::string path;
        if (td.data && td.width > 0 && td.height > 0) {
            path = write_env(td.data, td.width, td.height, td.components, true);
            r->tmpFiles.push_back(path);
        }
        return path;
    };
    auto texS = [&](const pbr_material_desc& m, int slot, const float* v) -> std::shared_ptr<Texture<Spectrum>> {
        if (!m.tex[slot]) return cs(v);
        const pbr_texture_desc& td = d->textures[m.tex[slot] - 1];
        return std::make_shared<ImageTexture<RGBSpectrum, Spectrum>>(std::make_unique<UVMapping2D>(td.su, td.sv, td.du, td.dv),
                                                                     image(td), td.trilinear != 0, td.max_aniso,
                                                                     (ImageWrap)td.wrap, td.scale, td.gamma != 0);
    };
    auto texF = [&](const pbr_material_desc& m, int slot, float v) -> std::shared_ptr<Texture<float>> {
        if (!m.tex[slot]) return cf(v);
        const pbr_texture_desc& td = d->textures[m.tex[slot] - 1];
        return std::make_shared<ImageTexture<float, float>>(std::make_unique<UVMapping2D>(td.su, td.sv, td.du, td.dv), image(td),
                                                            td.trilinear != 0, td.max_aniso, (ImageWrap)td.wrap, td.scale,
                                                            td.gamma != 0);
    };
    for (int i = 0; i < d->n_materials; ++i) {   // Main/main.cpp:147-239
        const pbr_material_desc& m = d->materials[i];
        std::shared_ptr<Material> mat;
        auto bump = cf(0.f);
        switch (m.type) {
        case PBR_MAT_NONE: break;
        case PBR_MAT_MATTE: mat = std::make_shared<MatteMaterial>(texS(m, PBR_TEX_KD, m.Kd), texF(m, PBR_TEX_SIGMA, m.sigma), bump); break;
        case PBR_MAT_MIRROR: mat = std::make_shared<MirrorMaterial>(texS(m, PBR_TEX_KR, m.Kr), bump); break;
        case PBR_MAT_GLASS:
            mat = std::make_shared<GlassMaterial>(texS(m, PBR_TEX_KR, m.Kr), texS(m, PBR_TEX_KT, m.Kt), cf(m.uroughness),
                                                  cf(m.vroughness), cf(m.eta), bump, m.remap_roughness != 0);
            break;
        case PBR_MAT_METAL:
            mat = std::make_shared<MetalMaterial>(cs(m.metal_eta), cs(m.metal_k), cf(m.roughness),
                                                  m.has_uv_roughness ? cf(m.uroughness) : nullptr,
                                                  m.has_uv_roughness ? cf(m.vroughness) : nullptr, bump, m.remap_roughness != 0);
            break;
        case PBR_MAT_PLASTIC:
            mat = std::make_shared<PlasticMaterial>(texS(m, PBR_TEX_KD, m.Kd), texS(m, PBR_TEX_KS, m.Ks),
                                                    texF(m, PBR_TEX_ROUGHNESS, m.roughness), bump, m.remap_roughness != 0);
            break;
        default: throw std::runtime_error("unknown material");
        }
        r->materials.push_back(mat);
    }
    // shapes, in descriptor order: the `prims` vector order BVHAccel receives (main.cpp:279-282)
    std::vector<std::vector<std::shared_ptr<Shape>>> shapeTris(d->n_shapes);
    std::vector<int> firstPrim(d->n_shapes, 0);
    for (int i = 0; i < d->n_shapes; ++i) {
        const pbr_shape_desc& s = d->shapes[i];
        if (s.type != PBR_SHAPE_TRIANGLE_MESH) throw std::runtime_error("the reference's Sphere is a stub (F2)");
        const Transform* o2w = r->keep(xf(s.object_to_world));
        const Transform* w2o = r->keep(Inverse(*o2w));
        std::vector<Point3f> P(s.n_vertices);
        for (int v = 0; v < s.n_vertices; ++v) P[v] = Point3f(s.P[3 * v], s.P[3 * v + 1], s.P[3 * v + 2]);
        std::vector<Point2f> UV;
        if (s.UV) {
            UV.resize(s.n_vertices);
            for (int v = 0; v < s.n_vertices; ++v) UV[v] = Point2f(s.UV[2 * v], s.UV[2 * v + 1]);
        }
        if (s.N) throw std::runtime_error("per-vertex normals are not supported");
        auto mesh = std::make_shared<TriangleMesh>(*o2w, s.n_triangles, s.indices, s.n_vertices, P.data(), nullptr, nullptr,
                                                   s.UV ? UV.data() : nullptr, nullptr);
        firstPrim[i] = (int)r->prims.size();
        for (int t = 0; t < s.n_triangles; ++t) {
            shapeTris[i].push_back(std::make_shared<Triangle>(o2w, w2o, s.reverse_orientation != 0, mesh, t));
            r->prims.push_back(nullptr);   // filled below, once area lights exist
        }
    }
    // lights (Light/*.h constructors as main.cpp calls them).  stb's vertical-flip-on-load flag is
    // process-global and SkyBoxLight::loadImage sets it and never clears it (SkyBoxLight.cpp:20):
    // each scene starts from stb's default (off), as a fresh reference process would.
    std::vector<std::shared_ptr<AreaLight>> areaOf(r->prims.size());
    stbi_set_flip_vertically_on_load(0);
    bool skyLoaded = false;
    for (int i = 0; i < d->n_lights; ++i) {
        const pbr_light_desc& l = d->lights[i];
        MediumInterface mi(r->medium(l.medium_inside), r->medium(l.medium_outside));
        const Transform l2w = xf(l.light_to_world);
        if (l.type == PBR_LIGHT_POINT) {
            r->lights.push_back(std::make_shared<PointLight>(l2w, mi, spec(l.I)));
        } else if (l.type == PBR_LIGHT_DIFFUSE_AREA) {
            auto area = std::make_shared<DiffuseAreaLight>(l2w, mi, spec(l.Le), l.n_samples, shapeTris[l.shape][l.triangle],
                                                           l.two_sided != 0);
            areaOf[firstPrim[l.shape] + l.triangle] = area;
            r->lights.push_back(area);
        } else if (l.type == PBR_LIGHT_SKYBOX) {
            if (!l.env_data) throw std::runtime_error("SkyBoxLight needs an image");
            std::string f = write_env(l.env_data, l.env_width, l.env_height, l.env_components, true);
            r->tmpFiles.push_back(f);
            r->lights.push_back(std::make_shared<SkyBoxLight>(
                l2w, Point3f(l.world_center[0], l.world_center[1], l.world_center[2]), l.world_radius, f.c_str(), l.n_samples));
            skyLoaded = true;   // SkyBoxLight::loadImage leaves stb's load flip on (SkyBoxLight.cpp:20)
        } else if (l.type == PBR_LIGHT_INFINITE_AREA) {
            std::string f;
            if (l.env_data && l.env_width > 0 && l.env_height > 0) {
                f = write_env(l.env_data, l.env_width, l.env_height, l.env_components, skyLoaded);
                r->tmpFiles.push_back(f);
            }
            r->lights.push_back(std::make_shared<InfiniteAreaLight>(l2w, spec(l.Le), l.n_samples, f));
        } else {
            throw std::runtime_error("unknown light");
        }
    }
    for (int i = 0; i < d->n_shapes; ++i) {
        const pbr_shape_desc& s = d->shapes[i];
        MediumInterface mi(r->medium(s.medium_inside), r->medium(s.medium_outside));
        std::shared_ptr<Material> mat = (s.material >= 0 && s.material < (int)r->materials.size()) ? r->materials[s.material] : nullptr;
        for (int t = 0; t < s.n_triangles; ++t) {
            const int k = firstPrim[i] + t;
            r->prims[k] = std::make_shared<GeometricPrimitive>(shapeTris[i][t], mat, areaOf[k], mi);
            r->primIndex[r->prims[k].get()] = k;
        }
    }
    r->bvh = std::make_shared<BVHAccel>(r->prims, d->max_prims_in_node > 0 ? d->max_prims_in_node : 1,
                                        (BVHAccel::SplitMethod)d->split_method);
    r->scene.reset(new Scene(r->bvh, r->lights));
    return r;
}

struct RefCamera {
    std::unique_ptr<Camera> cam;
};
// CreatePerspectiveCamera (Perspective.cpp:84-104) for pinhole cameras; a camera with an aperture
// (lens_radius > 0) is the reference's PerspectiveCamera constructor (Perspective.cpp:7-9) called
// with the screen window CreatePerspectiveCamera would pass, the descriptor's lens radius and focal
// distance, and fov 90.
std::shared_ptr<Camera> make_camera(const pbr_camera_desc& c) {
    if (c.fov != 90.f || c.lens_radius < 0.f) throw std::runtime_error("the reference camera is fov 90");
    if (c.use_raster_to_camera) throw std::runtime_error("a given RasterToCamera: build the reference camera itself");
    Transform c2w;
    if (c.use_look_at)
        c2w = Inverse(LookAt(Point3f(c.eye[0], c.eye[1], c.eye[2]), Point3f(c.look[0], c.look[1], c.look[2]),
                             Vector3f(c.up[0], c.up[1], c.up[2])));
    else
        c2w = xf(c.camera_to_world);
    if (c.lens_radius == 0.f) return std::shared_ptr<Camera>(CreatePerspectiveCamera(c.width, c.height, c2w, nullptr));
    const float frame = (float)c.width / (float)c.height;
    Bounds2f screen;
    if (frame > 1.f) { screen.pMin.x = -frame; screen.pMax.x = frame; screen.pMin.y = -1.f; screen.pMax.y = 1.f; }
    else { screen.pMin.x = -1.f; screen.pMax.x = 1.f; screen.pMin.y = -1.f / frame; screen.pMax.y = 1.f / frame; }
    return std::make_shared<PerspectiveCamera>(c.width, c.height, c2w, screen, c.lens_radius, c.focal_distance, 90.0f, nullptr);
}

std::shared_ptr<SamplerIntegrator> make_integrator(const pbr_render_desc* rd, std::shared_ptr<Camera> cam,
                                                   std::shared_ptr<Sampler> sampler, FrameBuffer* fb) {
    if (rd->sampler != PBR_SAMPLER_HALTON) throw std::runtime_error("the reference has no Sobol sampler (F3)");
    const Bounds2i bounds(Point2i(0, 0), Point2i(rd->camera.width, rd->camera.height));
    const std::string strategy = rd->light_strategy == PBR_LIGHTS_POWER ? "power" : "uniform";
    switch (rd->integrator) {
    case PBR_INTEGRATOR_WHITTED: return std::make_shared<WhittedIntegrator>(rd->max_depth, cam, sampler, bounds, fb);
    case PBR_INTEGRATOR_PATH:
        return std::make_shared<PathIntegrator>(rd->max_depth, cam, sampler, bounds, rd->rr_threshold, strategy, fb);
    case PBR_INTEGRATOR_VOLPATH:
        return std::make_shared<VolPathIntegrator>(rd->max_depth, cam, sampler, bounds, rd->rr_threshold, strategy, fb);
    default: throw std::runtime_error("unknown integrator");
    }
}

int fail(const std::exception& e) {
    std::fprintf(stderr, "ref harness: %s\n", e.what());
    return PBR_E_INVALID;
}

}  // namespace

extern "C" {

// Per-pixel float average (colObj / spp) and RGBA8 of SamplerIntegrator::Render's body, over the
// descriptor's tiles (packed tile after tile, row-major), with `threads` OpenMP threads (0 = all).
int ref_render(const pbr_scene_desc* sd, const pbr_render_desc* rd, float* rgb, uint8_t* rgba, int threads,
               double* seconds) {
    try {
        std::unique_ptr<RefScene> rs = build(sd);
        auto cam = make_camera(rd->camera);
        const Bounds2i bounds(Point2i(0, 0), Point2i(rd->camera.width, rd->camera.height));
        auto sampler = std::make_shared<HaltonSampler>(rd->spp, bounds);
        auto integ = make_integrator(rd, cam, sampler, nullptr);
        std::vector<pbr_tile> tiles;
        if (rd->n_tiles > 0) tiles.assign(rd->tiles, rd->tiles + rd->n_tiles);
        else tiles.push_back(pbr_tile{0, 0, rd->camera.width, rd->camera.height});
        std::vector<std::pair<int, int>> px;
        for (const pbr_tile& t : tiles)
            for (int y = t.y0; y < t.y1; ++y)
                for (int x = t.x0; x < t.x1; ++x) px.emplace_back(x, y);
        const double t0 = omp_get_wtime();
        integ->Preprocess(*rs->scene, *sampler);
        const int W = rd->camera.width;
#pragma omp parallel num_threads(threads > 0 ? threads : omp_get_max_threads())
        {
            arena_on((size_t)256 << 20);
#pragma omp for schedule(dynamic, 16)
            for (long long k = 0; k < (long long)px.size(); ++k) {
                arena_rewind();
                const int i = px[k].first, j = px[k].second;
                // Integrator.cpp:290-313 (pixel (i, j) = (x, y); the seed is the reference's offset)
                std::unique_ptr<Sampler> pixelSampler = sampler->Clone(W * j + i);
                Point2i pixel(i, j);
                pixelSampler->StartPixel(pixel);
                Spectrum colObj(0.0f);
                do {
                    CameraSample cameraSample = pixelSampler->GetCameraSample(pixel);
                    RayDifferential r;
                    cam->GenerateRayDifferential(cameraSample, &r);
                    r.ScaleDifferentials(1 / std::sqrt((float)pixelSampler->samplesPerPixel));
                    colObj += integ->Li(r, *rs->scene, *pixelSampler, 0);
                } while (pixelSampler->StartNextSample());
                colObj /= (float)pixelSampler->samplesPerPixel;
                if (rgb) for (int c = 0; c < 3; ++c) rgb[3 * k + c] = colObj[c];
                // Integrator.cpp:327-344
                float xyz[3], out[3];
                colObj.ToXYZ(xyz);
                XYZToRGB(xyz, out);
                if (rgba) {
                    for (int c = 0; c < 3; ++c)
                        rgba[4 * k + c] = (unsigned char)PBR::Clamp(255.f * GammaCorrect(out[c]) + 0.5f, 0.f, 255.f);
                    rgba[4 * k + 3] = 255;
                }
                pixelSampler.release();   // arena memory: never handed back to the heap
            }
            arena_off();
        }
        if (seconds) *seconds = omp_get_wtime() - t0;
        return PBR_OK;
    } catch (const std::exception& e) {
        return fail(e);
    }
}

// The reference's own Integrator::Render (Integrator.cpp:280-356, 4 OpenMP threads) on a SQUARE
// raster into its FrameBuffer; out = getUCbuffer() (W*H*4, row 0 = the image's bottom row, F1 note:
// only square rasters are fully written).
int ref_render_frame(const pbr_scene_desc* sd, const pbr_render_desc* rd, uint8_t* out, double* seconds) {
    try {
        if (rd->camera.width != rd->camera.height) throw std::runtime_error("Render writes only square rasters (F1)");
        if (rd->n_tiles > 0) throw std::runtime_error("Render renders whole frames");
        std::unique_ptr<RefScene> rs = build(sd);
        auto cam = make_camera(rd->camera);
        const Bounds2i bounds(Point2i(0, 0), Point2i(rd->camera.width, rd->camera.height));
        auto sampler = std::make_shared<HaltonSampler>(rd->spp, bounds);
        FrameBuffer fb;
        fb.InitBuffer(rd->camera.width, rd->camera.height, 4);
        auto integ = make_integrator(rd, cam, sampler, &fb);
        double t = 0;
        g_frameArena = true;
        integ->Render(*rs->scene, t);
        g_frameArena = false;
        if (tl_frame) { arena_off(); tl_frame = false; }
        std::memcpy(out, fb.getUCbuffer(), (size_t)rd->camera.width * rd->camera.height * 4);
        if (seconds) *seconds = t;
        return PBR_OK;
    } catch (const std::exception& e) {
        g_frameArena = false;
        return fail(e);
    }
}

// The frame arena of ref_render_frame for callers that run the reference's own Integrator::Render
// themselves (oracle/ref/refbind_scenes.cpp): on before Render, off after it.
void ref_frame_arena(int on) {
    g_frameArena = on != 0;
    if (!on && tl_frame) { arena_off(); tl_frame = false; }
}

// BVHAccel's flattened nodes (32-B LinearBVHNode, BVHAccel.cpp:46-55) and the original index of
// each primitive in BVH order; NULL buffers query the counts.
int ref_build_bvh(const pbr_scene_desc* sd, void* nodes_out, int* n_nodes, int32_t* prim_ids_out, int* n_prims) {
    try {
        std::unique_ptr<RefScene> rs = build(sd);
        BVHAccel& b = *rs->bvh;
        // the node count: walk the flattened tree (first child follows its parent, the second
        // child's offset is stored in the node; a leaf has nPrimitives > 0)
        struct Node { float b[6]; int offset; uint16_t nPrims; uint8_t axis, pad; };
        static_assert(sizeof(Node) == 32, "LinearBVHNode layout");
        const Node* nd = reinterpret_cast<const Node*>(b.nodes);
        int total = 0;
        if (nd && !b.primitives.empty()) {
            std::vector<int> stack{0};
            while (!stack.empty()) {
                const int i = stack.back();
                stack.pop_back();
                ++total;
                if (nd[i].nPrims == 0) { stack.push_back(nd[i].offset); stack.push_back(i + 1); }
            }
        }
        if (n_nodes) *n_nodes = total;
        if (n_prims) *n_prims = (int)b.primitives.size();
        if (nodes_out) std::memcpy(nodes_out, (const void*)b.nodes, (size_t)total * 32);
        if (prim_ids_out)
            for (size_t i = 0; i < b.primitives.size(); ++i) prim_ids_out[i] = rs->primIndex.at(b.primitives[i].get());
        return PBR_OK;
    } catch (const std::exception& e) {
        return fail(e);
    }
}

// Scene::Intersect (any_hit = 0) / IntersectP (1) for rays {o.xyz, d.xyz, tMax}:
// out = {hit, tMax after the query (the hit's t), original primitive index, p.x, p.y, p.z}.
int ref_intersect(const pbr_scene_desc* sd, int n, const float* rays, float* out, int any_hit) {
    try {
        std::unique_ptr<RefScene> rs = build(sd);
        for (int i = 0; i < n; ++i) {
            const float* q = rays + 7 * i;
            Ray r(Point3f(q[0], q[1], q[2]), Vector3f(q[3], q[4], q[5]), q[6]);
            float* o = out + 6 * i;
            if (any_hit) {
                o[0] = rs->scene->IntersectP(r) ? 1.f : 0.f;
                o[1] = r.tMax; o[2] = -1; o[3] = o[4] = o[5] = 0;
                continue;
            }
            SurfaceInteraction si;
            const bool hit = rs->scene->Intersect(r, &si);
            o[0] = hit ? 1.f : 0.f;
            o[1] = r.tMax;
            o[2] = hit ? (float)rs->primIndex.at(si.primitive) : -1.f;
            o[3] = hit ? si.p.x : 0.f; o[4] = hit ? si.p.y : 0.f; o[5] = hit ? si.p.z : 0.f;
        }
        return PBR_OK;
    } catch (const std::exception& e) {
        return fail(e);
    }
}

// PerspectiveCamera::GenerateRayDifferential for raster samples (pFilm; pLens (0.5, 0.5) or, with
// plens, the given lens samples; time 0): out = o.xyz, d.xyz.
int ref_camera_rays_lens(const pbr_camera_desc* cd, int n, const float* pfilm, const float* plens, float* out) {
    try {
        auto cam = make_camera(*cd);
        for (int i = 0; i < n; ++i) {
            CameraSample cs;
            cs.pFilm = Point2f(pfilm[2 * i], pfilm[2 * i + 1]);
            cs.pLens = plens ? Point2f(plens[2 * i], plens[2 * i + 1]) : Point2f(0.5f, 0.5f);
            cs.time = 0.f;
            RayDifferential r;
            cam->GenerateRayDifferential(cs, &r);
            out[6 * i] = r.o.x; out[6 * i + 1] = r.o.y; out[6 * i + 2] = r.o.z;
            out[6 * i + 3] = r.d.x; out[6 * i + 4] = r.d.y; out[6 * i + 5] = r.d.z;
        }
        return PBR_OK;
    } catch (const std::exception& e) {
        return fail(e);
    }
}

int ref_camera_rays(const pbr_camera_desc* cd, int n, const float* pfilm, float* out) {
    return ref_camera_rays_lens(cd, n, pfilm, nullptr, out);
}

// Shape/plyRead.h:22-47: the reference's ".3d" reader (vertices ×20); pass NULL arrays for counts.
int ref_ply_info(const char* path, int* n_vertices, int* n_triangles, float* verts, int32_t* indices) {
    try {
        PBR::plyInfo info(path);
        *n_vertices = info.nVertices;
        *n_triangles = info.nTriangles;
        if (verts)
            for (int i = 0; i < info.nVertices; ++i)
                for (int k = 0; k < 3; ++k) verts[3 * i + k] = info.vertexArray[i][k];
        if (indices)
            for (int i = 0; i < 3 * info.nTriangles; ++i) indices[i] = info.vertexIndices[i];
        delete[] info.vertexArray;
        delete[] info.vertexIndices;
        return 0;
    } catch (...) {
        return -1;
    }
}

}  // extern "C"
