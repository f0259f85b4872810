// host_api_test.cpp — the C++ host API (include/pbr/pbr.h) used exactly as the reference's
// Main/main.cpp uses its classes, checked against the oracle (test infrastructure) on the same
// flattened scene.
//
//   host_api_test cpu   no GPU needed: scene building, flattening, oracle sanity, Render fails loudly
//   host_api_test gpu   renders through WhittedIntegrator / PathIntegrator / VolPathIntegrator on
//                       the GPU and compares the FrameBuffer with the oracle (L∞ ≤ 1e-3; u8 identical where the float pixel is, else ≤ 1)
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <unistd.h>
#include <memory>
#include <string>
#include <vector>

#include "../../include/pbr/pbr.h"
#include "../../include/pbr_hip.h"
#include <hip/hip_runtime_api.h>
#include "../../oracle/pbr_oracle.h"

using namespace PBR;

namespace {

int failures = 0;
void expect(bool ok, const std::string& what) {
    std::printf("%s %s\n", ok ? "ok  " : "FAIL", what.c_str());
    if (!ok) ++failures;
}

std::shared_ptr<Texture<Spectrum>> rgbTex(float r, float g, float b) {
    float v[3] = {r, g, b};
    return std::make_shared<ConstantTexture<Spectrum>>(Spectrum::FromRGB(v));
}
std::shared_ptr<Texture<float>> fTex(float v) { return std::make_shared<ConstantTexture<float>>(v); }

struct Built {
    std::vector<std::unique_ptr<Transform>> xf;   // shapes keep raw Transform pointers
    std::vector<std::unique_ptr<Medium>> media;
    std::unique_ptr<Scene> scene;
    std::shared_ptr<Camera> cam;
    const Medium* camMedium = nullptr;
};

const Transform* keep(Built& b, const Transform& t) {
    b.xf.push_back(std::make_unique<Transform>(t));
    return b.xf.back().get();
}

// C1 of SURVEY §8(d): two matte spheres, point light I=20 at (0,4,4), camera (0,0,5) → origin.
void build_c1(Built& b, int W, int H) {
    std::vector<std::shared_ptr<Primitive>> prims;
    auto matte = std::make_shared<MatteMaterial>(rgbTex(0.5f, 0.5f, 0.5f), fTex(0.f), nullptr);
    const Vector3f centres[2] = {Vector3f(-1.f, 0.f, 0.f), Vector3f(1.2f, 0.f, -1.f)};
    for (const Vector3f& c : centres) {
        const Transform* o2w = keep(b, Translate(c));
        const Transform* w2o = keep(b, Inverse(*o2w));
        auto s = std::make_shared<Sphere>(o2w, w2o, false, 1.f);
        prims.push_back(std::make_shared<GeometricPrimitive>(s, matte, nullptr, MediumInterface()));
    }
    std::vector<std::shared_ptr<Light>> lights;
    lights.push_back(std::make_shared<PointLight>(Translate(Vector3f(0.f, 4.f, 4.f)), MediumInterface(), Spectrum(20.f)));
    b.scene = std::make_unique<Scene>(std::make_shared<BVHAccel>(prims, 1), lights);
    Transform lookat = LookAt(Point3f(0.f, 0.f, 5.f), Point3f(0.f, 0.f, 0.f), Vector3f(0.f, 1.f, 0.f));
    b.cam = std::shared_ptr<Camera>(CreatePerspectiveCamera(W, H, Inverse(lookat), nullptr));
}

// A C3/C5-shaped scene: a small tetrahedral mesh (glass, optionally filled with a homogeneous
// medium) over a matte floor, lit by a one-sided two-triangle area light at y = 2.45.
void build_area(Built& b, int W, int H, bool medium) {
    std::vector<std::shared_ptr<Primitive>> prims;
    const Medium* inside = nullptr;
    if (medium) {
        b.media.push_back(std::make_unique<HomogeneousMedium>(Spectrum(0.5f), Spectrum(4.4f), -0.5f));
        inside = b.media.back().get();
    }
    auto glass = std::make_shared<GlassMaterial>(rgbTex(1, 1, 1), rgbTex(1, 1, 1), fTex(0.1f), fTex(0.1f), fTex(1.5f), nullptr, false);
    auto floorMat = std::make_shared<MatteMaterial>(rgbTex(0.6f, 0.6f, 0.6f), fTex(0.f), nullptr);
    const Transform* id = keep(b, Transform());
    const Point3f tp[4] = {Point3f(-0.8f, -0.9f, -0.5f), Point3f(0.8f, -0.9f, -0.5f), Point3f(0.f, -0.9f, 0.8f), Point3f(0.f, 0.6f, 0.f)};
    const int ti[12] = {0, 2, 1, 0, 1, 3, 1, 2, 3, 2, 0, 3};
    for (auto& s : CreateTriangleMesh(id, id, false, 4, ti, 4, tp, nullptr, nullptr, nullptr))
        prims.push_back(std::make_shared<GeometricPrimitive>(s, glass, nullptr, MediumInterface(inside, nullptr)));
    const Point3f fp[4] = {Point3f(-5, -1, -5), Point3f(5, -1, -5), Point3f(5, -1, 5), Point3f(-5, -1, 5)};
    const int fi[6] = {0, 2, 1, 0, 3, 2};
    for (auto& s : CreateTriangleMesh(id, id, false, 2, fi, 4, fp, nullptr, nullptr, nullptr))
        prims.push_back(std::make_shared<GeometricPrimitive>(s, floorMat, nullptr, MediumInterface()));
    // area light: quad facing down (reverseOrientation flips the normal to -y)
    const Transform* lx = keep(b, Translate(Vector3f(0.f, 2.45f, 0.f)));
    const Transform* lxi = keep(b, Inverse(*lx));
    const Point3f lp[4] = {Point3f(-0.6f, 0, -0.6f), Point3f(0.6f, 0, -0.6f), Point3f(0.6f, 0, 0.6f), Point3f(-0.6f, 0, 0.6f)};
    const int li[6] = {0, 1, 2, 0, 2, 3};
    std::vector<std::shared_ptr<Light>> lights;
    auto lightMat = std::make_shared<MatteMaterial>(rgbTex(0, 0, 0), fTex(0.f), nullptr);
    for (auto& s : CreateTriangleMesh(lx, lxi, true, 2, li, 4, lp, nullptr, nullptr, nullptr)) {
        auto area = std::make_shared<DiffuseAreaLight>(*lx, MediumInterface(), Spectrum(5.f), 5, s, false);
        lights.push_back(area);
        prims.push_back(std::make_shared<GeometricPrimitive>(s, lightMat, area, MediumInterface()));
    }
    b.scene = std::make_unique<Scene>(std::make_shared<BVHAccel>(prims, 1), lights);
    Transform lookat = LookAt(Point3f(0.f, 0.3f, 3.2f), Point3f(0.f, -0.3f, 0.f), Vector3f(0.f, 1.f, 0.f));
    b.cam = std::shared_ptr<Camera>(CreatePerspectiveCamera(W, H, Inverse(lookat), nullptr));
}

// Nested closed boxes with no material (pbrt's medium-interface idiom): the outer one bounds a thin
// medium, the inner one a denser one, around a matte tetrahedron; matte floor, area light above.
void build_boxes(Built& b, int W, int H) {
    std::vector<std::shared_ptr<Primitive>> prims;
    b.media.push_back(std::make_unique<HomogeneousMedium>(Spectrum(0.05f), Spectrum(0.3f), 0.2f));
    b.media.push_back(std::make_unique<HomogeneousMedium>(Spectrum(0.1f), Spectrum(0.9f), -0.3f));
    const Medium* m1 = b.media[0].get();
    const Medium* m2 = b.media[1].get();
    const Transform* id = keep(b, Transform());
    auto box = [&](float h, const Medium* in, const Medium* out) {
        const Point3f p[8] = {Point3f(-h, -h, -h), Point3f(h, -h, -h), Point3f(h, h, -h), Point3f(-h, h, -h),
                              Point3f(-h, -h, h),  Point3f(h, -h, h),  Point3f(h, h, h),  Point3f(-h, h, h)};
        const int idx[36] = {0, 2, 1, 0, 3, 2, 4, 5, 6, 4, 6, 7, 0, 1, 5, 0, 5, 4, 3, 6, 2, 3, 7, 6, 0, 4, 7, 0, 7, 3, 1, 2, 6, 1, 6, 5};
        for (auto& s : CreateTriangleMesh(id, id, false, 12, idx, 8, p, nullptr, nullptr, nullptr))
            prims.push_back(std::make_shared<GeometricPrimitive>(s, nullptr, nullptr, MediumInterface(in, out)));
    };
    box(0.95f, m1, nullptr);
    box(0.6f, m2, m1);
    auto matte = std::make_shared<MatteMaterial>(rgbTex(0.7f, 0.5f, 0.3f), fTex(0.f), nullptr);
    const Point3f tp[4] = {Point3f(-0.3f, -0.3f, -0.2f), Point3f(0.3f, -0.3f, -0.2f), Point3f(0.f, -0.3f, 0.3f), Point3f(0.f, 0.3f, 0.f)};
    const int ti[12] = {0, 2, 1, 0, 1, 3, 1, 2, 3, 2, 0, 3};
    for (auto& s : CreateTriangleMesh(id, id, false, 4, ti, 4, tp, nullptr, nullptr, nullptr))
        prims.push_back(std::make_shared<GeometricPrimitive>(s, matte, nullptr, MediumInterface(m2, m2)));
    auto floorMat = std::make_shared<MatteMaterial>(rgbTex(0.6f, 0.6f, 0.6f), fTex(0.f), nullptr);
    const Point3f fp[4] = {Point3f(-5, -1, -5), Point3f(5, -1, -5), Point3f(5, -1, 5), Point3f(-5, -1, 5)};
    const int fi[6] = {0, 2, 1, 0, 3, 2};
    for (auto& s : CreateTriangleMesh(id, id, false, 2, fi, 4, fp, nullptr, nullptr, nullptr))
        prims.push_back(std::make_shared<GeometricPrimitive>(s, floorMat, nullptr, MediumInterface()));
    const Transform* lx = keep(b, Translate(Vector3f(0.f, 2.45f, 0.f)));
    const Transform* lxi = keep(b, Inverse(*lx));
    const Point3f lp[4] = {Point3f(-0.6f, 0, -0.6f), Point3f(0.6f, 0, -0.6f), Point3f(0.6f, 0, 0.6f), Point3f(-0.6f, 0, 0.6f)};
    const int li[6] = {0, 1, 2, 0, 2, 3};
    std::vector<std::shared_ptr<Light>> lights;
    auto lightMat = std::make_shared<MatteMaterial>(rgbTex(0, 0, 0), fTex(0.f), nullptr);
    for (auto& s : CreateTriangleMesh(lx, lxi, true, 2, li, 4, lp, nullptr, nullptr, nullptr)) {
        auto area = std::make_shared<DiffuseAreaLight>(*lx, MediumInterface(), Spectrum(5.f), 5, s, false);
        lights.push_back(area);
        prims.push_back(std::make_shared<GeometricPrimitive>(s, lightMat, area, MediumInterface()));
    }
    b.scene = std::make_unique<Scene>(std::make_shared<BVHAccel>(prims, 1), lights);
    Transform lookat = LookAt(Point3f(0.f, 0.3f, 3.2f), Point3f(0.f, -0.3f, 0.f), Vector3f(0.f, 1.f, 0.f));
    b.cam = std::shared_ptr<Camera>(CreatePerspectiveCamera(W, H, Inverse(lookat), nullptr));
}

// The reference's main.cpp light (main.cpp:377-381): InfiniteAreaLight(RotateX(-90) * RotateY(-0) *
// RotateZ(-50), power 1, nSamples 10, texmap) — here an in-memory 60x30 sky (not a power of two,
// so the MIPMap resamples it) added to a built scene.
void add_infinite(Built& b) {
    std::vector<float> img(60 * 30 * 3);
    for (int y = 0; y < 30; ++y)
        for (int x = 0; x < 60; ++x)
            for (int c = 0; c < 3; ++c)
                img[(y * 60 + x) * 3 + c] = 0.2f + 0.6f * (float)y / 30.f + (c == 2 ? 0.3f : 0.f) + ((x == 17 && y == 22) ? 50.f : 0.f);
    Transform l2w = RotateX(-90) * RotateY(-0) * RotateZ(-50);
    std::vector<std::shared_ptr<Light>> lights = b.scene->lights;
    lights.push_back(std::make_shared<InfiniteAreaLight>(l2w, Spectrum(1.f), 10, 60, 30, 3, img));
    b.scene = std::make_unique<Scene>(b.scene->GetAggregate(), lights);
}

// main.cpp's getSmileFacePlasticMaterial idiom (main.cpp:63-78): an ImageTexture<RGBSpectrum,
// Spectrum> with UVMapping2D(1, 1, 0, 0) as both Kd and Ks of a PlasticMaterial, here on a UV-mapped
// floor, plus a float ImageTexture as the roughness and a textured matte tetrahedron (default UVs).
void build_textured(Built& b, int W, int H) {
    std::vector<float> img(13 * 9 * 3), rough(6 * 5 * 3);
    for (int y = 0; y < 9; ++y)
        for (int x = 0; x < 13; ++x)
            for (int c = 0; c < 3; ++c) img[(y * 13 + x) * 3 + c] = ((x / 2 + y / 2) % 2 ? 0.8f : 0.15f) * (c == 1 ? 0.7f : 1.f);
    for (size_t i = 0; i < rough.size(); ++i) rough[i] = 0.05f + 0.5f * (float)(i % 7) / 7.f;
    std::shared_ptr<Texture<Spectrum>> kd = std::make_shared<ImageTexture<RGBSpectrum, Spectrum>>(
        std::make_unique<UVMapping2D>(1.f, 1.f, 0.f, 0.f), 13, 9, 3, img, false, 8.f, ImageWrap::Repeat, 1.f, false);
    std::shared_ptr<Texture<float>> rg = std::make_shared<ImageTexture<float, float>>(
        std::make_unique<UVMapping2D>(2.f, 2.f, 0.1f, 0.f), 6, 5, 3, rough, false, 8.f, ImageWrap::Clamp, 1.f, false);
    auto plastic = std::make_shared<PlasticMaterial>(kd, kd, rg, nullptr, true);
    auto matte = std::make_shared<MatteMaterial>(std::make_shared<ImageTexture<RGBSpectrum, Spectrum>>(
                                                     std::make_unique<UVMapping2D>(3.f, 3.f, 0.f, 0.f), 13, 9, 3, img, true, 8.f,
                                                     ImageWrap::Black, 0.9f, true),
                                                 fTex(0.f), nullptr);
    std::vector<std::shared_ptr<Primitive>> prims;
    const Transform* id = keep(b, Transform());
    const Point3f fp[4] = {Point3f(-3, -1, -3), Point3f(3, -1, -3), Point3f(3, -1, 3), Point3f(-3, -1, 3)};
    const Point2f fuv[4] = {Point2f(0, 0), Point2f(2.5f, 0), Point2f(2.5f, 2.f), Point2f(0, 2.f)};
    const int fi[6] = {0, 2, 1, 0, 3, 2};
    for (auto& s : CreateTriangleMesh(id, id, false, 2, fi, 4, fp, nullptr, nullptr, fuv))
        prims.push_back(std::make_shared<GeometricPrimitive>(s, plastic, nullptr, MediumInterface()));
    const Point3f tp[4] = {Point3f(-0.8f, -0.9f, -0.5f), Point3f(0.8f, -0.9f, -0.5f), Point3f(0.f, -0.9f, 0.8f), Point3f(0.f, 0.6f, 0.f)};
    const int ti[12] = {0, 2, 1, 0, 1, 3, 1, 2, 3, 2, 0, 3};
    for (auto& s : CreateTriangleMesh(id, id, false, 4, ti, 4, tp, nullptr, nullptr, nullptr))
        prims.push_back(std::make_shared<GeometricPrimitive>(s, matte, nullptr, MediumInterface()));
    std::vector<std::shared_ptr<Light>> lights;
    lights.push_back(std::make_shared<PointLight>(Translate(Vector3f(0.5f, 2.f, 1.5f)), MediumInterface(), Spectrum(8.f)));
    b.scene = std::make_unique<Scene>(std::make_shared<BVHAccel>(prims, 1), lights);
    Transform lookat = LookAt(Point3f(0.f, 0.8f, 3.2f), Point3f(0.f, -0.5f, 0.f), Vector3f(0.f, 1.f, 0.f));
    b.cam = std::shared_ptr<Camera>(CreatePerspectiveCamera(W, H, Inverse(lookat), nullptr));
}

// The same camera/render settings as SamplerIntegrator::Render builds, for the oracle.
pbr_render_desc oracle_desc(const Built& b, const FlatScene& flat, int integrator, int spp, int depth, float rr,
                            int sampler = PBR_SAMPLER_HALTON) {
    auto* cam = dynamic_cast<const PerspectiveCamera*>(b.cam.get());
    pbr_render_desc rd;
    std::memset(&rd, 0, sizeof(rd));
    rd.integrator = integrator;
    rd.max_depth = depth;
    rd.rr_threshold = rr;
    rd.sampler = sampler;
    rd.spp = spp;
    rd.camera.width = cam->RasterWidth;
    rd.camera.height = cam->RasterHeight;
    std::memcpy(rd.camera.camera_to_world.m, cam->CameraToWorld.GetMatrix().m, 64);
    std::memcpy(rd.camera.camera_to_world.m_inv, cam->CameraToWorld.GetInverseMatrix().m, 64);
    rd.camera.fov = cam->fov;
    rd.camera.medium = MediumIndex(flat, cam->medium);
    return rd;
}

// Renders `integrator` through the host API and compares its FrameBuffer with the oracle.
void compare(const char* name, Built& b, std::shared_ptr<SamplerIntegrator> integ, FrameBuffer& fb, int itype, int spp,
             int depth, float rr, int sampler = PBR_SAMPLER_HALTON) {
    double t = 0;
    integ->Render(*b.scene, t);
    auto flat = FlattenScene(*b.scene, nullptr);
    pbr_render_desc rd = oracle_desc(b, *flat, itype, spp, depth, rr, sampler);
    const int W = fb.width, H = fb.height;
    std::vector<float> rgb((size_t)W * H * 3);
    std::vector<uint8_t> rgba((size_t)W * H * 4);
    double sec = 0;
    int rc = oracle_render(SceneDesc(*flat), &rd, rgb.data(), rgba.data(), 0, &sec);
    expect(rc == 0, std::string(name) + ": oracle render");
    // floats within 1e-3; the 8-bit pixel is a function of the float pixel, so it must be identical
    // wherever the float pixel is bit-identical, and within one step elsewhere
    float linf = 0;
    int u8 = 0, u8Exact = 0;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            size_t k = (size_t)(y * W + x);
            size_t f0 = ((size_t)x + (size_t)(H - 1 - y) * W) * fb.channals;   // FrameBuffer is flipped
            bool same = std::memcmp(&fb.getFCbuffer()[f0], &rgb[3 * k], 3 * sizeof(float)) == 0;
            for (int c = 0; c < 3; ++c) {
                float d = std::fabs(fb.getFCbuffer()[f0 + c] - rgb[3 * k + c]);
                if (!(d <= linf)) linf = std::isnan(d) ? 1e30f : d;
                int du = std::abs((int)fb.getUCbuffer()[f0 + c] - (int)rgba[4 * k + c]);
                if (du > u8) u8 = du;
                if (same && du > u8Exact) u8Exact = du;
            }
        }
    char msg[256];
    std::snprintf(msg, sizeof msg, "%s %dx%d %d spp: L_inf %.3g (<= 1e-3), 8-bit max diff %d (<= 1; %d where the floats match, == 0), %.2f ms on device",
                  name, W, H, spp, linf, u8, u8Exact, integ->LastStats().kernel_ms);
    expect(linf <= 1e-3f && u8 <= 1 && u8Exact == 0, msg);
    expect(fb.getUCbuffer()[3] == 255, std::string(name) + ": alpha 255");
}

int run_cpu() {
    Built b;
    build_c1(b, 32, 32);
    auto flat = FlattenScene(*b.scene, nullptr);
    const pbr_scene_desc* d = SceneDesc(*flat);
    expect(d->n_shapes == 2 && d->shapes[0].type == PBR_SHAPE_SPHERE && d->n_lights == 1 && d->n_materials == 1,
           "C1 flattens to 2 spheres, 1 material, 1 point light");
    pbr_render_desc rd = oracle_desc(b, *flat, PBR_INTEGRATOR_WHITTED, 1, 5, 1.f);
    std::vector<float> rgb(32 * 32 * 3);
    std::vector<uint8_t> rgba(32 * 32 * 4);
    double sec;
    expect(oracle_render(d, &rd, rgb.data(), rgba.data(), 1, &sec) == 0 && rgba[0] == 231,
           "oracle on the flattened C1: corner is the F4 grey (231)");
    Built a;
    build_area(a, 16, 16, true);
    auto flat2 = FlattenScene(*a.scene, nullptr);
    const pbr_scene_desc* d2 = SceneDesc(*flat2);
    expect(d2->n_shapes == 3 && d2->shapes[0].n_triangles == 4 && d2->shapes[2].area_light_first == 0 && d2->n_media == 1 &&
               d2->shapes[0].medium_inside == 0 && d2->lights[1].triangle == 1,
           "area-light scene flattens to mesh runs with bound lights and a medium");
    add_infinite(a);
    auto flat3 = FlattenScene(*a.scene, nullptr);
    const pbr_scene_desc* d3 = SceneDesc(*flat3);
    expect(d3->n_lights == 3 && d3->lights[2].type == PBR_LIGHT_INFINITE_AREA && d3->lights[2].env_width == 60 &&
               d3->lights[2].env_data != nullptr && a.scene->infiniteLights.size() == 1,
           "InfiniteAreaLight flattens with its image and is an infinite light");
    Built t;
    build_textured(t, 16, 16);
    auto flat4 = FlattenScene(*t.scene, nullptr);
    const pbr_scene_desc* d4 = SceneDesc(*flat4);
    expect(d4->n_textures == 3 && d4->n_materials == 2 && d4->materials[0].tex[PBR_TEX_KD] == 1 &&
               d4->materials[0].tex[PBR_TEX_KS] == 1 && d4->materials[0].tex[PBR_TEX_ROUGHNESS] == 2 &&
               d4->textures[1].is_float == 1 && d4->textures[1].wrap == PBR_WRAP_CLAMP && d4->textures[2].gamma == 1 &&
               d4->textures[0].width == 13 && d4->textures[0].data != nullptr,
           "ImageTextures flatten once per texture, referenced from their material slots");
    // Render must fail loudly without a device (no CPU fallback)
    FrameBuffer fb;
    fb.InitBuffer(32, 32, 4);
    auto sampler = std::make_shared<HaltonSampler>(1, Bounds2i(Point2i(0, 0), Point2i(32, 32)));
    WhittedIntegrator w(5, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(32, 32)), &fb);
    bool threw = false;
    try {
        double t;
        w.Render(*b.scene, t);
    } catch (const std::runtime_error& e) {
        threw = std::string(e.what()).find("pbr_hip_create") != std::string::npos;
        std::printf("     (%s)\n", e.what());
    }
    expect(threw, "Render without a GPU throws from pbr_hip_create");
    // multi-GPU partition and assembly: every pixel in exactly one rank's tiles, tile i on rank
    // i mod world, and the packed spans scatter back to the frame
    {
        const int W = 100, H = 70, world = 3;
        std::vector<int> owner(W * H, -1);
        std::vector<uint32_t> frame(W * H, 0);
        bool ok = TileGrid(W, H).size() == 4 * 3;
        std::vector<Bounds2i> all = TileGrid(W, H);
        for (int r = 0; r < world; ++r) {
            std::vector<Bounds2i> mine = TilesForRank(W, H, r, world);
            std::vector<uint32_t> packed;
            for (size_t i = 0; i < mine.size(); ++i) {
                const Bounds2i& t = mine[i];
                ok &= t.pMin.x == all[r + i * world].pMin.x && t.pMin.y == all[r + i * world].pMin.y;
                for (int y = t.pMin.y; y < t.pMax.y; ++y)
                    for (int x = t.pMin.x; x < t.pMax.x; ++x) {
                        ok &= owner[y * W + x] < 0;
                        owner[y * W + x] = r;
                        packed.push_back((uint32_t)(y * W + x));
                    }
            }
            AssembleTiles(mine, reinterpret_cast<const uint8_t*>(packed.data()), 4, W, reinterpret_cast<uint8_t*>(frame.data()));
        }
        for (int k = 0; k < W * H; ++k) ok &= owner[k] >= 0 && frame[k] == (uint32_t)k;
        expect(ok, "TilesForRank deals 32x32 tiles round-robin, covering the frame once; AssembleTiles restores it");
    }
    Matrix4x4 m(2, 0, 0, 1, 0, 3, 0, 2, 0, 0, 4, 3, 0, 0, 0, 1);
    Matrix4x4 p = Mul(m, Inverse(m));
    bool ident = true;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) ident &= std::fabs(p.m[i][j] - (i == j ? 1.f : 0.f)) < 1e-6f;
    expect(ident, "Matrix4x4 Inverse");
    return failures ? 1 : 0;
}

// Scene::Intersect / IntersectP / WorldBound and the Primitive virtuals (Scene.h:19-21,
// Primitive.h:13-21) on the device, against the oracle's Scene::Intersect on the same scene.
void scene_queries() {
    Built b;
    build_area(b, 32, 24, true);
    const Scene& sc = *b.scene;
    auto flat = FlattenScene(sc, nullptr);
    // rays: a fan from two origins through the scene, plus a few that must miss
    std::vector<Ray> rays;
    for (int i = 0; i < 24; ++i)
        for (int j = 0; j < 16; ++j) {
            const float u = -1.5f + 3.f * (float)i / 23.f, v = -1.2f + 2.4f * (float)j / 15.f;
            rays.emplace_back(Point3f(0.1f, 0.6f, 3.f), Vector3f(u, v - 0.3f, -2.5f));
            rays.emplace_back(Point3f(-2.f, 2.5f, 0.3f), Vector3f(1.f + 0.2f * u, -1.f + 0.3f * v, -0.1f * v));
        }
    rays.emplace_back(Point3f(0.f, 0.f, 50.f), Vector3f(0.f, 0.f, 1.f));
    rays.emplace_back(Point3f(0.1f, 0.6f, 3.f), Vector3f(0.f, -0.3f, -2.5f), 0.01f);   // short tMax
    const int n = (int)rays.size();
    std::vector<float> rf((size_t)n * 7);
    for (int i = 0; i < n; ++i) {
        const Ray& r = rays[i];
        const float v[7] = {r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, r.tMax};
        std::memcpy(&rf[7 * (size_t)i], v, sizeof v);
    }
    std::vector<float> oc((size_t)n * 5), oa((size_t)n * 5);
    expect(oracle_intersect(SceneDesc(*flat), n, rf.data(), oc.data(), 0) == 0 &&
               oracle_intersect(SceneDesc(*flat), n, rf.data(), oa.data(), 1) == 0, "oracle Intersect / IntersectP");
    std::vector<Ray> batch = rays;
    std::vector<SurfaceInteraction> si;
    std::vector<char> hit, hitP;
    sc.Intersect(batch, &si, &hit);
    sc.IntersectP(rays, &hitP);
    auto* bvh = dynamic_cast<const BVHAccel*>(sc.GetAggregate().get());
    int nHit = 0, bad = 0, badP = 0, badSingle = 0, badPrim = 0, badBox = 0;
    const Bounds3f wb = sc.WorldBound();
    for (int i = 0; i < n; ++i) {
        const float* o = &oc[5 * (size_t)i];
        if ((o[0] != 0.f) != (hit[i] != 0)) { ++bad; continue; }
        if ((oa[5 * (size_t)i] != 0.f) != (hitP[i] != 0) || (sc.IntersectP(rays[i]) != (hitP[i] != 0))) ++badP;
        if (!hit[i]) continue;
        ++nHit;
        const SurfaceInteraction& s = si[i];
        if (batch[i].tMax != o[1] || s.primIndex != (int)o[2] || s.b1 != o[3] || s.b2 != o[4] ||
            s.primitive != bvh->Primitives()[s.primIndex].get())
            ++bad;
        // the single-ray call and the aggregate's own Intersect agree with the batch
        Ray r1 = rays[i];
        SurfaceInteraction s1;
        if (!sc.Intersect(r1, &s1) || r1.tMax != batch[i].tMax || std::memcmp(&s1.p, &s.p, sizeof(Point3f)) != 0) ++badSingle;
        Ray r2 = rays[i];
        SurfaceInteraction s2;
        if (!bvh->Intersect(r2, &s2) || r2.tMax != batch[i].tMax) ++badSingle;
        // GeometricPrimitive::Intersect of the hit primitive alone finds the same t
        Ray r3 = rays[i];
        SurfaceInteraction s3;
        if (!s.primitive->Intersect(r3, &s3) || r3.tMax != batch[i].tMax || !s.primitive->IntersectP(rays[i])) ++badPrim;
        s.primitive->ComputeScatteringFunctions(&s3, TransportMode::Radiance, true);
        if (s3.bsdfMaterial != s.primitive->GetMaterial()) ++badPrim;
        // the hit point lies in the primitive's and the scene's bounds (up to the hit's error bound)
        const Bounds3f pb = s.primitive->WorldBound();
        for (int a = 0; a < 3; ++a) {
            const float e = s.pError[a] + 1e-6f;
            if (s.p[a] < pb.pMin[a] - e || s.p[a] > pb.pMax[a] + e || s.p[a] < wb.pMin[a] - e || s.p[a] > wb.pMax[a] + e) ++badBox;
        }
    }
    char msg[200];
    std::snprintf(msg, sizeof msg, "Scene::Intersect batch = oracle on %d rays (%d hits): hit, tMax, primitive, b1, b2", n, nHit);
    expect(bad == 0 && nHit > n / 4, msg);
    expect(badP == 0, "Scene::IntersectP (batch and single) = oracle IntersectP");
    expect(badSingle == 0, "single-ray Scene::Intersect and BVHAccel::Intersect = the batch");
    expect(badPrim == 0, "GeometricPrimitive::Intersect / IntersectP / ComputeScatteringFunctions of the hit primitive");
    expect(badBox == 0, "hit points inside GeometricPrimitive::WorldBound and Scene::WorldBound");
    expect(bvh->WorldBound().pMin.x == wb.pMin.x && wb.pMin.x < wb.pMax.x, "BVHAccel::WorldBound = Scene::WorldBound");
    // a primitive outside any scene cannot answer
    auto lone = std::make_shared<GeometricPrimitive>(std::static_pointer_cast<GeometricPrimitive>(bvh->Primitives()[0])->shape,
                                                     nullptr, nullptr, MediumInterface());
    bool threw = false;
    try { lone->IntersectP(rays[0]); } catch (const std::logic_error&) { threw = true; }
    expect(threw, "GeometricPrimitive outside a Scene throws");
}

// The sampler surface of Sampler.h: Get1D / Get2D / GetCameraSample / the 1D-2D arrays of a
// GlobalSampler (Sampler.cpp:97-143) equal the oracle's SampleDimension for Halton and pbrt-v3's
// SobolSampler, and Clone copies the sampler.
void sampler_surface() {
    const int W = 37, H = 21;
    for (int kind = 0; kind < 2; ++kind) {
        std::unique_ptr<GlobalSampler> s;
        if (kind == 0) s.reset(new HaltonSampler(16, Bounds2i(Point2i(0, 0), Point2i(W, H))));
        else s.reset(new SobolSampler(12, Bounds2i(Point2i(0, 0), Point2i(W, H))));   // → 16 spp
        expect(s->samplesPerPixel == 16, kind ? "SobolSampler rounds spp up to a power of two" : "Halton spp");
        s->Request1DArray(2);
        s->Request2DArray(1);
        int bad = 0, n = 0;
        for (int px : {0, 5, 36})
            for (int py : {0, 7, 20}) {
                const Point2i pixel(px, py);
                auto c = s->Clone(py * W + px);
                c->StartPixel(pixel);
                int64_t sample = 0;
                do {
                    // expected dims: 0..4 (camera), the 1D array at 5, the 2D array at 6-7 (arrayEndDim = 8),
                    // then Get1D → 8, Get2D → 9, 10
                    CameraSample cs = c->GetCameraSample(pixel);
                    const float* a1 = c->Get1DArray(2);
                    const Point2f* a2 = c->Get2DArray(1);
                    const float u = c->Get1D();
                    const Point2f v = c->Get2D();
                    std::vector<int32_t> q;
                    const int dims[] = {0, 1, 2, 3, 4, 8, 9, 10};
                    for (int d : dims) q.insert(q.end(), {px, py, (int32_t)sample, d});
                    // the arrays: the 1D array at dim 5 (its k-th value of sample s is sample number 2·s + k),
                    // the 2D array at dims 6, 7
                    for (int k = 0; k < 2; ++k) q.insert(q.end(), {px, py, (int32_t)(2 * sample + k), 5});
                    q.insert(q.end(), {px, py, (int32_t)sample, 6});
                    q.insert(q.end(), {px, py, (int32_t)sample, 7});
                    const int nq = (int)q.size() / 4;
                    std::vector<float> ref(nq);
                    std::vector<int64_t> idx(nq);
                    if (kind == 0) expect(oracle_halton(W, H, 16, nq, q.data(), ref.data()) == 0, "oracle_halton");
                    else expect(oracle_sobol(W, H, nq, q.data(), nullptr, 0, ref.data(), idx.data()) == 0, "oracle_sobol");
                    const float got[] = {cs.pFilm.x - (float)px, cs.pFilm.y - (float)py, cs.time, cs.pLens.x, cs.pLens.y, u, v.x, v.y,
                                         a1[0], a1[1], a2[0].x, a2[0].y};
                    for (int k = 0; k < nq; ++k) {
                        const float g = got[k];
                        float want = ref[k];
                        if (k < 2) want = ((float)(k == 0 ? px : py) + ref[k]) - (float)(k == 0 ? px : py);
                        if (std::memcmp(&g, &want, 4) != 0) ++bad;
                        ++n;
                    }
                    ++sample;
                } while (c->StartNextSample());
                expect(sample == 16, "StartNextSample runs samplesPerPixel samples");
            }
        char msg[160];
        std::snprintf(msg, sizeof msg, "%s: GetCameraSample / Get1D / Get2D / Get1DArray / Get2DArray = the oracle's "
                      "SampleDimension (%d values, %d differ)", kind ? "SobolSampler" : "HaltonSampler", n, bad);
        expect(bad == 0, msg);
    }
}

// Sampler subclasses written against the reference's interface (Sampler/Sampler.h:13-82).
// A GlobalSampler that answers GetIndexForSample / SampleDimension itself — here by forwarding to
// a HaltonSampler, so the expected frame is known — renders through Render (the values are
// tabulated, PBR_SAMPLER_TABLE) bit for bit like the HaltonSampler; one shaped like the reference's
// ClockRandSampler (ClockRand.h: index 0, a value per call) renders a finite, deterministic frame; a
// PixelSampler subclass keeps the reference's 1D / 2D streams and RNG fallback and is refused by
// Render (its streams are not one dimension counter).
class ForwardingHalton : public GlobalSampler {
  public:
    ForwardingHalton(int spp, const Bounds2i& b) : GlobalSampler(spp), inner(spp, b) {}
    void StartPixel(const Point2i& p) override {
        inner.StartPixel(p);   // the inner sampler's pixel first: GetIndexForSample reads it
        GlobalSampler::StartPixel(p);
    }
    int64_t GetIndexForSample(int64_t sampleNum) const override { return inner.GetIndexForSample(sampleNum); }
    float SampleDimension(int64_t index, int dimension) const override { return inner.SampleDimension(index, dimension); }
    std::unique_ptr<Sampler> Clone(int) override { return std::unique_ptr<Sampler>(new ForwardingHalton(*this)); }

  private:
    HaltonSampler inner;
};
class HashSampler : public GlobalSampler {   // ClockRandSampler's shape with a deterministic value
  public:
    explicit HashSampler(int spp) : GlobalSampler(spp) {}
    int64_t GetIndexForSample(int64_t sampleNum) const override {
        return ((int64_t)currentPixel.y * 4096 + currentPixel.x) * samplesPerPixel + sampleNum;
    }
    float SampleDimension(int64_t index, int dimension) const override {
        uint64_t h = (uint64_t)index * 0x9E3779B97F4A7C15ull ^ (uint64_t)(dimension + 1) * 0xC2B2AE3D27D4EB4Full;
        h ^= h >> 31; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 29;
        return std::min(0.99999994f, (float)(h >> 40) * (1.f / 16777216.f));
    }
    std::unique_ptr<Sampler> Clone(int) override { return std::unique_ptr<Sampler>(new HashSampler(*this)); }
};
class FilledPixelSampler : public PixelSampler {
  public:
    FilledPixelSampler(int spp, int nDims) : PixelSampler(spp, nDims) {}
    void StartPixel(const Point2i& p) override {
        for (auto& d : samples1D) for (float& v : d) v = 0.25f;
        for (auto& d : samples2D) for (Point2f& v : d) v = Point2f(0.5f, 0.75f);
        Sampler::StartPixel(p);
    }
    std::unique_ptr<Sampler> Clone(int seed) override {
        auto c = std::unique_ptr<FilledPixelSampler>(new FilledPixelSampler(*this));
        c->rng.SetSequence(seed);
        return std::unique_ptr<Sampler>(c.release());
    }
};
void custom_samplers() {
    const int W = 40, H = 30, spp = 8;
    const Bounds2i bounds(Point2i(0, 0), Point2i(W, H));
    for (int itype = 0; itype < 2; ++itype) {
        Built b;
        if (itype == 0) build_c1(b, W, H);
        else build_area(b, W, H, false);
        auto render = [&](std::shared_ptr<Sampler> smp, FrameBuffer& fb) {
            std::shared_ptr<SamplerIntegrator> integ;
            if (itype == 0) integ = std::make_shared<WhittedIntegrator>(5, b.cam, smp, bounds, &fb);
            else integ = std::make_shared<PathIntegrator>(8, b.cam, smp, bounds, 0.8f, "uniform", &fb);
            double t = 0;
            integ->Render(*b.scene, t);
        };
        FrameBuffer ref, fwd, h1, h2;
        for (FrameBuffer* f : {&ref, &fwd, &h1, &h2}) f->InitBuffer(W, H, 4);
        render(std::make_shared<HaltonSampler>(spp, bounds), ref);
        render(std::make_shared<ForwardingHalton>(spp, bounds), fwd);
        const size_t nb = (size_t)W * H * 4;
        expect(std::memcmp(ref.getUCbuffer(), fwd.getUCbuffer(), nb) == 0 &&
                   std::memcmp(ref.getFCbuffer(), fwd.getFCbuffer(), nb * sizeof(float)) == 0,
               itype ? "Path: a GlobalSampler subclass (forwarding SampleDimension) renders = HaltonSampler, bit for bit"
                     : "Whitted: a GlobalSampler subclass (forwarding SampleDimension) renders = HaltonSampler, bit for bit");
        render(std::make_shared<HashSampler>(spp), h1);
        render(std::make_shared<HashSampler>(spp), h2);
        bool finite = true;
        double sum = 0;
        for (size_t k = 0; k < nb; ++k) { finite = finite && std::isfinite(h1.getFCbuffer()[k]); sum += h1.getFCbuffer()[k]; }
        expect(finite && sum > 0 && std::memcmp(h1.getFCbuffer(), h2.getFCbuffer(), nb * sizeof(float)) == 0,
               itype ? "Path: a ClockRandSampler-shaped GlobalSampler renders a finite, deterministic frame"
                     : "Whitted: a ClockRandSampler-shaped GlobalSampler renders a finite, deterministic frame");
    }
    {   // VolPath through media bounded by material-less surfaces: each crossing inside a
        // medium draws HomogeneousMedium::Sample's 2 dimensions without counting as a bounce
        // (VolPathIntegrator.cpp:68-71), so a path can ask for more dimensions than the first table
        // holds; Render tabulates again with more and the frame equals the HaltonSampler's.
        Built b;
        build_boxes(b, W, H);
        auto render = [&](std::shared_ptr<Sampler> smp, FrameBuffer& fb) {
            auto integ = std::make_shared<VolPathIntegrator>(1, b.cam, smp, bounds, 1.f, "uniform", &fb);
            double t = 0;
            integ->Render(*b.scene, t);
        };
        FrameBuffer ref, fwd;
        for (FrameBuffer* f : {&ref, &fwd}) f->InitBuffer(W, H, 4);
        render(std::make_shared<HaltonSampler>(spp, bounds), ref);
        render(std::make_shared<ForwardingHalton>(spp, bounds), fwd);
        const size_t nb = (size_t)W * H * 4;
        expect(std::memcmp(ref.getUCbuffer(), fwd.getUCbuffer(), nb) == 0 &&
                   std::memcmp(ref.getFCbuffer(), fwd.getFCbuffer(), nb * sizeof(float)) == 0,
               "VolPath: a GlobalSampler subclass through nested material-less medium boxes renders = HaltonSampler, bit for bit");
    }
    // PixelSampler: the reference's streams (Sampler.cpp:67-95), refused by Render
    FilledPixelSampler ps(4, 2);
    auto c = ps.Clone(7);
    c->StartPixel(Point2i(1, 2));
    const float a = c->Get1D(), bb = c->Get1D();
    const Point2f p2 = c->Get2D();
    const float beyond = c->Get1D();   // past nSampledDimensions: rng
    RNG rng;
    rng.SetSequence(7);
    const float want = rng.UniformFloat();
    expect(a == 0.25f && bb == 0.25f && p2.x == 0.5f && p2.y == 0.75f && beyond == want,
           "PixelSampler: sampled dimensions, then the RNG (Sampler.cpp:83-95)");
    bool threw = false;
    try {
        Built b;
        build_c1(b, W, H);
        FrameBuffer fb;
        fb.InitBuffer(W, H, 4);
        WhittedIntegrator w(5, b.cam, std::make_shared<FilledPixelSampler>(4, 2), bounds, &fb);
        double t = 0;
        w.Render(*b.scene, t);
    } catch (const std::invalid_argument&) { threw = true; }
    expect(threw, "Render refuses a PixelSampler (its 1D / 2D streams are not on the GPU path)");
}

// An ingested mesh through the C++ surface on the device: tests/golden/mesh_small.3d
// read by plyInfo and built as main.cpp:332-348 builds the dragon (TriangleMesh with an
// object-to-world translation, one Triangle per face, GeometricPrimitive with a glass material),
// rendered by PathIntegrator::Render = the oracle on the flattened scene.
void ply3d_render() {
    char exe[4096];
    const ssize_t len = readlink("/proc/self/exe", exe, sizeof exe - 1);
    if (len <= 0) { expect(false, "locate the test binary"); return; }
    exe[len] = 0;
    std::string dir(exe);
    dir = dir.substr(0, dir.rfind('/'));
    plyInfo plyi(dir + "/../golden/mesh_small.3d");
    expect(plyi.nVertices == 64 && plyi.nTriangles == 110, "plyInfo reads mesh_small.3d (64 vertices, 110 faces)");
    Built b;
    const int W = 40, H = 30, spp = 8;
    build_area(b, W, H, false);   // floor + area light + camera; its tetrahedron is replaced below
    std::vector<std::shared_ptr<Primitive>> prims;
    auto* agg = dynamic_cast<const BVHAccel*>(b.scene->GetAggregate().get());
    for (const auto& p : agg->Primitives()) {   // keep the floor and the light (not the glass tetrahedron)
        auto gp = std::dynamic_pointer_cast<GeometricPrimitive>(p);
        if (!gp || !dynamic_cast<const GlassMaterial*>(gp->material.get())) prims.push_back(p);
    }
    const Transform* o2w = keep(b, Translate(Vector3f(0.0f, -0.35f, 0.0f)));
    const Transform* w2o = keep(b, Inverse(*o2w));
    auto mesh = std::make_shared<TriangleMesh>(*o2w, plyi.nTriangles, plyi.vertexIndices.data(), plyi.nVertices,
                                               plyi.vertexArray.data(), nullptr, nullptr, nullptr, nullptr);
    auto glass = std::make_shared<GlassMaterial>(rgbTex(1, 1, 1), rgbTex(1, 1, 1), fTex(0.1f), fTex(0.1f), fTex(1.5f), nullptr, false);
    for (int i = 0; i < plyi.nTriangles; ++i)
        prims.push_back(std::make_shared<GeometricPrimitive>(std::make_shared<Triangle>(o2w, w2o, false, mesh, i), glass, nullptr,
                                                             MediumInterface()));
    b.scene = std::make_unique<Scene>(std::make_shared<BVHAccel>(prims, 1), b.scene->lights);
    FrameBuffer fb;
    fb.InitBuffer(W, H, 4);
    auto sampler = std::make_shared<HaltonSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
    auto p = std::make_shared<PathIntegrator>(8, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), 0.8f, "uniform", &fb);
    compare("Path, plyInfo mesh_small.3d (glass)", b, p, fb, PBR_INTEGRATOR_PATH, spp, 8, 0.8f);
}

// pbrt-v3's SobolSampler through PathIntegrator::Render (C3's sampler, area light) = the oracle.
void sobol_render() {
    Built b;
    const int W = 48, H = 40, spp = 16;
    build_area(b, W, H, false);
    FrameBuffer fb;
    fb.InitBuffer(W, H, 4);
    auto sampler = std::make_shared<SobolSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
    auto p = std::make_shared<PathIntegrator>(8, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), 0.8f, "uniform", &fb);
    compare("Path + area light, SobolSampler", b, p, fb, PBR_INTEGRATOR_PATH, spp, 8, 0.8f, PBR_SAMPLER_SOBOL);
    bool threw = false;
    try {   // Sobol's resolution comes from the camera raster: other bounds are refused
        auto other = std::make_shared<SobolSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W + 1, H)));
        PathIntegrator q(8, b.cam, other, Bounds2i(Point2i(0, 0), Point2i(W, H)), 0.8f, "uniform", &fb);
        double t = 0;
        q.Render(*b.scene, t);
    } catch (const std::invalid_argument&) { threw = true; }
    expect(threw, "SobolSampler bounds other than the camera raster are refused");
}

// The reference's per-sample loop (Integrator.cpp:286-313) written against the host API —
// StartPixel, GetCameraSample, GenerateRayDifferential, Li, colObj += L, StartNextSample,
// colObj / spp — gives bit for bit the frame Render gives.
void decomposed_render_loop() {
    for (int itype = 0; itype < 3; ++itype) {
        Built b;
        const int W = 20, H = 14, spp = 4;
        if (itype == 0) build_c1(b, W, H); else build_area(b, W, H, false);
        FrameBuffer fb;
        fb.InitBuffer(W, H, 4);
        std::shared_ptr<Sampler> sampler;
        if (itype == 2) sampler = std::make_shared<SobolSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
        else sampler = std::make_shared<HaltonSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
        std::shared_ptr<SamplerIntegrator> integ;
        if (itype == 0) integ = std::make_shared<WhittedIntegrator>(5, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), &fb);
        else integ = std::make_shared<PathIntegrator>(6, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), 0.8f, "uniform", &fb);
        double t = 0;
        integ->Render(*b.scene, t);
        integ->Preprocess(*b.scene, *sampler);
        int bad = 0, checked = 0;
        for (int y = 0; y < H; y += 3)
            for (int x = 0; x < W; x += 2) {
                const Point2i pixel(x, y);
                std::unique_ptr<Sampler> pixelSampler = sampler->Clone(W * y + x);
                pixelSampler->StartPixel(pixel);
                float col[3] = {0.f, 0.f, 0.f};
                do {
                    CameraSample cs = pixelSampler->GetCameraSample(pixel);
                    RayDifferential r;
                    b.cam->GenerateRayDifferential(cs, &r);
                    r.ScaleDifferentials(1 / std::sqrt((float)pixelSampler->samplesPerPixel));
                    Spectrum L = integ->Li(r, *b.scene, *pixelSampler, 0);
                    for (int c = 0; c < 3; ++c) col[c] = col[c] + L[c];
                } while (pixelSampler->StartNextSample());
                for (int c = 0; c < 3; ++c) col[c] = col[c] / (float)spp;
                const float* f = &fb.getFCbuffer()[((size_t)x + (size_t)(H - 1 - y) * W) * 4];
                if (std::memcmp(col, f, sizeof col) != 0) ++bad;
                ++checked;
            }
        char msg[200];
        std::snprintf(msg, sizeof msg, "%s: the reference's per-sample loop through Clone / StartPixel / GetCameraSample / "
                      "GenerateRay / Li = Render, bit for bit (%d pixels)",
                      itype == 0 ? "Whitted C1" : (itype == 1 ? "Path area light" : "Path area light, SobolSampler"), checked);
        expect(bad == 0, msg);
    }
}

// SetDevices: tiles dealt over devices, spans gathered (RCCL over distinct devices; a repeated
// device gets its own context and a copy) — the FrameBuffer equals the single-device Render's.
void multi_gpu_render() {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    std::vector<std::vector<int>> sets = {{0}, {0, 0}, {0, 0, 0}};
    if (ndev >= 2) sets.push_back({0, 1});
    Built b;
    const int W = 77, H = 45, spp = 4;
    build_area(b, W, H, false);
    FrameBuffer ref, fb;
    ref.InitBuffer(W, H, 4);
    fb.InitBuffer(W, H, 4);
    auto sampler = std::make_shared<HaltonSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
    PathIntegrator single(6, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), 0.8f, "uniform", &ref);
    double t = 0;
    single.Render(*b.scene, t);
    for (const auto& devs : sets) {
        PathIntegrator multi(6, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), 0.8f, "uniform", &fb);
        multi.SetDevices(devs);
        std::memset(fb.getUCbuffer(), 0, (size_t)W * H * 4);
        multi.Render(*b.scene, t);
        multi.Render(*b.scene, t);   // a second frame reuses contexts, buffers and communicator
        const bool same = std::memcmp(fb.getUCbuffer(), ref.getUCbuffer(), (size_t)W * H * 4) == 0 &&
                          std::memcmp(fb.getFCbuffer(), ref.getFCbuffer(), (size_t)W * H * 4 * sizeof(float)) == 0;
        std::string d;
        for (int x : devs) d += std::to_string(x) + " ";
        expect(same, "multi-GPU Render over devices { " + d + "}" + (devs.size() == 1 || devs[0] != devs[1] ? " (RCCL gather)" : " (copies)") +
                         " = single-device Render, bit for bit");
    }
}

int run_gpu() {
    {
        Built b;
        const int W = 96, H = 64, spp = 4;
        build_c1(b, W, H);
        FrameBuffer fb;
        fb.InitBuffer(W, H, 4);
        auto sampler = std::make_shared<HaltonSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
        auto w = std::make_shared<WhittedIntegrator>(5, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), &fb);
        compare("Whitted C1", b, w, fb, PBR_INTEGRATOR_WHITTED, spp, 5, 1.f);
    }
    {
        Built b;
        const int W = 48, H = 40, spp = 8;
        build_area(b, W, H, false);
        FrameBuffer fb;
        fb.InitBuffer(W, H, 4);
        auto sampler = std::make_shared<HaltonSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
        auto p = std::make_shared<PathIntegrator>(8, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), 0.8f, "uniform", &fb);
        compare("Path glass + area light", b, p, fb, PBR_INTEGRATOR_PATH, spp, 8, 0.8f);
    }
    {
        Built b;
        const int W = 40, H = 32, spp = 8;
        build_area(b, W, H, true);
        FrameBuffer fb;
        fb.InitBuffer(W, H, 4);
        auto sampler = std::make_shared<HaltonSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
        auto v = std::make_shared<VolPathIntegrator>(10, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), 1.f, "uniform", &fb);
        compare("VolPath homogeneous medium", b, v, fb, PBR_INTEGRATOR_VOLPATH, spp, 10, 1.f);
    }
    {
        Built b;
        const int W = 48, H = 36, spp = 8;
        build_textured(b, W, H);
        FrameBuffer fb;
        fb.InitBuffer(W, H, 4);
        auto sampler = std::make_shared<HaltonSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
        auto p = std::make_shared<PathIntegrator>(5, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), 1.f, "uniform", &fb);
        compare("Path ImageTexture plastic + matte", b, p, fb, PBR_INTEGRATOR_PATH, spp, 5, 1.f);
    }
    {   // main.cpp's own configuration: VolPath d10 "uniform" + the rotated InfiniteAreaLight
        Built b;
        const int W = 40, H = 32, spp = 8;
        build_area(b, W, H, true);
        add_infinite(b);
        FrameBuffer fb;
        fb.InitBuffer(W, H, 4);
        auto sampler = std::make_shared<HaltonSampler>(spp, Bounds2i(Point2i(0, 0), Point2i(W, H)));
        auto v = std::make_shared<VolPathIntegrator>(10, b.cam, sampler, Bounds2i(Point2i(0, 0), Point2i(W, H)), 1.f, "uniform", &fb);
        compare("VolPath medium + InfiniteAreaLight", b, v, fb, PBR_INTEGRATOR_VOLPATH, spp, 10, 1.f);
    }
    scene_queries();
    decomposed_render_loop();
    sampler_surface();
    sobol_render();
    custom_samplers();
    ply3d_render();
    multi_gpu_render();
    return failures ? 1 : 0;
}

// main.cpp's output stage (main.cpp:419-429) on a patterned FrameBuffer: set_uc, a few
// update_f_u_c averages, stbi_flip_vertically_on_write + stbi_write_png.  The raw ubuffer goes
// to <png>.raw; tests/test_host_cpp.py decodes the PNG and compares.
int run_png(const char* path) {
    const int W = 37, H = 23;
    FrameBuffer fb;
    fb.InitBuffer(W, H, 4);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 4; ++c) fb.set_uc(x, y, c, (unsigned char)((x * 7 + y * 13 + c * 29) & 255));
    for (int n = 1; n <= 3; ++n) fb.update_f_u_c(5, 6, 1, n, 0.25f * (float)n);   // f: .25, .375, .5 → u8 127
    if (fb.update_f_u_c(W, 0, 0, 1, 1.f) || fb.set_uc(-1, 0, 0, 0)) { std::printf("FAIL out-of-bounds write accepted\n"); return 1; }
    stbi_flip_vertically_on_write(1);
    if (!stbi_write_png(path, W, H, 4, fb.getUCbuffer(), W * 4)) { std::printf("FAIL stbi_write_png\n"); return 1; }
    FILE* f = std::fopen((std::string(path) + ".raw").c_str(), "wb");
    if (!f) return 1;
    std::fwrite(fb.getUCbuffer(), 1, (size_t)W * H * 4, f);
    std::fclose(f);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    std::string mode = argc > 1 ? argv[1] : "cpu";
    try {
        if (mode == "png") return run_png(argc > 2 ? argv[2] : "host_api_test.png");
        if ((mode == "ply3d" || mode == "ply") && argc > 2) {   // mesh readers: "v <hex x> <hex y> <hex z>", "f a b c"
            std::vector<Point3f> v;
            std::vector<int> idx;
            if (mode == "ply3d") { plyInfo info(argv[2]); v = info.vertexArray; idx = info.vertexIndices; }
            else { PlyMesh m = LoadPLY(argv[2]); v = m.vertices; idx = m.indices; }
            for (const Point3f& p : v) {
                uint32_t b[3];
                std::memcpy(&b[0], &p.x, 4); std::memcpy(&b[1], &p.y, 4); std::memcpy(&b[2], &p.z, 4);
                std::printf("v %08x %08x %08x\n", b[0], b[1], b[2]);
            }
            for (size_t k = 0; k + 2 < idx.size(); k += 3) std::printf("f %d %d %d\n", idx[k], idx[k + 1], idx[k + 2]);
            return 0;
        }
        if (mode == "tiles" && argc > 4) {   // tiles W H world: one "rank x0 y0 x1 y1" line per tile
            const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), world = std::atoi(argv[4]);
            for (int r = 0; r < world; ++r)
                for (const Bounds2i& t : TilesForRank(W, H, r, world)) std::printf("%d %d %d %d %d\n", r, t.pMin.x, t.pMin.y, t.pMax.x, t.pMax.y);
            return 0;
        }
        int rc = mode == "gpu" ? run_gpu() : run_cpu();
        std::printf("%s: %d failure(s)\n", mode.c_str(), failures);
        return rc;
    } catch (const std::exception& e) {
        std::printf("FAIL exception: %s\n", e.what());
        return 2;
    }
}
