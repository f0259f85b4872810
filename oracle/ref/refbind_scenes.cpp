// refbind_scenes.cpp — TEST INFRASTRUCTURE ONLY (oracle/_ref/libpbr_refbind.so).  Exercises the
// reference-side binding (integration/reference_binding/pbr_hip_integrator.{h,cpp}) the way a user of
// the reference would: scenes assembled from the reference's OWN classes as Main/main.cpp:186-413
// does (TriangleMesh / Triangle / GeometricPrimitive, Matte / Mirror / Glass / Metal / Plastic
// materials over ConstantTextures and ImageTextures, SkyBoxLight and InfiniteAreaLight from .hdr
// files, DiffuseAreaLight, HomogeneousMedium, BVHAccel(SAH), Scene, CreatePerspectiveCamera or a
// PerspectiveCamera of another fov / screen window, HaltonSampler), rendered once by the reference's
// own Integrator::Render (Integrator.cpp:280-356) and once by the binding's HipSamplerIntegrator — the
// drop-in that replaces it — into two FrameBuffers.  The reference's per-pixel float colObj / spp (its
// Render writes only the 8-bit buffer) comes from the same per-pixel body driven here
// (Clone, StartPixel, GetCameraSample, GenerateRayDifferential, Li), the drop-in's from the float
// buffer it fills.  tests/test_reference_binding.py compares them.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include <omp.h>
#include <unistd.h>

#define private public   // BVHAccel's node array (tree-identity check), FrameBuffer's float buffer
#define protected public
#include "Accelerator\BVHAccel.h"
#include "Core\FrameBuffer.h"
#undef protected
#undef private
#include "Camera\orthographic.h"
#include "Camera\Perspective.h"
#include "Core\Primitive.h"
#include "Core\Scene.h"
#include "Core\Transform.h"
#include "Integrator\PathIntegrator.h"
#include "Integrator\VolPathIntegrator.h"
#include "Integrator\WhittedIntegrator.h"
#include "Light\DiffuseLight.h"
#include "Sampler\Sampling.h"   // Distribution2D, before InfiniteAreaLight.h holds one
#include "Light\InfiniteAreaLight.h"
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

#include "../../integration/reference_binding/pbr_hip_integrator.h"

using namespace PBR;

// from oracle/ref/ref_harness.cpp (libpbr_ref.so): the arena that survives the reference's BSDF
// double destroy while its Render runs, and stb's HDR writer
extern "C" void ref_frame_arena(int on);
extern "C" int stbi_write_hdr(char const* filename, int w, int h, int comp, const float* data);
extern "C" void stbi_flip_vertically_on_write(int flag);
extern "C" void stbi_set_flip_vertically_on_load(int flag);

namespace {

std::shared_ptr<Texture<Spectrum>> cs(float r, float g, float b) {
    Spectrum s;
    s[0] = r; s[1] = g; s[2] = b;
    return std::make_shared<ConstantTexture<Spectrum>>(s);
}
std::shared_ptr<Texture<float>> cf(float v) { return std::make_shared<ConstantTexture<float>>(v); }

// the displaced-sphere dragon stand-in: (n+1) latitude rows × n longitudes, with
// (longitude, latitude) UVs for the textured scene
void standin(int n, std::vector<Point3f>* P, std::vector<int>* I, std::vector<Point2f>* UV = nullptr) {
    const double kPi = 3.14159265358979323846;
    for (int a = 0; a <= n; ++a)
        for (int b = 0; b < n; ++b) {
            const double th = kPi * a / n, ph = 2 * kPi * b / n;
            const double r = 1.0 + 0.08 * std::sin(7 * th) * std::cos(9 * ph) + 0.03 * std::sin(31 * th + 17 * ph);
            P->push_back(Point3f((float)(r * std::sin(th) * std::cos(ph)), (float)(r * std::cos(th)),
                                 (float)(r * std::sin(th) * std::sin(ph))));
            if (UV) UV->push_back(Point2f((float)b / n * 2.f, (float)a / n * 2.f));   // each tile repeats twice
        }
    for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) {
            const int i00 = a * n + b, i01 = a * n + (b + 1) % n, i10 = (a + 1) * n + b, i11 = (a + 1) * n + (b + 1) % n;
            I->insert(I->end(), {i00, i10, i11, i00, i11, i01});
        }
}

// an .hdr file with a procedural image (w × h RGB), removed with the scene
std::string write_hdr(int w, int h, float (*f)(int, int, int, int, int)) {
    std::vector<float> img((size_t)w * h * 3);
    for (int j = 0; j < h; ++j)
        for (int i = 0; i < w; ++i)
            for (int c = 0; c < 3; ++c) img[((size_t)j * w + i) * 3 + c] = f(i, j, c, w, h);
    char path[] = "/tmp/pbr_refbind_imgXXXXXX";
    const int fd = mkstemp(path);
    if (fd >= 0) close(fd);
    stbi_flip_vertically_on_write(0);
    if (!stbi_write_hdr(path, w, h, 3, img.data())) throw std::runtime_error("stbi_write_hdr failed");
    return path;
}

struct Built {
    std::vector<std::unique_ptr<Transform>> xf;
    std::vector<std::shared_ptr<Primitive>> prims;
    std::vector<std::shared_ptr<Light>> lights;
    std::unique_ptr<HomogeneousMedium> medium;
    std::shared_ptr<BVHAccel> bvh;
    std::unique_ptr<Scene> scene;
    std::shared_ptr<Camera> cam;
    std::vector<std::string> files;
    ~Built() {
        for (auto& f : files) unlink(f.c_str());
    }
    const Transform* keep(const Transform& t) {
        xf.emplace_back(new Transform(t));
        return xf.back().get();
    }
    // a triangle mesh as main.cpp builds one (:283-302): TriangleMesh, its Triangles, one
    // GeometricPrimitive each
    std::vector<std::shared_ptr<Shape>> mesh(const Transform& o2w, const std::vector<Point3f>& P, const std::vector<int>& I,
                                             const std::shared_ptr<Material>& m, const MediumInterface& mi,
                                             bool emissive = false, float Le = 0.f, const std::vector<Point2f>* UV = nullptr) {
        const Transform* a = keep(o2w);
        const Transform* b = keep(Inverse(o2w));
        auto tm = std::make_shared<TriangleMesh>(*a, (int)I.size() / 3, I.data(), (int)P.size(), P.data(), nullptr, nullptr,
                                                 UV ? UV->data() : nullptr, nullptr);
        std::vector<std::shared_ptr<Shape>> tris;
        for (int t = 0; t < (int)I.size() / 3; ++t) {
            tris.push_back(std::make_shared<Triangle>(a, b, false, tm, t));
            std::shared_ptr<AreaLight> area;
            if (emissive) {   // main.cpp's area light block (:360-372): DiffuseAreaLight(Le, 5 samples, one-sided)
                area = std::make_shared<DiffuseAreaLight>(*a, MediumInterface(), Spectrum(Le), 5, tris.back(), false);
                lights.push_back(area);
            }
            prims.push_back(std::make_shared<GeometricPrimitive>(tris.back(), m, area, mi));
        }
        return tris;
    }
};

// The scenes (integrator, depth, rr and light strategy in make_ref / make_hip below):
//   2: C2 shape — Whitted d5, green matte dragon on a mirror floor under a SkyBox
//   3: C3 shape — Path d8 rr 0.8, matte dragon + floor, one-sided area light
//   4: C4 shape — Path d8 rr 0.8, three dragons with main.cpp's glass, metal (u/v roughness) and
//      plastic (remapped roughness) recipes (:160-183, :228-239), matte floor, area light
//   5: C5 shape — VolPath d10, glass dragon bounding a HomogeneousMedium, area light
//   6: the scene main.cpp ships (:186-413) — VolPath d10 rr 1 "uniform", a mirror floor, an
//      InfiniteAreaLight (RotateX(-90)·RotateY(-0)·RotateZ(-50), power 1, 10 samples) from an .hdr,
//      and (the FBX knight needs assimp: the stand-in instead) an object in main.cpp's
//      getSmileFacePlasticMaterial (an ImageTexture as Kd and Ks, UVMapping2D, Repeat)
//   7: scene 2 through a PerspectiveCamera built directly with fov 65 and an off-centre screen window
//   8: scene 2 through an OrthographicCamera (the binding refuses it)
std::unique_ptr<Built> build(int config, int res) {
    std::unique_ptr<Built> B(new Built);
    std::vector<Point3f> P;
    std::vector<int> I;
    std::vector<Point2f> UV;
    standin(config == 4 || config == 6 ? 24 : 40, &P, &I, config == 6 ? &UV : nullptr);
    const auto bump = cf(0.f);
    const auto white = std::make_shared<MatteMaterial>(cs(0.8f, 0.8f, 0.8f), cf(0.f), bump);
    const auto green = std::make_shared<MatteMaterial>(cs(0.f, 1.f, 0.f), cf(0.f), bump);
    MediumInterface none;
    const std::vector<int> FI = {0, 1, 2, 3, 4, 5};
    auto floor = [&](float L, float y) {
        return std::vector<Point3f>{Point3f(-L, y, L), Point3f(L, y, L), Point3f(-L, y, -L),
                                    Point3f(L, y, L), Point3f(L, y, -L), Point3f(-L, y, -L)};
    };
    auto areaLight = [&](float a, float y) {
        std::vector<Point3f> Q = {Point3f(-a, 0.f, a), Point3f(-a, 0.f, -a), Point3f(a, 0.f, a),
                                  Point3f(a, 0.f, a), Point3f(-a, 0.f, -a), Point3f(a, 0.f, -a)};
        B->mesh(Translate(Vector3f(0.f, y, 0.f)), Q, FI, white, none, true, 5.f);
    };
    Transform c2w = Inverse(LookAt(Point3f(0.f, 0.55f, 2.6f), Point3f(0.f, -0.25f, 0.f), Vector3f(0.f, 1.f, 0.f)));
    if (config == 4) {
        // main.cpp's recipes: getWhiteGlassMaterial, getYellowMetalMaterial, plasticMaterial
        const auto glass = std::make_shared<GlassMaterial>(cs(0.98f, 0.98f, 0.98f), cs(0.98f, 0.98f, 0.98f), cf(0.1f), cf(0.1f),
                                                           cf(1.5f), bump, false);
        const auto metal = std::make_shared<MetalMaterial>(cs(0.2f, 0.2f, 0.8f), cs(0.11f, 0.11f, 0.11f), cf(0.15f), cf(0.15f),
                                                           cf(0.15f), bump, false);
        Spectrum purple;
        purple[0] = 0.35f; purple[1] = 0.12f; purple[2] = 0.48f;
        const auto plastic = std::make_shared<PlasticMaterial>(std::make_shared<ConstantTexture<Spectrum>>(purple),
                                                               std::make_shared<ConstantTexture<Spectrum>>(Spectrum(1.f) - purple),
                                                               cf(0.1f), bump, true);
        const std::shared_ptr<Material> mats[3] = {glass, metal, plastic};
        for (int k = 0; k < 3; ++k) B->mesh(Translate(Vector3f(-2.3f + 2.3f * k, 0.f, 0.f)), P, I, mats[k], none);
        B->mesh(Transform(), floor(10.f, -1.12f), FI, white, none);
        areaLight(1.8f, 2.9f);
        c2w = Inverse(LookAt(Point3f(0.f, 1.2f, 5.f), Point3f(0.f, -0.3f, 0.f), Vector3f(0.f, 1.f, 0.f)));
    } else if (config == 6) {
        // getSmileFacePlasticMaterial (main.cpp:63-78): awesomeface.jpg → a procedural image (non-power-
        // of-two, so the MIPMap resamples it), UVMapping2D(1, 1, 0, 0), Repeat, no trilinear, maxAniso 8
        const std::string face = write_hdr(40, 24, [](int i, int j, int c, int w, int h) {
            const float u = (i + 0.5f) / w - 0.5f, v = (j + 0.5f) / h - 0.5f;
            const bool eye = (std::fabs(std::fabs(u) - 0.18f) < 0.07f && std::fabs(v + 0.15f) < 0.08f);
            const bool mouth = std::fabs(v - 0.18f) < 0.05f && std::fabs(u) < 0.3f;
            const float base = c == 0 ? 0.95f : (c == 1 ? 0.8f : 0.1f);
            return eye || mouth ? 0.05f : base * (0.6f + 0.4f * (float)i / w);
        });
        B->files.push_back(face);
        std::unique_ptr<TextureMapping2D> map(new UVMapping2D(1.f, 1.f, 0.f, 0.f));
        std::shared_ptr<Texture<Spectrum>> Kt = std::make_shared<ImageTexture<RGBSpectrum, Spectrum>>(
            std::move(map), face, false, 8.f, ImageWrap::Repeat, 1.f, false);
        const auto smile = std::make_shared<PlasticMaterial>(Kt, Kt, cf(0.1f), bump, true);
        B->mesh(Translate(Vector3f(0.f, -120.f, -60.f)) * Scale(25.f, 25.f, 25.f), P, I, smile, none, false, 0.f, &UV);
        // main.cpp:255-282: the mirror floor, 2 triangles, length 200 at groundY -200
        const auto mirror = std::make_shared<MirrorMaterial>(cs(1.f, 1.f, 1.f), bump);
        std::vector<Point3f> Fl = {Point3f(-200.f, -200.f, 200.f), Point3f(200.f, -200.f, 200.f), Point3f(-200.f, -200.f, -200.f),
                                   Point3f(200.f, -200.f, 200.f), Point3f(200.f, -200.f, -200.f), Point3f(-200.f, -200.f, -200.f)};
        B->mesh(Transform(), Fl, FI, mirror, none);
        // main.cpp:377-382: the InfiniteAreaLight (Free8kalienatmosphereHDRI.hdr → a procedural sky
        // with a sun, 96 × 48: resampled to 128 × 64 by the light's MIPMap)
        const std::string sky = write_hdr(96, 48, [](int i, int j, int c, int w, int h) {
            const float u = (i + 0.5f) / w, v = (j + 0.5f) / h;
            const float du = u - 0.3f, dv = v - 0.35f;
            const float sun = (du * du + dv * dv < 0.004f) ? 40.f : 0.f;
            return sun + (c == 2 ? 0.9f : 0.35f + 0.3f * v) * (0.5f + 0.5f * std::sin(6.2831853f * u * 3.f) * 0.2f);
        });
        B->files.push_back(sky);
        const Transform l2w = RotateX(-90) * RotateY(-0) * RotateZ(-50);
        B->lights.push_back(std::make_shared<InfiniteAreaLight>(l2w, Spectrum(1.f), 10, sky));
        c2w = Inverse(LookAt(Point3f(0.f, -100.f, 40.f), Point3f(0.f, -102.f, 0.f), Vector3f(0.f, 1.f, 0.f)));
    } else {
        if (config == 5) {
            B->medium.reset(new HomogeneousMedium(Spectrum(0.5f), Spectrum(4.4f), -0.5f));   // main.cpp:242
            const auto glass = std::make_shared<GlassMaterial>(cs(1.f, 1.f, 1.f), cs(1.f, 1.f, 1.f), cf(0.f), cf(0.f), cf(1.5f),
                                                               bump, false);
            B->mesh(Transform(), P, I, glass, MediumInterface(B->medium.get(), nullptr));
        } else {
            B->mesh(Transform(), P, I, green, none);
        }
        const bool whitted = config == 2 || config == 7 || config == 8;
        if (whitted) B->mesh(Transform(), floor(40.f, -1.12f), FI, std::make_shared<MirrorMaterial>(cs(1.f, 1.f, 1.f), bump), none);
        else B->mesh(Transform(), floor(40.f, -1.12f), FI, white, none);
        if (whitted) {
            // SkyBoxLight reads its image from a file (SkyBoxLight.cpp:16-24): a procedural sky written as .hdr
            const std::string sky = write_hdr(64, 32, [](int i, int j, int c, int w, int h) {
                return c == 0 ? 0.25f + 0.5f * (float)j / h : (c == 1 ? 0.35f + 0.4f * (float)i / w : 0.9f - 0.3f * (float)j / h);
            });
            B->files.push_back(sky);
            stbi_set_flip_vertically_on_load(0);
            B->lights.push_back(std::make_shared<SkyBoxLight>(Transform(), Point3f(0.f, 0.f, 0.f), 60.f, sky.c_str(), 1));
        } else {
            areaLight(0.8f, 2.0f);
        }
    }
    B->bvh = std::make_shared<BVHAccel>(B->prims, 1, BVHAccel::SplitMethod::SAH);   // main.cpp:383
    B->scene.reset(new Scene(B->bvh, B->lights));
    if (config == 7) {   // PerspectiveCamera(…, screenWindow, lensRadius, focalDistance, fov, medium), Perspective.cpp:6-9
        Bounds2f screen;
        screen.pMin.x = -0.8f; screen.pMax.x = 1.2f; screen.pMin.y = -1.1f; screen.pMax.y = 0.9f;
        B->cam = std::make_shared<PerspectiveCamera>(res, res, c2w, screen, 0.f, 0.f, 65.f, nullptr);
    } else if (config == 8) {
        Bounds2f screen;
        screen.pMin.x = -1.5f; screen.pMax.x = 1.5f; screen.pMin.y = -1.5f; screen.pMax.y = 1.5f;
        B->cam = std::make_shared<OrthographicCamera>(res, res, c2w, screen, 0.f, 0.f, nullptr);
    } else {
        B->cam = std::shared_ptr<Camera>(CreatePerspectiveCamera(res, res, c2w, nullptr));
    }
    return B;
}

int integrator_of(int config) { return config == 2 || config == 7 || config == 8 ? 0 : (config == 3 || config == 4 ? 1 : 2); }

}  // namespace

extern "C" {

// Renders scene `config` at res × res, spp samples per pixel, with the reference's own integrator
// (ref_out) and with the binding's drop-in (hip_out): FrameBuffer bytes (getUCbuffer: res·res·4,
// row 0 = the image's bottom row).  ref_rgb / hip_rgb (optional, res·res·3, image rows top to
// bottom): the reference's colObj / spp from its per-pixel body, the drop-in's from the FrameBuffer's
// float buffer.  bvh_equal: the device's uploaded node array equals the reference BVHAccel's byte for
// byte.  Returns 0, or -1 with the message in err.
int refbind_render(int config, int res, int spp, uint8_t* ref_out, uint8_t* hip_out, float* ref_rgb, float* hip_rgb,
                   double* seconds, int* bvh_equal, char* err, int errlen) {
    try {
        std::unique_ptr<Built> B = build(config, res);
        const Bounds2i bounds(Point2i(0, 0), Point2i(res, res));
        auto sampler = std::make_shared<HaltonSampler>(spp, bounds);   // main.cpp:388-391
        const int integ = integrator_of(config);
        auto make_ref = [&](FrameBuffer* fb) -> std::shared_ptr<SamplerIntegrator> {
            if (integ == 0) return std::make_shared<WhittedIntegrator>(5, B->cam, sampler, bounds, fb);
            if (integ == 1) return std::make_shared<PathIntegrator>(8, B->cam, sampler, bounds, 0.8f, "uniform", fb);
            return std::make_shared<VolPathIntegrator>(10, B->cam, sampler, bounds, 1.f, "uniform", fb);
        };
        // the drop-in: the same arguments, pbrhip:: in front of the class name
        auto make_hip = [&](FrameBuffer* fb) -> std::shared_ptr<pbrhip::HipSamplerIntegrator> {
            if (integ == 0) return std::make_shared<pbrhip::HipWhittedIntegrator>(5, B->cam, sampler, bounds, fb);
            if (integ == 1) return std::make_shared<pbrhip::HipPathIntegrator>(8, B->cam, sampler, bounds, 0.8f, "uniform", fb);
            return std::make_shared<pbrhip::HipVolPathIntegrator>(10, B->cam, sampler, bounds, 1.f, "uniform", fb);
        };
        if (config != 8) {   // (the OrthographicCamera scene is only handed to the drop-in, which refuses it)
            FrameBuffer fb;
            fb.InitBuffer(res, res, 4);
            auto ref = make_ref(&fb);
            double t = 0;
            ref_frame_arena(1);
            ref->Render(*B->scene, t);
            ref_frame_arena(0);
            std::memcpy(ref_out, fb.getUCbuffer(), (size_t)res * res * 4);
            if (seconds) seconds[0] = t;
            if (ref_rgb) {
                // SamplerIntegrator::Render's per-pixel body (Integrator.cpp:288-313) on the same objects:
                // the float colObj / spp its u8 bytes come from (identical work: a square raster)
                auto li = make_ref(nullptr);
                li->Preprocess(*B->scene, *sampler);
                ref_frame_arena(1);
#pragma omp parallel for schedule(dynamic, 4)
                for (int k = 0; k < res * res; ++k) {
                    const int x = k % res, y = k / res;
                    std::unique_ptr<Sampler> ps = sampler->Clone(res * y + x);
                    const Point2i pixel(x, y);
                    ps->StartPixel(pixel);
                    Spectrum colObj(0.0f);
                    do {
                        CameraSample cs0 = ps->GetCameraSample(pixel);
                        RayDifferential r;
                        B->cam->GenerateRayDifferential(cs0, &r);
                        r.ScaleDifferentials(1 / std::sqrt((float)ps->samplesPerPixel));
                        colObj += li->Li(r, *B->scene, *ps, 0);
                    } while (ps->StartNextSample());
                    colObj /= (float)ps->samplesPerPixel;
                    for (int c = 0; c < 3; ++c) ref_rgb[3 * k + c] = colObj[c];
                    ps.release();   // arena memory (ref_harness.cpp): never handed back to the heap
                }
                ref_frame_arena(0);
            }
        }
        {
            FrameBuffer fb;
            fb.InitBuffer(res, res, 4);
            auto hip = make_hip(&fb);
            hip->SetWriteFloatBuffer(hip_rgb != nullptr);   // the device's floats, read back below
            double t = 0;
            hip->Render(*B->scene, t);
            std::memcpy(hip_out, fb.getUCbuffer(), (size_t)res * res * 4);
            if (hip_rgb)   // fbuffer rows as set_fc wrote them: row res-1-y holds image row y
                for (int y = 0; y < res; ++y)
                    for (int x = 0; x < res; ++x)
                        for (int c = 0; c < 3; ++c)
                            hip_rgb[((size_t)y * res + x) * 3 + c] = fb.fbuffer[((size_t)(res - 1 - y) * res + x) * 4 + c];
            if (seconds) seconds[1] = t;
            if (bvh_equal) {
                int nn = 0, np = 0;
                if (pbr_hip_get_bvh(hip->Context(), nullptr, &nn, nullptr, &np) != PBR_OK) throw std::runtime_error("get_bvh");
                std::vector<unsigned char> dev((size_t)nn * 32);
                std::vector<int32_t> ids(np);
                if (pbr_hip_get_bvh(hip->Context(), dev.data(), &nn, ids.data(), &np) != PBR_OK) throw std::runtime_error("get_bvh");
                const std::vector<unsigned char>& ref = hip->Flat()->nodes;
                *bvh_equal = dev.size() == ref.size() && std::memcmp(dev.data(), ref.data(), ref.size()) == 0 &&
                             np == (int)B->bvh->primitives.size();
            }
        }
        return 0;
    } catch (const std::exception& e) {
        ref_frame_arena(0);
        if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", e.what());
        return -1;
    }
}

// The binding's own flattened scene and render descriptor for scene `config` (what its Render hands
// the C-ABI) rendered by two CPU restatements whose oracle_render entry points the caller passes in:
// `oracle` (oracle/liboracle.so, correctly rounded transcendentals) into ora_rgb and `libm`
// (oracle/liboracle_libm.so, glibc's float functions as the reference calls them) into libm_rgb —
// res·res·3 floats, image rows top to bottom.  Test infrastructure: it separates the drop-in's
// differences from the reference into the restatement's (none: device = oracle) and libm's last bits
// (libm twin = reference).
typedef int (*oracle_render_fn)(const pbr_scene_desc*, const pbr_render_desc*, float*, uint8_t*, int, double*);
int refbind_render_oracles(int config, int res, int spp, void* oracle, void* libm, float* ora_rgb, float* libm_rgb,
                           char* err, int errlen) {
    try {
        std::unique_ptr<Built> B = build(config, res);
        const Bounds2i bounds(Point2i(0, 0), Point2i(res, res));
        auto sampler = std::make_shared<HaltonSampler>(spp, bounds);
        const int integ = integrator_of(config);
        FrameBuffer fb;
        fb.InitBuffer(res, res, 4);
        std::shared_ptr<pbrhip::HipSamplerIntegrator> hip;
        if (integ == 0) hip = std::make_shared<pbrhip::HipWhittedIntegrator>(5, B->cam, sampler, bounds, &fb);
        else if (integ == 1) hip = std::make_shared<pbrhip::HipPathIntegrator>(8, B->cam, sampler, bounds, 0.8f, "uniform", &fb);
        else hip = std::make_shared<pbrhip::HipVolPathIntegrator>(10, B->cam, sampler, bounds, 1.f, "uniform", &fb);
        double t = 0;
        hip->Render(*B->scene, t);
        pbr_render_desc rd = hip->LastRenderDesc();
        std::vector<uint8_t> rgba((size_t)res * res * 4);
        double sec = 0;
        if (ora_rgb && oracle_render_fn(oracle)(&hip->Flat()->desc, &rd, ora_rgb, rgba.data(), 0, &sec) != 0)
            throw std::runtime_error("oracle_render failed");
        if (libm_rgb && oracle_render_fn(libm)(&hip->Flat()->desc, &rd, libm_rgb, rgba.data(), 0, &sec) != 0)
            throw std::runtime_error("oracle_render (libm twin) failed");
        return 0;
    } catch (const std::exception& e) {
        if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", e.what());
        return -1;
    }
}

// The flattening alone (no device): counts of what SceneFlattener hands the C-ABI for scene
// `config` — shapes, triangles, materials, lights, media, BVH nodes, textures — and the reference's
// own primitive and light counts, for the CPU tests.  tex0 (optional, 4 ints): the first texture's
// width, height, components and level0 flag; light0 (optional, 4 ints): the first light's type,
// env_width, env_height and whether its Le is (1, 1, 1).
int refbind_flatten(int config, int* counts, int* tex0, int* light0, char* err, int errlen) {
    try {
        std::unique_ptr<Built> B = build(config, 16);
        auto F = pbrhip::SceneFlattener::Flatten(*B->scene);
        int tris = 0;
        for (const auto& sd : F->shapes) tris += sd.n_triangles;
        counts[0] = F->desc.n_shapes;
        counts[1] = tris;
        counts[2] = F->desc.n_materials;
        counts[3] = F->desc.n_lights;
        counts[4] = F->desc.n_media;
        counts[5] = F->desc.n_bvh_nodes;
        counts[6] = (int)B->bvh->primitives.size();
        counts[7] = (int)B->scene->lights.size();
        counts[8] = F->desc.n_textures;
        if (tex0 && F->desc.n_textures > 0) {
            const pbr_texture_desc& t = F->desc.textures[0];
            tex0[0] = t.width; tex0[1] = t.height; tex0[2] = t.components; tex0[3] = t.level0;
        }
        if (light0 && F->desc.n_lights > 0) {
            const pbr_light_desc& l = F->desc.lights[0];
            light0[0] = l.type; light0[1] = l.env_width; light0[2] = l.env_height;
            light0[3] = l.Le[0] == 1.f && l.Le[1] == 1.f && l.Le[2] == 1.f;
        }
        return 0;
    } catch (const std::exception& e) {
        if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", e.what());
        return -1;
    }
}

}  // extern "C"
