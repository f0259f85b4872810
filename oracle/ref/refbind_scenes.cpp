// refbind_scenes.cpp — TEST INFRASTRUCTURE ONLY (oracle/_ref/libpbr_refbind.so).  Exercises the
// reference-side binding (integration/reference_binding/pbr_hip_integrator.{h,cpp}) the way a user of
// the reference would: scenes assembled from the reference's OWN classes as Main/main.cpp:186-413
// does (TriangleMesh / Triangle / GeometricPrimitive, Matte / Mirror / Glass materials over
// ConstantTextures, SkyBoxLight from an .hdr file, DiffuseAreaLight, HomogeneousMedium, BVHAccel(SAH),
// Scene, CreatePerspectiveCamera, HaltonSampler), rendered once by the reference's own
// Integrator::Render (Integrator.cpp:280-356) and once by the binding's HipSamplerIntegrator — the
// drop-in that replaces it — into two FrameBuffers.  tests/test_reference_binding.py compares them.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include <unistd.h>

#define private public   // BVHAccel's node array, for the tree-identity check only
#include "Accelerator\BVHAccel.h"
#undef private
#include "Camera\Perspective.h"
#include "Core\FrameBuffer.h"
#include "Core\Primitive.h"
#include "Core\Scene.h"
#include "Core\Transform.h"
#include "Integrator\PathIntegrator.h"
#include "Integrator\VolPathIntegrator.h"
#include "Integrator\WhittedIntegrator.h"
#include "Light\DiffuseLight.h"
#include "Light\SkyBoxLight.h"
#include "Material\GlassMaterial.h"
#include "Material\MatteMaterial.h"
#include "Material\Mirror.h"
#include "Media\HomogeneousMedium.h"
#include "Sampler\Halton.h"
#include "Shape\Triangle.h"
#include "Texture\ConstantTexture.h"

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

// the displaced-sphere dragon stand-in: (n+1) latitude rows × n longitudes
void standin(int n, std::vector<Point3f>* P, std::vector<int>* I) {
    const double kPi = 3.14159265358979323846;
    for (int a = 0; a <= n; ++a)
        for (int b = 0; b < n; ++b) {
            const double th = kPi * a / n, ph = 2 * kPi * b / n;
            const double r = 1.0 + 0.08 * std::sin(7 * th) * std::cos(9 * ph) + 0.03 * std::sin(31 * th + 17 * ph);
            P->push_back(Point3f((float)(r * std::sin(th) * std::cos(ph)), (float)(r * std::cos(th)),
                                 (float)(r * std::sin(th) * std::sin(ph))));
        }
    for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) {
            const int i00 = a * n + b, i01 = a * n + (b + 1) % n, i10 = (a + 1) * n + b, i11 = (a + 1) * n + (b + 1) % n;
            I->insert(I->end(), {i00, i10, i11, i00, i11, i01});
        }
}

struct Built {
    std::vector<std::unique_ptr<Transform>> xf;
    std::vector<std::shared_ptr<Primitive>> prims;
    std::vector<std::shared_ptr<Light>> lights;
    std::unique_ptr<HomogeneousMedium> medium;
    std::shared_ptr<BVHAccel> bvh;
    std::unique_ptr<Scene> scene;
    std::shared_ptr<Camera> cam;
    std::string skyFile;
    ~Built() { if (!skyFile.empty()) unlink(skyFile.c_str()); }
    const Transform* keep(const Transform& t) {
        xf.emplace_back(new Transform(t));
        return xf.back().get();
    }
    // a triangle mesh as main.cpp builds one (:283-302): TriangleMesh, its Triangles, one
    // GeometricPrimitive each
    std::vector<std::shared_ptr<Shape>> mesh(const Transform& o2w, const std::vector<Point3f>& P, const std::vector<int>& I,
                                             const std::shared_ptr<Material>& m, const MediumInterface& mi,
                                             bool emissive = false, float Le = 0.f) {
        const Transform* a = keep(o2w);
        const Transform* b = keep(Inverse(o2w));
        auto tm = std::make_shared<TriangleMesh>(*a, (int)I.size() / 3, I.data(), (int)P.size(), P.data(), nullptr, nullptr,
                                                 nullptr, nullptr);
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

// config 2: C2 shape — Whitted, green matte dragon on a mirror floor under a SkyBox
// config 3: C3 shape — Path d8 rr 0.8, matte dragon + floor, one-sided area light
// config 5: C5 shape — VolPath d10, glass dragon bounding a HomogeneousMedium, area light
std::unique_ptr<Built> build(int config, int res) {
    std::unique_ptr<Built> B(new Built);
    std::vector<Point3f> P;
    std::vector<int> I;
    standin(40, &P, &I);
    const auto bump = cf(0.f);
    const auto white = std::make_shared<MatteMaterial>(cs(0.8f, 0.8f, 0.8f), cf(0.f), bump);
    const auto green = std::make_shared<MatteMaterial>(cs(0.f, 1.f, 0.f), cf(0.f), bump);
    MediumInterface none;
    if (config == 5) {
        B->medium.reset(new HomogeneousMedium(Spectrum(0.5f), Spectrum(4.4f), -0.5f));   // main.cpp:242
        const auto glass = std::make_shared<GlassMaterial>(cs(1.f, 1.f, 1.f), cs(1.f, 1.f, 1.f), cf(0.f), cf(0.f), cf(1.5f),
                                                           bump, false);
        B->mesh(Transform(), P, I, glass, MediumInterface(B->medium.get(), nullptr));
    } else {
        B->mesh(Transform(), P, I, green, none);
    }
    const float L = 40.f, y = -1.12f;
    std::vector<Point3f> F = {Point3f(-L, y, L), Point3f(L, y, L), Point3f(-L, y, -L),
                              Point3f(L, y, L), Point3f(L, y, -L), Point3f(-L, y, -L)};
    std::vector<int> FI = {0, 1, 2, 3, 4, 5};
    if (config == 2) B->mesh(Transform(), F, FI, std::make_shared<MirrorMaterial>(cs(1.f, 1.f, 1.f), bump), none);
    else B->mesh(Transform(), F, FI, white, none);
    if (config == 2) {
        // SkyBoxLight reads its image from a file (SkyBoxLight.cpp:16-24): a procedural sky written as .hdr
        const int w = 64, h = 32;
        std::vector<float> img((size_t)w * h * 3);
        for (int j = 0; j < h; ++j)
            for (int i = 0; i < w; ++i) {
                float* p = &img[((size_t)j * w + i) * 3];
                p[0] = 0.25f + 0.5f * (float)j / h;
                p[1] = 0.35f + 0.4f * (float)i / w;
                p[2] = 0.9f - 0.3f * (float)j / h;
            }
        char path[] = "/tmp/pbr_refbind_skyXXXXXX";
        const int fd = mkstemp(path);
        if (fd >= 0) close(fd);
        B->skyFile = path;
        stbi_flip_vertically_on_write(0);
        if (!stbi_write_hdr(path, w, h, 3, img.data())) throw std::runtime_error("stbi_write_hdr failed");
        stbi_set_flip_vertically_on_load(0);
        B->lights.push_back(std::make_shared<SkyBoxLight>(Transform(), Point3f(0.f, 0.f, 0.f), 60.f, path, 1));
    } else {
        const float a = 0.8f;
        std::vector<Point3f> Q = {Point3f(-a, 0.f, a), Point3f(-a, 0.f, -a), Point3f(a, 0.f, a),
                                  Point3f(a, 0.f, a), Point3f(-a, 0.f, -a), Point3f(a, 0.f, -a)};
        B->mesh(Translate(Vector3f(0.f, 2.0f, 0.f)), Q, FI, white, none, true, 5.f);
    }
    B->bvh = std::make_shared<BVHAccel>(B->prims, 1, BVHAccel::SplitMethod::SAH);   // main.cpp:383
    B->scene.reset(new Scene(B->bvh, B->lights));
    const Transform c2w = Inverse(LookAt(Point3f(0.f, 0.55f, 2.6f), Point3f(0.f, -0.25f, 0.f), Vector3f(0.f, 1.f, 0.f)));
    B->cam = std::shared_ptr<Camera>(CreatePerspectiveCamera(res, res, c2w, nullptr));
    return B;
}

}  // namespace

extern "C" {

// Renders scene `config` (2, 3, 5) at res × res, spp samples per pixel, with the reference's own
// integrator (ref_out) and with the binding's drop-in (hip_out): FrameBuffer bytes (getUCbuffer:
// res·res·4, row 0 = the image's bottom row).  bvh_equal: the device's uploaded node array equals the
// reference BVHAccel's byte for byte.  Returns 0, or -1 with the message in err.
int refbind_render(int config, int res, int spp, uint8_t* ref_out, uint8_t* hip_out, double* seconds, int* bvh_equal,
                   char* err, int errlen) {
    try {
        std::unique_ptr<Built> B = build(config, res);
        const Bounds2i bounds(Point2i(0, 0), Point2i(res, res));
        auto sampler = std::make_shared<HaltonSampler>(spp, bounds);   // main.cpp:388-391
        auto make_ref = [&](FrameBuffer* fb) -> std::shared_ptr<Integrator> {
            if (config == 2) return std::make_shared<WhittedIntegrator>(5, B->cam, sampler, bounds, fb);
            if (config == 3) return std::make_shared<PathIntegrator>(8, B->cam, sampler, bounds, 0.8f, "uniform", fb);
            return std::make_shared<VolPathIntegrator>(10, B->cam, sampler, bounds, 1.f, "uniform", fb);
        };
        // the drop-in: the same arguments, pbrhip:: in front of the class name
        auto make_hip = [&](FrameBuffer* fb) -> std::shared_ptr<pbrhip::HipSamplerIntegrator> {
            if (config == 2) return std::make_shared<pbrhip::HipWhittedIntegrator>(5, B->cam, sampler, bounds, fb);
            if (config == 3) return std::make_shared<pbrhip::HipPathIntegrator>(8, B->cam, sampler, bounds, 0.8f, "uniform", fb);
            return std::make_shared<pbrhip::HipVolPathIntegrator>(10, B->cam, sampler, bounds, 1.f, "uniform", fb);
        };
        {
            FrameBuffer fb;
            fb.InitBuffer(res, res, 4);
            auto integ = make_ref(&fb);
            double t = 0;
            ref_frame_arena(1);
            integ->Render(*B->scene, t);
            ref_frame_arena(0);
            std::memcpy(ref_out, fb.getUCbuffer(), (size_t)res * res * 4);
            if (seconds) seconds[0] = t;
        }
        {
            FrameBuffer fb;
            fb.InitBuffer(res, res, 4);
            auto integ = make_hip(&fb);
            double t = 0;
            integ->Render(*B->scene, t);
            std::memcpy(hip_out, fb.getUCbuffer(), (size_t)res * res * 4);
            if (seconds) seconds[1] = t;
            if (bvh_equal) {
                int nn = 0, np = 0;
                if (pbr_hip_get_bvh(integ->Context(), nullptr, &nn, nullptr, &np) != PBR_OK) throw std::runtime_error("get_bvh");
                std::vector<unsigned char> dev((size_t)nn * 32);
                std::vector<int32_t> ids(np);
                if (pbr_hip_get_bvh(integ->Context(), dev.data(), &nn, ids.data(), &np) != PBR_OK) throw std::runtime_error("get_bvh");
                const std::vector<unsigned char>& ref = integ->Flat()->nodes;
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

// The flattening alone (no device): counts of what SceneFlattener hands the C-ABI for scene
// `config` — shapes, triangles, materials, lights, media, BVH nodes — and the reference's own
// primitive and light counts, for the CPU tests.
int refbind_flatten(int config, int* counts, char* err, int errlen) {
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
        return 0;
    } catch (const std::exception& e) {
        if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", e.what());
        return -1;
    }
}

}  // extern "C"
