/*
 * pbr_hip.h — C-ABI drop-in boundary for the MI355X render path.
 *
 * The reference (G0T-cha/PysicalBasedRaytracer) has no FFI: its hot path is reached through the
 * C++ virtual `Integrator::Render(const Scene&, double&)` (Integrator/Integrator.h:14) after the
 * scene has been assembled from `GeometricPrimitive`s (Core/Primitive.h:30-33), a `BVHAccel`
 * (Accelerator/BVHAccel.h:19-21), lights (Light/Light.h:50-61), a `HaltonSampler`
 * (Sampler/Halton.h:18) and a `PerspectiveCamera` (Camera/Perspective.cpp:84-104).
 * The C++ host mirror in include/pbr/ keeps those class names and constructors; underneath, every
 * one of them flattens into the POD descriptors below and crosses into the HIP runtime through the
 * five `pbr_hip_*` entry points.  Nothing here uses torch or STL types: plain pointers and sizes.
 *
 * Entry point ↔ reference interface it replaces:
 *   pbr_hip_create        — (none; the reference has one implicit CPU "device")
 *   pbr_hip_upload_scene  — Scene::Scene (Core/Scene.cpp:7-17) + BVHAccel::BVHAccel
 *                           (Accelerator/BVHAccel.cpp:57-87) + TriangleMesh ctor (Shape/Triangle.cpp:12-44)
 *                           + HaltonSampler ctor (Sampler/Halton.cpp:30-58)
 *   pbr_hip_render        — SamplerIntegrator::Render (Integrator/Integrator.cpp:280-356), which
 *                           drives {Whitted,Path,VolPath}Integrator::Li per sample
 *   pbr_hip_destroy       — scene/integrator destructors
 *   pbr_hip_last_error    — (none; the reference fails silently)
 *   pbr_hip_sync          — (none; the reference's Render returns when the frame is done): waits
 *                           for asynchronous frames and reports a deferred failure
 *
 * Errors: every call returns 0 on success, a negative PBR_E_* code otherwise; the message is
 * kept per context and returned by pbr_hip_last_error.  Calls on one context are not thread-safe;
 * different contexts (one per device) are independent.
 *
 * Unbounded walks: the reference follows chains of material-less surfaces (medium boundaries)
 * without limit (WhittedIntegrator.cpp:26-28, PathIntegrator.cpp:70-75, Light.cpp:31-47).  The
 * device follows them too, up to safety bounds far beyond any sane scene — 1024 crossings in one
 * Whitted Li or Path/VolPath path, 256 interfaces on one transmittance walk — and a frame in which
 * a walk reaches a bound fails with PBR_E_UNSUPPORTED (synchronous renders: that call;
 * asynchronous ones: the next pbr_hip_render or pbr_hip_sync on the context) instead of returning
 * a truncated image.  BVH traversal keeps the reference's 64-entry stack (BVHAccel.cpp:293): an
 * upload whose tree could overflow it (or the 1.5-entries-per-level need of the two-level node walk)
 * fails with PBR_E_UNSUPPORTED.
 */
#ifndef PBR_HIP_H
#define PBR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBR_HIP_ABI_VERSION 5

/* ---- status codes ---- */
enum {
    PBR_OK = 0,
    PBR_E_INVALID = -1,   /* bad argument / descriptor */
    PBR_E_HIP = -2,       /* a HIP runtime call failed */
    PBR_E_NOSCENE = -3,   /* render before upload */
    PBR_E_UNSUPPORTED = -4,
    PBR_E_NODEVICE = -5
};

/* ---- enums mirroring the reference's class families ---- */
enum pbr_shape_type { PBR_SHAPE_TRIANGLE_MESH = 0, PBR_SHAPE_SPHERE = 1 };
enum pbr_material_type {
    PBR_MAT_NONE = 0,     /* GeometricPrimitive with material == nullptr (medium boundary) */
    PBR_MAT_MATTE = 1,    /* Material/MatteMaterial.cpp:13-28 */
    PBR_MAT_MIRROR = 2,   /* Material/Mirror.cpp:5-15 */
    PBR_MAT_GLASS = 3,    /* Material/GlassMaterial.cpp:9-57 */
    PBR_MAT_METAL = 4,    /* Material/MetalMaterial.cpp:25-43 */
    PBR_MAT_PLASTIC = 5   /* Material/PlasticMaterial.cpp:8-30 */
};
enum pbr_light_type {
    PBR_LIGHT_POINT = 0,        /* Light/PointLight.cpp */
    PBR_LIGHT_DIFFUSE_AREA = 1, /* Light/DiffuseLight.cpp */
    PBR_LIGHT_SKYBOX = 2,       /* Light/SkyBoxLight.cpp */
    PBR_LIGHT_INFINITE_AREA = 3 /* Light/InfiniteAreaLight.cpp: light_to_world, Le = the `power`
                                 * scale, n_samples, env_* = the image as stbi_loadf returned it
                                 * (NULL → a 1x1 map of Le); worldRadius from the scene bounds.
                                 * A caller holding only a built light's map — Lmap's level 0
                                 * (InfiniteAreaLight.h:33: powers of two, L already applied) —
                                 * passes those texels with Le = (1, 1, 1): 1·x is x, a power-of-two
                                 * image is not resampled (MIPMap.h:96), so the upload rebuilds the
                                 * same pyramid, Distribution2D and Power() */
};
enum pbr_integrator_type {
    PBR_INTEGRATOR_WHITTED = 0, /* Integrator/WhittedIntegrator.cpp:11-65 */
    PBR_INTEGRATOR_PATH = 1,    /* Integrator/PathIntegrator.cpp:32-110 */
    PBR_INTEGRATOR_VOLPATH = 2  /* Integrator/VolPathIntegrator.cpp:21-107 */
};
/* HALTON: Sampler/Halton.cpp; SOBOL: pbrt-v3's SobolSampler over the reference's SobolMatrices32;
 * TABLE: values supplied by the caller — a host sampler the device cannot compute, e.g. a custom
 * GlobalSampler subclass (Sampler/Sampler.h:62-82): see pbr_render_desc::sample_table. */
enum pbr_sampler_type { PBR_SAMPLER_HALTON = 0, PBR_SAMPLER_SOBOL = 1, PBR_SAMPLER_TABLE = 2 };
enum pbr_light_strategy { PBR_LIGHTS_UNIFORM = 0, PBR_LIGHTS_POWER = 1 };
/* BVHAccel::SplitMethod (Accelerator/BVHAccel.h:18); HLBVH falls through to SAH (BVHAccel.cpp:135-160). */
enum pbr_split_method { PBR_SPLIT_SAH = 0, PBR_SPLIT_HLBVH = 1, PBR_SPLIT_MIDDLE = 2, PBR_SPLIT_EQUAL_COUNTS = 3 };

/* A reference Transform holds both m and mInv (Core/Transform.h:49-60); so do we. Row-major. */
typedef struct pbr_transform {
    float m[16];
    float m_inv[16];
} pbr_transform;

/* One Shape family instance. Primitives are enumerated in shape order, triangles in index order:
 * this is the `prims` vector order the reference hands to BVHAccel (Main/main.cpp:279-282). */
typedef struct pbr_shape_desc {
    int type;                   /* pbr_shape_type */
    pbr_transform object_to_world;
    int reverse_orientation;
    /* triangle mesh (Shape/Triangle.h:11-24) */
    int n_triangles;
    int n_vertices;
    const int32_t* indices;     /* 3*n_triangles */
    const float* P;             /* 3*n_vertices, object space */
    const float* N;             /* optional 3*n_vertices per-vertex normals, or NULL */
    const float* UV;            /* optional 2*n_vertices, or NULL (default (0,0),(1,0),(1,1)) */
    /* sphere (Shape/Sphere.h) */
    float radius;
    /* GeometricPrimitive fields (Core/Primitive.h:30-33) */
    int material;               /* index into materials, -1 = nullptr */
    int area_light_first;       /* triangle t carries lights[area_light_first + t]; -1 = none */
    int medium_inside;          /* MediumInterface, -1 = nullptr */
    int medium_outside;
} pbr_shape_desc;

/* ImageTexture<RGBSpectrum, Spectrum> / <float, float> (Texture/ImageTexture.h:43-91,
 * ImageTexture.cpp:13-92) with a UVMapping2D (Texture/Texture.h:16-27).  The reference's ray
 * differentials are zero (dudx = dvdx = 0, F5), so both MIPMap filters — trilinear (MIPMap.h:193-211)
 * and EWA (:227-247) — reduce to the bilinear level-0 lookup triangle(0, st) (:240-252); the pyramid
 * above level 0 is never read.  Level 0 is the image resampled to powers of two with the texture's
 * wrap mode (MIPMap.h:86-150). */
enum pbr_image_wrap { PBR_WRAP_REPEAT = 0, PBR_WRAP_BLACK = 1, PBR_WRAP_CLAMP = 2 };   /* ImageWrap, MIPMap.h:21 */
typedef struct pbr_texture_desc {
    int is_float;               /* 1: ImageTexture<float, float> (convertIn: scale * y()), 0: RGB */
    int width, height, components;
    const float* data;          /* as loadImage's stbi_loadf returns it (flip-on-load set); NULL →
                                 * the 1x1 grey 0.5 image GetTexture substitutes (ImageTexture.cpp:60-66) */
    float scale;
    int gamma;                  /* convertIn applies InverseGammaCorrect (Core/PBR.h:126-129) */
    int wrap;                   /* pbr_image_wrap */
    int trilinear;              /* doTrilinear (no effect, see above) */
    float max_aniso;            /* maxAniso (no effect, see above) */
    float su, sv, du, dv;       /* UVMapping2D(su, sv, du, dv): st = (su·u + du, sv·v + dv) */
    int level0;                 /* 1: `data` is already the MIPMap's level 0 — what a built ImageTexture
                                 * holds (ImageTexture.h:88, MIPMap.h:150-153): width and height powers
                                 * of two, convertIn applied, `components` = 3 (RGB) or 1 (float
                                 * textures); used as is (scale and gamma ignored) */
} pbr_texture_desc;

/* Material parameter slots that may hold an image texture instead of the constant below
 * (pbr_material_desc.tex[slot] = index into pbr_scene_desc.textures + 1; 0 = the constant, so a
 * zero-initialised descriptor has no textures).  RGB slots need an RGB texture, scalar slots a
 * float one. */
enum pbr_texture_slot {
    PBR_TEX_KD = 0,             /* matte / plastic Kd (RGB) */
    PBR_TEX_KS = 1,             /* plastic Ks (RGB) */
    PBR_TEX_KR = 2,             /* mirror / glass Kr (RGB) */
    PBR_TEX_KT = 3,             /* glass Kt (RGB) */
    PBR_TEX_SIGMA = 4,          /* matte sigma (float) */
    PBR_TEX_ROUGHNESS = 5,      /* plastic roughness (float) */
    PBR_TEX_SLOTS = 6
};

typedef struct pbr_material_desc {
    int type;                   /* pbr_material_type */
    float Kd[3];                /* matte Kd, plastic Kd */
    float sigma;                /* matte sigma (degrees) */
    float Kr[3];                /* mirror Kr, glass Kr */
    float Kt[3];                /* glass Kt */
    float Ks[3];                /* plastic Ks */
    float eta;                  /* glass index */
    float metal_eta[3];         /* metal eta */
    float metal_k[3];           /* metal k */
    float roughness;            /* metal roughness / plastic roughness */
    float uroughness;           /* glass/metal u roughness (metal: used when has_uv_roughness) */
    float vroughness;
    int has_uv_roughness;       /* metal: uRoughness/vRoughness textures present */
    int remap_roughness;
    int tex[PBR_TEX_SLOTS];     /* pbr_texture_slot → texture index + 1, or 0 (triangle meshes only) */
} pbr_material_desc;

typedef struct pbr_light_desc {
    int type;                   /* pbr_light_type */
    pbr_transform light_to_world;
    float I[3];                 /* point intensity */
    float Le[3];                /* area emission */
    int shape;                  /* area light: index of the mesh shape ... */
    int triangle;               /* ... and the triangle in it */
    int two_sided;
    int n_samples;
    int medium_inside, medium_outside;
    /* SkyBoxLight (Light/SkyBoxLight.h): env data as stbi_loadf returns it with vertical flip */
    float world_center[3];
    float world_radius;
    int env_width, env_height, env_components;
    const float* env_data;      /* env_width*env_height*env_components, or NULL → black */
} pbr_light_desc;

typedef struct pbr_medium_desc {   /* Media/HomogeneousMedium.h */
    float sigma_a[3];
    float sigma_s[3];
    float g;
} pbr_medium_desc;

typedef struct pbr_scene_desc {
    int abi_version;            /* PBR_HIP_ABI_VERSION */
    int n_shapes;
    const pbr_shape_desc* shapes;
    int n_materials;
    const pbr_material_desc* materials;
    int n_lights;
    const pbr_light_desc* lights;
    int n_media;
    const pbr_medium_desc* media;
    int max_prims_in_node;      /* BVHAccel maxPrimsInNode (main.cpp:385 uses 1) */
    int n_textures;
    const pbr_texture_desc* textures;
    int split_method;           /* pbr_split_method (BVHAccel.h:18); Middle / EqualCounts build on the host */
    /* A BVHAccel already built over the primitives IN THE ORDER GIVEN HERE — the reference's own
     * flattened node array (LinearBVHNode, BVHAccel.cpp:46-55, 32 B each), as a Scene's aggregate
     * holds it after its constructor reordered `primitives` into leaf order.  The upload then uses
     * that tree as is instead of building one: the traversal tests the reference's boxes in the
     * reference's order.  It is checked to be a preorder tree whose leaves hold primitives 0..n-1
     * in order, each leaf box the union of its primitives' bounds (PBR_E_INVALID otherwise).
     * NULL = build one (split_method, max_prims_in_node). */
    const void* bvh_nodes;
    int n_bvh_nodes;
} pbr_scene_desc;

/* CreatePerspectiveCamera (Camera/Perspective.cpp:84-104) inputs. */
typedef struct pbr_camera_desc {
    int width, height;          /* raster resolution */
    pbr_transform camera_to_world;
    int use_look_at;            /* if set, camera_to_world = Inverse(LookAt(eye, look, up)) */
    float eye[3], look[3], up[3];
    float fov;                  /* degrees; the reference fixes 90 */
    float lens_radius;          /* the reference fixes 0 */
    float focal_distance;
    int medium;                 /* camera medium (dropped by CameraToWorld, F12) */
    /* 1: raster_to_camera is the camera's own ProjectiveCamera::RasterToCamera (Camera.h:36-53:
     * Inverse(CameraToScreen) · RasterToScreen of its screen window and fov), used instead of
     * CreatePerspectiveCamera's (fov above, the raster's aspect-ratio screen window): a reference
     * PerspectiveCamera built with any fov or screen window (Perspective.cpp:6-9) hands over exactly */
    int use_raster_to_camera;
    pbr_transform raster_to_camera;
} pbr_camera_desc;

typedef struct pbr_tile {
    int x0, y0, x1, y1;         /* half-open pixel rectangle */
} pbr_tile;

typedef struct pbr_render_desc {
    int integrator;             /* pbr_integrator_type */
    int max_depth;
    float rr_threshold;
    int light_strategy;         /* pbr_light_strategy ("spatial" falls back to uniform, LightDistrib.cpp:10-21) */
    int sampler;                /* pbr_sampler_type */
    int spp;
    pbr_camera_desc camera;
    /* pixels to render; n_tiles == 0 → whole frame. Output is packed tile after tile, each tile
     * row-major, 3 floats (linear RGB = colObj/spp) and 4 bytes (RGBA8) per pixel. */
    int n_tiles;
    const pbr_tile* tiles;
    int outputs_on_device;      /* 1: rgb_out/rgba_out are device pointers (e.g. torch tensors) */
    void* stream;               /* hipStream_t to launch on (NULL = context stream).  With
                                 * outputs_on_device, collect_stats == 0 and stats == NULL the call
                                 * is asynchronous: it returns once the frame is enqueued on `stream`
                                 * and the caller synchronises (frames queue back to back). */
    int collect_stats;          /* 1: also count BVH node visits / triangle tests (slower) */
    /* PBR_SAMPLER_SOBOL (pbrt-v3 SobolSampler; the reference ships only its tables, F3):
     * generator matrices in the layout of the reference's SobolMatrices32 (Sampler/SobolMatrices.h:
     * 42-47: [dims][52] uint32 columns).  NULL → the built-in matrices, which are the
     * reference's SobolMatrices32 (all 1024 dimensions, regenerated from the Joe-Kuo direction
     * numbers the table was built from; hash-checked against it).  spp is rounded up to a power of
     * two (GlobalSampler(RoundUpPow2(spp))).  Sample indices are 64-bit as pbrt-v3's: up to 2^52
     * (2·log2(resolution) + log2(spp) <= 52). */
    const uint32_t* sobol_matrices;
    int sobol_dims;
    /* PBR_SAMPLER_TABLE: every sample's dimensions as the caller's sampler gives them —
     * sample_table[((y * camera.width + x) * spp + s) * table_dims + d] = SampleDimension(
     * GetIndexForSample(s), d) at pixel (x, y), host memory, rows of pixels outside the tiles unused.
     * GlobalSampler's bookkeeping (a Get2D at dimension 4 moves to 5, Sampler.cpp:131-143) applies as
     * for the device samplers.  A path that asks for a dimension >= table_dims fails the frame
     * (PBR_E_UNSUPPORTED).  Frames with a table are synchronous; camera.width·height·spp < 2^32. */
    const float* sample_table;
    int table_dims;
} pbr_render_desc;

typedef struct pbr_render_stats {
    double seconds;             /* wall time of the render call (incl. launch + sync) */
    double kernel_ms;           /* device time of the integrator kernel(s), HIP events */
    double film_ms;             /* device time of the film/output kernel */
    uint64_t samples;           /* pixels * spp rendered */
    uint64_t rays;              /* rays traced (closest + any hit), if collect_stats */
    uint64_t node_visits;       /* LinearBVHNode visits, if collect_stats */
    uint64_t prim_tests;        /* primitive intersection tests, if collect_stats */
    uint64_t shading_events;    /* surface/medium interactions shaded, if collect_stats */
    int n_launches;
} pbr_render_stats;

typedef struct pbr_hip_ctx pbr_hip_ctx;

int pbr_hip_create(int device, pbr_hip_ctx** out);
int pbr_hip_upload_scene(pbr_hip_ctx* ctx, const pbr_scene_desc* scene);
int pbr_hip_render(pbr_hip_ctx* ctx, const pbr_render_desc* desc,
                   float* rgb_out, uint8_t* rgba_out, pbr_render_stats* stats);
int pbr_hip_destroy(pbr_hip_ctx* ctx);
const char* pbr_hip_last_error(const pbr_hip_ctx* ctx);
/* Waits for the context's asynchronous frames; returns PBR_E_UNSUPPORTED if one of them stopped at
 * a safety bound (see above). */
int pbr_hip_sync(pbr_hip_ctx* ctx);
/* n frames of one descriptor in one call — SamplerIntegrator::Render (Integrator.cpp:280-356) n
 * times, e.g. the frames of an animation or the timed frames of a benchmark.  The frames' chunks
 * continue one rotation over the chunk lanes with no join between frames, so the launches that end
 * one frame overlap the ones that start the next (a frame of few chunks — a multi-GPU rank's shard —
 * otherwise leaves the GPU part idle at its end).  Every frame is the same bits as pbr_hip_render's.
 * Frame f goes to rgb_outs[f] / rgba_outs[f] (device pointers; either array may be NULL).  Requires
 * desc->outputs_on_device = 1, collect_stats = 0, no sample table.  Asynchronous: returns once the
 * frames are enqueued; desc->stream (NULL: the context stream) reaches its tail when all are done;
 * pbr_hip_wait_frame orders another stream after one frame. */
int pbr_hip_render_frames(pbr_hip_ctx* ctx, const pbr_render_desc* desc, int n, float* const* rgb_outs,
                          uint8_t* const* rgba_outs);
/* Makes `stream` (hipStream_t; NULL = the context stream) wait until frame f of the last
 * pbr_hip_render_frames call is complete (e.g. before gathering it to another GPU). */
int pbr_hip_wait_frame(pbr_hip_ctx* ctx, void* stream, int f);

/* ---- schedule (no reference counterpart) ----
 * How a frame is cut into launches on the device.  Every setting renders the same bits (the GPU
 * tests compare them with each other and with the reference); the defaults — a zeroed struct or
 * NULL — are the measured schedule of DESIGN.md §4.  The library reads no environment variables:
 * this call is the only run-time switch.  The setting holds for the context's later renders. */
enum pbr_kernels_mode {
    PBR_KERNELS_AUTO = 0,       /* the wavefront schedule wherever the integrator and scene allow it */
    PBR_KERNELS_MEGAKERNEL = 1  /* one kernel per frame, whole Li per lane */
};
enum pbr_fuse_mode {
    PBR_FUSE_AUTO = 0,          /* Whitted's level-0 shade traces its own camera rays in frames of at
                                 * least max(2, lanes) chunks (a separate camera kernel otherwise) */
    PBR_FUSE_OFF = 1,
    PBR_FUSE_ON = 2
};
typedef struct pbr_schedule {
    int kernels;                /* pbr_kernels_mode */
    int chunk_log2;             /* at most 2^chunk_log2 samples per chunk (10..28; 0 = the default: 25 for
                                 * Whitted, less with several lights; for Path / VolPath the largest of
                                 * 2^20..2^27 whose lanes' queues fit 3/4 of the device memory free or held
                                 * by the context); capped at 25 (Whitted) and 27 (Path / VolPath) */
    int lanes;                  /* chunk lanes, each its own stream and queues (1..4); 0 = 3 (Path: 4 where
                                 * four lanes of 2^27-sample chunks fit the memory share above) */
    int fuse_camera;            /* pbr_fuse_mode */
    int serial;                 /* 1: every launch of a frame on the caller's stream, one after another
                                 * (one lane, no shadow stream) — measures each kernel on its own */
} pbr_schedule;
int pbr_hip_set_schedule(pbr_hip_ctx* ctx, const pbr_schedule* sched);

/* ---- per-kernel profile (measurement; no reference counterpart) ----
 * While profiling is on, every kernel launch of a render is bracketed by a HIP event pair on the
 * stream it runs on, and each kernel family counts the work units it processed.  `bytes` is the
 * family's ALGORITHMIC HBM traffic: the compulsory queue / per-sample record / output bytes of the
 * wavefront design per counted unit — BVH, mesh and texture fetches, which the
 * caches serve, are not counted. */
typedef struct pbr_kernel_profile {
    char name[40];              /* kernel family, e.g. "k_wf_shade" (rocprof adds template args) */
    int launches;
    double ms;                  /* summed HIP-event durations of the family's launches */
    uint64_t units;             /* work units: samples (camera), queued rays, pixels (finish) */
    uint64_t bytes;             /* algorithmic HBM bytes */
    uint64_t counts[8];         /* raw counters: [0] units, [1..4] pushes / rays that got through */
} pbr_kernel_profile;
/* on = 1: start a measurement window of event timings; on = 2: timings and work counters (the
 * counters add one small counting launch after each queue kernel); 0: stop.  Either resets. */
int pbr_hip_set_profiling(pbr_hip_ctx* ctx, int on);
/* Waits for the context's work, returns the window's per-family profile (n = families seen; at most
 * `max` written) and starts a new window. */
int pbr_hip_get_profile(pbr_hip_ctx* ctx, pbr_kernel_profile* out, int max, int* n);

/* ---- introspection used by the parity tests (no reference counterpart) ---- */
/* Flattened BVH after upload: 32-B LinearBVHNode records (BVHAccel.cpp:46-55) and the ordered
 * primitive ids (position in the `prims` vector).  Pass NULL buffers to query counts. */
int pbr_hip_get_bvh(pbr_hip_ctx* ctx, void* nodes_out, int* n_nodes, int32_t* prim_ids_out, int* n_prims);
/* Halton/Sobol samples computed ON THE DEVICE for (pixel, sample, dim) triples. */
int pbr_hip_sampler_values(pbr_hip_ctx* ctx, int sampler, int width, int height, int spp,
                           int n, const int32_t* px_py_sample_dim, float* out);
/* GlobalSampler::GetIndexForSample (Sampler.h:69; Halton.cpp:61-81, pbrt-v3 SobolSampler) on the
 * device: px_py_sample = 3 ints per query, out = the 64-bit interval sample index. */
int pbr_hip_sample_index(pbr_hip_ctx* ctx, int sampler, int width, int height, int spp, int n,
                         const int32_t* px_py_sample, int64_t* out);
/* GlobalSampler::SampleDimension(index, dimension) (Sampler.h:70; Halton.cpp:83-92, pbrt-v3
 * SobolSampler, whose dimensions 0 and 1 are taken relative to the current pixel: px_py_dim = 3 ints
 * per query, pixel then dimension). */
int pbr_hip_sample_dimensions(pbr_hip_ctx* ctx, int sampler, int width, int height, int n, const int64_t* index,
                              const int32_t* px_py_dim, float* out);
/* Camera rays computed on the device for raster samples (pFilm.x, pFilm.y): out = o.xyz, d.xyz */
int pbr_hip_camera_rays(pbr_hip_ctx* ctx, const pbr_camera_desc* cam, int n, const float* pfilm, float* out);
/* Closest-hit queries on the device: rays = o.xyz d.xyz tmax; out = {hit, t, prim_id, b1, b2} as floats */
int pbr_hip_intersect(pbr_hip_ctx* ctx, int n, const float* rays, float* out, int any_hit);
/* ---- the reference's C++ query surface, batched (include/pbr/pbr.h builds on these) ---- */
/* SurfaceInteraction fields of a hit (Core/Interaction.h:56-105), as GeometricPrimitive::Intersect
 * leaves them (Primitive.cpp:22-36): t = the ray's new tMax. */
typedef struct pbr_surface_hit {
    int hit;                    /* 0 / 1 */
    int prim;                   /* index in the prims vector (shape order), -1 on a miss */
    float t;
    float b[3];                 /* barycentrics of the watertight test (triangles; 0 for spheres) */
    float p[3], p_error[3];
    float n[3];                 /* geometric normal (Triangle.cpp:197-206 orientation rules) */
    float ns[3], dpdu[3];       /* shading frame after the per-vertex normals */
    float wo[3];
    float uv[2];                /* surface (u, v) of the hit (Triangle.cpp:160-190; sphere: phi/phiMax, (theta-thetaMin)/range) */
    int medium_inside, medium_outside;   /* the primitive's MediumInterface (indices, -1 = none) */
} pbr_surface_hit;
/* Scene::Intersect (Core/Scene.cpp:20-24) or, with any_hit, IntersectP (:26-28) for n rays
 * (7 floats each: o.xyz, d.xyz, tMax).  prim >= 0 restricts the query to that one primitive
 * (GeometricPrimitive::Intersect / IntersectP, Core/Primitive.cpp:22-44).  Any-hit queries fill
 * only `hit`. */
int pbr_hip_query(pbr_hip_ctx* ctx, int n, const float* rays, int any_hit, int prim, pbr_surface_hit* out);
/* World bounds (lo.xyz, hi.xyz): prim = -1 → Scene::WorldBound (the BVH root, Scene.cpp:7-17);
 * prim >= 0 → GeometricPrimitive::WorldBound of that primitive (Primitive.cpp:18-20). */
int pbr_hip_bounds(pbr_hip_ctx* ctx, int prim, float* out6);
/* SamplerIntegrator::Li (Integrator.h:44) for n rays (7 floats each) on the device, with the
 * integrator / sampler / light strategy of `desc` (its tiles and outputs are ignored): each ray's
 * sampler is GlobalSampler-positioned at (pixel x, y; sample s) with its next dimension `dim`
 * (px_py_sample_dim: 4 ints per ray; dim 5 after GetCameraSample of a pinhole camera).  depth is
 * the recursion depth argument (Whitted).  rgb_out: 3 floats per ray. */
int pbr_hip_li(pbr_hip_ctx* ctx, const pbr_render_desc* desc, int n, const float* rays,
               const int32_t* px_py_sample_dim, int depth, float* rgb_out);

/* ---- BVH construction (BVHAccel::BVHAccel, Accelerator/BVHAccel.cpp:57-87; SAH recursiveBuild
 * :97-260; flattenBVHTree :262-283) ----
 * Both builders produce the reference's node array and orderedPrims exactly (the host one is the
 * sequential algorithm; the device one, pbr_bvh_build.hip, reproduces its partitions level by level). */
enum pbr_bvh_build { PBR_BVH_BUILD_HOST = 0, PBR_BVH_BUILD_DEVICE = 1 };
/* Which builder pbr_hip_upload_scene runs (default PBR_BVH_BUILD_DEVICE). */
int pbr_hip_set_bvh_build(pbr_hip_ctx* ctx, int where);
/* The last upload's build: builder, wall ms (device: incl. the bounds upload and node download),
 * device kernel ms (0 for the host builder). */
int pbr_hip_bvh_build_info(pbr_hip_ctx* ctx, int* where, double* ms, double* kernel_ms);
/* Standalone build over n primitive world bounds (6 floats each, lo.xyz hi.xyz, prims order:
 * GeometricPrimitive::WorldBound): nodes_out has room for 2n-1 32-B LinearBVHNodes, prim_ids_out for
 * n ids; ms_out (optional, 2 doubles) = {wall ms, device kernel ms}. */
int pbr_hip_build_bvh(pbr_hip_ctx* ctx, int where, int n, const float* prim_bounds, int max_prims,
                      void* nodes_out, int* n_nodes, int32_t* prim_ids_out, double* ms_out);

/* Device build info: ABI version, gfx arch string. */
int pbr_hip_abi_version(void);
const char* pbr_hip_build_info(void);
/* The built-in Sobol' generator matrices (SobolMatrices32 layout, dims × 52 uint32, dims <= 1024):
 * the reference's SobolMatrices32; host only. */
int pbr_hip_sobol_matrices(int dims, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* PBR_HIP_H */
