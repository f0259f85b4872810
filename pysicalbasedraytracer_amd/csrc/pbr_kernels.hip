// pbr_kernels.hip — MI355X (gfx950) render path: sampler, camera, Whitted/Path/VolPath integrators
// and the film, behind the C-ABI of include/pbr_hip.h.
//
// Work decomposition.  One lane traces one camera sample (pixel, sample index); a 256-lane
// workgroup owns a run of whole pixels (4 pixels × 64 spp at the 1080p config, i.e. one pixel per
// wave, which keeps primary rays and their shadow rays coherent inside a wave).  Per-sample
// radiance is staged in LDS and summed per pixel in sample order, so the float sum is
// bit-identical to the reference's `colObj += Li` loop (Integrator.cpp:303-313), then the output
// transform runs in the same kernel (no second pass over HBM).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <memory>
#include <string>
#include <vector>

#include "../../include/pbr_hip.h"
#include "pbr_device.h"
#include "pbr_scene.h"

using namespace pbr;

namespace {

// ---------------------------------------------------------------- sampler (Sampler/Sampler.cpp)
// index: the low 32 bits of the GlobalSampler's intervalSampleIndex (pbrt-v3 int64_t; Halton's stays
// below 2^32); px, py: the current pixel (Sobol dims 0/1 remap); sid: any number ≡ the sample
// number mod spp (the sample number, or the wavefront's per-chunk sample id, pixel-major), from
// which a Sobol index's bits >= 32 follow — (frame << 2m) | j has frame << 2m >> 32 above bit 31 —
// so they need no register or queue storage of their own
struct SState { uint32_t index; int dim; int px, py; int sid; };
struct SIndex { uint32_t lo, hi; };

__host__ __device__ __forceinline__ HaltonParams hparams(const DeviceSampler& s) {
    HaltonParams h;
    h.baseExp0 = s.baseExp0; h.baseExp1 = s.baseExp1; h.baseScale1 = s.baseScale1; h.stride = s.stride;
    h.mult0 = s.mult0; h.mult1 = s.mult1; h.scaleRatio0 = s.ratio0; h.scaleRatio1 = s.ratio1;
    return h;
}

// The low sampler dimensions a bounce loop samples over and over, staged in LDS by the kernels
// that ask for it (LDS = true).  Halton: one scrambled radical inverse is a chain of dependent
// digit-permutation lookups, and ds_read latency is a fraction of an L1/L2 round trip.  Sobol: the
// nibble tables of the first kLdsSobolDims dimensions (below).  One LDS array serves both.
constexpr int kLdsDims = 64;
constexpr int kLdsPermEntries = 8893;              // Σ of the first 64 primes
constexpr int kSobolNib = 128;                     // words per dimension: 8 nibble positions × 16
constexpr int kSobolNibHi = 80;                    // index bits 32..51: 5 nibble positions × 16
constexpr int kLdsSobolDims = 34;                  // 34 × 512 B fit the Halton permutation array
static_assert(kLdsSobolDims * kSobolNib * 4 <= kLdsPermEntries * 2, "Sobol LDS tables share the Halton array");
__shared__ __align__(16) uint16_t s_halton_perm[kLdsPermEntries];
__shared__ uint4 s_halton_tab[kLdsDims];           // prime, floor(2^32/prime), primeSums, 1/prime (float bits)
__shared__ float s_halton_tail[kLdsDims];          // invBase·perm[0] / (1 - invBase), the digit series' tail

__device__ __forceinline__ int sobol_lds_dims(const DeviceSampler& s) {
    return min(min(s.ldsDims, kLdsSobolDims), s.nSobolDims);
}
// Whole workgroup; call before the first LDS sample and follow with __syncthreads().  Inlined: an
// out-of-line call taking the sampler by reference makes the compiler copy the whole by-value kernel
// parameter block into per-lane scratch and read every parameter back from there.
__device__ __forceinline__ void stage_halton_lds(const DeviceSampler& s) {
    if (s.type == PBR_SAMPLER_TABLE) return;
    if (s.type == PBR_SAMPLER_SOBOL) {
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_halton_perm);
        const int n = sobol_lds_dims(s) * kSobolNib;
        for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = s.sobol[i];
        return;
    }
    const int nd = s.ldsDims;
    for (int i = threadIdx.x; i < nd; i += blockDim.x) {
        // ScrambledRadicalInverse's two per-call divisions (LowDiscrepancy.cpp:2302, :2314), formed once:
        // the same operations on the same values, so the same bits
        const float invBase = 1.f / (float)s.primes[i];
        s_halton_tab[i] = make_uint4(s.primes[i], s.recips[i], s.primeSums[i], __float_as_uint(invBase));
        s_halton_tail[i] = invBase * (float)s.perms[s.primeSums[i]] / (1 - invBase);
    }
    const int n = nd > 0 ? (int)(s.primeSums[nd - 1] + s.primes[nd - 1]) : 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s_halton_perm[i] = s.perms[i];
}

// pbrt-v3 SobolSampler::SampleDimension (Sobol.cpp) over SobolSampleFloat (LowDiscrepancy.h):
// XOR of the generator columns of the set index bits, v·2^-32 narrowed, dims 0/1 remapped into
// the pixel.  Dimensions beyond the matrices read 0 (pbrt aborts there).  The XOR over the 32
// index bits is regrouped by nibble (XOR is associative and commutative, so v is unchanged):
// T[8k + n] = XOR of columns 4k..4k+3 selected by n (prepare_sobol), eight independent lookups
// instead of a loop of up to 32 dependent column loads.
__device__ __forceinline__ uint32_t sobol_nibbles(const uint32_t* T, uint32_t index) {
    return T[index & 15u] ^ T[16 + ((index >> 4) & 15u)] ^ T[32 + ((index >> 8) & 15u)] ^ T[48 + ((index >> 12) & 15u)] ^
           T[64 + ((index >> 16) & 15u)] ^ T[80 + ((index >> 20) & 15u)] ^ T[96 + ((index >> 24) & 15u)] ^
           T[112 + (index >> 28)];
}
// index bits 32..51 (columns 32..51 of the 52-column matrices): five more nibble tables, read from
// global memory only when a sample's index needs them
__device__ __forceinline__ uint32_t sobol_nibbles_hi(const uint32_t* T, uint32_t hi) {
    return T[hi & 15u] ^ T[16 + ((hi >> 4) & 15u)] ^ T[32 + ((hi >> 8) & 15u)] ^ T[48 + ((hi >> 12) & 15u)] ^
           T[64 + ((hi >> 16) & 15u)];
}
// SobolSampler::SampleDimension for a 64-bit index (lo, hi): dimensions 0 and 1 relative to the pixel
template <bool LDS = false>
__device__ __forceinline__ float sobol_value(const DeviceSampler& s, uint32_t lo, uint32_t hi, int dim, int px, int py) {
    if (dim >= s.nSobolDims) return 0.f;
    uint32_t v;
    if (LDS && dim < sobol_lds_dims(s)) v = sobol_nibbles(reinterpret_cast<const uint32_t*>(s_halton_perm) + dim * kSobolNib, lo);
    else v = sobol_nibbles(s.sobol + (size_t)dim * kSobolNib, lo);
    if (hi) v ^= sobol_nibbles_hi(s.sobolHi + (size_t)dim * kSobolNibHi, hi);
    float f = mn((float)v * 2.3283064365386963e-10f, kOneMinusEpsilon);
    if (dim <= 1) {
        f = f * (float)s.sobolRes;   // + sampleBounds.pMin[dim] == 0
        f = clampf(f - (float)(dim == 0 ? px : py), 0.f, kOneMinusEpsilon);
    }
    return f;
}
template <bool LDS = false>
__device__ __forceinline__ float sobol_dimension(const DeviceSampler& s, uint32_t index, int sid, int dim, int px, int py) {
    // index bits 32..51: the frame's bits above 31 - 2m (spp is a power of two)
    const uint32_t hi = s.wideIndex ? ((uint32_t)sid & (uint32_t)(s.spp - 1)) >> s.hiShift : 0u;
    return sobol_value<LDS>(s, index, hi, dim, px, py);
}
// PBR_SAMPLER_TABLE: the caller's SampleDimension values (pbr_render_desc::sample_table); a
// dimension the table lacks fails the frame instead of reading past it
__device__ __forceinline__ float table_dimension(const DeviceSampler& s, uint32_t index, int dim) {
    if (dim < s.tableDims) return s.table[(size_t)index * s.tableDims + dim];
    atomicOr(s.guard, kGuardSampleTable);
    return 0.f;
}
// SobolIntervalToIndex (LowDiscrepancy.h) via the GF(2) tables of sobol_pixel_tables; the index is
// (frame << 2m) | j, 64-bit as pbrt-v3's (bits >= 32 come from the frame alone)
__device__ __forceinline__ SIndex sobol_index(const DeviceSampler& s, int px, int py, uint32_t frame) {
    const int m = s.sobolLog2Res;
    if (m == 0) return SIndex{0u, 0u};   // pbrt-v3 returns 0 here (a 1×1 raster repeats sample 0)
    const uint32_t* T = s.sobolPix;
    uint32_t delta = 0;
    for (int k = 0; (frame >> k) != 0u; ++k)
        if ((frame >> k) & 1u) delta ^= T[2 * m + k];
    uint32_t b = (((uint32_t)px << m) | (uint32_t)py) ^ delta, j = 0;
    for (int r = 0; b != 0; b >>= 1, ++r)
        if (b & 1u) j ^= T[r];
    const uint64_t idx = ((uint64_t)frame << (2 * m)) | j;
    return SIndex{(uint32_t)idx, (uint32_t)(idx >> 32)};
}
// GlobalSampler::StartPixel / SetSampleNumber: the global index of sample s of pixel (x, y)
// KIND: the sampler type when the caller knows it (the other types' code is compiled out), else -1
template <int KIND = -1>
__device__ __forceinline__ SIndex sample_index(const DeviceSampler& smp, int x, int y, int s) {
    if (KIND == PBR_SAMPLER_SOBOL || (KIND < 0 && smp.type == PBR_SAMPLER_SOBOL)) return sobol_index(smp, x, y, (uint32_t)s);
    if (KIND == PBR_SAMPLER_TABLE || (KIND < 0 && smp.type == PBR_SAMPLER_TABLE))   // the table row of (pixel, sample)
        return SIndex{((uint32_t)y * (uint32_t)smp.tableW + (uint32_t)x) * (uint32_t)smp.spp + (uint32_t)s, 0u};
    return SIndex{halton_pixel_offset(hparams(smp), x, y) + (uint32_t)s * (uint32_t)smp.stride, 0u};   // Halton.cpp:61-81
}

template <bool LDS = false, int KIND = -1>
__device__ __forceinline__ float sample_dimension(const DeviceSampler& s, uint32_t index, int sid, int dim, int px = 0, int py = 0) {
    if (KIND == PBR_SAMPLER_SOBOL || (KIND < 0 && s.type == PBR_SAMPLER_SOBOL)) return sobol_dimension<LDS>(s, index, sid, dim, px, py);
    if (KIND == PBR_SAMPLER_TABLE || (KIND < 0 && s.type == PBR_SAMPLER_TABLE)) return table_dimension(s, index, dim);
    // HaltonSampler::SampleDimension (Halton.cpp:83-92)
    if (dim == 0) return radical_inverse_2(index >> s.baseExp0);
    if (dim == 1) return radical_inverse_b(3u, 0x55555555u, div_prime(index, (uint32_t)s.baseScale1, 0xffffffffu / (uint32_t)s.baseScale1));
    if (dim >= 1000) return 0.f;
    if constexpr (LDS) {
        if (dim < s.ldsDims) {
            uint4 t = s_halton_tab[dim];
            return scrambled_radical_inverse_pre(t.x, t.y, s_halton_perm + t.z, index, __uint_as_float(t.w), s_halton_tail[dim]);
        }
    }
    return scrambled_radical_inverse(s.primes[dim], s.recips[dim], s.perms + s.primeSums[dim], index);
}
// GlobalSampler::Get1D/Get2D (Sampler.cpp:131-143): with no requested sample arrays
// arrayStartDim == arrayEndDim == 5, so only a Get2D that would straddle dimension 5 is moved.
template <bool LDS = false, int KIND = -1>
__device__ __forceinline__ float get1d(const DeviceSampler& s, SState& st) {
    if constexpr (PBR_DIAG_SHADE & 8) {   // diagnostic: a hash instead of the sampler
        uint32_t h = st.index * 0x9E3779B1u ^ (uint32_t)(st.dim++) * 0x85EBCA77u ^ (uint32_t)st.sid * 0xC2B2AE3Du;
        h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12;
        return (float)(h >> 8) * (1.f / 16777216.f);
    }
    return sample_dimension<LDS, KIND>(s, st.index, st.sid, st.dim++, st.px, st.py);
}
template <bool LDS = false, int KIND = -1>
__device__ __forceinline__ void get2d(const DeviceSampler& s, SState& st, float* a, float* b) {
    if (st.dim == 4) st.dim = 5;
    if constexpr (PBR_DIAG_SHADE & 8) { *a = get1d<LDS, KIND>(s, st); *b = get1d<LDS, KIND>(s, st); return; }
    *a = sample_dimension<LDS, KIND>(s, st.index, st.sid, st.dim, st.px, st.py);
    *b = sample_dimension<LDS, KIND>(s, st.index, st.sid, st.dim + 1, st.px, st.py);
    st.dim += 2;
}

// ---------------------------------------------------------------- camera (Perspective.cpp:44-80)
// PINHOLE: the caller knows lensRadius == 0 (the lens branch is compiled out)
template <bool PINHOLE = false>
__device__ __forceinline__ Ray camera_ray(const DeviceCamera& c, float fx, float fy, float l0, float l1) {
    f3 pCam = xf_point(c.rasterToCamera, mk(fx, fy, 0));
    f3 dir = normalize(pCam);
    Ray r = mkray(mk(0, 0, 0), dir, PBR_INF, -1);
    if (!PINHOLE && c.lensRadius > 0) {
        float dx, dy;
        concentric_disk(l0, l1, &dx, &dy);
        float lx = c.lensRadius * dx, ly = c.lensRadius * dy;
        float ft = c.focalDistance / r.d.z;
        f3 pFocus = r.o + r.d * ft;
        r.o = mk(lx, ly, 0);
        r.d = normalize(pFocus - r.o);
    }
    // CameraToWorld drops the medium (F12)
    return mkray(xf_point(c.cameraToWorld, r.o), xf_vector(c.cameraToWorld, r.d), r.tMax, -1);
}

struct KParams {
    DeviceScene S;
    DeviceSampler smp;
    DeviceCamera cam;
    int integrator, maxDepth;
    float rrThreshold;
    int spp, ppb;              // samples per pixel, pixels per workgroup
    long long nPixels;
    const int4* tiles;         // x0 y0 x1 y1
    const long long* tileStart;
    int nTiles;
    float* rgbOut;
    uint8_t* rgbaOut;
    unsigned long long* stats; // rays, nodes, prims, shading
};

// GetCameraSample (Sampler.cpp:10-21) + GenerateRay: pFilm = dims 0,1; time = dim 2 (no motion
// blur: never read); pLens = dims 3,4, read only by a camera with an aperture (lensRadius > 0), so
// a pinhole camera skips their scrambled radical inverses and only advances the dimension to 5.
template <bool PINHOLE = false, int KIND = -1>
__device__ __forceinline__ Ray camera_sample_ray(const KParams& P, SState& st, int x, int y) {
    float u0, u1, l0 = 0.f, l1 = 0.f;
    get2d<false, KIND>(P.smp, st, &u0, &u1);
    if (!PINHOLE && P.cam.lensRadius > 0) {
        get1d(P.smp, st);
        get2d(P.smp, st, &l0, &l1);
    } else {
        st.dim = 5;
    }
    return camera_ray<PINHOLE>(P.cam, (float)x + u0, (float)y + u1, l0, l1);
}

// ---------------------------------------------------------------- direct lighting (Integrator.cpp:46-177)
template <bool STATS>
__device__ bool unoccluded(const DeviceScene& S, const Isect& p0, const VisPt& p1, Counters* c) {   // Light.cpp:19-22
    Ray r = spawn_ray_to(p0, p1.p, p1.pError, p1.n);
    HitRec h;
    return !traverse<true, STATS>(S, r, &h, c);
}
template <bool STATS>
__device__ rgb vis_tr(const DeviceScene& S, const Isect& p0, const VisPt& p1, Counters* c) {   // Light.cpp:31-47
    Ray ray = spawn_ray_to(p0, p1.p, p1.pError, p1.n);
    rgb Tr = sp(1.f);
    for (int guard = 0;; ++guard) {
        Isect isect;
        bool hit = intersect<STATS>(S, ray, &isect, c);
        if (hit && S.primInfo[isect.slot].y >= 0) return sp(0.0f);
        if (ray.medium >= 0) Tr = Tr * medium_tr(S, ray.medium, ray);
        if (!hit) break;
        if (guard == kMaxTrCrossings) { atomicOr(S.guard, kGuardTransmittance); break; }
        ray = spawn_ray_to(isect, p1.p, p1.pError, p1.n);
    }
    return Tr;
}

template <bool STATS>
__device__ rgb estimate_direct(const KParams& P, const Isect& it, const BSDF* bsdf, float g, float uS0, float uS1, int li,
                               float uL0, float uL1, bool handleMedia, Counters* c) {
    const DeviceScene& S = P.S;
    const DLight& light = S.lights[li];
    const bool delta = light.type == LT_POINT;
    const int flags = BSDF_ALL & ~BSDF_SPECULAR;
    const bool surface = !is_zero(it.n);
    rgb Ld = sp(0.f);
    f3 wi = mk(0, 0, 0);
    float lightPdf = 0, scatteringPdf = 0;
    VisPt vis;
    rgb Li = sample_li(S, light, it, uL0, uL1, &wi, &lightPdf, &vis);
    if (lightPdf > 0 && !black(Li)) {
        rgb f;
        if (surface) {
            f = bsdf_f(*bsdf, it.wo, wi, flags) * absdot(wi, it.sn);
            scatteringPdf = bsdf_pdf(*bsdf, it.wo, wi, flags);
        } else {
            f = sp(phase_hg(dot(it.wo, wi), g));
        }
        if (!black(f)) {
            if (handleMedia) Li = Li * vis_tr<STATS>(S, it, vis, c);
            else if (!unoccluded<STATS>(S, it, vis, c)) Li = sp(0.f);
            if (!black(Li)) {
                if (delta) Ld = Ld + f * Li / lightPdf;
                else {
                    float fp = 1 * lightPdf, gp = 1 * scatteringPdf;
                    float weight = (fp * fp) / (fp * fp + gp * gp);
                    Ld = Ld + f * Li * weight / lightPdf;
                }
            }
        }
    }
    if (!delta) {
        rgb f;
        bool sampledSpecular = false;
        if (surface) {
            int st = 0;
            f = bsdf_sample(*bsdf, it.wo, &wi, uS0, uS1, &scatteringPdf, flags, &st);
            f = f * absdot(wi, it.sn);
            sampledSpecular = (st & BSDF_SPECULAR) != 0;
        } else {
            float p = hg_sample(g, it.wo, &wi, uS0, uS1);
            f = sp(p);
            scatteringPdf = p;
        }
        if (!black(f) && scatteringPdf > 0) {
            float weight = 1;
            if (!sampledSpecular) {
                lightPdf = pdf_li(S, light, it, wi);
                if (lightPdf == 0) return Ld;
                float fp = 1 * scatteringPdf, gp = 1 * lightPdf;
                weight = (fp * fp) / (fp * fp + gp * gp);
            }
            Isect lightIsect;
            Ray ray = spawn_ray(it, wi);
            bool found = intersect<STATS>(S, ray, &lightIsect, c);
            rgb Li2 = sp(0.f);
            if (found) {
                if (S.primInfo[lightIsect.slot].z == li) Li2 = si_Le(S, lightIsect, -wi);
            } else {
                Li2 = light_Le(S, light, ray);
            }
            if (!black(Li2)) Ld = Ld + f * Li2 * weight / scatteringPdf;
        }
    }
    return Ld;
}

// Distribution1D::SampleDiscrete over the lights (Sampling.h:96-107)
__device__ __forceinline__ int sample_light(const DeviceScene& S, float u, float* pdf) {
    int size = S.nLights + 1;
    int first = 0, len_ = size;
    while (len_ > 0) {
        int half = len_ >> 1, middle = first + half;
        if (S.lightCdf[middle] <= u) { first = middle + 1; len_ -= half + 1; }
        else len_ = half;
    }
    int off = clampi(first - 1, 0, size - 2);
    *pdf = (S.lightFuncInt > 0) ? S.lightFunc[off] / (S.lightFuncInt * S.nLights) : 0;
    return off;
}
template <bool STATS>
__device__ rgb uniform_sample_one_light(const KParams& P, const Isect& it, const BSDF* bsdf, float g, SState& st,
                                        bool handleMedia, Counters* c) {
    if (P.S.nLights == 0) return sp(0.f);
    float lightPdf;
    int li = sample_light(P.S, get1d(P.smp, st), &lightPdf);
    if (lightPdf == 0) return sp(0.f);
    float uL0, uL1, uS0, uS1;
    get2d(P.smp, st, &uL0, &uL1);
    get2d(P.smp, st, &uS0, &uS1);
    return estimate_direct<STATS>(P, it, bsdf, g, uS0, uS1, li, uL0, uL1, handleMedia, c) / lightPdf;
}

// ---------------------------------------------------------------- Whitted (WhittedIntegrator.cpp:11-65)
// The recursion L_k = A_k + ((f_k · L_{k+1}) · c_k) / pdf_k is unrolled into a bounded loop; the
// per-level terms are kept and folded back deepest-first so the float result equals the
// recursive evaluation.
constexpr int kMaxWhittedDepth = 64;   // pbr_hip_render rejects a deeper Whitted maxDepth
template <bool STATS>
__device__ rgb whitted_li(const KParams& P, Ray ray, SState& st, Counters* c) {
    const DeviceScene& S = P.S;
    rgb A[kMaxWhittedDepth], F[kMaxWhittedDepth];
    float CC[kMaxWhittedDepth], PD[kMaxWhittedDepth];
    int depth = 0;
    rgb Llast;
    for (int guard = 0;; ++guard) {
        Isect isect;
        if (!intersect<STATS>(S, ray, &isect, c)) {
            rgb L = sp(0.f);
            for (int i = 0; i < S.nLights; ++i) L = L + light_Le(S, S.lights[i], ray);
            Llast = L;
            break;
        }
        if (STATS) c->shading++;
        f3 n = isect.sn, wo = isect.wo;
        BSDF bsdf;
        MatTemplate texLocal;   // a textured material's per-hit lobes (make_bsdf)
        if (!make_bsdf<true>(S, S.materials, isect, false, &bsdf, &texLocal)) {
            if (guard > kMaxPassThrough) { atomicOr(S.guard, kGuardWhittedPassThrough); Llast = sp(0.f); break; }
            ray = spawn_ray(isect, ray.d);     // Li(isect.SpawnRay(ray.d), depth)
            continue;
        }
        rgb L = sp(0.f);
        L = L + si_Le(S, isect, wo);
        for (int i = 0; i < S.nLights; ++i) {
            f3 wi;
            float pdf;
            VisPt vis;
            float u0, u1;
            get2d(P.smp, st, &u0, &u1);
            rgb Li = sample_li(S, S.lights[i], isect, u0, u1, &wi, &pdf, &vis);
            if (black(Li) || pdf == 0) continue;
            rgb f = bsdf_f(bsdf, wo, wi, BSDF_ALL);
            if (!black(f) && unoccluded<STATS>(S, isect, vis, c)) L = L + f * Li * absdot(wi, n) / pdf;
        }
        if (depth + 1 < P.maxDepth && depth + 1 < kMaxWhittedDepth) {   // SpecularReflect (Integrator.cpp:179-222)
            f3 wi = mk(0, 0, 0);
            float pdf = 0;
            int stype = 0;
            float u0, u1;
            get2d(P.smp, st, &u0, &u1);
            rgb f = bsdf_sample(bsdf, wo, &wi, u0, u1, &pdf, BSDF_REFLECTION | BSDF_SPECULAR, &stype);
            if (!black(f) && pdf > 0.f && absdot(wi, isect.sn) != 0.f) {
                A[depth] = L; F[depth] = f; CC[depth] = absdot(wi, isect.sn); PD[depth] = pdf;
                ray = spawn_ray(isect, wi);
                ++depth;
                continue;
            }
        }
        Llast = L + sp(0.f);
        break;
    }
    for (int k = depth - 1; k >= 0; --k) Llast = A[k] + F[k] * Llast * CC[k] / PD[k];
    return Llast;
}

// ---------------------------------------------------------------- Path (PathIntegrator.cpp:32-110)
template <bool STATS>
__device__ rgb path_li(const KParams& P, Ray ray, SState& st, Counters* c) {
    const DeviceScene& S = P.S;
    rgb L = sp(0.f), beta = sp(1.f);
    bool specularBounce = false;
    float etaScale = 1;
    for (int bounces = 0;; ++bounces) {
        Isect isect;
        bool found = intersect<STATS>(S, ray, &isect, c);
        if (bounces == 0 || specularBounce) {
            if (found) L = L + beta * si_Le(S, isect, -ray.d);
            else for (int i = 0; i < S.nInfinite; ++i) L = L + beta * light_Le(S, S.lights[S.infinite[i]], ray);
        }
        if (!found || bounces >= P.maxDepth) break;
        if (STATS) c->shading++;
        BSDF bsdf;
        MatTemplate texLocal;   // a textured material's per-hit lobes (make_bsdf)
        if (!make_bsdf<true>(S, S.materials, isect, true, &bsdf, &texLocal)) { ray = spawn_ray(isect, ray.d); bounces--; continue; }
        if (num_components(bsdf, BSDF_ALL & ~BSDF_SPECULAR) > 0) {
            rgb Ld = beta * uniform_sample_one_light<STATS>(P, isect, &bsdf, 0.f, st, false, c);
            L = L + Ld;
        }
        f3 wo = -ray.d, wi = mk(0, 0, 0);
        float pdf = 0;
        int flags = 0;
        float u0, u1;
        get2d(P.smp, st, &u0, &u1);
        rgb f = bsdf_sample(bsdf, wo, &wi, u0, u1, &pdf, BSDF_ALL, &flags);
        if (black(f) || pdf == 0.f) break;
        beta = beta * (f * absdot(wi, isect.sn) / pdf);
        specularBounce = (flags & BSDF_SPECULAR) != 0;
        if ((flags & BSDF_SPECULAR) && (flags & BSDF_TRANSMISSION)) {
            float eta = bsdf.mt->eta;
            etaScale *= (dot(wo, isect.n) > 0) ? (eta * eta) : 1 / (eta * eta);
        }
        ray = spawn_ray(isect, wi);
        rgb rrBeta = beta * etaScale;
        if (maxval(rrBeta) < P.rrThreshold && bounces > 3) {
            float q = mx((float).05, 1 - maxval(rrBeta));
            if (get1d(P.smp, st) < q) break;
            beta = beta / (1 - q);
        }
    }
    return L;
}

// ---------------------------------------------------------------- VolPath (VolPathIntegrator.cpp:21-107)
template <bool STATS>
__device__ rgb volpath_li(const KParams& P, Ray ray, SState& st, Counters* c) {
    const DeviceScene& S = P.S;
    rgb L = sp(0.f), beta = sp(1.f);
    bool specularBounce = false;
    float etaScale = 1;
    for (int bounces = 0;; ++bounces) {
        Isect isect;
        bool found = intersect<STATS>(S, ray, &isect, c);
        bool mediumEvent = false;
        Isect mi;
        float g = 0;
        if (ray.medium >= 0) {   // HomogeneousMedium::Sample (HomogeneousMedium.cpp:15-45)
            const float* md = S.media + 10 * ray.medium;
            int channel = (int)(get1d(P.smp, st) * 3);
            if (channel > 2) channel = 2;
            float dist = -t_log(1 - get1d(P.smp, st)) / md[6 + channel];
            float t = mn(dist / len(ray.d), ray.tMax);
            bool sampled = t < ray.tMax;
            if (sampled) {
                mi.p = ray.o + ray.d * t; mi.wo = -ray.d; mi.n = mk(0, 0, 0); mi.pError = mk(0, 0, 0);
                mi.medIn = mi.medOut = ray.medium; mi.slot = -1;
                g = md[9];
                mediumEvent = true;
            }
            rgb Tr = exp_s(sp3(-md[6], -md[7], -md[8]) * mn(t, kMaxFloat) * len(ray.d));
            rgb density = sampled ? (sp3(md[6], md[7], md[8]) * Tr) : Tr;
            float pdf = 0;
            pdf += density.r; pdf += density.g; pdf += density.b;
            pdf *= 1 / (float)3;
            if (pdf == 0) pdf = 1;
            beta = beta * (sampled ? (Tr * sp3(md[3], md[4], md[5]) / pdf) : (Tr / pdf));
        }
        if (black(beta)) break;
        if (mediumEvent) {
            if (bounces >= P.maxDepth) break;
            if (STATS) c->shading++;
            L = L + beta * uniform_sample_one_light<STATS>(P, mi, nullptr, g, st, true, c);
            f3 wo = -ray.d, wi;
            float u0, u1;
            get2d(P.smp, st, &u0, &u1);
            hg_sample(g, wo, &wi, u0, u1);
            ray = spawn_ray(mi, wi);
            specularBounce = false;
        } else {
            if (bounces == 0 || specularBounce) {
                if (found) L = L + beta * si_Le(S, isect, -ray.d);
                else for (int i = 0; i < S.nInfinite; ++i) L = L + beta * light_Le(S, S.lights[S.infinite[i]], ray);
            }
            if (!found || bounces >= P.maxDepth) break;
            if (STATS) c->shading++;
            BSDF bsdf;
            MatTemplate texLocal;   // a textured material's per-hit lobes (make_bsdf)
            if (!make_bsdf<true>(S, S.materials, isect, true, &bsdf, &texLocal)) { ray = spawn_ray(isect, ray.d); bounces--; continue; }
            L = L + beta * uniform_sample_one_light<STATS>(P, isect, &bsdf, 0.f, st, true, c);
            f3 wo = -ray.d, wi = mk(0, 0, 0);
            float pdf = 0;
            int flags = 0;
            float u0, u1;
            get2d(P.smp, st, &u0, &u1);
            rgb f = bsdf_sample(bsdf, wo, &wi, u0, u1, &pdf, BSDF_ALL, &flags);
            if (black(f) || pdf == 0.f) break;
            beta = beta * (f * absdot(wi, isect.sn) / pdf);
            specularBounce = (flags & BSDF_SPECULAR) != 0;
            if ((flags & BSDF_SPECULAR) && (flags & BSDF_TRANSMISSION)) {
                float eta = bsdf.mt->eta;
                etaScale *= (dot(wo, isect.n) > 0) ? (eta * eta) : 1 / (eta * eta);
            }
            ray = spawn_ray(isect, wi);
        }
        rgb rrBeta = beta * etaScale;
        if (maxval(rrBeta) < P.rrThreshold && bounces > 3) {
            float q = mx((float).05, 1 - maxval(rrBeta));
            if (get1d(P.smp, st) < q) break;
            beta = beta / (1 - q);
        }
    }
    return L;
}

__device__ __forceinline__ void pixel_xy(const KParams& P, long long q, int* x, int* y) {
    int lo = 0, hi = P.nTiles - 1;
    while (lo < hi) {   // last tile with start <= q
        int mid = (lo + hi + 1) >> 1;
        if (P.tileStart[mid] <= q) lo = mid; else hi = mid - 1;
    }
    int4 t = P.tiles[lo];
    long long local = q - P.tileStart[lo];
    int w = t.z - t.x;
    *x = t.x + (int)(local % w);
    *y = t.y + (int)(local / w);
}

// Output transform (Integrator.cpp:313-344): average, XYZ round trip, sRGB gamma, 8-bit.
__device__ __forceinline__ void film_out(const KParams& P, long long q, rgb col) {
    col = col / (float)P.spp;
    if (P.rgbOut) { P.rgbOut[3 * q] = col.r; P.rgbOut[3 * q + 1] = col.g; P.rgbOut[3 * q + 2] = col.b; }
    if (P.rgbaOut) {
        float X = 0.412453f * col.r + 0.357580f * col.g + 0.180423f * col.b;
        float Y = 0.212671f * col.r + 0.715160f * col.g + 0.072169f * col.b;
        float Z = 0.019334f * col.r + 0.119193f * col.g + 0.950227f * col.b;
        float o[3];
        o[0] = 3.240479f * X - 1.537150f * Y - 0.498535f * Z;
        o[1] = -0.969256f * X + 1.875991f * Y + 0.041556f * Z;
        o[2] = 0.055648f * X - 0.204043f * Y + 1.057311f * Z;
        uint32_t packed = 0xff000000u;
        for (int k = 0; k < 3; ++k) {
            float v = o[k];
            float gc = (v <= 0.0031308f) ? 12.92f * v : 1.055f * t_pow(v, (1.f / 2.4f)) - 0.055f;
            float b = clampf(255.f * gc + 0.5f, 0.f, 255.f);
            packed |= ((uint32_t)(int)b & 0xffu) << (8 * k);
        }
        reinterpret_cast<uint32_t*>(P.rgbaOut)[q] = packed;
    }
}

template <int INTEGRATOR, bool STATS, int OCC>
__global__ __launch_bounds__(256, OCC) void k_render(KParams P) {
    __shared__ float lds[256 * 3];
    const int tid = threadIdx.x;
    const long long pixBase = (long long)blockIdx.x * P.ppb;
    long long rem = P.nPixels - pixBase;
    const int npix = rem < P.ppb ? (int)rem : P.ppb;
    if (npix <= 0) return;
    const int spp = P.spp;
    const int total = npix * spp;
    Counters cnt = {0, 0, 0, 0};
    rgb acc = sp(0.0f);
    for (int base = 0; base < total; base += 256) {
        int slot = base + tid;
        rgb L = sp(0.f);
        if (slot < total) {
            int lp = slot / spp, s = slot - lp * spp;
            int x, y;
            pixel_xy(P, pixBase + lp, &x, &y);
            // GlobalSampler::StartPixel/SetSampleNumber (Sampler.cpp:97-130)
            SState st;
            st.index = sample_index(P.smp, x, y, s).lo;
            st.sid = s;
            st.dim = 0;
            st.px = x;
            st.py = y;
            // GetCameraSample (Sampler.cpp:10-21): pFilm, time, pLens
            Ray r = camera_sample_ray(P, st, x, y);
            if (INTEGRATOR == PBR_INTEGRATOR_WHITTED) L = whitted_li<STATS>(P, r, st, &cnt);
            else if (INTEGRATOR == PBR_INTEGRATOR_PATH) L = path_li<STATS>(P, r, st, &cnt);
            else L = volpath_li<STATS>(P, r, st, &cnt);
        }
        lds[3 * tid] = L.r; lds[3 * tid + 1] = L.g; lds[3 * tid + 2] = L.b;
        __syncthreads();
        if (tid < npix) {
            int lo = tid * spp > base ? tid * spp : base;
            int hi = (tid + 1) * spp < base + 256 ? (tid + 1) * spp : base + 256;
            for (int k = lo; k < hi; ++k) {
                int j = k - base;
                acc = acc + sp3(lds[3 * j], lds[3 * j + 1], lds[3 * j + 2]);
            }
        }
        __syncthreads();
    }
    if (tid < npix) film_out(P, pixBase + tid, acc);
    if (STATS) {
        atomicAdd(&P.stats[0], (unsigned long long)cnt.rays);
        atomicAdd(&P.stats[1], (unsigned long long)cnt.nodes);
        atomicAdd(&P.stats[2], (unsigned long long)cnt.prims);
        atomicAdd(&P.stats[3], (unsigned long long)cnt.shading);
    }
}

#include "pbr_wavefront.h"
#include "pbr_wavefront_path.h"
#include "pbr_wavefront_volpath.h"

// ---------------------------------------------------------------- introspection kernels
__global__ void k_sampler_values(DeviceSampler smp, HaltonParams hp, int n, const int32_t* q, float* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SIndex idx = sample_index(smp, q[4 * i], q[4 * i + 1], q[4 * i + 2]);
    out[i] = sample_dimension(smp, idx.lo, q[4 * i + 2], q[4 * i + 3], q[4 * i], q[4 * i + 1]);
}
// GlobalSampler::GetIndexForSample / SampleDimension for (pixel, sample) and (index, pixel, dim) queries
__global__ void k_sample_index(DeviceSampler smp, int n, const int32_t* q, long long* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int x = q[3 * i], y = q[3 * i + 1], s = q[3 * i + 2];
    if (smp.type == PBR_SAMPLER_SOBOL) {
        const SIndex k = sobol_index(smp, x, y, (uint32_t)s);
        out[i] = (long long)(((uint64_t)k.hi << 32) | k.lo);
    } else {   // Halton.cpp:61-81 in 64 bits: offsetForCurrentPixel + sampleNum * sampleStride
        out[i] = (long long)((uint64_t)halton_pixel_offset(hparams(smp), x, y) + (uint64_t)s * (uint64_t)smp.stride);
    }
}
__global__ void k_sample_dimensions(DeviceSampler smp, int n, const long long* idx, const int32_t* q, float* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t index = (uint64_t)idx[i];
    const int px = q[3 * i], py = q[3 * i + 1], dim = q[3 * i + 2];
    if (smp.type == PBR_SAMPLER_SOBOL) out[i] = sobol_value(smp, (uint32_t)index, (uint32_t)(index >> 32), dim, px, py);
    else out[i] = sample_dimension(smp, (uint32_t)index, 0, dim, px, py);
}
__global__ void k_camera_rays(DeviceCamera cam, int n, const float* pf, float* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r = camera_ray(cam, pf[2 * i], pf[2 * i + 1], 0.5f, 0.5f);
    out[6 * i] = r.o.x; out[6 * i + 1] = r.o.y; out[6 * i + 2] = r.o.z;
    out[6 * i + 3] = r.d.x; out[6 * i + 4] = r.d.y; out[6 * i + 5] = r.d.z;
}
__global__ void k_intersect(DeviceScene S, const int32_t* primIds, int n, const float* rays, float* out, int any) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* rr = rays + 7 * i;
    Ray r = mkray(mk(rr[0], rr[1], rr[2]), mk(rr[3], rr[4], rr[5]), rr[6], -1);
    HitRec h;
    Counters c;
    float* o = out + 5 * i;
    if (any) {
        o[0] = traverse<true, false>(S, r, &h, &c) ? 1.f : 0.f;
        o[1] = o[2] = o[3] = o[4] = 0.f;
    } else {
        bool hit = traverse<false, false>(S, r, &h, &c);
        o[0] = hit ? 1.f : 0.f;
        o[1] = hit ? r.tMax : 0.f;
        o[2] = hit ? (float)primIds[h.slot] : -1.f;
        o[3] = hit ? h.b1 : 0.f;
        o[4] = hit ? h.b2 : 0.f;
    }
}

// Scene::Intersect / IntersectP (or one primitive's GeometricPrimitive::Intersect / IntersectP when
// slotOnly >= 0) with the SurfaceInteraction fields of the hit (pbr_hip_query).
__global__ void k_query(DeviceScene S, const int32_t* primIds, int n, const float* rays, int any, int slotOnly,
                        pbr_surface_hit* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* rr = rays + 7 * i;
    Ray r = mkray(mk(rr[0], rr[1], rr[2]), mk(rr[3], rr[4], rr[5]), rr[6], -1);
    pbr_surface_hit o;
    memset(&o, 0, sizeof(o));
    o.prim = -1;
    o.medium_inside = o.medium_outside = -1;
    HitRec h;
    h.slot = -1; h.b0 = h.b1 = h.b2 = 0.f;
    bool hit;
    if (slotOnly >= 0) {   // GeometricPrimitive::Intersect: the shape's test against ray.tMax
        float t = 0.f;
        hit = prim_hit(S, slotOnly, r, &t, &h.b0, &h.b1, &h.b2);
        if (hit && !any) { r.tMax = t; h.slot = slotOnly; }
    } else {
        Counters c;
        hit = any ? traverse<true, false>(S, r, &h, &c) : traverse<false, false>(S, r, &h, &c);
    }
    o.hit = hit ? 1 : 0;
    if (hit && !any) {
        const int flags = __float_as_int(S.triVerts[3 * (size_t)h.slot].w);
        Isect si;
        if (flags & PRIM_SPHERE) {
            const SphereRec& sph = S.spheres[__float_as_int(S.triVerts[3 * (size_t)h.slot].x)];
            sphere_si(sph, r, r.tMax, &si);
            // pbrt-v3 Sphere::Intersect's (u, v): phi / phiMax, (theta - thetaMin) / (thetaMax - thetaMin)
            f3 ob = xf_point(sph.w2o, r.o), db = xf_vector(sph.w2o, r.d);
            f3 ph = ob + db * r.tMax;
            ph = ph * (sph.radius / len(ph));
            if (ph.x == 0 && ph.y == 0) ph.x = 1e-5f * sph.radius;
            float phi = t_atan2(ph.y, ph.x);
            if (phi < 0) phi += 2 * kPi;
            const float theta = t_acos(clampf(ph.z / sph.radius, -1, 1));
            o.uv[0] = phi / (2 * kPi);
            o.uv[1] = (theta - kPi) / (0.f - kPi);
        } else {
            triangle_si(S, h.slot, r, h.b0, h.b1, h.b2, flags, &si);
            float u0x = 0, u0y = 0, u1x = 1, u1y = 0, u2x = 1, u2y = 1;   // Triangle::GetUVs default
            if (flags & PRIM_HAS_UV) {
                const float2* uv = S.triUV + 3 * (size_t)h.slot;
                u0x = uv[0].x; u0y = uv[0].y; u1x = uv[1].x; u1y = uv[1].y; u2x = uv[2].x; u2y = uv[2].y;
            }
            o.uv[0] = h.b0 * u0x + h.b1 * u1x + h.b2 * u2x;   // Triangle.cpp:170
            o.uv[1] = h.b0 * u0y + h.b1 * u1y + h.b2 * u2y;
        }
        const int4 info = S.primInfo[h.slot];
        o.prim = primIds[h.slot];
        o.t = r.tMax;
        o.b[0] = h.b0; o.b[1] = h.b1; o.b[2] = h.b2;
        o.p[0] = si.p.x; o.p[1] = si.p.y; o.p[2] = si.p.z;
        o.p_error[0] = si.pError.x; o.p_error[1] = si.pError.y; o.p_error[2] = si.pError.z;
        o.n[0] = si.n.x; o.n[1] = si.n.y; o.n[2] = si.n.z;
        o.ns[0] = si.sn.x; o.ns[1] = si.sn.y; o.ns[2] = si.sn.z;
        o.dpdu[0] = si.dpdu.x; o.dpdu[1] = si.dpdu.y; o.dpdu[2] = si.dpdu.z;
        o.wo[0] = si.wo.x; o.wo[1] = si.wo.y; o.wo[2] = si.wo.z;
        o.medium_inside = (int)(short)(info.w & 0xffff);
        o.medium_outside = (int)(short)((info.w >> 16) & 0xffff);
    }
    out[i] = o;
}

// SamplerIntegrator::Li for caller-given rays (pbr_hip_li): each ray's sampler positioned at
// (pixel, sample) with its next dimension given.
template <int INTEGRATOR>
__global__ void k_li(KParams P, int n, const float* rays, const int32_t* q, float* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* rr = rays + 7 * i;
    Ray r = mkray(mk(rr[0], rr[1], rr[2]), mk(rr[3], rr[4], rr[5]), rr[6], -1);   // camera rays carry no medium (F12)
    SState st;
    st.index = sample_index(P.smp, q[4 * i], q[4 * i + 1], q[4 * i + 2]).lo;
    st.sid = q[4 * i + 2];
    st.dim = q[4 * i + 3];
    st.px = q[4 * i];
    st.py = q[4 * i + 1];
    Counters c = {0, 0, 0, 0};
    rgb L;
    if (INTEGRATOR == PBR_INTEGRATOR_WHITTED) L = whitted_li<false>(P, r, st, &c);
    else if (INTEGRATOR == PBR_INTEGRATOR_PATH) L = path_li<false>(P, r, st, &c);
    else L = volpath_li<false>(P, r, st, &c);
    out[3 * i] = L.r; out[3 * i + 1] = L.g; out[3 * i + 2] = L.b;
}

// Profiling: adds the sums of up to kProfFields segment-count arrays (kWfBlocks ints each) to the
// counter row dst[0..]; one workgroup, launched after the kernel it counts (outside its events).
struct ProfSums {
    const int* seg[kProfFields];
    unsigned long long* dst;
};
__global__ __launch_bounds__(256) void k_prof_count(ProfSums a) {
    for (int k = 0; k < kProfFields; ++k) {
        if (!a.seg[k]) continue;
        unsigned long long v = 0;
        for (int i = threadIdx.x; i < kWfBlocks; i += 256) v += (unsigned long long)a.seg[k][i];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(a.dst + k, v);
    }
}

}  // namespace

// ======================================================================== C-ABI
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t ensure(size_t n) {
        if (n <= bytes && p) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; bytes = 0; }
        hipError_t e = hipMalloc(&p, n ? n : 16);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    template <class T> hipError_t upload(const std::vector<T>& v, hipStream_t s) {
        hipError_t e = ensure(v.size() * sizeof(T));
        if (e != hipSuccess || v.empty()) return e;
        return hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
    }
};

// Wavefront queues, per-sample state and records of one chunk lane (pbr_wavefront*.h).
struct WfBufs {
    DevBuf wqO[2], wqD[2], wqId[2], wqHit[2], wsO, wsD, wsC, wsId, wRecA, wRecF, wRecP, wDepth, wIndex, wCnt;
    DevBuf wsO2, wsD2, wsC2, wsId2;   // Whitted: second shadow queue (levels alternate)
    DevBuf wsW, wsW2;                 // Whitted under a SkyBox: the shadow entries' directions
    DevBuf wRecC, wRecV;              // multi-light Whitted: per-light contributions, visibility
    // wavefront Path (pbr_wavefront_path.h): probe + direct queues, per-sample state and records
    DevBuf wqS0[2], wqS1[2];          // Path/VolPath: the path state carried with the ray
    DevBuf wPassList, wPassCnt;       // the classed Path shade: passes 1..'s queue positions, counts
    DevBuf wpO, wpD, wpId, sL, rA, rB, rBeta, rLi, rFlags, rLight, rTgt;
    DevBuf wtO, wtD, wtP, wtE, wtN, wtId, rLiA, rTr, rWA;   // VolPath transmittance walk
};
// Chunks alternate between two lanes (own buffers, own stream) so one chunk's launch tails overlap
// the other's work — what keeps a small per-GPU shard of a multi-GPU frame efficient.
// Lanes a frame may use (pbr_schedule::lanes), and the default.  Measured (frame ms, bit-identical):
// C2 2 lanes 17.73-17.80, 3: 17.49, 4: 17.97 (4 lanes of 2^24-sample chunks 19.10); C3 268.7 /
// 267.3 / 274.9; C5 1396 / 1379 / 1414.
constexpr int kWfLanes = 4;
#ifndef PBR_LANES_DEFAULT
#define PBR_LANES_DEFAULT 3
#endif
constexpr int kWfDefaultLanes = PBR_LANES_DEFAULT;

struct pbr_hip_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    bool haveScene = false;
    HostScene host;
    HaltonTables halton;
    DevBuf dInfTex, dInfCF, dInfCC, dInfMF, dInfMC, dInfRec;
    DevBuf dTexels, dTextures, dTexMats;   // ImageTextures and the textured materials' parameters
    DevBuf dNodes, dWide, dQuad, dTri, dInfo, dUV, dSph, dMat, dLights, dEnv, dCdf, dFunc, dMedia;
    DevBuf dPrimes, dRecips, dPrimeSums, dPerms, dPrimIds;
    DevBuf dSobol, dSobolHi, dSobolPix;  // active Sobol nibble tables (index bits 0-31, 32-51), pixel tables
    std::vector<uint32_t> sobolBuiltin;
    uint64_t sobolKey = 0;               // FNV-1a of the matrices dSobol was built from
    int sobolSrcDims = 0, sobolPixM = -1;
    DevBuf dTiles, dTileStart, dRgb, dRgba, dStats, dScratchIn, dScratchOut;
    DevBuf dTable;                       // PBR_SAMPLER_TABLE values of the current frame
    std::vector<int32_t> tilesHost;      // what dTiles / dTileStart hold (re-uploaded on change only)
    DevBuf dMatPass;                     // the classed Path shade: each material's pass
    std::vector<int32_t> matPassHost;
    std::vector<long long> startsHost;
    hipStream_t lastStream = nullptr;    // stream of the last asynchronous render (may still run)
    bool inFlight = false;
    // wavefront buffers of the two chunk lanes, and the lane-1 stream with its fork/join events
    WfBufs wb[kWfLanes];
    hipStream_t side[kWfLanes] = {};     // lanes 1.. (lane 0: the caller's stream, or ctx->stream — wf_fork)
    hipStream_t lane0 = nullptr;         // lane 0's stream in the current frame or batch (wf_fork)
    hipEvent_t evFork = nullptr, evJoin[kWfLanes] = {};
    struct FrameEv {                     // a batch: the end of frame f's last chunk on each lane it used
        hipEvent_t ev[kWfLanes] = {};
        unsigned used = 0;
    };
    std::vector<FrameEv> frameEv;        // (pbr_hip_wait_frame)
    int batchFrames = 0;                 // frames of the last batch
    // Whitted: per lane, a stream for the shadow rays and per-level events (shade done, shadow done)
    hipStream_t shadowStream[kWfLanes] = {};
    hipEvent_t evShade[kWfLanes][kWfMaxDepth + 2] = {}, evShadow[kWfLanes][kWfMaxDepth + 2] = {};
    int curStrategy = PBR_LIGHTS_UNIFORM;
    float funcInt = 0;
    pbr_schedule sched = {};             // pbr_hip_set_schedule (zero = the measured defaults)
    // per-kernel profile (pbr_hip_set_profiling): a HIP event pair around every launch, on the
    // launch's stream, and the work counters of each kernel family (device rows + host-known counts)
    bool profOn = false, profCount = false;
    struct ProfEv { int kind; hipEvent_t a, b; };
    std::vector<ProfEv> profEv;
    size_t profUsed = 0;
    DevBuf dProf;
    unsigned long long profHost[KP_COUNT][kProfFields] = {};
    int bvhBuild = PBR_BVH_BUILD_DEVICE; // which SAH builder pbr_hip_upload_scene runs
    double bvhMs = 0, bvhKernelMs = 0;   // the last upload's BVH build: wall / device time
    int bvhWhereLast = PBR_BVH_BUILD_HOST;   // ... and where it ran (Middle / EqualCounts: always the host)
    DevBuf dGuard;                       // DeviceScene::guard (kGuard* bits of tripped safety bounds)
    int* guardHost = nullptr;            // pinned copy, refreshed at the end of every frame
    hipEvent_t evGuard = nullptr;        // recorded after the last frame's guard copy, on that frame's stream
    bool guardPending = false;           // that copy may still be in flight: guardHost is read once it landed
};

namespace {

// Lobe kinds the scene's BSDFs can hold (selects the shading kernels' specialisation); a textured
// material's lobes are built per hit, so it may produce any kind.
int scene_lobe_kinds(const HostScene& h) {
    int lobes = 0;
    for (const MatTemplate& m : h.materials) {
        if (m.textured) lobes |= kAllLobes | kTexturedLobes;
        for (int i = 0; i < m.nLobes; ++i) lobes |= 1 << m.lobes[i].kind;
    }
    return lobes;
}

int set_err(pbr_hip_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}
#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return set_err(ctx, PBR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Wait for an asynchronous render still reading the context's buffers (see pbr_hip_render).
int drain(pbr_hip_ctx* ctx) {
    if (ctx->inFlight) HIP_TRY(hipStreamSynchronize(ctx->lastStream));
    ctx->inFlight = false;
    return PBR_OK;
}

// Every stream of the context idle: the caller's stream, the lane-1 stream and the shadow streams.
// Used after a schedule fails part-way (a side lane may still write lane buffers, dGuard or dProf)
// and where profiling state is reset or read — instead of a device-wide synchronisation, which
// would stall other contexts sharing the GPU.
void quiesce(pbr_hip_ctx* ctx, hipStream_t s) {
    if (s) (void)hipStreamSynchronize(s);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (int l = 0; l < kWfLanes; ++l)
        if (ctx->side[l]) (void)hipStreamSynchronize(ctx->side[l]);
    for (int l = 0; l < kWfLanes; ++l)
        if (ctx->shadowStream[l]) (void)hipStreamSynchronize(ctx->shadowStream[l]);
    ctx->inFlight = false;
}

// A frame whose walk reached a safety bound fails instead of returning a truncated image.  Frames
// that can trip one (scenes with material-less primitives) copy the flag to pinned memory at their
// end; synchronous renders check it before returning, asynchronous ones at the next call.
// The caller has made ctx->device current and drained the context (the pinned copy of an
// asynchronous frame lands only when that frame ends); the reset is ordered on the context's stream.
// The copy of an asynchronous frame is read only once its event has completed (a copy still in
// flight is checked by a later call or pbr_hip_sync, which drains first).  A tripped bit is reset on
// the context's stream ordered after that copy, and guardHost is cleared only after the reset has
// run, so no copy queued before it can land later and fail an unrelated frame.
int check_guard(pbr_hip_ctx* ctx) {
    if (ctx->guardPending) {
        const hipError_t q = hipEventQuery(ctx->evGuard);
        if (q == hipErrorNotReady) return PBR_OK;
        HIP_TRY(q);
        ctx->guardPending = false;
    }
    const int g = ctx->guardHost ? *(volatile int*)ctx->guardHost : 0;
    if (!g) return PBR_OK;
    HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->evGuard, 0));
    HIP_TRY(hipMemsetAsync(ctx->dGuard.p, 0, sizeof(int), ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    *ctx->guardHost = 0;
    std::string what;
    if (g & kGuardWhittedPassThrough) what += "a Whitted path crossed more than 1024 material-less surfaces; ";
    if (g & kGuardTransmittance) what += "a transmittance walk crossed more than 256 medium interfaces; ";
    if (g & kGuardStack) what += "a BVH traversal stack was full; ";
    if (g & kGuardSampleTable) what += "a path asked the sample table for a dimension beyond table_dims; ";
    return set_err(ctx, PBR_E_UNSUPPORTED, what + "the frame is incomplete");
}

DeviceScene device_scene(pbr_hip_ctx* ctx) {
    const HostScene& h = ctx->host;
    DeviceScene S;
    std::memset(&S, 0, sizeof(S));
    S.nodes = (const float4*)ctx->dNodes.p;
    S.wide = (const float4*)ctx->dWide.p;
    S.rootRef = h.rootRef;
    S.quad = (const float4*)ctx->dQuad.p;
    S.quadRootRef = h.quadRootRef;
    S.binaryWalk = h.quadStackNeed > kQuadStackLimit ? 1 : 0;
    S.triVerts = (const float4*)ctx->dTri.p;
    S.guard = (int*)ctx->dGuard.p;
    S.primInfo = (const int4*)ctx->dInfo.p;
    S.triUV = h.triUV.empty() ? nullptr : (const float2*)ctx->dUV.p;
    S.spheres = (const SphereRec*)ctx->dSph.p;
    S.materials = (const MatTemplate*)ctx->dMat.p;
    S.lights = (const DLight*)ctx->dLights.p;
    S.env = h.env.empty() ? nullptr : (const float4*)ctx->dEnv.p;
    S.nNodes = (int)h.nodes.size();
    S.nPrims = (int)h.primIds.size();
    S.nLights = (int)h.lights.size();
    S.nMaterials = (int)h.materials.size() / 2;
    S.envLight = h.envLight;
    S.nInfinite = (int)h.infinite.size();
    for (int i = 0; i < S.nInfinite && i < 4; ++i) S.infinite[i] = h.infinite[i];
    S.lightCdf = (const float*)ctx->dCdf.p;
    S.lightFunc = (const float*)ctx->dFunc.p;
    S.lightFuncInt = ctx->funcInt;
    S.media = (const float*)ctx->dMedia.p;
    S.nMedia = (int)h.media.size() / 10;
    S.inf = h.inf.light >= 0 ? (const InfDev*)ctx->dInfRec.p : nullptr;
    S.texels = h.texTexels.empty() ? nullptr : (const float4*)ctx->dTexels.p;
    S.textures = h.textures.empty() ? nullptr : (const TexDev*)ctx->dTextures.p;
    S.texMats = h.texMats.empty() ? nullptr : (const TexMat*)ctx->dTexMats.p;
    return S;
}

DeviceSampler device_sampler(pbr_hip_ctx* ctx, int type, int spp, int w, int h) {
    DeviceSampler s;
    std::memset(&s, 0, sizeof(s));
    s.type = type;
    s.spp = spp;
    halton_params(w, h, &s);
    s.primes = (const uint32_t*)ctx->dPrimes.p;
    s.recips = (const uint32_t*)ctx->dRecips.p;
    s.primeSums = (const uint32_t*)ctx->dPrimeSums.p;
    s.perms = (const uint16_t*)ctx->dPerms.p;
    s.guard = (int*)ctx->dGuard.p;
    return s;
}

// SobolSampler(spp, sampleBounds) (Sobol.h): resolution = RoundUpPow2(max(w, h)); matrices from
// the caller (the reference's SobolMatrices32) or the built-in ones; GF(2) pixel tables per m.
int prepare_sobol(pbr_hip_ctx* ctx, const uint32_t* user, int userDims, int w, int h, DeviceSampler* s) {
    const uint32_t* src = user;
    int dims = userDims;
    if (!user) {
        if (ctx->sobolBuiltin.empty()) build_sobol_matrices(1024, &ctx->sobolBuiltin);
        src = ctx->sobolBuiltin.data();
        dims = 1024;
    }
    if (dims < 2) return set_err(ctx, PBR_E_INVALID, "Sobol needs at least 2 dimensions of matrices");
    // the cached device tables are keyed on the matrices' contents, not on the caller's pointer (a
    // reused or reallocated buffer can hold new matrices at the same address)
    uint64_t key = 1469598103934665603ull;
    for (size_t i = 0; i < (size_t)dims * kSobolMatrixSize; ++i) key = (key ^ src[i]) * 1099511628211ull;
    if (key != ctx->sobolKey || dims != ctx->sobolSrcDims) {
        if (int rc = drain(ctx)) return rc;
        // nibble tables: index bits 0..31 (sobol_nibbles) and 32..51 (sobol_nibbles_hi)
        std::vector<uint32_t> nib((size_t)dims * kSobolNib, 0u), nibHi((size_t)dims * kSobolNibHi, 0u);
        for (int d = 0; d < dims; ++d)
            for (int k = 0; k < 13; ++k)
                for (int n = 0; n < 16; ++n) {
                    uint32_t v = 0;
                    for (int b = 0; b < 4; ++b)
                        if ((n >> b) & 1) v ^= src[(size_t)d * kSobolMatrixSize + 4 * k + b];
                    if (k < 8) nib[(size_t)d * kSobolNib + 16 * k + n] = v;
                    else nibHi[(size_t)d * kSobolNibHi + 16 * (k - 8) + n] = v;
                }
        HIP_TRY(ctx->dSobol.upload(nib, ctx->stream));
        HIP_TRY(ctx->dSobolHi.upload(nibHi, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        ctx->sobolKey = key;
        ctx->sobolSrcDims = dims;
        ctx->sobolPixM = -1;
    }
    int res = 1, m = 0;
    while (res < std::max(w, h)) { res <<= 1; ++m; }
    if (m != ctx->sobolPixM) {
        if (int rc = drain(ctx)) return rc;
        std::vector<uint32_t> t;
        try {
            sobol_pixel_tables(src, m, &t);
        } catch (const std::exception& e) {
            return set_err(ctx, PBR_E_UNSUPPORTED, e.what());
        }
        if (t.empty()) t.push_back(0);
        HIP_TRY(ctx->dSobolPix.upload(t, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        ctx->sobolPixM = m;
    }
    s->sobol = (const uint32_t*)ctx->dSobol.p;
    s->sobolHi = (const uint32_t*)ctx->dSobolHi.p;
    s->nSobolDims = dims;
    s->sobolLog2Res = m;
    s->sobolRes = res;
    s->sobolPix = (const uint32_t*)ctx->dSobolPix.p;
    return PBR_OK;
}

int upload_light_distribution(pbr_hip_ctx* ctx, int strategy) {
    std::vector<float> cdf, func;
    float fi = 0;
    light_distribution(ctx->host, strategy, &cdf, &func, &fi);
    if (func.empty()) func.push_back(0.f);
    if (int rc = drain(ctx)) return rc;
    HIP_TRY(ctx->dCdf.upload(cdf, ctx->stream));
    HIP_TRY(ctx->dFunc.upload(func, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));   // the host vectors die on return
    ctx->funcInt = fi;
    ctx->curStrategy = strategy;
    return PBR_OK;
}


// Chunking of the wavefront schedules: at most 2^chunkLog2 samples per chunk; chunks alternate
// over the lanes.  Measured on C2: two lanes 23.4 ms vs 24.9 for one; forcing a one-chunk
// (1/8-frame shard) frame into two concurrent half chunks was slower (4.00 vs 3.86 ms).
struct WfChunks {
    long long chunkPix = 1;
    int lanes = 1;
    size_t cap = 0;   // samples of the largest chunk
    int segCap = 0;   // capacity of one queue segment
    size_t qcap = 0;  // queue entries
};
// A batch's one-chunk frames rotate over the lanes, and every lane holds queue and record buffers for
// the whole frame: they keep several lanes only while the lanes' buffers together stay within this
// many bytes (bytesPerSample × samples per lane, estimated from the schedule's buffers).  A C2 rank
// shard (≤ 2^25 samples, ≈ 12 GB per lane) keeps three; a Path frame at the 2^26-sample cap (≈ 23
// GB per lane) two; the single-frame call would run such a frame on one lane.
constexpr double kBatchLaneBytes = 48e9;
// The largest chunk a Whitted schedule accepts (its default is 2^25, less with several lights).
// Measured, C2 in 5-frame batches (bit-identical): 2^25 (four chunks) 13.62-13.69 ms, 2^26 14.39-14.61,
// 2^27 14.16-14.25 (profiles/r6_c2_chunk_ab.log).
#ifndef PBR_WF_WHITTED_MAXLOG2
#define PBR_WF_WHITTED_MAXLOG2 25
#endif
// laneBudget > 0 (the Path / VolPath schedules, lane_budget): the default chunk is the largest
// 2^k <= 2^maxLog2 samples whose lanes' buffers fit that many bytes (not below 2^minLog2), and a
// batch's one-chunk frames keep as many lanes as fit it; 0: the default is 2^maxLog2 and the batch
// budget kBatchLaneBytes.  A requested chunk_log2 is capped at maxLog2 either way.
// wideLanes > the default lane count: the default lanes when that many lanes of 2^maxLog2-sample
// chunks fit laneBudget (the Path schedule: 4).
WfChunks wf_chunks(const pbr_schedule& sch, const KParams& P, int maxLog2 = 25, bool batch = false,
                   double bytesPerSample = 0, double laneBudget = 0, int defLog2 = 0, int minLog2 = 20,
                   int wideLanes = 0) {
    WfChunks c;
    c.lanes = sch.serial ? 1 : (sch.lanes > 0 ? sch.lanes : kWfDefaultLanes);
    if (!sch.serial && sch.lanes == 0 && wideLanes > c.lanes && sch.chunk_log2 == 0 && defLog2 == 0 &&
        wideLanes * bytesPerSample * (double)(1LL << maxLog2) <= laneBudget)
        c.lanes = std::min(wideLanes, kWfLanes);
    int chunkLog2 = maxLog2;
    if (sch.chunk_log2 > 0) chunkLog2 = std::min(sch.chunk_log2, maxLog2);
    else if (defLog2 > 0) chunkLog2 = std::min(defLog2, maxLog2);
    else if (laneBudget > 0 && bytesPerSample > 0)
        while (chunkLog2 > minLog2 && c.lanes * bytesPerSample * (double)(1LL << chunkLog2) > laneBudget) --chunkLog2;
    c.chunkPix = std::max(1LL, (1LL << chunkLog2) / P.spp);
    if (c.chunkPix >= P.nPixels) {   // one chunk: splitting a small frame only adds launch tails
        c.chunkPix = P.nPixels;
        if (!batch) c.lanes = 1;     // (a batch's one-chunk frames rotate over the lanes)
        else if (c.lanes > 1 && bytesPerSample > 0) {
            const double perLane = bytesPerSample * (double)P.nPixels * (double)P.spp;
            const double budget = laneBudget > 0 ? laneBudget : kBatchLaneBytes;
            c.lanes = (int)std::max(1.0, std::min((double)c.lanes, std::floor(budget / perLane)));
        }
    } else {
        // Many chunks: make them equal and a whole number per lane (the count rounded down to a
        // multiple of the lanes), so no lane runs a last chunk alone.  Measured (bit-identical,
        // frame ms; default / rounded down / rounded up): C5 (32 chunks) 1215 / 1193 / 1200, C4
        // (254) 6628 / 6587 / 6572, C3 (16) 257.0 / 257.5 / 268.3, C2 (4) 17.5 / 18.6 / 18.3 —
        // with few chunks the power-of-two size wins, so only 24 or more are balanced.
        long long n = (P.nPixels + c.chunkPix - 1) / c.chunkPix;
        if (n >= 24) {
            n = std::max<long long>(c.lanes, n / c.lanes * c.lanes);
            c.chunkPix = (P.nPixels + n - 1) / n;
        }
    }
    c.cap = (size_t)c.chunkPix * P.spp;
    // a shade workgroup processes at most ceil(cap / (kWfBlocks·256)) rounds of 256
    c.segCap = (int)((c.cap + (size_t)kWfBlocks * 256 - 1) / ((size_t)kWfBlocks * 256) * 256);
    c.qcap = std::max(c.cap, (size_t)c.segCap * kWfBlocks);
    return c;
}
// Bytes the Path / VolPath lane buffers may take: a share of the device memory that is free or
// already held by this context's lanes (their buffers are reused and grown, never shrunk).  On an
// MI355X (288 GB) that is room for three lanes of 2^27-sample chunks; another large allocation on the
// device (a second context) leaves less and the chunks shrink.  Measured (bit-identical, frame ms of
// single frames, three lanes): C4 2^26 4379 → 2^27 4189, C5 815.6 → 771.4, C3 205.0 → 203.6; 2^24
// and 2^23 were 25-50% slower (profiles/r6_sched_sweep*.log).
constexpr double kLaneMemShare = 0.75;
double lane_budget(pbr_hip_ctx* ctx) {
    size_t freeB = 0, totalB = 0;
    if (hipMemGetInfo(&freeB, &totalB) != hipSuccess) return 0;   // the fixed defaults
    static_assert(sizeof(WfBufs) % sizeof(DevBuf) == 0, "WfBufs holds DevBuf members only");
    double held = 0;
    for (int l = 0; l < kWfLanes; ++l) {
        const DevBuf* b = reinterpret_cast<const DevBuf*>(&ctx->wb[l]);
        for (size_t i = 0; i < sizeof(WfBufs) / sizeof(DevBuf); ++i) held += (double)b[i].bytes;
    }
    return kLaneMemShare * ((double)freeB + held);
}

// The frames of one render call.  One frame (pbr_hip_render): its chunks alternate over the lanes,
// lane 0 on the caller's stream, forked at the start and joined at the end.  A batch
// (pbr_hip_render_frames): the frames' chunks continue one rotation over the same lanes, forked once
// and joined once, so one frame's last launches overlap the next frame's first ones.  No stream
// waits between frames: frame f's end is one event per lane it used (frameEv[f]), which
// pbr_hip_wait_frame hands to the caller's other streams.  (A first version ran every lane on a side
// stream and made the caller's stream wait for each frame: C2 15.7 → 17.0 ms — that stream's waits
// sat in a hardware queue it shares with a lane, holding the lane's next frame behind them.)
struct FrameSet {
    int n = 1;
    float* const* rgb = nullptr;     // per frame (batch); the single frame's outputs are in KParams
    uint8_t* const* rgba = nullptr;
    bool batch = false;
};
// Lanes and hardware queues (PBR_OWN_LANES).  HIP gives a process a few hardware queues (4 by
// default) and deals them to streams in creation order, so lanes only run side by side when their
// streams hold different queues.  The context creates its stream and the lane streams 1-3 together
// (create_lane_streams); a caller's own stream, made at some other time, may share a queue with a
// lane, whose launches then wait behind the other's.  So with four lanes (as many as the default
// queues) and a caller's stream, lane 0 runs on the context's stream, forked from and joined back
// into the caller's.  With fewer lanes the caller's stream keeps lane 0: its fork/join waits would
// otherwise sit in a queue it may share with a lane.  Measured (bit-identical, frame ms in batches
// on a torch stream as bench.py's, profiles/r6_own_lanes_ab.log): four lanes, C3 206.8-207.4 →
// 194.7-196.0, C4 4310 → 4156; three lanes, C5 772.1 → 772.8, C2 13.57-13.59 → 13.75-13.89.
#ifndef PBR_OWN_LANES
#define PBR_OWN_LANES 1
#endif
int create_lane_streams(pbr_hip_ctx* ctx) {
    for (int l = 1; l < kWfLanes; ++l)
        if (!ctx->side[l]) {
            HIP_TRY(hipStreamCreateWithFlags(&ctx->side[l], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&ctx->evJoin[l], hipEventDisableTiming));
        }
    if (!ctx->evJoin[0]) HIP_TRY(hipEventCreateWithFlags(&ctx->evJoin[0], hipEventDisableTiming));
    if (!ctx->evFork) HIP_TRY(hipEventCreateWithFlags(&ctx->evFork, hipEventDisableTiming));
    return PBR_OK;
}
hipStream_t lane_stream(pbr_hip_ctx* ctx, hipStream_t s, int l) { return l ? ctx->side[l] : (ctx->lane0 ? ctx->lane0 : s); }
// Fork the lanes off `s` at the start of a frame (a batch), join them back at the end.
int wf_fork(pbr_hip_ctx* ctx, hipStream_t s, int lanes) {
    const bool own = PBR_OWN_LANES && lanes >= kWfLanes && s != ctx->stream;
    ctx->lane0 = own ? ctx->stream : s;
    if (lanes < 2) return PBR_OK;
    if (int rc = create_lane_streams(ctx)) return rc;
    HIP_TRY(hipEventRecord(ctx->evFork, s));
    for (int l = own ? 0 : 1; l < lanes; ++l) HIP_TRY(hipStreamWaitEvent(lane_stream(ctx, s, l), ctx->evFork, 0));
    return PBR_OK;
}
int wf_join(pbr_hip_ctx* ctx, hipStream_t s, int lanes) {
    if (lanes < 2) return PBR_OK;
    for (int l = ctx->lane0 != s ? 0 : 1; l < lanes; ++l) {
        HIP_TRY(hipEventRecord(ctx->evJoin[l], lane_stream(ctx, s, l)));
        HIP_TRY(hipStreamWaitEvent(s, ctx->evJoin[l], 0));
    }
    return PBR_OK;
}
// A batch: frame f's chunks ended on the lanes in `used` (bit mask; lane 0 is `s`): one event per
// lane, recorded after the lane's last launch of the frame (pbr_hip_wait_frame waits on them).
int wf_frame_done(pbr_hip_ctx* ctx, hipStream_t s, int f, unsigned used) {
    if ((int)ctx->frameEv.size() <= f) ctx->frameEv.resize(f + 1);
    pbr_hip_ctx::FrameEv& e = ctx->frameEv[f];
    e.used = used;
    for (int l = 0; l < kWfLanes; ++l) {
        if (!(used & (1u << l))) continue;
        if (!e.ev[l]) HIP_TRY(hipEventCreateWithFlags(&e.ev[l], hipEventDisableTiming));
        HIP_TRY(hipEventRecord(e.ev[l], lane_stream(ctx, s, l)));
    }
    return PBR_OK;
}
dim3 resident_grid(pbr_hip_ctx* ctx, const void* fn) {
    int perCU = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, fn, 256, 0) != hipSuccess || perCU <= 0) perCU = 4;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0) cus = 256;
    return dim3((unsigned)(perCU * cus));
}

// ---- per-kernel profiling helpers
int prof_begin(pbr_hip_ctx* ctx, int kind, hipStream_t st, int* idx) {
    if (ctx->profUsed == ctx->profEv.size()) {
        pbr_hip_ctx::ProfEv e{kind, nullptr, nullptr};
        HIP_TRY(hipEventCreate(&e.a));
        HIP_TRY(hipEventCreate(&e.b));
        ctx->profEv.push_back(e);
    }
    pbr_hip_ctx::ProfEv& e = ctx->profEv[ctx->profUsed];
    e.kind = kind;
    *idx = (int)ctx->profUsed++;
    HIP_TRY(hipEventRecord(e.a, st));
    return PBR_OK;
}
// counts the segmented queues a launch consumed / filled into row `kind` (fields in order; null = skip)
int prof_sums(pbr_hip_ctx* ctx, hipStream_t st, int kind, std::initializer_list<const int*> segs) {
    if (!ctx->profCount) return PBR_OK;
    ProfSums a;
    std::memset(&a, 0, sizeof(a));
    int k = 0;
    for (const int* p : segs) a.seg[k++] = p;
    a.dst = (unsigned long long*)ctx->dProf.p + (size_t)kind * kProfFields;
    hipLaunchKernelGGL(k_prof_count, dim3(1), dim3(256), 0, st, a);
    return PBR_OK;
}
void prof_host(pbr_hip_ctx* ctx, int kind, int field, unsigned long long v) {
    if (ctx->profCount) ctx->profHost[kind][field] += v;
}
// a launch (any statement list) bracketed by the profile events of `kind` on stream ST
#define PROF_LAUNCH(KIND, ST, ...)                                                  \
    do {                                                                            \
        int pi_ = -1;                                                               \
        if (ctx->profOn) { if (int rc_ = prof_begin(ctx, KIND, ST, &pi_)) return rc_; } \
        __VA_ARGS__;                                                                \
        if (pi_ >= 0) HIP_TRY(hipEventRecord(ctx->profEv[pi_].b, ST));              \
    } while (0)

// Wavefront Whitted: chunks of up to 2^25 samples on two lanes, per level shade → shadow → extend
// (pbr_wavefront.h).
int render_wavefront(pbr_hip_ctx* ctx, KParams& P, hipStream_t s, const FrameSet& F) {
    const int spp = P.spp;
    // samples per chunk: queue + record memory ≈ 370 B per sample at depth 5 (12 GB at 2^25);
    // measured on C2 (one lane): 2^23 29.4 ms, 2^24 28.1, 2^25 26.6, 2^27 (whole frame) 26.6
    const int levels = P.maxDepth < 1 ? 1 : P.maxDepth;
    // multi-light scenes (k_wf_shade_ml): per (level, light) records of 17 B per sample and up to
    // nL shadow rays per shading event; the chunk shrinks so those stay near 6 GB per lane
    const int nL = (int)ctx->host.lights.size();
    const bool ml = nL != 1;
    // one SkyBox light: its radiance is looked up by the shadow kernel (k_wf_shade)
    const bool skyDeferred = !ml && ctx->host.lights[0].type == LT_SKY;
    const bool skyHalton = skyDeferred && P.smp.type == PBR_SAMPLER_HALTON;   // the SkyBox shade variants (C2)
    // records per sample and level: A, F+cos, pdf (36 B) + per light 17 B; the chunk shrinks so
    // they stay under 8 GB per lane (C2: 5 levels × 36 B × 2^25 = 6 GB)
    int maxLog2 = 25;
    while (maxLog2 > 20 && (double)levels * (36.0 + (ml ? 17.0 * nL : 0.0)) * (double)(1LL << maxLog2) > 8e9) --maxLog2;
    const int lightsPerShade = ml ? std::max(1, nL) : 1;
    // the lane buffers below, per sample: two ray queues, the shadow queue(s), the records
    const double bytesPerSample = 2 * 52.0 + (52.0 + (skyDeferred ? 16.0 : 0.0)) * lightsPerShade + 16.0 +
                                  levels * (36.0 + (ml ? 17.0 * nL : 0.0)) + 8.0;
    const WfChunks ch = wf_chunks(ctx->sched, P, PBR_WF_WHITTED_MAXLOG2, F.batch, bytesPerSample, lane_budget(ctx), maxLog2);
    const size_t cap = ch.cap, qcap = ch.qcap;
    const size_t sqcap = qcap * (size_t)lightsPerShade;   // shadow-queue entries
    const int lobes = scene_lobe_kinds(ctx->host);
    const bool simple = (lobes & ~kSimpleLobes) == 0;
    const bool mm = (lobes & ~kMatteMirrorLobes) == 0;   // Lambert + mirror only (C2)
    const bool textured = (lobes & kTexturedLobes) != 0;
    const bool matsLds = ctx->host.materials.size() <= (size_t)kLdsMats;   // templates staged in LDS
    // The level-0 shade traces its own camera rays (no camera kernel and queue).  Frames with fewer
    // chunks than lanes (rank shards of a multi-GPU C2 job) keep the separate kernels by default:
    // there the camera kernel's 8 waves per SIMD win (C2 shard 0/8, one chunk: 2.58 → 3.10 ms fused;
    // shard 0/2, two chunks: 9.58-9.63 → 10.12-10.22).
    // Round 6: a batch whose few-chunk frames rotate over the lanes (a rank's shard) fuses as well — its
    // frames overlap on the lanes, which hides the fused kernel's lower occupancy: C2 8-rank shards
    // 2.10-2.19 → 1.99-2.02 ms, 4-rank 4.13-4.31 → 3.95-4.01 (profiles/r6_shard_c2*.json).
    const long long nChunks = (P.nPixels + ch.chunkPix - 1) / ch.chunkPix;
    const int fuse = ctx->sched.fuse_camera;
    const bool rotating = F.batch && nChunks < ch.lanes;
    const bool fuseCamera = kPacket && kQuadTraversal && fuse != PBR_FUSE_OFF && (mm || simple) && matsLds && !textured &&
                            !ml && (nChunks >= std::max(2, ch.lanes) || fuse == PBR_FUSE_ON || rotating);
    // + pass-through levels only when some primitive has no material (Whitted's no-BSDF branch)
    const int maxLevels = levels;   // no material-less primitives here (those scenes run the megakernel)
    // Shadow rays of level L run on a second stream, overlapping extend(L+1) and shade(L+1) (they
    // only read what shade(L) wrote); the shadow queue alternates between two buffers by level.
    // Default: when the frame is one chunk (no lane overlap).  Measured on C2: a 1/8 shard
    // 3.97 → 3.54 ms; the whole frame (two lanes) 23.43 → 23.76 ms, so off there.
    const bool shadowOverlap = ch.lanes == 1 && !F.batch && !ctx->sched.serial && maxLevels <= kWfMaxDepth + 2;
    WfParams WL[kWfLanes];
    int* cntL[kWfLanes];
    for (int l = 0; l < ch.lanes; ++l) {
        WfBufs& B = ctx->wb[l];
        for (int k = 0; k < 2; ++k) {
            HIP_TRY(B.wqO[k].ensure(qcap * 16)); HIP_TRY(B.wqD[k].ensure(qcap * 16));
            HIP_TRY(B.wqId[k].ensure(qcap * 4)); HIP_TRY(B.wqHit[k].ensure(qcap * 16));
        }
        HIP_TRY(B.wsO.ensure(sqcap * 16)); HIP_TRY(B.wsD.ensure(sqcap * 16));
        HIP_TRY(B.wsC.ensure(qcap * 16)); HIP_TRY(B.wsId.ensure(sqcap * 4));
        if (skyDeferred) HIP_TRY(B.wsW.ensure(sqcap * 16));
        if (ml) { HIP_TRY(B.wRecC.ensure(cap * 16 * levels * nL)); HIP_TRY(B.wRecV.ensure(cap * levels * nL)); }
        HIP_TRY(B.wRecA.ensure(cap * 16 * levels)); HIP_TRY(B.wRecF.ensure(cap * 16 * levels));
        HIP_TRY(B.wRecP.ensure(cap * 4 * levels)); HIP_TRY(B.wDepth.ensure(cap * 4));
        HIP_TRY(B.wIndex.ensure(cap * 4));
        if (shadowOverlap) {
            HIP_TRY(B.wsO2.ensure(sqcap * 16)); HIP_TRY(B.wsD2.ensure(sqcap * 16));
            HIP_TRY(B.wsC2.ensure(qcap * 16)); HIP_TRY(B.wsId2.ensure(sqcap * 4));
            if (skyDeferred) HIP_TRY(B.wsW2.ensure(sqcap * 16));
            if (!ctx->shadowStream[l]) {
                HIP_TRY(hipStreamCreateWithFlags(&ctx->shadowStream[l], hipStreamNonBlocking));
                for (int k = 0; k < kWfMaxDepth + 2; ++k) {
                    HIP_TRY(hipEventCreateWithFlags(&ctx->evShade[l][k], hipEventDisableTiming));
                    HIP_TRY(hipEventCreateWithFlags(&ctx->evShadow[l][k], hipEventDisableTiming));
                }
            }
        }
        HIP_TRY(B.wCnt.ensure(4 * kWfBlocks * sizeof(int)));
        int* cnt = cntL[l] = (int*)B.wCnt.p;   // segment counts: queue 0, queue 1, shadow queues 0, 1
        WfParams& W = WL[l];
        std::memset(&W, 0, sizeof(W));
        W.P = P;
        W.so = (float4*)B.wsO.p; W.sd = (float4*)B.wsD.p; W.sc = (float4*)B.wsC.p; W.sid = (int*)B.wsId.p;
        W.sw = (float4*)B.wsW.p;
        W.skyDeferred = skyDeferred ? 1 : 0;
        W.shadowSeg = cnt + 2 * kWfBlocks;
        W.segCap = ch.segCap;
        W.shadowSegCap = ch.segCap * lightsPerShade;
        W.nLightsML = ml ? nL : 0;
        W.recC = ml ? (float4*)B.wRecC.p : nullptr;
        W.recV = ml ? (uint8_t*)B.wRecV.p : nullptr;
        W.recA = (float4*)B.wRecA.p; W.recF = (float4*)B.wRecF.p; W.recP = (float*)B.wRecP.p;
        W.depthOf = (int*)B.wDepth.p;
        W.sampleIndex = (uint32_t*)B.wIndex.p;
        W.initRecords = ctx->host.anyNoMaterial ? 1 : 0;
        W.prof = ctx->profCount ? (unsigned long long*)ctx->dProf.p : nullptr;
        // Halton dims one sample reaches: 5 camera + per level 2 per light + 2 (SpecularReflect)
        W.P.smp.ldsDims = std::min(kLdsDims, 5 + (2 * lightsPerShade + 2) * levels + 2);
        W.cap = (int)cap;
    }
    auto queue = [&](int l, int k) {
        WfBufs& B = ctx->wb[l];
        WfQueue q;
        q.o = (float4*)B.wqO[k].p; q.d = (float4*)B.wqD[k].p; q.id = (int*)B.wqId[k].p; q.hit = (float4*)B.wqHit[k].p;
        q.s0 = (float4*)B.wqS0[k].p; q.s1 = (float4*)B.wqS1[k].p;
        q.segCount = cntL[l] + k * kWfBlocks;
        return q;
    };
    const dim3 blk(256), gstride(kWfBlocks);
    // The queue consumers (extend, shadow) run exactly one resident wave of workgroups: a grid of
    // kWfBlocks would leave a partial second round (2048 = 1.33 × the 1536 resident at 6/CU).
    const dim3 gShadow = resident_grid(ctx, (const void*)k_wf_shadow<kShortStack>);
    const dim3 gShadowML = resident_grid(ctx, (const void*)k_wf_shadow_ml<kShortStack>);
    const dim3 gExtend = resident_grid(ctx, (const void*)k_wf_extend<kShortStack>);
    // A batch of frames with fewer chunks than lanes (a rank's shard) continues one rotation over the
    // lanes through all its frames; frames of more chunks fork and join per frame, as single frames do
    // (C2, four chunks on three lanes: 15.65 ms per frame joined, 16.11 rotating).
    const bool rotate = F.batch && nChunks < ch.lanes;
    if (rotate) { if (int rc = wf_fork(ctx, s, ch.lanes)) return rc; }
    int chunk = 0;
    for (int f = 0; f < F.n; ++f) {
    if (!rotate) {
        if (int rc = wf_fork(ctx, s, ch.lanes)) return rc;
        chunk = 0;
    }
    unsigned used = 0;
    for (long long p0 = 0; p0 < P.nPixels; p0 += ch.chunkPix, ++chunk) {
        const int l = chunk % ch.lanes;
        const hipStream_t st = lane_stream(ctx, s, l);
        WfParams& W = WL[l];
        if (F.batch) {
            W.P.rgbOut = F.rgb ? F.rgb[f] : nullptr;
            W.P.rgbaOut = F.rgba ? F.rgba[f] : nullptr;
            used |= 1u << l;
        }
        W.chunkPix0 = p0;
        W.chunkPix = (int)std::min<long long>(ch.chunkPix, P.nPixels - p0);
        W.nSamples = W.chunkPix * spp;
        int cur = 0;
        W.cur = queue(l, 0);
        if (!fuseCamera) {
            PROF_LAUNCH(KP_WF_CAMERA, st,
                hipLaunchKernelGGL(k_wf_camera_extend<kCameraShort>, dim3((W.nSamples + 255) / 256), blk, 0, st, W));
        }
        prof_host(ctx, KP_WF_CAMERA, 0, (unsigned long long)W.nSamples);
        const hipStream_t sst = shadowOverlap ? ctx->shadowStream[l] : st;
        WfBufs& B = ctx->wb[l];
        for (int level = 0; level < maxLevels; ++level) {
            W.cur = queue(l, cur);
            W.next = queue(l, cur ^ 1);
            if (shadowOverlap) {
                const bool odd = level & 1;
                W.so = (float4*)(odd ? B.wsO2.p : B.wsO.p); W.sd = (float4*)(odd ? B.wsD2.p : B.wsD.p);
                W.sc = (float4*)(odd ? B.wsC2.p : B.wsC.p); W.sid = (int*)(odd ? B.wsId2.p : B.wsId.p);
                W.sw = (float4*)(odd ? B.wsW2.p : B.wsW.p);
                W.shadowSeg = cntL[l] + (odd ? 3 : 2) * kWfBlocks;
                // shade(L) refills the queue shadow(L-2) read
                if (level >= 2) HIP_TRY(hipStreamWaitEvent(st, ctx->evShadow[l][level - 2], 0));
            }
            const int l0 = level == 0 ? 1 : 0;
            const int kShade = l0 && fuseCamera ? KP_WF_SHADE0 : KP_WF_SHADE;   // (the fused level 0: its own family)
            PROF_LAUNCH(kShade, st,
            if (textured) {
                if (ml) hipLaunchKernelGGL((k_wf_shade_ml<kAllLobes | kTexturedLobes, false>), gstride, blk, 0, st, W, l0);
                else hipLaunchKernelGGL((k_wf_shade<kAllLobes | kTexturedLobes, false>), gstride, blk, 0, st, W, l0);
            } else if (ml) {
                if (simple && matsLds) hipLaunchKernelGGL((k_wf_shade_ml<kSimpleLobes, true>), gstride, blk, 0, st, W, l0);
                else if (simple) hipLaunchKernelGGL((k_wf_shade_ml<kSimpleLobes, false>), gstride, blk, 0, st, W, l0);
                else if (matsLds) hipLaunchKernelGGL((k_wf_shade_ml<kAllLobes, true>), gstride, blk, 0, st, W, l0);
                else hipLaunchKernelGGL((k_wf_shade_ml<kAllLobes, false>), gstride, blk, 0, st, W, l0);
            } else if (fuseCamera && l0 && mm && skyHalton && !(P.cam.lensRadius > 0)) hipLaunchKernelGGL((k_wf_shade<kMatteMirrorLobes, PBR_WF_FUSED_MATS_LDS != 0, PBR_WF_FUSED_OCC, true, true>), gstride, blk, 0, st, W, l0);
            else if (fuseCamera && l0 && mm) hipLaunchKernelGGL((k_wf_shade<kMatteMirrorLobes, true, PBR_WF_SHADE_OCC, true>), gstride, blk, 0, st, W, l0);
            else if (fuseCamera && l0) hipLaunchKernelGGL((k_wf_shade<kSimpleLobes, true, PBR_WF_SHADE_OCC, true>), gstride, blk, 0, st, W, l0);
            else if (mm && matsLds && skyHalton) hipLaunchKernelGGL((k_wf_shade<kMatteMirrorLobes, true, PBR_WF_SHADE_OCC_MM, false, true>), gstride, blk, 0, st, W, l0);
            else if (mm && matsLds) hipLaunchKernelGGL((k_wf_shade<kMatteMirrorLobes, true>), gstride, blk, 0, st, W, l0);
            else if (simple && matsLds) hipLaunchKernelGGL((k_wf_shade<kSimpleLobes, true>), gstride, blk, 0, st, W, l0);
            else if (simple) hipLaunchKernelGGL((k_wf_shade<kSimpleLobes, false>), gstride, blk, 0, st, W, l0);
            else if (matsLds) hipLaunchKernelGGL((k_wf_shade<kAllLobes, true>), gstride, blk, 0, st, W, l0);
            else hipLaunchKernelGGL((k_wf_shade<kAllLobes, false>), gstride, blk, 0, st, W, l0));
            if (l0) prof_host(ctx, kShade, 0, (unsigned long long)W.nSamples);
            if (l0 && fuseCamera && !textured && !ml) prof_host(ctx, kShade, 6, (unsigned long long)W.nSamples);
            if (int rc = prof_sums(ctx, st, kShade, {l0 ? nullptr : W.cur.segCount, W.shadowSeg, nullptr, nullptr,
                                                          W.next.segCount, l0 ? nullptr : W.cur.segCount, nullptr,
                                                          skyDeferred ? W.shadowSeg : nullptr})) return rc;
            if (shadowOverlap) {
                HIP_TRY(hipEventRecord(ctx->evShade[l][level], st));
                HIP_TRY(hipStreamWaitEvent(sst, ctx->evShade[l][level], 0));
            }
            PROF_LAUNCH(KP_WF_SHADOW, sst,
                if (ml) hipLaunchKernelGGL(k_wf_shadow_ml<kShortStack>, gShadowML, blk, 0, sst, W);
                else hipLaunchKernelGGL(k_wf_shadow<kShortStack>, gShadow, blk, 0, sst, W));
            if (int rc = prof_sums(ctx, sst, KP_WF_SHADOW, {W.shadowSeg})) return rc;
            if (shadowOverlap) HIP_TRY(hipEventRecord(ctx->evShadow[l][level], sst));
            if (level + 1 == maxLevels) break;
            cur ^= 1;
            W.cur = queue(l, cur);
            PROF_LAUNCH(KP_WF_EXTEND, st, hipLaunchKernelGGL(k_wf_extend<kShortStack>, gExtend, blk, 0, st, W));
            if (int rc = prof_sums(ctx, st, KP_WF_EXTEND, {W.cur.segCount})) return rc;
        }
        // the fold reads every level's records: after the last shadow launch (stream order on sst)
        if (shadowOverlap) HIP_TRY(hipStreamWaitEvent(st, ctx->evShadow[l][maxLevels - 1], 0));
        const int pb = finish_pixels(spp);
        PROF_LAUNCH(KP_WF_FINISH, st, hipLaunchKernelGGL(k_wf_finish<0>, dim3((W.chunkPix + pb - 1) / pb), blk, 0, st, W));
        prof_host(ctx, KP_WF_FINISH, 0, (unsigned long long)W.chunkPix);
        prof_host(ctx, KP_WF_FINISH, 1, (unsigned long long)W.nSamples);
    }
    if (!rotate) { if (int rc = wf_join(ctx, s, ch.lanes)) return rc; }
    if (F.batch) { if (int rc = wf_frame_done(ctx, s, f, rotate ? used : 1u)) return rc; }
    }
    HIP_TRY(hipGetLastError());
    return rotate ? wf_join(ctx, s, ch.lanes) : PBR_OK;
}

// Wavefront Path: per bounce shade → shadow → probe → resolve → extend (pbr_wavefront_path.h).
int render_wavefront_path(pbr_hip_ctx* ctx, KParams& P, hipStream_t s, bool vol, const FrameSet& F) {
    const int spp = P.spp;
    // ≈ 290 B of queues + state per sample: 19.5 GB per 2^26 chunk and lane.  Measured (bit-identical):
    // C3 2^25 349.4 ms, 2^26 336.1, 2^27 340.4; C5 2^25 1979 ms, 2^26 1939, 2^27 1919
    // the lane buffers below, per sample: two ray queues with their state (84 B each), shadow and probe
    // queues, the direct records, the sample's L and index (+ VolPath's transmittance walk and
    // records), and the class pass lists (at most 5 passes)
    // Path: four lanes where four lanes of 2^27-sample chunks fit the budget (bit-identical, 2^27
    // chunks, frame ms in batches: C3 204.5 → 195.8, C4 4217 → 4160; VolPath's four lanes would have to
    // drop to 2^26 chunks: C5 776.6 → 806.0, profiles/r6_lanes4_batch.log)
    const WfChunks ch = wf_chunks(ctx->sched, P, 27, F.batch, (vol ? 460.0 : 340.0) + 4.0 * 5, lane_budget(ctx), 0, 20,
                                  vol ? 0 : 4);
    const size_t cap = ch.cap, qcap = ch.qcap;
    const long long nChunks = (P.nPixels + ch.chunkPix - 1) / ch.chunkPix;
    const int lobes = scene_lobe_kinds(ctx->host);
    const bool simple = (lobes & ~kSimpleLobes) == 0;
    const bool micro = (lobes & ~kMicroLobes) == 0;   // Lambert + microfacet reflection/transmission (C4, C5)
    // the frame's sampler, for the shade variants specialised on it (C3 Sobol, C4 / C5 Halton)
    const bool halton = P.smp.type == PBR_SAMPLER_HALTON, sobol = P.smp.type == PBR_SAMPLER_SOBOL;
    const bool mm = (lobes & ~kMatteMirrorLobes) == 0;   // Lambert + mirror only (C3)
    const bool textured = (lobes & kTexturedLobes) != 0;
    const bool matsLds = ctx->host.materials.size() <= (size_t)kLdsMats;   // templates staged in LDS
    // The classed Path/VolPath shade (k_wfp_shade / k_wfv_shade CLASSED): with materials of several
    // lobe sets (C4's glass, metal, plastic and matte), one launch per lobe set shades that set's hits
    // with a kernel compiled for it.  A material goes to the first of these sets that holds its lobes;
    // misses and material-less hits to pass 0.  VolPath: pass 0 is the medium pass (no lobes: the
    // rays inside a medium, misses, material-less hits) and every lobe set present has a pass.
    static constexpr int kPassLobes[] = {1 << L_LAMBERT, 1 << L_MF_R, (1 << L_LAMBERT) | (1 << L_MF_R),
                                         (1 << L_MF_R) | (1 << L_MF_T), kMicroLobes};
    constexpr int kMediumPassKind = 5;                          // VolPath's pass 0 (k_wfv_shade<0, …>)
    std::vector<int> passKind;                                   // pass → kPassLobes index
    std::vector<int32_t> matPass(ctx->host.materials.size() / 2, 0);
    if (PBR_CLASSED_SHADE && !textured && matsLds && halton && micro) {
        std::vector<int> kindOf(matPass.size(), -1);
        for (size_t m = 0; m < matPass.size(); ++m) {
            const MatTemplate& mt = ctx->host.materials[2 * m + 1];   // the Path/VolPath lobes (make_bsdf)
            if (!mt.valid) continue;
            int mask = 0;
            for (int i = 0; i < mt.nLobes; ++i) mask |= 1 << mt.lobes[i].kind;
            for (int k = 0; k < 5; ++k)
                if ((mask & ~kPassLobes[k]) == 0) { kindOf[m] = k; break; }
        }
        if (vol) passKind.push_back(kMediumPassKind);
        for (int k = 0; k < 5; ++k)
            for (size_t m = 0; m < matPass.size(); ++m)
                if (kindOf[m] == k) {
                    for (size_t j = 0; j < matPass.size(); ++j)
                        if (kindOf[j] == k) matPass[j] = (int32_t)passKind.size();
                    passKind.push_back(k);
                    break;
                }
        if (passKind.size() < 2) passKind.clear();
    }
    const bool classed = !passKind.empty();
    if (classed && matPass != ctx->matPassHost) {
        HIP_TRY(hipStreamSynchronize(s));   // an earlier async copy may still read the host copy
        ctx->matPassHost = matPass;
        HIP_TRY(ctx->dMatPass.upload(ctx->matPassHost, s));
    }
    // (the level-0 shade tracing its own camera rays, as Whitted's does, measured slower here: C3
    // 254 → 268-271 ms, C4 6575 → 6702 ms at 3 shading waves per SIMD; profiles/r3_fused_ab.log)
    WfvParams VL[kWfLanes];
    int* cntL[kWfLanes];
    for (int l = 0; l < ch.lanes; ++l) {
        WfBufs& B = ctx->wb[l];
        for (int k = 0; k < 2; ++k) {
            HIP_TRY(B.wqO[k].ensure(qcap * 16)); HIP_TRY(B.wqD[k].ensure(qcap * 16));
            HIP_TRY(B.wqId[k].ensure(qcap * 4)); HIP_TRY(B.wqHit[k].ensure(qcap * 16));
            HIP_TRY(B.wqS0[k].ensure(qcap * 16)); HIP_TRY(B.wqS1[k].ensure(qcap * 16));
        }
        HIP_TRY(B.wsO.ensure(qcap * 16)); HIP_TRY(B.wsD.ensure(qcap * 16)); HIP_TRY(B.wsId.ensure(qcap * 4));
        HIP_TRY(B.wpO.ensure(qcap * 16)); HIP_TRY(B.wpD.ensure(qcap * 16)); HIP_TRY(B.wpId.ensure(qcap * 4));
        HIP_TRY(B.sL.ensure(cap * 16));
        // direct records live at the direct queue's positions (segmented, like the ray queues)
        HIP_TRY(B.rA.ensure(qcap * 16)); HIP_TRY(B.rB.ensure(qcap * 16)); HIP_TRY(B.rBeta.ensure(qcap * 16));
        HIP_TRY(B.rLi.ensure(qcap * 16)); HIP_TRY(B.rFlags.ensure(qcap * 4)); HIP_TRY(B.rLight.ensure(qcap * 4));
        HIP_TRY(B.rTgt.ensure(qcap * 4));
        HIP_TRY(B.wIndex.ensure(cap * 4));
        HIP_TRY(B.wCnt.ensure(6 * kWfBlocks * sizeof(int)));
        int* cnt = cntL[l] = (int*)B.wCnt.p;   // segment counts: ray queues 0/1, shadow, probe, direct, Tr walk
        WfvParams& V = VL[l];
        std::memset(&V, 0, sizeof(V));
        WfpParams& X = V.X;
        WfParams& W = X.W;
        X.matPass = classed ? (const int*)ctx->dMatPass.p : nullptr;
        X.nPasses = classed ? (int)passKind.size() : 0;
        if (classed) {   // pass 0 files the entries of passes 1.. per segment
            HIP_TRY(B.wPassList.ensure((passKind.size() - 1) * qcap * 4));
            HIP_TRY(B.wPassCnt.ensure((passKind.size() - 1) * kWfBlocks * sizeof(int)));
            X.passList = (int*)B.wPassList.p;
            X.passCnt = (int*)B.wPassCnt.p;
            X.passStride = (int)qcap;
        }
        if (vol) {
            V.anyHitTr = ctx->host.anyNoMaterial ? 0 : 1;
            HIP_TRY(B.wtO.ensure(qcap * 16)); HIP_TRY(B.wtD.ensure(qcap * 16)); HIP_TRY(B.wtP.ensure(qcap * 16));
            HIP_TRY(B.wtE.ensure(qcap * 16)); HIP_TRY(B.wtN.ensure(qcap * 16)); HIP_TRY(B.wtId.ensure(qcap * 4));
            HIP_TRY(B.rLiA.ensure(qcap * 16)); HIP_TRY(B.rTr.ensure(qcap * 16)); HIP_TRY(B.rWA.ensure(qcap * 4));
            V.to = (float4*)B.wtO.p; V.td = (float4*)B.wtD.p; V.tp = (float4*)B.wtP.p;
            V.te = (float4*)B.wtE.p; V.tn = (float4*)B.wtN.p; V.tid = (int*)B.wtId.p;
            V.trSeg = cnt + 5 * kWfBlocks;
            V.dLiA = (float4*)B.rLiA.p; V.dTr = (float4*)B.rTr.p; V.dWA = (float*)B.rWA.p;
        }
        W.P = P;
        W.prof = ctx->profCount ? (unsigned long long*)ctx->dProf.p : nullptr;
        W.so = (float4*)B.wsO.p; W.sd = (float4*)B.wsD.p; W.sid = (int*)B.wsId.p;
        W.shadowSeg = cnt + 2 * kWfBlocks;
        W.segCap = ch.segCap;
        W.shadowSegCap = ch.segCap;
        W.sampleIndex = (uint32_t*)B.wIndex.p;
        W.cap = (int)cap;
        X.po = (float4*)B.wpO.p; X.pd = (float4*)B.wpD.p; X.pid = (int*)B.wpId.p;
        X.probeSeg = cnt + 3 * kWfBlocks;
        X.directSeg = cnt + 4 * kWfBlocks;
        X.stL = (float4*)B.sL.p;
        X.dA = (float4*)B.rA.p; X.dB = (float4*)B.rB.p; X.dBeta = (float4*)B.rBeta.p; X.dLi = (float4*)B.rLi.p;
        X.dFlags = (int*)B.rFlags.p; X.dLight = (int*)B.rLight.p; X.dTgt = (int*)B.rTgt.p;
        // Path: 5 camera dims + per bounce 1 + 2 + 2 (light) + 2 (BSDF) + 1 (RR)
        W.P.smp.ldsDims = std::min(kLdsDims, 5 + 8 * std::max(1, P.maxDepth) + 2);
    }
    auto queue = [&](int l, int k) {
        WfBufs& B = ctx->wb[l];
        WfQueue q;
        q.o = (float4*)B.wqO[k].p; q.d = (float4*)B.wqD[k].p; q.id = (int*)B.wqId[k].p; q.hit = (float4*)B.wqHit[k].p;
        q.s0 = (float4*)B.wqS0[k].p; q.s1 = (float4*)B.wqS1[k].p;
        q.segCount = cntL[l] + k * kWfBlocks;
        return q;
    };
    const dim3 blk(256), gshade(kWfBlocks);
    const dim3 gShadow = resident_grid(ctx, (const void*)k_wfp_shadow<kShortStack>);
    const dim3 gProbe = resident_grid(ctx, (const void*)k_wfp_probe<kShortStack>);
    const dim3 gExtend = resident_grid(ctx, (const void*)k_wf_extend<kShortStack, true>);
    const dim3 gResolve = resident_grid(ctx, (const void*)k_wfp_resolve);
    // Material-less primitives (medium interfaces) continue a path without a bounce
    // (PathIntegrator.cpp:70-75), one level per crossing.  With such primitives the schedule runs
    // 32 extra levels and then keeps going while continuation rays are queued (a host read of the
    // queue's segment counts per extra level), so no path is cut short; a chain of more than
    // kMaxPassThrough crossings fails the render.
    const int maxLevels = std::max(1, P.maxDepth) + 1 + (ctx->host.anyNoMaterial ? 32 : 0);
    std::vector<int> segHost(kWfBlocks);
    // A batch of frames with fewer chunks than lanes (a rank's shard) continues one rotation over the
    // lanes through all its frames; frames of more chunks fork and join per frame, as single frames do
    // (C2, four chunks on three lanes: 15.65 ms per frame joined, 16.11 rotating).
    const bool rotate = F.batch && nChunks < ch.lanes;
    if (rotate) { if (int rc = wf_fork(ctx, s, ch.lanes)) return rc; }
    int chunk = 0;
    for (int f = 0; f < F.n; ++f) {
    if (!rotate) {
        if (int rc = wf_fork(ctx, s, ch.lanes)) return rc;
        chunk = 0;
    }
    unsigned used = 0;
    for (long long p0 = 0; p0 < P.nPixels; p0 += ch.chunkPix, ++chunk) {
        const int l = chunk % ch.lanes;
        const hipStream_t st = lane_stream(ctx, s, l);
        WfvParams& V = VL[l];
        WfpParams& X = V.X;
        WfParams& W = X.W;
        if (F.batch) {
            W.P.rgbOut = F.rgb ? F.rgb[f] : nullptr;
            W.P.rgbaOut = F.rgba ? F.rgba[f] : nullptr;
            used |= 1u << l;
        }
        W.chunkPix0 = p0;
        W.chunkPix = (int)std::min<long long>(ch.chunkPix, P.nPixels - p0);
        W.nSamples = W.chunkPix * spp;
        int cur = 0;
        W.cur = queue(l, 0);
        PROF_LAUNCH(KP_WFP_CAMERA, st, hipLaunchKernelGGL(k_wfp_camera_extend<kCameraShort>, dim3((W.nSamples + 255) / 256), blk, 0, st, X));
        prof_host(ctx, KP_WFP_CAMERA, 0, (unsigned long long)W.nSamples);
        for (int level = 0;; ++level) {   // ends below: at maxLevels, or when no continuation is queued
            W.cur = queue(l, cur);
            W.next = queue(l, cur ^ 1);
            const int l0 = level == 0 ? 1 : 0;
            const int kShade = vol ? KP_WFV_SHADE : KP_WFP_SHADE;
            X.lastLevel = level + 1 >= maxLevels && !ctx->host.anyNoMaterial;
            if (vol && classed) {   // one launch per pass (pass 0: the medium pass)
                for (int p = 0; p < (int)passKind.size(); ++p) {
                    constexpr int H = PBR_SAMPLER_HALTON, O = PBR_WFV_OCC;
                    PROF_LAUNCH(KP_WFV_SHADE, st,
                        switch (passKind[p]) {
                        case 0: hipLaunchKernelGGL((k_wfv_shade<kPassLobes[0], true, O, H, true>), gshade, blk, 0, st, V, l0, p); break;
                        case 1: hipLaunchKernelGGL((k_wfv_shade<kPassLobes[1], true, O, H, true>), gshade, blk, 0, st, V, l0, p); break;
                        case 2: hipLaunchKernelGGL((k_wfv_shade<kPassLobes[2], true, O, H, true>), gshade, blk, 0, st, V, l0, p); break;
                        case 3: hipLaunchKernelGGL((k_wfv_shade<kPassLobes[3], true, O, H, true>), gshade, blk, 0, st, V, l0, p); break;
                        case 4: hipLaunchKernelGGL((k_wfv_shade<kPassLobes[4], true, O, H, true>), gshade, blk, 0, st, V, l0, p); break;
                        default: hipLaunchKernelGGL((k_wfv_shade<0, true, O, H, true>), gshade, blk, 0, st, V, l0, p); break;
                        });
                }
            } else if (vol) {
                PROF_LAUNCH(KP_WFV_SHADE, st,
                    if (textured) hipLaunchKernelGGL((k_wfv_shade<kAllLobes | kTexturedLobes, false>), gshade, blk, 0, st, V, l0, 0);
                    else if (simple && matsLds) hipLaunchKernelGGL((k_wfv_shade<kSimpleLobes, true>), gshade, blk, 0, st, V, l0, 0);
                    else if (simple) hipLaunchKernelGGL((k_wfv_shade<kSimpleLobes, false>), gshade, blk, 0, st, V, l0, 0);
                    else if (micro && matsLds && halton) hipLaunchKernelGGL((k_wfv_shade<kMicroLobes, true, PBR_WFV_OCC, PBR_SAMPLER_HALTON>), gshade, blk, 0, st, V, l0, 0);
                    else if (micro && matsLds) hipLaunchKernelGGL((k_wfv_shade<kMicroLobes, true>), gshade, blk, 0, st, V, l0, 0);
                    else if (matsLds) hipLaunchKernelGGL((k_wfv_shade<kAllLobes, true>), gshade, blk, 0, st, V, l0, 0);
                    else hipLaunchKernelGGL((k_wfv_shade<kAllLobes, false>), gshade, blk, 0, st, V, l0, 0));
            } else if (classed) {   // one launch per material pass, each compiled for its lobes
                for (int p = 0; p < (int)passKind.size(); ++p) {
                    constexpr int H = PBR_SAMPLER_HALTON, O = PBR_WFP_OCC;
                    PROF_LAUNCH(KP_WFP_SHADE, st,
                        switch (passKind[p]) {
                        case 0: hipLaunchKernelGGL((k_wfp_shade<kPassLobes[0], true, PBR_WFP_OCC_L, H, true>), gshade, blk, 0, st, X, l0, p); break;
                        case 1: hipLaunchKernelGGL((k_wfp_shade<kPassLobes[1], true, O, H, true>), gshade, blk, 0, st, X, l0, p); break;
                        case 2: hipLaunchKernelGGL((k_wfp_shade<kPassLobes[2], true, O, H, true>), gshade, blk, 0, st, X, l0, p); break;
                        case 3: hipLaunchKernelGGL((k_wfp_shade<kPassLobes[3], true, O, H, true>), gshade, blk, 0, st, X, l0, p); break;
                        default: hipLaunchKernelGGL((k_wfp_shade<kPassLobes[4], true, O, H, true>), gshade, blk, 0, st, X, l0, p); break;
                        });
                }
            } else {
                PROF_LAUNCH(KP_WFP_SHADE, st,
                    if (textured) hipLaunchKernelGGL((k_wfp_shade<kAllLobes | kTexturedLobes, false>), gshade, blk, 0, st, X, l0, 0);
                    else if (mm && matsLds && sobol) hipLaunchKernelGGL((k_wfp_shade<kMatteMirrorLobes, true, PBR_WFP_OCC_MM, PBR_SAMPLER_SOBOL>), gshade, blk, 0, st, X, l0, 0);
                    else if (mm && matsLds) hipLaunchKernelGGL((k_wfp_shade<kMatteMirrorLobes, true>), gshade, blk, 0, st, X, l0, 0);
                    else if (simple && matsLds) hipLaunchKernelGGL((k_wfp_shade<kSimpleLobes, true>), gshade, blk, 0, st, X, l0, 0);
                    else if (simple) hipLaunchKernelGGL((k_wfp_shade<kSimpleLobes, false>), gshade, blk, 0, st, X, l0, 0);
                    else if (micro && matsLds && halton) hipLaunchKernelGGL((k_wfp_shade<kMicroLobes, true, PBR_WFP_OCC, PBR_SAMPLER_HALTON>), gshade, blk, 0, st, X, l0, 0);
                    else if (micro && matsLds) hipLaunchKernelGGL((k_wfp_shade<kMicroLobes, true>), gshade, blk, 0, st, X, l0, 0);
                    else if (matsLds) hipLaunchKernelGGL((k_wfp_shade<kAllLobes, true>), gshade, blk, 0, st, X, l0, 0);
                    else hipLaunchKernelGGL((k_wfp_shade<kAllLobes, false>), gshade, blk, 0, st, X, l0, 0));
            }
            if (l0) prof_host(ctx, kShade, 0, (unsigned long long)W.nSamples);
            if (int rc = prof_sums(ctx, st, kShade, {l0 ? nullptr : W.cur.segCount, vol ? V.trSeg : W.shadowSeg, X.probeSeg,
                                                     X.directSeg, W.next.segCount, l0 ? nullptr : W.cur.segCount})) return rc;
            if (vol) {
                PROF_LAUNCH(KP_WFV_TR, st, hipLaunchKernelGGL(k_wfv_tr<kShortStack>, gShadow, blk, 0, st, V));
                if (int rc = prof_sums(ctx, st, KP_WFV_TR, {V.trSeg})) return rc;
            } else {
                PROF_LAUNCH(KP_WFP_SHADOW, st, hipLaunchKernelGGL(k_wfp_shadow<kShortStack>, gShadow, blk, 0, st, X));
                if (int rc = prof_sums(ctx, st, KP_WFP_SHADOW, {W.shadowSeg})) return rc;
            }
            PROF_LAUNCH(KP_WFP_PROBE, st, hipLaunchKernelGGL(k_wfp_probe<kShortStack>, gProbe, blk, 0, st, X));
            if (int rc = prof_sums(ctx, st, KP_WFP_PROBE, {X.probeSeg})) return rc;
            if (vol) PROF_LAUNCH(KP_WFV_RESOLVE, st, hipLaunchKernelGGL(k_wfv_resolve, gResolve, blk, 0, st, V));
            else PROF_LAUNCH(KP_WFP_RESOLVE, st, hipLaunchKernelGGL(k_wfp_resolve, gResolve, blk, 0, st, X));
            if (int rc = prof_sums(ctx, st, vol ? KP_WFV_RESOLVE : KP_WFP_RESOLVE, {X.directSeg})) return rc;
            if (level + 1 >= maxLevels) {
                if (!ctx->host.anyNoMaterial) break;
                HIP_TRY(hipMemcpyAsync(segHost.data(), W.next.segCount, kWfBlocks * sizeof(int), hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                long long pending = 0;
                for (int c : segHost) pending += c;
                if (pending == 0) break;
                if (level + 1 >= maxLevels + kMaxPassThrough)
                    return set_err(ctx, PBR_E_UNSUPPORTED, "a path crossed more than 1024 material-less surfaces");
            }
            cur ^= 1;
            W.cur = queue(l, cur);
            PROF_LAUNCH(KP_WF_EXTEND, st, hipLaunchKernelGGL((k_wf_extend<kShortStack, true>), gExtend, blk, 0, st, W));
            if (int rc = prof_sums(ctx, st, KP_WF_EXTEND, {W.cur.segCount})) return rc;
        }
        const int pb = finish_pixels(spp);
        PROF_LAUNCH(KP_WFP_FINISH, st, hipLaunchKernelGGL(k_wfp_finish, dim3((W.chunkPix + pb - 1) / pb), blk, 0, st, X));
        prof_host(ctx, KP_WFP_FINISH, 0, (unsigned long long)W.chunkPix);
        prof_host(ctx, KP_WFP_FINISH, 1, (unsigned long long)W.nSamples);
    }
    if (!rotate) { if (int rc = wf_join(ctx, s, ch.lanes)) return rc; }
    if (F.batch) { if (int rc = wf_frame_done(ctx, s, f, rotate ? used : 1u)) return rc; }
    }
    HIP_TRY(hipGetLastError());
    return rotate ? wf_join(ctx, s, ch.lanes) : PBR_OK;
}

// The integrator, sampler and scene parameters of a render descriptor (validated): shared by
// pbr_hip_render and the per-ray pbr_hip_li.
int make_params(pbr_hip_ctx* ctx, const pbr_render_desc* d, KParams* out) {
    if (d->spp <= 0) return set_err(ctx, PBR_E_INVALID, "spp must be positive");
    if (d->max_depth < 0) return set_err(ctx, PBR_E_INVALID, "max_depth must be >= 0");
    if (d->integrator == PBR_INTEGRATOR_WHITTED && d->max_depth > kMaxWhittedDepth)
        return set_err(ctx, PBR_E_UNSUPPORTED, "Whitted max_depth above 64 is not supported");
    if (d->integrator < PBR_INTEGRATOR_WHITTED || d->integrator > PBR_INTEGRATOR_VOLPATH)
        return set_err(ctx, PBR_E_INVALID, "unknown integrator");
    if (d->sampler != PBR_SAMPLER_HALTON && d->sampler != PBR_SAMPLER_SOBOL && d->sampler != PBR_SAMPLER_TABLE)
        return set_err(ctx, PBR_E_INVALID, "unknown sampler");
    // SobolSampler rounds spp up to a power of two (GlobalSampler(RoundUpPow2(spp)), Sobol.h)
    int spp = d->spp;
    if (d->sampler == PBR_SAMPLER_SOBOL) {
        int p2 = 1;
        while (p2 < spp) p2 <<= 1;
        spp = p2;
        int res = 1, m = 0;
        while (res < std::max(d->camera.width, d->camera.height)) { res <<= 1; ++m; }
        // pbrt-v3's SobolSampleFloat reads one 52-column matrix per dimension: indices below 2^52
        if (2 * m + 31 - __builtin_clz((unsigned)spp) > kSobolMatrixSize) return set_err(ctx, PBR_E_UNSUPPORTED, "Sobol sample index beyond 52 bits");
        // the device index keeps (px << m) | py and its low 32 bits in 32-bit words, and bits >= 32
        // come from frame >> (32 - 2m): rasters of 2^16 or more (max(w, h) > 32768) are refused
        if (m >= 16) return set_err(ctx, PBR_E_UNSUPPORTED, "Sobol raster above 32768 pixels per side");
    } else if (d->sampler == PBR_SAMPLER_TABLE) {
        if (!d->sample_table || d->table_dims < 1) return set_err(ctx, PBR_E_INVALID, "PBR_SAMPLER_TABLE needs sample_table and table_dims");
        if ((long long)d->camera.width * d->camera.height * spp >= (1ll << 32))
            return set_err(ctx, PBR_E_UNSUPPORTED, "sample table rows beyond 32-bit indices");
    } else if ((long long)spp * (long long)31104 >= (1ll << 32)) {
        return set_err(ctx, PBR_E_UNSUPPORTED, "spp too large for 32-bit sample indices");
    }
    KParams& P = *out;
    std::memset(&P, 0, sizeof(P));
    try {
        build_camera(&d->camera, &P.cam);
    } catch (const std::exception& e) {
        return set_err(ctx, PBR_E_INVALID, e.what());
    }
    if (d->light_strategy != ctx->curStrategy) {
        int rc = upload_light_distribution(ctx, d->light_strategy);
        if (rc) return rc;
    }
    P.S = device_scene(ctx);
    P.smp = device_sampler(ctx, d->sampler, spp, d->camera.width, d->camera.height);
    if (d->sampler == PBR_SAMPLER_TABLE) {   // the caller's values, copied before the call returns
        const size_t bytes = (size_t)d->camera.width * d->camera.height * spp * d->table_dims * sizeof(float);
        if (int rc = drain(ctx)) return rc;
        HIP_TRY(ctx->dTable.ensure(bytes));
        HIP_TRY(hipMemcpyAsync(ctx->dTable.p, d->sample_table, bytes, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        P.smp.table = (const float*)ctx->dTable.p;
        P.smp.tableDims = d->table_dims;
        P.smp.tableW = d->camera.width;
    }
    if (d->sampler == PBR_SAMPLER_SOBOL) {
        int rc = prepare_sobol(ctx, d->sobol_matrices, d->sobol_dims, d->camera.width, d->camera.height, &P.smp);
        if (rc) return rc;
        // sample indices (frame << 2m) | j with frame < spp: bits >= 32 exist iff 2m + log2(spp) > 32
        P.smp.wideIndex = 2 * P.smp.sobolLog2Res + 31 - __builtin_clz((unsigned)spp) > 32;
        P.smp.hiShift = 32 - 2 * P.smp.sobolLog2Res;
    }
    P.integrator = d->integrator;
    P.maxDepth = d->max_depth;
    P.rrThreshold = d->rr_threshold;
    P.spp = spp;
    P.ppb = spp >= 256 ? 1 : 256 / spp;
    return PBR_OK;
}

}  // namespace

extern "C" {

int pbr_hip_abi_version(void) { return PBR_HIP_ABI_VERSION; }

int pbr_hip_query(pbr_hip_ctx* ctx, int n, const float* rays, int any_hit, int prim, pbr_surface_hit* out) {
    if (!ctx || n < 0 || (n > 0 && (!rays || !out))) return PBR_E_INVALID;
    if (!ctx->haveScene) return set_err(ctx, PBR_E_NOSCENE, "no scene uploaded");
    if (prim >= (int)ctx->host.slotOf.size()) return set_err(ctx, PBR_E_INVALID, "primitive index out of range");
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;
    if (n == 0) return PBR_OK;
    const int slot = prim >= 0 ? ctx->host.slotOf[prim] : -1;
    HIP_TRY(ctx->dScratchIn.ensure((size_t)n * 7 * sizeof(float)));
    HIP_TRY(ctx->dScratchOut.ensure((size_t)n * sizeof(pbr_surface_hit)));
    HIP_TRY(hipMemcpyAsync(ctx->dScratchIn.p, rays, (size_t)n * 7 * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_query, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, device_scene(ctx),
                       (const int32_t*)ctx->dPrimIds.p, n, (const float*)ctx->dScratchIn.p, any_hit ? 1 : 0, slot,
                       (pbr_surface_hit*)ctx->dScratchOut.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, ctx->dScratchOut.p, (size_t)n * sizeof(pbr_surface_hit), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return PBR_OK;
}

int pbr_hip_bounds(pbr_hip_ctx* ctx, int prim, float* out6) {
    if (!ctx || !out6) return PBR_E_INVALID;
    if (!ctx->haveScene) return set_err(ctx, PBR_E_NOSCENE, "no scene uploaded");
    const HostScene& h = ctx->host;
    if (prim < 0) {
        if (h.nodes.empty()) {   // an empty scene: Bounds3f() (pMin = +max, pMax = -max)
            const float M = 3.40282347e+38f;
            const float e[6] = {M, M, M, -M, -M, -M};
            std::memcpy(out6, e, sizeof(e));
            return PBR_OK;
        }
        std::memcpy(out6, h.nodes[0].pMin, 12);
        std::memcpy(out6 + 3, h.nodes[0].pMax, 12);
        return PBR_OK;
    }
    if ((size_t)prim * 6 + 6 > h.primBounds.size()) return set_err(ctx, PBR_E_INVALID, "primitive index out of range");
    std::memcpy(out6, &h.primBounds[(size_t)prim * 6], 24);
    return PBR_OK;
}

int pbr_hip_li(pbr_hip_ctx* ctx, const pbr_render_desc* d, int n, const float* rays, const int32_t* q, int depth,
               float* rgb_out) {
    if (!ctx || !d || n < 0 || (n > 0 && (!rays || !q || !rgb_out)) || depth < 0) return PBR_E_INVALID;
    if (!ctx->haveScene) return set_err(ctx, PBR_E_NOSCENE, "no scene uploaded");
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;
    if (int rc = check_guard(ctx)) return rc;
    KParams P;
    if (int rc = make_params(ctx, d, &P)) return rc;
    // Whitted recurses while depth + 1 < maxDepth: starting at `depth` is starting at 0 with
    // maxDepth - depth levels left
    if (d->integrator == PBR_INTEGRATOR_WHITTED) P.maxDepth = std::max(0, P.maxDepth - depth);
    if (n == 0) return PBR_OK;
    for (int i = 0; i < n; ++i) {
        if (q[4 * i] < 0 || q[4 * i + 1] < 0 || q[4 * i] >= d->camera.width || q[4 * i + 1] >= d->camera.height ||
            q[4 * i + 2] < 0 || q[4 * i + 2] >= P.spp || q[4 * i + 3] < 0)
            return set_err(ctx, PBR_E_INVALID, "pixel / sample / dimension out of range");
    }
    const size_t rb = (size_t)n * 7 * 4, qb = (size_t)n * 16, ob = (size_t)n * 12;
    HIP_TRY(ctx->dScratchIn.ensure(rb + qb));
    HIP_TRY(ctx->dScratchOut.ensure(ob));
    char* in = (char*)ctx->dScratchIn.p;
    HIP_TRY(hipMemcpyAsync(in, rays, rb, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(in + rb, q, qb, hipMemcpyHostToDevice, ctx->stream));
    const dim3 g((n + 63) / 64), b(64);
    float* o = (float*)ctx->dScratchOut.p;
    const int32_t* qd = (const int32_t*)(in + rb);
    if (d->integrator == PBR_INTEGRATOR_WHITTED) hipLaunchKernelGGL(k_li<PBR_INTEGRATOR_WHITTED>, g, b, 0, ctx->stream, P, n, (const float*)in, qd, o);
    else if (d->integrator == PBR_INTEGRATOR_PATH) hipLaunchKernelGGL(k_li<PBR_INTEGRATOR_PATH>, g, b, 0, ctx->stream, P, n, (const float*)in, qd, o);
    else hipLaunchKernelGGL(k_li<PBR_INTEGRATOR_VOLPATH>, g, b, 0, ctx->stream, P, n, (const float*)in, qd, o);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(rgb_out, o, ob, hipMemcpyDeviceToHost, ctx->stream));
    if (ctx->host.anyNoMaterial || d->sampler == PBR_SAMPLER_TABLE) {
        HIP_TRY(hipMemcpyAsync(ctx->guardHost, ctx->dGuard.p, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipEventRecord(ctx->evGuard, ctx->stream));
        ctx->guardPending = true;
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return check_guard(ctx);
}

int pbr_hip_set_bvh_build(pbr_hip_ctx* ctx, int where) {
    if (!ctx || (where != PBR_BVH_BUILD_HOST && where != PBR_BVH_BUILD_DEVICE)) return PBR_E_INVALID;
    ctx->bvhBuild = where;
    return PBR_OK;
}

int pbr_hip_bvh_build_info(pbr_hip_ctx* ctx, int* where, double* ms, double* kernel_ms) {
    if (!ctx) return PBR_E_INVALID;
    if (!ctx->haveScene) return set_err(ctx, PBR_E_NOSCENE, "no scene uploaded");
    if (where) *where = ctx->bvhWhereLast;
    if (ms) *ms = ctx->bvhMs;
    if (kernel_ms) *kernel_ms = ctx->bvhKernelMs;
    return PBR_OK;
}

int pbr_hip_build_bvh(pbr_hip_ctx* ctx, int where, int n, const float* prim_bounds, int max_prims, void* nodes_out,
                      int* n_nodes, int32_t* prim_ids_out, double* ms_out) {
    if (!ctx || n < 0 || (n > 0 && !prim_bounds) || !nodes_out || !n_nodes || (n > 0 && !prim_ids_out) ||
        (where != PBR_BVH_BUILD_HOST && where != PBR_BVH_BUILD_DEVICE))
        return PBR_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;
    std::vector<float> pb(prim_bounds, prim_bounds + (size_t)n * 6);
    std::vector<LinearBVHNode> nodes;
    std::vector<int32_t> ids;
    double kms = 0;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        if (where == PBR_BVH_BUILD_DEVICE) device_build_bvh(ctx->stream, pb, max_prims > 0 ? max_prims : 1, &nodes, &ids, &kms);
        else host_build_bvh(pb, max_prims > 0 ? max_prims : 1, &nodes, &ids);
    } catch (const std::invalid_argument& e) {
        return set_err(ctx, PBR_E_INVALID, e.what());
    } catch (const std::exception& e) {
        return set_err(ctx, PBR_E_HIP, e.what());
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms_out) { ms_out[0] = ms; ms_out[1] = kms; }
    *n_nodes = (int)nodes.size();
    if (!nodes.empty()) std::memcpy(nodes_out, nodes.data(), nodes.size() * sizeof(LinearBVHNode));
    if (!ids.empty()) std::memcpy(prim_ids_out, ids.data(), ids.size() * 4);
    return PBR_OK;
}

int pbr_hip_sobol_matrices(int dims, uint32_t* out) {
    if (dims < 1 || dims > kSobolMaxDims || !out) return PBR_E_INVALID;
    std::vector<uint32_t> m;
    build_sobol_matrices(dims, &m);
    std::memcpy(out, m.data(), m.size() * 4);
    return PBR_OK;
}

int pbr_hip_create(int device, pbr_hip_ctx** out) {
    if (!out) return PBR_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return PBR_E_NODEVICE;
    if (device < 0 || device >= n) return PBR_E_INVALID;
    std::unique_ptr<pbr_hip_ctx> ctx(new pbr_hip_ctx);
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess) return PBR_E_HIP;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) return PBR_E_HIP;
    if (hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->evGuard, hipEventDisableTiming) != hipSuccess) return PBR_E_HIP;
    build_halton_tables(1000, &ctx->halton);
    pbr_hip_ctx* c = ctx.get();
    {
        pbr_hip_ctx* ctx = c;   // for HIP_TRY
        if (PBR_OWN_LANES) { if (int rc = create_lane_streams(ctx)) return rc; }   // right after ctx->stream
        HIP_TRY(hipHostMalloc((void**)&ctx->guardHost, sizeof(int), hipHostMallocDefault));
        *ctx->guardHost = 0;
        HIP_TRY(ctx->dGuard.ensure(sizeof(int)));
        HIP_TRY(hipMemsetAsync(ctx->dGuard.p, 0, sizeof(int), ctx->stream));
        HIP_TRY(ctx->dPrimes.upload(ctx->halton.primes, ctx->stream));
        HIP_TRY(ctx->dRecips.upload(ctx->halton.recips, ctx->stream));
        HIP_TRY(ctx->dPrimeSums.upload(ctx->halton.primeSums, ctx->stream));
        HIP_TRY(ctx->dPerms.upload(ctx->halton.perms, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    *out = ctx.release();
    return PBR_OK;
}

int pbr_hip_destroy(pbr_hip_ctx* ctx) {
    if (!ctx) return PBR_E_INVALID;
    (void)hipSetDevice(ctx->device);
    (void)drain(ctx);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (int l = 0; l < kWfLanes; ++l)
        if (ctx->side[l]) (void)hipStreamSynchronize(ctx->side[l]);
    for (int l = 0; l < kWfLanes; ++l) {
        if (ctx->shadowStream[l]) (void)hipStreamSynchronize(ctx->shadowStream[l]);
        for (int k = 0; k < kWfMaxDepth + 2; ++k) {
            if (ctx->evShade[l][k]) (void)hipEventDestroy(ctx->evShade[l][k]);
            if (ctx->evShadow[l][k]) (void)hipEventDestroy(ctx->evShadow[l][k]);
        }
        if (ctx->shadowStream[l]) (void)hipStreamDestroy(ctx->shadowStream[l]);
    }
    if (ctx->evFork) (void)hipEventDestroy(ctx->evFork);
    for (const pbr_hip_ctx::FrameEv& e : ctx->frameEv)
        for (int l = 0; l < kWfLanes; ++l)
            if (e.ev[l]) (void)hipEventDestroy(e.ev[l]);
    for (int l = 0; l < kWfLanes; ++l) {
        if (ctx->evJoin[l]) (void)hipEventDestroy(ctx->evJoin[l]);
        if (ctx->side[l]) (void)hipStreamDestroy(ctx->side[l]);
    }
    for (auto& e : ctx->profEv) {
        if (e.a) (void)hipEventDestroy(e.a);
        if (e.b) (void)hipEventDestroy(e.b);
    }
    ctx->profEv.clear();
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->evGuard) (void)hipEventDestroy(ctx->evGuard);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->guardHost) (void)hipHostFree(ctx->guardHost);
    hipStream_t s = ctx->stream;
    delete ctx;
    if (s) (void)hipStreamDestroy(s);
    return PBR_OK;
}

const char* pbr_hip_last_error(const pbr_hip_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int pbr_hip_sync(pbr_hip_ctx* ctx) {
    if (!ctx) return PBR_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;
    return check_guard(ctx);
}

int pbr_hip_upload_scene(pbr_hip_ctx* ctx, const pbr_scene_desc* desc) {
    if (!ctx) return PBR_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;
    try {
        ctx->bvhMs = ctx->bvhKernelMs = 0;
        ctx->bvhWhereLast = PBR_BVH_BUILD_HOST;
        BvhBuildFn timed = [ctx](const std::vector<float>& pb, int maxPrims, std::vector<LinearBVHNode>* nodes,
                                 std::vector<int32_t>* ids) {
            const auto t0 = std::chrono::steady_clock::now();
            ctx->bvhWhereLast = ctx->bvhBuild;
            if (ctx->bvhBuild == PBR_BVH_BUILD_DEVICE) device_build_bvh(ctx->stream, pb, maxPrims, nodes, ids, &ctx->bvhKernelMs);
            else host_build_bvh(pb, maxPrims, nodes, ids);
            ctx->bvhMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        };
        build_host_scene(desc, &ctx->host, &timed);
    } catch (const std::invalid_argument& e) {
        ctx->haveScene = false;
        return set_err(ctx, PBR_E_INVALID, e.what());
    } catch (const std::exception& e) {
        ctx->haveScene = false;
        return set_err(ctx, PBR_E_HIP, e.what());
    }
    const HostScene& h = ctx->host;
    // BVHAccel's 64-entry stack (BVHAccel.cpp:293) bounds the trees the reference can walk (deeper
    // ones overflow it): those are refused rather than rendered with truncated traversals.  The
    // quad walk needs up to 1.5 entries per binary level; a tree it could overflow (never an SAH
    // tree of a real mesh) renders through the binary walk (device_scene: binaryWalk).
    if (h.binaryStackNeed > kTraversalStack) {
        ctx->haveScene = false;
        return set_err(ctx, PBR_E_UNSUPPORTED, "BVH deeper than BVHAccel's 64-entry traversal stack (" +
                                                   std::to_string(h.binaryStackNeed) + " interior levels)");
    }
    HIP_TRY(hipMemsetAsync(ctx->dGuard.p, 0, sizeof(int), ctx->stream));
    *ctx->guardHost = 0;
    HIP_TRY(ctx->dNodes.upload(h.nodes, ctx->stream));
    HIP_TRY(ctx->dWide.upload(h.wide, ctx->stream));
    HIP_TRY(ctx->dQuad.upload(h.quad, ctx->stream));
    HIP_TRY(ctx->dTri.upload(h.triVerts, ctx->stream));
    HIP_TRY(ctx->dInfo.upload(h.primInfo, ctx->stream));
    HIP_TRY(ctx->dUV.upload(h.triUV, ctx->stream));
    HIP_TRY(ctx->dSph.upload(h.spheres, ctx->stream));
    HIP_TRY(ctx->dMat.upload(h.materials, ctx->stream));
    HIP_TRY(ctx->dLights.upload(h.lights, ctx->stream));
    HIP_TRY(ctx->dEnv.upload(h.env, ctx->stream));
    HIP_TRY(ctx->dMedia.upload(h.media, ctx->stream));
    HIP_TRY(ctx->dInfTex.upload(h.inf.tex, ctx->stream));
    HIP_TRY(ctx->dInfCF.upload(h.inf.condFunc, ctx->stream));
    HIP_TRY(ctx->dInfCC.upload(h.inf.condCdf, ctx->stream));
    HIP_TRY(ctx->dInfMF.upload(h.inf.margFunc, ctx->stream));
    HIP_TRY(ctx->dInfMC.upload(h.inf.margCdf, ctx->stream));
    {   // the InfiniteAreaLight record the device functions read (pbr_layout.h InfDev)
        std::vector<InfDev> rec(1);
        std::memset(rec.data(), 0, sizeof(InfDev));
        rec[0].tex = (const float4*)ctx->dInfTex.p;
        rec[0].condFunc = (const float*)ctx->dInfCF.p;
        rec[0].condCdf = (const float*)ctx->dInfCC.p;
        rec[0].margFunc = (const float*)ctx->dInfMF.p;
        rec[0].margCdf = (const float*)ctx->dInfMC.p;
        rec[0].margInt = h.inf.margInt;
        rec[0].w = h.inf.w;
        rec[0].h = h.inf.h;
        std::memcpy(rec[0].l2w, h.inf.l2w, sizeof(rec[0].l2w));
        std::memcpy(rec[0].w2l, h.inf.w2l, sizeof(rec[0].w2l));
        HIP_TRY(ctx->dInfRec.upload(rec, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));   // rec is a host temporary
    }
    HIP_TRY(ctx->dPrimIds.upload(h.primIds, ctx->stream));
    HIP_TRY(ctx->dTexels.upload(h.texTexels, ctx->stream));
    HIP_TRY(ctx->dTextures.upload(h.textures, ctx->stream));
    HIP_TRY(ctx->dTexMats.upload(h.texMats, ctx->stream));
    int rc = upload_light_distribution(ctx, PBR_LIGHTS_UNIFORM);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->haveScene = true;
    return PBR_OK;
}

static int render_impl(pbr_hip_ctx* ctx, const pbr_render_desc* d, float* rgb_out, uint8_t* rgba_out, pbr_render_stats* stats,
                       const FrameSet& F) {
    if (!ctx) return PBR_E_INVALID;
    if (!d) return set_err(ctx, PBR_E_INVALID, "null render desc");
    if (!ctx->haveScene) return set_err(ctx, PBR_E_NOSCENE, "no scene uploaded");
    if (F.batch && (!d->outputs_on_device || d->collect_stats || stats || d->sampler == PBR_SAMPLER_TABLE || F.n < 1))
        return set_err(ctx, PBR_E_INVALID, "render_frames: device outputs, no stats, no sample table, n >= 1");
    if (F.batch) ctx->batchFrames = 0;   // (set when the batch is queued)
    auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(ctx->device));
    // An earlier asynchronous frame that stopped at a safety bound fails this call.  Only scenes with
    // material-less primitives can trip one in an asynchronous frame (and copy the flag out at the
    // end of their frames), so only those wait for the previous frame here; every other frame stays
    // queued back to back.  Frames with a caller's sample table run synchronously.
    const bool guardFrame = ctx->host.anyNoMaterial || d->sampler == PBR_SAMPLER_TABLE;
    if (guardFrame) {
        if (int rc = drain(ctx)) return rc;
    }
    if (int rc = check_guard(ctx)) return rc;
    hipStream_t s = d->stream ? (hipStream_t)d->stream : ctx->stream;
    KParams P;
    if (int rc = make_params(ctx, d, &P)) return rc;
    const int spp = P.spp;
    // tiles
    std::vector<int32_t> tiles;
    std::vector<long long> starts;
    long long npx = 0;
    if (d->n_tiles > 0) {
        if (!d->tiles) return set_err(ctx, PBR_E_INVALID, "tiles == NULL");
        for (int i = 0; i < d->n_tiles; ++i) {
            const pbr_tile& t = d->tiles[i];
            if (t.x0 < 0 || t.y0 < 0 || t.x1 > d->camera.width || t.y1 > d->camera.height || t.x1 <= t.x0 || t.y1 <= t.y0)
                return set_err(ctx, PBR_E_INVALID, "tile outside the raster");
            tiles.insert(tiles.end(), {t.x0, t.y0, t.x1, t.y1});
            starts.push_back(npx);
            npx += (long long)(t.x1 - t.x0) * (t.y1 - t.y0);
        }
    } else {
        tiles = {0, 0, d->camera.width, d->camera.height};
        starts.push_back(0);
        npx = (long long)d->camera.width * d->camera.height;
    }
    // Device-output renders without host-side stats return without synchronising, so frames can
    // queue back to back.  The context's queues are reused by every frame: a render on another
    // stream first drains the previous one.
    if (ctx->lastStream != s) {
        if (int rc = drain(ctx)) return rc;
    }
    if (tiles != ctx->tilesHost || starts != ctx->startsHost) {
        HIP_TRY(hipStreamSynchronize(s));   // an earlier async copy may still read the host copies
        ctx->tilesHost = tiles;
        ctx->startsHost = starts;
        HIP_TRY(ctx->dTiles.upload(ctx->tilesHost, s));
        HIP_TRY(ctx->dTileStart.upload(ctx->startsHost, s));
    }
    P.tiles = (const int4*)ctx->dTiles.p;
    P.tileStart = (const long long*)ctx->dTileStart.p;
    P.nTiles = (int)starts.size();
    P.nPixels = npx;
    // outputs
    if (d->outputs_on_device) {
        P.rgbOut = rgb_out;
        P.rgbaOut = rgba_out;
    } else {
        if (rgb_out) { HIP_TRY(ctx->dRgb.ensure((size_t)npx * 12)); P.rgbOut = (float*)ctx->dRgb.p; }
        if (rgba_out) { HIP_TRY(ctx->dRgba.ensure((size_t)npx * 4)); P.rgbaOut = (uint8_t*)ctx->dRgba.p; }
    }
    if (d->collect_stats) {
        HIP_TRY(ctx->dStats.ensure(4 * sizeof(unsigned long long)));
        HIP_TRY(hipMemsetAsync(ctx->dStats.p, 0, 4 * sizeof(unsigned long long), s));
        P.stats = (unsigned long long*)ctx->dStats.p;
    }
    long long blocks = (npx + P.ppb - 1) / P.ppb;
    if (blocks > 0x7fffffffLL) return set_err(ctx, PBR_E_UNSUPPORTED, "frame too large");
    dim3 grid((unsigned)blocks), block(256);
    HIP_TRY(hipEventRecord(ctx->ev0, s));
    if (blocks > 0) {
        bool st = d->collect_stats != 0;
        // (a tree too deep for the quad walk's stack runs the megakernel's binary walk)
        const bool mega = ctx->sched.kernels == PBR_KERNELS_MEGAKERNEL || ctx->host.quadStackNeed > kQuadStackLimit;
        // Whitted through material-less primitives recurses at the same depth without bound
        // (WhittedIntegrator.cpp:26-28): only the megakernel follows such chains to the end
        bool wavefront = d->integrator == PBR_INTEGRATOR_WHITTED && !st && ctx->host.lights.size() <= (size_t)kWfMaxLightsML &&
                         !ctx->host.anyNoMaterial &&
                         d->max_depth <= kWfMaxDepth && !mega;
        bool wavefrontPath = (d->integrator == PBR_INTEGRATOR_PATH || d->integrator == PBR_INTEGRATOR_VOLPATH) && !st &&
                             d->max_depth <= 120 && ctx->host.media.size() / 10 < 255 && !mega;
        // the megakernel at 2 waves per SIMD (it trades VGPRs for scratch): 2 beat 1 by 1.78x on C2
        // and tied 4
#define PBR_LAUNCH(I)                                                                                 \
    if (st) hipLaunchKernelGGL((k_render<I, true, 1>), grid, block, 0, s, P);                        \
    else hipLaunchKernelGGL((k_render<I, false, 2>), grid, block, 0, s, P);
        if (wavefront || wavefrontPath) {
            int rc = wavefront ? render_wavefront(ctx, P, s, F) : render_wavefront_path(ctx, P, s, d->integrator == PBR_INTEGRATOR_VOLPATH, F);
            if (rc) {   // stopped part-way: the forked lane / shadow streams may still run
                quiesce(ctx, s);
                return rc;
            }
        } else {
            for (int f = 0; f < F.n; ++f) {   // (a batch: frame after frame on `s`)
                if (F.batch) {
                    P.rgbOut = F.rgb ? F.rgb[f] : nullptr;
                    P.rgbaOut = F.rgba ? F.rgba[f] : nullptr;
                }
                PROF_LAUNCH(KP_MEGA, s,
                    switch (d->integrator) {
                    case PBR_INTEGRATOR_WHITTED: PBR_LAUNCH(PBR_INTEGRATOR_WHITTED) break;
                    case PBR_INTEGRATOR_PATH: PBR_LAUNCH(PBR_INTEGRATOR_PATH) break;
                    default: PBR_LAUNCH(PBR_INTEGRATOR_VOLPATH) break;
                    });
                prof_host(ctx, KP_MEGA, 0, (unsigned long long)npx * (unsigned long long)spp);
                prof_host(ctx, KP_MEGA, 1, (unsigned long long)npx);
                if (F.batch) { if (int rc = wf_frame_done(ctx, s, f, 1u)) return rc; }
            }
        }
#undef PBR_LAUNCH
        HIP_TRY(hipGetLastError());
    }
    if (F.batch) ctx->batchFrames = F.n;
    HIP_TRY(hipEventRecord(ctx->ev1, s));
    if (!d->outputs_on_device) {
        if (rgb_out) HIP_TRY(hipMemcpyAsync(rgb_out, P.rgbOut, (size_t)npx * 12, hipMemcpyDeviceToHost, s));
        if (rgba_out) HIP_TRY(hipMemcpyAsync(rgba_out, P.rgbaOut, (size_t)npx * 4, hipMemcpyDeviceToHost, s));
    }
    unsigned long long hs[4] = {0, 0, 0, 0};
    if (d->collect_stats) HIP_TRY(hipMemcpyAsync(hs, ctx->dStats.p, sizeof(hs), hipMemcpyDeviceToHost, s));
    // every frame copies the guard word out (4 B, asynchronous): a bound or a full traversal stack
    // fails this call (synchronous frames) or the next one / pbr_hip_sync (asynchronous ones), and a
    // bit is never left behind to fail an unrelated later frame
    HIP_TRY(hipMemcpyAsync(ctx->guardHost, ctx->dGuard.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(ctx->evGuard, s));
    ctx->guardPending = true;
    if (!d->outputs_on_device || d->collect_stats || stats || d->sampler == PBR_SAMPLER_TABLE) {
        HIP_TRY(hipStreamSynchronize(s));
        if (int rc = check_guard(ctx)) return rc;
    } else {
        ctx->inFlight = true;
        ctx->lastStream = s;
        return PBR_OK;
    }
    auto t1 = std::chrono::steady_clock::now();
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
        stats->kernel_ms = ms;
        stats->film_ms = 0;
        stats->seconds = std::chrono::duration<double>(t1 - t0).count();
        stats->samples = (uint64_t)npx * (uint64_t)spp;
        stats->rays = hs[0];
        stats->node_visits = hs[1];
        stats->prim_tests = hs[2];
        stats->shading_events = hs[3];
        stats->n_launches = blocks > 0 ? 1 : 0;
    }
    return PBR_OK;
}

int pbr_hip_render(pbr_hip_ctx* ctx, const pbr_render_desc* d, float* rgb_out, uint8_t* rgba_out, pbr_render_stats* stats) {
    return render_impl(ctx, d, rgb_out, rgba_out, stats, FrameSet{});
}

int pbr_hip_render_frames(pbr_hip_ctx* ctx, const pbr_render_desc* d, int n, float* const* rgb_outs, uint8_t* const* rgba_outs) {
    if (!ctx) return PBR_E_INVALID;
    if (n < 1) return set_err(ctx, PBR_E_INVALID, "render_frames: n must be >= 1");
    FrameSet F;
    F.n = n;
    F.rgb = rgb_outs;
    F.rgba = rgba_outs;
    F.batch = true;
    return render_impl(ctx, d, nullptr, nullptr, nullptr, F);
}

int pbr_hip_wait_frame(pbr_hip_ctx* ctx, void* stream, int f) {
    if (!ctx) return PBR_E_INVALID;
    if (f < 0 || f >= ctx->batchFrames) return set_err(ctx, PBR_E_INVALID, "wait_frame: no such frame in the last batch");
    HIP_TRY(hipSetDevice(ctx->device));
    const pbr_hip_ctx::FrameEv& e = ctx->frameEv[f];
    for (int l = 0; l < kWfLanes; ++l)
        if (e.used & (1u << l)) HIP_TRY(hipStreamWaitEvent(stream ? (hipStream_t)stream : ctx->stream, e.ev[l], 0));
    return PBR_OK;
}

int pbr_hip_set_schedule(pbr_hip_ctx* ctx, const pbr_schedule* sched) {
    if (!ctx) return PBR_E_INVALID;
    pbr_schedule s = {};
    if (sched) s = *sched;
    if (s.kernels != PBR_KERNELS_AUTO && s.kernels != PBR_KERNELS_MEGAKERNEL)
        return set_err(ctx, PBR_E_INVALID, "schedule: unknown kernels mode");
    if (s.chunk_log2 != 0 && (s.chunk_log2 < 10 || s.chunk_log2 > 28))
        return set_err(ctx, PBR_E_INVALID, "schedule: chunk_log2 must be 0 or 10..28");
    if (s.lanes < 0 || s.lanes > kWfLanes) return set_err(ctx, PBR_E_INVALID, "schedule: lanes must be 0..4");
    if (s.fuse_camera < PBR_FUSE_AUTO || s.fuse_camera > PBR_FUSE_ON) return set_err(ctx, PBR_E_INVALID, "schedule: unknown fuse mode");
    if (s.serial != 0 && s.serial != 1) return set_err(ctx, PBR_E_INVALID, "schedule: serial must be 0 or 1");
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;   // an asynchronous frame may still use the lane buffers
    ctx->sched = s;
    return PBR_OK;
}

int pbr_hip_set_profiling(pbr_hip_ctx* ctx, int on) {
    if (!ctx) return PBR_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;
    quiesce(ctx, nullptr);
    ctx->profOn = on != 0;
    ctx->profCount = on >= 2;
    ctx->profUsed = 0;
    std::memset(ctx->profHost, 0, sizeof(ctx->profHost));
    if (ctx->profOn) {
        const size_t bytes = (size_t)KP_COUNT * kProfFields * sizeof(unsigned long long);
        HIP_TRY(ctx->dProf.ensure(bytes));
        HIP_TRY(hipMemsetAsync(ctx->dProf.p, 0, bytes, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    return PBR_OK;
}

int pbr_hip_get_profile(pbr_hip_ctx* ctx, pbr_kernel_profile* out, int max, int* n) {
    if (!ctx || !n || (max > 0 && !out)) return PBR_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;
    quiesce(ctx, nullptr);
    static const char* kNames[KP_COUNT] = {
        "k_wf_camera_extend", "k_wf_shade", "k_wf_shadow", "k_wf_extend", "k_wf_finish",
        "k_wfp_camera_extend", "k_wfp_shade", "k_wfp_shadow", "k_wfp_probe", "k_wfp_resolve", "k_wfp_finish",
        "k_wfv_shade", "k_wfv_tr", "k_wfv_resolve", "k_render", "k_wf_shade_l0"};
    unsigned long long c[KP_COUNT][kProfFields];
    std::memset(c, 0, sizeof(c));
    if (ctx->profOn) HIP_TRY(hipMemcpy(c, ctx->dProf.p, sizeof(c), hipMemcpyDeviceToHost));
    for (int k = 0; k < KP_COUNT; ++k)
        for (int f = 0; f < kProfFields; ++f) c[k][f] += ctx->profHost[k][f];
    int launches[KP_COUNT] = {};
    double ms[KP_COUNT] = {};
    for (size_t i = 0; i < ctx->profUsed; ++i) {
        float t = 0;
        HIP_TRY(hipEventElapsedTime(&t, ctx->profEv[i].a, ctx->profEv[i].b));
        ms[ctx->profEv[i].kind] += t;
        launches[ctx->profEv[i].kind] += 1;
    }
    // Algorithmic HBM bytes of each family: the compulsory queue / record / output traffic of the
    // wavefront design, per counted unit; BVH, mesh and texture reads are cacheable
    // and not counted.  f[0] units, f[1..4] pushes (any-hit kernels: f[1] = rays that got through),
    // f[5] units read from a segmented queue (+4 B id each).
    auto bytes = [&](int k) -> unsigned long long {
        const unsigned long long* f = c[k];
        switch (k) {
        case KP_WF_CAMERA: return 52 * f[0];                                   // o, d, hit, index
        case KP_WF_SHADE: case KP_WF_SHADE0:   // ray + hit + index + recA + depth; shadow; next + recF/P
            // (f[6] level-0 samples of fused launches: those read no ray, hit or index; they write the
            // index, 4 B; f[7] shadow pushes carrying a SkyBox direction, 16 B)
            return 72 * f[0] - 48 * f[6] + 4 * f[5] + 52 * f[1] + 52 * f[4] + 16 * f[7];
        case KP_WF_SHADOW:   // o, d, contribution, id; recA RMW (f[2] of the visible: + the SkyBox direction)
            return 52 * f[0] + 32 * f[1] + 16 * f[2];
        case KP_WF_EXTEND: return 64 * f[0];                                   // o, d read; o, hit written
        case KP_WF_FINISH:
            return 16 * f[0] + 4 * f[1] + 16 * (c[KP_WF_SHADE][0] + c[KP_WF_SHADE0][0]) + 20 * (c[KP_WF_SHADE][4] + c[KP_WF_SHADE0][4]);
        case KP_WFP_CAMERA: return 52 * f[0];                                  // o, d, hit, index
        // ray + hit + index (level 0) or id + carried state (queued); stL of the paths that end;
        // shadow, probe, direct record, continuation with its state
        case KP_WFP_SHADE: return 52 * f[0] + 32 * f[5] + 16 * (f[0] - f[4]) + 36 * f[1] + 36 * f[2] + 60 * f[3] + 68 * f[4];
        case KP_WFP_SHADOW: return 36 * f[0] + 8 * f[1];
        case KP_WFP_PROBE: return 56 * f[0];
        case KP_WFP_RESOLVE: return 104 * f[0];                                // record 72 + L RMW 32
        case KP_WFP_FINISH: return 16 * f[0] + 16 * f[1];
        case KP_WFV_SHADE: return 52 * f[0] + 36 * f[5] + 16 * (f[0] - f[4]) + 84 * f[1] + 36 * f[2] + 80 * f[3] + 68 * f[4];
        case KP_WFV_TR: return 100 * f[0];
        case KP_WFV_RESOLVE: return 140 * f[0];
        default: return 16 * f[1];                                             // megakernel: the film output
        }
    };
    int m = 0;
    for (int k = 0; k < KP_COUNT; ++k) {
        if (!launches[k]) continue;
        if (m < max) {
            pbr_kernel_profile& o = out[m];
            std::memset(&o, 0, sizeof(o));
            std::snprintf(o.name, sizeof(o.name), "%s", kNames[k]);
            o.launches = launches[k];
            o.ms = ms[k];
            o.units = c[k][0];
            o.bytes = bytes(k);
            for (int f = 0; f < kProfFields && f < 8; ++f) o.counts[f] = c[k][f];
        }
        ++m;
    }
    *n = m;
    // reset for the next measurement window
    ctx->profUsed = 0;
    std::memset(ctx->profHost, 0, sizeof(ctx->profHost));
    if (ctx->profOn) HIP_TRY(hipMemset(ctx->dProf.p, 0, sizeof(c)));
    return PBR_OK;
}

int pbr_hip_get_bvh(pbr_hip_ctx* ctx, void* nodes_out, int* n_nodes, int32_t* prim_ids_out, int* n_prims) {
    if (!ctx) return PBR_E_INVALID;
    if (!ctx->haveScene) return set_err(ctx, PBR_E_NOSCENE, "no scene uploaded");
    const HostScene& h = ctx->host;
    if (n_nodes) *n_nodes = (int)h.nodes.size();
    if (n_prims) *n_prims = (int)h.primIds.size();
    if (nodes_out) {   // read back what the device traverses
        HIP_TRY(hipMemcpy(nodes_out, ctx->dNodes.p, h.nodes.size() * sizeof(LinearBVHNode), hipMemcpyDeviceToHost));
    }
    if (prim_ids_out) std::memcpy(prim_ids_out, h.primIds.data(), h.primIds.size() * sizeof(int32_t));
    return PBR_OK;
}

int pbr_hip_sampler_values(pbr_hip_ctx* ctx, int sampler, int width, int height, int spp, int n, const int32_t* q, float* out) {
    if (!ctx || !q || !out || n < 0 || width <= 0 || height <= 0) return PBR_E_INVALID;
    if (sampler != PBR_SAMPLER_HALTON && sampler != PBR_SAMPLER_SOBOL) return set_err(ctx, PBR_E_INVALID, "unknown sampler");
    HIP_TRY(hipSetDevice(ctx->device));
    DeviceSampler s = device_sampler(ctx, sampler, spp, width, height);
    if (sampler == PBR_SAMPLER_SOBOL) {
        int rc = prepare_sobol(ctx, nullptr, 0, width, height, &s);
        if (rc) return rc;
        // queries name their sample numbers directly (any int32): keep all of their bits
        s.wideIndex = s.sobolLog2Res > 0;
        s.hiShift = 32 - 2 * s.sobolLog2Res;
        s.spp = 0;   // the mask (spp - 1) of sobol_dimension becomes all ones
    }
    // queries index the prime / permutation (Halton: 1000 dimensions) and matrix (Sobol) tables
    const int maxDims = sampler == PBR_SAMPLER_SOBOL ? s.nSobolDims : 1000;
    for (int i = 0; i < n; ++i)
        if (q[4 * i] < 0 || q[4 * i + 1] < 0 || q[4 * i + 2] < 0 || q[4 * i + 3] < 0 || q[4 * i + 3] >= maxDims)
            return set_err(ctx, PBR_E_INVALID, "sampler query: negative pixel / sample or dimension beyond the tables");
    HaltonParams hp = hparams(s);
    HIP_TRY(ctx->dScratchIn.ensure((size_t)n * 16));
    HIP_TRY(ctx->dScratchOut.ensure((size_t)n * 4));
    HIP_TRY(hipMemcpyAsync(ctx->dScratchIn.p, q, (size_t)n * 16, hipMemcpyHostToDevice, ctx->stream));
    if (n > 0) hipLaunchKernelGGL(k_sampler_values, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, s, hp, n,
                                  (const int32_t*)ctx->dScratchIn.p, (float*)ctx->dScratchOut.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, ctx->dScratchOut.p, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return PBR_OK;
}

// The device samplers as queried by the host API's GlobalSampler (include/pbr/pbr.h): the
// sampler tables for a raster, as pbr_hip_sampler_values prepares them.
static int query_sampler(pbr_hip_ctx* ctx, int sampler, int width, int height, int spp, DeviceSampler* s) {
    if (sampler != PBR_SAMPLER_HALTON && sampler != PBR_SAMPLER_SOBOL) return set_err(ctx, PBR_E_INVALID, "sampler queries: Halton or Sobol");
    if (width <= 0 || height <= 0 || spp <= 0) return set_err(ctx, PBR_E_INVALID, "sampler queries: empty raster or spp");
    *s = device_sampler(ctx, sampler, spp, width, height);
    if (sampler == PBR_SAMPLER_SOBOL) {
        if (int rc = prepare_sobol(ctx, nullptr, 0, width, height, s)) return rc;
        int p2 = 1;
        while (p2 < spp) p2 <<= 1;
        s->spp = p2;
    }
    return PBR_OK;
}

int pbr_hip_sample_index(pbr_hip_ctx* ctx, int sampler, int width, int height, int spp, int n, const int32_t* q, int64_t* out) {
    if (!ctx || n < 0 || (n > 0 && (!q || !out))) return PBR_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;
    DeviceSampler s;
    if (int rc = query_sampler(ctx, sampler, width, height, spp, &s)) return rc;
    for (int i = 0; i < n; ++i)
        if (q[3 * i] < 0 || q[3 * i + 1] < 0 || q[3 * i + 2] < 0) return set_err(ctx, PBR_E_INVALID, "sample_index: negative pixel or sample");
    if (n == 0) return PBR_OK;
    HIP_TRY(ctx->dScratchIn.ensure((size_t)n * 12));
    HIP_TRY(ctx->dScratchOut.ensure((size_t)n * 8));
    HIP_TRY(hipMemcpyAsync(ctx->dScratchIn.p, q, (size_t)n * 12, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_sample_index, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, s, n, (const int32_t*)ctx->dScratchIn.p,
                       (long long*)ctx->dScratchOut.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, ctx->dScratchOut.p, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return PBR_OK;
}

int pbr_hip_sample_dimensions(pbr_hip_ctx* ctx, int sampler, int width, int height, int n, const int64_t* index, const int32_t* q,
                              float* out) {
    if (!ctx || n < 0 || (n > 0 && (!index || !q || !out))) return PBR_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = drain(ctx)) return rc;
    DeviceSampler s;
    if (int rc = query_sampler(ctx, sampler, width, height, 1, &s)) return rc;
    const int maxDims = sampler == PBR_SAMPLER_SOBOL ? s.nSobolDims : 1000;
    for (int i = 0; i < n; ++i) {
        if (q[3 * i + 2] < 0 || q[3 * i + 2] >= maxDims) return set_err(ctx, PBR_E_INVALID, "sample_dimensions: dimension beyond the tables");
        // the device Halton evaluates 32-bit indices (pbr_hip_render refuses spp that would need more)
        if (index[i] < 0 || (sampler == PBR_SAMPLER_HALTON && index[i] >= (1ll << 32)) || index[i] >= (1ll << 52))
            return set_err(ctx, PBR_E_INVALID, "sample_dimensions: index out of range");
    }
    if (n == 0) return PBR_OK;
    HIP_TRY(ctx->dScratchIn.ensure((size_t)n * 20));
    HIP_TRY(ctx->dScratchOut.ensure((size_t)n * 4));
    char* in = (char*)ctx->dScratchIn.p;
    HIP_TRY(hipMemcpyAsync(in, index, (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(in + (size_t)n * 8, q, (size_t)n * 12, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_sample_dimensions, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, s, n, (const long long*)in,
                       (const int32_t*)(in + (size_t)n * 8), (float*)ctx->dScratchOut.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, ctx->dScratchOut.p, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return PBR_OK;
}

int pbr_hip_camera_rays(pbr_hip_ctx* ctx, const pbr_camera_desc* cam, int n, const float* pf, float* out) {
    if (!ctx || !cam || !pf || !out || n < 0) return PBR_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    DeviceCamera dc;
    try {
        build_camera(cam, &dc);
    } catch (const std::exception& e) {
        return set_err(ctx, PBR_E_INVALID, e.what());
    }
    HIP_TRY(ctx->dScratchIn.ensure((size_t)n * 8));
    HIP_TRY(ctx->dScratchOut.ensure((size_t)n * 24));
    HIP_TRY(hipMemcpyAsync(ctx->dScratchIn.p, pf, (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream));
    if (n > 0) hipLaunchKernelGGL(k_camera_rays, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, dc, n,
                                  (const float*)ctx->dScratchIn.p, (float*)ctx->dScratchOut.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, ctx->dScratchOut.p, (size_t)n * 24, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return PBR_OK;
}

int pbr_hip_intersect(pbr_hip_ctx* ctx, int n, const float* rays, float* out, int any_hit) {
    if (!ctx || !rays || !out || n < 0) return PBR_E_INVALID;
    if (!ctx->haveScene) return set_err(ctx, PBR_E_NOSCENE, "no scene uploaded");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(ctx->dScratchIn.ensure((size_t)n * 28));
    HIP_TRY(ctx->dScratchOut.ensure((size_t)n * 20));
    HIP_TRY(hipMemcpyAsync(ctx->dScratchIn.p, rays, (size_t)n * 28, hipMemcpyHostToDevice, ctx->stream));
    DeviceScene S = device_scene(ctx);
    if (n > 0) hipLaunchKernelGGL(k_intersect, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, S,
                                  (const int32_t*)ctx->dPrimIds.p, n, (const float*)ctx->dScratchIn.p,
                                  (float*)ctx->dScratchOut.p, any_hit);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, ctx->dScratchOut.p, (size_t)n * 20, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return PBR_OK;
}

}  // extern "C"
