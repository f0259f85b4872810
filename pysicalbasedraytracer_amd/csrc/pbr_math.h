// pbr_math.h — arithmetic core of the MI355X render path, compiled for both gfx950 and the host.
//
// Every operation keeps the reference's float op sequence (no contraction: built with
// -ffp-contract=off; HIP's default correctly-rounded fp32 div/sqrt), because the parity bar is a
// per-pixel L∞ on the CPU render and discrete branches (BVH ties, shadow occlusion, texel choice,
// lobe choice) must resolve identically.  Where the reference crosses to double (Cross, the
// watertight fallback, gamma(n)), so do we — fp64 is cheap on CDNA4.  Transcendentals are
// evaluated as (float)f((double)x) on both sides of the parity check.
#pragma once
#include "pbr_config.h"
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define PBR_HD __host__ __device__ __forceinline__
#else
#define PBR_HD inline
#endif

namespace pbr {

// Core/PBR.h:12-24
constexpr float kPi = 3.14159265358979323846;
constexpr float kInvPi = 0.31830988618379067154;
constexpr float kInv2Pi = 0.15915494309189533577;
constexpr float kInv4Pi = 0.07957747154594766788;
constexpr float kPiOver2 = 1.57079632679489661923;
constexpr float kPiOver4 = 0.78539816339744830961;
constexpr float kShadowEpsilon = 0.0001f;
constexpr float kOneMinusEpsilon = 0.99999994f;
constexpr float kMaxFloat = 3.402823466e+38f;
#define PBR_INF __builtin_huge_valf()

// gamma(n) = (n·ε/2)/(1 − n·ε/2) evaluated in double, narrowed once (Core/PBR.h:21-24)
constexpr float gamma_n(int n) {
    return (float)((n * (1.1920928955078125e-07 * 0.5)) / (1 - n * (1.1920928955078125e-07 * 0.5)));
}

#if defined(__HIP_DEVICE_COMPILE__) && defined(PBR_INLINE_TRANS)
#define PBR_TRANS PBR_HD
#elif defined(__HIP_DEVICE_COMPILE__)
#define PBR_TRANS __host__ __device__ __attribute__((noinline))
#else
#define PBR_TRANS PBR_HD
#endif
PBR_TRANS float t_sin(float x) { return (float)sin((double)x); }
PBR_TRANS float t_cos(float x) { return (float)cos((double)x); }
PBR_TRANS float t_exp(float x) { return (float)exp((double)x); }
PBR_TRANS float t_log(float x) { return (float)log((double)x); }
PBR_TRANS float t_pow(float x, float y) { return (float)pow((double)x, (double)y); }
PBR_TRANS float t_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
PBR_TRANS float t_asin(float x) { return (float)asin((double)x); }
PBR_TRANS float t_acos(float x) { return (float)acos((double)x); }
// sin and cos of one argument in one out-of-line call (each call clobbers every caller-saved VGPR,
// so the shading kernels spill their live state around it): same values as t_sin / t_cos.  Used by
// the SkyBox light sample (uniform_sphere); in the Path/VolPath shades (concentric disk, phase
// function, InfiniteAreaLight) the pair measured slower than two calls (C3 +1.0%, C5 +2.4%).
struct SinCos { float s, c; };
PBR_TRANS SinCos t_sincos(float x) { return SinCos{(float)sin((double)x), (float)cos((double)x)}; }
// atan2(y, x) and asin(z) in one call (SkyBoxLight's direction → map coordinates)
struct Atan2Asin { float phi, theta; };
PBR_TRANS Atan2Asin t_atan2_asin(float y, float x, float z) {
    return Atan2Asin{(float)atan2((double)y, (double)x), (float)asin((double)z)};
}

// std::min/std::max/Clamp with the reference's NaN behaviour
PBR_HD float mn(float a, float b) { return (b < a) ? b : a; }
PBR_HD float mx(float a, float b) { return (a < b) ? b : a; }
PBR_HD float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
PBR_HD int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
PBR_HD float fabs_(float x) { return x < 0 ? -x : (x == 0 ? 0.f : x); }
PBR_HD float fsqrt(float x) { return sqrtf(x); }

PBR_HD uint32_t fbits(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
PBR_HD float bitsf(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }
PBR_HD bool is_inf(float v) { return (fbits(v) & 0x7fffffffu) == 0x7f800000u; }
// Core/PBR.h:142-165
PBR_HD float next_up(float v) {
    if (is_inf(v) && v > 0.f) return v;
    if (v == -0.f) v = 0.f;
    uint32_t u = fbits(v);
    if (v >= 0) ++u; else --u;
    return bitsf(u);
}
PBR_HD float next_down(float v) {
    if (is_inf(v) && v < 0.f) return v;
    if (v == 0.f) v = -0.f;
    uint32_t u = fbits(v);
    if (v > 0) --u; else ++u;
    return bitsf(u);
}

struct f3 { float x, y, z; };
PBR_HD f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
PBR_HD f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
PBR_HD f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
PBR_HD f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
PBR_HD f3 operator*(f3 a, float s) { return mk(s * a.x, s * a.y, s * a.z); }
PBR_HD f3 operator*(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
PBR_HD f3 operator/(f3 a, float f) { float inv = 1.f / f; return mk(a.x * inv, a.y * inv, a.z * inv); }
PBR_HD float get(f3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
PBR_HD void set(f3& v, int i, float x) { if (i == 0) v.x = x; else if (i == 1) v.y = x; else v.z = x; }
PBR_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PBR_HD float absdot(f3 a, f3 b) { return fabsf(dot(a, b)); }
PBR_HD f3 vabs(f3 a) { return mk(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
PBR_HD f3 cross(f3 a, f3 b) {   // Geometry.h:705-714: one narrowing per component
    double ax = a.x, ay = a.y, az = a.z, bx = b.x, by = b.y, bz = b.z;
    return mk((float)((ay * bz) - (az * by)), (float)((az * bx) - (ax * bz)), (float)((ax * by) - (ay * bx)));
}
PBR_HD float len2(f3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
PBR_HD float len(f3 a) { return sqrtf(len2(a)); }
PBR_HD f3 normalize(f3 a) { return a / len(a); }
PBR_HD float maxcomp(f3 v) { return mx(v.x, mx(v.y, v.z)); }
PBR_HD int maxdim(f3 v) { return (v.x > v.y) ? ((v.x > v.z) ? 0 : 2) : ((v.y > v.z) ? 1 : 2); }
PBR_HD f3 permute(f3 v, int x, int y, int z) { return mk(get(v, x), get(v, y), get(v, z)); }
PBR_HD f3 faceforward(f3 n, f3 v) { return (dot(n, v) < 0.f) ? -n : n; }
PBR_HD f3 vmin(f3 a, f3 b) { return mk(mn(a.x, b.x), mn(a.y, b.y), mn(a.z, b.z)); }
PBR_HD f3 vmax(f3 a, f3 b) { return mk(mx(a.x, b.x), mx(a.y, b.y), mx(a.z, b.z)); }
PBR_HD bool is_zero(f3 n) { return n.x == 0 && n.y == 0 && n.z == 0; }
PBR_HD void coordinate_system(f3 v1, f3* v2, f3* v3) {   // Geometry.h:770-777
    if (fabsf(v1.x) > fabsf(v1.y)) *v2 = mk(-v1.z, 0, v1.x) / sqrtf(v1.x * v1.x + v1.z * v1.z);
    else *v2 = mk(0, v1.z, -v1.y) / sqrtf(v1.y * v1.y + v1.z * v1.z);
    *v3 = cross(v1, *v2);
}
PBR_HD f3 spherical_direction(float sinTheta, float cosTheta, float phi, f3 x, f3 y, f3 z) {
    return sinTheta * t_cos(phi) * x + sinTheta * t_sin(phi) * y + cosTheta * z;
}

// RGB spectrum: component-wise, true division by scalars (Spectrum.h:103-109)
struct rgb { float r, g, b; };
PBR_HD rgb sp(float v) { rgb s; s.r = s.g = s.b = v; return s; }
PBR_HD rgb sp3(float r, float g, float b) { rgb s; s.r = r; s.g = g; s.b = b; return s; }
PBR_HD rgb operator+(rgb a, rgb b) { return sp3(a.r + b.r, a.g + b.g, a.b + b.b); }
PBR_HD rgb operator-(rgb a, rgb b) { return sp3(a.r - b.r, a.g - b.g, a.b - b.b); }
PBR_HD rgb operator*(rgb a, rgb b) { return sp3(a.r * b.r, a.g * b.g, a.b * b.b); }
PBR_HD rgb operator/(rgb a, rgb b) { return sp3(a.r / b.r, a.g / b.g, a.b / b.b); }
PBR_HD rgb operator*(rgb a, float s) { return sp3(a.r * s, a.g * s, a.b * s); }
PBR_HD rgb operator*(float s, rgb a) { return sp3(a.r * s, a.g * s, a.b * s); }
PBR_HD rgb operator/(rgb a, float s) { return sp3(a.r / s, a.g / s, a.b / s); }
PBR_HD bool black(rgb a) { return a.r == 0.f && a.g == 0.f && a.b == 0.f; }
PBR_HD float maxval(rgb a) { return mx(mx(a.r, a.g), a.b); }
PBR_HD rgb sqrt_s(rgb a) { return sp3(sqrtf(a.r), sqrtf(a.g), sqrtf(a.b)); }
// Spectrum Exp, per channel.  Three equal channels (a grey medium's transmittance: C5's) take one
// evaluation — the same input gives the same bits — instead of three out-of-line fp64 calls.
PBR_HD rgb exp_s(rgb a) {
    if (a.r == a.g && a.g == a.b) {   // (±0 compare equal and exp(+0) == exp(-0); a NaN takes the general path)
        const float e = t_exp(a.r);
        return sp3(e, e, e);
    }
    return sp3(t_exp(a.r), t_exp(a.g), t_exp(a.b));
}
PBR_HD rgb clamp_s(rgb a) { return sp3(clampf(a.r, 0, PBR_INF), clampf(a.g, 0, PBR_INF), clampf(a.b, 0, PBR_INF)); }

// 4x4 row-major transforms (Core/Transform.h)
struct m44 { float m[16]; };
PBR_HD f3 xf_point(const float* m, f3 p) {
    float x = p.x, y = p.y, z = p.z;
    float xp = m[0] * x + m[1] * y + m[2] * z + m[3];
    float yp = m[4] * x + m[5] * y + m[6] * z + m[7];
    float zp = m[8] * x + m[9] * y + m[10] * z + m[11];
    float wp = m[12] * x + m[13] * y + m[14] * z + m[15];
    if (wp == 1) return mk(xp, yp, zp);
    float inv = 1.f / wp;
    return mk(inv * xp, inv * yp, inv * zp);
}
PBR_HD f3 xf_vector(const float* m, f3 v) {
    float x = v.x, y = v.y, z = v.z;
    return mk(m[0] * x + m[1] * y + m[2] * z, m[4] * x + m[5] * y + m[6] * z, m[8] * x + m[9] * y + m[10] * z);
}

// Geometry.h:1470-1484
PBR_HD f3 offset_ray_origin(f3 p, f3 pError, f3 n, f3 w) {
    float d = dot(vabs(n), pError);
    f3 off = d * n;
    if (dot(w, n) < 0) off = -off;
    f3 po = p + off;
    if (off.x > 0) po.x = next_up(po.x); else if (off.x < 0) po.x = next_down(po.x);
    if (off.y > 0) po.y = next_up(po.y); else if (off.y < 0) po.y = next_down(po.y);
    if (off.z > 0) po.z = next_up(po.z); else if (off.z < 0) po.z = next_down(po.z);
    return po;
}

// ---------------------------------------------------------------- Halton (Sampler/Halton.cpp)
// Exact 32-bit division by a runtime prime: approximate quotient from a 32-bit reciprocal,
// corrected by at most two steps. Valid for every 32-bit numerator.
// recip <= 2^32/d makes the estimate at most floor(n/d) and n·recip/2^32 > n/d − 1 at least
// floor(n/d) − 1, so one conditional step corrects it (and the remainder, the digit, comes with it).
PBR_HD uint32_t divrem_prime(uint32_t n, uint32_t d, uint32_t recip /* floor(2^32/d) */, uint32_t* rem) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t q = __umulhi(n, recip);
#else
    uint32_t q = (uint32_t)(((uint64_t)n * recip) >> 32);
#endif
    uint32_t r = n - q * d;
    const bool c = r >= d;
    q += c ? 1u : 0u;
    r -= c ? d : 0u;
    *rem = r;
    return q;
}
PBR_HD uint32_t div_prime(uint32_t n, uint32_t d, uint32_t recip /* floor(2^32/d) */) {
    uint32_t r;
    return divrem_prime(n, d, recip, &r);
}
// LowDiscrepancy.cpp:212-225 RadicalInverseSpecialized<base> (64-bit digit accumulator)
PBR_HD float radical_inverse_b(uint32_t base, uint32_t recip, uint32_t a) {
    const float invBase = 1.f / (float)base;
    uint64_t rev = 0;
    float invBaseN = 1;
    while (a) {
        uint32_t next = div_prime(a, base, recip);
        uint32_t digit = a - next * base;
        rev = rev * base + digit;
        invBaseN *= invBase;
        a = next;
    }
    return mn((float)rev * invBaseN, kOneMinusEpsilon);
}
// LowDiscrepancy.cpp:2300-2315
PBR_HD float scrambled_radical_inverse(uint32_t base, uint32_t recip, const uint16_t* perm, uint32_t a) {
    const float invBase = 1.f / (float)base;
    uint64_t rev = 0;
    float invBaseN = 1;
    while (a) {
        uint32_t next = div_prime(a, base, recip);
        uint32_t digit = a - next * base;
        rev = rev * base + perm[digit];
        invBaseN *= invBase;
        a = next;
    }
    return mn(invBaseN * ((float)rev + invBase * (float)perm[0] / (1 - invBase)), kOneMinusEpsilon);
}
// the same with invBase = 1 / base and tail = invBase·perm[0] / (1 - invBase) formed by the caller
// (per dimension, once: stage_halton_lds)
// Two digits per step while two remain: both permutation lookups are issued together (they are
// independent), rev gets the same integer and invBaseN the same sequence of products.
PBR_HD float scrambled_radical_inverse_pre(uint32_t base, uint32_t recip, const uint16_t* perm, uint32_t a, float invBase,
                                           float tail) {
    uint64_t rev = 0;
    float invBaseN = 1;
    while (a >= base) {
        uint32_t d0, d1;
        const uint32_t a1 = divrem_prime(a, base, recip, &d0);
        a = divrem_prime(a1, base, recip, &d1);
        const uint32_t p0 = perm[d0], p1 = perm[d1];
        rev = (rev * base + p0) * base + p1;
        invBaseN *= invBase;
        invBaseN *= invBase;
    }
    if (a) {   // the last digit is a itself
        rev = rev * base + perm[a];
        invBaseN *= invBase;
    }
    return mn(invBaseN * ((float)rev + tail), kOneMinusEpsilon);
}
PBR_HD uint32_t reverse_bits32(uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __brev(n);
#else
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ffu) << 8) | ((n & 0xff00ff00u) >> 8);
    n = ((n & 0x0f0f0f0fu) << 4) | ((n & 0xf0f0f0f0u) >> 4);
    n = ((n & 0x33333333u) << 2) | ((n & 0xccccccccu) >> 2);
    n = ((n & 0x55555555u) << 1) | ((n & 0xaaaaaaaau) >> 1);
    return n;
#endif
}
// base 2: ReverseBits64(a)·2^-64 narrowed from double == (float)ReverseBits32(a)·2^-32 for a < 2^32
PBR_HD float radical_inverse_2(uint32_t a) { return (float)reverse_bits32(a) * 2.3283064365386963e-10f; }

struct HaltonParams {
    int baseExp0, baseExp1, baseScale1, stride;
    int mult0, mult1, scaleRatio0, scaleRatio1;   // sampleStride/baseScales[i]
};
// HaltonSampler::GetIndexForSample (Halton.cpp:61-81) — per-pixel offset, exact in 32 bits
PBR_HD uint32_t halton_pixel_offset(const HaltonParams& h, int px, int py) {
    if (h.stride <= 1) return 0;
    int pm0 = px % 128; if (pm0 < 0) pm0 += 128;
    int pm1 = py % 128; if (pm1 < 0) pm1 += 128;
    uint32_t d0 = 0, v = (uint32_t)pm0;
    for (int i = 0; i < h.baseExp0; ++i) { d0 = d0 * 2 + (v & 1u); v >>= 1; }
    uint32_t d1 = 0; v = (uint32_t)pm1;
    for (int i = 0; i < h.baseExp1; ++i) { uint32_t q = v / 3u; d1 = d1 * 3 + (v - q * 3u); v = q; }
    // d_i < baseScale_i, scaleRatio_i = stride / baseScale_i, mult_i < baseScale_i: each term is
    // below baseScale_i · stride <= 243 · 31104, so the sum fits 32 bits and the reference's
    // 64-bit arithmetic (Halton.cpp:61-81) gives the same value
    uint32_t off = d0 * (uint32_t)h.scaleRatio0 * (uint32_t)h.mult0 + d1 * (uint32_t)h.scaleRatio1 * (uint32_t)h.mult1;
    return off % (uint32_t)h.stride;
}

}  // namespace pbr
