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
// The out-of-line fp64 library calls (ocml on the device, libm on the host).
PBR_TRANS float c_sin(float x) { return (float)sin((double)x); }
PBR_TRANS float c_cos(float x) { return (float)cos((double)x); }
PBR_TRANS float c_exp(float x) { return (float)exp((double)x); }
PBR_TRANS float c_log(float x) { return (float)log((double)x); }
PBR_TRANS float t_pow(float x, float y) { return (float)pow((double)x, (double)y); }
PBR_TRANS float c_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
PBR_TRANS float c_asin(float x) { return (float)asin((double)x); }
PBR_TRANS float c_acos(float x) { return (float)acos((double)x); }
PBR_TRANS double c_cos_d(double x) { return cos(x); }
PBR_TRANS double c_sin_d(double x) { return sin(x); }

// Device fast path of the transcendentals, same results.  Each t_f(x) is (float)f((double)x).  On
// the device it is first evaluated inline in fp64 — Cody-Waite reduction + fdlibm's sin/cos kernels,
// atan over a k/8 table, log via atanh, exp via ln2 reduction — to within 2^-50 relative (measured
// 2^-51 against glibc over 4·10^7 arguments incl. the floats nearest multiples of π/2:
// tests/test_fast_trans.py).  If every value within 2^-40 relative of that approximation rounds to
// the same float, that float is the correctly rounded f(x), and so exactly what the fp64 library
// call rounds to (its result lies in the same interval); otherwise — about once in 2^15 — the call
// is made.  The calls stay on a cold branch: they clobber every caller-saved VGPR, so a shading
// kernel that called them on its hot path spilled its live state around each one.
namespace fastm {
PBR_HD bool rounds_to(double v, float* out) {
    const double t = fabs(v) * 0x1p-40;
    const float lo = (float)(v - t), hi = (float)(v + t);
    *out = hi;
    return lo == hi;
}
// sin / cos of a float with |x| <= 64 (fdlibm's __kernel_sin / __kernel_cos polynomials on
// |y| <= π/4; π/2 in three parts, the first two of 33 bits so n·part is exact)
PBR_HD bool sincos(float x, double* s, double* c) {
    const double xd = x;
    if (!(fabs(xd) <= 64.0) || x == 0) return false;
    const double n = rint(xd * 6.36619772367581382433e-01);
    const double y = ((xd - n * 1.57079632673412561417e+00) - n * 6.07710050630396597660e-11) - n * 2.02226624879595063154e-21;
    const double z = y * y;
    const double ps = 8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 + z * (2.75573137070700676789e-06 +
                      z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
    const double sy = y + y * z * (-1.66666666666666324348e-01 + z * ps);
    const double pc = 4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 + z * (2.48015872894767294178e-05 +
                      z * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11))));
    const double cy = (1.0 - 0.5 * z) + z * z * pc;
    const int q = (int)n & 3;
    *s = q == 0 ? sy : (q == 1 ? cy : (q == 2 ? -sy : -cy));
    *c = q == 0 ? cy : (q == 1 ? -sy : (q == 2 ? -cy : sy));
    return true;
}
// atan(t), t in [0, 1]: atan(k/8) + atan((t − k/8) / (1 + t·k/8)), |u| <= 1/16, Taylor to u^13
PBR_HD double atan01(double t) {
    const double kd = rint(t * 8.0);
    const double c = kd * 0.125;
    const double u = (t - c) / (1.0 + t * c);
    const double z = u * u;
    const double p = -1.0 / 3 + z * (1.0 / 5 + z * (-1.0 / 7 + z * (1.0 / 9 + z * (-1.0 / 11 + z * (1.0 / 13)))));
    const int k = (int)kd;
    const double tk = k < 4 ? (k < 2 ? (k == 0 ? 0.0 : 0x1.fd5ba9aac2f6ep-4) : (k == 2 ? 0x1.f5b75f92c80ddp-3 : 0x1.6f61941e4def1p-2))
                            : (k < 6 ? (k == 4 ? 0x1.dac670561bb4fp-2 : 0x1.1e00babdefeb4p-1)
                                     : (k == 6 ? 0x1.4978fa3269ee1p-1 : (k == 7 ? 0x1.700a7c5784634p-1 : 0x1.921fb54442d18p-1)));
    return tk + (u + u * z * p);
}
PBR_HD bool atan2(double y, double x, double* r) {   // finite, both nonzero
    if (!(x != 0 && y != 0 && fabs(x) <= 1e300 && fabs(y) <= 1e300)) return false;
    const double ax = fabs(x), ay = fabs(y);
    const bool sw = ay > ax;
    double a = atan01(sw ? ax / ay : ay / ax);
    if (sw) a = 0x1.921fb54442d18p+0 - a;
    if (x < 0) a = 0x1.921fb54442d18p+1 - a;
    *r = y < 0 ? -a : a;
    return true;
}
// log(x), x > 0 normal: e·ln2 + 2·atanh(s), s = (m − 1)/(m + 1), m in [√½, √2), |s| <= 0.1716
PBR_HD bool log(float x, double* r) {
    if (!(x >= 1.17549435e-38f && x <= 3.40282347e+38f)) return false;
    int e = (int)((__builtin_bit_cast(uint32_t, x) >> 23) & 0xff) - 127;
    double md = (double)__builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, x) & 0x7fffffu) | 0x3f800000u);   // [1, 2)
    if (md > 1.41421356237309504880) { md *= 0.5; e += 1; }
    const double s = (md - 1.0) / (md + 1.0), z = s * s;
    const double p = 1.0 / 3 + z * (1.0 / 5 + z * (1.0 / 7 + z * (1.0 / 9 + z * (1.0 / 11 + z * (1.0 / 13 + z * (1.0 / 15 +
                     z * (1.0 / 17 + z * (1.0 / 19 + z * (1.0 / 21 + z * (1.0 / 23))))))))));
    const double lm = 2.0 * (s + s * z * p);
    *r = e == 0 ? lm : (double)e * 0x1.62e42fefa39efp-1 + lm;
    return true;
}
// exp(x), |x| <= 100: 2^n · exp(r), r = x − n·ln2 (ln2 in two parts, the first of 32 bits), Taylor to r^13
PBR_HD bool exp(float x, double* r) {
    if (!(fabs(x) <= 100.f)) return false;
    const double xd = x;
    const double n = rint(xd * 0x1.71547652b82fep+0);
    const double y = (xd - n * 0x1.62e42feep-1) - n * 0x1.a39ef35793c76p-33;
    double p = 1.0 / 6227020800.0;
    p = 1.0 / 479001600.0 + y * p; p = 1.0 / 39916800.0 + y * p; p = 1.0 / 3628800.0 + y * p;
    p = 1.0 / 362880.0 + y * p; p = 1.0 / 40320.0 + y * p; p = 1.0 / 5040.0 + y * p; p = 1.0 / 720.0 + y * p;
    p = 1.0 / 120.0 + y * p; p = 1.0 / 24.0 + y * p; p = 1.0 / 6.0 + y * p; p = 0.5 + y * p; p = 1.0 + y * p;
    const double ey = 1.0 + y * p;
    *r = ey * __builtin_bit_cast(double, (uint64_t)((int64_t)n + 1023) << 52);
    return true;
}
}  // namespace fastm

#if defined(__HIP_DEVICE_COMPILE__) && !defined(PBR_INLINE_TRANS)
#define PBR_FAST(call, expr)                                                        \
    do {                                                                            \
        double v_;                                                                  \
        float o_;                                                                   \
        if (__builtin_expect(call && fastm::rounds_to(expr, &o_), 1)) return o_;   \
    } while (0)
#else
#define PBR_FAST(call, expr) do { } while (0)
#endif
PBR_HD float t_sin(float x) { double c_; (void)c_; PBR_FAST(fastm::sincos(x, &v_, &c_), v_); return c_sin(x); }
PBR_HD float t_cos(float x) { double s_; (void)s_; PBR_FAST(fastm::sincos(x, &s_, &v_), v_); return c_cos(x); }
PBR_HD float t_exp(float x) { PBR_FAST(fastm::exp(x, &v_), v_); return c_exp(x); }
PBR_HD float t_log(float x) { PBR_FAST(fastm::log(x, &v_), v_); return c_log(x); }
PBR_HD float t_atan2(float y, float x) { PBR_FAST(fastm::atan2((double)y, (double)x, &v_), v_); return c_atan2(y, x); }
PBR_HD float t_asin(float x) {   // asin(x) = atan2(x, sqrt((1 − x)(1 + x)))
    PBR_FAST(fabsf(x) < 1.f && fastm::atan2((double)x, sqrt((1.0 - (double)x) * (1.0 + (double)x)), &v_), v_);
    return c_asin(x);
}
PBR_HD float t_acos(float x) {   // acos(x) = atan2(sqrt((1 − x)(1 + x)), x)
    PBR_FAST(fabsf(x) < 1.f && fastm::atan2(sqrt((1.0 - (double)x) * (1.0 + (double)x)), (double)x, &v_), v_);
    return c_acos(x);
}
// (float)(r · cos(phi)) / (float)(r · sin(phi)) with the products in double (TrowbridgeReitzSample11)
PBR_HD float t_rcos_d(double r, float phi) {
    double s_; (void)s_; PBR_FAST(fastm::sincos(phi, &s_, &v_), r * v_); return (float)(r * c_cos_d((double)phi));
}
PBR_HD float t_rsin_d(double r, float phi) {
    double c_; (void)c_; PBR_FAST(fastm::sincos(phi, &v_, &c_), r * v_); return (float)(r * c_sin_d((double)phi));
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
PBR_HD rgb exp_s(rgb a) { return sp3(t_exp(a.r), t_exp(a.g), t_exp(a.b)); }
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
PBR_HD uint32_t div_prime(uint32_t n, uint32_t d, uint32_t recip /* floor(2^32/d) */) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t q = __umulhi(n, recip);
#else
    uint32_t q = (uint32_t)(((uint64_t)n * recip) >> 32);
#endif
    uint32_t r = n - q * d;
    while (r >= d) { ++q; r -= d; }
    return q;
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
