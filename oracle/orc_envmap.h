// orc_envmap.h — TEST INFRASTRUCTURE ONLY (part of the CPU restatement, see pbr_oracle.h).
//
// InfiniteAreaLight support of the oracle: Lanczos (Texture/Texture.cpp:16-24), MIPMap<Spectrum>
// with ImageWrap::Repeat — power-of-two resampling, box pyramid, trilinear Lookup(st, width)
// (Texture/MIPMap.h:37-53, 86-211, 240-252) — Distribution1D::SampleContinuous and
// Distribution2D (Sampler/Sampling.h:117-171, Sampling.cpp:121-133).  Written class for class
// after the reference so the device tables (pysicalbasedraytracer_amd/csrc/pbr_infinite.cpp) can be
// checked against an independent evaluation.
#pragma once
#include <memory>
#include <vector>

#include "orc_core.h"

namespace orc {

inline float Lanczos(float x, float tau = 2) {   // Texture.cpp:16-24
    x = std::abs(x);
    if (x < 1e-5f) return 1;
    if (x > 1.f) return 0;
    x *= Pi;
    float s = t_sin(x * tau) / (x * tau);
    float lanczos = t_sin(x) / x;
    return s * lanczos;
}
inline int ModI(int a, int b) {   // Mod (PBR.h:194-197)
    int result = a - (a / b) * b;
    return (result < 0) ? result + b : result;
}
inline int RoundUpPow2I(int v) {   // PBR.h:262-270
    v--;
    v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
    return v + 1;
}
inline int Log2IntI(uint32_t v) { return v ? 31 - __builtin_clz(v) : 0; }   // PBR.h:290-297

enum class ImageWrapO { Repeat = 0, Black = 1, Clamp = 2 };   // MIPMap.h:21
inline Spec ClampInf(const Spec& v) { return v.Clamp(0.f, Infinity); }
inline float ClampInf(float v) { return Clampf(v, 0.f, Infinity); }

// MIPMap<T> (T = Spectrum or float), Texture/MIPMap.h:37-252
template <class T>
class MIPMapT {
  public:
    MIPMapT(int resX, int resY, const T* img, ImageWrapO wrap = ImageWrapO::Repeat) : wrapMode(wrap) {   // MIPMap.h:86-155
        std::vector<T> resampled;
        const T* level0 = img;
        if (!IsPow2(resX) || !IsPow2(resY)) {
            int rx = RoundUpPow2I(resX), ry = RoundUpPow2I(resY);
            std::vector<RW> sW = Weights(resX, rx);
            resampled.assign((size_t)rx * ry, T(0.f));
            for (int t = 0; t < resY; ++t)
                for (int s = 0; s < rx; ++s) {
                    resampled[(size_t)t * rx + s] = 0.f;
                    for (int j = 0; j < 4; ++j) {
                        int origS = WrapI(sW[s].firstTexel + j, resX);
                        if (origS >= 0 && origS < resX)
                            resampled[(size_t)t * rx + s] += sW[s].weight[j] * img[(size_t)t * resX + origS];
                    }
                }
            std::vector<RW> tW = Weights(resY, ry);
            std::vector<T> work(ry);
            for (int s = 0; s < rx; ++s) {
                for (int t = 0; t < ry; ++t) {
                    work[t] = 0.f;
                    for (int j = 0; j < 4; ++j) {
                        int offset = WrapI(tW[t].firstTexel + j, resY);
                        if (offset >= 0 && offset < resY) work[t] += tW[t].weight[j] * resampled[(size_t)offset * rx + s];
                    }
                }
                for (int t = 0; t < ry; ++t) resampled[(size_t)t * rx + s] = ClampInf(work[t]);
            }
            resX = rx;
            resY = ry;
            level0 = resampled.data();
        }
        int nLevels = 1 + Log2IntI((uint32_t)std::max(resX, resY));
        us.resize(nLevels);
        vs.resize(nLevels);
        pyr.resize(nLevels);
        us[0] = resX;
        vs[0] = resY;
        pyr[0].assign(level0, level0 + (size_t)resX * resY);
        for (int i = 1; i < nLevels; ++i) {
            int sRes = std::max(1, us[i - 1] / 2), tRes = std::max(1, vs[i - 1] / 2);
            us[i] = sRes;
            vs[i] = tRes;
            pyr[i].assign((size_t)sRes * tRes, T(0.f));
            for (int t = 0; t < tRes; ++t)
                for (int s = 0; s < sRes; ++s)
                    pyr[i][(size_t)t * sRes + s] = .25f * (Texel(i - 1, 2 * s, 2 * t) + Texel(i - 1, 2 * s + 1, 2 * t) +
                                                           Texel(i - 1, 2 * s, 2 * t + 1) + Texel(i - 1, 2 * s + 1, 2 * t + 1));
        }
    }
    int Width() const { return us[0]; }
    int Height() const { return vs[0]; }
    int Levels() const { return (int)pyr.size(); }
    T Texel(int level, int s, int t) const {   // MIPMap.h:166-190
        switch (wrapMode) {
        case ImageWrapO::Repeat: s = ModI(s, us[level]); t = ModI(t, vs[level]); break;
        case ImageWrapO::Clamp: s = Clampi(s, 0, us[level] - 1); t = Clampi(t, 0, vs[level] - 1); break;
        case ImageWrapO::Black:
            if (s < 0 || s >= us[level] || t < 0 || t >= vs[level]) return T(0.f);
            break;
        }
        return pyr[level][(size_t)t * us[level] + s];
    }
    T Lookup(P2 st, float width = 0.f) const {   // MIPMap.h:193-211
        float level = Levels() - 1 + Log2(std::max(width, (float)1e-8));
        if (level < 0) return triangle(0, st);
        else if (level >= Levels() - 1) return Texel(Levels() - 1, 0, 0);
        int iLevel = (int)std::floor(level);
        float delta = level - iLevel;
        return (1 - delta) * triangle(iLevel, st) + delta * triangle(iLevel + 1, st);   // Lerp
    }
    // Lookup(st, dst0, dst1) (MIPMap.h:227-247) with the zero differentials every hit carries (F5):
    // trilinear → Lookup(st, 0) → triangle(0, st); EWA → minorLength == 0 → triangle(0, st)
    T LookupZeroDifferentials(P2 st, bool doTrilinear) const { return doTrilinear ? Lookup(st, 0.f) : triangle(0, st); }

  private:
    struct RW { int firstTexel; float weight[4]; };
    int WrapI(int i, int res) const {
        if (wrapMode == ImageWrapO::Repeat) return ModI(i, res);
        if (wrapMode == ImageWrapO::Clamp) return Clampi(i, 0, res - 1);
        return i;
    }
    static bool IsPow2(int v) { return v && !(v & (v - 1)); }
    static float Log2(float x) {   // PBR.h:283-286
        const float invLog2 = 1.442695040888963387004650940071;
        return t_log(x) * invLog2;
    }
    static std::vector<RW> Weights(int oldRes, int newRes) {   // MIPMap.h:37-53
        std::vector<RW> wt(newRes);
        float filterwidth = 2.f;
        for (int i = 0; i < newRes; ++i) {
            float center = (i + .5f) * oldRes / newRes;
            wt[i].firstTexel = (int)std::floor((center - filterwidth) + 0.5f);
            for (int j = 0; j < 4; ++j) {
                float pos = wt[i].firstTexel + j + .5f;
                wt[i].weight[j] = Lanczos((pos - center) / filterwidth);
            }
            float invSumWts = 1 / (wt[i].weight[0] + wt[i].weight[1] + wt[i].weight[2] + wt[i].weight[3]);
            for (int j = 0; j < 4; ++j) wt[i].weight[j] *= invSumWts;
        }
        return wt;
    }
    T triangle(int level, P2 st) const {   // MIPMap.h:240-252
        level = Clampi(level, 0, Levels() - 1);
        float s = st.x * us[level] - 0.5f;
        float t = st.y * vs[level] - 0.5f;
        int s0 = (int)std::floor(s), t0 = (int)std::floor(t);
        float ds = s - s0, dt = t - t0;
        return (1 - ds) * (1 - dt) * Texel(level, s0, t0) + (1 - ds) * dt * Texel(level, s0, t0 + 1) +
               ds * (1 - dt) * Texel(level, s0 + 1, t0) + ds * dt * Texel(level, s0 + 1, t0 + 1);
    }
    ImageWrapO wrapMode;
    std::vector<int> us, vs;
    std::vector<std::vector<T>> pyr;
};
using MIPMapS = MIPMapT<Spec>;

// Distribution1D::SampleContinuous (Sampling.h:117-131)
inline float SampleContinuous(const Distribution1D& d, float u, float* pdf, int* off) {
    int size = (int)d.cdf.size();
    int first = 0, len = size;
    while (len > 0) {   // FindInterval (PBR.h:167-181)
        int half = len >> 1, middle = first + half;
        if (d.cdf[middle] <= u) { first = middle + 1; len -= half + 1; } else len = half;
    }
    int offset = Clampi(first - 1, 0, size - 2);
    if (off) *off = offset;
    float du = u - d.cdf[offset];
    if ((d.cdf[offset + 1] - d.cdf[offset]) > 0) du /= (d.cdf[offset + 1] - d.cdf[offset]);
    if (pdf) *pdf = (d.funcInt > 0) ? d.func[offset] / d.funcInt : 0;
    return (offset + du) / d.Count();
}

class Distribution2D {   // Sampling.h:134-171, Sampling.cpp:121-133
  public:
    Distribution2D(const float* func, int nu, int nv) {
        for (int v = 0; v < nv; ++v) cond.emplace_back(&func[(size_t)v * nu], nu);
        std::vector<float> marginalFunc;
        for (int v = 0; v < nv; ++v) marginalFunc.push_back(cond[v].funcInt);
        marg = Distribution1D(marginalFunc.data(), nv);
    }
    P2 SampleContinuous2(P2 u, float* pdf) const {
        float pdfs[2];
        int v;
        float d1 = SampleContinuous(marg, u.y, &pdfs[1], &v);
        float d0 = SampleContinuous(cond[v], u.x, &pdfs[0], nullptr);
        *pdf = pdfs[0] * pdfs[1];
        return P2(d0, d1);
    }
    float Pdf(P2 p) const {
        int iu = Clampi(int(p.x * cond[0].Count()), 0, cond[0].Count() - 1);
        int iv = Clampi(int(p.y * marg.Count()), 0, marg.Count() - 1);
        return cond[iv].func[iu] / marg.funcInt;
    }

  private:
    std::vector<Distribution1D> cond;
    Distribution1D marg;
};

}  // namespace orc
