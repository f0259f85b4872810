// pbr_infinite.cpp — host half of the InfiniteAreaLight (Light/InfiniteAreaLight.cpp:7-68) and of
// ImageTexture (Texture/ImageTexture.cpp:13-92: its MIPMap's level 0, see build_image_texture): the
// MIPMap<RGBSpectrum> built from the environment image (Texture/MIPMap.h:86-187), its level-0
// texels for the device's bilinear Lookup(st, 0), the Distribution2D over luminance × sinθ
// (Sampler/Sampling.h:76-171, Sampling.cpp:121-133) and Power() for the power light distribution.
//
// Float operations follow the reference's order one for one (per channel for RGBSpectrum), with
// the transcendentals of pbr_math.h (correctly rounded) so the oracle reproduces the same bits.
#include "pbr_scene.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

namespace pbr {

namespace {

struct RGB { float c[3]; };
inline RGB rgb0() { return RGB{{0.f, 0.f, 0.f}}; }
inline RGB operator+(const RGB& a, const RGB& b) { return RGB{{a.c[0] + b.c[0], a.c[1] + b.c[1], a.c[2] + b.c[2]}}; }
inline RGB operator*(float s, const RGB& a) { return RGB{{s * a.c[0], s * a.c[1], s * a.c[2]}}; }

int imod(int a, int b) {   // Mod (Core/PBR.h:194-197)
    int r = a - (a / b) * b;
    return r < 0 ? r + b : r;
}
bool is_pow2(int v) { return v && !(v & (v - 1)); }
int round_up_pow2(int v) {   // RoundUpPow2 (PBR.h:262-270)
    v--;
    v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
    return v + 1;
}
int log2_int(uint32_t v) { return v ? 31 - __builtin_clz(v) : 0; }

float lanczos(float x, float tau) {   // Texture/Texture.cpp:16-24
    x = std::fabs(x);
    if (x < 1e-5f) return 1;
    if (x > 1.f) return 0;
    x *= kPi;
    float s = t_sin(x * tau) / (x * tau);
    float l = t_sin(x) / x;
    return s * l;
}

struct Weight { int first; float w[4]; };
std::vector<Weight> resample_weights(int oldRes, int newRes) {   // MIPMap.h:37-53
    std::vector<Weight> wt(newRes);
    const float filterwidth = 2.f;
    for (int i = 0; i < newRes; ++i) {
        float center = (i + .5f) * oldRes / newRes;
        wt[i].first = (int)std::floor((center - filterwidth) + 0.5f);
        for (int j = 0; j < 4; ++j) {
            float pos = wt[i].first + j + .5f;
            wt[i].w[j] = lanczos((pos - center) / filterwidth, 2.f);
        }
        float invSumWts = 1 / (wt[i].w[0] + wt[i].w[1] + wt[i].w[2] + wt[i].w[3]);
        for (int j = 0; j < 4; ++j) wt[i].w[j] *= invSumWts;
    }
    return wt;
}

float clamp_inf(float v) {   // Clamp(v, 0, Infinity)
    const float inf = std::numeric_limits<float>::infinity();
    return v < 0.f ? 0.f : (v > inf ? inf : v);
}

// MIPMap<RGBSpectrum> with ImageWrap::Repeat (the InfiniteAreaLight's default).
struct Pyramid {
    std::vector<int> W, H;
    std::vector<std::vector<RGB>> lv;
    int levels() const { return (int)lv.size(); }
    const RGB& texel(int l, int s, int t) const {   // MIPMap.h:166-190
        s = imod(s, W[l]);
        t = imod(t, H[l]);
        return lv[l][(size_t)t * W[l] + s];
    }
    RGB triangle(int l, float s0f, float t0f) const {   // MIPMap.h:240-252
        l = l < 0 ? 0 : (l > levels() - 1 ? levels() - 1 : l);
        float s = s0f * W[l] - 0.5f;
        float t = t0f * H[l] - 0.5f;
        int s0 = (int)std::floor(s), t0 = (int)std::floor(t);
        float ds = s - s0, dt = t - t0;
        return (1 - ds) * (1 - dt) * texel(l, s0, t0) + (1 - ds) * dt * texel(l, s0, t0 + 1) +
               ds * (1 - dt) * texel(l, s0 + 1, t0) + ds * dt * texel(l, s0 + 1, t0 + 1);
    }
    RGB lookup(float s, float t, float width) const {   // MIPMap.h:193-211
        const float invLog2 = 1.442695040888963387004650940071f;
        float level = levels() - 1 + t_log(width > 1e-8f ? width : 1e-8f) * invLog2;
        if (level < 0) return triangle(0, s, t);
        if (level >= levels() - 1) return texel(levels() - 1, 0, 0);
        int il = (int)std::floor(level);
        float delta = level - il;
        return (1 - delta) * triangle(il, s, t) + delta * triangle(il + 1, s, t);
    }
};

void build_pyramid(int resW, int resH, std::vector<RGB> img, Pyramid* P) {   // MIPMap.h:86-155
    if (!is_pow2(resW) || !is_pow2(resH)) {
        const int pw = round_up_pow2(resW), ph = round_up_pow2(resH);
        std::vector<Weight> sw = resample_weights(resW, pw);
        std::vector<RGB> re((size_t)pw * ph, rgb0());
        for (int t = 0; t < resH; ++t)
            for (int s = 0; s < pw; ++s) {
                RGB acc = rgb0();
                for (int j = 0; j < 4; ++j) {
                    int os = imod(sw[s].first + j, resW);
                    if (os >= 0 && os < resW) acc = acc + sw[s].w[j] * img[(size_t)t * resW + os];
                }
                re[(size_t)t * pw + s] = acc;
            }
        std::vector<Weight> tw = resample_weights(resH, ph);
        std::vector<RGB> work(ph);
        for (int s = 0; s < pw; ++s) {
            for (int t = 0; t < ph; ++t) {
                RGB acc = rgb0();
                for (int j = 0; j < 4; ++j) {
                    int off = imod(tw[t].first + j, resH);
                    if (off >= 0 && off < resH) acc = acc + tw[t].w[j] * re[(size_t)off * pw + s];
                }
                work[t] = acc;
            }
            for (int t = 0; t < ph; ++t)
                for (int k = 0; k < 3; ++k) re[(size_t)t * pw + s].c[k] = clamp_inf(work[t].c[k]);
        }
        img.swap(re);
        resW = pw;
        resH = ph;
    }
    const int n = 1 + log2_int((uint32_t)std::max(resW, resH));
    P->W.assign(n, 0);
    P->H.assign(n, 0);
    P->lv.assign(n, {});
    P->W[0] = resW;
    P->H[0] = resH;
    P->lv[0] = std::move(img);
    for (int i = 1; i < n; ++i) {
        const int sr = std::max(1, P->W[i - 1] / 2), tr = std::max(1, P->H[i - 1] / 2);
        P->W[i] = sr;
        P->H[i] = tr;
        P->lv[i].assign((size_t)sr * tr, rgb0());
        for (int t = 0; t < tr; ++t)
            for (int s = 0; s < sr; ++s)
                P->lv[i][(size_t)t * sr + s] = .25f * (P->texel(i - 1, 2 * s, 2 * t) + P->texel(i - 1, 2 * s + 1, 2 * t) +
                                                       P->texel(i - 1, 2 * s, 2 * t + 1) + P->texel(i - 1, 2 * s + 1, 2 * t + 1));
    }
}

float lum(const RGB& a) { return 0.212671f * a.c[0] + 0.715160f * a.c[1] + 0.072169f * a.c[2]; }   // RGBSpectrum::y

// Distribution1D (Sampling.h:78-91); func kept as given
void dist1d(const float* f, int n, std::vector<float>* cdf, float* funcInt) {
    cdf->assign(n + 1, 0.f);
    for (int i = 1; i < n + 1; ++i) (*cdf)[i] = (*cdf)[i - 1] + f[i - 1] / n;
    *funcInt = (*cdf)[n];
    if (*funcInt == 0) for (int i = 1; i < n + 1; ++i) (*cdf)[i] = float(i) / float(n);
    else for (int i = 1; i < n + 1; ++i) (*cdf)[i] /= *funcInt;
}

float inverse_gamma(float v) {   // InverseGammaCorrect (Core/PBR.h:126-129)
    if (v <= 0.04045f) return v * 1.f / 12.92f;
    return t_pow((v + 0.055f) * 1.f / 1.055f, (float)2.4f);
}

// MIPMap<T> constructor's power-of-two resample (MIPMap.h:86-150) with the texture's wrap mode, for
// T = RGBSpectrum (nc = 3) or float (nc = 1); img is row-major, nc floats per texel.
void resample_pow2(int wrap, int nc, int* resW, int* resH, std::vector<float>* img) {
    const int W0 = *resW, H0 = *resH;
    if (is_pow2(W0) && is_pow2(H0)) return;
    const int pw = round_up_pow2(W0), ph = round_up_pow2(H0);
    auto wrapIdx = [wrap](int i, int res) {
        if (wrap == PBR_WRAP_REPEAT) return imod(i, res);
        if (wrap == PBR_WRAP_CLAMP) return i < 0 ? 0 : (i > res - 1 ? res - 1 : i);
        return i;
    };
    std::vector<Weight> sw = resample_weights(W0, pw);
    std::vector<float> re((size_t)pw * ph * nc, 0.f);
    for (int t = 0; t < H0; ++t)
        for (int s = 0; s < pw; ++s)
            for (int j = 0; j < 4; ++j) {
                const int os = wrapIdx(sw[s].first + j, W0);
                if (os >= 0 && os < W0)
                    for (int k = 0; k < nc; ++k)
                        re[((size_t)t * pw + s) * nc + k] += sw[s].w[j] * (*img)[((size_t)t * W0 + os) * nc + k];
            }
    std::vector<Weight> tw = resample_weights(H0, ph);
    std::vector<float> work((size_t)ph * nc);
    for (int s = 0; s < pw; ++s) {
        for (int t = 0; t < ph; ++t) {
            for (int k = 0; k < nc; ++k) work[(size_t)t * nc + k] = 0.f;
            for (int j = 0; j < 4; ++j) {
                const int off = wrapIdx(tw[t].first + j, H0);
                if (off >= 0 && off < H0)
                    for (int k = 0; k < nc; ++k) work[(size_t)t * nc + k] += tw[t].w[j] * re[((size_t)off * pw + s) * nc + k];
            }
        }
        for (int t = 0; t < ph; ++t)
            for (int k = 0; k < nc; ++k) re[((size_t)t * pw + s) * nc + k] = clamp_inf(work[(size_t)t * nc + k]);
    }
    img->swap(re);
    *resW = pw;
    *resH = ph;
}

}  // namespace

void build_image_texture(const pbr_texture_desc& td, TexDev* out, std::vector<float>* texels) {
    // loadImage (ImageTexture.cpp:13-37) → GetTexture's substitute for a missing image (:60-66) →
    // convertIn per texel (ImageTexture.h:69-78) → MIPMap level 0 (MIPMap.h:86-150)
    int w = 1, h = 1;
    std::vector<RGB> rgb;
    if (td.wrap < PBR_WRAP_REPEAT || td.wrap > PBR_WRAP_CLAMP) throw std::invalid_argument("bad texture wrap mode");
    if (td.level0) {   // a built ImageTexture's MIPMap level 0 (MIPMap.h:150-153): used as is
        const int nc = td.is_float ? 1 : 3;
        if (!td.data || td.width <= 0 || td.height <= 0 || !is_pow2(td.width) || !is_pow2(td.height))
            throw std::invalid_argument("a level-0 texture needs data with power-of-two width and height");
        if (td.components != nc) throw std::invalid_argument("a level-0 texture has 3 (RGB) or 1 (float) components");
        std::memset(out, 0, sizeof(*out));
        out->offset = (int)(texels->size() / 4);
        out->w = td.width;
        out->h = td.height;
        out->wrap = td.wrap;
        out->isFloat = td.is_float ? 1 : 0;
        out->su = td.su; out->sv = td.sv; out->du = td.du; out->dv = td.dv;
        for (size_t i = 0; i < (size_t)td.width * td.height; ++i)
            for (int k = 0; k < 4; ++k) texels->push_back(k < nc ? td.data[i * nc + k] : 0.f);
        return;
    }
    if (td.data && td.width > 0 && td.height > 0) {
        if (td.components < 3) throw std::invalid_argument("ImageTexture image needs >= 3 components");
        w = td.width;
        h = td.height;
        rgb.resize((size_t)w * h);
        for (size_t i = 0; i < rgb.size(); ++i)
            for (int k = 0; k < 3; ++k) rgb[i].c[k] = td.data[i * td.components + k];
    } else {
        rgb.assign(1, RGB{{0.5f, 0.5f, 0.5f}});
    }
    const int nc = td.is_float ? 1 : 3;
    std::vector<float> img((size_t)w * h * nc);
    for (size_t i = 0; i < rgb.size(); ++i) {
        if (td.is_float) {
            const float y = lum(rgb[i]);
            img[i] = td.scale * (td.gamma ? inverse_gamma(y) : y);
        } else {
            for (int k = 0; k < 3; ++k) img[i * 3 + k] = td.scale * (td.gamma ? inverse_gamma(rgb[i].c[k]) : rgb[i].c[k]);
        }
    }
    resample_pow2(td.wrap, nc, &w, &h, &img);
    std::memset(out, 0, sizeof(*out));
    out->offset = (int)(texels->size() / 4);
    out->w = w;
    out->h = h;
    out->wrap = td.wrap;
    out->isFloat = td.is_float ? 1 : 0;
    out->su = td.su; out->sv = td.sv; out->du = td.du; out->dv = td.dv;
    for (size_t i = 0; i < (size_t)w * h; ++i)
        for (int k = 0; k < 4; ++k) texels->push_back(k < nc ? img[i * nc + k] : 0.f);
}

void build_infinite_light(const pbr_light_desc& ld, const float worldMin[3], const float worldMax[3],
                          InfiniteHost* out, float power[3]) {
    // texels = L × image (InfiniteAreaLight.cpp:12-40); no image → a 1×1 map of L
    int w = 1, h = 1;
    std::vector<RGB> tex;
    if (ld.env_data && ld.env_width > 0 && ld.env_height > 0) {
        if (ld.env_components < 3) throw std::invalid_argument("InfiniteAreaLight image needs >= 3 components");
        w = ld.env_width;
        h = ld.env_height;
        tex.resize((size_t)w * h);
        for (size_t i = 0; i < tex.size(); ++i)
            for (int k = 0; k < 3; ++k) tex[i].c[k] = ld.Le[k] * ld.env_data[i * ld.env_components + k];
    } else {
        tex.assign(1, RGB{{ld.Le[0], ld.Le[1], ld.Le[2]}});
    }
    Pyramid P;
    build_pyramid(w, h, std::move(tex), &P);
    const int W = P.W[0], H = P.H[0];
    out->w = W;
    out->h = H;
    out->tex.assign((size_t)W * H * 4, 0.f);
    for (size_t i = 0; i < (size_t)W * H; ++i)
        for (int k = 0; k < 3; ++k) out->tex[4 * i + k] = P.lv[0][i].c[k];
    // Distribution2D over Lookup(center, 0).y() · sinθ (InfiniteAreaLight.cpp:46-58)
    std::vector<float> img((size_t)W * H);
    for (int v = 0; v < H; ++v) {
        float vp = (v + .5f) / (float)H;
        float sinTheta = t_sin(kPi * (v + .5f) / H);
        for (int u = 0; u < W; ++u) {
            float up = (u + .5f) / (float)W;
            img[u + (size_t)v * W] = lum(P.lookup(up, vp, 0.f));
            img[u + (size_t)v * W] *= sinTheta;
        }
    }
    out->condFunc = img;
    out->condCdf.assign((size_t)H * (W + 1), 0.f);
    out->margFunc.assign(H, 0.f);
    for (int v = 0; v < H; ++v) {
        std::vector<float> cdf;
        dist1d(&img[(size_t)v * W], W, &cdf, &out->margFunc[v]);
        std::copy(cdf.begin(), cdf.end(), out->condCdf.begin() + (size_t)v * (W + 1));
    }
    dist1d(out->margFunc.data(), H, &out->margCdf, &out->margInt);
    std::memcpy(out->l2w, ld.light_to_world.m, 64);
    std::memcpy(out->w2l, ld.light_to_world.m_inv, 64);
    // Preprocess: scene.WorldBound().BoundingSphere (Geometry.h:1250-1254)
    f3 lo = mk(worldMin[0], worldMin[1], worldMin[2]), hi = mk(worldMax[0], worldMax[1], worldMax[2]);
    f3 c = (lo + hi) * 0.5f;
    bool inside = c.x >= lo.x && c.x <= hi.x && c.y >= lo.y && c.y <= hi.y && c.z >= lo.z && c.z <= hi.z;
    out->worldRadius = inside ? len(c - hi) : 0.f;
    // Power (InfiniteAreaLight.cpp:63-67)
    RGB mid = P.lookup(.5f, .5f, .5f);
    float k = (4 * kPi) * kPi * out->worldRadius * out->worldRadius;
    for (int i = 0; i < 3; ++i) power[i] = k * mid.c[i];
}

}  // namespace pbr
