// pbr_material.h — Material::ComputeScatteringFunctions (Material/*.cpp) as a lobe template, shared by
// the host (constant textures, folded once at upload: pbr_scene.cpp) and the device (image textures,
// evaluated per hit: pbr_device.h textured_template).
#pragma once
#include "pbr_layout.h"
#include "pbr_math.h"

namespace pbr {

// A material's parameters with every texture already evaluated (Texture::Evaluate at the hit).
struct MatParams {
    int type;                     // pbr_material_type
    float Kd[3], Kr[3], Kt[3], Ks[3];
    float sigma, eta;
    float metal_eta[3], metal_k[3];
    float roughness, uroughness, vroughness;
    int has_uv_roughness, remap_roughness;
};

// A textured material: its constant parameters and, per pbr_texture_slot, the texture (-1: constant).
struct TexMat {
    MatParams p;
    int tex[6];
};

PBR_HD float roughness_to_alpha(float roughness) {   // Microfacet.h:78-83
    roughness = mx(roughness, (float)1e-3);
    float x = t_log(roughness);
    return 1.62142f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x + 0.000640711f * x * x * x * x;
}
PBR_HD void mt_put3(float* d, const float* s) { d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; }
PBR_HD bool mt_black3(const float* v) { return v[0] == 0.f && v[1] == 0.f && v[2] == 0.f; }
PBR_HD void mt_clamp3(float* d, const float* s) { for (int i = 0; i < 3; ++i) d[i] = clampf(s[i], 0, PBR_INF); }
PBR_HD Lobe lobe0() {
    Lobe l;
    int* w = (int*)&l;
    for (unsigned i = 0; i < sizeof(Lobe) / 4; ++i) w[i] = 0;
    return l;
}
PBR_HD void set_tr(Lobe& l, float ax, float ay) { l.ax = mx(float(0.001), ax); l.ay = mx(float(0.001), ay); }

// The BxDFs each material adds, allowMultipleLobes = multi.  Returns false for an unknown type.
PBR_HD bool material_template(const MatParams& m, bool multi, MatTemplate* out) {
    MatTemplate& t = *out;
    {
        int* w = (int*)&t;
        for (unsigned i = 0; i < sizeof(MatTemplate) / 4; ++i) w[i] = 0;
    }
    if (m.type == 0) return true;   // PBR_MAT_NONE: material == nullptr
    t.valid = 1;
    t.eta = 1;
    switch (m.type) {
    case 1: {   // MatteMaterial.cpp:13-28
        float r[3];
        mt_clamp3(r, m.Kd);
        float sig = clampf(m.sigma, 0, 90);
        if (!mt_black3(r)) {
            Lobe l = lobe0();
            mt_put3(l.R, r);
            l.type = BSDF_REFLECTION | BSDF_DIFFUSE;
            if (sig == 0) l.kind = L_LAMBERT;
            else {
                l.kind = L_OREN;
                float s = (kPi / 180) * sig;
                float s2 = s * s;
                l.A = 1.f - (s2 / (2.f * (s2 + 0.33f)));
                l.B = 0.45f * s2 / (s2 + 0.09f);
            }
            t.lobes[t.nLobes++] = l;
        }
        return true;
    }
    case 2: {   // Mirror.cpp:5-15
        float r[3];
        mt_clamp3(r, m.Kr);
        if (!mt_black3(r)) {
            Lobe l = lobe0();
            l.kind = L_SPEC_R; l.type = BSDF_REFLECTION | BSDF_SPECULAR; l.fresnel = FR_NOOP;
            mt_put3(l.R, r);
            t.lobes[t.nLobes++] = l;
        }
        return true;
    }
    case 3: {   // GlassMaterial.cpp:9-57
        t.eta = m.eta;
        float R[3], T[3];
        mt_clamp3(R, m.Kr);
        mt_clamp3(T, m.Kt);
        float ur = m.uroughness, vr = m.vroughness;
        if (mt_black3(R) && mt_black3(T)) return true;
        bool spec = ur == 0 && vr == 0;
        if (spec && multi) {
            Lobe l = lobe0();
            l.kind = L_FRESNEL_SPEC; l.type = BSDF_REFLECTION | BSDF_TRANSMISSION | BSDF_SPECULAR;
            mt_put3(l.R, R); mt_put3(l.T, T); l.etaA = 1.f; l.etaB = m.eta;
            t.lobes[t.nLobes++] = l;
            return true;
        }
        if (m.remap_roughness) { ur = roughness_to_alpha(ur); vr = roughness_to_alpha(vr); }
        if (!mt_black3(R)) {
            Lobe l = lobe0();
            mt_put3(l.R, R); l.fresnel = FR_DIEL; l.fEtaI = 1.f; l.fEtaT = m.eta;
            if (spec) { l.kind = L_SPEC_R; l.type = BSDF_REFLECTION | BSDF_SPECULAR; }
            else { l.kind = L_MF_R; l.type = BSDF_REFLECTION | BSDF_GLOSSY; set_tr(l, ur, vr); }
            t.lobes[t.nLobes++] = l;
        }
        if (!mt_black3(T)) {
            Lobe l = lobe0();
            mt_put3(l.T, T); l.etaA = 1.f; l.etaB = m.eta;
            if (spec) { l.kind = L_SPEC_T; l.type = BSDF_TRANSMISSION | BSDF_SPECULAR; }
            else { l.kind = L_MF_T; l.type = BSDF_TRANSMISSION | BSDF_GLOSSY; set_tr(l, ur, vr); }
            t.lobes[t.nLobes++] = l;
        }
        return true;
    }
    case 4: {   // MetalMaterial.cpp:25-43
        float ur = m.has_uv_roughness ? m.uroughness : m.roughness;
        float vr = m.has_uv_roughness ? m.vroughness : m.roughness;
        if (m.remap_roughness) { ur = roughness_to_alpha(ur); vr = roughness_to_alpha(vr); }
        Lobe l = lobe0();
        l.kind = L_MF_R; l.type = BSDF_REFLECTION | BSDF_GLOSSY;
        l.R[0] = l.R[1] = l.R[2] = 1.f;
        l.fresnel = FR_COND;
        l.cEtaI[0] = l.cEtaI[1] = l.cEtaI[2] = 1.f;
        mt_put3(l.cEtaT, m.metal_eta);
        mt_put3(l.cK, m.metal_k);
        set_tr(l, ur, vr);
        t.lobes[t.nLobes++] = l;
        return true;
    }
    case 5: {   // PlasticMaterial.cpp:8-30
        float kd[3], ks[3];
        mt_clamp3(kd, m.Kd);
        if (!mt_black3(kd)) {
            Lobe l = lobe0();
            l.kind = L_LAMBERT; l.type = BSDF_REFLECTION | BSDF_DIFFUSE;
            mt_put3(l.R, kd);
            t.lobes[t.nLobes++] = l;
        }
        mt_clamp3(ks, m.Ks);
        if (!mt_black3(ks)) {
            float r = m.roughness;
            if (m.remap_roughness) r = roughness_to_alpha(r);
            Lobe l = lobe0();
            l.kind = L_MF_R; l.type = BSDF_REFLECTION | BSDF_GLOSSY;
            mt_put3(l.R, ks);
            l.fresnel = FR_DIEL; l.fEtaI = 1.5f; l.fEtaT = 1.f;
            set_tr(l, r, r);
            t.lobes[t.nLobes++] = l;
        }
        return true;
    }
    default:
        return false;
    }
}

}  // namespace pbr
