// pbr_wavefront_volpath.h — wavefront schedule for VolPathIntegrator::Li (VolPathIntegrator.cpp:
// 21-107) over homogeneous media.  Included after pbr_wavefront_path.h; shares its queues, camera
// kernel, probe kernel (the BSDF/phase-sampled ray of EstimateDirect is a plain Scene::Intersect,
// Integrator.cpp:159) and finish.  Differences from the Path schedule:
//   * rays carry their medium (packed into the queue's dim word);
//   * every bounce first samples the ray's medium (HomogeneousMedium::Sample, two Get1D), which can
//     turn the bounce into a medium interaction (HG phase function instead of a BSDF);
//   * the light sample's visibility is VisibilityTester::Tr (Light.cpp:31-47): k_wfv_tr walks the
//     shadow ray through medium interfaces, multiplying homogeneous transmittance, and the
//     resolve multiplies Li by it before the !IsBlack test, in the reference's op order.
#pragma once

constexpr int kWfvDelta = 8;   // dFlags: the estimate's light is a delta light

struct WfvParams {
    WfpParams X;
    // transmittance-walk queue (segmented): origin+tMax, dir + medium, target p, pError, n, the
    // direct record it fills
    float4* to; float4* td; float4* tp; float4* te; float4* tn; int* tid; int* trSeg;
    // direct records (at the direct queue position, like WfpParams' d*)
    float4* dLiA;          // light sample Li.rgb, lightPdf
    float4* dTr;           // transmittance to the light sample
    float* dWA;            // MIS weight of the light sample
    int anyHitTr;          // every primitive has a material: the walk is one any-hit query
};

__device__ __forceinline__ int pack_vol(int dim, int bounces, bool specular, int medium) {
    return pack_path(dim, bounces, specular) | ((medium + 1) << 24);
}

// Scene::Intersect's medium interface on a hit (Primitive.cpp:30-34)
__device__ __forceinline__ void set_interface(const DeviceScene& S, Isect* it, int rayMedium) {
    int4 info = S.primInfo[it->slot];
    int mi = (int)(short)(info.w & 0xffff), mo = (int)(short)((info.w >> 16) & 0xffff);
    if (mi != mo) { it->medIn = mi; it->medOut = mo; }
    else { it->medIn = rayMedium; it->medOut = rayMedium; }
}

// Waves per SIMD (C5: 2 → 1940 ms, 3 → 1832-1846, 4 → 1898)
#ifndef PBR_WFV_OCC
#define PBR_WFV_OCC 3
#endif
// The material pass of a queued VolPath ray (the classed shade): a ray inside a medium goes to pass
// 0, as do misses and material-less hits; a ray outside media goes to its hit material's pass.
// Pass 0 is the medium pass (k_wfv_shade<0, …, CLASSED>: no BSDF lobes): it samples the medium of
// every ray inside one and shades the medium events; a ray that reaches a surface with a material
// instead leaves its state after the medium sample (β, the sampler dimension) in its queue entry
// and is filed, flagged kDeferred, into that material's pass, which continues it from there.
__device__ __forceinline__ int entry_pass_vol(const WfpParams& X, int q) {
    if (((__float_as_int(X.W.cur.d[q].w) >> 24) & 0xff) != 0) return 0;   // in a medium (pack_vol)
    return entry_pass(X, q);
}
constexpr int kDeferred = (int)0x80000000;   // pass-list entry: the medium pass sampled its medium
// CLASSED: as k_wfp_shade's (pass 0 classifies and files, later passes read their lists)
template <int LOBES, bool MATS_LDS, int OCC = PBR_WFV_OCC, int SMP = -1, bool CLASSED = false>   // SMP: as k_wfp_shade's
__global__ __launch_bounds__(256, OCC) void k_wfv_shade(WfvParams V, int level0, int pass) {
    constexpr bool kMediumPass = CLASSED && LOBES == 0;   // pass 0 of the classed shade
    WfpParams& X = V.X;
    WfParams& W = X.W;
    const KParams& P = W.P;
    const DeviceScene& S = P.S;
    stage_halton_lds(P.smp);
    const MatTemplate* mats = S.materials;
    if constexpr (MATS_LDS) {
        constexpr int words = (int)(sizeof(MatTemplate) / 4);
        const int n = 2 * S.nMaterials * words;
        const uint32_t* src = (const uint32_t*)S.materials;
        uint32_t* dst = (uint32_t*)s_mats;
        for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
        mats = s_mats;
    }
    __shared__ int s_push[4];   // transmittance walk, probe, direct, next
    __shared__ int s_list[8];   // the classed shade's pass 0: entries filed into passes 1..
    if (threadIdx.x < 4) {
        int v = 0;   // (a later pass of the classed shade continues the segments)
        if (CLASSED && pass > 0) {
            const int b = wf_block();
            v = threadIdx.x == 0 ? V.trSeg[b] : threadIdx.x == 1 ? X.probeSeg[b] : threadIdx.x == 2 ? X.directSeg[b] : W.next.segCount[b];
        }
        s_push[threadIdx.x] = v;
    }
    __syncthreads();
    const int n = level0 ? W.nSamples : seg_scan(W.cur.segCount);
    const int stride = gridDim.x * blockDim.x;
    const int nIter = (n + stride - 1) / stride;
    const int base = wf_block() * W.segCap;
    // one queued ray; every lane of the workgroup calls it together (wave_push needs convergent lanes).
    // (As a lambda the body's registers are allocated apart from the loop's: k_wfp_shade 149 → 115
    // VGPRs for C3, profiles/r5_classed_shade_ab.log.)
    // deferredIn: the medium pass left this entry after its medium sample.  Returns the pass a
    // medium-pass entry was deferred to (0: shaded here).
    auto shade = [&](const bool active, const int q, const bool deferredIn) -> int {
        // Two phases around the light-estimate pushes (as k_wfp_shade): the record, the transmittance
        // walk and the probe ray are written before the path's phase-function / BSDF sample.
        bool pushTr = false, pushProbe = false, pushDirect = false, pushNext = false;
        int id = 0, dim = 0, bounces = 0;
        bool specularBounce = false;
        Ray cont, ray;
        rgb L, beta;
        float etaScale = 1.f;
        uint32_t sIndex = 0;
        SState st;
        st.index = 0; st.sid = 0; st.dim = 0; st.px = st.py = 0;
        Isect isect;   // the surface hit, or the medium interaction once one is sampled
        BSDF bsdf;
        MatTemplate texLocal;   // a textured material's per-hit lobes (make_bsdf)
        bool estimate = false, mediumEvent = false;
        float g = 0;
        int di = -1;
        int deferTo = 0;
        {
        Ray shadow, probe;
        VisPt vis;
        rgb fA, fB, Li;
        float pmfD = 0.f, weightA = 0.f, weightB = 1.f, lightPdf = 0.f, scatPdfD = 0.f;
        int dflagsD = 0, lightD = 0;
        if (active) {
            float4 o = W.cur.o[q], d = W.cur.d[q], hr = W.cur.hit[q];
            id = level0 ? q : W.cur.id[q];
            const int dd = __float_as_int(d.w);
            dim = dd & 0xffff;
            bounces = (dd >> 16) & 0x7f;
            specularBounce = (dd >> 23) & 1;
            const int medium = ((dd >> 24) & 0xff) - 1;
            ray = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, medium);
            const int slot = __float_as_int(hr.x);
            const bool found = slot >= 0;
            if (level0 && !deferredIn) {
                L = sp(0.f); beta = sp(1.f); etaScale = 1.f;
                sIndex = W.sampleIndex[q];
            } else {
                const float4 a = W.cur.s0[q], b = W.cur.s1[q];
                L = sp3(a.x, a.y, a.z); beta = sp3(a.w, b.x, b.y);
                etaScale = b.z;
                sIndex = __float_as_uint(b.w);
            }
            st.index = sIndex;
            st.sid = id;   // ≡ the sample number mod spp (pixel-major ids)
            st.dim = dim;
            if (found) {
                int flags = __float_as_int(S.triVerts[3 * (size_t)slot].w);
                if (flags & PRIM_SPHERE) sphere_si(S.spheres[__float_as_int(S.triVerts[3 * (size_t)slot].x)], ray, ray.tMax, &isect);
                else triangle_si(S, slot, ray, hr.y, hr.z, hr.w, flags, &isect);
                isect.slot = slot;
                set_interface(S, &isect, ray.medium);
            }
            // HomogeneousMedium::Sample (HomogeneousMedium.cpp:15-45)
            if (ray.medium >= 0 && !deferredIn) {
                const float* md = S.media + 10 * ray.medium;
                int channel = (int)(get1d<true, SMP>(P.smp, st) * 3);
                if (channel > 2) channel = 2;
                float dist = -t_log(1 - get1d<true, SMP>(P.smp, st)) / md[6 + channel];
                float t = mn(dist / len(ray.d), ray.tMax);
                bool sampled = t < ray.tMax;
                if (sampled) {
                    // MediumInteraction: it replaces the surface record, which a medium event never
                    // reads again (one record, no pointer select between two: that kept both in scratch)
                    isect.p = ray.o + ray.d * t; isect.wo = -ray.d; isect.n = mk(0, 0, 0); isect.pError = mk(0, 0, 0);
                    isect.sn = mk(0, 0, 0); isect.dpdu = mk(0, 0, 0);
                    isect.medIn = isect.medOut = ray.medium; isect.slot = -1;
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
            if constexpr (kMediumPass) {
                // a surface with a material reached from inside the medium: its material's pass
                // continues the path from the state after the medium sample
                if (ray.medium >= 0 && !mediumEvent && found) {
                    const int mat = S.primInfo[slot].y;
                    if (mat >= 0 && mats[2 * mat + 1].valid) deferTo = X.matPass[mat];
                }
                if (deferTo > 0) {
                    W.cur.d[q] = make_float4(d.x, d.y, d.z, __int_as_float(pack_vol(st.dim, bounces, specularBounce, ray.medium)));
                    W.cur.s0[q] = make_float4(L.r, L.g, L.b, beta.r);
                    W.cur.s1[q] = make_float4(beta.g, beta.b, etaScale, __uint_as_float(sIndex));
                }
            }
            bool alive = deferTo == 0 && !black(beta);
            if (alive && mediumEvent) {
                if (bounces >= P.maxDepth) alive = false;
                else estimate = true;
            } else if (alive) {
                if (bounces == 0 || specularBounce) {
                    if (found) L = L + beta * si_Le(S, isect, -ray.d);
                    else for (int k = 0; k < S.nInfinite; ++k) L = L + beta * light_Le(S, S.lights[S.infinite[k]], ray);
                }
                if (!found || bounces >= P.maxDepth) alive = false;
                else if (!make_bsdf<(LOBES & kTexturedLobes) != 0>(S, mats, isect, true, &bsdf, &texLocal)) {
                    cont = spawn_ray(isect, ray.d);   // bounces--; continue: no Russian roulette
                    pushNext = true;
                    alive = false;
                } else {
                    estimate = true;
                }
            }
            if (estimate && S.nLights > 0) {
                // UniformSampleOneLight(handleMedia = true) / EstimateDirect
                const Isect& ref = isect;
                float pmf;
                const int li = sample_light(S, get1d<true, SMP>(P.smp, st), &pmf);
                if (pmf != 0) {
                    float uL0, uL1, uS0, uS1;
                    get2d<true, SMP>(P.smp, st, &uL0, &uL1);
                    get2d<true, SMP>(P.smp, st, &uS0, &uS1);
                    const DLight& light = S.lights[li];
                    const bool delta = light.type == LT_POINT;
                    const int flagsNS = BSDF_ALL & ~BSDF_SPECULAR;
                    int dflags = delta ? kWfvDelta : 0;
                    f3 wi = mk(0, 0, 0);
                    float scatteringPdf = 0;
                    lightPdf = 0;
                    weightA = 0;
                    // Lambda(wo) of the microfacet lobes, once for the estimate's two strategies
                    const float lamL = mediumEvent ? kNoLambda : mf_lambda<LOBES>(bsdf, bsdf.to_local(ref.wo));
                    Li = sample_li(S, light, ref, uL0, uL1, &wi, &lightPdf, &vis);
                    fA = sp(0.f);
                    if (lightPdf > 0 && !black(Li)) {
                        if (!mediumEvent) {
                            fA = bsdf_f_pdf<LOBES>(bsdf, ref.wo, wi, flagsNS, &scatteringPdf, lamL) * absdot(wi, ref.sn);
                        } else {
                            fA = sp(phase_hg(dot(ref.wo, wi), g));
                        }
                        if (!black(fA)) {
                            float fp = 1 * lightPdf, gp = 1 * scatteringPdf;
                            weightA = (fp * fp) / (fp * fp + gp * gp);
                            shadow = spawn_ray_to(ref, vis.p, vis.pError, vis.n);
                            pushTr = true;
                            dflags |= kWfpAPending;
                        }
                    }
                    fB = sp(0.f);
                    weightB = 1.f;
                    if (!delta && !mediumEvent) {
                        // EstimateDirect's BSDF sample (Integrator.cpp:126-174).  Its value f·|cos| is
                        // only read when the sampled direction can reach the light — a specular
                        // sample, or Pdf_Li != 0 — so it is formed only then (the checks are pure,
                        // so their order does not change the outcome): most sampled directions miss
                        // a small area light and skip the sum over the lobes.
                        int stype = 0;
                        BsdfDraw draw;
                        if (bsdf_sample_dir<LOBES>(bsdf, ref.wo, &wi, uS0, uS1, &scatteringPdf, flagsNS, &stype, &draw, lamL) &&
                            scatteringPdf > 0) {
                            const bool sampledSpecular = (stype & BSDF_SPECULAR) != 0;
                            const float lp = sampledSpecular ? 0.f : pdf_li(S, light, ref, wi);
                            if (sampledSpecular || lp != 0) {
                                fB = bsdf_sample_sum<LOBES>(bsdf, ref.wo, wi, flagsNS, draw) * absdot(wi, ref.sn);
                                if (!black(fB)) {
                                    if (!sampledSpecular) {
                                        float fp = 1 * scatteringPdf, gp = 1 * lp;
                                        weightB = (fp * fp) / (fp * fp + gp * gp);
                                    }
                                    probe = spawn_ray(ref, wi);
                                    pushProbe = true;
                                    dflags |= kWfpBPending;
                                }
                            }
                        }
                    } else if (!delta) {
                        const bool sampledSpecular = false;
                        float p = hg_sample(g, ref.wo, &wi, uS0, uS1);
                        fB = sp(p);
                        scatteringPdf = p;
                        if (!black(fB) && scatteringPdf > 0) {
                            bool probeIt = true;
                            if (!sampledSpecular) {
                                float lp = pdf_li(S, light, ref, wi);
                                if (lp == 0) probeIt = false;
                                else {
                                    float fp = 1 * scatteringPdf, gp = 1 * lp;
                                    weightB = (fp * fp) / (fp * fp + gp * gp);
                                }
                            }
                            if (probeIt) {
                                probe = spawn_ray(ref, wi);
                                pushProbe = true;
                                dflags |= kWfpBPending;
                            }
                        }
                    }
                    if (dflags & (kWfpAPending | kWfpBPending)) {   // written at its queue position below
                        pmfD = pmf;
                        scatPdfD = scatteringPdf;
                        dflagsD = dflags;
                        lightD = li;
                        pushDirect = true;
                    }
                }
            }
        }
            // the estimate's record (beta at the estimate), its transmittance walk and probe ray
            di = base + wave_push(&s_push[2], pushDirect);
            if (pushDirect) {
                X.dA[di] = make_float4(fA.r, fA.g, fA.b, pmfD);
                V.dLiA[di] = make_float4(Li.r, Li.g, Li.b, lightPdf);
                V.dWA[di] = weightA;
                X.dB[di] = make_float4(fB.r, fB.g, fB.b, weightB);
                X.dBeta[di] = make_float4(beta.r, beta.g, beta.b, scatPdfD);
                X.dFlags[di] = dflagsD;
                X.dLight[di] = lightD;
            }
            const int ti = base + wave_push(&s_push[0], pushTr);
            if (pushTr) {
                V.to[ti] = make_float4(shadow.o.x, shadow.o.y, shadow.o.z, shadow.tMax);
                V.td[ti] = make_float4(shadow.d.x, shadow.d.y, shadow.d.z, __int_as_float(shadow.medium));
                if (!V.anyHitTr) {   // the walk's target; one any-hit query needs none of it
                    V.tp[ti] = make_float4(vis.p.x, vis.p.y, vis.p.z, 0.f);
                    V.te[ti] = make_float4(vis.pError.x, vis.pError.y, vis.pError.z, 0.f);
                    V.tn[ti] = make_float4(vis.n.x, vis.n.y, vis.n.z, 0.f);
                }
                V.tid[ti] = di;
            }
            const int pi = base + wave_push(&s_push[1], pushProbe);
            if (pushProbe) {
                X.po[pi] = make_float4(probe.o.x, probe.o.y, probe.o.z, probe.tMax);
                X.pd[pi] = make_float4(probe.d.x, probe.d.y, probe.d.z, 0.f);
                X.pid[pi] = di;
            }
        }
        if (active && deferTo == 0) {
            bool doRR = false;
            if (estimate) {
                if (mediumEvent) {   // HenyeyGreenstein::Sample_p, then the ray leaves the interaction
                    f3 wo = -ray.d, wi;
                    float u0, u1;
                    get2d<true, SMP>(P.smp, st, &u0, &u1);
                    hg_sample(g, wo, &wi, u0, u1);
                    cont = spawn_ray(isect, wi);
                    specularBounce = false;
                    doRR = true;
                } else {
                    const f3 wo = -ray.d;
                    f3 wi = mk(0, 0, 0);
                    float pdf = 0;
                    int flags = 0;
                    float u0, u1;
                    get2d<true, SMP>(P.smp, st, &u0, &u1);
                    rgb f = bsdf_sample<LOBES>(bsdf, wo, &wi, u0, u1, &pdf, BSDF_ALL, &flags);
                    if (!(black(f) || pdf == 0.f)) {
                        beta = beta * (f * absdot(wi, isect.sn) / pdf);
                        specularBounce = (flags & BSDF_SPECULAR) != 0;
                        if ((flags & BSDF_SPECULAR) && (flags & BSDF_TRANSMISSION)) {
                            float eta = bsdf.mt->eta;
                            etaScale *= (dot(wo, isect.n) > 0) ? (eta * eta) : 1 / (eta * eta);
                        }
                        cont = spawn_ray(isect, wi);
                        doRR = true;
                    }
                }
            }
            if (doRR) {
                bool stop = false;
                rgb rrBeta = beta * etaScale;
                if (maxval(rrBeta) < P.rrThreshold && bounces > 3) {
                    float qq = mx((float).05, 1 - maxval(rrBeta));
                    if (get1d<true, SMP>(P.smp, st) < qq) stop = true;
                    else beta = beta / (1 - qq);
                }
                if (!stop) {
                    pushNext = true;
                    bounces += 1;
                }
            }
            dim = st.dim;
            if (X.lastLevel) pushNext = false;   // never taken: no bounce is left at the last level
            if (!pushNext) X.stL[id] = make_float4(L.r, L.g, L.b, 0.f);   // the path ends here
        }
        const int ni = base + wave_push(&s_push[3], pushNext);
        if (pushNext) {
            W.next.o[ni] = make_float4(cont.o.x, cont.o.y, cont.o.z, cont.tMax);
            W.next.d[ni] = make_float4(cont.d.x, cont.d.y, cont.d.z, __int_as_float(pack_vol(dim, bounces, specularBounce, cont.medium)));
            W.next.id[ni] = id;
            W.next.s0[ni] = make_float4(L.r, L.g, L.b, beta.r);
            W.next.s1[ni] = make_float4(beta.g, beta.b, etaScale, __uint_as_float(sIndex));
        }
        if (pushDirect) X.dTgt[di] = pushNext ? ni : ~id;
        return deferTo;
    };
    // the medium pass files a deferred entry into its material's pass list (convergent lanes)
    auto file_deferred = [&](const int dp, const int q) {
        if constexpr (kMediumPass) {
            for (int c = 1; c < X.nPasses; ++c) {
                const int at = wave_push(&s_list[c - 1], dp == c);
                if (dp == c) X.passList[(size_t)(c - 1) * X.passStride + base + at] = q | kDeferred;
            }
        }
    };
    if constexpr (!CLASSED) {
        for (int it = 0; it < nIter; ++it) {   // uniform trip count: wave_push needs convergent lanes
            const int i = it * stride + wf_block() * blockDim.x + threadIdx.x;
            const bool active = i < n;
            const int q = level0 ? i : seg_pos_dense(W.segCap, i, n);
            shade(active, active ? q : 0, false);
        }
    } else if (pass > 0) {   // this pass's list, filed by pass 0
        const int cnt = X.passCnt[(pass - 1) * kWfBlocks + wf_block()];
        const int* list = X.passList + (size_t)(pass - 1) * X.passStride + base;
        for (int k0 = 0; k0 < cnt; k0 += 256) {
            const int k = k0 + (int)threadIdx.x;
            const bool active = k < cnt;
            const int e = active ? list[k] : 0;
            shade(active, e & ~kDeferred, (e & kDeferred) != 0);
        }
    } else {   // pass 0: k_wfp_shade's ring, and the other passes' lists
        __shared__ int s_ring[512];
        __shared__ int s_tail;
        if (threadIdx.x == 0) s_tail = 0;
        if (threadIdx.x < 8) s_list[threadIdx.x] = 0;
        __syncthreads();
        int head = 0;
        for (int it = 0; it < nIter; ++it) {
            const int i = it * stride + wf_block() * blockDim.x + threadIdx.x;
            const int qd = level0 ? i : seg_pos_dense(W.segCap, i, n);
            const int q = i < n ? qd : 0;
            const int cls = i < n ? entry_pass_vol(X, q) : -1;
            for (int c = 1; c < X.nPasses; ++c) {
                const int at = wave_push(&s_list[c - 1], cls == c);
                if (cls == c) X.passList[(size_t)(c - 1) * X.passStride + base + at] = q;
            }
            const int at = wave_push(&s_tail, cls == 0);
            if (cls == 0) s_ring[at & 511] = q;
            __syncthreads();
            const bool full = s_tail - head >= 256;
            const int qq = full ? s_ring[(head + threadIdx.x) & 511] : 0;
            __syncthreads();
            if (full) {
                file_deferred(shade(true, qq, false), qq);
                head += 256;
            }
        }
        __syncthreads();
        const int tail = s_tail;
        if (head < tail) {
            const bool active = head + (int)threadIdx.x < tail;
            const int qq = active ? s_ring[(head + threadIdx.x) & 511] : 0;
            file_deferred(shade(active, qq, false), qq);
        }
        if constexpr (kMediumPass) __syncthreads();   // every wave's deferred entries are filed
        if ((int)threadIdx.x + 1 < X.nPasses) X.passCnt[threadIdx.x * kWfBlocks + wf_block()] = s_list[threadIdx.x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        V.trSeg[wf_block()] = s_push[0];
        X.probeSeg[wf_block()] = s_push[1];
        X.directSeg[wf_block()] = s_push[2];
        W.next.segCount[wf_block()] = s_push[3];
    }
}

// VisibilityTester::Tr (Light.cpp:31-47): walk to the light sample through medium interfaces.
// Its lane-refill walk fetches near/far plane rows (PBR_NF_ROWS) although that spills 9 VGPRs here:
// C5 transmittance 340.8 ms/frame without the rows, 327.3 with them at 5 workgroups per CU (no
// spill), 321.5 with them at 6 (kept; serial schedule, profiles/r6_ab_tr.log).
template <int SHORT>
__global__ __launch_bounds__(256, PBR_REFILL_OCC_TR) void k_wfv_tr(WfvParams V) {
    WfpParams& X = V.X;
    const DeviceScene& S = X.W.P.S;
    const int n = seg_scan(V.trSeg);
    if constexpr (kRefill > 0 && SHORT > 0 && kQuadTraversal) {
        if (V.anyHitTr) {   // the walk is one any-hit query (below): lane-refill traversal
            traverse_stream<true, SHORT>(   // (not kAnyShort: see pbr_device.h)
                S, n, X.W.segCap,
                [&](int q, int* key) {
                    *key = q;
                    const float4 o = V.to[q], d = V.td[q];
                    return mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, __float_as_int(d.w));
                },
                [&](int q, bool hit, const Ray& ray, const HitRec&) {
                    rgb Tr = sp(1.f);
                    if (hit) Tr = sp(0.0f);
                    else if (ray.medium >= 0) Tr = Tr * medium_tr(S, ray.medium, ray);
                    V.dTr[V.tid[q]] = make_float4(Tr.r, Tr.g, Tr.b, 0.f);
                },
                X.W.prof, KP_WFV_TR);
            return;
        }
    }
    for (int i0 = wf_block() * blockDim.x + ((int)threadIdx.x & ~63); i0 < n; i0 += gridDim.x * blockDim.x) {   // per wave
        const int i = i0 + (int)__lane_id();
        const int q = seg_pos_dense(X.W.segCap, i, n);
        if (i >= n) continue;
        float4 o = V.to[q], d = V.td[q], tp = V.tp[q], te = V.te[q], tn = V.tn[q];
        const f3 p1 = mk(tp.x, tp.y, tp.z), e1 = mk(te.x, te.y, te.z), n1 = mk(tn.x, tn.y, tn.z);
        Ray ray = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, __float_as_int(d.w));
        rgb Tr = sp(1.f);
        if (V.anyHitTr) {
            // Every surface has a material, so the walk's first hit, if any, returns 0 and a miss
            // multiplies the medium's Tr over the unchanged ray: whether anything is hit is all that
            // matters, and IntersectP answers that (same boolean, same ray on a miss).
            HitRec h;
            Counters c;
            if (traverse<true, false, SHORT>(S, ray, &h, &c)) Tr = sp(0.0f);
            else if (ray.medium >= 0) Tr = Tr * medium_tr(S, ray.medium, ray);
            V.dTr[V.tid[q]] = make_float4(Tr.r, Tr.g, Tr.b, 0.f);
            continue;
        }
        for (int guard = 0;; ++guard) {
            HitRec h;
            Counters c;
            const bool hit = traverse<false, false, SHORT>(S, ray, &h, &c);
            if (hit && S.primInfo[h.slot].y >= 0) { Tr = sp(0.0f); break; }
            if (ray.medium >= 0) Tr = Tr * medium_tr(S, ray.medium, ray);
            if (!hit) break;
            if (guard == kMaxTrCrossings) { atomicOr(S.guard, kGuardTransmittance); break; }
            Isect isect;
            int flags = __float_as_int(S.triVerts[3 * (size_t)h.slot].w);
            if (flags & PRIM_SPHERE) sphere_si(S.spheres[__float_as_int(S.triVerts[3 * (size_t)h.slot].x)], ray, ray.tMax, &isect);
            else triangle_si(S, h.slot, ray, h.b0, h.b1, h.b2, flags, &isect);
            isect.slot = h.slot;
            set_interface(S, &isect, ray.medium);
            ray = spawn_ray_to(isect, p1, e1, n1);
        }
        V.dTr[V.tid[q]] = make_float4(Tr.r, Tr.g, Tr.b, 0.f);
    }
}

// Ld = [f·(Li·Tr)·w/lightPdf if Li·Tr is not black] + [f·Li·w/scatteringPdf if Li is not black];
// L += beta · (Ld / pmf)
__global__ __launch_bounds__(256) void k_wfv_resolve(WfvParams V) {
    WfpParams& X = V.X;
    const int n = seg_scan(X.directSeg);
    for (int i0 = wf_block() * blockDim.x + ((int)threadIdx.x & ~63); i0 < n; i0 += gridDim.x * blockDim.x) {   // per wave
        const int i = i0 + (int)__lane_id();
        const int di = seg_pos_dense(X.W.segCap, i, n);
        if (i >= n) continue;
        const int fl = X.dFlags[di];
        const float4 a = X.dA[di], bt = X.dBeta[di];
        rgb Ld = sp(0.f);
        if (fl & kWfpAPending) {
            const float4 la = V.dLiA[di], tr = V.dTr[di];
            const rgb Lt = sp3(la.x, la.y, la.z) * sp3(tr.x, tr.y, tr.z);
            if (!black(Lt)) {
                const rgb fA = sp3(a.x, a.y, a.z);
                if (fl & kWfvDelta) Ld = Ld + fA * Lt / la.w;
                else Ld = Ld + fA * Lt * V.dWA[di] / la.w;
            }
        }
        if (fl & kWfpBPending) {
            const float4 li = X.dLi[di], b = X.dB[di];
            const rgb Li2 = sp3(li.x, li.y, li.z);
            if (!black(Li2)) Ld = Ld + sp3(b.x, b.y, b.z) * Li2 * b.w / bt.w;
        }
        const rgb beta = sp3(bt.x, bt.y, bt.z);
        add_direct(X, X.dTgt[di], beta * (Ld / a.w));
    }
}
