// pbr_wavefront_path.h — wavefront schedule for PathIntegrator::Li (PathIntegrator.cpp:32-110) with
// UniformSampleOneLight / EstimateDirect (Integrator.cpp:46-177).  Included by pbr_kernels.hip
// after pbr_wavefront.h (queues, segment scan, wave_push, the camera/extend kernels).
//
// Per bounce k:
//   k_wfp_shade    emission (bounce 0 / after specular), BSDF, the one-light estimate's two
//                  candidate terms — light sample (needs a shadow ray) and BSDF sample (needs a
//                  probe ray) — and the continuation (BSDF sample, beta update, Russian roulette)
//   k_wfp_shadow   any-hit for the light-sample rays → "visible" flag in the direct record
//   k_wfp_probe    closest hit for the BSDF-sample rays → the radiance the sampled light shows there
//   k_wfp_resolve  Ld = [A if visible] + [f·Li·weight/scatteringPdf]; L += beta · (Ld / pmf)
//   k_wf_extend    closest hit for the continuation queue (shared with Whitted)
// then k_wfp_finish sums each pixel's per-sample L in sample order and runs the film.
//
// The path state — L, beta, etaScale and the sample's global index — travels with the ray in the
// queues (WfQueue s0/s1, compacted with the ray), and the direct-light estimate of bounce k is a
// record at its own position of the direct queue, which the shadow/probe entries point at: every
// kernel reads and writes its queue entries densely instead of gathering per-sample state by
// sample id from a compacted queue (which moved 3.5-8x the algorithmic bytes: partial lines).
// A path's L leaves the queues once, when the path ends (stL[id], read by the finish).  The
// estimate's record names where L is at resolve time — the continuation entry the same shade
// pushed, or stL[id] — and resolve adds the direct term there.  Every L update therefore happens
// in the reference's order (emission of bounce k, direct light of bounce k, emission of bounce
// k+1, ...), so the per-sample radiance is bit-identical to the recursive megakernel's.  Sampler
// dimensions travel in the ray queue.
#pragma once

constexpr int kWfpAPending = 1, kWfpBPending = 2, kWfpVisible = 4;

struct WfpParams {
    WfParams W;            // queues (cur/next rays with the path state, shadow), chunk geometry, sample index table
    // probe queue (segmented): origin+tMax, dir, the direct record it fills
    float4* po; float4* pd; int* pid; int* probeSeg;
    int* directSeg;        // direct-light records, segmented like the queues (at the shade's push position)
    float4* stL;           // the finished path's L.rgb, per sample (the finish's input)
    float4* dA;            // light-sample term f·Li·w/lightPdf (if unoccluded), pmf
    float4* dB;            // BSDF-sample f (× |cos|), weight
    float4* dBeta;         // beta at the estimate, scatteringPdf
    float4* dLi;           // probe result: Li at the BSDF-sampled direction
    int* dFlags;           // kWfp* bits
    int* dLight;           // light index of the estimate
    int* dTgt;             // where the path's L is when the estimate resolves: the continuation's
                           // position in the next queue, or ~id (stL[id]) when the path ended
    int lastLevel;         // this shade is the schedule's last: a continuation ends the path instead
    const int* matPass;    // the classed shade (CLASSED): the pass that shades each material's hits
    int* passList;         // ... the queue positions of passes 1.. ([pass - 1][segmented], filed by pass 0)
    int* passCnt;          // ... their counts ([pass - 1][workgroup])
    int passStride;        // ... entries per pass list
    int nPasses;
};

// The material pass of a queued hit (the classed shade): misses and material-less hits go to pass 0.
__device__ __forceinline__ int entry_pass(const WfpParams& X, int q) {
    const int slot = __float_as_int(X.W.cur.hit[q].x);
    if (slot < 0) return 0;
    const int mat = X.W.P.S.primInfo[slot].y;
    return mat < 0 ? 0 : X.matPass[mat];
}

__device__ __forceinline__ int pack_path(int dim, int bounces, bool specular) {
    return (dim & 0xffff) | ((bounces & 0x7f) << 16) | (specular ? (1 << 23) : 0);
}

template <int SHORT>
__global__ __launch_bounds__(256, PBR_TRAV_OCC) void k_wfp_camera_extend(WfpParams X) {
    WfParams& W = X.W;
    const KParams& P = W.P;
    int q = wf_block() * blockDim.x + threadIdx.x;
    if (q >= W.nSamples) return;
    int lp = q / P.spp, s = q - lp * P.spp;
    int x, y;
    pixel_xy(P, W.chunkPix0 + lp, &x, &y);
    SState st;
    st.index = sample_index(P.smp, x, y, s).lo;
    st.sid = s;
    st.dim = 0;
    st.px = x;
    st.py = y;
    Ray r = camera_sample_ray(P, st, x, y);
    HitRec h;
    Counters c;
    bool hit;
    if constexpr (kPacket && kQuadTraversal) {   // a wave holds (part of) one pixel's samples
        h.slot = -1; h.b0 = h.b1 = h.b2 = 0.f;
        hit = traverse_wave<false>(P.S, r, &h, true);
    } else {
        hit = traverse<false, false, SHORT>(P.S, r, &h, &c);
    }
    trav_diag(W.prof, KP_WFP_CAMERA, h);
    W.cur.o[q] = make_float4(r.o.x, r.o.y, r.o.z, r.tMax);
    W.cur.d[q] = make_float4(r.d.x, r.d.y, r.d.z, __int_as_float(pack_path(st.dim, 0, false)));
    W.cur.hit[q] = make_float4(__int_as_float(hit ? h.slot : -1), h.b0, h.b1, h.b2);
    W.sampleIndex[q] = st.index;   // the level-0 state (L = 0, beta = 1, etaScale = 1) is implied
}

// (A workgroup-local stable sort of each iteration's 256 shading events by miss / medium / material
// before shading was measured and removed: bit-identical, but C4 7711 → 7865 ms, C5 1373 → 1429,
// C3 269.7 → 270.8 — its barriers and key loads cost more than the divergence they removed.)

// One bounce of PathIntegrator::Li for every queued ray.
// Waves per SIMD: 3 for either lobe set (all lobes, C4: 2 → 9.58 s, 3 → 8.86 s, 4 → 9.32 s)
#ifndef PBR_WFP_OCC
#define PBR_WFP_OCC 3
#endif
// the Lambert + mirror kernel on Sobol frames (C3) and the classed shade's Lambert pass
#ifndef PBR_WFP_OCC_MM
#define PBR_WFP_OCC_MM PBR_WFP_OCC
#endif
#ifndef PBR_WFP_OCC_L
#define PBR_WFP_OCC_L PBR_WFP_OCC
#endif
// SMP: the frame's sampler type when the launch knows it (the other samplers' code — and the kernel
// parameters it reads, which otherwise spill from SGPRs into VGPR lanes — is compiled out), else -1.
// CLASSED: one of several launches per bounce, each shading the hits of the materials whose lobe set
// it is compiled for (X.matPass, pass `pass`).  Pass 0 walks the workgroup's queue entries as before,
// gathers its own into an LDS ring and shades them 256 at a time, and files every other entry's
// position in the list of its pass; a later pass shades its list, dense, 256 at a time.  So every
// wave runs one material class with that class's registers, and only pass 0 reads every entry's
// hit to classify it.  Pushes continue the segment counts of the pass before.
// Entries land in the queues in another order, which nothing depends on (records are indexed by
// sample or by queue position, and every L update keeps its order: pbr_wavefront_path.h header).
template <int LOBES, bool MATS_LDS, int OCC = PBR_WFP_OCC, int SMP = -1, bool CLASSED = false>
__global__ __launch_bounds__(256, OCC) void k_wfp_shade(WfpParams X, int level0, int pass) {
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
    __shared__ int s_push[4];   // shadow, probe, direct, next
    if (threadIdx.x < 4) {
        int v = 0;   // (a later pass of the classed shade continues the segments)
        if (CLASSED && pass > 0) {
            const int b = wf_block();
            v = threadIdx.x == 0 ? W.shadowSeg[b] : threadIdx.x == 1 ? X.probeSeg[b] : threadIdx.x == 2 ? X.directSeg[b] : W.next.segCount[b];
        }
        s_push[threadIdx.x] = v;
    }
    __syncthreads();
    const int n = level0 ? W.nSamples : seg_scan(W.cur.segCount);
    const int stride = gridDim.x * blockDim.x;
    const int nIter = (n + stride - 1) / stride;
    const int base = wf_block() * W.segCap;
    // one queued ray; every lane of the workgroup calls it together (wave_push needs convergent lanes)
    auto shade = [&](const bool active, const int q) {
        // Two phases around the light-estimate pushes: the estimate's record, shadow and probe rays
        // are written as soon as they exist, so their registers are free during the path's BSDF
        // sample; only the record's target (the continuation's position) is written at the end.
        bool pushShadow = false, pushProbe = false, pushDirect = false, pushNext = false;
        bool cont2 = false;   // phase 2 runs: the path samples its BSDF
        int id = 0, dim = 0, bounces = 0;
        bool specularBounce = false;
        Ray cont, ray;
        rgb L, beta;
        float etaScale = 1.f;
        uint32_t sIndex = 0;
        Isect isect;
        BSDF bsdf;
        MatTemplate texLocal;   // a textured material's per-hit lobes (make_bsdf)
        SState st;
        st.index = 0; st.sid = 0; st.dim = 0; st.px = st.py = 0;
        int di = -1;
        {
            Ray shadow, probe;
            rgb A, fB;
            float pmfD = 0.f, weightB = 1.f, scatPdfD = 0.f;
            int dflagsD = 0, lightD = 0;
            if (active) {
                float4 o = W.cur.o[q], d = W.cur.d[q], hr = W.cur.hit[q];
                id = level0 ? q : W.cur.id[q];
                const int dd = __float_as_int(d.w);
                dim = dd & 0xffff;
                bounces = (dd >> 16) & 0x7f;
                specularBounce = (dd >> 23) & 1;
                ray = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
                const int slot = __float_as_int(hr.x);
                const bool found = slot >= 0;
                if (level0) {
                    L = sp(0.f); beta = sp(1.f); etaScale = 1.f;
                    sIndex = W.sampleIndex[q];
                } else {
                    const float4 a = W.cur.s0[q], b = W.cur.s1[q];
                    L = sp3(a.x, a.y, a.z); beta = sp3(a.w, b.x, b.y);
                    etaScale = b.z;
                    sIndex = __float_as_uint(b.w);
                }
                if (found) {
                    int flags = __float_as_int(S.triVerts[3 * (size_t)slot].w);
                    if (flags & PRIM_SPHERE) sphere_si(S.spheres[__float_as_int(S.triVerts[3 * (size_t)slot].x)], ray, ray.tMax, &isect);
                    else triangle_si(S, slot, ray, hr.y, hr.z, hr.w, flags, &isect);
                    isect.slot = slot;
                    isect.medIn = isect.medOut = -1;
                }
                if (bounces == 0 || specularBounce) {
                    if (found) L = L + beta * si_Le(S, isect, -ray.d);
                    else for (int k = 0; k < S.nInfinite; ++k) L = L + beta * light_Le(S, S.lights[S.infinite[k]], ray);
                }
                bool alive = found && bounces < P.maxDepth;
                if (alive && !make_bsdf<(LOBES & kTexturedLobes) != 0>(S, mats, isect, true, &bsdf, &texLocal)) {
                    cont = spawn_ray(isect, ray.d);   // isect.SpawnRay(ray.d); bounces-- then ++: same bounce
                    pushNext = true;
                    alive = false;
                } else if (alive) {
                    cont2 = true;
                    st.index = sIndex;
                    st.sid = id;   // ≡ the sample number mod spp (pixel-major ids)
                    st.dim = dim;
                    const f3 wo = isect.wo;
                    if (num_components(bsdf, BSDF_ALL & ~BSDF_SPECULAR) > 0 && S.nLights > 0) {
                        // UniformSampleOneLight: light choice, then EstimateDirect's two strategies
                        float pmf;
                        const int li = sample_light(S, get1d<true, SMP>(P.smp, st), &pmf);
                        if (pmf != 0) {
                            float uL0, uL1, uS0, uS1;
                            get2d<true, SMP>(P.smp, st, &uL0, &uL1);
                            get2d<true, SMP>(P.smp, st, &uS0, &uS1);
                            const DLight& light = S.lights[li];
                            const bool delta = light.type == LT_POINT;
                            const int flagsNS = BSDF_ALL & ~BSDF_SPECULAR;
                            int dflags = 0;
                            f3 wi = mk(0, 0, 0);
                            float lightPdf = 0, scatteringPdf = 0;
                            VisPt vis;
                            // Lambda(wo) of the microfacet lobes, once for the estimate's two strategies
                            const float lamL = mf_lambda<LOBES>(bsdf, bsdf.to_local(wo));
                            rgb Li = sample_li(S, light, isect, uL0, uL1, &wi, &lightPdf, &vis);
                            A = sp(0.f);
                            if (lightPdf > 0 && !black(Li)) {
                                rgb f;
                                if constexpr (PBR_DIAG_SHADE & 1) { f = sp(0.25f); scatteringPdf = 0.5f; }
                                else {
                                f = bsdf_f_pdf<LOBES>(bsdf, wo, wi, flagsNS, &scatteringPdf, lamL) * absdot(wi, isect.sn);
                                }
                                if (!black(f)) {
                                    if (delta) A = f * Li / lightPdf;
                                    else {
                                        float fp = 1 * lightPdf, gp = 1 * scatteringPdf;
                                        float weight = (fp * fp) / (fp * fp + gp * gp);
                                        A = f * Li * weight / lightPdf;
                                    }
                                    shadow = spawn_ray_to(isect, vis.p, vis.pError, vis.n);
                                    pushShadow = true;
                                    dflags |= kWfpAPending;
                                }
                            }
                            fB = sp(0.f);
                            weightB = 1.f;
                            if (!delta && !(PBR_DIAG_SHADE & 2)) {
                                // EstimateDirect's BSDF sample (Integrator.cpp:126-174).  Its value f·|cos|
                                // is only read when the sampled direction can reach the light — a specular
                                // sample, or Pdf_Li != 0 — so it is formed only then (the checks are pure,
                                // so their order does not change the outcome): most sampled directions miss
                                // a small area light and skip the sum over the lobes.
                                int stype = 0;
                                BsdfDraw draw;
                                if (bsdf_sample_dir<LOBES>(bsdf, wo, &wi, uS0, uS1, &scatteringPdf, flagsNS, &stype, &draw, lamL) &&
                                    scatteringPdf > 0) {
                                    const bool sampledSpecular = (stype & BSDF_SPECULAR) != 0;
                                    const float lp = sampledSpecular ? 0.f : ((PBR_DIAG_SHADE & 4) ? 0.5f : pdf_li(S, light, isect, wi));
                                    if (sampledSpecular || lp != 0) {
                                        fB = bsdf_sample_sum<LOBES>(bsdf, wo, wi, flagsNS, draw) * absdot(wi, isect.sn);
                                        if (!black(fB)) {
                                            if (!sampledSpecular) {
                                                float fp = 1 * scatteringPdf, gp = 1 * lp;
                                                weightB = (fp * fp) / (fp * fp + gp * gp);
                                            }
                                            probe = spawn_ray(isect, wi);
                                            pushProbe = true;
                                            dflags |= kWfpBPending;
                                        }
                                    }
                                }
                            }
                            if (dflags) {
                                pmfD = pmf;
                                scatPdfD = scatteringPdf;
                                dflagsD = dflags;
                                lightD = li;
                                pushDirect = true;
                            }
                        }
                    }
                }
            }
            // the estimate's record (beta at the estimate: the path's beta before its BSDF sample),
            // its shadow and probe rays
            di = base + wave_push(&s_push[2], pushDirect);
            if (pushDirect) {
                X.dA[di] = make_float4(A.r, A.g, A.b, pmfD);
                X.dB[di] = make_float4(fB.r, fB.g, fB.b, weightB);
                X.dBeta[di] = make_float4(beta.r, beta.g, beta.b, scatPdfD);
                X.dFlags[di] = dflagsD;
                X.dLight[di] = lightD;
            }
            const int si = base + wave_push(&s_push[0], pushShadow);
            if (pushShadow) {
                W.so[si] = make_float4(shadow.o.x, shadow.o.y, shadow.o.z, shadow.tMax);
                W.sd[si] = make_float4(shadow.d.x, shadow.d.y, shadow.d.z, 0.f);
                W.sid[si] = di;
            }
            const int pi = base + wave_push(&s_push[1], pushProbe);
            if (pushProbe) {
                X.po[pi] = make_float4(probe.o.x, probe.o.y, probe.o.z, probe.tMax);
                X.pd[pi] = make_float4(probe.d.x, probe.d.y, probe.d.z, 0.f);
                X.pid[pi] = di;
            }
        }
        if (cont2) {
            // BSDF sample for the path (PathIntegrator.cpp:80-105): wo is -ray.d here, not the
            // normalised isect.wo the light estimate uses
            const f3 woPath = -ray.d;
            f3 wi = mk(0, 0, 0);
            float pdf = 0;
            int flags = 0;
            float u0, u1;
            get2d<true, SMP>(P.smp, st, &u0, &u1);
            rgb f = bsdf_sample<LOBES>(bsdf, woPath, &wi, u0, u1, &pdf, BSDF_ALL, &flags);
            if (!(black(f) || pdf == 0.f)) {
                beta = beta * (f * absdot(wi, isect.sn) / pdf);
                specularBounce = (flags & BSDF_SPECULAR) != 0;
                if ((flags & BSDF_SPECULAR) && (flags & BSDF_TRANSMISSION)) {
                    float eta = bsdf.mt->eta;
                    etaScale *= (dot(woPath, isect.n) > 0) ? (eta * eta) : 1 / (eta * eta);
                }
                cont = spawn_ray(isect, wi);
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
        }
        if (active) {
            if (X.lastLevel) pushNext = false;   // never taken: no bounce is left at the last level
            if (!pushNext) X.stL[id] = make_float4(L.r, L.g, L.b, 0.f);   // the path ends here
        }
        const int ni = base + wave_push(&s_push[3], pushNext);
        if (pushNext) {
            W.next.o[ni] = make_float4(cont.o.x, cont.o.y, cont.o.z, cont.tMax);
            W.next.d[ni] = make_float4(cont.d.x, cont.d.y, cont.d.z, __int_as_float(pack_path(dim, bounces, specularBounce)));
            W.next.id[ni] = id;
            W.next.s0[ni] = make_float4(L.r, L.g, L.b, beta.r);
            W.next.s1[ni] = make_float4(beta.g, beta.b, etaScale, __uint_as_float(sIndex));
        }
        if (pushDirect) X.dTgt[di] = pushNext ? ni : ~id;
    };
    if constexpr (!CLASSED) {
        for (int it = 0; it < nIter; ++it) {   // uniform trip count: wave_push needs convergent lanes
            const int i = it * stride + wf_block() * blockDim.x + threadIdx.x;
            const bool active = i < n;
            const int q = level0 ? i : seg_pos_dense(W.segCap, i, n);
            shade(active, active ? q : 0);
        }
    } else if (pass > 0) {   // this pass's list, filed by pass 0
        const int cnt = X.passCnt[(pass - 1) * kWfBlocks + wf_block()];
        const int* list = X.passList + (size_t)(pass - 1) * X.passStride + base;
        for (int k0 = 0; k0 < cnt; k0 += 256) {   // uniform trip count
            const int k = k0 + (int)threadIdx.x;
            const bool active = k < cnt;
            shade(active, active ? list[k] : 0);
        }
    } else {
        // ring of queue positions of this pass: appended per iteration (at most 256), shaded 256 at a
        // time once that many are pending, so fewer than 256 wait and 512 slots never overrun
        __shared__ int s_ring[512];
        __shared__ int s_tail;
        __shared__ int s_list[8];   // entries filed per later pass
        if (threadIdx.x == 0) s_tail = 0;
        if (threadIdx.x < 8) s_list[threadIdx.x] = 0;
        __syncthreads();
        int head = 0;   // workgroup-uniform
        for (int it = 0; it < nIter; ++it) {
            const int i = it * stride + wf_block() * blockDim.x + threadIdx.x;
            const int qd = level0 ? i : seg_pos_dense(W.segCap, i, n);
            const int q = i < n ? qd : 0;
            const int cls = i < n ? entry_pass(X, q) : -1;
            const bool mine = cls == 0;
            for (int c = 1; c < X.nPasses; ++c) {   // file the other passes' entries (per segment, dense)
                const int at = wave_push(&s_list[c - 1], cls == c);
                if (cls == c) X.passList[(size_t)(c - 1) * X.passStride + base + at] = q;
            }
            const int at = wave_push(&s_tail, mine);
            if (mine) s_ring[at & 511] = q;
            __syncthreads();
            const bool full = s_tail - head >= 256;   // (the same for every lane: no append until the barrier below)
            const int qq = full ? s_ring[(head + threadIdx.x) & 511] : 0;
            __syncthreads();   // the counter and the entries are read before any wave appends again
            if (full) {
                shade(true, qq);
                head += 256;
            }
        }
        __syncthreads();
        const int tail = s_tail;
        if (head < tail) {
            const bool active = head + (int)threadIdx.x < tail;
            const int qq = active ? s_ring[(head + threadIdx.x) & 511] : 0;
            shade(active, qq);
        }
        if ((int)threadIdx.x + 1 < X.nPasses) X.passCnt[threadIdx.x * kWfBlocks + wf_block()] = s_list[threadIdx.x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        W.shadowSeg[wf_block()] = s_push[0];
        X.probeSeg[wf_block()] = s_push[1];
        X.directSeg[wf_block()] = s_push[2];
        W.next.segCount[wf_block()] = s_push[3];
    }
}

// VisibilityTester::Unoccluded for the light-sample rays
template <int SHORT>
__global__ __launch_bounds__(256, PBR_REFILL_OCC_ANY) void k_wfp_shadow(WfpParams X) {
    WfParams& W = X.W;
    const int n = seg_scan(W.shadowSeg);
    if constexpr (kRefill > 0 && SHORT > 0 && kQuadTraversal) {
        unsigned visible = 0;   // profile field 1, added once per wave at the end
        traverse_stream<true, kAnyShort>(
            W.P.S, n, W.segCap,
            [&](int q, int* key) {
                *key = q;
                const float4 o = W.so[q], d = W.sd[q];
                return mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
            },
            [&](int q, bool hit, const Ray&, const HitRec&) {
                if (!hit) {
                    ++visible;
                    X.dFlags[W.sid[q]] |= kWfpVisible;   // the only writer of this record in this launch
                }
            },
            W.prof, KP_WFP_SHADOW);
        if (W.prof) prof_add(W.prof + KP_WFP_SHADOW * kProfFields + 1, visible);
        return;
    }
    for (int i0 = wf_block() * blockDim.x + ((int)threadIdx.x & ~63); i0 < n; i0 += gridDim.x * blockDim.x) {   // per wave
        const int i = i0 + (int)__lane_id();
        const int q = seg_pos_dense(W.segCap, i, n);
        if (i >= n) continue;
        float4 o = W.so[q], d = W.sd[q];
        Ray r = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
        HitRec h;
        Counters c;
        const bool visible = !traverse<true, false, SHORT>(W.P.S, r, &h, &c);
        trav_diag(W.prof, KP_WFP_SHADOW, h);
        if (W.prof) prof_count(W.prof + KP_WFP_SHADOW * kProfFields + 1, visible);
        if (visible) X.dFlags[W.sid[q]] |= kWfpVisible;   // the only writer of this record in this launch
    }
}

// EstimateDirect's BSDF-sampled ray: closest hit; Li = the sampled light's emission if that is
// what it hits (si.Le), light.Le(ray) if it escapes (Light::Le, F4 for non-infinite lights).
template <int SHORT>
__global__ __launch_bounds__(256, PBR_REFILL_OCC) void k_wfp_probe(WfpParams X) {
    WfParams& W = X.W;
    const DeviceScene& S = W.P.S;
    const int n = seg_scan(X.probeSeg);
    if constexpr (kRefill > 0 && SHORT > 0 && kQuadTraversal) {
        traverse_stream<false, kRefillShort>(
            S, n, W.segCap,
            [&](int q, int* key) {
                *key = q;
                const float4 o = X.po[q], d = X.pd[q];
                return mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
            },
            [&](int q, bool hit, const Ray& ray, const HitRec& h) {
                const int di = X.pid[q];
                const int li = X.dLight[di];
                rgb Li2 = sp(0.f);
                if (hit) {
                    if (S.primInfo[h.slot].z == li) {
                        Isect lightIsect;
                        int flags = __float_as_int(S.triVerts[3 * (size_t)h.slot].w);
                        if (flags & PRIM_SPHERE) sphere_si(S.spheres[__float_as_int(S.triVerts[3 * (size_t)h.slot].x)], ray, ray.tMax, &lightIsect);
                        else triangle_si(S, h.slot, ray, h.b0, h.b1, h.b2, flags, &lightIsect);
                        lightIsect.slot = h.slot;
                        Li2 = si_Le(S, lightIsect, -ray.d);
                    }
                } else {
                    Li2 = light_Le(S, S.lights[li], ray);
                }
                X.dLi[di] = make_float4(Li2.r, Li2.g, Li2.b, 0.f);
            },
            W.prof, KP_WFP_PROBE);
        return;
    }
    for (int i0 = wf_block() * blockDim.x + ((int)threadIdx.x & ~63); i0 < n; i0 += gridDim.x * blockDim.x) {   // per wave
        const int i = i0 + (int)__lane_id();
        const int q = seg_pos_dense(W.segCap, i, n);
        if (i >= n) continue;
        float4 o = X.po[q], d = X.pd[q];
        Ray ray = mkray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, -1);
        const int di = X.pid[q];
        const int li = X.dLight[di];
        HitRec h;
        Counters c;
        rgb Li2 = sp(0.f);
        const bool hitP = traverse<false, false, SHORT>(S, ray, &h, &c);
        trav_diag(W.prof, KP_WFP_PROBE, h);
        if (hitP) {
            if (S.primInfo[h.slot].z == li) {
                Isect lightIsect;
                int flags = __float_as_int(S.triVerts[3 * (size_t)h.slot].w);
                if (flags & PRIM_SPHERE) sphere_si(S.spheres[__float_as_int(S.triVerts[3 * (size_t)h.slot].x)], ray, ray.tMax, &lightIsect);
                else triangle_si(S, h.slot, ray, h.b0, h.b1, h.b2, flags, &lightIsect);
                lightIsect.slot = h.slot;
                Li2 = si_Le(S, lightIsect, -ray.d);
            }
        } else {
            Li2 = light_Le(S, S.lights[li], ray);
        }
        X.dLi[di] = make_float4(Li2.r, Li2.g, Li2.b, 0.f);
    }
}

// the path's L where the estimate resolves: its continuation entry, or stL[id] if the path ended
__device__ __forceinline__ void add_direct(const WfpParams& X, int tgt, rgb direct) {
    float4* p = tgt >= 0 ? &X.W.next.s0[tgt] : &X.stL[~tgt];
    float4 L = *p;
    L.x = L.x + direct.r; L.y = L.y + direct.g; L.z = L.z + direct.b;
    *p = L;
}

// Ld = [A if the light sample is unoccluded] + [f·Li·weight/scatteringPdf if Li is not black];
// L += beta · (Ld / pmf) — UniformSampleOneLight's division, then PathIntegrator's beta product.
__global__ __launch_bounds__(256) void k_wfp_resolve(WfpParams X) {
    WfParams& W = X.W;
    const int n = seg_scan(X.directSeg);
    for (int i0 = wf_block() * blockDim.x + ((int)threadIdx.x & ~63); i0 < n; i0 += gridDim.x * blockDim.x) {   // per wave
        const int i = i0 + (int)__lane_id();
        const int di = seg_pos_dense(W.segCap, i, n);
        if (i >= n) continue;
        const int fl = X.dFlags[di];
        const float4 a = X.dA[di], bt = X.dBeta[di];
        rgb Ld = sp(0.f);
        if ((fl & kWfpAPending) && (fl & kWfpVisible)) Ld = Ld + sp3(a.x, a.y, a.z);
        if (fl & kWfpBPending) {
            const float4 li = X.dLi[di], b = X.dB[di];
            const rgb Li2 = sp3(li.x, li.y, li.z);
            if (!black(Li2)) Ld = Ld + sp3(b.x, b.y, b.z) * Li2 * b.w / bt.w;
        }
        const rgb beta = sp3(bt.x, bt.y, bt.z);
        add_direct(X, X.dTgt[di], beta * (Ld / a.w));
    }
}

// Per-pixel in-order sum of the per-sample L (colObj += Li) and the film; layout as k_wf_finish.
__global__ __launch_bounds__(256) void k_wfp_finish(WfpParams X) {
    WfParams& W = X.W;
    __shared__ float lds[3 * (kFinishSamples + 64)];
    __shared__ float sum[64 * 3];
    const KParams& P = W.P;
    const int spp = P.spp, pitch = min(spp, kFinishSamples) + 1;
    const int pb = finish_pixels(spp);
    const int lp0 = blockIdx.x * pb;   // dispatch order: the XCD-run order made finish 28% slower
    const int npx = min(pb, W.chunkPix - lp0);
    const int slice = min(spp, kFinishSamples);
    float acc = 0.f;
    for (int s0 = 0; s0 < spp; s0 += slice) {
        const int ns = npx * min(slice, spp - s0);
        for (int t = threadIdx.x; t < ns; t += blockDim.x) {
            const int p = spp <= kFinishSamples ? t / spp : 0, k = spp <= kFinishSamples ? t - p * spp : s0 + t;
            const float4 L = X.stL[(lp0 + p) * spp + k];
            const int kk = k - s0;
            lds[(p * 3 + 0) * pitch + kk] = L.x;
            lds[(p * 3 + 1) * pitch + kk] = L.y;
            lds[(p * 3 + 2) * pitch + kk] = L.z;
        }
        __syncthreads();
        if ((int)threadIdx.x < 3 * npx) {
            const int cnt = min(slice, spp - s0);
            const float* row = lds + threadIdx.x * pitch;
            for (int k = 0; k < cnt; ++k) acc = acc + row[k];
        }
        __syncthreads();
    }
    if ((int)threadIdx.x < 3 * npx) sum[threadIdx.x] = acc;
    __syncthreads();
    if ((int)threadIdx.x < npx)
        film_out(P, W.chunkPix0 + lp0 + threadIdx.x, sp3(sum[3 * threadIdx.x], sum[3 * threadIdx.x + 1], sum[3 * threadIdx.x + 2]));
}
