// path_kernel.hip -- the `direct` integrator, batch ray queries, the film
// reduction and the launchers of Mitsuba 0.6's `path` integrator megakernel
// (dmega.h; its variants are compiled per scene feature set in path_f.hip).
#include "dmega.h"


// ===========================================================================
// The `direct` integrator: MIDirectIntegrator::Li (integrators/direct/direct.cpp:
// 144-306) at rRec.depth = 1, one lane per (sample, pixel) item.  Per item: the
// camera ray; at its hit, `emitterSamples` emitter samples (each with its shadow
// ray) and `bsdfSamples` BSDF samples (each with its closest-hit ray), MIS-
// weighted with the integrator's fractions and per-technique weights.
// ===========================================================================

// SobolSampler with requested 2D arrays: next1D/next2D skip dims [5, arrayEnd)
// (sobol.cpp:219-250)
__device__ __forceinline__ float next1d_a(const SobolCtx &C, SamplerState &s, uint32_t arrayEnd) {
    if (s.dim >= 5 && s.dim < arrayEnd) s.dim = arrayEnd;
    return next1d(C, s);
}
__device__ __forceinline__ void next2d_a(const SobolCtx &C, float res, SamplerState &s, int px, int py,
                                         uint32_t arrayEnd, float &u, float &v) {
    if (s.dim + 1 >= 5 && s.dim < arrayEnd) s.dim = arrayEnd;
    next2d(C, res, s, px, py, u, v);
}
// element k of the sample's `size`-point 2D array at dimension `dim`: Sampler::
// next2DArray (sampler.cpp:82-92) over SobolSampler::generate's arrays (sobol.cpp:188-197)
template <typename T>
__device__ __forceinline__ void sobol_array2d(const SobolCtx &C, const MtsgLookup &Lu, T *ycolTab, uint32_t nibbles,
                                              uint32_t j, uint32_t size, uint32_t k, int px, int py,
                                              uint64_t scramble64, uint32_t dim, float &u, float &v) {
    const uint32_t frame = j * size + k;
    const uint64_t idx = C.indep ? indep_key((uint32_t)px, (uint32_t)py, frame)
                       : Lu.m >= 1 ? sobol_lookup_lds(Lu, ycolTab, nibbles, frame, (uint32_t)px, (uint32_t)py, scramble64)
                                   : (uint64_t)frame;
    u = sobol_sample(C, idx, dim);
    v = sobol_sample(C, idx, dim + 1);
}

// PerspectiveCameraImpl::sampleRayDifferential (perspective.cpp:271-298): origin, direction, [mint, maxt]
__device__ __forceinline__ void camera_ray(const MtsgCamera &cam, float sx, float sy, f3 &ro, f3 &rd, float &mint,
                                           float &maxt) {
    const f3 nearP = xf_point(cam.sample_to_camera, mk(sx * cam.inv_res_x, sy * cam.inv_res_y, 0.0f));
    const f3 dl = normalize(nearP);
    const float invZ = 1.0f / dl.z;
    mint = cam.near_clip * invZ;
    maxt = cam.far_clip * invZ;
    const float *W = cam.to_world;
    ro = mk(W[0] * 0.0f + W[1] * 0.0f + W[2] * 0.0f + W[3], W[4] * 0.0f + W[5] * 0.0f + W[6] * 0.0f + W[7],
            W[8] * 0.0f + W[9] * 0.0f + W[10] * 0.0f + W[11]);
    rd = mk(W[0] * dl.x + W[1] * dl.y + W[2] * dl.z, W[4] * dl.x + W[5] * dl.y + W[6] * dl.z,
            W[8] * dl.x + W[9] * dl.y + W[10] * dl.z);
}

// Scene::evalEnvironment of a camera ray with its (scaled) differentials
__device__ __forceinline__ f3 env_camera(const MtsgLaunch &L, float sx, float sy, f3 rd) {
    glb_env *E = (glb_env *)L.scene.env;
    if (E->constant) return mk(E->radiance[0], E->radiance[1], E->radiance[2]);
    const MtsgCamera &cam = L.scene.cam;
    const f3 nearP = xf_point(cam.sample_to_camera, mk(sx * cam.inv_res_x, sy * cam.inv_res_y, 0.0f));
    const f3 rxl = normalize(add(nearP, ld3(cam.dx))), ryl = normalize(add(nearP, ld3(cam.dy)));
    const float *W = cam.to_world;
    f3 rxd = mk(W[0] * rxl.x + W[1] * rxl.y + W[2] * rxl.z, W[4] * rxl.x + W[5] * rxl.y + W[6] * rxl.z,
                W[8] * rxl.x + W[9] * rxl.y + W[10] * rxl.z);
    f3 ryd = mk(W[0] * ryl.x + W[1] * ryl.y + W[2] * ryl.z, W[4] * ryl.x + W[5] * ryl.y + W[6] * ryl.z,
                W[8] * ryl.x + W[9] * ryl.y + W[10] * ryl.z);
    rxd = add(rd, mul(sub(rxd, rd), L.diff_scale));
    ryd = add(rd, mul(sub(ryd, rd), L.diff_scale));
    return env_eval_diff(E, rd, rxd, ryd);
}

// Scene::sampleEmitterDirect without the visibility test (scene.cpp:828-852):
// value = radiance / (pdf * emPdf) and pdf = dRec.pdf * emPdf when pdf != 0
struct NeeSample { f3 value, d; float dist, pdf; };
template <bool ENV, bool ANA, typename HS>
__device__ __forceinline__ NeeSample emitter_sample(const MtsgDeviceScene &S, const HS &hs, f3 ref, f3 refN, float ex,
                                                    float ey) {
    NeeSample r;
    r.value = mk(0, 0, 0); r.d = mk(0, 0, 1); r.dist = 0.0f; r.pdf = 0.0f;
    float emPdf;
    const uint32_t ei = dd_sample_reuse(S.em_cdf, S.num_emitters, ex, &emPdf);
    const MtsgEmitter &e = S.emitters[ei];
    f3 value = mk(0, 0, 0);
    float pdf = 0.0f;
    if (ENV && e.type != MTSG_EMITTER_AREA) {
        glb_env *E = (glb_env *)S.env;
        const EnvSample es = E->constant ? const_sample_direct(E, ref, refN, ex, ey) : env_sample_direct(E, ref, ex, ey);
        value = es.value; r.d = es.d; r.dist = es.dist; pdf = es.pdf;
    } else if (ANA && S.shapes[e.shape].analytic >= 0) {
        const AnaSample as = ana_sample_direct(((GAna *)S.analytic)[S.shapes[e.shape].analytic], ref, ex, ey);
        r.d = as.d; r.dist = as.dist; pdf = as.pdf;
        if (dot(r.d, refN) >= 0 && dot(r.d, as.n) < 0 && pdf != 0) value = divs(ld3(e.radiance), pdf);   // area.cpp:158-173
        else pdf = 0.0f;
    } else {
        // TriMesh::samplePosition (trimesh.cpp:412-425), Triangle::sample (triangle.cpp:24-58)
        float py2 = ey;
        const uint32_t lt = dd_sample_reuse(S.area_cdf + e.cdf_offset, e.tri_count, py2, nullptr);
        const uint32_t prim = e.tri_first + lt;
        const uint4 pv = make_uint4(hs.pv[4 * prim], hs.pv[4 * prim + 1], hs.pv[4 * prim + 2], hs.pv[4 * prim + 3]);
        const float a = safe_sqrt(1.0f - ex);
        const float bx = 1 - a, by = a * py2;
        const f3 p0 = ldp3(hs.pos + 3 * (size_t)pv.x), p1 = ldp3(hs.pos + 3 * (size_t)pv.y),
                 p2 = ldp3(hs.pos + 3 * (size_t)pv.z);
        const f3 sideA = sub(p1, p0), sideB = sub(p2, p0);
        const f3 lp = add(add(p0, mul(sideA, bx)), mul(sideB, by));
        f3 ln;
        if (hs.shapes[e.shape].has_normals) {
            const f3 n0 = ldp3(hs.nrm + 3 * (size_t)pv.x), n1 = ldp3(hs.nrm + 3 * (size_t)pv.y),
                     n2 = ldp3(hs.nrm + 3 * (size_t)pv.z);
            ln = normalize(add(add(mul(n0, 1.0f - bx - by), mul(n1, bx)), mul(n2, by)));
        } else {
            ln = normalize(cross(sideA, sideB));
        }
        pdf = e.inv_area;
        r.d = sub(lp, ref);   // Shape::sampleDirect (shape.cpp:102-115)
        const float distSquared = len2(r.d);
        r.dist = dsqrt(distSquared);
        r.d = divs(r.d, r.dist);
        const float dp = absdot(r.d, ln);
        pdf *= dp != 0 ? (distSquared / dp) : 0.0f;
        if (dot(r.d, refN) >= 0 && dot(r.d, ln) < 0 && pdf != 0) value = divs(ld3(e.radiance), pdf);
        else pdf = 0.0f;
    }
    if (pdf != 0) {
        r.pdf = pdf * emPdf;
        r.value = divs(value, emPdf);
    }
    return r;
}

// Scene::pdfEmitterDirect for an area-light hit h reached along d from `ref`
// (area.cpp:175-181, shape.cpp:117-126 / sphere.cpp:357-387, scene.h:848-850)
template <bool ANA>
__device__ __forceinline__ float area_hit_pdf(const MtsgDeviceScene &S, const Hit &h, f3 ref, f3 d, f3 refN) {
    const MtsgEmitter &e = S.emitters[S.shapes[h.shape].emitter];
    const f3 dn = h.sh.n;
    float pdf = 0.0f;
    if (dot(d, refN) >= 0 && dot(d, dn) < 0) {
        if (ANA && S.shapes[h.shape].analytic >= 0)
            pdf = ana_pdf_direct(((GAna *)S.analytic)[S.shapes[h.shape].analytic], ref, d, dn, h.t);
        else
            pdf = e.inv_area * (h.t * h.t) / absdot(d, dn);
    }
    return pdf * (e.weight * S.em_norm);
}

// BSDF eval/pdf/sample through a twosided wrapper (twosided.cpp:105-172)
template <bool EXT>
__device__ __forceinline__ void bsdf_eval_pdf_2s(const MtsgDeviceScene &S, GBsdf &bsdf, const Hit &h, f3 wo, f3 &val,
                                                 float *pdf) {
    f3 qwi = h.wi, qwo = wo;
    GBsdf *qb = &bsdf;
    if constexpr (EXT) {
        if (bsdf.type == BSDF_TWOSIDED) {
            const bool flip = !(qwi.z > 0);
            qb = &((GBsdf *)S.bsdfs)[bsdf.nested[flip ? 1 : 0]];
            if (flip) { qwi.z = -qwi.z; qwo.z = -qwo.z; }
        }
    }
    val = bsdf_eval_fast<(EXT ? (int)MTSG_FEAT_EXT : 0)>(*qb, (glb_f32 *)S.rtrans, qwi, qwo, h.u, h.v);
    if (pdf) *pdf = bsdf_pdf_fast<(EXT ? (int)MTSG_FEAT_EXT : 0)>(*qb, (glb_f32 *)S.rtrans, qwi, qwo, h.u, h.v);
}
template <bool EXT>
__device__ __forceinline__ BSample bsdf_sample_2s(const MtsgDeviceScene &S, GBsdf &bsdf, const Hit &h, float bx,
                                                  float by, float u1d) {
    if (EXT && bsdf.type == BSDF_TWOSIDED) {
        const bool flip = h.wi.z < 0;
        f3 qwi = h.wi;
        if (flip) qwi.z = -qwi.z;
        constexpr int BS = EXT ? (int)MTSG_FEAT_EXT : 0;
        GBsdf &nb = ((GBsdf *)S.bsdfs)[bsdf.nested[flip ? 1 : 0]];
        BSample bs = bsdf_sample_fast<BS>(nb, (glb_f32 *)S.rtrans, qwi, bx, by, u1d, h.u, h.v,
                                          rp_pre_for<BS>(nb, (glb_f32 *)S.rtrans, qwi, h.u, h.v));
        if (flip && !is_zero(bs.weight) && bs.pdf != 0) bs.wo.z = -bs.wo.z;
        return bs;
    }
    return bsdf_sample_fast<(EXT ? (int)MTSG_FEAT_EXT : 0)>(
        bsdf, (glb_f32 *)S.rtrans, h.wi, bx, by, u1d, h.u, h.v,
        rp_pre_for<(EXT ? (int)MTSG_FEAT_EXT : 0)>(bsdf, (glb_f32 *)S.rtrans, h.wi, h.u, h.v));
}

// direct_kernel's shadow rays: the any-hit traversal.  Inlined into
// direct_kernel's nested divergent loops at -O3, hipcc (ROCm 7.2, gfx950)
// produced wrong occlusion answers for 15% of the samples of the analytic-shape
// scene; the pass bisection pinned it to GVN's scalar PRE on that kernel
// (DESIGN.md 4).  This translation unit is therefore compiled with
// -mllvm -enable-pre=false (Makefile), and the traversal is inlined again;
// -DMTSG_SHADOW_ANY_NOINLINE restores the round-2 workaround (a call)
#ifdef MTSG_SHADOW_ANY_NOINLINE
#define SHADOW_ANY_CALL __device__ __noinline__
#else
#define SHADOW_ANY_CALL __device__ __forceinline__
#endif
template <bool ANA, typename NodeT, typename TriT>
SHADOW_ANY_CALL bool shadow_any(NodeT *nodes, TriT *tris, f3 o, f3 d, float mint, float maxt,
                                        lds_stk_n *stkN, lds_stk_d *stkD, unsigned long long &cN,
                                        unsigned long long &cT, const MtsgAnalytic *ana) {
    uint32_t sl = 0;
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
    return traverse<true, false, ANA>(nodes, tris, o, d, mint, maxt, stkN, stkD, sl, a0, a1, a2, cN, cT, ana);
}
template <bool SCENE_LDS, int FEAT>
__global__ __launch_bounds__(BLOCK, MTSG_WAVES_PER_EU) void direct_kernel(MtsgLaunch L) {
    constexpr bool ENV = (FEAT & MTSG_FEAT_ENV) != 0, EXT = (FEAT & MTSG_FEAT_EXT) != 0,
                   ANA = (FEAT & MTSG_FEAT_ANA) != 0;
    extern __shared__ uint32_t lds[];
    const MtsgDeviceScene &S = L.scene;
    // LDS as path_kernel: [Sobol nibble tables][look_up column tables][scene (small scenes)][stacks]
    const uint32_t tabWords = L.lds_dims * L.nibbles * 16;
    for (uint32_t i = threadIdx.x; i < tabWords; i += BLOCK) {
        const uint32_t d = i / (L.nibbles * 16), r = i % (L.nibbles * 16);
        lds[i] = L.sobol_nib[(size_t)d * MTSG_NIBBLES * 16 + r];
    }
    for (uint32_t i = threadIdx.x; i < 16 * 16; i += BLOCK) {
        const uint32_t c = i >> 4, v = i & 15;
        uint32_t r = 0;
        for (int b = 0; b < 4; ++b)
            if ((v >> b) & 1) r ^= L.lut.ycol[4 * c + b];
        lds[tabWords + i] = r;
    }
    const uint32_t base2 = tabWords + 16 * 16;
    uint32_t sceneWords = 0;
    if (SCENE_LDS) {
        const uint32_t nodeWords = L.num_nodes * 16, triWords = S.num_prims * 12;
        const uint32_t *gn = reinterpret_cast<const uint32_t *>(S.nodes);
        const uint32_t *gt = reinterpret_cast<const uint32_t *>(S.tris);
        for (uint32_t i = threadIdx.x; i < nodeWords; i += BLOCK) lds[base2 + i] = gn[i];
        for (uint32_t i = threadIdx.x; i < triWords; i += BLOCK) lds[base2 + nodeWords + i] = gt[i];
        sceneWords = nodeWords + triWords;
        const uint32_t np = S.num_prims, nv = L.num_verts, ns = L.num_shapes * (sizeof(MtsgShape) / 4);
        const uint32_t *srcs[5] = {S.prim_vtx, reinterpret_cast<const uint32_t *>(S.dpdu),
                                   reinterpret_cast<const uint32_t *>(S.positions),
                                   reinterpret_cast<const uint32_t *>(S.normals),
                                   reinterpret_cast<const uint32_t *>(S.shapes)};
        const uint32_t lens[5] = {4 * np, 3 * np, 3 * nv, 3 * nv, ns};
        for (int a = 0; a < 5; ++a) {
            for (uint32_t i = threadIdx.x; i < lens[a]; i += BLOCK) lds[base2 + sceneWords + i] = srcs[a][i];
            sceneWords += lens[a];
        }
    }
    __syncthreads();
    lds_u32 *ycolTab = (lds_u32 *)(lds + tabWords);
    lds_node *ldsNodes = (lds_node *)__builtin_assume_aligned((const void *)(lds + base2), 16);
    lds_tri *ldsTris = (lds_tri *)__builtin_assume_aligned((const void *)(lds + base2 + L.num_nodes * 16), 16);
    HitSrc<SCENE_LDS> hs;
    if constexpr (SCENE_LDS) {
        const uint32_t np = S.num_prims, nv = L.num_verts;
        lds_u32 *b = (lds_u32 *)(lds + base2 + L.num_nodes * 16 + np * 12);
        hs.pv = b;
        hs.dpdu = (lds_f32 *)(b + 4 * np);
        hs.pos = (lds_f32 *)(b + 7 * np);
        hs.nrm = (lds_f32 *)(b + 7 * np + 3 * nv);
        hs.shapes = (lds_shape *)(b + 7 * np + 6 * nv);
    } else {
        hs.pv = (glb_u32 *)S.prim_vtx;
        hs.dpdu = (glb_f32 *)S.dpdu;
        hs.pos = (glb_f32 *)S.positions;
        hs.nrm = (glb_f32 *)S.normals;
        hs.shapes = (glb_shape *)S.shapes;
    }
    SobolCtx SC;
    SC.lds = (lds_u32 *)lds;
    SC.glob = (glb_u32 *)L.sobol_nib;
    SC.lds_dims = L.lds_dims;
    SC.nibbles = L.nibbles;
    SC.scramble = L.scramble;
    SC.indep = L.sampler == MTSG_SAMPLER_INDEPENDENT;
    SC.replay = false;   // the SFMT replay renders path / volpath only (capi.cpp)
    SC.sfmt = nullptr;
    lds_stk_n *stkN = (lds_stk_n *)(lds + base2 + sceneWords) + threadIdx.x;
    lds_stk_d *stkD = (lds_stk_d *)(lds + base2 + sceneWords + L.stack_depth * BLOCK) + threadIdx.x;
    unsigned long long cRays = 0, cShadow = 0, cSamples = 0, cErr = 0, cN = 0, cT = 0;

    // closest hit / occlusion through the scene's structure (scan, LDS BVH or HBM BVH)
    auto closest = [&](f3 o, f3 d, float rmint, float rmaxt, Hit &h) -> bool {
        cRays++;
        float mint, maxt;
        uint32_t slot = 0;
        float hu = 0, hv = 0, ht = 0;
        bool hit = false;
        if (ray_interval(S, o, d, rmint, rmaxt, false, mint, maxt)) {
            if (SCENE_LDS && L.scan)
                hit = scan_tris<false, false>(L, o, d, mint, maxt, slot, hu, hv, ht, cT);
            else if (SCENE_LDS)
                hit = traverse<false, false, ANA>(ldsNodes, ldsTris, o, d, mint, maxt, stkN, stkD, slot, hu, hv, ht, cN,
                                                  cT, S.analytic);
            else
                hit = traverse<false, false, ANA>((glb_node *)S.nodes, (glb_tri *)S.tris, o, d, mint, maxt, stkN, stkD,
                                                  slot, hu, hv, ht, cN, cT, S.analytic);
        }
        if (hit) {
            const uint32_t prim = (SCENE_LDS && L.scan) ? slot : SCENE_LDS ? ldsTris[slot].prim : S.tris[slot].prim;
            fill_hit<EXT, ANA>(S, hs, slot, prim, hu, hv, ht, o, d, h);
        } else {
            h = Hit{};
        }
        return hit;
    };
    auto occluded = [&](f3 o, f3 d, float dist) -> bool {   // Ray(ref, d, Epsilon, dist*(1-ShadowEpsilon))
        cShadow++;
        float mint, maxt;
        if (!ray_interval(S, o, d, D_EPSILON, dist * (1 - D_SHADOW_EPSILON), true, mint, maxt)) return false;
        if (SCENE_LDS && L.scan) {
            uint32_t sl; float a0, a1, a2;
            return scan_tris<true, false>(L, o, d, mint, maxt, sl, a0, a1, a2, cT);
        }
        if (SCENE_LDS) return shadow_any<ANA>(ldsNodes, ldsTris, o, d, mint, maxt, stkN, stkD, cN, cT, S.analytic);
        return shadow_any<ANA>((glb_node *)S.nodes, (glb_tri *)S.tris, o, d, mint, maxt, stkN, stkD, cN, cT,
                               S.analytic);
    };

    const uint64_t lanes = (uint64_t)gridDim.x * BLOCK;
    for (uint64_t it = (uint64_t)xcd_block(L.xcds) * BLOCK + threadIdx.x; it < L.num_items; it += lanes) {
        const uint32_t jj = (uint32_t)(it / L.num_pixels);
        const uint32_t pix = (uint32_t)(it - (uint64_t)jj * L.num_pixels);
        int px, py;
        if (!pixel_of(L, pix, px, py)) continue;
        const uint32_t j = L.j0 + jj;
        SamplerState smp;
        smp.dim = 0;
        smp.sampleIndex = j;
        smp.err = false;
        smp.sobolIndex = SC.indep ? indep_key((uint32_t)px, (uint32_t)py, j)
                       : (L.lut.m > 1) ? sobol_lookup_lds(L.lut, ycolTab, L.nibbles, j, (uint32_t)px, (uint32_t)py,
                                                          L.scramble64)
                                       : (uint64_t)j;
        float u, v;
        next2d(SC, L.resolution, smp, px, py, u, v);
        const float sx = (float)px + u, sy = (float)py + v;
        f3 ro, rd;
        float rmint, rmaxt;
        camera_ray(S.cam, sx, sy, ro, rd, rmint, rmaxt);
        f3 Li = mk(0, 0, 0);
        Hit its;
        const bool hit = closest(ro, rd, rmint, rmaxt, its);
        const float alpha = L.has_alpha ? (hit ? 1.0f : 0.0f) : 1.0f;
        if (!hit) {
            if (ENV && !L.hide_emitters) Li = env_camera(L, sx, sy, rd);
        } else {
            auto &sh = hs.shapes[its.shape];
            GBsdf &bsdf = ((GBsdf *)S.bsdfs)[sh.bsdf];
            if (sh.emitter >= 0 && !L.hide_emitters) Li = add(Li, area_Le(S, its, neg(rd)));
            if (!(L.strict_normals && dot(rd, its.geoN) * its.wi.z >= 0)) {
                const f3 refN = (bsdf.flags & (MTSG_F_TRANSMISSION | MTSG_F_BACK)) == 0 ? its.sh.n : mk(0, 0, 0);
                // emitter sampling (direct.cpp:199-239)
                float su = 0, sv = 0;
                if (L.lum_samples <= 1) next2d_a(SC, L.resolution, smp, px, py, L.array_end, su, sv);
                if (bsdf.flags & MTSG_F_SMOOTH) {
                    for (uint32_t i = 0; i < L.lum_samples; ++i) {
                        float nx = su, ny = sv;
                        if (L.lum_samples > 1)
                            sobol_array2d(SC, L.lut, ycolTab, L.nibbles, j, L.lum_samples, i, px, py, L.scramble64,
                                          L.lum_dim, nx, ny);
                        NeeSample ns = emitter_sample<ENV, ANA>(S, hs, its.p, refN, nx, ny);
                        if (ns.pdf != 0 && occluded(its.p, ns.d, ns.dist)) ns.value = mk(0, 0, 0);
                        if (ns.pdf == 0) ns.value = mk(0, 0, 0);
                        if (!is_zero(ns.value)) {
                            const f3 wo = to_local(its.sh, ns.d);
                            f3 bsdfVal;
                            float bsdfPdf;
                            bsdf_eval_pdf_2s<EXT>(S, bsdf, its, wo, bsdfVal, &bsdfPdf);
                            if (!is_zero(bsdfVal) && (!L.strict_normals || dot(its.geoN, ns.d) * wo.z > 0)) {
                                const float pa = ns.pdf * L.frac_lum, pb = bsdfPdf * L.frac_bsdf;
                                const float weight = (pa * pa) / (pa * pa + pb * pb) * L.weight_lum;
                                Li = add(Li, mul(mulv(ns.value, bsdfVal), weight));
                            }
                        }
                    }
                }
                // BSDF sampling (direct.cpp:241-304)
                if (L.bsdf_samples <= 1) next2d_a(SC, L.resolution, smp, px, py, L.array_end, su, sv);
                for (uint32_t i = 0; i < L.bsdf_samples; ++i) {
                    float bx = su, by = sv;
                    if (L.bsdf_samples > 1)
                        sobol_array2d(SC, L.lut, ycolTab, L.nibbles, j, L.bsdf_samples, i, px, py, L.scramble64,
                                      L.bsdf_dim, bx, by);
                    float u1d = 0.0f;
                    if (bsdf.type == BSDF_ROUGHDIELECTRIC) u1d = next1d_a(SC, smp, L.array_end);
                    const BSample bs = bsdf_sample_2s<EXT>(S, bsdf, its, bx, by, u1d);
                    if (is_zero(bs.weight)) continue;
                    const f3 wo = to_world(its.sh, bs.wo);
                    if (L.strict_normals && dot(its.geoN, wo) * bs.wo.z <= 0) continue;
                    Hit h2;
                    f3 value;
                    float lumPdf = 0.0f;
                    if (closest(its.p, wo, D_EPSILON, INFINITY, h2)) {
                        if (hs.shapes[h2.shape].emitter < 0) continue;
                        value = area_Le(S, h2, neg(wo));
                        if (!(bs.sampledType & MTSG_F_DELTA)) lumPdf = area_hit_pdf<ANA>(S, h2, its.p, wo, refN);
                    } else {
                        if (!ENV || (L.hide_emitters && bs.sampledType == MTSG_F_NULL)) continue;
                        glb_env *E = (glb_env *)S.env;
                        value = E->constant ? mk(E->radiance[0], E->radiance[1], E->radiance[2]) : env_eval(E, wo);
                        float nT, fT;
                        if (!env_bsphere(E, its.p, wo, nT, fT) || nT > 0 || fT < 0) continue;
                        if (!(bs.sampledType & MTSG_F_DELTA))
                            lumPdf = (E->constant ? const_pdf_direct(wo, refN) : env_pdf_direction(E, wo)) *
                                     (S.emitters[S.env_emitter].weight * S.em_norm);
                    }
                    const float pa = bs.pdf * L.frac_bsdf, pb = lumPdf * L.frac_lum;
                    const float weight = (pa * pa) / (pa * pa + pb * pb) * L.weight_bsdf;
                    Li = add(Li, mul(mulv(value, bs.weight), weight));
                }
            }
        }
        // block->put(samplePos, spec, alpha) (integrator.cpp:184), as path_kernel
        const float val[5] = {Li.x, Li.y, Li.z, alpha, 1.0f};
        film_record(L, film_slot(L, j - L.j0, pix), px, py, sx, sy, val, alpha != 0.0f);
        if (L.samples) {
            const uint32_t pixIdx = (uint32_t)(py - (int)L.y0) * L.width + (uint32_t)(px - (int)L.x0);
            float *rec = L.samples + ((size_t)pixIdx * L.spp + j) * 8;
            rec[0] = Li.x; rec[1] = Li.y; rec[2] = Li.z; rec[3] = alpha;
            rec[4] = sx; rec[5] = sy; rec[6] = 1.0f; rec[7] = smp.err ? 1.0f : 0.0f;
        }
        cSamples++;
        if (smp.err) cErr++;
    }
    atomicAdd(L.counters + 0, cSamples);
    atomicAdd(L.counters + 1, cRays);
    atomicAdd(L.counters + 2, cShadow);
    atomicAdd(L.counters + 3, cSamples);   // rRec.depth = 1 per sample
    if (cErr) atomicAdd(L.counters + 6, cErr);
}

// Scene::rayIntersect / Scene::isOccluded on a batch of rays (one ray per lane):
// rays[2i] = {o, mint}, rays[2i+1] = {d, maxt}; out[i] = {t, u, v, prim bits}
// (prim 0xffffffff and t = inf: no hit; the shadow query writes t = 1 / 0)
template <bool ANY, int WAVES, bool ANA>
__global__ __launch_bounds__(BLOCK, WAVES) void trace_kernel(MtsgDeviceScene S, const float4 *__restrict__ rays,
                                                              uint32_t n, float4 *__restrict__ out,
                                                              uint32_t stackDepth) {
    extern __shared__ uint32_t lds[];
    lds_stk_n *stkN = (lds_stk_n *)lds + threadIdx.x;
    lds_stk_d *stkD = (lds_stk_d *)(lds + stackDepth * BLOCK) + threadIdx.x;
    unsigned long long cn = 0, ct = 0;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        const float4 a = rays[2 * (size_t)i], b = rays[2 * (size_t)i + 1];
        const f3 o = mk(a.x, a.y, a.z), d = mk(b.x, b.y, b.z);
        float4 r = make_float4(INFINITY, 0.0f, 0.0f, __uint_as_float(0xffffffffu));
        float mint, maxt;
        if (ray_interval(S, o, d, a.w, b.w, ANY, mint, maxt)) {
            uint32_t slot = 0;
            float u = 0, v = 0, t = 0;
            const bool hit = traverse<ANY, false, ANA>((glb_node *)S.nodes, (glb_tri *)S.tris, o, d, mint, maxt, stkN,
                                                       stkD, slot, u, v, t, cn, ct, S.analytic);
            if (ANY) r.x = hit ? 1.0f : 0.0f;
            else if (hit) r = make_float4(t, u, v, __uint_as_float(S.tris[slot].prim));
        } else if (ANY) {
            r.x = 0.0f;
        }
        out[i] = r;
    }
}

template <bool ANY>
__global__ __launch_bounds__(BLOCK) void trace_kd_kernel(MtsgDeviceScene S, const uint2 *__restrict__ kdNodes,
                                                         const uint32_t *__restrict__ kdIndices,
                                                         const MtsgTri *__restrict__ kdTris,
                                                         const float4 *__restrict__ rays, uint32_t n,
                                                         float4 *__restrict__ out) {
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        const float4 a = rays[2 * (size_t)i], b = rays[2 * (size_t)i + 1];
        const f3 o = mk(a.x, a.y, a.z), d = mk(b.x, b.y, b.z);
        float4 r = make_float4(INFINITY, 0.0f, 0.0f, __uint_as_float(0xffffffffu));
        float mint, maxt;
        if (ray_interval(S, o, d, a.w, b.w, ANY, mint, maxt)) {
            float t = 0, u = 0, v = 0;
            uint32_t prim = 0;
            const bool hit = kd_traverse<ANY>(kdNodes, kdIndices, kdTris, o, d, mint, maxt, t, u, v, prim);
            if (ANY) r.x = hit ? 1.0f : 0.0f;
            else if (hit) r = make_float4(t, u, v, __uint_as_float(prim));
        } else if (ANY) {
            r.x = 0.0f;
        }
        out[i] = r;
    }
}

// per-pixel ordered sum of the own-pixel splats: film_own[p] (+)= c[0] + c[1] + ...
// in sample order -- the reference's `*dest++ += weight * value[k]` sequence
__global__ void film_reduce(MtsgLaunch L) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= L.num_pixels) return;
    int px, py;
    if (!pixel_of(L, p, px, py)) return;
    float *dst = L.film_own + ((size_t)(py + L.filter.border) * L.fw + (px + L.filter.border)) * 5;
    float acc[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) acc[k] = dst[k];
    const float4 *c = reinterpret_cast<const float4 *>(L.contrib);
    for (uint32_t jj = 0; jj < L.chunk_spp; ++jj) {
        const float4 r = c[film_slot(L, jj, p)];
        const float w = fabsf(r.w);
        const float alpha = signbit(r.w) ? 0.0f : 1.0f;
        acc[0] += w * r.x;
        acc[1] += w * r.y;
        acc[2] += w * r.z;
        acc[3] += w * alpha;
        acc[4] += w * 1.0f;
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) dst[k] = acc[k];
}

// ---------------------------------------------------------------------------
// gather mode (gaussian and other filters whose footprint covers neighbours):
// every film pixel forms its own sum from the sample records of the pixels
// around it, in one fixed order, so the film is deterministic and equal to the
// oracle's (oracle/mts_oracle.c film_gather) bit for bit: for each sample
// index j (ascending), the source pixels q of the (2H+1)^2 neighbourhood in
// row-major order, each adding weight * value[k] with weight =
// weightsX[x] * weightsY[y] as ImageBlock::put forms them (imageblock.h:
// 124-204; footprint and discretised filter exactly as film_splat, so the
// 32x32 block bitmap's clip and the film edge are kept).  The reference's own
// order is its block schedule's (Film::put merges blocks as they finish,
// renderproc.cpp:142-149); this one replaces the atomic neighbour splats, which
// had no order at all.
//
// One workgroup: a 16 x 16R tile of film pixels, R = gather_rows(H) vertically
// adjacent pixels per thread.  Per sample index the tile's (16+2H) x (16R+2H)
// source records are staged in LDS together with their per-axis weights towards
// every offset -H..H (formed once per record, not once per neighbour), then each
// thread adds the (2H+1)^2 neighbours of each of its pixels from LDS.
// ---------------------------------------------------------------------------
// the compact pixel index p (work items' pixel, pixel_of's inverse) of image
// pixel (qx, qy), or -1 when this launch does not render it (outside the
// window, or another shard's rows / tiles)
__device__ __forceinline__ long long pix_index(const MtsgLaunch &L, int qx, int qy) {
    const int lx = qx - (int)L.x0, ly = qy - (int)L.y0;
    if (lx < 0 || ly < 0 || lx >= (int)L.width || ly >= (int)L.height) return -1;
    uint32_t tile, in;
    if (L.tile_shard) {
        const uint32_t t = (uint32_t)(ly >> 3) * L.tiles_x + (uint32_t)(lx >> 3);
        if (t % L.row_stride != L.row_phase) return -1;
        tile = t / L.row_stride;
        in = (uint32_t)(ly & 7) * 8u + (uint32_t)(lx & 7);
    } else {
        const uint32_t blkAbs = (uint32_t)ly / L.row_block;
        if (blkAbs % L.row_stride != L.row_phase) return -1;
        const uint32_t r = (blkAbs / L.row_stride) * L.row_block + (uint32_t)ly % L.row_block;
        tile = (r >> 3) * L.tiles_x + (uint32_t)(lx >> 3);
        in = (r & 7u) * 8u + (uint32_t)(lx & 7);
    }
    return (long long)tile * 64 + in;
}

typedef float f2v __attribute__((ext_vector_type(2)));
#ifndef MTSG_GATHER_PK
#define MTSG_GATHER_PK 1
#endif
#define GATHER_T 16
// output rows per thread: a thread sums GATHER_ROWS vertically adjacent film pixels, so each
// staged source record and x weight read from LDS serves up to GATHER_ROWS of its sums
#ifndef MTSG_GATHER_ROWS
#define MTSG_GATHER_ROWS 2
#endif
// (H = 4 keeps one row: two would need 85 KB of LDS per block)
__host__ __device__ constexpr int gather_rows(int H) { return H <= 3 ? MTSG_GATHER_ROWS : 1; }
__host__ __device__ constexpr size_t gather_lds_floats(int H) {
    return (size_t)(GATHER_T + 2 * H) * (GATHER_T * gather_rows(H) + 2 * H) * (4 + 2 * (2 * H + 1)) + 32;
}

template <int H>
__global__ __launch_bounds__(256) void film_gather(MtsgLaunch L, int gx0, int gy0, int gx1, int gy1) {
    constexpr int R = gather_rows(H), TY = GATHER_T * R;
    constexpr int SWX = GATHER_T + 2 * H, SWY = TY + 2 * H, S = SWX * SWY, NW = 2 * H + 1;
    constexpr int SLOTS = (S + 255) / 256;
    extern __shared__ float glds[];
    float4 *val = reinterpret_cast<float4 *>(glds);   // [S] {L.rgb, alpha}
    float *wxs = glds + 4 * S;                          // [NW][S] weight towards film x = q's + (o - H)
    float *wys = wxs + NW * S;                          // [NW][S]
    float *fv = wys + NW * S;                           // the discretised filter (32 values)
    const MtsgFilter &F = L.filter;
    const int b = F.border, bw = MTSG_BLOCK_SIZE + 2 * b;
    const int tx = threadIdx.x & (GATHER_T - 1), tr = threadIdx.x / GATHER_T;   // output rows tr * R + i
    const int ox = gx0 + blockIdx.x * GATHER_T, oy = gy0 + blockIdx.y * TY;
    const int gx = ox + tx;
    // source s = image pixel (sx0 + s % SWX, sy0 + s / SWX): film position q + b = g + d, d in [-H, H]
    const int sx0 = ox - b - H, sy0 = oy - b - H;
    for (int i = threadIdx.x; i <= MTSG_FILTER_RES; i += 256) fv[i] = F.values[i];
    long long pi[SLOTS];
    int rendered = 0;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) {
        const int s = threadIdx.x + 256 * k;
        pi[k] = s < S ? pix_index(L, sx0 + s % SWX, sy0 + s / SWX) : -1;
        rendered |= pi[k] >= 0;
    }
    // a tile none of whose sources this launch renders (another shard's part of the
    // window: with N-way tile sharding a rank renders every N-th tile column) keeps
    // its film values: the whole block leaves before the first barrier
    if (!__syncthreads_or(rendered)) return;
    bool live[R];
    float *dst[R];
    f2v a01[R], a23[R];
    float aw[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int gy = oy + tr * R + i;
        live[i] = gx < gx1 && gy < gy1;
        dst[i] = L.film_own + ((size_t)gy * L.fw + gx) * 5;
        float acc[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        if (live[i]) {
#pragma unroll
            for (int k = 0; k < 5; ++k) acc[k] = dst[i][k];   // the previous chunks' running sums
        }
        a01[i] = f2v{acc[0], acc[1]};
        a23[i] = f2v{acc[2], acc[3]};
        aw[i] = acc[4];
    }
    bool anyLive = false;
#pragma unroll
    for (int i = 0; i < R; ++i) anyLive |= live[i];
    const float4 *rec = reinterpret_cast<const float4 *>(L.contrib);
    for (uint32_t jj = 0; jj < L.chunk_spp; ++jj) {
        __syncthreads();   // the previous sample's neighbours are summed
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) {
            const int s = threadIdx.x + 256 * k;
            if (s >= S) break;
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            float wx[NW], wy[NW];
#pragma unroll
            for (int o = 0; o < NW; ++o) wx[o] = wy[o] = 0.0f;
            if (pi[k] >= 0) {
                const size_t slot = (size_t)jj * L.num_pixels + (size_t)pi[k];
                const float4 r = rec[2 * slot];
                const float sy = rec[2 * slot + 1].x;
                if (!signbit(sy)) {
                    const int qx = sx0 + s % SWX, qy = sy0 + s / SWX;
                    const float sx = fabsf(r.w);
                    v = make_float4(r.x, r.y, r.z, signbit(r.w) ? 0.0f : 1.0f);
                    // film_splat's footprint in the block bitmap of q's 32x32 block
                    const int bx = (qx / MTSG_BLOCK_SIZE) * MTSG_BLOCK_SIZE, by = (qy / MTSG_BLOCK_SIZE) * MTSG_BLOCK_SIZE;
                    const float posx = sx - 0.5f - (float)(bx - b), posy = sy - 0.5f - (float)(by - b);
                    const int minx = max((int)ceilf(posx - F.radius), 0), miny = max((int)ceilf(posy - F.radius), 0);
                    const int maxx = min((int)floorf(posx + F.radius), bw - 1), maxy = min((int)floorf(posy + F.radius), bw - 1);
#pragma unroll
                    for (int o = 0; o < NW; ++o) {
                        const int x = qx + b + (o - H) - bx, y = qy + b + (o - H) - by;   // block-local
                        if (x >= minx && x <= maxx && qx + b + (o - H) < L.fw) {
                            int i = (int)fabsf(((float)x - posx) * F.scale);
                            wx[o] = fv[min(i, MTSG_FILTER_RES)];
                        }
                        if (y >= miny && y <= maxy && qy + b + (o - H) < L.fh) {
                            int i = (int)fabsf(((float)y - posy) * F.scale);
                            wy[o] = fv[min(i, MTSG_FILTER_RES)];
                        }
                    }
                }
            }
            val[s] = v;
#pragma unroll
            for (int o = 0; o < NW; ++o) {
                wxs[o * S + s] = wx[o];
                wys[o * S + s] = wy[o];
            }
        }
        __syncthreads();
        if (anyLive) {
            // source row rr of the thread's window (film rows tr * R - H .. tr * R + R - 1 + H):
            // output i takes it as neighbour row dy = rr - i - H, so each output still adds its
            // neighbours in row-major order.  neighbour d = (dx, dy): source q at film position
            // g + d; g sits at offset -d from it.  The four value channels as two packed pairs
            // (v_pk_mul_f32 + v_pk_add_f32: each half the IEEE product and sum of its own channel)
#pragma unroll
            for (int rr = 0; rr < 2 * H + R; ++rr) {
#pragma unroll
                for (int dx = -H; dx <= H; ++dx) {
                    const int s = (tr * R + rr) * SWX + (tx + H + dx);
                    const float wxv = wxs[(H - dx) * S + s];
                    const float4 v = val[s];
#pragma unroll
                    for (int i = 0; i < R; ++i) {
                        const int dy = rr - i - H;
                        if (dy < -H || dy > H) continue;
                        const float w = wxv * wys[(H - dy) * S + s];
#if MTSG_GATHER_PK
                        const f2v ww = {w, w};
                        a01[i] += ww * f2v{v.x, v.y};
                        a23[i] += ww * f2v{v.z, v.w};
#else
                        a01[i].x += w * v.x;
                        a01[i].y += w * v.y;
                        a23[i].x += w * v.z;
                        a23[i].y += w * v.w;
#endif
                        aw[i] += w * 1.0f;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
        if (!live[i]) continue;
        dst[i][0] = a01[i].x; dst[i][1] = a01[i].y; dst[i][2] = a23[i].x; dst[i][3] = a23[i].y; dst[i][4] = aw[i];
    }
}

__global__ void film_finalize(float *__restrict__ own, const double *__restrict__ spill, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) own[i] += (float)spill[i];
}

// the device's SFMT19937 stream: n nextULong draws from the stream at w (one lane)
__global__ void sfmt_probe(uint32_t *w, unsigned long long *out, int n) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    for (int i = 0; i < n; ++i) out[i] = sfmt_next_ulong((glb_w32 *)w);
}

hipError_t mtsg_launch_sfmt_probe(uint32_t *w, unsigned long long *out, int n, hipStream_t s) {
    hipLaunchKernelGGL(sfmt_probe, dim3(1), dim3(64), 0, s, w, out, n);
    return hipGetLastError();
}

// element-wise IEEE checks of the device arithmetic the path relies on
__global__ void arith_probe(const float *a, const float *b, float *out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s, c;
    d_sincos(a[i], &s, &c);
    out[8 * i + 0] = a[i] / b[i];
    out[8 * i + 1] = dsqrt(fabsf(a[i]));
    out[8 * i + 2] = s;
    out[8 * i + 3] = c;
    out[8 * i + 4] = d_acos(fminf(fmaxf(a[i], -1.0f), 1.0f));
    out[8 * i + 5] = d_atan2(a[i], b[i]);
    out[8 * i + 6] = d_fastexp(-fabsf(a[i]));
    out[8 * i + 7] = a[i] * b[i] + a[i];
}

// ---------------------------------------------------------------------------
// host-side launchers (called by capi.cpp)
// ---------------------------------------------------------------------------
size_t mtsg_path_lds_bytes(const MtsgLaunch &L) {
    const size_t scene = L.scene_lds ? ((size_t)L.num_nodes * 16 + (size_t)L.scene.num_prims * (12 + 7) +
                                        (size_t)L.num_verts * 6 + (size_t)L.num_shapes * (sizeof(MtsgShape) / 4))
                                     : 0;
    return ((size_t)L.lds_dims * L.nibbles * 16 + 16 * 16 + scene + ((size_t)L.stack_depth * 3 * BLOCK + 1) / 2) * 4;
}

// the megakernel variants, one object per scene feature set (path_f.hip)
#define MTSG_PATH_F_DECL(N)                                                                                  \
    hipError_t mtsg_launch_path_f##N(const MtsgLaunch &L, int grid, bool instr, hipStream_t s, int bits);   \
    int mtsg_path_occupancy_f##N(const MtsgLaunch &L, int bits, int *bpc);
MTSG_PATH_F_DECL(0) MTSG_PATH_F_DECL(1) MTSG_PATH_F_DECL(2) MTSG_PATH_F_DECL(3) MTSG_PATH_F_DECL(6)
MTSG_PATH_F_DECL(7)
#undef MTSG_PATH_F_DECL

int mtsg_path_features(const MtsgLaunch &L) {
    return (L.scene.env_emitter >= 0 ? MTSG_FEAT_ENV : 0) | ((L.ext || L.ana) ? MTSG_FEAT_EXT : 0) |
           (L.ana ? MTSG_FEAT_ANA : 0);
}

// The BSDF-set specialisation (dbsdf.h BSet) of large scenes: bit 0 = every
// rough BSDF uses GGX, bit 1 = no roughdielectric, bit 2 = no roughconductor
// (capi.cpp L.bset).  Every feature set has all 7 sets compiled (path_f.hip);
// small scenes staged in LDS and the direct integrator take the generic kernel.
static int spec_bits(const MtsgLaunch &L) {
    if (L.scene_lds || L.integrator == MTSG_INTEGRATOR_DIRECT) return 0;
    const int b = ((L.bset & MTSG_FEAT_GGX) ? 1 : 0) | ((L.bset & MTSG_FEAT_NORD) ? 2 : 0) | ((L.bset & MTSG_FEAT_NORC) ? 4 : 0);
    return b | ((b && (L.bset & MTSG_FEAT_NOREFN) && (mtsg_path_features(L) & MTSG_FEAT_ENV)) ? 8 : 0);
}

template <int FEAT>
static void launch_direct(const MtsgLaunch &L, int grid, hipStream_t stream) {
    const size_t lds = mtsg_path_lds_bytes(L);
    if (L.scene_lds) hipLaunchKernelGGL((direct_kernel<true, FEAT>), dim3(grid), dim3(BLOCK), lds, stream, L);
    else hipLaunchKernelGGL((direct_kernel<false, FEAT>), dim3(grid), dim3(BLOCK), lds, stream, L);
}

hipError_t mtsg_launch_path(const MtsgLaunch &L, int grid, bool samples, bool stats, hipStream_t stream) {
    const bool instr = samples || stats;
    if (L.integrator == MTSG_INTEGRATOR_DIRECT) {
        switch (mtsg_path_features(L)) {
            case 0: launch_direct<0>(L, grid, stream); break;
            case MTSG_FEAT_ENV: launch_direct<MTSG_FEAT_ENV>(L, grid, stream); break;
            case MTSG_FEAT_EXT: launch_direct<MTSG_FEAT_EXT>(L, grid, stream); break;
            case MTSG_FEAT_ENV | MTSG_FEAT_EXT: launch_direct<MTSG_FEAT_ENV | MTSG_FEAT_EXT>(L, grid, stream); break;
            case MTSG_FEAT_EXT | MTSG_FEAT_ANA: launch_direct<MTSG_FEAT_EXT | MTSG_FEAT_ANA>(L, grid, stream); break;
            default: launch_direct<MTSG_FEAT_ENV | MTSG_FEAT_EXT | MTSG_FEAT_ANA>(L, grid, stream); break;
        }
        return hipGetLastError();
    }
    const int bits = spec_bits(L);
    switch (mtsg_path_features(L)) {
        case 0: return mtsg_launch_path_f0(L, grid, instr, stream, bits);
        case MTSG_FEAT_ENV: return mtsg_launch_path_f1(L, grid, instr, stream, bits);
        case MTSG_FEAT_EXT: return mtsg_launch_path_f2(L, grid, instr, stream, bits);
        case MTSG_FEAT_ENV | MTSG_FEAT_EXT: return mtsg_launch_path_f3(L, grid, instr, stream, bits);
        case MTSG_FEAT_EXT | MTSG_FEAT_ANA: return mtsg_launch_path_f6(L, grid, instr, stream, bits);
        default: return mtsg_launch_path_f7(L, grid, instr, stream, bits);
    }
}

hipError_t mtsg_launch_reduce(const MtsgLaunch &L, hipStream_t stream) {
    const int threads = 256;
    const int blocks = (int)((L.num_pixels + threads - 1) / threads);
    hipLaunchKernelGGL(film_reduce, dim3(blocks), dim3(threads), 0, stream, L);
    return hipGetLastError();
}

// gather mode: the film pixels the launch's samples can reach, [x0 + b - H, x0 + w + b + H)
// x [y0 + b - H, y0 + h + b + H) clipped to the film, in tiles of 16 x (16 * gather_rows(H))
hipError_t mtsg_launch_gather(const MtsgLaunch &L, hipStream_t stream) {
    const int H = (int)L.gather_h, b = L.filter.border;
    const int gx0 = std::max(0, (int)L.x0 + b - H), gy0 = std::max(0, (int)L.y0 + b - H);
    const int gx1 = std::min(L.fw, (int)(L.x0 + L.width) + b + H), gy1 = std::min(L.fh, (int)(L.y0 + L.height) + b + H);
    if (gx1 <= gx0 || gy1 <= gy0) return hipSuccess;
    const int ty = GATHER_T * gather_rows(H);
    const dim3 grid((gx1 - gx0 + GATHER_T - 1) / GATHER_T, (gy1 - gy0 + ty - 1) / ty);
    const size_t lds = gather_lds_floats(H) * 4;
    switch (H) {
        case 1: hipLaunchKernelGGL(film_gather<1>, grid, dim3(256), lds, stream, L, gx0, gy0, gx1, gy1); break;
        case 2: hipLaunchKernelGGL(film_gather<2>, grid, dim3(256), lds, stream, L, gx0, gy0, gx1, gy1); break;
        case 3: hipLaunchKernelGGL(film_gather<3>, grid, dim3(256), lds, stream, L, gx0, gy0, gx1, gy1); break;
        case 4: hipLaunchKernelGGL(film_gather<4>, grid, dim3(256), lds, stream, L, gx0, gy0, gx1, gy1); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t mtsg_launch_finalize(float *own, const double *spill, size_t n, hipStream_t stream) {
    const int threads = 256;
    const int blocks = (int)((n + threads - 1) / threads);
    if (blocks > 0) hipLaunchKernelGGL(film_finalize, dim3(blocks), dim3(threads), 0, stream, own, spill, n);
    return hipGetLastError();
}

hipError_t mtsg_launch_trace(const MtsgDeviceScene &S, const float *rays, uint32_t n, float *out, bool shadow,
                             uint32_t stackDepth, int numCUs, hipStream_t stream) {
    const size_t lds = (size_t)stackDepth * 3 * BLOCK / 2 * 4 + 16;
    int bpc = 1;
    if (shadow) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, trace_kernel<true, 8, false>, BLOCK, lds);
    else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, trace_kernel<false, 8, false>, BLOCK, lds);
    const uint32_t want = (n + BLOCK - 1) / BLOCK;
    const int grid = (int)std::max<uint32_t>(1, std::min<uint32_t>(want, (uint32_t)(std::max(bpc, 1) * numCUs)));
    const bool ana = S.analytic != nullptr;
#define MTSG_TRACE(A, N) hipLaunchKernelGGL((trace_kernel<A, 8, N>), dim3(grid), dim3(BLOCK), lds, stream, S, \
                                            (const float4 *)rays, n, (float4 *)out, stackDepth)
    if (shadow) { if (ana) MTSG_TRACE(true, true); else MTSG_TRACE(true, false); }
    else { if (ana) MTSG_TRACE(false, true); else MTSG_TRACE(false, false); }
#undef MTSG_TRACE
    return hipGetLastError();
}

hipError_t mtsg_launch_trace_kd(const MtsgDeviceScene &S, const uint32_t *kdNodes, const uint32_t *kdIndices,
                                const MtsgTri *kdTris, const float *rays, uint32_t n, float *out, bool shadow,
                                int numCUs, hipStream_t stream) {
    const uint32_t want = (n + BLOCK - 1) / BLOCK;
    const int grid = (int)std::max<uint32_t>(1, std::min<uint32_t>(want, (uint32_t)(4 * numCUs)));
    if (shadow)
        hipLaunchKernelGGL(trace_kd_kernel<true>, dim3(grid), dim3(BLOCK), 0, stream, S, (const uint2 *)kdNodes,
                           kdIndices, kdTris, (const float4 *)rays, n, (float4 *)out);
    else
        hipLaunchKernelGGL(trace_kd_kernel<false>, dim3(grid), dim3(BLOCK), 0, stream, S, (const uint2 *)kdNodes,
                           kdIndices, kdTris, (const float4 *)rays, n, (float4 *)out);
    return hipGetLastError();
}

hipError_t mtsg_launch_arith_probe(const float *a, const float *b, float *out, int n, hipStream_t stream) {
    hipLaunchKernelGGL(arith_probe, dim3((n + 255) / 256), dim3(256), 0, stream, a, b, out, n);
    return hipGetLastError();
}

// the FEAT template argument of the megakernel mtsg_launch_path runs for L
// (reported through debug counter 15 so the tests can see which one ran)
int mtsg_path_variant(const MtsgLaunch &L) {
    const int bits = spec_bits(L), f = mtsg_path_features(L);
    if (bits) return f | MTSG_FEAT_NOSTRICT | ((bits & 1) ? MTSG_FEAT_GGX : 0) | ((bits & 2) ? MTSG_FEAT_NORD : 0) |
                     ((bits & 4) ? MTSG_FEAT_NORC : 0) | ((bits & 8) ? MTSG_FEAT_NOREFN : 0);
    return (f == 0 && L.all_diffuse) ? (int)MTSG_FEAT_DIFF : f;
}

int mtsg_path_kernel_occupancy(const MtsgLaunch &L, int *blocksPerCU) {
    const int bits = spec_bits(L);
    switch (mtsg_path_features(L)) {
        case 0: return mtsg_path_occupancy_f0(L, bits, blocksPerCU);
        case MTSG_FEAT_ENV: return mtsg_path_occupancy_f1(L, bits, blocksPerCU);
        case MTSG_FEAT_EXT: return mtsg_path_occupancy_f2(L, bits, blocksPerCU);
        case MTSG_FEAT_ENV | MTSG_FEAT_EXT: return mtsg_path_occupancy_f3(L, bits, blocksPerCU);
        case MTSG_FEAT_EXT | MTSG_FEAT_ANA: return mtsg_path_occupancy_f6(L, bits, blocksPerCU);
        default: return mtsg_path_occupancy_f7(L, bits, blocksPerCU);
    }
}
