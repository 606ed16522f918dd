// dmega.h -- the persistent megakernel of Mitsuba 0.6's `path` integrator
// (MIPathTracer::Li, src/integrators/path/path.cpp:119-294, inside
// SamplingIntegrator::renderBlock, src/librender/integrator.cpp:140-188),
// instantiated per scene feature set in path_f.hip:
//
//  * lane g of the persistent grid takes sample runs g, g + lanes, g + 2 lanes, ...
//    (static striding: no queue, no tail of long per-pixel tasks), a run being
//    2^round_shift consecutive samples of one pixel, one after the other;
//  * a lane whose path ends starts its next item immediately (regeneration);
//  * each loop iteration traces the lane's pending shadow ray and its
//    closest-hit ray, then shades (PathShader, dpath.h);
//  * LDS holds the Sobol tables and the lane-strided traversal stacks (and
//    the whole scene for small ones).
#pragma once
#include "dpath.h"

size_t mtsg_path_lds_bytes(const MtsgLaunch &L);   // path_kernel.hip

// tiny-scene kernels keep a pair's first splat record in registers (PathShader::finish)
#ifndef MTSG_HOLD_PAIR
#define MTSG_HOLD_PAIR 1
#endif

// diagnostic build (-DMTSG_MK_STAMPS): wave cycles per megakernel section,
// summed into counters 11-14 (start, shadow trace, closest trace, shade) by
// lane 0 of each wave.  s_memtime without draining the memory counters: a
// section's loads are consumed inside it (traversal, shading), so the split is
// close; read shares, not times (tools/mk_stamps.py)
#ifdef MTSG_MK_STAMPS
#define MK_STAMP(acc, t0)                                                        \
    do {                                                                         \
        unsigned long long t1_;                                                  \
        __builtin_amdgcn_sched_barrier(0);                                       \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                       \
        acc += t1_ - t0;                                                         \
        t0 = t1_;                                                                \
    } while (0)
#else
#define MK_STAMP(acc, t0) (void)0
#endif


// The persistent megakernel: grid = CUs x resident blocks; every lane runs
// PathShader steps with both traversals inline
template <bool INSTR, bool SCENE_LDS, int FEAT, int WAVES>
__global__ __launch_bounds__(BLOCK, WAVES) void path_kernel(MtsgLaunch L) {   // L: the first argument (launch_fresh)
    constexpr bool STATS = INSTR;
    constexpr bool ANA = (FEAT & MTSG_FEAT_ANA) != 0;
    constexpr bool HNODES = (FEAT & (MTSG_FEAT_GGX | MTSG_FEAT_NORD | MTSG_FEAT_NORC)) != 0;
    extern __shared__ uint32_t lds[];
    (void)stage_lds<SCENE_LDS>(L, lds);
    PathCounters c = {};   // INSTR statistics only: the always-on counts are wave-uniform (wc)
    WaveCounters wc = {};

    // static striding: lane g takes sample runs g + k * lanes, k = 0, 1, ... (`round`
    // counts the lane's samples, or the SFMT replay's position in its unit: 32 bits,
    // not a 64-bit item index, live across the bounce loop)
    const uint64_t lanes = (uint64_t)gridDim.x * BLOCK;
    const uint32_t g = xcd_block(L.xcds) * BLOCK + threadIdx.x;
    uint32_t round = 0;
    bool done = false;
    float4 held = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // PathShader::finish's held splat record
    PathState st;
    st.active = false;
    st.pix = 0;
    st.smp.sobolIndex = 0; st.smp.sampleIndex = 0; st.smp.dim = 0; st.smp.err = false;
    st.sx = st.sy = 0;
    st.haveRay = st.primary = st.haveShadow = false;
    st.P.its.p = mk(0, 0, 0); st.rd = mk(0, 0, 1); st.sd = mk(0, 0, 1);
    st.rmint = st.rmaxt = st.smaxt = 0;
#ifdef MTSG_MK_STAMPS
    unsigned long long mkT[4] = {0, 0, 0, 0}, mkT0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(mkT0)::"memory");
#endif

    while (true) {
        // the launch record re-read per bounce instead of held (dpath.h launch_fresh),
        // and the LDS / scene pointers re-derived from it (dpath.h lds_view): C2 +2.0%,
        // C4 +3.8%, C5 +0.7%, C3 0 (profiles/r04_ab_fresh_view.log)
        const MtsgLaunch &L = launch_fresh();
        const MtsgDeviceScene &S = L.scene;
        const LdsView<SCENE_LDS> V = lds_view<SCENE_LDS>(L, lds);
        lds_node *ldsNodes = V.nodes;
        lds_tri *ldsTris = V.tris;
        lds_stk_n *stkN = (lds_stk_n *)(lds + V.stackBase) + threadIdx.x;
        lds_stk_d *stkD = (lds_stk_d *)(lds + V.stackBase + L.stack_depth * BLOCK) + threadIdx.x;
        const PathShader<INSTR, SCENE_LDS, FEAT> sh{L, V.hs, V.SC, V.ycolTab, c};
        // ---- A: start the next sample
        while (!st.active && !done) {
            if (L.replay) {   // SFMT replay: this lane's unit, pixel after pixel, in order
                const uint32_t unit = blockIdx.x * BLOCK + threadIdx.x;
                if (unit >= L.units) { done = true; break; }
                const uint32_t k0 = L.unit_start[unit], n = L.unit_start[unit + 1] - k0;
                if ((uint64_t)round >= (uint64_t)n * L.chunk_spp) { done = true; break; }
                const uint32_t k = k0 + round / L.chunk_spp, jj = round % L.chunk_spp;
                ++round;
                sh.start_xy(st, L.order[k], jj);
                break;
            }
            // sample runs: the lane's rounds r * 2^s .. r * 2^s + 2^s - 1 render samples
            // k * 2^s .. of one pixel back to back (run q = g + r * lanes; s = L.round_shift):
            // a box-filter record sector (film_slot: samples 2k, 2k + 1) has both halves
            // stored one path apart, while the line is still in this XCD's L2, and the
            // wave's primary rays revisit the same pixels
            const uint32_t rs = L.round_shift;
            const uint64_t q = g + (uint64_t)(round >> rs) * lanes;
            const uint32_t jq = (uint32_t)(q / L.num_pixels), jr = jq << rs, jj = jr + (round & ((1u << rs) - 1u));
            if (jr >= L.chunk_spp) { done = true; break; }
            ++round;
            if (jj < L.chunk_spp) sh.start_jp(st, jj, (uint32_t)(q - (uint64_t)jq * L.num_pixels));
        }
        if (__all(done)) break;
        MK_STAMP(mkT[0], mkT0);

        // ---- B: trace the shadow ray, then the closest-hit ray ---------------
        bool occluded = false;
        bool hit = false;
        uint32_t slot = 0, prim = 0;
        float hu = 0, hv = 0, ht = 0;
        if (SCENE_LDS && L.scan) {
            // tiny scene: both rays of the bounce in one pass (scan_pair); both
            // leave the same point, P.its.p
            float minS = INFINITY, maxS = -INFINITY, minC = INFINITY, maxC = -INFINITY;
            bool okS = false, okC = false;
            wc.shadow += wave_count(st.active && st.haveShadow);
            wc.rays += wave_count(st.active && st.haveRay);
            if (st.active && st.haveShadow) {
                if (!is_zero(st.P.neeC)) okS = ray_interval(S, st.P.its.p, st.sd, D_EPSILON, st.smaxt, true, minS, maxS);
                if (!okS) { minS = INFINITY; maxS = -INFINITY; }
            }
            if (st.active && st.haveRay) {
                okC = ray_interval(S, st.P.its.p, st.rd, st.rmint, st.rmaxt, false, minC, maxC);
                if (!okC) { minC = INFINITY; maxC = -INFINITY; }
            }
            if (__any(okS || okC))
                scan_pair<STATS>(L, st.P.its.p, st.sd, st.rd, minS, maxS, minC, maxC, occluded, hit,
                                 prim, hu, hv, ht, c.tests);
            hit = hit && okC;
            occluded = occluded && okS;
        } else {
        // (round 4 measured both rays of a bounce through one per-lane loop, traverse_seq:
        // bit-identical, but C3 -5.5%, C4 -10%, C5 -1.7%, profiles/r04_ab_seq_traversal.log; removed)
        wc.shadow += wave_count(st.active && st.haveShadow);
        if (st.active && st.haveShadow) {
            float mint, maxt;
            // a shadow ray whose estimate is zero cannot change Li: skip its traversal
            if (!is_zero(st.P.neeC) && ray_interval(S, st.P.its.p, st.sd, D_EPSILON, st.smaxt, true, mint, maxt)) {
                uint32_t sl; float a0, a1, a2;
                if (SCENE_LDS)
                    occluded = traverse<true, STATS, ANA>(ldsNodes, ldsTris, st.P.its.p, st.sd, mint, maxt, stkN,
                                                                stkD, sl, a0, a1, a2, c.nodes, c.tests, S.analytic);
                else if constexpr (HNODES)
                    occluded = traverse<true, STATS, ANA>((glb_hnode *)S.hnodes, (glb_tri *)S.tris, st.P.its.p,
                                                                st.sd, mint, maxt, stkN, stkD, sl, a0, a1, a2, c.nodes,
                                                                c.tests, S.analytic);
                else
                    occluded = traverse<true, STATS, ANA>((glb_node *)S.nodes, (glb_tri *)S.tris, st.P.its.p,
                                                                st.sd, mint, maxt, stkN, stkD, sl, a0, a1, a2, c.nodes,
                                                                c.tests, S.analytic);
            }
        }
        // the NEE estimate is added now (as shade() would first thing), so it
        // is not live across the closest-hit traversal
        if (st.active && st.haveShadow) {
            if (!occluded) st.P.L = add(st.P.L, st.P.neeC);
            st.haveShadow = false;
        }
        MK_STAMP(mkT[1], mkT0);
        wc.rays += wave_count(st.active && st.haveRay);
        if (st.active && st.haveRay) {
            float mint, maxt;
            if (ray_interval(S, st.P.its.p, st.rd, st.rmint, st.rmaxt, false, mint, maxt)) {
                if (SCENE_LDS)
                    hit = traverse<false, STATS, ANA>(ldsNodes, ldsTris, st.P.its.p, st.rd, mint, maxt, stkN, stkD,
                                                            slot, hu, hv, ht, c.nodes, c.tests, S.analytic);
                else if constexpr (HNODES)
                    hit = traverse<false, STATS, ANA>((glb_hnode *)S.hnodes, (glb_tri *)S.tris, st.P.its.p, st.rd,
                                                            mint, maxt, stkN, stkD, slot, hu, hv, ht, c.nodes, c.tests,
                                                            S.analytic);
                else
                    hit = traverse<false, STATS, ANA>((glb_node *)S.nodes, (glb_tri *)S.tris, st.P.its.p, st.rd,
                                                            mint, maxt, stkN, stkD, slot, hu, hv, ht, c.nodes, c.tests,
                                                            S.analytic);
            }
            if (hit) prim = SCENE_LDS ? ldsTris[slot].prim : S.tris[slot].prim;
        }
        }
        if (st.active && st.haveShadow) {   // scan_pair case
            if (!occluded) st.P.L = add(st.P.L, st.P.neeC);
            st.haveShadow = false;
        }

        MK_STAMP(mkT[2], mkT0);

        // ---- C: shade -------------------------------------------------------
        // wave-uniform counts: a path's length is 1 + the bounces that advanced its
        // depth (shade() advances it at most once), summed over finished samples
        const bool was = st.active;
        const int d0 = st.P.depth;
        bool ended = false;
        if (st.active && sh.shade(st, occluded, hit, slot, prim, hu, hv, ht)) {
            ended = true;
            sh.template finish<false>(st, MTSG_HOLD_PAIR && SCENE_LDS ? &held : nullptr);
        }
        wc.len += wave_count(was && st.P.depth != d0);
        wc.samples += wave_count(ended);
        wc.err += wave_count(ended && st.smp.err);
        if (__builtin_expect((wc.len | wc.rays | wc.shadow) >= 0x80000000u, 0)) {   // uniform: flush before a wrap
            wc.len += wc.samples;
            wave_counters_flush(L, wc);
            wc = WaveCounters{};
        }
        MK_STAMP(mkT[3], mkT0);
    }
    wc.len += wc.samples;
    wave_counters_flush(L, wc);
    path_counters_flush<STATS>(L, c);
#ifdef MTSG_MK_STAMPS
    if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0)
        for (int k = 0; k < 4; ++k) atomicAdd(L.counters + 11 + k, mkT[k]);
#endif
}


// one megakernel variant: its launch and its resident blocks per CU
template <bool SCENE_LDS, int FEAT, int WAVES>
static void launch_path_w(const MtsgLaunch &L, int grid, bool instr, hipStream_t stream) {
    const size_t lds = mtsg_path_lds_bytes(L);
    if (instr) hipLaunchKernelGGL((path_kernel<true, SCENE_LDS, FEAT, WAVES>), dim3(grid), dim3(BLOCK), lds, stream, L);
    else hipLaunchKernelGGL((path_kernel<false, SCENE_LDS, FEAT, WAVES>), dim3(grid), dim3(BLOCK), lds, stream, L);
}
template <bool SCENE_LDS, int FEAT, int WAVES>
static int occupancy_w(const MtsgLaunch &L, int *bpc) {
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(bpc, path_kernel<false, SCENE_LDS, FEAT, WAVES>, BLOCK,
                                                             mtsg_path_lds_bytes(L));
}
