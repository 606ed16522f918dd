// wf_impl.h -- the wavefront engine of Mitsuba 0.6's `path` integrator
// (MIPathTracer::Li, src/integrators/path/path.cpp:119-294, inside
// SamplingIntegrator::renderBlock, src/librender/integrator.cpp:140-188) as
// per-bounce kernels over SoA queues in HBM (BASELINE.json north star).
//
// The reference picks the BSDF per vertex through BSDF's virtual eval/sample
// (path.cpp:171-211).  Here the trace kernel that finds a path's next vertex
// sorts the path's slot into the queue of that vertex's BSDF type, and one
// shade kernel per type runs the rest of the bounce (PathShader, dpath.h,
// with KIND = that type): its BSDF code is inline and alone in the kernel, so
// each kernel keeps few registers and runs at its own occupancy, and a wave
// never executes two BSDFs' code.  Misses (and slots with no closest-hit ray)
// go to the MISS kernel, which also starts every slot's first path.
//
// Per bounce (parity p = bounce & 1):
//   shade_k  consumes cls[p][k]: shade / finish / regenerate; appends the next
//            closest-hit and shadow rays to ray[p], slots without a closest-hit
//            ray to cls[p^1][MISS];
//   trace    consumes ray[p]: writes hit[slot] / occl[slot], appends each
//            closest-hit ray's slot to cls[p^1][kind of the hit]; block 0 zeroes
//            the counters of the queues nobody reads or writes any more.
// Appends are one ballot + one atomic per wave and queue (wave_append); the
// results of every sample equal the megakernel's and the oracle's bit for bit
// (PathShader is the same code; only the order the slots take items differs).
#pragma once
#include "dpath.h"

#define WF_R MTSG_WF_REGIONS
#ifndef MTSG_WF_TRACE_WAVES
#define MTSG_WF_TRACE_WAVES 8
#endif


// per-wave append: one atomic for the wave, positions in lane order
__device__ __forceinline__ uint32_t wave_append(uint32_t *counter, bool pred) {
    const unsigned long long m = __ballot(pred);
    if (m == 0) return MTSG_WF_NONE;
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if ((int)lane_id() == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    return pred ? base + rank : MTSG_WF_NONE;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// per-block partial counters: [block][16] (MtsgLaunch::counters indices), summed by wf_flush;
// counter `atomicK` (if any) is instead added to *atomicDst (one atomic per block)
__device__ __forceinline__ void block_counters(unsigned long long *part, const uint32_t *v, uint32_t *red,
                                               int atomicK = -1, uint32_t *atomicDst = nullptr) {
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t s = wave_sum(v[k]);
        if (lane == 0) red[w * 16 + k] = s;
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        unsigned long long t = 0;
        for (uint32_t i = 0; i < BLOCK / 64; ++i) t += red[i * 16 + threadIdx.x];
        if ((int)threadIdx.x == atomicK) {
            if (t) atomicAdd(atomicDst, (uint32_t)t);
        } else if (t) {
            part[(size_t)blockIdx.x * 16 + threadIdx.x] += t;
        }
    }
}

// A queue's regions as one index space: the (wave-uniform) counts, their
// prefix, and entry i's position region * cap + offset
struct QueueView {
    uint32_t pre[WF_R + 1];
    __device__ __forceinline__ void load(const uint32_t *c) {
        pre[0] = 0;
#pragma unroll
        for (int r = 0; r < WF_R; ++r) pre[r + 1] = pre[r] + c[r];
    }
    __device__ __forceinline__ uint32_t total() const { return pre[WF_R]; }
    __device__ __forceinline__ size_t pos(uint32_t i, uint32_t cap) const {
        uint32_t r = 0;
#pragma unroll
        for (int k = 1; k < WF_R; ++k) r += i >= pre[k] ? 1u : 0u;
        uint32_t base = 0;
#pragma unroll
        for (int k = 0; k < WF_R; ++k) base = (uint32_t)k == r ? pre[k] : base;
        return (size_t)r * cap + (i - base);
    }
};

__device__ __forceinline__ uint32_t *wf_cnt(const MtsgWave &W, uint32_t parity, uint32_t queue) {
    return W.cnt + ((size_t)parity * MTSG_WF_QUEUES + queue) * WF_R;
}

// path state <-> slot s (AoS, 128 B): [0] L, eta  [1] thr, bsdfPdf  [2] neeC, alpha
// [3] refN, sx  [4] ray origin (P.its.p), sy  [5] rd, depth  [6] pix, j, sobol index
// [7] flags | dim << 16, sampledType, -, -
enum { WF_ACTIVE = 1, WF_RAY = 2, WF_PRIMARY = 4, WF_SHADOW = 8, WF_SCATTERED = 16, WF_EMITTED = 32, WF_ERR = 64,
       WF_DONE = 128,      // the slot's items are used up
       WF_SQUEUED = 256 }; // the shadow ray was queued (occl[slot] holds its answer)
__device__ __forceinline__ bool wf_load(const MtsgLaunch &L, const MtsgWave &W, uint32_t s, PathState &st,
                                        uint32_t &flags) {
    const float4 *v = W.state + (size_t)s * MTSG_WF_STATE_VECS;
    const uint4 f = reinterpret_cast<const uint4 *>(v)[7];
    const float4 a = v[0], b = v[1], c = v[2], d = v[3], e = v[4], g = v[5];
    const uint4 h = reinterpret_cast<const uint4 *>(v)[6];
    flags = f.x;
    st.active = (f.x & WF_ACTIVE) != 0;
    if (!st.active) {
        st.smp.sampleIndex = h.y; st.pix = h.x;   // the last item's (sample, pixel): regeneration continues after it
        return false;
    }
    st.P.L = mk(a.x, a.y, a.z); st.P.eta = a.w;
    st.P.thr = mk(b.x, b.y, b.z); st.P.bsdfPdf = b.w;
    st.P.neeC = mk(c.x, c.y, c.z); st.P.alpha = c.w != 0.0f;
    st.P.refN = mk(d.x, d.y, d.z); st.sx = d.w;
    st.P.its.p = mk(e.x, e.y, e.z); st.sy = e.w;
    st.rd = mk(g.x, g.y, g.z); st.P.depth = __float_as_int(g.w);
    st.pix = h.x;
    st.smp.sobolIndex = (uint64_t)h.z | ((uint64_t)h.w << 32);
    st.smp.sampleIndex = h.y;
    st.smp.dim = f.x >> 16;
    st.smp.err = (f.x & WF_ERR) != 0;
    PV_SET_DELTA(st.P, (int)f.y);
    st.haveRay = (f.x & WF_RAY) != 0;
    st.primary = (f.x & WF_PRIMARY) != 0;
    st.haveShadow = (f.x & WF_SHADOW) != 0;
    st.P.scattered = (f.x & WF_SCATTERED) != 0;
    st.P.emitted = (f.x & WF_EMITTED) != 0;
    return true;
}

__device__ __forceinline__ void wf_store(const MtsgWave &W, uint32_t s, const PathState &st, uint32_t extra) {
    float4 *v = W.state + (size_t)s * MTSG_WF_STATE_VECS;
    uint4 f;
    f.x = extra | (st.active ? WF_ACTIVE : 0) | (st.haveRay ? WF_RAY : 0) | (st.primary ? WF_PRIMARY : 0) |
          (st.haveShadow ? WF_SHADOW : 0) | (st.P.scattered ? WF_SCATTERED : 0) | (st.P.emitted ? WF_EMITTED : 0) |
          (st.smp.err ? WF_ERR : 0) | (st.smp.dim << 16);
    f.y = PV_DELTA(st.P) ? (uint32_t)MTSG_F_DELTA : 0u;
    f.z = f.w = 0;
    reinterpret_cast<uint4 *>(v)[7] = f;
    reinterpret_cast<uint4 *>(v)[6] =
        make_uint4(st.pix, st.smp.sampleIndex, (uint32_t)st.smp.sobolIndex, (uint32_t)(st.smp.sobolIndex >> 32));
    if (!st.active) return;
    v[0] = make_float4(st.P.L.x, st.P.L.y, st.P.L.z, st.P.eta);
    v[1] = make_float4(st.P.thr.x, st.P.thr.y, st.P.thr.z, st.P.bsdfPdf);
    v[2] = make_float4(st.P.neeC.x, st.P.neeC.y, st.P.neeC.z, st.P.alpha ? 1.0f : 0.0f);
    v[3] = make_float4(st.P.refN.x, st.P.refN.y, st.P.refN.z, st.sx);
    v[4] = make_float4(st.P.its.p.x, st.P.its.p.y, st.P.its.p.z, st.sy);
    v[5] = make_float4(st.rd.x, st.rd.y, st.rd.z, __int_as_float(st.P.depth));
}

// ---------------------------------------------------------------------------
// shade kernels: KIND = BSDF_* type of the queue's vertices (-1: any, the GEN
// queue), HITK = 1 (every closest-hit ray hit) or 2 (the MISS queue)
// ---------------------------------------------------------------------------
// One block of a shade kind's queue: queue entries kb * BLOCK + threadIdx of
// queue `queue` (n entries, view Q), one per thread.  No persistent loop, so
// nothing is carried or hoisted across items (a grid-stride loop kept the
// launch fields and the loop state live across the whole shading and spilled
// 170-560 VGPRs)
template <bool INSTR, int FEAT, int KIND, int HITK>
__device__ __forceinline__ void wf_shade_block(const MtsgLaunch &L, const MtsgWave &W, unsigned long long *part,
                                               uint32_t queue, const QueueView &Q, uint32_t n, uint32_t kb,
                                               uint32_t *lds, uint32_t *red) {
    const uint32_t p = W.parity, region = blockIdx.x % WF_R;
    const MtsgDeviceScene &S = L.scene;
    const LdsView<false> V = stage_lds<false>(L, lds);   // ends with a barrier
    PathCounters c = {};
    const PathShader<INSTR, false, FEAT, KIND, HITK> sh{L, V.hs, V.SC, V.ycolTab, c};
    const uint32_t *cls = W.cls[p] + (size_t)queue * WF_R * W.cap_cls;
    float4 *qray = W.ray[p], *sray = W.ray[p] + (size_t)2 * WF_R * W.cap;
    uint32_t *qslot = W.rslot[p], *sslot = W.rslot[p] + (size_t)WF_R * W.cap;
    uint32_t *missQ = W.cls[p ^ 1u];   // MTSG_WK_MISS = 0: the first kind queue
    uint32_t *cq = wf_cnt(W, p, 0) + region, *cs = wf_cnt(W, p, 1) + region;
    uint32_t *cm = wf_cnt(W, p ^ 1u, 2 + MTSG_WK_MISS) + region;
    const uint32_t i = kb * BLOCK + threadIdx.x;
    const bool valid = i < n;
    const uint32_t s = !valid ? 0u : W.seed ? i : cls[Q.pos(i, W.cap_cls)];
    PathState st;
    uint32_t flags = 0;
    st.active = false;
    const bool was = valid && !W.seed && wf_load(L, W, s, st, flags);
    bool occluded = false, hit = false;
    uint32_t slot = 0, prim = 0;
    float hu = 0, hv = 0, ht = 0;
    Hit pre;
    const bool usePre = HITK == 1 && W.hitrec != nullptr;   // launch-uniform
    if (was) {
        occluded = (flags & WF_SQUEUED) != 0 && W.occl[s] != 0;
        if constexpr (HITK == 1) {
            hit = true;
            if (usePre) {
                hit_load<(FEAT & MTSG_FEAT_EXT) != 0>(W.hitrec + (size_t)s * MTSG_WF_HIT_VECS, pre);
            } else {
                // the hit record's 4th word: the TriAccel slot with analytic shapes (fill_hit
                // reads the slot's record), else the primitive index itself
                const float4 h = W.hit[s];
                const uint32_t w = __float_as_uint(h.w);
                ht = h.x; hu = h.y; hv = h.z;
                if ((FEAT & MTSG_FEAT_ANA) != 0) { slot = w; prim = S.tris[slot].prim; }
                else prim = w;
            }
        }
    }
    // a slot in a queue is live, or (first bounce) not started yet
    bool done = false;
    if (was && sh.shade(st, occluded, hit, slot, prim, hu, hv, ht, usePre, pre)) {
        sh.finish(st);
        // regeneration: slot s takes items s, s + slots, s + 2 slots, ...
        uint64_t it = (uint64_t)(st.smp.sampleIndex - L.j0) * L.num_pixels + st.pix + W.slots;
        while (true) {
            if (it >= L.num_items) { done = true; break; }
            if (sh.start(st, it)) break;
            it += W.slots;   // padding pixel of a partial tile
        }
    } else if (valid && W.seed) {
        uint64_t it = s;
        while (true) {
            if (it >= L.num_items) { done = true; break; }
            if (sh.start(st, it)) break;
            it += W.slots;
        }
    }
    // the next bounce's rays (the megakernel's intervals and counts)
    float4 r0 = make_float4(0, 0, 0, 0), r1 = r0, s0 = r0, s1 = r0;
    bool ps = false, pr = false;
    if (st.active && st.haveShadow) {
        c.shadow++;
        float mint, maxt;
        if (!is_zero(st.P.neeC) && ray_interval(S, st.P.its.p, st.sd, D_EPSILON, st.smaxt, true, mint, maxt)) {
            ps = true;
            s0 = make_float4(st.P.its.p.x, st.P.its.p.y, st.P.its.p.z, mint);
            s1 = make_float4(st.sd.x, st.sd.y, st.sd.z, maxt);
        }
    }
    if (st.active && st.haveRay) {
        c.rays++;
        float mint, maxt;
        if (ray_interval(S, st.P.its.p, st.rd, st.rmint, st.rmaxt, false, mint, maxt)) {
            pr = true;
            r0 = make_float4(st.P.its.p.x, st.P.its.p.y, st.P.its.p.z, mint);
            r1 = make_float4(st.rd.x, st.rd.y, st.rd.z, maxt);
        }
    }
    const uint32_t spos = wave_append(cs, ps);
    const uint32_t qpos = wave_append(cq, pr);
    // a live path without a closest-hit ray (none sampled, or outside the scene
    // box): its next shade step is a miss
    const bool pm = st.active && !pr;
    const uint32_t mpos = wave_append(cm, pm);
    if (ps) {
        const size_t k = (size_t)region * W.cap + spos;
        sray[2 * k] = s0; sray[2 * k + 1] = s1; sslot[k] = s;
    }
    if (pr) {
        const size_t k = (size_t)region * W.cap + qpos;
        qray[2 * k] = r0; qray[2 * k + 1] = r1; qslot[k] = s;
    }
    if (pm) missQ[(size_t)region * W.cap_cls + mpos] = s;
    if (valid) wf_store(W, s, st, (done ? WF_DONE : 0u) | (ps ? WF_SQUEUED : 0u));
    uint32_t v[16] = {};
    v[0] = (uint32_t)c.samples; v[1] = (uint32_t)c.rays; v[2] = (uint32_t)c.shadow; v[3] = (uint32_t)c.len;
    v[6] = (uint32_t)c.err;
    v[8] = st.active ? 1u : 0u;   // (slot 8 is otherwise unused) live slots: one atomic per block
    if (INSTR) { v[7] = (uint32_t)c.hits; v[9] = (uint32_t)c.nee; v[10] = (uint32_t)c.sobol; }
    block_counters(part, v, red, 8, W.live + p);
}

// a shade kind's kernel: the grid covers the largest queue possible (all
// slots) and blocks past the queue's end leave at once
template <bool INSTR, int FEAT, int KIND, int HITK, int WAVES>
__global__ __launch_bounds__(BLOCK, WAVES) void wf_shade(MtsgLaunch L, MtsgWave W, unsigned long long *part,
                                                         uint32_t queue) {
    QueueView Q;
    Q.load(wf_cnt(W, W.parity, 2 + queue));
    const uint32_t n = W.seed ? W.slots : Q.total();
    if (blockIdx.x * BLOCK >= n) return;   // block-uniform
    extern __shared__ uint32_t lds[];
    __shared__ uint32_t red[BLOCK / 64 * 16];
    wf_shade_block<INSTR, FEAT, KIND, HITK>(L, W, part, queue, Q, n, blockIdx.x, lds, red);
}

// ---------------------------------------------------------------------------
// the trace kernel: both ray queues of the bounce; closest-hit rays' slots are
// sorted into the next bounce's per-kind queues
// ---------------------------------------------------------------------------
// KD: the reference's kd-tree (kd_traverse); its first KDK stack entries
// (16 B per lane each) and, KDMB, its mailbox (32 B per lane) in LDS.  Up to
// 80 B per lane the kernel keeps MTSG_WF_KD_TRACE_WAVES = 7 waves/SIMD (160 KB
// of LDS over 2048 lanes); above, it is compiled for 4
#ifndef MTSG_WF_KD_LDSK
#define MTSG_WF_KD_LDSK 0
#endif
#ifndef MTSG_WF_KD_MBL
#define MTSG_WF_KD_MBL 1
#endif
constexpr uint32_t wf_kd_lds_lane_bytes(int kdk, bool kdmb) { return (uint32_t)kdk * 16u + (kdmb ? 32u : 0u); }
// the kd trace kernel at 7 waves/SIMD: 70 VGPRs and no spills, against 64 VGPRs
// and 19 spilled at 8: C4 91.3 -> 93.4, C3 451.1 -> 456.0 Msamples/s, bit-identical
// (round 5, profiles/r05_ab_kd_waves.log; 6 waves compiles to the same 70 VGPRs)
#ifndef MTSG_WF_KD_TRACE_WAVES
#define MTSG_WF_KD_TRACE_WAVES 7
#endif
template <bool STATS, bool SCENE_LDS, bool ANA, bool KD, int KDK = 0, bool KDMB = false>
__global__ __launch_bounds__(BLOCK, KD ? (wf_kd_lds_lane_bytes(KDK, KDMB) > 80 ? 4 : MTSG_WF_KD_TRACE_WAVES) : MTSG_WF_TRACE_WAVES) void wf_trace(
    MtsgLaunch L, MtsgWave W, unsigned long long *part) {
    extern __shared__ uint32_t lds[];
    __shared__ uint32_t red[BLOCK / 64 * 16];
    const MtsgDeviceScene &S = L.scene;
    const uint32_t p = W.parity, region = blockIdx.x % WF_R;
    if (blockIdx.x == 0) {
        // queues whose bounce is over: this bounce's kind queues (its shade kernels
        // have run), the other parity's ray queues (traced last bounce), and the
        // next bounce's live count
        if (threadIdx.x < MTSG_WK_KINDS * WF_R) wf_cnt(W, p, 2)[threadIdx.x] = 0;
        else if (threadIdx.x < MTSG_WK_KINDS * WF_R + 2 * WF_R) wf_cnt(W, p ^ 1u, 0)[threadIdx.x - MTSG_WK_KINDS * WF_R] = 0;
        else if (threadIdx.x == MTSG_WK_KINDS * WF_R + 2 * WF_R) W.live[p ^ 1u] = 0;
    }
    QueueView Qc, Qs;
    Qc.load(wf_cnt(W, p, 0));
    Qs.load(wf_cnt(W, p, 1));
    const uint32_t nc = Qc.total(), n = nc + Qs.total();
    // one ray per thread: the grid covers both queues' largest size (2 x slots);
    // blocks past the end leave at once (no persistent loop: DESIGN.md 4)
    if (blockIdx.x * BLOCK >= n) return;   // block-uniform
    uint32_t stackBase = 0;
    if (SCENE_LDS && !L.scan && !KD) {
        const uint32_t nodeWords = L.num_nodes * 16, triWords = S.num_prims * 12;
        const uint32_t *gn = reinterpret_cast<const uint32_t *>(S.nodes);
        const uint32_t *gt = reinterpret_cast<const uint32_t *>(S.tris);
        for (uint32_t i = threadIdx.x; i < nodeWords; i += BLOCK) lds[i] = gn[i];
        for (uint32_t i = threadIdx.x; i < triWords; i += BLOCK) lds[nodeWords + i] = gt[i];
        stackBase = nodeWords + triWords;
        __syncthreads();
    }
    const uint32_t K = L.stack_depth < MTSG_WF_LDS_STACK ? L.stack_depth : MTSG_WF_LDS_STACK;
    lds_node *ldsNodes = (lds_node *)__builtin_assume_aligned((const void *)lds, 16);
    lds_tri *ldsTris = (lds_tri *)__builtin_assume_aligned((const void *)(lds + L.num_nodes * 16), 16);
    lds_stk_n *stkN = (lds_stk_n *)(lds + stackBase) + threadIdx.x;
    lds_stk_d *stkD = (lds_stk_d *)(lds + stackBase + K * BLOCK) + threadIdx.x;
    uint2 *ovf = W.ovf + ((size_t)blockIdx.x * BLOCK + threadIdx.x) * W.ovf_depth;
    const uint2 *kn = (const uint2 *)L.kd_nodes;
    lds_kdent *kstk = (lds_kdent *)lds + threadIdx.x;
    lds_w32 *kmb = (lds_w32 *)(lds + KDK * BLOCK * 4) + threadIdx.x;
    unsigned long long cN = 0, cT = 0;
    const float4 *rays = W.ray[p];
    const uint32_t *rslot = W.rslot[p];
    uint32_t *next = W.cls[p ^ 1u];
    {
        const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
        const bool valid = i < n;
        const bool shadow = i >= nc;
        const size_t k = !valid ? 0 : shadow ? (size_t)WF_R * W.cap + Qs.pos(i - nc, W.cap) : Qc.pos(i, W.cap);
        float4 a = make_float4(0, 0, 0, 1), b = make_float4(0, 0, 1, 0);
        uint32_t s = 0;
        if (valid) { a = rays[2 * k]; b = rays[2 * k + 1]; s = rslot[k]; }
        const f3 o = mk(a.x, a.y, a.z), d = mk(b.x, b.y, b.z);
        const float mint = a.w, maxt = b.w;
        uint32_t slot = 0;
        float hu = 0, hv = 0, ht = 0;
        uint32_t kind = MTSG_WK_KINDS;   // no append
        if (!valid) {
        } else if (shadow) {
            bool occ;
            if constexpr (KD) occ = kd_traverse<true, KDK, KDMB>(kn, L.kd_indices, L.kd_tris, o, d, mint, maxt, ht, hu, hv, slot, kstk, kmb);
            else if (SCENE_LDS && L.scan)
                occ = scan_tris<true, STATS>(L, o, d, mint, maxt, slot, hu, hv, ht, cT);
            else if (SCENE_LDS)
                occ = traverse<true, STATS, ANA, MTSG_WF_LDS_STACK>(ldsNodes, ldsTris, o, d, mint, maxt, stkN, stkD,
                                                                    slot, hu, hv, ht, cN, cT, S.analytic, ovf);
            else
                occ = traverse<true, STATS, ANA, MTSG_WF_LDS_STACK>((glb_node *)S.nodes, (glb_tri *)S.tris, o, d, mint,
                                                                    maxt, stkN, stkD, slot, hu, hv, ht, cN, cT,
                                                                    S.analytic, ovf);
            W.occl[s] = occ ? 1u : 0u;
        } else {
            bool hit;
            uint32_t w = MTSG_WF_NONE, shape = 0, prim = slot;
            if constexpr (KD) {
                hit = kd_traverse<false, KDK, KDMB>(kn, L.kd_indices, L.kd_tris, o, d, mint, maxt, ht, hu, hv, slot, kstk, kmb);
                if (hit) { w = prim = slot; shape = S.prim_vtx[4 * (size_t)slot + 3]; }
            } else if (SCENE_LDS && L.scan) {
                hit = scan_tris<false, STATS>(L, o, d, mint, maxt, slot, hu, hv, ht, cT);
                if (hit) { w = prim = slot; shape = S.prim_vtx[4 * (size_t)slot + 3]; }
            } else {
                if (SCENE_LDS)
                    hit = traverse<false, STATS, ANA, MTSG_WF_LDS_STACK>(ldsNodes, ldsTris, o, d, mint, maxt, stkN,
                                                                         stkD, slot, hu, hv, ht, cN, cT, S.analytic, ovf);
                else
                    hit = traverse<false, STATS, ANA, MTSG_WF_LDS_STACK>((glb_node *)S.nodes, (glb_tri *)S.tris, o, d,
                                                                         mint, maxt, stkN, stkD, slot, hu, hv, ht, cN,
                                                                         cT, S.analytic, ovf);
                if (hit) {
                    const uint2 ps = *reinterpret_cast<const uint2 *>(&S.tris[slot].prim);   // prim, shape
                    w = ANA ? slot : ps.x;
                    prim = ps.x;
                    shape = ps.y;
                }
            }
            if (W.hitrec) {   // the shade kernels read the whole record (hit_store)
                if (hit) {
                    constexpr bool A = ANA && !KD;
                    const HitSrc<false> hs{(glb_u32 *)S.prim_vtx, (glb_f32 *)S.positions, (glb_f32 *)S.normals,
                                           (glb_f32 *)S.dpdu, (glb_shape *)S.shapes};
                    Hit h;
                    if (W.hitrec_uv) fill_hit<true, A>(S, hs, slot, prim, hu, hv, ht, o, d, h);
                    else fill_hit<false, A>(S, hs, slot, prim, hu, hv, ht, o, d, h);
                    hit_store(W.hitrec + (size_t)s * MTSG_WF_HIT_VECS, h, W.hitrec_uv != 0);
                }
            } else {
                W.hit[s] = make_float4(ht, hu, hv, __uint_as_float(w));
            }
            kind = hit ? W.shape_kind[shape] : (uint32_t)MTSG_WK_MISS;
        }
#pragma unroll
        for (uint32_t q = 0; q < MTSG_WK_KINDS; ++q) {
            const uint32_t pos = wave_append(wf_cnt(W, p ^ 1u, 2 + q) + region, kind == q);
            if (kind == q) next[((size_t)q * WF_R + region) * W.cap_cls + pos] = s;
        }
    }
    if (STATS) {
        uint32_t v[16] = {};
        v[4] = (uint32_t)cN;
        v[5] = (uint32_t)cT;
        block_counters(part, v, red);
    }
}


// (Round 4 measured a persistent trace kernel with dynamic ray fetch, Aila & Laine's
// while-while with terminated rays replaced: bit-identical, but C3 604 -> 489,
// C4 172 -> 149, C5 607 -> 497 Msamples/s, profiles/r04_ab_wf_dyn.log; removed.)

// waves per SIMD each shade kind is compiled for
#ifndef MTSG_WF_WAVES_MISS
#define MTSG_WF_WAVES_MISS 4
#endif
#ifndef MTSG_WF_WAVES_DIFF
#define MTSG_WF_WAVES_DIFF 4
#endif
#ifndef MTSG_WF_WAVES_ROUGH
#define MTSG_WF_WAVES_ROUGH 4
#endif
#ifndef MTSG_WF_WAVES_GEN
#define MTSG_WF_WAVES_GEN 3
#endif
template <int KIND, int HITK> struct WfWaves {
    static constexpr int W = HITK == 2 ? MTSG_WF_WAVES_MISS : KIND == BSDF_DIFFUSE ? MTSG_WF_WAVES_DIFF
                           : KIND < 0 ? MTSG_WF_WAVES_GEN : MTSG_WF_WAVES_ROUGH;
};

// shade kernel of (FEAT, kind, GGX): FEAT = the scene's ENV / EXT / ANA bits
template <bool INSTR, int FEAT, int WK, bool GGX>
struct WfShadeK {
    static constexpr int KIND = WK == MTSG_WK_DIFF ? (int)BSDF_DIFFUSE : WK == MTSG_WK_RC ? (int)BSDF_ROUGHCONDUCTOR
                              : WK == MTSG_WK_RD ? (int)BSDF_ROUGHDIELECTRIC : WK == MTSG_WK_RP ? (int)BSDF_ROUGHPLASTIC : -1;
    static constexpr int HITK = WK == MTSG_WK_MISS ? 2 : 1;
    static constexpr int BS = FEAT | (KIND >= 0 ? (int)MTSG_FEAT_INL : 0) | (GGX ? (int)MTSG_FEAT_GGX : 0);
    static constexpr auto fn() { return &wf_shade<INSTR, BS, KIND, HITK, WfWaves<KIND, HITK>::W>; }
};

template <int FEAT, int WK, bool GGX>
__host__ auto wf_shade_fn(bool instr) {
    return instr ? WfShadeK<true, FEAT, WK, GGX>::fn() : WfShadeK<false, FEAT, WK, GGX>::fn();
}
template <int FEAT, int WK>
__host__ auto wf_shade_fn_g(bool instr, bool ggx) {
    if constexpr (WK == MTSG_WK_RC || WK == MTSG_WK_RD || WK == MTSG_WK_RP)
        return ggx ? wf_shade_fn<FEAT, WK, true>(instr) : wf_shade_fn<FEAT, WK, false>(instr);
    else
        return wf_shade_fn<FEAT, WK, false>(instr);
}
typedef void (*WfShadeFn)(MtsgLaunch, MtsgWave, unsigned long long *, uint32_t);
template <int FEAT>
__host__ WfShadeFn wf_shade_pick_f(int wk, bool instr, bool ggx) {

    switch (wk) {
        case MTSG_WK_MISS: return wf_shade_fn_g<FEAT, MTSG_WK_MISS>(instr, ggx);
        case MTSG_WK_DIFF: return wf_shade_fn_g<FEAT, MTSG_WK_DIFF>(instr, ggx);
        case MTSG_WK_RC: return wf_shade_fn_g<FEAT, MTSG_WK_RC>(instr, ggx);
        case MTSG_WK_RD: return wf_shade_fn_g<FEAT, MTSG_WK_RD>(instr, ggx);
        case MTSG_WK_RP:
            if constexpr ((FEAT & MTSG_FEAT_EXT) != 0) return wf_shade_fn_g<FEAT, MTSG_WK_RP>(instr, ggx);
            else return nullptr;   // roughplastic implies EXT
        default: return wf_shade_fn_g<FEAT, MTSG_WK_GEN>(instr, ggx);
    }
}
