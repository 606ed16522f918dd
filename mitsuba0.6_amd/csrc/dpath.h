// dpath.h -- the device side of Mitsuba 0.6's `path` integrator shared by both
// execution engines (path_kernel.hip: the persistent megakernel, the `direct`
// integrator and batch ray queries; wf_kernel.hip: the wavefront engine):
// SamplingIntegrator::renderBlock's per-sample loop body
// (src/librender/integrator.cpp:140-188) around MIPathTracer::Li
// (src/integrators/path/path.cpp:119-294) as a per-path state machine
// (PathShader), the Sobol / independent samplers, the BVH2 and kd-tree
// traversals, the hit record and the film splat.
//
// Work items are (sample j, pixel p) pairs, pixels in 8x8 tiles; the megakernel
// hands them out as runs of consecutive samples of one pixel (dmega.h).
// The own-pixel splat of every sample is stored to HBM ([spp][pixels], film_slot)
// and a second kernel sums each pixel in sample order -- the reference's
// ImageBlock accumulation order, bit for bit; splats into other pixels (box
// filter edges) go to a spill film with double atomics, gaussian footprints are
// gathered per pixel in a fixed order (film_gather).  LDS holds the Sobol
// direction numbers of the first dimensions as 4-bit lookup tables (8
// independent reads per 32-bit sample instead of up to 32 dependent ones).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "danalytic.h"
#include "dbsdf.h"
#include "denv.h"
#include "layout.h"
#include "sfmt.h"

#define BLOCK 256

// ---------------------------------------------------------------------------
// Sobol sampler (samplers/sobol.cpp:147-258, sobolseq.h:43-130)
// ---------------------------------------------------------------------------
// sobol::sampleSingle (sobolseq.h:43-57): XOR of the direction-number columns
// selected by the bits of `index`, evaluated 4 bits at a time through
// precomputed XOR tables (exactly the same XOR, so the same result)
typedef __attribute__((address_space(3))) const uint32_t lds_u32;     // LDS
typedef __attribute__((address_space(1))) const uint32_t glb_u32;     // global
typedef __attribute__((address_space(3))) const MtsgNode lds_node;
typedef __attribute__((address_space(1))) const MtsgNode glb_node;
typedef __attribute__((address_space(3))) const MtsgTri lds_tri;
typedef __attribute__((address_space(1))) const MtsgTri glb_tri;
typedef float vf4 __attribute__((ext_vector_type(4)));
typedef int vi4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const vf4 lds_f4;
typedef __attribute__((address_space(1))) const vf4 glb_f4;
typedef __attribute__((address_space(3))) const vi4 lds_i4;
typedef __attribute__((address_space(1))) const vi4 glb_i4;
typedef unsigned int vu4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const vu4 glb_u4;
typedef __attribute__((address_space(1))) const MtsgHNode glb_hnode;

// one BVH2 node's two child boxes and child references: the 64 B MtsgNode
// (LDS or HBM) in four 16 B loads, or the 32 B MtsgHNode in two, its half
// bounds widened exactly to float (the conversions fold into the slab FMAs)
__device__ __forceinline__ float half_lo(uint32_t w) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu)); }
__device__ __forceinline__ float half_hi(uint32_t w) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16)); }
template <typename NodeT>
__device__ __forceinline__ void load_node(NodeT *n, vf4 &a, vf4 &b, vf4 &c, int &c0, int &c1) {
    if constexpr (std::is_same<NodeT, glb_hnode>::value) {
        const vu4 p = *reinterpret_cast<glb_u4 *>(&n->box[0]);
        const vu4 q = *reinterpret_cast<glb_u4 *>(&n->box[4]);
        a = vf4{half_lo(p.x), half_hi(p.x), half_lo(p.y), half_hi(p.y)};
        b = vf4{half_lo(p.z), half_hi(p.z), half_lo(p.w), half_hi(p.w)};
        c = vf4{half_lo(q.x), half_hi(q.x), half_lo(q.y), half_hi(q.y)};
        c0 = (int)q.z;
        c1 = (int)q.w;
    } else {
        typedef typename std::conditional<std::is_same<NodeT, lds_node>::value, lds_f4, glb_f4>::type F4;
        typedef typename std::conditional<std::is_same<NodeT, lds_node>::value, lds_i4, glb_i4>::type I4;
        a = *reinterpret_cast<F4 *>(&n->c0lox);
        b = *reinterpret_cast<F4 *>(&n->c1lox);
        c = *reinterpret_cast<F4 *>(&n->c0loz);
        const vi4 e = *reinterpret_cast<I4 *>(&n->c0);
        c0 = e.x;
        c1 = e.y;
    }
}

template <int NIB, typename T>
__device__ __forceinline__ uint32_t sobol_bits(T *tab, uint64_t index) {
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < NIB; ++c) r ^= tab[c * 16 + (uint32_t)((index >> (4 * c)) & 15u)];
    return r;
}

struct SobolCtx {
    lds_u32 *lds;             // [lds_dims][nibbles][16]
    glb_u32 *glob;            // [1024][MTSG_NIBBLES][16]
    uint32_t lds_dims, nibbles, scramble;
    bool indep;               // the `independent` sampler: `index` is a stream key
    bool replay;              // SFMT replay: draws come from the lane's SFMT stream
    uint32_t *sfmt;           // the streams (lane u: sfmt + u * MTSG_SFMT_WORDS)
};

// the SFMT replay stream of this lane (MtsgLaunch::sfmt; unit = global lane index)
typedef __attribute__((address_space(1))) uint32_t glb_w32;
__device__ __forceinline__ glb_w32 *lane_sfmt(const SobolCtx &C) {
    return (glb_w32 *)C.sfmt + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * MTSG_SFMT_WORDS;
}

// The independent sampler (independent.cpp:82-104): a counter-based stream per
// (pixel, sample) -- splitmix64-finalised key, one finalised draw per dimension
// -- in place of the reference's per-thread SFMT19937, whose values depend on
// the thread schedule; Random::nextFloat's [1,2) - 1 conversion
// (random.cpp:630-639).  The oracle's indep_* functions are the same.
__device__ __forceinline__ uint64_t indep_mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t indep_key(uint32_t px, uint32_t py, uint32_t frame) {
    return indep_mix64((((uint64_t)px << 48) | ((uint64_t)py << 32) | frame) ^ 0x6A09E667F3BCC909ull);
}
__device__ __forceinline__ float indep_float(uint64_t key, uint32_t dim) {
    const uint32_t u = (uint32_t)indep_mix64(key + (uint64_t)(dim + 1) * 0x9E3779B97F4A7C15ull);
    return __uint_as_float((u >> 9) | 0x3f800000u) - 1.0f;
}

__device__ __forceinline__ float sobol_sample(const SobolCtx &C, uint64_t index, uint32_t dim) {
    if (C.indep) return indep_float(index, dim);
    uint32_t bits;
    if (dim < C.lds_dims) {
        lds_u32 *t = C.lds + dim * C.nibbles * 16;
        bits = (C.nibbles == 8) ? sobol_bits<8>(t, index) : sobol_bits<MTSG_NIBBLES>(t, index);
    } else {
        glb_u32 *t = C.glob + (size_t)dim * MTSG_NIBBLES * 16;
        bits = (C.nibbles == 8) ? sobol_bits<8>(t, index) : sobol_bits<MTSG_NIBBLES>(t, index);
    }
    const uint32_t result = C.scramble ^ bits;
    float v = (float)result * (1.0f / 4294967296.0f);
    return smin(v, D_ONE_MINUS_EPS);
}

// sobol::look_up restated as the GF(2) solve it encodes (host precomputes inv/ycol)
__device__ __forceinline__ uint64_t sobol_lookup(const MtsgLookup &L, uint32_t frame, uint32_t px, uint32_t py,
                                                 uint64_t scramble) {
    const uint32_t m = L.m;
    uint32_t s = (uint32_t)((scramble & 0xFFFFFFFFull) >> (32 - m));
    uint32_t mask = (1u << m) - 1u;
    uint32_t sx = (px ^ s) & mask, sy = (py ^ s) & mask;
    uint32_t jlo = __builtin_bitreverse32(sx) >> (32 - m);
    uint64_t index = ((uint64_t)frame << (2 * m)) | jlo;
    uint32_t K = 0;
    uint64_t bits = index;
    while (bits) {
        uint32_t b = (uint32_t)__builtin_ctzll(bits);
        K ^= L.ycol[b];
        bits &= bits - 1;
    }
    uint32_t rhs = (sy ^ K) & mask, jhi = 0;
    for (uint32_t t = 0; t < m; ++t) jhi |= (uint32_t)(__builtin_popcount(L.inv[t] & rhs) & 1) << t;
    return index | ((uint64_t)jhi << m);
}

// Workgroups are dispatched round-robin over the 8 XCDs, each with its own L2.
// Renumber them so that XCD x runs the x-th contiguous eighth of the grid: the
// items (pixels in 8x8 tiles) the lanes of one XCD hold at a time are then
// neighbours, and their rays share BVH nodes and triangles in that XCD's L2.
// `xcds` comes from the host (MtsgLaunch::xcds: CUs / 32 on gfx950, 1 on a
// CPX partition); no remap when it is 1 or does not divide the grid.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb, uint32_t xcds) {
    return (xcds > 1u && nb % xcds == 0) ? (b % xcds) * (nb / xcds) + b / xcds : b;
}
__device__ __forceinline__ uint32_t xcd_block(uint32_t xcds) { return xcd_remap(blockIdx.x, gridDim.x, xcds); }

// The kernel's launch record (its first argument), re-read through a pointer
// the compiler cannot follow.  A persistent loop otherwise has LICM hoist every
// launch field and every product of them it finds invariant (camera rows,
// scene pointers, sampler constants) out of the loop; they then stay live
// across the whole bounce, as SGPRs spilled into VGPR lanes or as VGPR copies,
// and push the shading state into scratch.  Re-read per iteration they are
// s_loads from the kernarg segment (scalar cache) at their point of use.
// Requires MtsgLaunch to be the kernel's first argument (kernarg offset 0).
__device__ __forceinline__ const MtsgLaunch &launch_fresh() {
    typedef __attribute__((address_space(4))) const MtsgLaunch KernargLaunch;
    KernargLaunch *kp = (KernargLaunch *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *(const MtsgLaunch *)kp;
}

struct SamplerState {
    uint64_t sobolIndex;
    uint32_t sampleIndex;
    uint32_t dim;
    bool err;
};

// ---------------------------------------------------------------------------
// per-lane path state
// ---------------------------------------------------------------------------
enum { ST_NEWSAMPLE = 0, ST_PRIMARY = 1, ST_SHADOW = 2, ST_EXT = 3, ST_DONE = 4 };

struct Hit {
    int valid;
    float t;
    f3 p, geoN, wi;
    ShFrame sh;
    int shape;
    float u, v;       // its.uv (textured scenes only; dead otherwise)
};

// ---------------------------------------------------------------------------
// BVH2 traversal
// ---------------------------------------------------------------------------
// LDS traversal stack, lane-strided: node index (4 B) + entry distance as the
// top 16 bits of the (non-negative) float, i.e. bfloat16 rounded toward zero:
// a lower bound of the true entry distance, so culling on pop stays
// conservative (6 B/entry keeps 3 blocks per CU on large scenes)
typedef __attribute__((address_space(3))) int lds_stk_n;
typedef __attribute__((address_space(3))) uint16_t lds_stk_d;
__device__ __forceinline__ uint16_t dist_down16(float t) { return (uint16_t)(__float_as_uint(fmaxf(t, 0.0f)) >> 16); }
__device__ __forceinline__ float dist_up16(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
// Speculative while-while traversal (Aila & Laine 2009): a lane that reaches a
// leaf parks it and keeps descending until every lane of the wave holds a
// leaf; then all lanes test their parked leaves together.  Same closest hit
// (tie rule included) as a plain depth-first traversal.
// LDSK > 0: the first LDSK stack entries live in LDS, deeper ones in a per-lane
// global array `ovf` ({node, distance} pairs): a short LDS stack keeps the
// traversal kernel's LDS per lane small (wf_trace occupancy); 0: all in LDS
// (Round 4 measured the stack's top entry cached in two registers: bit-identical,
// but C2 -0.9%, C3 -4.2%, C4 -5.2%, C5 -3.9%, profiles/r04_ab_reg_top.log; removed.)
template <bool ANY, bool STATS, bool ANA = false, int LDSK = 0, typename NodeT, typename TriT>
__device__ __forceinline__ bool traverse(NodeT *nodesArr, TriT *trisArr, f3 o, f3 d, float mint, float maxt,
                                         lds_stk_n *stkN, lds_stk_d *stkD, uint32_t &bestSlot, float &bu, float &bv,
                                         float &bt, unsigned long long &nodes, unsigned long long &tests,
                                         const MtsgAnalytic *anaArr = nullptr, uint2 *ovf = nullptr) {
    typedef typename std::conditional<std::is_same<NodeT, lds_node>::value, lds_f4, glb_f4>::type F4;
    const float ix = (d.x == 0.0f) ? copysignf(1e30f, d.x) : 1.0f / d.x;
    const float iy = (d.y == 0.0f) ? copysignf(1e30f, d.y) : 1.0f / d.y;
    const float iz = (d.z == 0.0f) ? copysignf(1e30f, d.z) : 1.0f / d.z;
    const float ox = o.x * ix, oy = o.y * iy, oz = o.z * iz;
    constexpr int DONE = 0x7fffffff;
    bool found = false;
    uint32_t bestPrim = 0;
    bt = maxt;
    int sp = 0;
    int node = 0, leaf = 0;
    auto pop = [&]() -> int {
        while (sp > 0) {
            --sp;
            if (LDSK == 0 || sp < LDSK) {
                // the entry's node read ahead of the cull test (the empty asm pins it
                // there) instead of inside the taken branch: C3 +2.0%, C4 +1.6%, C5
                // +1.2% (round 5, profiles/r05_ab_pop_both.log).  Both reads issued
                // before one wait lost 1.1-1.6% against this (r05_ab_pop_onewait.log),
                // so the gain is in the shape of the compiled pop loop, not in LDS
                // round trips
                int n = stkN[sp * BLOCK];
                asm volatile("" : "+v"(n));
                if (ANY || dist_up16(stkD[sp * BLOCK]) <= bt) return n;
            } else {
                const uint2 e = ovf[sp - LDSK];
                if (ANY || dist_up16((uint16_t)e.y) <= bt) return (int)e.x;
            }
        }
        return DONE;
    };
    while (node != DONE) {
        // inner nodes
        while ((uint32_t)node < (uint32_t)DONE) {
            if (STATS) nodes++;
            vf4 a, b, c;
            int ec0, ec1;
            load_node(nodesArr + node, a, b, c, ec0, ec1);
            // slab tests; node boxes are conservatively inflated on the host
            const float t0x = __builtin_fmaf(a.x, ix, -ox), t1x = __builtin_fmaf(a.y, ix, -ox);
            const float t0y = __builtin_fmaf(a.z, iy, -oy), t1y = __builtin_fmaf(a.w, iy, -oy);
            const float t0z = __builtin_fmaf(c.x, iz, -oz), t1z = __builtin_fmaf(c.y, iz, -oz);
            const float n0 = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), mint));
            const float f0 = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), bt));
            const float u0x = __builtin_fmaf(b.x, ix, -ox), u1x = __builtin_fmaf(b.y, ix, -ox);
            const float u0y = __builtin_fmaf(b.z, iy, -oy), u1y = __builtin_fmaf(b.w, iy, -oy);
            const float u0z = __builtin_fmaf(c.z, iz, -oz), u1z = __builtin_fmaf(c.w, iz, -oz);
            const float n1 = fmaxf(fmaxf(fminf(u0x, u1x), fminf(u0y, u1y)), fmaxf(fminf(u0z, u1z), mint));
            const float f1 = fminf(fminf(fmaxf(u0x, u1x), fmaxf(u0y, u1y)), fminf(fmaxf(u0z, u1z), bt));
            const bool h0 = n0 <= f0, h1 = n1 <= f1;
            if (h0 && h1) {
                int nearC = ec0, farC = ec1;
                float farT = n1;
                if (n1 < n0) { nearC = ec1; farC = ec0; farT = n0; }
                if (LDSK == 0 || sp < LDSK) {
                    stkN[sp * BLOCK] = farC;
                    stkD[sp * BLOCK] = dist_down16(farT);
                } else {
                    ovf[sp - LDSK] = make_uint2((uint32_t)farC, dist_down16(farT));
                }
                ++sp;
                node = nearC;
            } else if (h0) {
                node = ec0;
            } else if (h1) {
                node = ec1;
            } else {
                node = pop();
            }
            // park the first leaf reached and keep descending
            if (node < 0 && leaf == 0) {
                leaf = node;
                node = pop();
            }
            if (!__any(leaf == 0)) break;
        }
        // leaves
        while (leaf < 0) {
            const uint32_t ref = (uint32_t)(~leaf);
            const uint32_t first = ref >> 4, count = ref & 15u, end = first + count;
            // the next record's loads are in flight during a record's test (round 5:
            // C4 +1.7%, C3 +1.3%, C5 +0.4%, profiles/r05_ab_leaf_prefetch.log)
            vf4 p0 = *reinterpret_cast<F4 *>(&trisArr[first].k);
            vf4 p1 = *reinterpret_cast<F4 *>(&trisArr[first].a_u);
            vf4 p2 = *reinterpret_cast<F4 *>(&trisArr[first].c_nu);
            for (uint32_t i = first; i < end; ++i) {
                if (STATS) tests++;
                const vf4 q0 = p0, q1 = p1, q2 = p2;
                if (i + 1 < end) {
                    TriT *tn = trisArr + i + 1;
                    p0 = *reinterpret_cast<F4 *>(&tn->k);
                    p1 = *reinterpret_cast<F4 *>(&tn->a_u);
                    p2 = *reinterpret_cast<F4 *>(&tn->c_nu);
                }
                const uint32_t k = __float_as_uint(q0.x);
                // TriAccel::rayIntersect (triaccel.h:92-160)
                float o_u, o_v, o_k, d_u, d_v, d_k;
                if (k == 0) { o_u = o.y; o_v = o.z; o_k = o.x; d_u = d.y; d_v = d.z; d_k = d.x; }
                else if (k == 1) { o_u = o.z; o_v = o.x; o_k = o.y; d_u = d.z; d_v = d.x; d_k = d.y; }
                else if (k == 2) { o_u = o.x; o_v = o.y; o_k = o.z; d_u = d.x; d_v = d.y; d_k = d.z; }
                else {
                    if constexpr (ANA) {
                        // analytic primitive (skdtree.h:280-290: Shape::rayIntersect on [mint, maxt])
                        float at, alx, aly;
                        if (k == MTSG_K_ANALYTIC &&
                            ana_intersect<ANY>(((GAna *)anaArr)[__float_as_uint(q0.y)], o, d, mint, bt, at, alx, aly)) {
                            if (ANY) return true;
                            const uint32_t prim = __float_as_uint(q2.z);
                            if (!found || at < bt || prim > bestPrim) {
                                found = true; bestPrim = prim; bestSlot = i; bt = at; bu = alx; bv = aly;
                            }
                        }
                    }
                    continue;
                }
                const float n_u = q0.y, n_v = q0.z, n_d = q0.w;
                const float a_u = q1.x, a_v = q1.y, b_nu = q1.z, b_nv = q1.w;
                const float c_nu = q2.x, c_nv = q2.y;
                const float t = (n_d - o_u * n_u - o_v * n_v - o_k) / (d_u * n_u + d_v * n_v + d_k);
                if (t < mint || t > bt) continue;
                const float hu = o_u + t * d_u - a_u;
                const float hv = o_v + t * d_v - a_v;
                const float u = hv * b_nu + hu * b_nv;
                const float v = hu * c_nu + hv * c_nv;
                if (u >= 0 && v >= 0 && u + v <= 1.0f) {
                    if (ANY) return true;
                    const uint32_t prim = __float_as_uint(q2.z);
                    // ties (t == bt): the larger primitive index wins
                    if (!found || t < bt || prim > bestPrim) {
                        found = true; bestPrim = prim; bestSlot = i; bt = t; bu = u; bv = v;
                    }
                }
            }
            leaf = 0;
            if (node < 0) {   // the next stack entry is a leaf too: take it now
                leaf = node;
                node = pop();
            }
        }
    }
    return found;
}

typedef __attribute__((address_space(4))) const MtsgTri cst_tri;
// one projection axis' records: the coordinate permutation is a compile-time
// constant, so the loop is straight-line code around the correctly rounded
// division; each record is read whole (two scalar loads) at the loop head
// AL: the group whose plane normal lies along axis K (n_u and n_v both +-0,
// L.scan_n): then the numerator is n_d - o_k and the denominator d_k,
// exactly (a +-0 product added to a nonzero value leaves it unchanged).  Where
// the sum is zero the two forms may differ in the sign of that zero only: a
// zero numerator gives t = +-0 either way, and +0 and -0 pass every comparison
// alike; a zero d_k gives +-inf (rejected by the finite clipped [mint, maxt])
// or NaN (rejected by the barycentric test).  C2 +1.75%
// (profiles/r05_ab_aligned_scan.log)
template <int K, bool AL, bool ANY, bool STATS>
__device__ __forceinline__ bool scan_k(cst_tri *tris, uint32_t n, f3 o, f3 d, float mint, bool &found,
                                       uint32_t &bestPrim, float &bu, float &bv, float &bt,
                                       unsigned long long &tests) {
    const float o_u = K == 0 ? o.y : K == 1 ? o.z : o.x, o_v = K == 0 ? o.z : K == 1 ? o.x : o.y,
                o_k = K == 0 ? o.x : K == 1 ? o.y : o.z;
    const float d_u = K == 0 ? d.y : K == 1 ? d.z : d.x, d_v = K == 0 ? d.z : K == 1 ? d.x : d.y,
                d_k = K == 0 ? d.x : K == 1 ? d.y : d.z;
    for (uint32_t i = 0; i < n; ++i) {
        if (STATS) tests++;
        cst_tri &tr = tris[i];
        const float n_u = tr.n_u, n_v = tr.n_v, n_d = tr.n_d, a_u = tr.a_u, a_v = tr.a_v, b_nu = tr.b_nu,
                    b_nv = tr.b_nv, c_nu = tr.c_nu, c_nv = tr.c_nv;
        const uint32_t prim = tr.prim;
        // TriAccel::rayIntersect (triaccel.h:92-160)
        const float t = AL ? (n_d - o_k) / d_k : (n_d - o_u * n_u - o_v * n_v - o_k) / (d_u * n_u + d_v * n_v + d_k);
        if (t < mint || t > bt) continue;
        const float hu = o_u + t * d_u - a_u;
        const float hv = o_v + t * d_v - a_v;
        const float u = hv * b_nu + hu * b_nv;
        const float v = hu * c_nu + hv * c_nv;
        if (u >= 0 && v >= 0 && u + v <= 1.0f) {
            if (ANY) return true;
            if (!found || t < bt || prim > bestPrim) {
                found = true; bestPrim = prim; bt = t; bu = u; bv = v;
            }
        }
    }
    return false;
}

// Tiny scenes (<= MTSG_SCAN_MAX triangles, no analytic shapes): every lane
// tests every TriAccel record, read from the constant address space with a
// uniform index (scalar loads into SGPRs): no traversal stack, no divergent
// node loop.  The records come grouped by projection axis (L.scan_tris, each
// axis' records with an axis-aligned plane last); the
// result -- the closest t, ties to the larger primitive index as in
// traverse() -- does not depend on the test order.  Returns the
// primitive index (not a slot) in bestPrim.
template <bool ANY, bool STATS>
__device__ __forceinline__ bool scan_tris(const MtsgLaunch &L, f3 o, f3 d, float mint, float maxt,
                                          uint32_t &bestPrim, float &bu, float &bv, float &bt,
                                          unsigned long long &tests) {
    cst_tri *tris = (cst_tri *)L.scan_tris;
    bool found = false;
    bestPrim = 0;
    bt = maxt;
#define MTSG_SCAN_GROUP(K, AL)                                                                                   \
    if (scan_k<K, AL, ANY, STATS>(tris, L.scan_n[2 * K + AL], o, d, mint, found, bestPrim, bu, bv, bt, tests)) \
        return true;                                                                                             \
    tris += L.scan_n[2 * K + AL];
    MTSG_SCAN_GROUP(0, false) MTSG_SCAN_GROUP(0, true) MTSG_SCAN_GROUP(1, false) MTSG_SCAN_GROUP(1, true)
    MTSG_SCAN_GROUP(2, false) MTSG_SCAN_GROUP(2, true)
#undef MTSG_SCAN_GROUP
    return found;
}

// The megakernel's two rays of one bounce leave the same vertex (the NEE
// shadow ray and the next closest-hit ray, both from its.p), so a tiny scene
// tests them in one pass over the records: the TriAccel numerator is shared,
// the records are loaded once, and the pairs of products pack into
// v_pk_mul/v_pk_add.  Each ray's result is exactly that of its own scan_tris
// (an empty interval, mint = +inf and maxt = -inf, disables a ray).
// a / b from y = RN(1/b) (correctly rounded, computed once per ray): the
// quotient a * y with two residual corrections, r = a - b q exact by FMA and
// q' = RN(q + r y) (Markstein's theorem: with y = RN(1/b) and q within an ulp
// of a/b, q' = RN(a/b)).  It equals IEEE a / b wherever nothing underflows;
// scan_pair takes it only for rays with |b| >= 2^-60 and mint >= 2^-30, where
// a quotient small enough to underflow is rejected by mint either way.  Host
// check: 1.6e9 random and edge-mantissa pairs over that range, bit-equal to
// IEEE division (tools/gpu_runs/r05/fast_div_check.c).
__device__ __forceinline__ float div_by_rcp(float a, float b, float y) {
    float q = a * y;
    float r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}

// FAST (axis-aligned groups only): the two quotients through div_by_rcp with
// the rays' reciprocals yS = RN(1/s_k), yC = RN(1/c_k)
template <int K, bool AL, bool FAST, bool STATS>
__device__ __forceinline__ void scan_pair_k(cst_tri *tris, uint32_t n, f3 o, f3 ds, f3 dc, float minS, float maxS,
                                            float minC, bool &occ, bool &found, uint32_t &bestPrim, float &bu,
                                            float &bv, float &bt, unsigned long long &tests, float yS = 0,
                                            float yC = 0) {
    const float o_u = K == 0 ? o.y : K == 1 ? o.z : o.x, o_v = K == 0 ? o.z : K == 1 ? o.x : o.y,
                o_k = K == 0 ? o.x : K == 1 ? o.y : o.z;
    const float s_u = K == 0 ? ds.y : K == 1 ? ds.z : ds.x, s_v = K == 0 ? ds.z : K == 1 ? ds.x : ds.y,
                s_k = K == 0 ? ds.x : K == 1 ? ds.y : ds.z;
    const float c_u = K == 0 ? dc.y : K == 1 ? dc.z : dc.x, c_v = K == 0 ? dc.z : K == 1 ? dc.x : dc.y,
                c_k = K == 0 ? dc.x : K == 1 ? dc.y : dc.z;
    for (uint32_t i = 0; i < n; ++i) {
        if (STATS) tests += 2;
        cst_tri &tr = tris[i];
        const float n_u = tr.n_u, n_v = tr.n_v, n_d = tr.n_d, a_u = tr.a_u, a_v = tr.a_v, b_nu = tr.b_nu,
                    b_nv = tr.b_nv, c_nu = tr.c_nu, c_nv = tr.c_nv;
        const uint32_t prim = tr.prim;
        // TriAccel::rayIntersect (triaccel.h:92-160) for both rays
        // (AL: as in scan_k)
        const float num = AL ? n_d - o_k : n_d - o_u * n_u - o_v * n_v - o_k;
        const float tS = (AL && FAST) ? div_by_rcp(num, s_k, yS) : num / (AL ? s_k : s_u * n_u + s_v * n_v + s_k);
        const float tC = (AL && FAST) ? div_by_rcp(num, c_k, yC) : num / (AL ? c_k : c_u * n_u + c_v * n_v + c_k);
        if (!(tS < minS || tS > maxS)) {
            const float hu = o_u + tS * s_u - a_u;
            const float hv = o_v + tS * s_v - a_v;
            const float u = hv * b_nu + hu * b_nv;
            const float v = hu * c_nu + hv * c_nv;
            if (u >= 0 && v >= 0 && u + v <= 1.0f) occ = true;
        }
        if (!(tC < minC || tC > bt)) {
            const float hu = o_u + tC * c_u - a_u;
            const float hv = o_v + tC * c_v - a_v;
            const float u = hv * b_nu + hu * b_nv;
            const float v = hu * c_nu + hv * c_nv;
            if (u >= 0 && v >= 0 && u + v <= 1.0f) {
                if (!found || tC < bt || prim > bestPrim) {
                    found = true; bestPrim = prim; bt = tC; bu = u; bv = v;
                }
            }
        }
    }
}

template <bool STATS>
__device__ __forceinline__ void scan_pair(const MtsgLaunch &L, f3 o, f3 ds, f3 dc, float minS, float maxS, float minC,
                                          float maxC, bool &occ, bool &found, uint32_t &bestPrim, float &bu,
                                          float &bv, float &bt, unsigned long long &tests) {
    cst_tri *tris = (cst_tri *)L.scan_tris;
    occ = false;
    found = false;
    bestPrim = 0;
    bt = maxC;
    // a disabled ray (empty interval) may take the fast quotient whatever its direction
    const bool offS = !(minS <= maxS), offC = !(minC <= maxC);
#define MTSG_SCAN_GROUP(K)                                                                                         \
    scan_pair_k<K, false, false, STATS>(tris, L.scan_n[2 * K], o, ds, dc, minS, maxS, minC, occ, found, bestPrim,   \
                                        bu, bv, bt, tests);                                                        \
    tris += L.scan_n[2 * K];                                                                                       \
    if (L.scan_n[2 * K + 1]) {                                                                                     \
        const float s_k = K == 0 ? ds.x : K == 1 ? ds.y : ds.z, c_k = K == 0 ? dc.x : K == 1 ? dc.y : dc.z;        \
        const bool fast = (offS || (minS >= 0x1p-30f && fabsf(s_k) >= 0x1p-60f)) &&                                \
                          (offC || (minC >= 0x1p-30f && fabsf(c_k) >= 0x1p-60f));                                  \
        if (__all(fast))                                                                                           \
            scan_pair_k<K, true, true, STATS>(tris, L.scan_n[2 * K + 1], o, ds, dc, minS, maxS, minC, occ, found,  \
                                              bestPrim, bu, bv, bt, tests, 1.0f / s_k, 1.0f / c_k);                \
        else                                                                                                       \
            scan_pair_k<K, true, false, STATS>(tris, L.scan_n[2 * K + 1], o, ds, dc, minS, maxS, minC, occ, found, \
                                               bestPrim, bu, bv, bt, tests);                                       \
        tris += L.scan_n[2 * K + 1];                                                                               \
    }
    MTSG_SCAN_GROUP(0) MTSG_SCAN_GROUP(1) MTSG_SCAN_GROUP(2)
#undef MTSG_SCAN_GROUP
}

// AABB::rayIntersect (core/aabb.h:308-338) against the scene bounds
__device__ __forceinline__ bool aabb_clip(const MtsgDeviceScene &S, f3 o, f3 d, float &nearT, float &farT) {
    nearT = -INFINITY; farT = INFINITY;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float origin = comp(o, i), di = comp(d, i);
        const float minVal = S.aabb_min[i], maxVal = S.aabb_max[i];
        if (di == 0) {
            if (origin < minVal || origin > maxVal) return false;
        } else {
            const float rcp = (float)1 / di;                 // ray.dRcp (ray.h:86-93)
            float t1 = (minVal - origin) * rcp;
            float t2 = (maxVal - origin) * rcp;
            if (t1 > t2) { float t = t1; t1 = t2; t2 = t; }
            nearT = smax(t1, nearT);
            farT = smin(t2, farT);
            if (!(nearT <= farT)) return false;
        }
    }
    return true;
}

// The reference's own kd-tree (kdtree_build.cpp) traversed as
// SAHKDTree3D::rayIntersectHavran (sahkdtree3.h:178-308): entry/exit points on
// a stack of MTS_KD_MAXDEPTH entries, leaves tested over the global [mint,
// maxt] with the 8-entry hashed mailbox (:138-152, MTS_KD_MAILBOX_ENABLED),
// and ShapeKDTree::intersect's TriAccel test (skdtree.h:248-338), which keeps
// a hit at t == maxt: among exactly tied triangles the last one tested wins,
// as in the reference.  TriAccel records are in leaf-list order (tris[e] is
// the record of primitive indices[e], duplicated where leaves share one).
// The reference's stack (entries indexed by enPt / exPt, each with a prev
// link to the exit point below it) holds the pending far children in push
// order: every pop takes the most recent live push, and a push never
// overwrites a live entry (it lands above exPt, skipping enPt).  So here it is
// a plain LIFO whose entry keeps the far child and, by value, the exit point
// that was current when it was pushed -- what the reference reaches through
// prev -- and a pop is one stack read instead of three dependent ones.  A
// point (t, split, axis) is p = ray(t) with p[axis] = split; p[a] is re-formed
// as split (a == axis) or o[a] + d[a] * t, the same rounded product and sum
// the reference stores, so every comparison sees the same floats.  The entry
// and exit points the descent compares against are held in registers (only a
// push or a pop changes them), so a descent step reads no stack memory.  The
// reference's bottom entries, ray(mint) and ray(maxt) with node NONE, become
// the initial registers and the empty stack.  LDSK = 0: the stack lives in
// scratch; LDSK > 0: its first LDSK entries live in LDS, lane-strided
// (lstk[entry * BLOCK]), deeper entries in scratch; MBL: the mailbox in LDS
// (lmbox[slot * BLOCK]), else in scratch.
struct KdEnt { uint32_t node; float t; float split; uint32_t axis; };
typedef __attribute__((address_space(3))) vu4 lds_kdent;
typedef __attribute__((address_space(3))) uint32_t lds_w32;
template <bool ANY, int LDSK = 0, bool MBL = (LDSK > 0)>
__device__ bool kd_traverse(const uint2 *__restrict__ nodes, const uint32_t *__restrict__ indices,
                            const MtsgTri *__restrict__ tris, f3 o, f3 d, float mint, float maxt, float &bt,
                            float &bu, float &bv, uint32_t &bprim, lds_kdent *lstk = nullptr,
                            lds_w32 *lmbox = nullptr) {
    typedef KdEnt Ent;
    constexpr uint32_t NOAXIS = 3u, DEPTH = 46;   // MTS_KD_MAXDEPTH = 48 entries, two of them the bottom
    Ent stackS[DEPTH - LDSK];
    uint32_t mboxS[MBL ? 1 : 8];
    // entry i: LDS below LDSK, scratch above
    auto ld = [&](uint32_t i) -> Ent {
        if (LDSK && i < (uint32_t)LDSK) {
            const vu4 v = lstk[i * BLOCK];
            return Ent{v.x, __uint_as_float(v.y), __uint_as_float(v.z), v.w};
        }
        return stackS[i - LDSK];
    };
    auto st = [&](uint32_t i, const Ent &e) {
        if (LDSK && i < (uint32_t)LDSK) lstk[i * BLOCK] = vu4{e.node, __float_as_uint(e.t), __float_as_uint(e.split), e.axis};
        else stackS[i - LDSK] = e;
    };
    auto mb = [&](uint32_t k) -> uint32_t { if constexpr (MBL) return lmbox[k * BLOCK]; else return mboxS[k]; };
    auto mbset = [&](uint32_t k, uint32_t v) { if constexpr (MBL) lmbox[k * BLOCK] = v; else mboxS[k] = v; };
#pragma unroll
    for (int i = 0; i < 8; ++i) mbset(i, 0xffffffffu);
    const float rcp[3] = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};   // Ray::setDirection (ray.h:86-93)
    // p[a] of a point (t, split, eaxis): the stored point of sahkdtree3.h:239-244
    auto pt = [&](float t, float split, uint32_t eaxis, int a) -> float {
        if ((uint32_t)a == eaxis) return split;
        const float oa = a == 0 ? o.x : (a == 1 ? o.y : o.z);
        const float da = a == 0 ? d.x : (a == 1 ? d.y : d.z);
        return oa + da * t;
    };
    uint32_t sp = 0;
    // the two newest stack entries held in registers (entries sp - 1 and sp - 2
    // when nr = 2), the rest in memory; a cached entry packs its axis into the
    // node word's top bits (kd node indices stay below 2^30, capi.cpp)
    uint32_t nr = 0, c0n = 0, c1n = 0;
    float c0t = 0, c0s = 0, c1t = 0, c1s = 0;
    float en_t = mint, en_split = 0, ex_t = maxt, ex_split = 0;   // ray(mint), ray(maxt)
    uint32_t en_axis = NOAXIS, ex_axis = NOAXIS;
    bool found = false;
    uint32_t node = 0;
    while (true) {
        uint2 n = nodes[node];
        while (!(n.x & 0x80000000u)) {
            const float split = __uint_as_float(n.y);
            const int axis = (int)(n.x & 3u);
            const uint32_t left = node + ((n.x & ~(3u | 0x40000000u)) >> 2);
            const float enP = pt(en_t, en_split, en_axis, axis);
            const float exP = pt(ex_t, ex_split, ex_axis, axis);
            uint32_t farChild;
            if (enP <= split) {
                if (exP <= split) { node = left; n = nodes[node]; continue; }
                if (enP == split) { node = left + 1; n = nodes[node]; continue; }
                node = left;
                farChild = left + 1;
            } else {
                if (split < exP) { node = left + 1; n = nodes[node]; continue; }
                farChild = left;
                node = left + 1;
            }
            const float oa = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
            const float distToSplit = (split - oa) * rcp[axis];
            if (sp >= DEPTH) return found;   // MTS_KD_MAXDEPTH bounds the tree depth; never taken
            if (nr == 2) st(sp - 2, Ent{c1n & 0x3fffffffu, c1t, c1s, c1n >> 30});
            c1n = c0n; c1t = c0t; c1s = c0s;
            c0n = farChild | (ex_axis << 30); c0t = ex_t; c0s = ex_split;
            nr = nr < 2 ? nr + 1 : 2;
            ++sp;
            ex_t = distToSplit;
            ex_split = split;
            ex_axis = (uint32_t)axis;
            n = nodes[node];
        }
        for (uint32_t e = n.x & 0x7fffffffu; e != n.y; ++e) {
            // the record of list entry e (tris in leaf-list order): its loads do
            // not wait on indices[e], and the test is formed before the mailbox
            // decides whether it counts, so no load sits behind that branch
            const MtsgTri &tr = tris[e];
            const uint32_t prim = tr.prim;
            const uint32_t k = tr.k;
            float o_u, o_v, o_k, d_u, d_v, d_k;
            if (k == 0) { o_u = o.y; o_v = o.z; o_k = o.x; d_u = d.y; d_v = d.z; d_k = d.x; }
            else if (k == 1) { o_u = o.z; o_v = o.x; o_k = o.y; d_u = d.z; d_v = d.x; d_k = d.y; }
            else { o_u = o.x; o_v = o.y; o_k = o.z; d_u = d.x; d_v = d.y; d_k = d.z; }
            // TriAccel::rayIntersect (triaccel.h:92-160) on [mint, maxt]
            const float t = (tr.n_d - o_u * tr.n_u - o_v * tr.n_v - o_k) / (d_u * tr.n_u + d_v * tr.n_v + d_k);
            const float hu = o_u + t * d_u - tr.a_u;
            const float hv = o_v + t * d_v - tr.a_v;
            const float u = hv * tr.b_nu + hu * tr.b_nv;
            const float v = hu * tr.c_nu + hv * tr.c_nv;
            if (mb(prim & 7u) == prim) continue;   // the hashed mailbox (sahkdtree3.h:138-152)
            if (!(t < mint || t > maxt) && u >= 0 && v >= 0 && u + v <= 1.0f) {
                if (ANY) return true;
                maxt = t;
                found = true;
                bt = t; bu = u; bv = v; bprim = prim;
            }
            mbset(prim & 7u, prim);
        }
        if (ex_t > maxt) break;
        if (sp == 0) break;   // the exit point was ray(maxt), whose node is NONE
        en_t = ex_t;
        en_split = ex_split;
        en_axis = ex_axis;
        Ent e;
        if (nr) {
            e = Ent{c0n & 0x3fffffffu, c0t, c0s, c0n >> 30};
            c0n = c1n; c0t = c1t; c0s = c1s;
            --nr;
        } else {
            e = ld(sp - 1);
        }
        --sp;
        node = e.node;
        ex_t = e.t;
        ex_split = e.split;
        ex_axis = e.axis;
    }
    return found;
}

// ShapeKDTree::rayIntersect (skdtree.cpp:112-142 closest, :207-226 shadow):
// scene-AABB clip + adaptive ray epsilon -> [mint, maxt] for the traversal
__device__ __forceinline__ bool ray_interval(const MtsgDeviceScene &S, f3 o, f3 d, float rmint, float rmaxt,
                                             bool shadow, float &mint, float &maxt) {
    if (!aabb_clip(S, o, d, mint, maxt)) return false;
    float rayMinT = rmint;
    if (rayMinT == D_EPSILON) {
        if (shadow) rayMinT *= smax(smax(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
        else rayMinT *= smax(smax(smax(fabsf(o.x), fabsf(o.y)), fabsf(o.z)), D_EPSILON);
    }
    if (rayMinT > mint) mint = rayMinT;
    if (rmaxt < maxt) maxt = rmaxt;
    return maxt > mint;
}

// computeShadingFrame (util.cpp:603-608); t = cross(n, s) is ShFrame::t()
__device__ __forceinline__ ShFrame shading_frame(f3 n, f3 dpdu) {
    ShFrame f;
    f.n = n;
    f.s = normalize(sub(dpdu, mul(f.n, dot(f.n, dpdu))));
    return f;
}

// Where a vertex's triangle data comes from: HBM, or (small scenes, SCENE_LDS)
// the LDS copy every workgroup stages next to the BVH
typedef __attribute__((address_space(3))) const float lds_f32;
typedef __attribute__((address_space(1))) const MtsgShape glb_shape;
typedef __attribute__((address_space(3))) const MtsgShape lds_shape;
template <bool INLDS> struct HitSrc;
template <> struct HitSrc<false> { glb_u32 *pv; glb_f32 *pos, *nrm, *dpdu; glb_shape *shapes; };
template <> struct HitSrc<true> { lds_u32 *pv; lds_f32 *pos, *nrm, *dpdu; lds_shape *shapes; };
template <typename P> __device__ __forceinline__ f3 ldp3(P p) { return mk(p[0], p[1], p[2]); }

// fillIntersectionRecord<true> (skdtree.h:343-429); UV = TEX
template <bool TEX, bool ANA, typename HS>
__device__ __forceinline__ void fill_hit(const MtsgDeviceScene &S, const HS &hs, uint32_t slot, uint32_t prim, float u,
                                         float v, float t, f3 o, f3 d, Hit &h) {
    if constexpr (ANA) {
        const MtsgTri &tr = S.tris[slot];
        if (tr.k == MTSG_K_ANALYTIC) {   // Shape::fillIntersectionRecord + skdtree.h:425-427
            const AnaHit a = ana_fill(((GAna *)S.analytic)[__float_as_uint(tr.n_u)], o, d, t, u, v);
            h.valid = 1;
            h.t = t;
            h.shape = (int)tr.shape;
            h.p = a.p;
            h.geoN = a.geoN;
            h.sh = shading_frame(a.shN, a.dpdu);
            h.wi = to_local(h.sh, neg(d));
            if constexpr (TEX) { h.u = a.u; h.v = a.v; }
            return;
        }
    }
    const uint4 pv = make_uint4(hs.pv[4 * prim], hs.pv[4 * prim + 1], hs.pv[4 * prim + 2], hs.pv[4 * prim + 3]);
    h.valid = 1;
    h.t = t;
    h.shape = (int)pv.w;
    const float bx = 1 - u - v, by = u, bz = v;
    const f3 p0 = ldp3(hs.pos + 3 * (size_t)pv.x), p1 = ldp3(hs.pos + 3 * (size_t)pv.y),
             p2 = ldp3(hs.pos + 3 * (size_t)pv.z);
    h.p = add(add(mul(p0, bx), mul(p1, by)), mul(p2, bz));
    const f3 side1 = sub(p1, p0), side2 = sub(p2, p0);
    f3 faceNormal = cross(side1, side2);
    const float length = len(faceNormal);
    if (!is_zero(faceNormal)) faceNormal = divs(faceNormal, length);
    const f3 dpdu = ldp3(hs.dpdu + 3 * (size_t)prim);
    f3 shN;
    if (hs.shapes[h.shape].has_normals) {
        const f3 n0 = ldp3(hs.nrm + 3 * (size_t)pv.x), n1 = ldp3(hs.nrm + 3 * (size_t)pv.y),
                 n2 = ldp3(hs.nrm + 3 * (size_t)pv.z);
        shN = normalize(add(add(mul(n0, bx), mul(n1, by)), mul(n2, bz)));
        if (dot(faceNormal, shN) < 0) faceNormal = neg(faceNormal);
    } else {
        shN = faceNormal;
    }
    h.geoN = faceNormal;
    h.sh = shading_frame(shN, dpdu);
    h.wi = to_local(h.sh, neg(d));
    if constexpr (TEX) {   // skdtree.h:398-405: t0*b.x + t1*b.y + t2*b.z, else (b.y, b.z)
        if (hs.shapes[h.shape].has_uv) {
            const float *tc = S.texcoords;
            h.u = tc[2 * (size_t)pv.x] * bx + tc[2 * (size_t)pv.y] * by + tc[2 * (size_t)pv.z] * bz;
            h.v = tc[2 * (size_t)pv.x + 1] * bx + tc[2 * (size_t)pv.y + 1] * by + tc[2 * (size_t)pv.z + 1] * bz;
        } else {
            h.u = by;
            h.v = bz;
        }
    }
}

// The wavefront engine's hit record formed by the trace kernel (MtsgWave::hitrec,
// MTSG_WF_HIT_VECS float4 per slot): fill_hit's result, bit for bit, so a shade
// kernel starts from one contiguous record instead of the slot -> prim -> vertex
// chain of dependent loads.  The 6th vector (UVs) is written for textured scenes only.
__device__ __forceinline__ void hit_store(float4 *r, const Hit &h, bool uv) {
    r[0] = make_float4(h.t, h.p.x, h.p.y, h.p.z);
    r[1] = make_float4(h.geoN.x, h.geoN.y, h.geoN.z, h.wi.x);
    const f3 t = h.sh.t();
    r[2] = make_float4(h.wi.y, h.wi.z, h.sh.s.x, h.sh.s.y);
    r[3] = make_float4(h.sh.s.z, t.x, t.y, t.z);
    r[4] = make_float4(h.sh.n.x, h.sh.n.y, h.sh.n.z, __int_as_float(h.shape));
    if (uv) r[5] = make_float4(h.u, h.v, 0.0f, 0.0f);
}
template <bool UV> __device__ __forceinline__ void hit_load(const float4 *r, Hit &h) {
    const float4 a = r[0], b = r[1], c = r[2], d = r[3], e = r[4];
    h.valid = 1;
    h.t = a.x;
    h.p = mk(a.y, a.z, a.w);
    h.geoN = mk(b.x, b.y, b.z);
    h.wi = mk(b.w, c.x, c.y);
    h.sh.s = mk(c.z, c.w, d.x);
    h.sh.n = mk(e.x, e.y, e.z);   // (d.yzw: t, re-formed as cross(n, s))
    h.shape = __float_as_int(e.w);
    if constexpr (UV) { const float4 f = r[5]; h.u = f.x; h.v = f.y; }
}

// DiscreteDistribution::sample/sampleReuse (core/pmf.h:124-169)
__device__ __forceinline__ uint32_t dd_sample_reuse(const float *__restrict__ cdf, uint32_t n, float &value,
                                                   float *pdf) {
    uint32_t lo = 0, hi = n + 1;                          // std::lower_bound
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] < value) lo = mid + 1; else hi = mid;
    }
    int idx = (int)lo - 1;
    if (idx < 0) idx = 0;
    uint32_t index = (uint32_t)idx;
    if (index > n - 1) index = n - 1;
    while (cdf[index + 1] - cdf[index] == 0 && index < n - 1) ++index;
    const float c0 = cdf[index], c1 = cdf[index + 1];
    if (pdf) *pdf = c1 - c0;
    value = (value - c0) / (c1 - c0);
    return index;
}

// ---------------------------------------------------------------------------
// film splat: ImageBlock::put (render/imageblock.h:124-204) into the 32x32
// block that owns pixel (px, py); own-pixel weight goes to the lane's
// registers, other touched pixels to the spill film (double atomics)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float filter_disc(const MtsgFilter &F, float x) {
    int i = (int)fabsf(x * F.scale);
    if (MTSG_FILTER_RES < i) i = MTSG_FILTER_RES;
    return F.values[i];
}

__device__ __forceinline__ bool film_splat(const MtsgLaunch &L, int px, int py, float sx, float sy,
                                           const float *val, float &ownW) {
#pragma unroll
    for (int i = 0; i < 5; ++i)
        if (!isfinite(val[i]) || val[i] < 0) return false;
    const MtsgFilter &F = L.filter;
    const int b = F.border;
    const int bx = (px / MTSG_BLOCK_SIZE) * MTSG_BLOCK_SIZE, by = (py / MTSG_BLOCK_SIZE) * MTSG_BLOCK_SIZE;
    const int bw = MTSG_BLOCK_SIZE + 2 * b;
    const float posx = sx - 0.5f - (float)(bx - b), posy = sy - 0.5f - (float)(by - b);
    int minx = (int)ceilf(posx - F.radius), miny = (int)ceilf(posy - F.radius);
    int maxx = (int)floorf(posx + F.radius), maxy = (int)floorf(posy + F.radius);
    if (minx < 0) minx = 0;
    if (miny < 0) miny = 0;
    if (maxx > bw - 1) maxx = bw - 1;
    if (maxy > bw - 1) maxy = bw - 1;
    for (int y = miny; y <= maxy; ++y) {
        const float wy = filter_disc(F, (float)y - posy);
        for (int x = minx; x <= maxx; ++x) {
            const float weight = filter_disc(F, (float)x - posx) * wy;
            const int gx = x + bx, gy = y + by;
            if (gx >= L.fw || gy >= L.fh) continue;
            if (gx == px + b && gy == py + b) {
                ownW = weight;
            } else {
                // weight * value[k] in float as the reference forms it, summed in double:
                // exact for contributions within 2^29 of each other, so the spill film
                // does not depend on the order the atomics land (film_finalize rounds once)
                double *dst = L.film_spill + ((size_t)gy * L.fw + gx) * 5;
#pragma unroll
                for (int k = 0; k < 5; ++k) atomicAdd(dst + k, (double)(weight * val[k]));
            }
        }
    }
    return true;
}

// block->put(samplePos, spec, alpha) (integrator.cpp:184) as the sample's record in
// the splat buffer (slot = (j - j0) * num_pixels + pix).  Box filter: {L.rgb, w} with
// the own-pixel weight w (alpha in {0,1} in its sign bit; film_reduce re-forms
// weight * value[k]) and the rare neighbour splats as atomics.  Gather mode: the
// sample's value and film position, {L.rgb, sx (alpha in its sign bit: sx >= +0)}
// and {sy (-1: an invalid sample, which ImageBlock::put drops whole), 0, 0, 0} in one
// 32 B record: HBM writes whole 32 B sectors (profiles/r06_write_gran), so the
// record costs what a lone 16 B store costs, where a separate 4 B sy array cost
// another sector; film_gather forms every footprint weight with film_splat's arithmetic.
#ifndef MTSG_SPLAT_PAIR
#define MTSG_SPLAT_PAIR 1
#endif
// the record slot of sample jj (= j - j0) of compact pixel pix.  Box filter: the records
// of samples 2k and 2k+1 of a pixel share one 32 B sector (the lanes that write them
// run at different times; the sector is written to HBM once if both halves meet in L2).
// Gather mode: one 32 B record per slot.
__device__ __forceinline__ size_t film_slot(const MtsgLaunch &L, uint32_t jj, uint32_t pix) {
    if (MTSG_SPLAT_PAIR && !L.gather) return ((size_t)(jj >> 1) * L.num_pixels + pix) * 2 + (jj & 1);
    return (size_t)jj * L.num_pixels + pix;
}

__device__ __forceinline__ void film_record(const MtsgLaunch &L, size_t slot, int px, int py, float sx, float sy,
                                            const float *val, bool alpha) {
    float4 rec4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (L.gather) {
        bool valid = true;
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (!isfinite(val[i]) || val[i] < 0) valid = false;   // (alpha and 1 are valid)
        if (valid) rec4 = make_float4(val[0], val[1], val[2], alpha ? sx : -sx);
        float4 *r = reinterpret_cast<float4 *>(L.contrib) + 2 * slot;
        r[0] = rec4;
        r[1] = make_float4(valid ? sy : -1.0f, 0.0f, 0.0f, 0.0f);
        return;
    }
    float ownW = 0.0f;
    if (film_splat(L, px, py, sx, sy, val, ownW)) rec4 = make_float4(val[0], val[1], val[2], alpha ? ownW : -ownW);
    reinterpret_cast<float4 *>(L.contrib)[slot] = rec4;
}

// ---------------------------------------------------------------------------
// the persistent path kernel
// ---------------------------------------------------------------------------
// whether the BSDF sample that spawned the current ray chose a delta lobe
// (BSDFSamplingRecord::sampledType & EDelta, path.cpp:262,280): one bit
#define PV_DELTA(P) ((P).delta != 0)
#define PV_SET_DELTA(P, t) ((P).delta = ((t) & MTSG_F_DELTA) != 0)
struct PathVars {
    f3 L, thr;
    float eta;
    int depth;
    // flags as bits of one word (bools each took a lane-mask SGPR pair across the loop);
    // alpha is the sample's film alpha, 0 or 1 (path.cpp:125-131, records.inl:117-144)
    uint32_t scattered : 1, emitted : 1, delta : 1, alpha : 1;
    Hit its;          // current vertex
    f3 neeC;          // throughput*value*bsdfVal*weight, committed if the shadow ray is unoccluded
    f3 refN;          // DirectSamplingRecord::refN of the current vertex
    float bsdfPdf;
};

__device__ __forceinline__ float next1d(const SobolCtx &C, SamplerState &s) {   // sobol.cpp:219-229
    if (C.replay) { s.dim++; return sfmt_next_float(lane_sfmt(C)); }   // independent.cpp:97-99
    if (s.dim >= MTSG_SOBOL_DIMS && !C.indep) { s.err = true; return 0.0f; }
    return sobol_sample(C, s.sobolIndex, s.dim++);
}
__device__ __forceinline__ void next2d(const SobolCtx &C, float resolution, SamplerState &s, int px, int py,
                                       float &u, float &v) {                       // sobol.cpp:231-250
    if (C.replay) {   // independent.cpp:101-105: value1, then value2
        u = sfmt_next_float(lane_sfmt(C));
        v = sfmt_next_float(lane_sfmt(C));
        s.dim += 2;
        return;
    }
    if (s.dim + 1 >= 5 && s.dim < 5) s.dim = 5;   // skip the (empty) array dimensions [5,5)
    if (s.dim + 1 >= MTSG_SOBOL_DIMS && !C.indep) { s.err = true; u = v = 0.0f; return; }
    if (!C.indep && s.dim == 0 && s.sobolIndex != (uint64_t)s.sampleIndex) {
        u = sobol_sample(C, s.sobolIndex, s.dim++) * resolution - (float)px;
        v = sobol_sample(C, s.sobolIndex, s.dim++) * resolution - (float)py;
    } else {
        u = sobol_sample(C, s.sobolIndex, s.dim++);
        v = sobol_sample(C, s.sobolIndex, s.dim++);
    }
}

__device__ __forceinline__ f3 xf_point(const float *m, f3 p) {         // transform.h:108-125
    float x = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float y = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float z = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float w = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (w == 1.0f) return mk(x, y, z);
    return divs(mk(x, y, z), w);
}

__device__ __forceinline__ f3 area_Le(const MtsgDeviceScene &S, const Hit &h, f3 d) {   // area.cpp:104-109
    const MtsgEmitter &e = S.emitters[S.shapes[h.shape].emitter];
    if (dot(h.sh.n, d) <= 0) return mk(0, 0, 0);
    return ld3(e.radiance);
}

// ConstantBackgroundEmitter (emitters/constant.cpp): pdfDirect in solid angle
// (:216-231) and sampleDirect (:167-214) on the scene's bounding sphere
#define D_INV_FOURPI 0.07957747154594766788f
__device__ __forceinline__ float const_pdf_direct(f3 d, f3 refN) {
    if (!is_zero(refN)) return D_INV_PI * smax(0.0f, dot(d, refN));
    return D_INV_FOURPI;   // warp::squareToUniformSpherePdf
}
__device__ __noinline__ EnvSample const_sample_direct(glb_env *E, f3 ref, f3 refN, float sx, float sy) {
    EnvSample r;
    r.value = mk(0, 0, 0); r.pdf = 0.0f; r.dist = 0.0f;
    f3 d;
    float pdf;
    if (!is_zero(refN)) {
        d = square_to_cosine_hemisphere(sx, sy);
        pdf = D_INV_PI * d.z;
        Frame F;
        F.n = refN;
        coordinate_system(refN, F.s, F.t);
        d = to_world(F, d);
    } else {
        const float z = 1.0f - 2.0f * sy;   // warp::squareToUniformSphere (warp.cpp:25-31)
        const float rr = safe_sqrt(1.0f - z * z);
        float sinPhi, cosPhi;
        d_sincos(2.0f * D_PI * sx, &sinPhi, &cosPhi);
        d = mk(rr * cosPhi, rr * sinPhi, z);
        pdf = D_INV_FOURPI;
    }
    r.d = d;
    float nearT, farT;
    if (!env_bsphere(E, ref, d, nearT, farT)) return r;
    if (!(nearT < 0 && farT > 0)) return r;
    r.dist = farT;
    r.pdf = pdf;
    if (!is_zero(refN) && dot(d, refN) <= 0) return r;   // roundoff moved the sample to the backside
    r.value = divs(mk(E->radiance[0], E->radiance[1], E->radiance[2]), pdf);
    return r;
}

// compact pixel index (8x8 tiles over the window's active rows, or the
// window's every row_stride-th tile) -> image pixel
__device__ __forceinline__ bool pixel_of(const MtsgLaunch &L, uint32_t p, int &px, int &py) {
    const uint32_t tile = p >> 6, in = p & 63;
    if (L.tile_shard) {
        const uint32_t t = tile * L.row_stride + L.row_phase;
        const uint32_t lx = (t % L.tiles_x) * 8 + (in & 7), ly = (t / L.tiles_x) * 8 + (in >> 3);
        if (lx >= L.width || ly >= L.height) return false;
        px = (int)(L.x0 + lx);
        py = (int)(L.y0 + ly);
        return true;
    }
    const uint32_t lx = (tile % L.tiles_x) * 8 + (in & 7);
    const uint32_t r = (tile / L.tiles_x) * 8 + (in >> 3);
    if (lx >= L.width) return false;
    const uint32_t blk = r / L.row_block, off = r % L.row_block;
    const uint32_t ly = (blk * L.row_stride + L.row_phase) * L.row_block + off;
    if (ly >= L.height) return false;
    px = (int)(L.x0 + lx);
    py = (int)(L.y0 + ly);
    return true;
}

#ifndef MTSG_WAVES_PER_EU
#define MTSG_WAVES_PER_EU 3
#endif

// sobol::look_up (sobolseq.h:93-125) as the GF(2) solve it encodes; the XOR of
// the second dimension's (top m bits of) columns over the index bits comes from
// 4-bit tables in LDS (ycolTab[c][v]), the m x m inverse from the kernel args
template <typename T>
__device__ __forceinline__ uint64_t sobol_lookup_lds(const MtsgLookup &Lu, T *ycolTab, uint32_t nibbles,
                                                     uint32_t frame, uint32_t px, uint32_t py, uint64_t scramble) {
    const uint32_t m = Lu.m;
    const uint32_t s = (uint32_t)((scramble & 0xFFFFFFFFull) >> (32 - m));
    const uint32_t mask = (1u << m) - 1u;
    const uint32_t sx = (px ^ s) & mask, sy = (py ^ s) & mask;
    const uint32_t jlo = __builtin_bitreverse32(sx) >> (32 - m);
    const uint64_t index = ((uint64_t)frame << (2 * m)) | jlo;
    const uint32_t K = (nibbles == 8) ? sobol_bits<8>(ycolTab, index) : sobol_bits<MTSG_NIBBLES>(ycolTab, index);
    const uint32_t rhs = (sy ^ K) & mask;
    uint32_t jhi = 0;
    for (uint32_t t = 0; t < m; ++t) jhi |= (uint32_t)(__builtin_popcount(Lu.inv[t] & rhs) & 1) << t;
    return index | ((uint64_t)jhi << m);
}

// ---------------------------------------------------------------------------
// Li() as a per-path state machine, one bounce per step.  One step traces the
// path's pending shadow ray (NEE of the previous vertex) and its closest-hit
// ray (camera or BSDF-sampled), then shades the new vertex: add the NEE
// estimate if unoccluded, the MIS-weighted emission of the hit, Russian
// roulette, then at the new vertex draw the NEE sample and the BSDF sample,
// which produce the next step's two rays.  Sampler dimensions are consumed in
// the reference's order (NEE 2D, BSDF 2D [+1D], RR 1D), and radiance is
// accumulated in the reference's order (NEE term before the BSDF-hit term).
// PathShader holds the three pieces both execution models share: start (the
// renderBlock loop body up to Li's prologue), shade (the rest of one bounce)
// and finish (block->put).  The persistent megakernel (path_kernel) runs them
// with both traversals inline; the wavefront pipeline (wf_shade / wf_trace)
// runs the traversals as separate kernels over compacted ray queues.
// ---------------------------------------------------------------------------
// (the pixel's coordinates and the sample index are not kept: pixel_of(pix)
// and smp.sampleIndex give them where needed, two and one fewer registers
// live across every bounce)
struct PathState {
    uint32_t active : 1, haveRay : 1, primary : 1, haveShadow : 1;   // one word of bits
    uint32_t pix;
    float sx, sy;
    SamplerState smp;
    PathVars P;
    // rays of the next trace step: closest (camera / extension) and shadow (NEE).
    // Both leave P.its.p (the camera position for the primary ray, set by begin()):
    // the closest-hit ray's origin is not held separately
    f3 rd, sd;
    float rmint, rmaxt, smaxt;
};

// per-lane counts: 32-bit for the always-on ones (fewer live VGPRs in the
// persistent loop; finish() flushes them long before they could wrap),
// 64-bit for the INSTR-only traversal statistics
struct PathCounters {
    uint32_t rays, shadow, len, samples, err;
    unsigned long long nodes, tests, hits, nee, sobol;
};

// LDS of path_kernel / wf_shade: [Sobol nibble tables][look_up column tables]
// [BVH + TriAccel + hit data (SCENE_LDS)][traversal stacks]
template <bool SCENE_LDS>
struct LdsView {
    lds_u32 *ycolTab;
    lds_node *nodes;
    lds_tri *tris;
    HitSrc<SCENE_LDS> hs;
    SobolCtx SC;
    uint32_t stackBase;   // word offset of the traversal stacks
};

template <bool SCENE_LDS>
__device__ __forceinline__ LdsView<SCENE_LDS> lds_view(const MtsgLaunch &L, uint32_t *lds);

template <bool SCENE_LDS>
__device__ __forceinline__ LdsView<SCENE_LDS> stage_lds(const MtsgLaunch &L, uint32_t *lds) {
    const MtsgDeviceScene &S = L.scene;
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
        // the vertices' triangle data: prim_vtx, dpdu, positions, normals, shape records
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
    return lds_view<SCENE_LDS>(L, lds);
}

// the pointers into the staged LDS (and the scene buffers it mirrors), derived
// from the launch record alone: the persistent megakernel re-derives them per
// bounce from launch_fresh() instead of holding them live across it
template <bool SCENE_LDS>
__device__ __forceinline__ LdsView<SCENE_LDS> lds_view(const MtsgLaunch &L, uint32_t *lds) {
    const MtsgDeviceScene &S = L.scene;
    const uint32_t tabWords = L.lds_dims * L.nibbles * 16;
    const uint32_t base2 = tabWords + 16 * 16;
    uint32_t sceneWords = 0;
    if (SCENE_LDS) {
        sceneWords = L.num_nodes * 16 + S.num_prims * 12 + 4 * S.num_prims + 3 * S.num_prims + 3 * L.num_verts +
                     3 * L.num_verts + L.num_shapes * (uint32_t)(sizeof(MtsgShape) / 4);
    }
    LdsView<SCENE_LDS> v;
    v.ycolTab = (lds_u32 *)(lds + tabWords);
    // base2 and the node array size are multiples of 4 words: 16-byte aligned (ds_read_b128)
    v.nodes = (lds_node *)__builtin_assume_aligned((const void *)(lds + base2), 16);
    v.tris = (lds_tri *)__builtin_assume_aligned((const void *)(lds + base2 + L.num_nodes * 16), 16);
    // triangle data of hit records and emitter samples (HitSrc)
    if constexpr (SCENE_LDS) {
        const uint32_t np = S.num_prims, nv = L.num_verts;
        lds_u32 *b = (lds_u32 *)(lds + base2 + L.num_nodes * 16 + np * 12);
        v.hs.pv = b;
        v.hs.dpdu = (lds_f32 *)(b + 4 * np);
        v.hs.pos = (lds_f32 *)(b + 7 * np);
        v.hs.nrm = (lds_f32 *)(b + 7 * np + 3 * nv);
        v.hs.shapes = (lds_shape *)(b + 7 * np + 6 * nv);
    } else {
        v.hs.pv = (glb_u32 *)S.prim_vtx;
        v.hs.dpdu = (glb_f32 *)S.dpdu;
        v.hs.pos = (glb_f32 *)S.positions;
        v.hs.nrm = (glb_f32 *)S.normals;
        v.hs.shapes = (glb_shape *)S.shapes;
    }
    v.SC.lds = (lds_u32 *)lds;
    v.SC.glob = (glb_u32 *)L.sobol_nib;
    v.SC.lds_dims = L.lds_dims;
    v.SC.nibbles = L.nibbles;
    v.SC.scramble = L.scramble;
    v.SC.indep = L.sampler != MTSG_SAMPLER_SOBOL;
    v.SC.replay = L.replay != 0;
    v.SC.sfmt = L.sfmt;
    v.stackBase = base2 + sceneWords;
    return v;
}

// INSTR: traversal statistics + optional per-sample records (tests, roofline
// pass); SCENE_LDS: BVH + TriAccel staged in LDS; FEAT: MTSG_FEAT_ENV (scene
// has an environment emitter) | MTSG_FEAT_EXT (roughplastic, textures, smooth
// BSDFs, twosided) | MTSG_FEAT_ANA (analytic shapes)
// KIND / HITK (the wavefront engine's per-type shade kernels, wf_kernel.hip):
// the BSDF type at the vertex (BSDF_*, -1: any) and whether the step's
// closest-hit ray is known to have hit (1), known to have missed or not to
// exist (2), or unknown (0, the megakernel)
template <bool INSTR, bool SCENE_LDS, int FEAT, int KIND = -1, int HITK = 0>
struct PathShader {
    static constexpr bool STATS = INSTR;
    static constexpr bool ENV = (FEAT & MTSG_FEAT_ENV) != 0, EXT = (FEAT & MTSG_FEAT_EXT) != 0,
                          ANA = (FEAT & MTSG_FEAT_ANA) != 0, DIFF = (FEAT & MTSG_FEAT_DIFF) != 0;
    static constexpr int BSF = FEAT & BSET_BITS;   // the variant's BSDF set (dbsdf.h BSet)
    // the BSDF-set megakernels are built without strictNormals (the geometric normal
    // is then dead once the hit is formed); scenes with it run the generic kernel
    static constexpr bool NOSTRICT = (FEAT & MTSG_FEAT_NOSTRICT) != 0;
    // REFN false (MTSG_FEAT_NOREFN, capi.cpp): the scene's only emitter is a non-constant
    // envmap, whose sampleDirect / pdfDirect do not read refN (envmap.cpp:516-556): the area
    // light and constant-emitter code is compiled out and refN (three floats live across the
    // NEE and BSDF calls and the next traversal) is not kept
    static constexpr bool REFN = (FEAT & MTSG_FEAT_NOREFN) == 0;
    const MtsgLaunch &L;
    const HitSrc<SCENE_LDS> &hs;
    const SobolCtx &SC;
    lds_u32 *ycolTab;
    PathCounters &c;

    // the renderBlock loop body for item `it` up to Li()'s prologue
    // (integrator.cpp:165-186, path.cpp:119-133); false for a padding pixel
    __device__ __forceinline__ bool start(PathState &st, uint64_t it) const {
        const uint32_t jj = (uint32_t)(it / L.num_pixels);
        return start_jp(st, jj, (uint32_t)(it - (uint64_t)jj * L.num_pixels));
    }
    // sample jj of the chunk at compact pixel pix
    __device__ __forceinline__ bool start_jp(PathState &st, uint32_t jj, uint32_t pix) const {
        st.pix = pix;
        int px, py;
        if (!pixel_of(L, st.pix, px, py)) return false;
        begin(st, jj, px, py);
        return true;
    }
    // the SFMT replay's next sample: crop pixel xy (x | y << 16), sample jj of the chunk
    __device__ __forceinline__ void start_xy(PathState &st, uint32_t xy, uint32_t jj) const {
        const uint32_t lx = xy & 0xffffu, ly = xy >> 16;   // row_stride 1: compact row = ly
        st.pix = ((ly >> 3) * L.tiles_x + (lx >> 3)) * 64u + (ly & 7u) * 8u + (lx & 7u);   // pixel_of's inverse
        begin(st, jj, (int)(L.x0 + lx), (int)(L.y0 + ly));
    }

    __device__ __forceinline__ void begin(PathState &st, uint32_t jj, const int px, const int py) const {
        const MtsgDeviceScene &S = L.scene;
        SamplerState &smp = st.smp;
        PathVars &P = st.P;
        const uint32_t j = L.j0 + jj;
        float &sx = st.sx, &sy = st.sy;
        f3 &rd = st.rd;
        float &rmint = st.rmint, &rmaxt = st.rmaxt;
        smp.dim = 0;
        smp.sampleIndex = j;
        smp.err = false;
        if (SC.indep)
            smp.sobolIndex = indep_key((uint32_t)px, (uint32_t)py, j);
        else if (L.lut.m > 1)
            smp.sobolIndex = sobol_lookup_lds(L.lut, ycolTab, L.nibbles, j, (uint32_t)px, (uint32_t)py, L.scramble64);
        else
            smp.sobolIndex = j;
        float u, v;
        next2d(SC, L.resolution, smp, px, py, u, v);
        sx = (float)px + u;
        sy = (float)py + v;
        // PerspectiveCameraImpl::sampleRayDifferential (perspective.cpp:271-298)
        const MtsgCamera &cam = S.cam;
        const f3 nearP = xf_point(cam.sample_to_camera, mk(sx * cam.inv_res_x, sy * cam.inv_res_y, 0.0f));
        const f3 dl = normalize(nearP);
        const float invZ = 1.0f / dl.z;
        rmint = cam.near_clip * invZ;
        rmaxt = cam.far_clip * invZ;
        const float *W = cam.to_world;
        P.its.p = mk(W[0] * 0.0f + W[1] * 0.0f + W[2] * 0.0f + W[3], W[4] * 0.0f + W[5] * 0.0f + W[6] * 0.0f + W[7],
                     W[8] * 0.0f + W[9] * 0.0f + W[10] * 0.0f + W[11]);   // the ray's origin
        rd = mk(W[0] * dl.x + W[1] * dl.y + W[2] * dl.z, W[4] * dl.x + W[5] * dl.y + W[6] * dl.z,
                W[8] * dl.x + W[9] * dl.y + W[10] * dl.z);
        // Li() prologue (path.cpp:119-133)
        P.L = mk(0, 0, 0);
        P.thr = mk(1.0f, 1.0f, 1.0f);
        P.eta = 1.0f;
        P.depth = 1;
        P.scattered = false;
        P.emitted = true;
        st.haveRay = true;
        st.primary = true;
        st.haveShadow = false;
        st.active = true;
    }

    // the rest of one bounce, given the step's trace results: returns true
    // when the path ends (path.cpp:135-292).  usePre: the hit record `pre` is already
    // formed (the wavefront's trace kernel), else fill_hit forms it from (slot, prim, u, v, t)
    __device__ __forceinline__ bool shade(PathState &st, bool occluded, bool hit, uint32_t slot, uint32_t prim,
                                          float hu, float hv, float ht, bool usePre = false, const Hit &pre = Hit{}) const {
        const MtsgDeviceScene &S = L.scene;
        PathVars &P = st.P;
        SamplerState &smp = st.smp;
        // next2d reads the pixel only for dimensions 0-1 (begin() has drawn them)
        const int px = 0, py = 0;
        const float sx = st.sx, sy = st.sy;
        if constexpr (HITK == 1) hit = true;
        if constexpr (HITK == 2) hit = false;
        f3 &rd = st.rd, &sd = st.sd;
        const f3 ro = P.its.p;   // the ray's origin: the previous vertex (or the camera)
        float &rmint = st.rmint, &rmaxt = st.rmaxt, &smaxt = st.smaxt;
        bool endPath = false;
        // NEE of the previous vertex (scene.cpp:838-842, path.cpp:176-199)
        if (st.haveShadow && !occluded) P.L = add(P.L, P.neeC);
        st.haveShadow = false;
        bool vertex = false;
        if (!st.haveRay) {
            endPath = true;   // the BSDF sample at the previous vertex failed
        } else {
            // rRec.rayIntersect / scene->rayIntersect (records.inl:117-144, path.cpp:226)
            // a miss overwrites the whole record: no field of the previous vertex stays
            // live across the next traversal except through an explicit use
            if (hit) {
                if (usePre) P.its = pre;
                else fill_hit<EXT, ANA>(S, hs, slot, prim, hu, hv, ht, ro, rd, P.its);
            } else {
                P.its = Hit{};
            }
            if (STATS && hit) c.hits++;
            if (st.primary) {
                P.alpha = L.has_alpha ? (P.its.valid ? 1u : 0u) : 1u;
                vertex = true;
            } else if (HITK == 2 || !P.its.valid) {
                // missed: the environment emitter, if any (path.cpp:233-247)
                if (ENV && !(L.hide_emitters && !P.scattered)) {
                    glb_env *E = (glb_env *)S.env;
                    const bool cst = REFN && E->constant;
                    EnvValPdf vp = {mk(0, 0, 0), 0.0f};
                    if (!cst) vp = env_eval_pdf_at(E, env_uv(E, rd));   // one (u, v) and texel set for both
                    const f3 value = cst ? mk(E->radiance[0], E->radiance[1], E->radiance[2]) : vp.value;
                    float nT, fT;
                    // EnvironmentMap::fillDirectSamplingRecord (envmap.cpp:358-374)
                    if (env_bsphere(E, ro, rd, nT, fT) && !(nT > 0 || fT < 0)) {
                        float lumPdf = 0;
                        if (!PV_DELTA(P))   // pdfDirect (envmap.cpp:545-556) x pdfEmitterDiscrete
                            lumPdf = (cst ? const_pdf_direct(rd, P.refN) : vp.pdf) *
                                     (S.emitters[S.env_emitter].weight * S.em_norm);
                        const float a2 = P.bsdfPdf * P.bsdfPdf, b2 = lumPdf * lumPdf;
                        P.L = add(P.L, mul(mulv(P.thr, value), a2 / (a2 + b2)));
                    }
                }
                // volpath.cpp:326-336: the miss still passes the RR step before the loop ends
                if (L.integrator == MTSG_INTEGRATOR_VOLPATH && P.depth++ >= L.rr_depth) (void)next1d(SC, smp);
                endPath = true;   // !its.isValid(): break after the environment term
            } else if constexpr (HITK != 2) {
                auto &sh = hs.shapes[P.its.shape];
                if (REFN && sh.emitter >= 0) {
                    const f3 value = area_Le(S, P.its, neg(rd));
                    float lumPdf = 0;
                    if (!PV_DELTA(P)) {
                        // Scene::pdfEmitterDirect (scene.cpp:949-952), area.cpp:175-181, shape.cpp:117-126;
                        // dRec after setQuery (records.inl:168-176): d = ray.d, n = its.shFrame.n, dist = its.t
                        const MtsgEmitter &e = S.emitters[sh.emitter];
                        const f3 dn = P.its.sh.n;
                        float pdf = 0.0f;
                        if (dot(rd, P.refN) >= 0 && dot(rd, dn) < 0) {
                            if (ANA && S.shapes[P.its.shape].analytic >= 0)   // dRec.ref = the previous vertex
                                pdf = ana_pdf_direct(((GAna *)S.analytic)[S.shapes[P.its.shape].analytic], ro, rd,
                                                     dn, P.its.t);
                            else
                                pdf = e.inv_area * (P.its.t * P.its.t) / absdot(rd, dn);
                        }
                        lumPdf = pdf * (e.weight * S.em_norm);
                    }
                    const float a2 = P.bsdfPdf * P.bsdfPdf, b2 = lumPdf * lumPdf;
                    P.L = add(P.L, mul(mulv(P.thr, value), a2 / (a2 + b2)));
                }
                P.emitted = false;
                if (P.depth++ >= L.rr_depth) {
                    const float q = smin(smaxc(P.thr) * P.eta * P.eta, (float)0.95f);
                    if (next1d(SC, smp) >= q) endPath = true;
                    else P.thr = divs(P.thr, q);
                }
                if (smp.err) endPath = true;
                vertex = !endPath;
            }
        }
        st.haveRay = false;
        st.primary = false;

        if (vertex) {
            // loop head of Li() (path.cpp:135-200); rd is the incoming ray direction
            if (!(P.depth <= L.max_depth || L.max_depth < 0)) {
                endPath = true;
            } else if (HITK == 2 || !P.its.valid) {
                // camera ray missed: scene->evalEnvironment(ray) with the sensor's ray
                // differentials (path.cpp:136-142, perspective.cpp:271-298, integrator.cpp:181)
                if (ENV && P.emitted && (!L.hide_emitters || P.scattered)) {
                    const MtsgCamera &cam = S.cam;
                    const f3 nearP = xf_point(cam.sample_to_camera, mk(sx * cam.inv_res_x, sy * cam.inv_res_y, 0.0f));
                    const f3 rxl = normalize(add(nearP, ld3(cam.dx))), ryl = normalize(add(nearP, ld3(cam.dy)));
                    const float *W = cam.to_world;
                    f3 rxd = mk(W[0] * rxl.x + W[1] * rxl.y + W[2] * rxl.z, W[4] * rxl.x + W[5] * rxl.y + W[6] * rxl.z,
                                W[8] * rxl.x + W[9] * rxl.y + W[10] * rxl.z);
                    f3 ryd = mk(W[0] * ryl.x + W[1] * ryl.y + W[2] * ryl.z, W[4] * ryl.x + W[5] * ryl.y + W[6] * ryl.z,
                                W[8] * ryl.x + W[9] * ryl.y + W[10] * ryl.z);
                    rxd = add(rd, mul(sub(rxd, rd), L.diff_scale));   // RayDifferential::scaleDifferential (ray.h:163-168)
                    ryd = add(rd, mul(sub(ryd, rd), L.diff_scale));
                    glb_env *E = (glb_env *)S.env;
                    if (REFN && E->constant) {   // ConstantBackgroundEmitter::evalEnvironment (constant.cpp:241-243)
                        P.L = add(P.L, mulv(P.thr, mk(E->radiance[0], E->radiance[1], E->radiance[2])));
                    } else {
                    P.L = add(P.L, mulv(P.thr, env_eval_diff(E, rd, rxd, ryd)));
                    }
                }
                endPath = true;
            } else if constexpr (HITK != 2) {
                auto &sh = hs.shapes[P.its.shape];
                GBsdf &bsdf = ((GBsdf *)S.bsdfs)[sh.bsdf];
                // roughplastic's per-vertex transmittance terms (dbsdf.h rp_pre), formed
                // at the first query of this vertex and reused for the same BSDF and wi
                RpPre rpc = {0.0f, 0.0f, 0.0f};
                GBsdf *rpB = nullptr;
                float rpZ = 0.0f;
                auto rpPre = [&](GBsdf *qb, f3 qwi) -> RpPre {
                    if constexpr (EXT && (KIND < 0 || KIND == BSDF_ROUGHPLASTIC)) {
                        if ((KIND == BSDF_ROUGHPLASTIC || qb->type == BSDF_ROUGHPLASTIC) &&
                            !(rpB == qb && __float_as_uint(rpZ) == __float_as_uint(qwi.z))) {
                            rpc = rp_pre<BSF>(*qb, (glb_f32 *)S.rtrans, qwi, P.its.u, P.its.v);
                            rpB = qb;
                            rpZ = qwi.z;
                        }
                    }
                    return rpc;
                };
                if (REFN && sh.emitter >= 0 && P.emitted && (!L.hide_emitters || P.scattered))
                    P.L = add(P.L, mulv(P.thr, area_Le(S, P.its, neg(rd))));
                // volpath.cpp:214-221 stops only for a strictly negative -dot(geoN, d) * cosTheta(wi)
                const float snp = dot(rd, P.its.geoN) * P.its.wi.z;
                if ((P.depth >= L.max_depth && L.max_depth > 0) ||
                    (!NOSTRICT && L.strict_normals && (L.integrator == MTSG_INTEGRATOR_VOLPATH ? snp > 0 : snp >= 0))) {
                    endPath = true;
                } else {
                    if constexpr (REFN)
                        P.refN = (bsdf.flags & (MTSG_F_TRANSMISSION | MTSG_F_BACK)) == 0 ? P.its.sh.n : mk(0, 0, 0);
                    if (bsdf.flags & MTSG_F_SMOOTH) {
                        // Scene::sampleEmitterDirect (scene.cpp:828-852)
                        float ex, ey;
                        next2d(SC, L.resolution, smp, px, py, ex, ey);
                        float emPdf;
                        const uint32_t ei = dd_sample_reuse(S.em_cdf, S.num_emitters, ex, &emPdf);
                        if (STATS) c.nee++;
                        const MtsgEmitter &e = S.emitters[ei];
                        f3 value = mk(0, 0, 0), dd = mk(0, 0, 1);
                        float pdf = 0.0f, dist = 0.0f;
                        f3 vlp = mk(0, 0, 0);   // dRec.p where it does not define dRec.d exactly (volpath)
                        bool vrecomp = false;
                        if (ENV && (!REFN || e.type != MTSG_EMITTER_AREA)) {
                            glb_env *E = (glb_env *)S.env;
                            const EnvSample es = (REFN && E->constant) ? const_sample_direct(E, P.its.p, P.refN, ex, ey)
                                                                       : env_sample_direct(E, P.its.p, ex, ey);
                            value = es.value; dd = es.d; dist = es.dist; pdf = es.pdf;
                            vlp = add(P.its.p, mul(dd, dist));   // dRec.p = ray(farT) (envmap.cpp:536, constant.cpp:254)
                            vrecomp = true;
                        } else if constexpr (!REFN) {
                        } else if (ANA && S.shapes[e.shape].analytic >= 0) {
                            const AnaSample as =
                                ana_sample_direct(((GAna *)S.analytic)[S.shapes[e.shape].analytic], P.its.p, ex, ey);
                            dd = as.d; dist = as.dist; pdf = as.pdf;
                            vlp = as.p; vrecomp = true;
                            // AreaLight::sampleDirect (area.cpp:158-173)
                            if (dot(dd, P.refN) >= 0 && dot(dd, as.n) < 0 && pdf != 0) value = divs(ld3(e.radiance), pdf);
                            else pdf = 0.0f;
                        } else {
                        // TriMesh::samplePosition (trimesh.cpp:412-425), Triangle::sample (triangle.cpp:24-58)
                        float py2 = ey;
                        const uint32_t lt = dd_sample_reuse(S.area_cdf + e.cdf_offset, e.tri_count, py2, nullptr);
                        const uint32_t prim = e.tri_first + lt;
                        const uint4 pv = make_uint4(hs.pv[4 * prim], hs.pv[4 * prim + 1], hs.pv[4 * prim + 2],
                                                    hs.pv[4 * prim + 3]);
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
                        // Shape::sampleDirect (shape.cpp:102-115)
                        dd = sub(lp, P.its.p);
                        const float distSquared = len2(dd);
                        dist = dsqrt(distSquared);
                        dd = divs(dd, dist);
                        const float dp = absdot(dd, ln);
                        pdf *= dp != 0 ? (distSquared / dp) : 0.0f;
                        // AreaLight::sampleDirect (area.cpp:158-173)
                        if (dot(dd, P.refN) >= 0 && dot(dd, ln) < 0 && pdf != 0) value = divs(ld3(e.radiance), pdf);
                        else pdf = 0.0f;
                        }
                        if (pdf != 0) {
                            // the NEE estimate but for visibility (path.cpp:176-199)
                            const float dpdf = pdf * emPdf;
                            value = divs(value, emPdf);
                            f3 c = mk(0, 0, 0);
                            if (!is_zero(value)) {
                                const f3 wo = to_local(P.its.sh, dd);
                                // twosided (twosided.cpp:105-131): the nested BSDF of the side wi is on
                                f3 qwi = P.its.wi, qwo = wo;
                                GBsdf *qb = &bsdf;
                                if constexpr (EXT && KIND < 0) {
                                    if (bsdf.type == BSDF_TWOSIDED) {
                                        const bool flip = !(qwi.z > 0);
                                        qb = &((GBsdf *)S.bsdfs)[bsdf.nested[flip ? 1 : 0]];
                                        if (flip) { qwi.z = -qwi.z; qwo.z = -qwo.z; }
                                    }
                                }
                                const EvalPdf ep = bsdf_eval_pdf_k<BSF, KIND>(*qb, (glb_f32 *)S.rtrans, qwi, qwo,
                                                                              P.its.u, P.its.v, rpPre(qb, qwi));
                                const f3 bsdfVal = ep.val;
                                if (!is_zero(bsdfVal) && (NOSTRICT || !L.strict_normals || dot(P.its.geoN, dd) * wo.z > 0)) {
                                    const float bsdfPdf = ep.pdf;
                                    const float pa = dpdf * dpdf, pb = bsdfPdf * bsdfPdf;
                                    const float weight = pa / (pa + pb);
                                    c = mul(mulv(mulv(P.thr, value), bsdfVal), weight);
                                }
                            }
                            // Ray(dRec.ref, dRec.d, Epsilon, dRec.dist*(1-ShadowEpsilon)) (scene.cpp:839-840)
                            P.neeC = c;
                            sd = dd;
                            smaxt = dist * (1 - D_SHADOW_EPSILON);
                            if (L.integrator == MTSG_INTEGRATOR_VOLPATH && vrecomp) {
                                // Scene::evalTransmittance (scene.cpp:619-679, 890): the segment to dRec.p,
                                // re-normalised; every supported emitter is EOnSurface (envmap.cpp:107,
                                // constant.cpp:48, area lights), so the shadow epsilon always applies
                                const f3 v = sub(vlp, P.its.p);
                                const float rem = dsqrt(len2(v));
                                sd = divs(v, rem);
                                smaxt = rem * (1 - D_SHADOW_EPSILON);
                            }
                            st.haveShadow = true;
                        }
                    }
                    // BSDF sampling (path.cpp:206-226)
                    float bx2, by2;
                    next2d(SC, L.resolution, smp, px, py, bx2, by2);
                    float u1d = 0.0f;
                    if (KIND >= 0 ? KIND == BSDF_ROUGHDIELECTRIC : bsdf.type == BSDF_ROUGHDIELECTRIC)
                        u1d = next1d(SC, smp);   // roughdielectric.cpp:554
                    BSample bs;
                    if (EXT && KIND < 0 && bsdf.type == BSDF_TWOSIDED) {
                        // TwoSidedBRDF::sample(bRec, pdf, sample) (twosided.cpp:151-172)
                        const bool flip = P.its.wi.z < 0;
                        f3 qwi = P.its.wi;
                        if (flip) qwi.z = -qwi.z;
                        GBsdf *nb = &((GBsdf *)S.bsdfs)[bsdf.nested[flip ? 1 : 0]];
                        bs = bsdf_sample_fast<BSF>(*nb, (glb_f32 *)S.rtrans, qwi, bx2, by2, u1d, P.its.u, P.its.v,
                                                   rpPre(nb, qwi));
                        if (flip && !is_zero(bs.weight) && bs.pdf != 0) bs.wo.z = -bs.wo.z;
                    } else {
                        bs = bsdf_sample_k<BSF, KIND>(bsdf, (glb_f32 *)S.rtrans, P.its.wi, bx2, by2, u1d, P.its.u,
                                                      P.its.v, rpPre(&bsdf, P.its.wi));
                    }
                    if (!is_zero(bs.weight) && !smp.err) {
                        P.scattered |= bs.sampledType != MTSG_F_NULL;
                        const f3 wo = to_world(P.its.sh, bs.wo);
                        if (NOSTRICT || !L.strict_normals || dot(P.its.geoN, wo) * bs.wo.z > 0) {
                            // throughput *= bsdfWeight; eta *= bRec.eta (path.cpp:256-257): the same
                            // products as after the hit, formed now so they need not stay live
                            P.thr = mulv(P.thr, bs.weight);
                            P.bsdfPdf = bs.pdf;
                            P.eta *= bs.eta;
                            PV_SET_DELTA(P, bs.sampledType);
                            // Ray(its.p, wo, ray.time): mint = Epsilon, maxt = inf (origin P.its.p)
                            rd = wo;
                            rmint = D_EPSILON;
                            rmaxt = INFINITY;
                            st.haveRay = true;
                        }
                    }
                    // no next ray: the path ends once the pending shadow ray is resolved
                    if (!st.haveRay && !st.haveShadow) endPath = true;
                }
            }
        }
        return endPath;
    }

    // block->put(samplePos, spec, alpha) (integrator.cpp:184) and the sample's records
    // LANE_COUNTS: count the sample into c (the wavefront engine); the megakernel
    // counts finished samples per wave instead (WaveCounters)
    // hold (megakernel, box filter, sample runs of 2 or more): the record of sample 2k is
    // kept in *hold and stored with sample 2k + 1's, which the same lane renders next, as
    // one whole 32 B sector (film_slot)
    template <bool LANE_COUNTS = true>
    __device__ __forceinline__ void finish(PathState &st, float4 *hold = nullptr) const {
        PathVars &P = st.P;
        SamplerState &smp = st.smp;
        const uint32_t j = smp.sampleIndex, pix = st.pix;
        int px = 0, py = 0;
        pixel_of(L, pix, px, py);
        const float sx = st.sx, sy = st.sy;
        // block->put(samplePos, spec, alpha) (integrator.cpp:184): the own-pixel
        // splat is stored as {L.rgb, w} (alpha in {0,1} in the sign bit of w) and
        // film_reduce re-forms weight * value[k] -- the same products
        const float alpha = P.alpha ? 1.0f : 0.0f;
        const float val[5] = {P.L.x, P.L.y, P.L.z, alpha, 1.0f};
        const uint32_t jj = j - L.j0;
        if (hold && !L.gather && L.round_shift != 0 && MTSG_SPLAT_PAIR) {
            float ownW = 0.0f;
            float4 rec4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (film_splat(L, px, py, sx, sy, val, ownW)) rec4 = make_float4(val[0], val[1], val[2], P.alpha ? ownW : -ownW);
            float4 *c4 = reinterpret_cast<float4 *>(L.contrib);
            const size_t slot = film_slot(L, jj, pix);
            if ((jj & 1u) == 0 && jj + 1 < L.chunk_spp) {
                *hold = rec4;
            } else if (jj & 1u) {
                c4[slot - 1] = *hold;
                c4[slot] = rec4;
            } else {
                c4[slot] = rec4;
            }
        } else {
            film_record(L, film_slot(L, jj, pix), px, py, sx, sy, val, P.alpha);
        }
        if (INSTR && L.samples) {
            const uint32_t pixIdx = (uint32_t)(py - (int)L.y0) * L.width + (uint32_t)(px - (int)L.x0);
            float *rec = L.samples + ((size_t)pixIdx * L.spp + j) * 8;
            rec[0] = P.L.x; rec[1] = P.L.y; rec[2] = P.L.z; rec[3] = alpha;
            rec[4] = sx; rec[5] = sy; rec[6] = (float)P.depth; rec[7] = smp.err ? 1.0f : 0.0f;
        }
        if (STATS) c.sobol += (unsigned long long)smp.dim * (smp.dim < L.lds_dims ? 0 : L.nibbles);
        if (!LANE_COUNTS) {
            st.active = false;
            st.haveRay = st.haveShadow = false;
            return;
        }
        c.len += (uint32_t)P.depth;
        c.samples++;
        if (smp.err) c.err++;
        // a lane's rays and shadow rays never exceed its path lengths plus samples:
        // flush the 32-bit counts well before any of them can wrap
        if (__builtin_expect((c.len | c.samples) >= 0x40000000u, 0)) {
            atomicAdd(L.counters + 0, (unsigned long long)c.samples);
            atomicAdd(L.counters + 1, (unsigned long long)c.rays);
            atomicAdd(L.counters + 2, (unsigned long long)c.shadow);
            atomicAdd(L.counters + 3, (unsigned long long)c.len);
            c.samples = c.rays = c.shadow = c.len = 0;
        }
        st.active = false;
        st.haveRay = st.haveShadow = false;
    }
};

// the megakernel's always-on counts, summed per wave (uniform: SGPRs, not a VGPR
// per lane across the whole bounce loop)
struct WaveCounters {
    uint32_t rays, shadow, len, samples, err;
};
__device__ __forceinline__ uint32_t wave_count(bool b) { return (uint32_t)__popcll(__ballot(b)); }
__device__ __forceinline__ void wave_counters_flush(const MtsgLaunch &L, const WaveCounters &w) {
    if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0) {
        atomicAdd(L.counters + 0, (unsigned long long)w.samples);
        atomicAdd(L.counters + 1, (unsigned long long)w.rays);
        atomicAdd(L.counters + 2, (unsigned long long)w.shadow);
        atomicAdd(L.counters + 3, (unsigned long long)w.len);
        if (w.err) atomicAdd(L.counters + 6, (unsigned long long)w.err);
    }
}

template <bool STATS>
__device__ __forceinline__ void path_counters_flush(const MtsgLaunch &L, const PathCounters &c) {
    atomicAdd(L.counters + 0, (unsigned long long)c.samples);
    atomicAdd(L.counters + 1, (unsigned long long)c.rays);
    atomicAdd(L.counters + 2, (unsigned long long)c.shadow);
    atomicAdd(L.counters + 3, (unsigned long long)c.len);
    if (STATS) {
        atomicAdd(L.counters + 4, c.nodes);
        atomicAdd(L.counters + 5, c.tests);
        atomicAdd(L.counters + 7, c.hits);
        atomicAdd(L.counters + 9, c.nee);
        atomicAdd(L.counters + 10, c.sobol);
    }
    if (c.err) atomicAdd(L.counters + 6, (unsigned long long)c.err);
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
