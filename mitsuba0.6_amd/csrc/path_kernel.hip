// path_kernel.hip -- the MI355X (gfx950) hot path of Mitsuba 0.6's `path`
// integrator: SamplingIntegrator::renderBlock's per-sample loop
// (src/librender/integrator.cpp:140-188) around MIPathTracer::Li
// (src/integrators/path/path.cpp:119-294), as one persistent HIP kernel.
//
// Execution model:
//  * work items are (sample j, pixel p) pairs, j-major, pixels in 8x8 tiles;
//    lane g of the persistent grid takes items g, g + lanes, g + 2 lanes, ...
//    (static striding: no queue, no tail of long per-pixel tasks);
//  * a lane whose path ends starts its next item immediately (regeneration);
//  * each loop iteration traces exactly one ray per active lane (primary,
//    shadow or extension) through one shared BVH2 traversal, then advances that
//    lane's path state machine to its next ray;
//  * the own-pixel splat of every sample is stored to HBM ([5][spp][pixels])
//    and a second kernel sums each pixel in sample order -- the reference's
//    ImageBlock accumulation order, bit for bit; splats into other pixels (box
//    filter edges, gaussian) go to a spill film with float atomics;
//  * LDS holds the Sobol direction numbers of the first dimensions as 4-bit
//    lookup tables (8 independent reads per 32-bit sample instead of up to 32
//    dependent ones) and the lane-strided traversal stacks.
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
typedef __attribute__((address_space(1))) const MtsgQNode glb_qnode;

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
#ifdef MTSG_NO_XCD_REMAP
    return b;
#else
    return (xcds > 1u && nb % xcds == 0) ? (b % xcds) * (nb / xcds) + b / xcds : b;
#endif
}
__device__ __forceinline__ uint32_t xcd_block(uint32_t xcds) { return xcd_remap(blockIdx.x, gridDim.x, xcds); }

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
    Frame sh;
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
#ifndef MTSG_TRAV_IFIF
// Speculative while-while traversal (Aila & Laine 2009): a lane that reaches a
// leaf parks it and keeps descending until every lane of the wave holds a
// leaf; then all lanes test their parked leaves together.  Same closest hit
// (tie rule included) as a plain depth-first traversal.
// LDSK > 0: the first LDSK stack entries live in LDS, deeper ones in a per-lane
// global array `ovf` ({node, distance} pairs): a short LDS stack keeps the
// traversal kernel's LDS per lane small (wf_trace occupancy); 0: all in LDS
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
                if (ANY || dist_up16(stkD[sp * BLOCK]) <= bt) return stkN[sp * BLOCK];
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
            if constexpr (std::is_same<NodeT, glb_qnode>::value) {
                // 4-wide node: slab-test the four child boxes, visit the nearest
                // hit child next and push the other hit ones farthest first
                NodeT *q = nodesArr + node;
                const vu4 B0 = *reinterpret_cast<glb_u4 *>(&q->box[0]);
                const vu4 B1 = *reinterpret_cast<glb_u4 *>(&q->box[4]);
                const vu4 B2 = *reinterpret_cast<glb_u4 *>(&q->box[8]);
                const vi4 C = *reinterpret_cast<glb_i4 *>(&q->child[0]);
                auto slab = [&](uint32_t wx, uint32_t wy, uint32_t wz, int ch) -> float {
                    const float t0x = __builtin_fmaf(half_lo(wx), ix, -ox), t1x = __builtin_fmaf(half_hi(wx), ix, -ox);
                    const float t0y = __builtin_fmaf(half_lo(wy), iy, -oy), t1y = __builtin_fmaf(half_hi(wy), iy, -oy);
                    const float t0z = __builtin_fmaf(half_lo(wz), iz, -oz), t1z = __builtin_fmaf(half_hi(wz), iz, -oz);
                    const float nn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), mint));
                    const float ff = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), bt));
                    return (ch != 0 && nn <= ff) ? nn : INFINITY;
                };
                float d0 = slab(B0.x, B0.y, B0.z, C.x), d1 = slab(B0.w, B1.x, B1.y, C.y);
                float d2 = slab(B1.z, B1.w, B2.x, C.z), d3 = slab(B2.y, B2.z, B2.w, C.w);
                int k0 = C.x, k1 = C.y, k2 = C.z, k3 = C.w;
                auto cx = [](float &da, int &ka, float &db, int &kb) {
                    const bool sw = db < da;
                    const float td = sw ? db : da, tk_d = sw ? da : db;
                    const int tk = sw ? kb : ka, tk2 = sw ? ka : kb;
                    da = td; db = tk_d; ka = tk; kb = tk2;
                };
#ifdef MTSG_BVH4_NEAREST   // only the nearest hit child first; the others pushed in slot order
                cx(d0, k0, d1, k1); cx(d0, k0, d2, k2); cx(d0, k0, d3, k3);
#else
                cx(d0, k0, d1, k1); cx(d2, k2, d3, k3); cx(d0, k0, d2, k2); cx(d1, k1, d3, k3); cx(d1, k1, d2, k2);
#endif
                auto push = [&](int ref, float t) {
                    if (LDSK == 0 || sp < LDSK) {
                        stkN[sp * BLOCK] = ref;
                        stkD[sp * BLOCK] = dist_down16(t);
                    } else {
                        ovf[sp - LDSK] = make_uint2((uint32_t)ref, dist_down16(t));
                    }
                    ++sp;
                };
                if (d3 < INFINITY) push(k3, d3);
                if (d2 < INFINITY) push(k2, d2);
                if (d1 < INFINITY) push(k1, d1);
                node = d0 < INFINITY ? k0 : pop();
            } else {
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
#ifdef MTSG_LEAF_PREFETCH
            // the next record is loaded while the current one is tested
            vf4 p0 = {}, p1 = {}, p2 = {};
            if (count) {
                TriT *tr = trisArr + first;
                p0 = *reinterpret_cast<F4 *>(&tr->k);
                p1 = *reinterpret_cast<F4 *>(&tr->a_u);
                p2 = *reinterpret_cast<F4 *>(&tr->c_nu);
            }
#endif
            for (uint32_t i = first; i < end; ++i) {
                if (STATS) tests++;
#ifdef MTSG_LEAF_PREFETCH
                const vf4 q0 = p0, q1 = p1, q2 = p2;
                {
                    TriT *tn = trisArr + (i + 1 < end ? i + 1 : i);
                    p0 = *reinterpret_cast<F4 *>(&tn->k);
                    p1 = *reinterpret_cast<F4 *>(&tn->a_u);
                    p2 = *reinterpret_cast<F4 *>(&tn->c_nu);
                }
#else
                TriT *tr = trisArr + i;
                const vf4 q0 = *reinterpret_cast<F4 *>(&tr->k);
                const vf4 q1 = *reinterpret_cast<F4 *>(&tr->a_u);
                const vf4 q2 = *reinterpret_cast<F4 *>(&tr->c_nu);
#endif
                const uint32_t k = __float_as_uint(q0.x);
                // TriAccel::rayIntersect (triaccel.h:92-160)
                float o_u, o_v, o_k, d_u, d_v, d_k;
#ifdef MTSG_LEAF_SELECT
                if (!ANA || k < 3) {   // triangle: the projection axes as selects, no branches
                    const bool k0 = k == 0, k1 = k == 1;
                    o_u = k0 ? o.y : k1 ? o.z : o.x; o_v = k0 ? o.z : k1 ? o.x : o.y; o_k = k0 ? o.x : k1 ? o.y : o.z;
                    d_u = k0 ? d.y : k1 ? d.z : d.x; d_v = k0 ? d.z : k1 ? d.x : d.y; d_k = k0 ? d.x : k1 ? d.y : d.z;
                }
#else
                if (k == 0) { o_u = o.y; o_v = o.z; o_k = o.x; d_u = d.y; d_v = d.z; d_k = d.x; }
                else if (k == 1) { o_u = o.z; o_v = o.x; o_k = o.y; d_u = d.z; d_v = d.x; d_k = d.y; }
                else if (k == 2) { o_u = o.x; o_v = o.y; o_k = o.z; d_u = d.x; d_v = d.y; d_k = d.z; }
#endif
                else {
                    if constexpr (ANA) {
                        // analytic primitive (skdtree.h:280-290: Shape::rayIntersect on [mint, maxt])
                        float at, alx, aly;
                        if (k == MTSG_K_ANALYTIC &&
                            ana_intersect<ANY>(((GAna *)anaArr)[__float_as_uint(q0.y)], o, d, mint, bt, at, alx, aly)) {
#ifdef MTSG_ANYHIT_XC_SLOT   // diagnostic build: which test accepted the shadow ray
                            if (ANY) { bestSlot = i | 0x80000000u; bu = at; bv = alx; bt = aly; }
#endif
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
#ifdef MTSG_ANYHIT_XC_SLOT
                    if (ANY) { bestSlot = i; bu = t; bv = u; bt = v; }
#endif
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
#else
template <bool ANY, bool STATS, bool ANA = false, typename NodeT, typename TriT>
__device__ __forceinline__ bool traverse(NodeT *nodesArr, TriT *trisArr, f3 o, f3 d, float mint, float maxt,
                                         lds_stk_n *stkN, lds_stk_d *stkD, uint32_t &bestSlot, float &bu, float &bv,
                                         float &bt, unsigned long long &nodes, unsigned long long &tests,
                                         const MtsgAnalytic *anaArr = nullptr) {
    static_assert(!ANA, "the if-if traversal ablation has no analytic primitives");
    typedef typename std::conditional<std::is_same<NodeT, lds_node>::value, lds_f4, glb_f4>::type F4;
    typedef typename std::conditional<std::is_same<NodeT, lds_node>::value, lds_i4, glb_i4>::type I4;
    // reciprocal direction for the (conservative) node tests; exact zeros use
    // +-1e30 so that 0 * inf never produces NaN (TriAccel uses the exact ray)
    const float ix = (d.x == 0.0f) ? copysignf(1e30f, d.x) : 1.0f / d.x;
    const float iy = (d.y == 0.0f) ? copysignf(1e30f, d.y) : 1.0f / d.y;
    const float iz = (d.z == 0.0f) ? copysignf(1e30f, d.z) : 1.0f / d.z;
    const float ox = o.x * ix, oy = o.y * iy, oz = o.z * iz;
    bool found = false;
    uint32_t bestPrim = 0;
    bt = maxt;
    int sp = 0;
    int node = 0;
    while (true) {
        if (node >= 0) {
            if (STATS) nodes++;
            NodeT *n = nodesArr + node;
            const vf4 a = *reinterpret_cast<F4 *>(&n->c0lox);
            const vf4 b = *reinterpret_cast<F4 *>(&n->c1lox);
            const vf4 c = *reinterpret_cast<F4 *>(&n->c0loz);
            const vi4 e = *reinterpret_cast<I4 *>(&n->c0);
            // slab tests; node boxes are conservatively inflated on the host, so the
            // fused (o*inv precomputed) form needs no bit-exactness
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
                int nearC = e.x, farC = e.y;
                float farT = n1;
                if (n1 < n0) { nearC = e.y; farC = e.x; farT = n0; }
                stkN[sp * BLOCK] = farC;
                stkD[sp * BLOCK] = dist_down16(farT);
                ++sp;
                node = nearC;
                continue;
            } else if (h0) {
                node = e.x;
                continue;
            } else if (h1) {
                node = e.y;
                continue;
            }
        } else {
            const uint32_t ref = (uint32_t)(~node);
            const uint32_t first = ref >> 4, count = ref & 15u;
            for (uint32_t i = first; i < first + count; ++i) {
                if (STATS) tests++;
                TriT *tr = trisArr + i;
                const vf4 q0 = *reinterpret_cast<F4 *>(&tr->k);
                const vf4 q1 = *reinterpret_cast<F4 *>(&tr->a_u);
                const vf4 q2 = *reinterpret_cast<F4 *>(&tr->c_nu);
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
#ifdef MTSG_ANYHIT_XC_SLOT   // diagnostic build: which test accepted the shadow ray
                            if (ANY) { bestSlot = i | 0x80000000u; bu = at; bv = alx; bt = aly; }
#endif
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
#ifdef MTSG_ANYHIT_XC_SLOT
                    if (ANY) { bestSlot = i; bu = t; bv = u; bt = v; }
#endif
                    if (ANY) return true;
                    const uint32_t prim = __float_as_uint(q2.z);
                    // ties (t == bt): the larger primitive index wins
                    if (!found || t < bt || prim > bestPrim) {
                        found = true; bestPrim = prim; bestSlot = i; bt = t; bu = u; bv = v;
                    }
                }
            }
        }
        // pop, skipping subtrees that start beyond the closest hit found so far
        bool popped = false;
        while (sp > 0) {
            --sp;
            if (ANY || dist_up16(stkD[sp * BLOCK]) <= bt) { node = stkN[sp * BLOCK]; popped = true; break; }
        }
        if (!popped) break;
    }
    return found;
}

#endif

// A bounce's shadow ray and closest-hit ray through the BVH together (the
// BVH analogue of scan_pair): one traversal whose stack entries carry a 2-bit
// mask of the rays that still need the subtree (bit 0 closest, bit 1 shadow,
// in the low bits of the bf16 entry distance -- truncating it further keeps it
// a lower bound), so the nodes both rays visit are fetched and tested once and
// the two chains of dependent node loads overlap.  Results equal the separate
// traversals': the closest hit is the smallest t (ties: larger primitive
// index) over every triangle whose leaf the closest ray reaches, culling only
// by the closest ray's own entry distance; the shadow ray's answer is whether
// any triangle in its interval is hit (ShapeKDTree::rayIntersect(ray), its
// traversal stops at the first hit).  Each ray keeps its own origin.
template <bool STATS, typename NodeT, typename TriT>
__device__ __forceinline__ void tri_test(TriT *tr, f3 o, f3 d, float mint, float maxt, bool &hit, float &t_, float &u_,
                                         float &v_, uint32_t &prim) {
    typedef typename std::conditional<std::is_same<NodeT, lds_node>::value, lds_f4, glb_f4>::type F4;
    const vf4 q0 = *reinterpret_cast<F4 *>(&tr->k);
    const vf4 q1 = *reinterpret_cast<F4 *>(&tr->a_u);
    const vf4 q2 = *reinterpret_cast<F4 *>(&tr->c_nu);
    const uint32_t k = __float_as_uint(q0.x);
    hit = false;
    float o_u, o_v, o_k, d_u, d_v, d_k;   // TriAccel::rayIntersect (triaccel.h:92-160)
    if (k == 0) { o_u = o.y; o_v = o.z; o_k = o.x; d_u = d.y; d_v = d.z; d_k = d.x; }
    else if (k == 1) { o_u = o.z; o_v = o.x; o_k = o.y; d_u = d.z; d_v = d.x; d_k = d.y; }
    else { o_u = o.x; o_v = o.y; o_k = o.z; d_u = d.x; d_v = d.y; d_k = d.z; }
    const float n_u = q0.y, n_v = q0.z, n_d = q0.w;
    const float t = (n_d - o_u * n_u - o_v * n_v - o_k) / (d_u * n_u + d_v * n_v + d_k);
    if (t < mint || t > maxt) return;
    const float hu = o_u + t * d_u - q1.x;
    const float hv = o_v + t * d_v - q1.y;
    const float u = hv * q1.z + hu * q1.w;
    const float v = hu * q2.x + hv * q2.y;
    if (u >= 0 && v >= 0 && u + v <= 1.0f) {
        hit = true; t_ = t; u_ = u; v_ = v; prim = __float_as_uint(q2.z);
    }
}

template <bool STATS, typename NodeT, typename TriT>
__device__ __forceinline__ void traverse_pair(NodeT *nodesArr, TriT *trisArr, f3 oc, f3 dc, float mintC, float maxtC,
                                              bool actC, f3 os, f3 ds, float mintS, float maxtS, bool actS,
                                              lds_stk_n *stkN, lds_stk_d *stkD, bool &found, uint32_t &bestSlot,
                                              float &bu, float &bv, float &bt, bool &occluded,
                                              unsigned long long &nodes, unsigned long long &tests) {
    typedef typename std::conditional<std::is_same<NodeT, lds_node>::value, lds_f4, glb_f4>::type F4;
    typedef typename std::conditional<std::is_same<NodeT, lds_node>::value, lds_i4, glb_i4>::type I4;
    const float icx = (dc.x == 0.0f) ? copysignf(1e30f, dc.x) : 1.0f / dc.x;
    const float icy = (dc.y == 0.0f) ? copysignf(1e30f, dc.y) : 1.0f / dc.y;
    const float icz = (dc.z == 0.0f) ? copysignf(1e30f, dc.z) : 1.0f / dc.z;
    const float ocx = oc.x * icx, ocy = oc.y * icy, ocz = oc.z * icz;
    const float isx = (ds.x == 0.0f) ? copysignf(1e30f, ds.x) : 1.0f / ds.x;
    const float isy = (ds.y == 0.0f) ? copysignf(1e30f, ds.y) : 1.0f / ds.y;
    const float isz = (ds.z == 0.0f) ? copysignf(1e30f, ds.z) : 1.0f / ds.z;
    const float osx = os.x * isx, osy = os.y * isy, osz = os.z * isz;
    constexpr int DONE = 0x7fffffff;
    found = false;
    occluded = false;
    uint32_t bestPrim = 0;
    bt = maxtC;
    uint32_t live = (actC ? 1u : 0u) | (actS ? 2u : 0u);   // rays not finished
    int sp = 0;
    int node = live ? 0 : DONE, leaf = 0;
    uint32_t m = live, lm = 0;   // masks of `node` and of the parked leaf
    auto pop = [&](uint32_t &pm) -> int {
        while (sp > 0) {
            --sp;
            const uint32_t h = stkD[sp * BLOCK];
            uint32_t em = h & 3u & live;
            if ((em & 1u) && dist_up16((uint16_t)(h & ~3u)) > bt) em &= ~1u;
            if (em) { pm = em; return stkN[sp * BLOCK]; }
        }
        pm = 0;
        return DONE;
    };
    while (node != DONE || leaf < 0) {
        while ((uint32_t)node < (uint32_t)DONE) {
            m &= live;   // the shadow ray may have been answered since this entry was pushed
            if (m == 0) {
                node = pop(m);
                if (node < 0 && leaf == 0) { leaf = node; lm = m; node = pop(m); }
                if (!__any(leaf == 0)) break;
                continue;
            }
            if (STATS) nodes++;
            NodeT *n = nodesArr + node;
            const vf4 a = *reinterpret_cast<F4 *>(&n->c0lox);
            const vf4 b = *reinterpret_cast<F4 *>(&n->c1lox);
            const vf4 c = *reinterpret_cast<F4 *>(&n->c0loz);
            const vi4 e = *reinterpret_cast<I4 *>(&n->c0);
            // closest ray: slab tests (boxes conservatively inflated on the host)
            float t0x = __builtin_fmaf(a.x, icx, -ocx), t1x = __builtin_fmaf(a.y, icx, -ocx);
            float t0y = __builtin_fmaf(a.z, icy, -ocy), t1y = __builtin_fmaf(a.w, icy, -ocy);
            float t0z = __builtin_fmaf(c.x, icz, -ocz), t1z = __builtin_fmaf(c.y, icz, -ocz);
            const float n0c = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), mintC));
            const float f0c = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), bt));
            t0x = __builtin_fmaf(b.x, icx, -ocx); t1x = __builtin_fmaf(b.y, icx, -ocx);
            t0y = __builtin_fmaf(b.z, icy, -ocy); t1y = __builtin_fmaf(b.w, icy, -ocy);
            t0z = __builtin_fmaf(c.z, icz, -ocz); t1z = __builtin_fmaf(c.w, icz, -ocz);
            const float n1c = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), mintC));
            const float f1c = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), bt));
            // shadow ray
            t0x = __builtin_fmaf(a.x, isx, -osx); t1x = __builtin_fmaf(a.y, isx, -osx);
            t0y = __builtin_fmaf(a.z, isy, -osy); t1y = __builtin_fmaf(a.w, isy, -osy);
            t0z = __builtin_fmaf(c.x, isz, -osz); t1z = __builtin_fmaf(c.y, isz, -osz);
            const float n0s = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), mintS));
            const float f0s = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), maxtS));
            t0x = __builtin_fmaf(b.x, isx, -osx); t1x = __builtin_fmaf(b.y, isx, -osx);
            t0y = __builtin_fmaf(b.z, isy, -osy); t1y = __builtin_fmaf(b.w, isy, -osy);
            t0z = __builtin_fmaf(c.z, isz, -osz); t1z = __builtin_fmaf(c.w, isz, -osz);
            const float n1s = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), mintS));
            const float f1s = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), maxtS));
            const uint32_t m0 = m & ((n0c <= f0c ? 1u : 0u) | (n0s <= f0s ? 2u : 0u));
            const uint32_t m1 = m & ((n1c <= f1c ? 1u : 0u) | (n1s <= f1s ? 2u : 0u));
            if (m0 && m1) {
                // near child first by the closest ray's entry distance where it enters
                // both, else by the shadow ray's
                const bool swap = ((m0 & m1 & 1u) ? n1c < n0c : n1s < n0s);
                const int nearC = swap ? e.y : e.x, farC = swap ? e.x : e.y;
                const uint32_t nm = swap ? m1 : m0, fm = swap ? m0 : m1;
                const float farT = (fm & 1u) ? (swap ? n0c : n1c) : 0.0f;
                stkN[sp * BLOCK] = farC;
                stkD[sp * BLOCK] = (uint16_t)((dist_down16(farT) & ~3u) | fm);
                ++sp;
                node = nearC;
                m = nm;
            } else if (m0) {
                node = e.x; m = m0;
            } else if (m1) {
                node = e.y; m = m1;
            } else {
                node = pop(m);
            }
            // park the first leaf reached and keep descending
            if (node < 0 && leaf == 0) {
                leaf = node;
                lm = m;
                node = pop(m);
            }
            if (!__any(leaf == 0)) break;
        }
        // leaves
        while (leaf < 0) {
            const uint32_t ref = (uint32_t)(~leaf);
            const uint32_t first = ref >> 4, count = ref & 15u;
            lm &= live;
            for (uint32_t i = first; i < first + count && lm; ++i) {
                TriT *tr = trisArr + i;
                if (lm & 1u) {
                    if (STATS) tests++;
                    bool h; float t, u, v; uint32_t prim;
                    tri_test<STATS, NodeT>(tr, oc, dc, mintC, bt, h, t, u, v, prim);
                    // ties (t == bt): the larger primitive index wins
                    if (h && (!found || t < bt || prim > bestPrim)) {
                        found = true; bestPrim = prim; bestSlot = i; bt = t; bu = u; bv = v;
                    }
                }
                if (lm & 2u) {
                    if (STATS) tests++;
                    bool h; float t, u, v; uint32_t prim;
                    tri_test<STATS, NodeT>(tr, os, ds, mintS, maxtS, h, t, u, v, prim);
                    if (h) { occluded = true; live &= ~2u; lm &= ~2u; }
                }
            }
            leaf = 0;
            if (live == 0) { node = DONE; break; }   // no closest ray, shadow answered
            if (node < 0) {   // the next stack entry is a leaf too: take it now
                leaf = node;
                lm = m;
                node = pop(m);
            }
        }
    }
}

typedef __attribute__((address_space(4))) const MtsgTri cst_tri;
// one projection axis' records: the coordinate permutation is a compile-time
// constant, so the loop is straight-line code around the correctly rounded
// division; each record is read whole (two scalar loads) at the loop head
template <int K, bool ANY, bool STATS>
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
        const float t = (n_d - o_u * n_u - o_v * n_v - o_k) / (d_u * n_u + d_v * n_v + d_k);
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
// node loop.  The records come grouped by projection axis (L.scan_tris); the
// result -- the closest t, ties to the larger primitive index as in
// traverse() -- does not depend on the test order.  Returns the
// primitive index (not a slot) in bestPrim.
template <bool ANY, bool STATS>
__device__ __forceinline__ bool scan_tris(const MtsgLaunch &L, f3 o, f3 d, float mint, float maxt,
                                          uint32_t &bestPrim, float &bu, float &bv, float &bt,
                                          unsigned long long &tests) {
    cst_tri *tris = (cst_tri *)L.scan_tris;
    const uint32_t n0 = L.scan_n[0], n1 = L.scan_n[1], n2 = L.scan_n[2];
    bool found = false;
    bestPrim = 0;
    bt = maxt;
    if (scan_k<0, ANY, STATS>(tris, n0, o, d, mint, found, bestPrim, bu, bv, bt, tests)) return true;
    if (scan_k<1, ANY, STATS>(tris + n0, n1, o, d, mint, found, bestPrim, bu, bv, bt, tests)) return true;
    if (scan_k<2, ANY, STATS>(tris + n0 + n1, n2, o, d, mint, found, bestPrim, bu, bv, bt, tests)) return true;
    return found;
}

#ifndef MTSG_SCAN_UNROLL
#define MTSG_SCAN_UNROLL 1
#endif
// The megakernel's two rays of one bounce leave the same vertex (the NEE
// shadow ray and the next closest-hit ray, both from its.p), so a tiny scene
// tests them in one pass over the records: the TriAccel numerator is shared,
// the records are loaded once, and the pairs of products pack into
// v_pk_mul/v_pk_add.  Each ray's result is exactly that of its own scan_tris
// (an empty interval, mint = +inf and maxt = -inf, disables a ray).
template <int K, bool STATS>
__device__ __forceinline__ void scan_pair_k(cst_tri *tris, uint32_t n, f3 o, f3 ds, f3 dc, float minS, float maxS,
                                            float minC, bool &occ, bool &found, uint32_t &bestPrim, float &bu,
                                            float &bv, float &bt, unsigned long long &tests) {
    const float o_u = K == 0 ? o.y : K == 1 ? o.z : o.x, o_v = K == 0 ? o.z : K == 1 ? o.x : o.y,
                o_k = K == 0 ? o.x : K == 1 ? o.y : o.z;
    const float s_u = K == 0 ? ds.y : K == 1 ? ds.z : ds.x, s_v = K == 0 ? ds.z : K == 1 ? ds.x : ds.y,
                s_k = K == 0 ? ds.x : K == 1 ? ds.y : ds.z;
    const float c_u = K == 0 ? dc.y : K == 1 ? dc.z : dc.x, c_v = K == 0 ? dc.z : K == 1 ? dc.x : dc.y,
                c_k = K == 0 ? dc.x : K == 1 ? dc.y : dc.z;
#pragma unroll MTSG_SCAN_UNROLL
    for (uint32_t i = 0; i < n; ++i) {
        if (STATS) tests += 2;
        cst_tri &tr = tris[i];
        const float n_u = tr.n_u, n_v = tr.n_v, n_d = tr.n_d, a_u = tr.a_u, a_v = tr.a_v, b_nu = tr.b_nu,
                    b_nv = tr.b_nv, c_nu = tr.c_nu, c_nv = tr.c_nv;
        const uint32_t prim = tr.prim;
        // TriAccel::rayIntersect (triaccel.h:92-160) for both rays
        const float num = n_d - o_u * n_u - o_v * n_v - o_k;
        const float tS = num / (s_u * n_u + s_v * n_v + s_k);
        const float tC = num / (c_u * n_u + c_v * n_v + c_k);
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
    const uint32_t n0 = L.scan_n[0], n1 = L.scan_n[1], n2 = L.scan_n[2];
    occ = false;
    found = false;
    bestPrim = 0;
    bt = maxC;
    scan_pair_k<0, STATS>(tris, n0, o, ds, dc, minS, maxS, minC, occ, found, bestPrim, bu, bv, bt, tests);
    scan_pair_k<1, STATS>(tris + n0, n1, o, ds, dc, minS, maxS, minC, occ, found, bestPrim, bu, bv, bt, tests);
    scan_pair_k<2, STATS>(tris + n0 + n1, n2, o, ds, dc, minS, maxS, minC, occ, found, bestPrim, bu, bv, bt, tests);
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
// as in the reference.  TriAccel records are in global primitive order.
// The reference's stack entry holds the entry/exit point p = ray(t) with
// p[axis] = split; here an entry keeps (node, t, split, prev | axis << 8),
// 16 B instead of 24, and p[a] is re-formed as split (a == axis) or o[a] +
// d[a] * t — the same rounded product and sum the reference stores, so every
// comparison sees the same floats.  The entry and exit points the descent
// compares against are held in registers (only a push or a pop changes them),
// so a descent step reads no stack memory; the stack itself lives in scratch.
template <bool ANY>
__device__ bool kd_traverse(const uint2 *__restrict__ nodes, const uint32_t *__restrict__ indices,
                            const MtsgTri *__restrict__ tris, f3 o, f3 d, float mint, float maxt, float &bt,
                            float &bu, float &bv, uint32_t &bprim) {
    struct Ent { uint32_t node; float t; float split; uint32_t prev_axis; };
    constexpr uint32_t NONE = 0xffffffffu, NOAXIS = 3u;
    Ent stack[48];
    uint32_t mbox[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) mbox[i] = 0xffffffffu;
    const float rcp[3] = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};   // Ray::setDirection (ray.h:86-93)
    // p[a] of an entry (t, split, eaxis): the stored point of sahkdtree3.h:239-244
    auto pt = [&](float t, float split, uint32_t eaxis, int a) -> float {
        if ((uint32_t)a == eaxis) return split;
        const float oa = a == 0 ? o.x : (a == 1 ? o.y : o.z);
        const float da = a == 0 ? d.x : (a == 1 ? d.y : d.z);
        return oa + da * t;
    };
    uint32_t enPt = 0, exPt = 1;
    stack[0].t = mint;                                    // ray(mint)
    stack[0].prev_axis = NOAXIS << 8;
    stack[1].t = maxt;                                    // ray(maxt)
    stack[1].prev_axis = NOAXIS << 8;
    stack[1].node = NONE;
    float en_t = mint, en_split = 0, ex_t = maxt, ex_split = 0;
    uint32_t en_axis = NOAXIS, ex_axis = NOAXIS;
    bool found = false;
    uint32_t node = 0;
    while (node != NONE) {
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
            const uint32_t tmp = exPt++;
            if (exPt == enPt) ++exPt;
            if (exPt >= 48) return found;   // MTS_KD_MAXDEPTH bounds the tree depth; never taken
            stack[exPt].prev_axis = tmp | ((uint32_t)axis << 8);
            stack[exPt].t = distToSplit;
            stack[exPt].split = split;
            stack[exPt].node = farChild;
            ex_t = distToSplit;
            ex_split = split;
            ex_axis = (uint32_t)axis;
            n = nodes[node];
        }
        for (uint32_t e = n.x & 0x7fffffffu; e != n.y; ++e) {
            const uint32_t prim = indices[e];
#ifndef MTSG_KD_MBOX_REGS
            if (mbox[prim & 7u] == prim) continue;   // the hashed mailbox (sahkdtree3.h:138-152)
#else
            // A/B only (C3 -2%, C4 -9%): the mailbox held in registers.  A
            // primitive is only ever stored in slot prim & 7, so "slot prim & 7
            // holds prim" is "some slot holds prim": 8 compares and 8 selects
            // instead of a dynamically indexed scratch load and store
            bool seen = false;
#pragma unroll
            for (int i = 0; i < 8; ++i) seen |= mbox[i] == prim;
            if (seen) continue;
#endif
            const MtsgTri &tr = tris[prim];
            const uint32_t k = tr.k;
            float o_u, o_v, o_k, d_u, d_v, d_k;
            if (k == 0) { o_u = o.y; o_v = o.z; o_k = o.x; d_u = d.y; d_v = d.z; d_k = d.x; }
            else if (k == 1) { o_u = o.z; o_v = o.x; o_k = o.y; d_u = d.z; d_v = d.x; d_k = d.y; }
            else { o_u = o.x; o_v = o.y; o_k = o.z; d_u = d.x; d_v = d.y; d_k = d.z; }
            // TriAccel::rayIntersect (triaccel.h:92-160) on [mint, maxt]
            const float t = (tr.n_d - o_u * tr.n_u - o_v * tr.n_v - o_k) / (d_u * tr.n_u + d_v * tr.n_v + d_k);
            if (!(t < mint || t > maxt)) {
                const float hu = o_u + t * d_u - tr.a_u;
                const float hv = o_v + t * d_v - tr.a_v;
                const float u = hv * tr.b_nu + hu * tr.b_nv;
                const float v = hu * tr.c_nu + hv * tr.c_nv;
                if (u >= 0 && v >= 0 && u + v <= 1.0f) {
                    if (ANY) return true;
                    maxt = t;
                    found = true;
                    bt = t; bu = u; bv = v; bprim = prim;
                }
            }
#ifndef MTSG_KD_MBOX_REGS
            mbox[prim & 7u] = prim;
#else
#pragma unroll
            for (int i = 0; i < 8; ++i) mbox[i] = (prim & 7u) == (uint32_t)i ? prim : mbox[i];
#endif
        }
        if (ex_t > maxt) break;
        enPt = exPt;
        en_t = ex_t;
        en_split = ex_split;
        en_axis = ex_axis;
        node = stack[exPt].node;
        exPt = stack[enPt].prev_axis & 0xffu;
        const Ent e = stack[exPt];
        ex_t = e.t;
        ex_split = e.split;
        ex_axis = e.prev_axis >> 8;
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

// computeShadingFrame (util.cpp:603-608)
__device__ __forceinline__ Frame shading_frame(f3 n, f3 dpdu) {
    Frame f;
    f.n = n;
    f.s = normalize(sub(dpdu, mul(f.n, dot(f.n, dpdu))));
    f.t = cross(f.n, f.s);
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
// registers, other touched pixels to the spill film (atomics)
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
                float *dst = L.film_spill + ((size_t)gy * L.fw + gx) * 5;
#pragma unroll
                for (int k = 0; k < 5; ++k) atomicAdd(dst + k, weight * val[k]);
            }
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// the persistent path kernel
// ---------------------------------------------------------------------------
struct PathVars {
    f3 L, thr;
    float eta;
    int depth;
    bool scattered, emitted;
    float alpha;
    Hit its;          // current vertex
    f3 neeC;          // throughput*value*bsdfVal*weight, committed if the shadow ray is unoccluded
    f3 refN;          // DirectSamplingRecord::refN of the current vertex
    float bsdfPdf;
    int sampledType;
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
struct PathState {
    bool active;
    int px, py;
    uint32_t j, pix;
    float sx, sy;
    SamplerState smp;
    PathVars P;
    // rays of the next trace step: closest (camera / extension) and shadow (NEE)
    bool haveRay, primary, haveShadow;
    f3 ro, rd, sd;
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
template <bool INSTR, bool SCENE_LDS, int FEAT>
struct PathShader {
    static constexpr bool STATS = INSTR;
    static constexpr bool ENV = (FEAT & MTSG_FEAT_ENV) != 0, EXT = (FEAT & MTSG_FEAT_EXT) != 0,
                          ANA = (FEAT & MTSG_FEAT_ANA) != 0, DIFF = (FEAT & MTSG_FEAT_DIFF) != 0;
    static constexpr int BSF = FEAT & BSET_BITS;   // the variant's BSDF set (dbsdf.h BSet)
    const MtsgLaunch &L;
    const HitSrc<SCENE_LDS> &hs;
    const SobolCtx &SC;
    lds_u32 *ycolTab;
    PathCounters &c;

    // the renderBlock loop body for item `it` up to Li()'s prologue
    // (integrator.cpp:165-186, path.cpp:119-133); false for a padding pixel
    __device__ __forceinline__ bool start(PathState &st, uint64_t it) const {
        const uint32_t jj = (uint32_t)(it / L.num_pixels);
        st.pix = (uint32_t)(it - (uint64_t)jj * L.num_pixels);
        if (!pixel_of(L, st.pix, st.px, st.py)) return false;
        begin(st, jj);
        return true;
    }

    // the SFMT replay's next sample: crop pixel xy (x | y << 16), sample jj of the chunk
    __device__ __forceinline__ void start_xy(PathState &st, uint32_t xy, uint32_t jj) const {
        const uint32_t lx = xy & 0xffffu, ly = xy >> 16;   // row_stride 1: compact row = ly
        st.px = (int)(L.x0 + lx);
        st.py = (int)(L.y0 + ly);
        st.pix = ((ly >> 3) * L.tiles_x + (lx >> 3)) * 64u + (ly & 7u) * 8u + (lx & 7u);   // pixel_of's inverse
        begin(st, jj);
    }

    __device__ __forceinline__ void begin(PathState &st, uint32_t jj) const {
        const MtsgDeviceScene &S = L.scene;
        SamplerState &smp = st.smp;
        PathVars &P = st.P;
        const int px = st.px, py = st.py;
        uint32_t &j = st.j;
        float &sx = st.sx, &sy = st.sy;
        bool &haveRay = st.haveRay, &primary = st.primary, &haveShadow = st.haveShadow;
        f3 &ro = st.ro, &rd = st.rd;
        float &rmint = st.rmint, &rmaxt = st.rmaxt;
        j = L.j0 + jj;
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
        ro = mk(W[0] * 0.0f + W[1] * 0.0f + W[2] * 0.0f + W[3], W[4] * 0.0f + W[5] * 0.0f + W[6] * 0.0f + W[7],
                W[8] * 0.0f + W[9] * 0.0f + W[10] * 0.0f + W[11]);
        rd = mk(W[0] * dl.x + W[1] * dl.y + W[2] * dl.z, W[4] * dl.x + W[5] * dl.y + W[6] * dl.z,
                W[8] * dl.x + W[9] * dl.y + W[10] * dl.z);
        // Li() prologue (path.cpp:119-133)
        P.L = mk(0, 0, 0);
        P.thr = mk(1.0f, 1.0f, 1.0f);
        P.eta = 1.0f;
        P.depth = 1;
        P.scattered = false;
        P.emitted = true;
        haveRay = true;
        primary = true;
        haveShadow = false;
        st.active = true;
    }

    // the rest of one bounce, given the step's trace results: returns true
    // when the path ends (path.cpp:135-292)
    __device__ __forceinline__ bool shade(PathState &st, bool occluded, bool hit, uint32_t slot, uint32_t prim,
                                          float hu, float hv, float ht) const {
        const MtsgDeviceScene &S = L.scene;
        PathVars &P = st.P;
        SamplerState &smp = st.smp;
        const int px = st.px, py = st.py;
        const float sx = st.sx, sy = st.sy;
        bool &haveRay = st.haveRay, &primary = st.primary, &haveShadow = st.haveShadow;
        f3 &ro = st.ro, &rd = st.rd, &sd = st.sd;
        float &rmint = st.rmint, &rmaxt = st.rmaxt, &smaxt = st.smaxt;
        bool endPath = false;
        // NEE of the previous vertex (scene.cpp:838-842, path.cpp:176-199)
        if (haveShadow && !occluded) P.L = add(P.L, P.neeC);
        haveShadow = false;
        bool vertex = false;
        if (!haveRay) {
            endPath = true;   // the BSDF sample at the previous vertex failed
        } else {
            // rRec.rayIntersect / scene->rayIntersect (records.inl:117-144, path.cpp:226)
            // a miss overwrites the whole record: no field of the previous vertex stays
            // live across the next traversal except through an explicit use
            if (hit) {
                fill_hit<EXT, ANA>(S, hs, slot, prim, hu, hv, ht, ro, rd, P.its);
            } else {
                P.its = Hit{};
            }
            if (STATS && hit) c.hits++;
            if (primary) {
                P.alpha = L.has_alpha ? (P.its.valid ? 1.0f : 0.0f) : 1.0f;
                vertex = true;
            } else if (!P.its.valid) {
                // missed: the environment emitter, if any (path.cpp:233-247)
                if (ENV && !(L.hide_emitters && !P.scattered)) {
                    glb_env *E = (glb_env *)S.env;
                    const f3 value = E->constant ? mk(E->radiance[0], E->radiance[1], E->radiance[2]) : env_eval(E, rd);
                    float nT, fT;
                    // EnvironmentMap::fillDirectSamplingRecord (envmap.cpp:358-374)
                    if (env_bsphere(E, ro, rd, nT, fT) && !(nT > 0 || fT < 0)) {
                        float lumPdf = 0;
                        if (!(P.sampledType & MTSG_F_DELTA))   // pdfDirect (envmap.cpp:545-556) x pdfEmitterDiscrete
                            lumPdf = (E->constant ? const_pdf_direct(rd, P.refN) : env_pdf_direction(E, rd)) *
                                     (S.emitters[S.env_emitter].weight * S.em_norm);
                        const float a2 = P.bsdfPdf * P.bsdfPdf, b2 = lumPdf * lumPdf;
                        P.L = add(P.L, mul(mulv(P.thr, value), a2 / (a2 + b2)));
                    }
                }
                // volpath.cpp:326-336: the miss still passes the RR step before the loop ends
                if (L.integrator == MTSG_INTEGRATOR_VOLPATH && P.depth++ >= L.rr_depth) (void)next1d(SC, smp);
                endPath = true;   // !its.isValid(): break after the environment term
            } else {
                auto &sh = hs.shapes[P.its.shape];
                if (sh.emitter >= 0) {
                    const f3 value = area_Le(S, P.its, neg(rd));
                    float lumPdf = 0;
                    if (!(P.sampledType & MTSG_F_DELTA)) {
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
        haveRay = false;
        primary = false;

        if (vertex) {
            // loop head of Li() (path.cpp:135-200); rd is the incoming ray direction
            if (!(P.depth <= L.max_depth || L.max_depth < 0)) {
                endPath = true;
            } else if (!P.its.valid) {
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
                    if (E->constant) {   // ConstantBackgroundEmitter::evalEnvironment (constant.cpp:241-243)
                        P.L = add(P.L, mulv(P.thr, mk(E->radiance[0], E->radiance[1], E->radiance[2])));
                    } else {
#ifdef MTSG_ABL_BILINEAR_PRIMARY   // timing ablation only
                    P.L = add(P.L, mulv(P.thr, env_eval(E, rd)));
#else
                    P.L = add(P.L, mulv(P.thr, env_eval_diff(E, rd, rxd, ryd)));
#endif
                    }
                }
                endPath = true;
            } else {
                auto &sh = hs.shapes[P.its.shape];
                GBsdf &bsdf = ((GBsdf *)S.bsdfs)[sh.bsdf];
                // roughplastic's per-vertex transmittance terms (dbsdf.h rp_pre), formed
                // at the first query of this vertex and reused for the same BSDF and wi
                RpPre rpc = {0.0f, 0.0f};
                GBsdf *rpB = nullptr;
                float rpZ = 0.0f;
                auto rpPre = [&](GBsdf *qb, f3 qwi) -> RpPre {
                    if constexpr (EXT) {
                        if (qb->type == BSDF_ROUGHPLASTIC &&
                            !(rpB == qb && __float_as_uint(rpZ) == __float_as_uint(qwi.z))) {
                            rpc = rp_pre<BSF>(*qb, (glb_f32 *)S.rtrans, qwi, P.its.u, P.its.v);
                            rpB = qb;
                            rpZ = qwi.z;
                        }
                    }
                    return rpc;
                };
                if (sh.emitter >= 0 && P.emitted && (!L.hide_emitters || P.scattered))
                    P.L = add(P.L, mulv(P.thr, area_Le(S, P.its, neg(rd))));
                // volpath.cpp:214-221 stops only for a strictly negative -dot(geoN, d) * cosTheta(wi)
                const float snp = dot(rd, P.its.geoN) * P.its.wi.z;
                if ((P.depth >= L.max_depth && L.max_depth > 0) ||
                    (L.strict_normals && (L.integrator == MTSG_INTEGRATOR_VOLPATH ? snp > 0 : snp >= 0))) {
                    endPath = true;
                } else {
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
                        if (ENV && e.type != MTSG_EMITTER_AREA) {
#ifndef MTSG_ABL_NO_ENV_NEE   // timing ablation only
                            glb_env *E = (glb_env *)S.env;
                            const EnvSample es = E->constant ? const_sample_direct(E, P.its.p, P.refN, ex, ey)
                                                             : env_sample_direct(E, P.its.p, ex, ey);
                            value = es.value; dd = es.d; dist = es.dist; pdf = es.pdf;
                            vlp = add(P.its.p, mul(dd, dist));   // dRec.p = ray(farT) (envmap.cpp:536, constant.cpp:254)
                            vrecomp = true;
#endif
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
                                if constexpr (EXT) {
                                    if (bsdf.type == BSDF_TWOSIDED) {
                                        const bool flip = !(qwi.z > 0);
                                        qb = &((GBsdf *)S.bsdfs)[bsdf.nested[flip ? 1 : 0]];
                                        if (flip) { qwi.z = -qwi.z; qwo.z = -qwo.z; }
                                    }
                                }
                                const EvalPdf ep = bsdf_eval_pdf_fast<BSF>(*qb, (glb_f32 *)S.rtrans, qwi, qwo,
                                                                           P.its.u, P.its.v, rpPre(qb, qwi));
                                const f3 bsdfVal = ep.val;
                                if (!is_zero(bsdfVal) && (!L.strict_normals || dot(P.its.geoN, dd) * wo.z > 0)) {
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
                            haveShadow = true;
                        }
                    }
                    // BSDF sampling (path.cpp:206-226)
                    float bx2, by2;
                    next2d(SC, L.resolution, smp, px, py, bx2, by2);
                    float u1d = 0.0f;
                    if (bsdf.type == BSDF_ROUGHDIELECTRIC) u1d = next1d(SC, smp);   // roughdielectric.cpp:554
                    BSample bs;
                    if (EXT && bsdf.type == BSDF_TWOSIDED) {
                        // TwoSidedBRDF::sample(bRec, pdf, sample) (twosided.cpp:151-172)
                        const bool flip = P.its.wi.z < 0;
                        f3 qwi = P.its.wi;
                        if (flip) qwi.z = -qwi.z;
                        GBsdf *nb = &((GBsdf *)S.bsdfs)[bsdf.nested[flip ? 1 : 0]];
                        bs = bsdf_sample_fast<BSF>(*nb, (glb_f32 *)S.rtrans, qwi, bx2, by2, u1d, P.its.u, P.its.v,
                                                   rpPre(nb, qwi));
                        if (flip && !is_zero(bs.weight) && bs.pdf != 0) bs.wo.z = -bs.wo.z;
                    } else {
                        bs = bsdf_sample_fast<BSF>(bsdf, (glb_f32 *)S.rtrans, P.its.wi, bx2, by2, u1d, P.its.u, P.its.v,
                                                   rpPre(&bsdf, P.its.wi));
                    }
                    if (!is_zero(bs.weight) && !smp.err) {
                        P.scattered |= bs.sampledType != MTSG_F_NULL;
                        const f3 wo = to_world(P.its.sh, bs.wo);
                        if (!L.strict_normals || dot(P.its.geoN, wo) * bs.wo.z > 0) {
                            // throughput *= bsdfWeight; eta *= bRec.eta (path.cpp:256-257): the same
                            // products as after the hit, formed now so they need not stay live
                            P.thr = mulv(P.thr, bs.weight);
                            P.bsdfPdf = bs.pdf;
                            P.eta *= bs.eta;
                            P.sampledType = bs.sampledType;
                            ro = P.its.p;         // Ray(its.p, wo, ray.time): mint = Epsilon, maxt = inf
                            rd = wo;
                            rmint = D_EPSILON;
                            rmaxt = INFINITY;
                            haveRay = true;
                        }
                    }
                    // no next ray: the path ends once the pending shadow ray is resolved
                    if (!haveRay && !haveShadow) endPath = true;
                }
            }
        }
        return endPath;
    }

    // block->put(samplePos, spec, alpha) (integrator.cpp:184) and the sample's records
    __device__ __forceinline__ void finish(PathState &st) const {
        PathVars &P = st.P;
        SamplerState &smp = st.smp;
        const int px = st.px, py = st.py;
        const uint32_t j = st.j, pix = st.pix;
        const float sx = st.sx, sy = st.sy;
        bool &haveRay = st.haveRay, &haveShadow = st.haveShadow;
        // block->put(samplePos, spec, alpha) (integrator.cpp:184): the own-pixel
        // splat is stored as {L.rgb, w} (alpha in {0,1} in the sign bit of w) and
        // film_reduce re-forms weight * value[k] -- the same products
        const float val[5] = {P.L.x, P.L.y, P.L.z, P.alpha, 1.0f};
        float ownW = 0.0f;
        const bool valid = film_splat(L, px, py, sx, sy, val, ownW);
        float4 rec4;
        if (valid) rec4 = make_float4(P.L.x, P.L.y, P.L.z, P.alpha == 0.0f ? -ownW : ownW);
        else rec4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        reinterpret_cast<float4 *>(L.contrib)[(size_t)(j - L.j0) * L.num_pixels + pix] = rec4;
        if (INSTR && L.samples) {
            const uint32_t pixIdx = (uint32_t)(py - (int)L.y0) * L.width + (uint32_t)(px - (int)L.x0);
            float *rec = L.samples + ((size_t)pixIdx * L.spp + j) * 8;
            rec[0] = P.L.x; rec[1] = P.L.y; rec[2] = P.L.z; rec[3] = P.alpha;
            rec[4] = sx; rec[5] = sy; rec[6] = (float)P.depth; rec[7] = smp.err ? 1.0f : 0.0f;
        }
        c.len += (uint32_t)P.depth;
        c.samples++;
        if (STATS) c.sobol += (unsigned long long)smp.dim * (smp.dim < L.lds_dims ? 0 : L.nibbles);
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
        haveRay = haveShadow = false;
    }
};

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

// -DMTSG_PAIR_TRAVERSAL: a bounce's shadow and closest-hit rays through the
// BVH in one traversal (traverse_pair).  Off: its second ray's registers made
// the large-scene variants spill (C4 35 -> 127 VGPRs) and it lost C3 -9%,
// C4 -19%, C5 -4% (profiles/r03_ab_pair_C*.log)
#ifdef MTSG_PAIR_TRAVERSAL
#define PAIR_TRAVERSAL true
#else
#define PAIR_TRAVERSAL false
#endif

// The persistent megakernel: grid = CUs x resident blocks; every lane runs
// PathShader steps with both traversals inline
template <bool INSTR, bool SCENE_LDS, int FEAT, int WAVES>
__global__ __launch_bounds__(BLOCK, WAVES) void path_kernel(MtsgLaunch L) {
    constexpr bool STATS = INSTR;
    constexpr bool ANA = (FEAT & MTSG_FEAT_ANA) != 0;
#ifndef MTSG_FULL_NODES   // the BSDF-set variants (large scenes) traverse the 32 B half-box nodes
    constexpr bool HNODES = (FEAT & (MTSG_FEAT_GGX | MTSG_FEAT_NORD | MTSG_FEAT_NORC)) != 0;
#else
    constexpr bool HNODES = false;
#endif
#ifdef MTSG_BVH4   // ... or the 4-wide BVH (layout.h MtsgQNode)
    constexpr bool QNODES = HNODES;
    uint2 *qovf = (uint2 *)L.trav_ovf + (size_t)(blockIdx.x * BLOCK + threadIdx.x) * L.ovf_depth;
#else
    constexpr bool QNODES = false;
    uint2 *qovf = nullptr;
#endif
    extern __shared__ uint32_t lds[];
    const MtsgDeviceScene &S = L.scene;
    const LdsView<SCENE_LDS> V = stage_lds<SCENE_LDS>(L, lds);
    lds_node *ldsNodes = V.nodes;
    lds_tri *ldsTris = V.tris;
    lds_stk_n *stkN = (lds_stk_n *)(lds + V.stackBase) + threadIdx.x;
    lds_stk_d *stkD = (lds_stk_d *)(lds + V.stackBase + L.stack_depth * BLOCK) + threadIdx.x;
    PathCounters c = {};
    const PathShader<INSTR, SCENE_LDS, FEAT> sh{L, V.hs, V.SC, V.ycolTab, c};

    const uint64_t lanes = (uint64_t)gridDim.x * BLOCK;
    uint64_t item = L.replay ? 0 : (uint64_t)xcd_block(L.xcds) * BLOCK + threadIdx.x;
    bool done = false;
    PathState st;
    st.active = false;
    st.px = st.py = 0;
    st.j = st.pix = 0;
    st.smp.sobolIndex = 0; st.smp.sampleIndex = 0; st.smp.dim = 0; st.smp.err = false;
    st.sx = st.sy = 0;
    st.haveRay = st.primary = st.haveShadow = false;
    st.ro = mk(0, 0, 0); st.rd = mk(0, 0, 1); st.sd = mk(0, 0, 1);
    st.rmint = st.rmaxt = st.smaxt = 0;
#ifdef MTSG_MK_STAMPS
    unsigned long long mkT[4] = {0, 0, 0, 0}, mkT0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(mkT0)::"memory");
#endif

    while (true) {
        // ---- A: start the next sample
        while (!st.active && !done) {
            if (L.replay) {   // SFMT replay: this lane's unit, pixel after pixel, in order
                const uint32_t unit = blockIdx.x * BLOCK + threadIdx.x;
                if (unit >= L.units) { done = true; break; }
                const uint32_t k0 = L.unit_start[unit], n = L.unit_start[unit + 1] - k0;
                if (item >= (uint64_t)n * L.chunk_spp) { done = true; break; }
                const uint32_t k = k0 + (uint32_t)(item / L.chunk_spp), jj = (uint32_t)(item % L.chunk_spp);
                ++item;
                sh.start_xy(st, L.order[k], jj);
                break;
            }
            if (item >= L.num_items) { done = true; break; }
            const uint64_t it = item;
            item += lanes;
            sh.start(st, it);
        }
        if (__all(done)) break;
        MK_STAMP(mkT[0], mkT0);

        // ---- B: trace the shadow ray, then the closest-hit ray ---------------
        bool occluded = false;
        bool hit = false;
        uint32_t slot = 0, prim = 0;
        float hu = 0, hv = 0, ht = 0;
        if (SCENE_LDS && L.scan) {
            // tiny scene: both rays of the bounce in one pass (scan_pair); when
            // both exist they leave the same point (ro was set to its.p)
            float minS = INFINITY, maxS = -INFINITY, minC = INFINITY, maxC = -INFINITY;
            bool okS = false, okC = false;
            if (st.active && st.haveShadow) {
                c.shadow++;
#ifndef MTSG_ABL_NO_SHADOW
                if (!is_zero(st.P.neeC)) okS = ray_interval(S, st.P.its.p, st.sd, D_EPSILON, st.smaxt, true, minS, maxS);
#endif
                if (!okS) { minS = INFINITY; maxS = -INFINITY; }
            }
            if (st.active && st.haveRay) {
                c.rays++;
                okC = ray_interval(S, st.ro, st.rd, st.rmint, st.rmaxt, false, minC, maxC);
                if (!okC) { minC = INFINITY; maxC = -INFINITY; }
            }
            if (__any(okS || okC))
                scan_pair<STATS>(L, okC ? st.ro : st.P.its.p, st.sd, st.rd, minS, maxS, minC, maxC, occluded, hit,
                                 prim, hu, hv, ht, c.tests);
            hit = hit && okC;
            occluded = occluded && okS;
        } else if (PAIR_TRAVERSAL && !ANA) {
            // both rays of the bounce in one BVH traversal (traverse_pair)
            float minS = 0, maxS = 0, minC = 0, maxC = 0;
            bool okS = false, okC = false;
            if (st.active && st.haveShadow) {
                c.shadow++;
#ifndef MTSG_ABL_NO_SHADOW
                if (!is_zero(st.P.neeC)) okS = ray_interval(S, st.P.its.p, st.sd, D_EPSILON, st.smaxt, true, minS, maxS);
#endif
            }
            if (st.active && st.haveRay) {
                c.rays++;
                okC = ray_interval(S, st.ro, st.rd, st.rmint, st.rmaxt, false, minC, maxC);
            }
            if (SCENE_LDS)
                traverse_pair<STATS>(ldsNodes, ldsTris, st.ro, st.rd, minC, maxC, okC, st.P.its.p, st.sd, minS, maxS,
                                     okS, stkN, stkD, hit, slot, hu, hv, ht, occluded, c.nodes, c.tests);
            else
                traverse_pair<STATS>((glb_node *)S.nodes, (glb_tri *)S.tris, st.ro, st.rd, minC, maxC, okC,
                                     st.P.its.p, st.sd, minS, maxS, okS, stkN, stkD, hit, slot, hu, hv, ht, occluded,
                                     c.nodes, c.tests);
            if (hit) prim = SCENE_LDS ? ldsTris[slot].prim : S.tris[slot].prim;
        } else {
        if (st.active && st.haveShadow) {
            c.shadow++;
            float mint, maxt;
            // a shadow ray whose estimate is zero cannot change Li: skip its traversal
#ifdef MTSG_ABL_NO_SHADOW
            if (false) {
#else
            if (!is_zero(st.P.neeC) && ray_interval(S, st.P.its.p, st.sd, D_EPSILON, st.smaxt, true, mint, maxt)) {
#endif
                uint32_t sl; float a0, a1, a2;
                if (SCENE_LDS)
                    occluded = traverse<true, STATS, ANA>(ldsNodes, ldsTris, st.P.its.p, st.sd, mint, maxt, stkN, stkD,
                                                          sl, a0, a1, a2, c.nodes, c.tests, S.analytic);
                else if constexpr (QNODES)
                    occluded = traverse<true, STATS, ANA, MTSG_Q_LDS_STACK>((glb_qnode *)S.qnodes, (glb_tri *)S.tris,
                                                                            st.P.its.p, st.sd, mint, maxt, stkN, stkD,
                                                                            sl, a0, a1, a2, c.nodes, c.tests,
                                                                            S.analytic, qovf);
                else if constexpr (HNODES)
                    occluded = traverse<true, STATS, ANA>((glb_hnode *)S.hnodes, (glb_tri *)S.tris, st.P.its.p, st.sd,
                                                          mint, maxt, stkN, stkD, sl, a0, a1, a2, c.nodes, c.tests,
                                                          S.analytic);
                else
                    occluded = traverse<true, STATS, ANA>((glb_node *)S.nodes, (glb_tri *)S.tris, st.P.its.p, st.sd,
                                                          mint, maxt, stkN, stkD, sl, a0, a1, a2, c.nodes, c.tests,
                                                          S.analytic);
            }
        }
        // the NEE estimate is added now (as shade() would first thing), so it
        // is not live across the closest-hit traversal
        if (st.active && st.haveShadow) {
            if (!occluded) st.P.L = add(st.P.L, st.P.neeC);
            st.haveShadow = false;
        }
        MK_STAMP(mkT[1], mkT0);
        if (st.active && st.haveRay) {
            c.rays++;
            float mint, maxt;
            if (ray_interval(S, st.ro, st.rd, st.rmint, st.rmaxt, false, mint, maxt)) {
                if (SCENE_LDS)
                    hit = traverse<false, STATS, ANA>(ldsNodes, ldsTris, st.ro, st.rd, mint, maxt, stkN, stkD, slot,
                                                      hu, hv, ht, c.nodes, c.tests, S.analytic);
                else if constexpr (QNODES)
                    hit = traverse<false, STATS, ANA, MTSG_Q_LDS_STACK>((glb_qnode *)S.qnodes, (glb_tri *)S.tris,
                                                                        st.ro, st.rd, mint, maxt, stkN, stkD, slot,
                                                                        hu, hv, ht, c.nodes, c.tests, S.analytic, qovf);
                else if constexpr (HNODES)
                    hit = traverse<false, STATS, ANA>((glb_hnode *)S.hnodes, (glb_tri *)S.tris, st.ro, st.rd, mint,
                                                      maxt, stkN, stkD, slot, hu, hv, ht, c.nodes, c.tests,
                                                      S.analytic);
                else
                    hit = traverse<false, STATS, ANA>((glb_node *)S.nodes, (glb_tri *)S.tris, st.ro, st.rd, mint,
                                                      maxt, stkN, stkD, slot, hu, hv, ht, c.nodes, c.tests,
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
        if (st.active && sh.shade(st, occluded, hit, slot, prim, hu, hv, ht)) sh.finish(st);
        MK_STAMP(mkT[3], mkT0);
    }
    path_counters_flush<STATS>(L, c);
#ifdef MTSG_MK_STAMPS
    if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0)
        for (int k = 0; k < 4; ++k) atomicAdd(L.counters + 11 + k, mkT[k]);
#endif
}

// ===========================================================================
// The wavefront pipeline (north star: per-bounce SoA ray queues in HBM,
// ballot-compacted).  One bounce = wf_shade (every path slot: consume the
// previous trace results, run PathShader::shade / finish, regenerate ended
// paths from the pixel bands, append the next closest-hit and shadow rays to
// the queues with one atomic per wave) + wf_trace (both queues, dense, at the
// traversal's own occupancy).  Same PathShader code, same per-sample results
// as the megakernel; the traversals no longer run with the shading's register
// budget, and a shadow traversal no longer idles the lanes without one.
// ===========================================================================
#ifndef MTSG_WF_SHADE_WAVES
#define MTSG_WF_SHADE_WAVES 3
#endif
#ifndef MTSG_WF_TRACE_WAVES
#define MTSG_WF_TRACE_WAVES 8
#endif

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// diagnostic section stamps (guide: in-kernel stamps; shares only, never timing)
#ifdef MTSG_WF_STAMPS
#define WF_STAMP(t)                                                                                   \
    do {                                                                                              \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                                            \
    } while (0)
#else
#define WF_STAMP(t) (void)(t = 0)
#endif

// per-wave queue append: one atomic for the wave, positions in lane order
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

// path state <-> SoA slot s: [0] L, eta  [1] thr, bsdfPdf  [2] neeC, alpha
// [3] refN, sx  [4] ro, sy  [5] rd, depth  [6] pix, j, sobol index
// [7] flags | dim << 16, sampledType, closest queue pos, shadow queue pos
enum { WF_ACTIVE = 1, WF_RAY = 2, WF_PRIMARY = 4, WF_SHADOW = 8, WF_SCATTERED = 16, WF_EMITTED = 32, WF_ERR = 64 };
__device__ __forceinline__ bool wf_load(const MtsgLaunch &L, const MtsgWave &W, uint32_t s, PathState &st,
                                        uint32_t &qpos, uint32_t &spos, uint32_t &flags) {
    const size_t n = W.slots;
    // all eight vectors in flight at once (an inactive slot's are simply unused)
    const uint4 f = reinterpret_cast<const uint4 *>(W.state)[7 * n + s];
    const float4 a = W.state[s], b = W.state[n + s], c = W.state[2 * n + s], d = W.state[3 * n + s],
                 e = W.state[4 * n + s], g = W.state[5 * n + s];
    const uint4 h = reinterpret_cast<const uint4 *>(W.state)[6 * n + s];
    st.active = (f.x & WF_ACTIVE) != 0;
    qpos = f.z;
    spos = f.w;
    flags = f.x;
    if (!st.active) return false;
    st.P.L = mk(a.x, a.y, a.z); st.P.eta = a.w;
    st.P.thr = mk(b.x, b.y, b.z); st.P.bsdfPdf = b.w;
    st.P.neeC = mk(c.x, c.y, c.z); st.P.alpha = c.w;
    st.P.refN = mk(d.x, d.y, d.z); st.sx = d.w;
    st.ro = mk(e.x, e.y, e.z); st.sy = e.w;
    st.rd = mk(g.x, g.y, g.z); st.P.depth = __float_as_int(g.w);
    st.pix = h.x; st.j = h.y;
    st.smp.sobolIndex = (uint64_t)h.z | ((uint64_t)h.w << 32);
    st.smp.sampleIndex = h.y;
    st.smp.dim = f.x >> 16;
    st.smp.err = (f.x & WF_ERR) != 0;
    st.P.sampledType = (int)f.y;
    st.haveRay = (f.x & WF_RAY) != 0;
    st.primary = (f.x & WF_PRIMARY) != 0;
    st.haveShadow = (f.x & WF_SHADOW) != 0;
    st.P.scattered = (f.x & WF_SCATTERED) != 0;
    st.P.emitted = (f.x & WF_EMITTED) != 0;
    pixel_of(L, st.pix, st.px, st.py);
    return true;
}

__device__ __forceinline__ void wf_store(const MtsgWave &W, uint32_t s, const PathState &st, uint32_t qpos,
                                         uint32_t spos, uint32_t extra) {
    const size_t n = W.slots;
    uint4 f;
    f.x = extra | (st.active ? WF_ACTIVE : 0) | (st.haveRay ? WF_RAY : 0) | (st.primary ? WF_PRIMARY : 0) |
          (st.haveShadow ? WF_SHADOW : 0) | (st.P.scattered ? WF_SCATTERED : 0) | (st.P.emitted ? WF_EMITTED : 0) |
          (st.smp.err ? WF_ERR : 0) | (st.smp.dim << 16);
    f.y = (uint32_t)st.P.sampledType;
    f.z = qpos;
    f.w = spos;
    reinterpret_cast<uint4 *>(W.state)[7 * n + s] = f;
    if (!st.active) return;
    W.state[s] = make_float4(st.P.L.x, st.P.L.y, st.P.L.z, st.P.eta);
    W.state[n + s] = make_float4(st.P.thr.x, st.P.thr.y, st.P.thr.z, st.P.bsdfPdf);
    W.state[2 * n + s] = make_float4(st.P.neeC.x, st.P.neeC.y, st.P.neeC.z, st.P.alpha);
    W.state[3 * n + s] = make_float4(st.P.refN.x, st.P.refN.y, st.P.refN.z, st.sx);
    W.state[4 * n + s] = make_float4(st.ro.x, st.ro.y, st.ro.z, st.sy);
    W.state[5 * n + s] = make_float4(st.rd.x, st.rd.y, st.rd.z, __int_as_float(st.P.depth));
    reinterpret_cast<uint4 *>(W.state)[6 * n + s] =
        make_uint4(st.pix, st.j, (uint32_t)st.smp.sobolIndex, (uint32_t)(st.smp.sobolIndex >> 32));
}

// Slot s of wf_shade runs items v, v + slots, v + 2 slots, ... (v = the slot's
// XCD-aware lane index: each XCD's slots hold neighbouring pixels, as the
// megakernel's xcd_block), regenerating as soon as a path ends; flag WF_DONE
// marks a slot whose items are used up.
enum { WF_DONE = 128 };
__device__ __forceinline__ uint64_t wf_lane_index(uint32_t s, uint32_t xcds) {
    const uint32_t G = gridDim.x, t = s % BLOCK, b = (s / BLOCK) % G, r = s / (BLOCK * G);
    const uint32_t pb = xcd_remap(b, G, xcds);
    return ((uint64_t)r * G + pb) * BLOCK + t;
}

template <bool INSTR, bool SCENE_LDS, int FEAT>
__global__ __launch_bounds__(BLOCK, MTSG_WF_SHADE_WAVES) void wf_shade(MtsgLaunch L, MtsgWave W,
                                                                       unsigned long long *part) {
    extern __shared__ uint32_t lds[];
    __shared__ uint32_t red[BLOCK / 64 * 16];
    __shared__ uint32_t qcnt[2];   // this block's region: closest, shadow entries
    if (threadIdx.x < 2) qcnt[threadIdx.x] = 0;
    const MtsgDeviceScene &S = L.scene;
    const LdsView<SCENE_LDS> V = stage_lds<SCENE_LDS>(L, lds);   // ends with a barrier
    PathCounters c = {};
    const PathShader<INSTR, SCENE_LDS, FEAT> sh{L, V.hs, V.SC, V.ycolTab, c};
    const uint32_t lanes = gridDim.x * BLOCK;
    const uint32_t region = blockIdx.x * W.rounds * BLOCK;
    uint32_t live = 0;
    uint32_t stamp[5] = {0, 0, 0, 0, 0};
    for (uint32_t s = blockIdx.x * BLOCK + threadIdx.x; s < W.slots; s += lanes) {   // same trip count in a block
        unsigned long long t0, t1, t2, t3, t4, t5;
        WF_STAMP(t0);
        PathState st;
        uint32_t qpos, spos, flags;
        const bool was = wf_load(L, W, s, st, qpos, spos, flags);
        bool occluded = false, hit = false;
        uint32_t slot = 0, prim = 0;
        float hu = 0, hv = 0, ht = 0;
        if (st.active) {
            occluded = st.haveShadow && spos != MTSG_WF_NONE && W.occl[spos] != 0;
            if (st.haveRay && qpos != MTSG_WF_NONE) {
                // the hit record's 4th word: the TriAccel slot with analytic shapes (fill_hit reads
                // the slot's record), else the primitive index itself
                const float4 h = W.hit[qpos];
                const uint32_t w = __float_as_uint(h.w);
                hit = w != MTSG_WF_NONE;
                if (hit) {
                    ht = h.x; hu = h.y; hv = h.z;
                    if ((FEAT & MTSG_FEAT_ANA) != 0) { slot = w; prim = S.tris[slot].prim; }
                    else prim = w;
                }
            }
        }
        WF_STAMP(t1);
        bool ended = false;
        if (st.active && sh.shade(st, occluded, hit, slot, prim, hu, hv, ht)) { sh.finish(st); ended = true; }
        WF_STAMP(t2);
        // regeneration: the slot's next item (static stride, no atomics)
        bool done = (flags & WF_DONE) != 0;
        if (!st.active && !done) {
            uint64_t it = (ended || was) ? (uint64_t)(st.j - L.j0) * L.num_pixels + st.pix + W.slots : wf_lane_index(s, L.xcds);
            while (true) {
                if (it >= L.num_items) { done = true; break; }
                if (sh.start(st, it)) break;
                it += W.slots;   // padding pixel of a partial tile
            }
        }
        WF_STAMP(t3);
        // the next bounce's rays (megakernel step B's intervals and counts)
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
            if (ray_interval(S, st.ro, st.rd, st.rmint, st.rmaxt, false, mint, maxt)) {
                pr = true;
                r0 = make_float4(st.ro.x, st.ro.y, st.ro.z, mint);
                r1 = make_float4(st.rd.x, st.rd.y, st.rd.z, maxt);
            }
        }
        spos = wave_append(qcnt + 1, ps);
        qpos = wave_append(qcnt + 0, pr);
        if (ps) { spos += region; W.sray[2 * (size_t)spos] = s0; W.sray[2 * (size_t)spos + 1] = s1; }
        if (pr) { qpos += region; W.qray[2 * (size_t)qpos] = r0; W.qray[2 * (size_t)qpos + 1] = r1; }
        WF_STAMP(t4);
        live += st.active ? 1u : 0u;
        if (st.active || was || ended || done != ((flags & WF_DONE) != 0))
            wf_store(W, s, st, qpos, spos, done ? WF_DONE : 0u);
        WF_STAMP(t5);
#ifdef MTSG_WF_STAMPS
        stamp[0] += (uint32_t)(t1 - t0); stamp[1] += (uint32_t)(t2 - t1); stamp[2] += (uint32_t)(t3 - t2);
        stamp[3] += (uint32_t)(t4 - t3); stamp[4] += (uint32_t)(t5 - t4);
#endif
    }
    uint32_t v[16] = {};
    v[0] = (uint32_t)c.samples; v[1] = (uint32_t)c.rays; v[2] = (uint32_t)c.shadow; v[3] = (uint32_t)c.len;
    v[6] = (uint32_t)c.err;
    v[8] = live;   // (slot 8 is otherwise unused) live slots: this block's region count below
    if (INSTR) { v[7] = (uint32_t)c.hits; v[9] = (uint32_t)c.nee; v[10] = (uint32_t)c.sobol; }
#ifdef MTSG_WF_STAMPS   // diagnostic build: cycles per section, summed over waves (counters 11-15)
    if (lane_id() == 0)
        for (int k = 0; k < 5; ++k) v[11 + k] = stamp[k] >> 4;
#endif
    (void)stamp;
    block_counters(part, v, red, 8, W.live + W.parity);   // ends with a barrier: qcnt is final
    if (threadIdx.x < 2) W.rcnt[(W.parity * 2 + threadIdx.x) * W.regions + blockIdx.x] = qcnt[threadIdx.x];
}

// both queues of one bounce, region by region: block t works on wf_shade
// region t / split, entries [0, nc) closest hit then [nc, nc + ns) shadow, in
// steps of split x 256; block 0 also clears the other parity's live count
template <bool STATS, bool SCENE_LDS, bool ANA>
__global__ __launch_bounds__(BLOCK, MTSG_WF_TRACE_WAVES) void wf_trace(MtsgLaunch L, MtsgWave W,
                                                                       unsigned long long *part) {
    extern __shared__ uint32_t lds[];
    __shared__ uint32_t red[BLOCK / 64 * 16];
    const MtsgDeviceScene &S = L.scene;
    if (blockIdx.x == 0 && threadIdx.x == 0) W.live[W.parity ^ 1u] = 0;
    const uint32_t region = blockIdx.x / W.split, part0 = blockIdx.x % W.split;
    if (region >= W.regions) return;
    const uint32_t nc = W.rcnt[(W.parity * 2 + 0) * W.regions + region];
    const uint32_t ns = W.rcnt[(W.parity * 2 + 1) * W.regions + region];
    if (part0 * BLOCK >= nc + ns) return;   // block-uniform
    uint32_t stackBase = 0;
    if (SCENE_LDS && !L.scan) {
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
    unsigned long long cN = 0, cT = 0;
    const uint32_t n = nc + ns, base = region * W.rounds * BLOCK;
    for (uint32_t i = part0 * BLOCK + threadIdx.x; i < n; i += W.split * BLOCK) {
        const bool shadow = i >= nc;
        const uint32_t k = base + (shadow ? i - nc : i);
        const float4 *q = shadow ? W.sray : W.qray;
        const float4 a = q[2 * (size_t)k], b = q[2 * (size_t)k + 1];
        const f3 o = mk(a.x, a.y, a.z), d = mk(b.x, b.y, b.z);
        const float mint = a.w, maxt = b.w;
        uint32_t slot = 0;
        float hu = 0, hv = 0, ht = 0;
        if (shadow) {
            bool occ;
            if (SCENE_LDS && L.scan)
                occ = scan_tris<true, STATS>(L, o, d, mint, maxt, slot, hu, hv, ht, cT);
            else if (SCENE_LDS)
                occ = traverse<true, STATS, ANA, MTSG_WF_LDS_STACK>(ldsNodes, ldsTris, o, d, mint, maxt, stkN, stkD,
                                                                    slot, hu, hv, ht, cN, cT, S.analytic, ovf);
            else
                occ = traverse<true, STATS, ANA, MTSG_WF_LDS_STACK>((glb_node *)S.nodes, (glb_tri *)S.tris, o, d, mint,
                                                                    maxt, stkN, stkD, slot, hu, hv, ht, cN, cT,
                                                                    S.analytic, ovf);
            W.occl[k] = occ ? 1u : 0u;
        } else {
            bool hit;
            if (SCENE_LDS && L.scan)
                hit = scan_tris<false, STATS>(L, o, d, mint, maxt, slot, hu, hv, ht, cT);
            else if (SCENE_LDS)
                hit = traverse<false, STATS, ANA, MTSG_WF_LDS_STACK>(ldsNodes, ldsTris, o, d, mint, maxt, stkN, stkD,
                                                                     slot, hu, hv, ht, cN, cT, S.analytic, ovf);
            else
                hit = traverse<false, STATS, ANA, MTSG_WF_LDS_STACK>((glb_node *)S.nodes, (glb_tri *)S.tris, o, d,
                                                                     mint, maxt, stkN, stkD, slot, hu, hv, ht, cN, cT,
                                                                     S.analytic, ovf);
            const uint32_t w = !hit ? MTSG_WF_NONE : ANA ? slot
                             : (SCENE_LDS && L.scan) ? slot : SCENE_LDS ? ldsTris[slot].prim : S.tris[slot].prim;
            W.hit[k] = make_float4(ht, hu, hv, __uint_as_float(w));
        }
    }
    if (STATS) {
        uint32_t v[16] = {};
        v[4] = (uint32_t)cN;
        v[5] = (uint32_t)cT;
        block_counters(part, v, red);
    }
}

// wf_trace over the reference's kd-tree (MTSGPU_FLAG_KDTREE): the same queues,
// kd_traverse (SAHKDTree3D::rayIntersectHavran) per ray; hits carry the global
// primitive number, as wf_trace's do for triangle scenes
template <bool STATS>
__global__ __launch_bounds__(BLOCK) void wf_trace_kd(MtsgLaunch L, MtsgWave W, unsigned long long *part) {
    __shared__ uint32_t red[BLOCK / 64 * 16];
    if (blockIdx.x == 0 && threadIdx.x == 0) W.live[W.parity ^ 1u] = 0;
    const uint32_t region = blockIdx.x / W.split, part0 = blockIdx.x % W.split;
    if (region >= W.regions) return;
    const uint32_t nc = W.rcnt[(W.parity * 2 + 0) * W.regions + region];
    const uint32_t ns = W.rcnt[(W.parity * 2 + 1) * W.regions + region];
    if (part0 * BLOCK >= nc + ns) return;   // block-uniform
    const uint2 *kn = (const uint2 *)L.kd_nodes;
    const uint32_t n = nc + ns, base = region * W.rounds * BLOCK;
    for (uint32_t i = part0 * BLOCK + threadIdx.x; i < n; i += W.split * BLOCK) {
        const bool shadow = i >= nc;
        const uint32_t k = base + (shadow ? i - nc : i);
        const float4 *q = shadow ? W.sray : W.qray;
        const float4 a = q[2 * (size_t)k], b = q[2 * (size_t)k + 1];
        const f3 o = mk(a.x, a.y, a.z), d = mk(b.x, b.y, b.z);
        float ht = 0, hu = 0, hv = 0;
        uint32_t prim = 0;
        if (shadow) {
            W.occl[k] = kd_traverse<true>(kn, L.kd_indices, L.kd_tris, o, d, a.w, b.w, ht, hu, hv, prim) ? 1u : 0u;
        } else {
            const bool hit = kd_traverse<false>(kn, L.kd_indices, L.kd_tris, o, d, a.w, b.w, ht, hu, hv, prim);
            W.hit[k] = make_float4(ht, hu, hv, __uint_as_float(hit ? prim : MTSG_WF_NONE));
        }
    }
    if (STATS) {
        uint32_t v[16] = {};
        block_counters(part, v, red);
    }
}

// the per-block partial counters of a chunk -> MtsgLaunch::counters
__global__ void wf_flush(const unsigned long long *part, uint32_t blocks, unsigned long long *counters) {
    const uint32_t k = threadIdx.x & 15u;   // 256 threads: counter k, blocks b = threadIdx / 16 (mod 16)
    unsigned long long t = 0;
    for (uint32_t b = threadIdx.x >> 4; b < blocks; b += 16) t += part[(size_t)b * 16 + k];
    if (t) atomicAdd(counters + k, t);
}

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

// direct_kernel's shadow rays: the any-hit traversal as a separate (not
// inlined) function.  Inlined into direct_kernel's nested divergent loops at
// -O3, hipcc (ROCm 7.2, gfx950) produced wrong occlusion answers for 15% of the
// samples of the analytic-shape scene; the same source is exact at -O1, as a
// call, with the NaN-aware (closest-hit) form of the sphere predicate, and
// inlined into path_kernel / trace_kernel (DESIGN.md 4 has the bisection)
#ifdef MTSG_ANYHIT_INLINE   // diagnostic build: the round-1 inlined form (tools/diag_parity.py)
#define SHADOW_ANY_CALL __device__ __forceinline__
#else
#define SHADOW_ANY_CALL __device__ __noinline__
#endif
template <bool ANA, typename NodeT, typename TriT>
SHADOW_ANY_CALL bool shadow_any(NodeT *nodes, TriT *tris, f3 o, f3 d, float mint, float maxt,
                                        lds_stk_n *stkN, lds_stk_d *stkD, unsigned long long &cN,
                                        unsigned long long &cT, const MtsgAnalytic *ana) {
    uint32_t sl = 0;
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
    return traverse<true, false, ANA>(nodes, tris, o, d, mint, maxt, stkN, stkD, sl, a0, a1, a2, cN, cT, ana);
}
#ifdef MTSG_ANYHIT_CROSSCHECK   // diagnostic build: the inlined any-hit query beside the call, disagreements printed
template <bool ANA, typename NodeT, typename TriT>
__device__ __forceinline__ bool shadow_any_inl(NodeT *nodes, TriT *tris, f3 o, f3 d, float mint, float maxt,
                                               lds_stk_n *stkN, lds_stk_d *stkD, unsigned long long &cN,
                                               unsigned long long &cT, const MtsgAnalytic *ana, uint32_t &sl,
                                               float &a0, float &a1, float &a2) {
    sl = 0xffffffffu;
    a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
    return traverse<true, false, ANA>(nodes, tris, o, d, mint, maxt, stkN, stkD, sl, a0, a1, a2, cN, cT, ana);
}
__device__ unsigned int g_anyhit_xc;
#endif
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
#ifdef MTSG_ANYHIT_CROSSCHECK
        {
            uint32_t xs;
            float x0, x1, x2;
            const bool ri = SCENE_LDS ? shadow_any_inl<ANA>(ldsNodes, ldsTris, o, d, mint, maxt, stkN, stkD, cN, cT,
                                                            S.analytic, xs, x0, x1, x2)
                                      : shadow_any_inl<ANA>((glb_node *)S.nodes, (glb_tri *)S.tris, o, d, mint, maxt,
                                                            stkN, stkD, cN, cT, S.analytic, xs, x0, x1, x2);
            const bool rc = SCENE_LDS ? shadow_any<ANA>(ldsNodes, ldsTris, o, d, mint, maxt, stkN, stkD, cN, cT,
                                                        S.analytic)
                                      : shadow_any<ANA>((glb_node *)S.nodes, (glb_tri *)S.tris, o, d, mint, maxt,
                                                        stkN, stkD, cN, cT, S.analytic);
            if (ri != rc) {
                const unsigned int k = atomicAdd(&g_anyhit_xc, 1u);
                if (k < 48)
                    printf("XC %u inl %d call %d o %08x %08x %08x d %08x %08x %08x dist %08x mint %08x maxt %08x "
                           "lane %u slot %08x a %.9g %.9g %.9g\n", k, (int)ri, (int)rc, __float_as_uint(o.x),
                           __float_as_uint(o.y), __float_as_uint(o.z), __float_as_uint(d.x), __float_as_uint(d.y),
                           __float_as_uint(d.z), __float_as_uint(dist), __float_as_uint(mint), __float_as_uint(maxt),
                           threadIdx.x, xs, x0, x1, x2);
            }
            return rc;
        }
#endif
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
        float ownW = 0.0f;
        const bool valid = film_splat(L, px, py, sx, sy, val, ownW);
        float4 rec4 = valid ? make_float4(Li.x, Li.y, Li.z, alpha == 0.0f ? -ownW : ownW) : make_float4(0, 0, 0, 0);
        reinterpret_cast<float4 *>(L.contrib)[(size_t)(j - L.j0) * L.num_pixels + pix] = rec4;
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
    const float4 *c = reinterpret_cast<const float4 *>(L.contrib) + p;
    for (uint32_t jj = 0; jj < L.chunk_spp; ++jj) {
        const float4 r = c[(size_t)jj * L.num_pixels];
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

__global__ void film_finalize(float *__restrict__ own, const float *__restrict__ spill, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) own[i] += spill[i];
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

// variants: small scenes (BVH in LDS) run 3 waves/SIMD with 32 Sobol dims in
// LDS; large scenes run 4 waves/SIMD (128 VGPRs) when the traversal stacks fit
// 4 blocks per CU, else 3 (capi.cpp picks L.waves and L.lds_dims)
template <bool SCENE_LDS, int FEAT, int WAVES>
static void launch_path_w(const MtsgLaunch &L, int grid, bool instr, hipStream_t stream) {
    const size_t lds = mtsg_path_lds_bytes(L);
    if (instr) hipLaunchKernelGGL((path_kernel<true, SCENE_LDS, FEAT, WAVES>), dim3(grid), dim3(BLOCK), lds, stream, L);
    else hipLaunchKernelGGL((path_kernel<false, SCENE_LDS, FEAT, WAVES>), dim3(grid), dim3(BLOCK), lds, stream, L);
}

int mtsg_path_features(const MtsgLaunch &L) {
    return (L.scene.env_emitter >= 0 ? MTSG_FEAT_ENV : 0) | ((L.ext || L.ana) ? MTSG_FEAT_EXT : 0) |
           (L.ana ? MTSG_FEAT_ANA : 0);
}

// the specialised BSDF sets compiled for the large-scene megakernel: the
// scene's features (ENV / EXT / ANA) must match, and the set's restrictions
// (GGX / NORD / NORC) must hold for the scene (L.bset); dbsdf.h BSet
#define MTSG_SPEC_BITS (MTSG_FEAT_GGX | MTSG_FEAT_NORD | MTSG_FEAT_NORC)
#define MTSG_SPEC_SETS(X)                                                                         \
    X(MTSG_FEAT_ENV | MTSG_FEAT_GGX | MTSG_FEAT_NORD)             /* rough conductors, envmap  */ \
    X(MTSG_FEAT_GGX | MTSG_FEAT_NORC)                             /* rough glass, area lights  */ \
    X(MTSG_FEAT_ENV | MTSG_FEAT_EXT | MTSG_FEAT_GGX | MTSG_FEAT_NORD | MTSG_FEAT_NORC) /* plastic */
static int spec_variant(const MtsgLaunch &L) {
    if (L.scene_lds || L.integrator == MTSG_INTEGRATOR_DIRECT) return 0;
    const int f = mtsg_path_features(L);
#define MTSG_SPEC_PICK(V) \
    if (((V) & ~MTSG_SPEC_BITS) == f && ((V) & MTSG_SPEC_BITS & ~(int)L.bset) == 0) return (V);
    MTSG_SPEC_SETS(MTSG_SPEC_PICK)
#undef MTSG_SPEC_PICK
    return 0;
}

template <int FEAT>
static void launch_path(const MtsgLaunch &L, int grid, bool instr, hipStream_t stream) {
    if constexpr ((FEAT & MTSG_SPEC_BITS) != 0) {   // large scenes only (spec_variant)
        if (L.waves == 4) launch_path_w<false, FEAT, 4>(L, grid, instr, stream);
        else launch_path_w<false, FEAT, MTSG_WAVES_PER_EU>(L, grid, instr, stream);
    } else {
        if (L.scene_lds) {
            if constexpr ((FEAT & MTSG_FEAT_DIFF) != 0) {   // no calls: room for 4 waves (capi.cpp)
                if (L.waves == 4) { launch_path_w<true, FEAT, 4>(L, grid, instr, stream); return; }
            }
            launch_path_w<true, FEAT, MTSG_WAVES_PER_EU>(L, grid, instr, stream);
        }
        else if (L.waves == 4) launch_path_w<false, FEAT, 4>(L, grid, instr, stream);
        else launch_path_w<false, FEAT, MTSG_WAVES_PER_EU>(L, grid, instr, stream);
    }
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
    switch (spec_variant(L)) {
#define MTSG_SPEC_CASE(V) \
        case (V): launch_path<(V)>(L, grid, instr, stream); return hipGetLastError();
        MTSG_SPEC_SETS(MTSG_SPEC_CASE)
#undef MTSG_SPEC_CASE
        default: break;
    }
    switch (mtsg_path_features(L)) {
        case 0:
            if (L.all_diffuse) launch_path<MTSG_FEAT_DIFF>(L, grid, instr, stream);
            else launch_path<0>(L, grid, instr, stream);
            break;
        case MTSG_FEAT_ENV: launch_path<MTSG_FEAT_ENV>(L, grid, instr, stream); break;
        case MTSG_FEAT_EXT: launch_path<MTSG_FEAT_EXT>(L, grid, instr, stream); break;
        case MTSG_FEAT_ENV | MTSG_FEAT_EXT: launch_path<MTSG_FEAT_ENV | MTSG_FEAT_EXT>(L, grid, instr, stream); break;
        case MTSG_FEAT_EXT | MTSG_FEAT_ANA: launch_path<MTSG_FEAT_EXT | MTSG_FEAT_ANA>(L, grid, instr, stream); break;
        default: launch_path<MTSG_FEAT_ENV | MTSG_FEAT_EXT | MTSG_FEAT_ANA>(L, grid, instr, stream); break;
    }
    return hipGetLastError();
}

hipError_t mtsg_launch_reduce(const MtsgLaunch &L, hipStream_t stream) {
    const int threads = 256;
    const int blocks = (int)((L.num_pixels + threads - 1) / threads);
    hipLaunchKernelGGL(film_reduce, dim3(blocks), dim3(threads), 0, stream, L);
    return hipGetLastError();
}

hipError_t mtsg_launch_finalize(float *own, const float *spill, size_t n, hipStream_t stream) {
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

// wavefront launchers: wf_shade needs no traversal stacks; wf_trace stages
// the BVH of SCENE_LDS scenes (not the linear-scan ones) and holds the stacks
size_t mtsg_wf_shade_lds_bytes(const MtsgLaunch &L) {
    const size_t scene = L.scene_lds ? ((size_t)L.num_nodes * 16 + (size_t)L.scene.num_prims * (12 + 7) +
                                        (size_t)L.num_verts * 6 + (size_t)L.num_shapes * (sizeof(MtsgShape) / 4))
                                     : 0;
    return ((size_t)L.lds_dims * L.nibbles * 16 + 16 * 16 + scene) * 4;
}
size_t mtsg_wf_trace_lds_bytes(const MtsgLaunch &L) {
    const bool scan = L.scene_lds && L.scan;
    const size_t scene = (L.scene_lds && !L.scan) ? ((size_t)L.num_nodes * 16 + (size_t)L.scene.num_prims * 12) : 0;
    const size_t K = std::min<size_t>(L.stack_depth, MTSG_WF_LDS_STACK);
    const size_t stack = scan ? 0 : (K * 3 * BLOCK + 1) / 2;
    return (scene + stack) * 4 + 16;
}

template <int FEAT>
static void launch_wf_shade_f(const MtsgLaunch &L, const MtsgWave &W, unsigned long long *part, int grid, bool instr,
                              hipStream_t s) {
    const size_t lds = mtsg_wf_shade_lds_bytes(L);
#define MTSG_SHADE(I, SL) hipLaunchKernelGGL((wf_shade<I, SL, FEAT>), dim3(grid), dim3(BLOCK), lds, s, L, W, part)
    if (L.scene_lds) { if (instr) MTSG_SHADE(true, true); else MTSG_SHADE(false, true); }
    else { if (instr) MTSG_SHADE(true, false); else MTSG_SHADE(false, false); }
#undef MTSG_SHADE
}

hipError_t mtsg_launch_wf_shade(const MtsgLaunch &L, const MtsgWave &W, unsigned long long *part, int grid,
                                bool instr, hipStream_t s) {
    switch (mtsg_path_features(L)) {
        case 0: launch_wf_shade_f<0>(L, W, part, grid, instr, s); break;
        case MTSG_FEAT_ENV: launch_wf_shade_f<MTSG_FEAT_ENV>(L, W, part, grid, instr, s); break;
        case MTSG_FEAT_EXT: launch_wf_shade_f<MTSG_FEAT_EXT>(L, W, part, grid, instr, s); break;
        case MTSG_FEAT_ENV | MTSG_FEAT_EXT: launch_wf_shade_f<MTSG_FEAT_ENV | MTSG_FEAT_EXT>(L, W, part, grid, instr, s); break;
        case MTSG_FEAT_EXT | MTSG_FEAT_ANA: launch_wf_shade_f<MTSG_FEAT_EXT | MTSG_FEAT_ANA>(L, W, part, grid, instr, s); break;
        default: launch_wf_shade_f<MTSG_FEAT_ENV | MTSG_FEAT_EXT | MTSG_FEAT_ANA>(L, W, part, grid, instr, s); break;
    }
    return hipGetLastError();
}

hipError_t mtsg_launch_wf_trace(const MtsgLaunch &L, const MtsgWave &W, unsigned long long *part, int grid,
                                bool stats, hipStream_t s) {
    if (L.kd_nodes) {
        if (stats) hipLaunchKernelGGL(wf_trace_kd<true>, dim3(grid), dim3(BLOCK), 0, s, L, W, part);
        else hipLaunchKernelGGL(wf_trace_kd<false>, dim3(grid), dim3(BLOCK), 0, s, L, W, part);
        return hipGetLastError();
    }
    const size_t lds = mtsg_wf_trace_lds_bytes(L);
#define MTSG_WFT(ST, SL, A) hipLaunchKernelGGL((wf_trace<ST, SL, A>), dim3(grid), dim3(BLOCK), lds, s, L, W, part)
    const bool ana = L.ana != 0;
    if (stats) {
        if (L.scene_lds) { if (ana) MTSG_WFT(true, true, true); else MTSG_WFT(true, true, false); }
        else { if (ana) MTSG_WFT(true, false, true); else MTSG_WFT(true, false, false); }
    } else {
        if (L.scene_lds) { if (ana) MTSG_WFT(false, true, true); else MTSG_WFT(false, true, false); }
        else { if (ana) MTSG_WFT(false, false, true); else MTSG_WFT(false, false, false); }
    }
#undef MTSG_WFT
    return hipGetLastError();
}

hipError_t mtsg_launch_wf_flush(const unsigned long long *part, uint32_t blocks, unsigned long long *counters,
                                hipStream_t s) {
    hipLaunchKernelGGL(wf_flush, dim3(1), dim3(256), 0, s, part, blocks, counters);
    return hipGetLastError();
}

// resident blocks per CU of the two wavefront kernels (their grids)
int mtsg_wf_occupancy(const MtsgLaunch &L, int *shadeBpc, int *traceBpc) {
    *shadeBpc = *traceBpc = 0;
    const size_t ls = mtsg_wf_shade_lds_bytes(L), lt = mtsg_wf_trace_lds_bytes(L);
    int r = 0;
    switch (mtsg_path_features(L)) {   // the instrumented variants run on the same grid
#define MTSG_OCC(F) \
        r = L.scene_lds ? (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(shadeBpc, wf_shade<false, true, F>, BLOCK, ls) \
                        : (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(shadeBpc, wf_shade<false, false, F>, BLOCK, ls); \
        break;
        case 0: MTSG_OCC(0)
        case MTSG_FEAT_ENV: MTSG_OCC(MTSG_FEAT_ENV)
        case MTSG_FEAT_EXT: MTSG_OCC(MTSG_FEAT_EXT)
        case MTSG_FEAT_ENV | MTSG_FEAT_EXT: MTSG_OCC(MTSG_FEAT_ENV | MTSG_FEAT_EXT)
        case MTSG_FEAT_EXT | MTSG_FEAT_ANA: MTSG_OCC(MTSG_FEAT_EXT | MTSG_FEAT_ANA)
        default: MTSG_OCC(MTSG_FEAT_ENV | MTSG_FEAT_EXT | MTSG_FEAT_ANA)
#undef MTSG_OCC
    }
    if (r) return r;
    const bool ana = L.ana != 0;
    if (L.scene_lds) r = ana ? (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(traceBpc, wf_trace<false, true, true>, BLOCK, lt)
                             : (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(traceBpc, wf_trace<false, true, false>, BLOCK, lt);
    else r = ana ? (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(traceBpc, wf_trace<false, false, true>, BLOCK, lt)
                 : (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(traceBpc, wf_trace<false, false, false>, BLOCK, lt);
    return r;
}

template <bool SCENE_LDS, int FEAT, int WAVES>
static int occupancy_w(const MtsgLaunch &L, int *bpc) {
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(bpc, path_kernel<false, SCENE_LDS, FEAT, WAVES>, BLOCK,
                                                             mtsg_path_lds_bytes(L));
}
template <int FEAT>
static int occupancy_e(const MtsgLaunch &L, int *bpc) {
    if constexpr ((FEAT & MTSG_SPEC_BITS) != 0) {
        if (L.waves == 4) return occupancy_w<false, FEAT, 4>(L, bpc);
        return occupancy_w<false, FEAT, MTSG_WAVES_PER_EU>(L, bpc);
    } else {
        if (L.scene_lds) {
            if constexpr ((FEAT & MTSG_FEAT_DIFF) != 0) {
                if (L.waves == 4) return occupancy_w<true, FEAT, 4>(L, bpc);
            }
            return occupancy_w<true, FEAT, MTSG_WAVES_PER_EU>(L, bpc);
        }
        if (L.waves == 4) return occupancy_w<false, FEAT, 4>(L, bpc);
        return occupancy_w<false, FEAT, MTSG_WAVES_PER_EU>(L, bpc);
    }
}
int mtsg_path_kernel_occupancy(const MtsgLaunch &L, int *blocksPerCU) {
    switch (spec_variant(L)) {
#define MTSG_SPEC_CASE(V) \
        case (V): return occupancy_e<(V)>(L, blocksPerCU);
        MTSG_SPEC_SETS(MTSG_SPEC_CASE)
#undef MTSG_SPEC_CASE
        default: break;
    }
    switch (mtsg_path_features(L)) {
        case 0: return L.all_diffuse ? occupancy_e<MTSG_FEAT_DIFF>(L, blocksPerCU) : occupancy_e<0>(L, blocksPerCU);
        case MTSG_FEAT_ENV: return occupancy_e<MTSG_FEAT_ENV>(L, blocksPerCU);
        case MTSG_FEAT_EXT: return occupancy_e<MTSG_FEAT_EXT>(L, blocksPerCU);
        case MTSG_FEAT_ENV | MTSG_FEAT_EXT: return occupancy_e<MTSG_FEAT_ENV | MTSG_FEAT_EXT>(L, blocksPerCU);
        case MTSG_FEAT_EXT | MTSG_FEAT_ANA: return occupancy_e<MTSG_FEAT_EXT | MTSG_FEAT_ANA>(L, blocksPerCU);
        default: return occupancy_e<MTSG_FEAT_ENV | MTSG_FEAT_EXT | MTSG_FEAT_ANA>(L, blocksPerCU);
    }
}
