// sfmt.h -- SFMT19937, Mitsuba's Random (src/libcore/random.cpp), for the
// `independent` sampler replay (MTSGPU_SAMPLER_SFMT_*).  The host seeds the
// streams (init_gen_rand / init_by_array / Random(Random *) clones, done once
// per render); the device only advances them (gen_rand_all, nextULong,
// nextFloat).  A stream is MTSG_SFMT_WORDS 32-bit words: the 624-word state,
// then the index into it.
#pragma once
#include <stdint.h>

#define MTSG_SFMT_N 156          // 128-bit state words (MEXP 19937)
#define MTSG_SFMT_N32 624
#define MTSG_SFMT_N64 312
#define MTSG_SFMT_WORDS 628      // state + idx, padded to 16 bytes

#if defined(__HIPCC__)
#define SFMT_FN __host__ __device__ __forceinline__
#else
#define SFMT_FN inline
#endif

// do_recursion on one 128-bit word (random.cpp:204-219): 128-bit shifts by
// SL2 = SR2 = 1 byte, 32-bit shifts SR1 = 11, SL1 = 18, masks MSK1..4
SFMT_FN void sfmt_step(uint32_t *r, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    const uint32_t msk[4] = {0xdfffffefu, 0xddfecb7fu, 0xbffaffffu, 0xbffffff6u};
    const uint64_t alo = (uint64_t)a[0] | ((uint64_t)a[1] << 32), ahi = (uint64_t)a[2] | ((uint64_t)a[3] << 32);
    const uint64_t clo = (uint64_t)c[0] | ((uint64_t)c[1] << 32), chi = (uint64_t)c[2] | ((uint64_t)c[3] << 32);
    const uint64_t xlo = alo << 8, xhi = (ahi << 8) | (alo >> 56);   // lshift128(a, 1)
    const uint64_t ylo = (clo >> 8) | (chi << 56), yhi = chi >> 8;   // rshift128(c, 1)
    const uint32_t x[4] = {(uint32_t)xlo, (uint32_t)(xlo >> 32), (uint32_t)xhi, (uint32_t)(xhi >> 32)};
    const uint32_t y[4] = {(uint32_t)ylo, (uint32_t)(ylo >> 32), (uint32_t)yhi, (uint32_t)(yhi >> 32)};
    for (int k = 0; k < 4; ++k) r[k] = a[k] ^ x[k] ^ ((b[k] >> 11) & msk[k]) ^ y[k] ^ (d[k] << 18);
}

// gen_rand_all (random.cpp:353-390), in place
template <typename P>
SFMT_FN void sfmt_refill(P w) {
    uint32_t r1[4], r2[4];
    for (int k = 0; k < 4; ++k) { r1[k] = w[4 * (MTSG_SFMT_N - 2) + k]; r2[k] = w[4 * (MTSG_SFMT_N - 1) + k]; }
    for (int i = 0; i < MTSG_SFMT_N; ++i) {
        const int j = i < MTSG_SFMT_N - 122 ? i + 122 : i + 122 - MTSG_SFMT_N;   // POS1 = 122
        uint32_t a[4], b[4], r[4];
        for (int k = 0; k < 4; ++k) { a[k] = w[4 * i + k]; b[k] = w[4 * j + k]; }
        sfmt_step(r, a, b, r1, r2);
        for (int k = 0; k < 4; ++k) { w[4 * i + k] = r[k]; r1[k] = r2[k]; r2[k] = r[k]; }
    }
}

// gen_rand64 (random.cpp:288-297)
template <typename P>
SFMT_FN uint64_t sfmt_next_ulong(P w) {
    uint32_t idx = w[MTSG_SFMT_N32];
    if (idx >= MTSG_SFMT_N32) { sfmt_refill(w); idx = 0; }
    const uint64_t r = (uint64_t)w[idx] | ((uint64_t)w[idx + 1] << 32);
    w[MTSG_SFMT_N32] = idx + 2;
    return r;
}

// Random::nextFloat, SINGLE_PRECISION: ((low 32 bits) >> 9) | 1.0f, minus 1 (random.cpp:630-639)
template <typename P>
SFMT_FN float sfmt_next_float(P w) {
    const uint32_t u = ((uint32_t)(sfmt_next_ulong(w) & 0xFFFFFFFFull) >> 9) | 0x3f800000u;
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f - 1.0f;
}

// host-side seeding (Random(seed), Random(&parent)): capi.cpp mtsg_sfmt_seed / mtsg_sfmt_clone
