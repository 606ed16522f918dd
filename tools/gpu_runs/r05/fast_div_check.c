/* Host check of div_by_rcp (csrc/dpath.h): a / b as a * RN(1/b) with two
 * FMA residual corrections, against IEEE division, bit for bit, over the range
 * the scan's fast path admits (|b| in [2^-60, 2), quotients >= 2^-31 in
 * magnitude; smaller ones fall below every admitted mint).  Random signs,
 * exponents and mantissas, 3 in 8 of them edge mantissas (near all-ones, near
 * zero, near the half).
 *   gcc -O2 -ffp-contract=off -mfma -o /tmp/fdc tools/gpu_runs/r05/fast_div_check.c -lm && /tmp/fdc 400000000
 * r05: 1.6e9 pairs over three runs (numerators 2^-40..2^20 and 2^-40..2^60), 0 mismatches. */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static inline float fdiv(float a, float b, float y) {
    float q = a * y;
    float r = fmaf(-b, q, a);
    q = fmaf(r, y, q);
    r = fmaf(-b, q, a);
    return fmaf(r, y, q);
}
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline float rf(int elo, int ehi) {  // random sign/exponent in [elo, ehi], random mantissa
    uint64_t r = xr();
    int e = elo + (int)(r % (uint64_t)(ehi - elo + 1));
    uint32_t m = (uint32_t)(r >> 20) & 0x7fffff;
    switch ((r >> 8) & 7) {   // edge mantissas
        case 0: m = 0x7fffff - (uint32_t)((r >> 11) & 15); break;
        case 1: m = (uint32_t)((r >> 11) & 15); break;
        case 2: m = 0x400000 ^ (uint32_t)((r >> 11) & 15); break;
        default: break;
    }
    uint32_t sg = (uint32_t)(r >> 60) & 1;
    uint32_t bits = (sg << 31) | ((uint32_t)(e + 127) << 23) | m;
    float f; memcpy(&f, &bits, 4); return f;
}
int main(int argc, char **argv) {
    long n = atol(argv[1]); long bad = 0, checked = 0;
    for (long i = 0; i < n; ++i) {
        float b = rf(-60, 0);            // direction component, |b| in [2^-60, 2)
        float a = rf(-40, 60);           // numerator n_d - o_k
        volatile float y = 1.0f / b;
        float q = a / b;
        if (fabsf(q) < 0x1p-31f) continue;   // below every guarded mint: rejected both ways
        float f = fdiv(a, b, y);
        ++checked;
        if (memcmp(&f, &q, 4)) { if (bad < 10) printf("a=%a b=%a ieee=%a fast=%a\n", a, b, q, f); ++bad; }
    }
    printf("checked %ld bad %ld\n", checked, bad);
    return 0;
}
