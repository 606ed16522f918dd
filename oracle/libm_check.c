/* libm_check.c -- TEST INFRASTRUCTURE: checks the host build of the product's
 * glibc restatement (mitsuba0.6_amd/csrc/glibc_f32.h) against this machine's
 * libm.so.6, bit for bit.  Unary functions run over all 2^32 float inputs;
 * atan2f and powf over seeded random pairs plus dense grids.  NaN results
 * compare as a class (glibc returns x86's default NaN, sign bit set).
 * Also exports glibc_eval() for tests/test_gpu_libm.py (ctypes, _build/liblibm_check.so): the host
 * libm's values for given inputs.
 *
 * usage: libm_check <fn> [pairs]   fn: sincosf expf acosf atanf tanf atan2f powf
 * prints "<fn> checked=<n> mismatches=<m>" and the first mismatches. */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../mitsuba0.6_amd/csrc/glibc_f32.h"

static int same(float a, float b) {
    if (a != a && b != b) return 1;
    return glf_asuint(a) == glf_asuint(b);
}

static uint64_t splitmix(uint64_t *s) {
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

/* fn ids shared with the GPU probe (mtsgpu_debug_libm) */
enum { F_SIN = 0, F_COS, F_EXP, F_ACOS, F_ATAN, F_TAN, F_ATAN2, F_POW, F_FASTEXP, F_FASTLOG };

static float ref1(int fn, float x, float y) {
    float s, c;
    switch (fn) {
    case F_SIN: sincosf(x, &s, &c); return s;
    case F_COS: sincosf(x, &s, &c); return c;
    case F_EXP: return expf(x);
    case F_ACOS: return acosf(x);
    case F_ATAN: return atanf(x);
    case F_TAN: return tanf(x);
    case F_ATAN2: return atan2f(x, y);
    case F_POW: return powf(x, y);
    case F_FASTEXP: return (float)exp((double)x);
    case F_FASTLOG: return (float)log((double)x);
    }
    return 0;
}

static float mine1(int fn, float x, float y) {
    float s, c;
    switch (fn) {
    case F_SIN: glf_sincosf(x, &s, &c); return s;
    case F_COS: glf_sincosf(x, &s, &c); return c;
    case F_EXP: return glf_expf(x);
    case F_ACOS: return glf_acosf(x);
    case F_ATAN: return glf_atanf(x);
    case F_TAN: return glf_tanf(x);
    case F_ATAN2: return glf_atan2f(x, y);
    case F_POW: return glf_powf(x, y);
    }
    return 0;
}

/* host libm values for the GPU test: out[i] = f(a[i], b[i]) */
void glibc_eval(int fn, const float *a, const float *b, float *out, long n) {
#pragma omp parallel for schedule(static)
    for (long i = 0; i < n; ++i) out[i] = ref1(fn, a[i], b ? b[i] : 0.0f);
}

/* mismatches between dev[i] and glibc's f(bits first + i) for i < n (unary fns);
   the first mismatching index goes to *first_bad (-1 if none) */
long glibc_compare_range(int fn, uint32_t first, long n, const float *dev, long *first_bad) {
    long bad = 0, fb = n;
#pragma omp parallel for schedule(static) reduction(+ : bad) reduction(min : fb)
    for (long i = 0; i < n; ++i) {
        if (!same(ref1(fn, glf_asfloat(first + (uint32_t)i), 0.0f), dev[i])) {
            ++bad;
            if (i < fb) fb = i;
        }
    }
    *first_bad = bad ? fb : -1;
    return bad;
}

static long report(const char *name, long checked, long bad, float *bx, float *by, int nb, int fn) {
    printf("%s checked=%ld mismatches=%ld\n", name, checked, bad);
    for (int i = 0; i < nb; ++i) {
        float r = ref1(fn, bx[i], by[i]), m = mine1(fn, bx[i], by[i]);
        printf("  x=%a (0x%08x) y=%a glibc=%a (0x%08x) mine=%a (0x%08x)\n", bx[i], glf_asuint(bx[i]), by[i], r,
               glf_asuint(r), m, glf_asuint(m));
    }
    return bad;
}

#define MAXB 8
static long check_unary(const char *name, int fn, int fn2) {
    long bad = 0;
    float bx[MAXB], by[MAXB];
    int nb = 0;
#pragma omp parallel for schedule(dynamic, 1 << 20) reduction(+ : bad)
    for (long i = 0; i < (1L << 32); ++i) {
        const float x = glf_asfloat((uint32_t)i);
        int ok = same(ref1(fn, x, 0), mine1(fn, x, 0));
        if (fn2 >= 0) ok = ok && same(ref1(fn2, x, 0), mine1(fn2, x, 0));
        if (!ok) {
            ++bad;
#pragma omp critical
            if (nb < MAXB) { bx[nb] = x; by[nb] = 0; ++nb; }
        }
    }
    return report(name, 1L << 32, bad, bx, by, nb, fn);
}

/* pairs: seeded random bit patterns, random values in [-8, 8], and for powf
   bases in (0, 2] with the exponents the path uses (0.25, 1/(e+2), e+1) */
static long check_binary(const char *name, int fn, long pairs) {
    long bad = 0;
    float bx[MAXB], by[MAXB];
    int nb = 0;
#pragma omp parallel for schedule(dynamic, 1 << 16) reduction(+ : bad)
    for (long i = 0; i < pairs; ++i) {
        uint64_t st = 0x1234567ull + (uint64_t)i * 0x9e3779b97f4a7c15ull;
        const uint64_t r = splitmix(&st);
        float x, y;
        switch (i % 4) {
        case 0: x = glf_asfloat((uint32_t)r); y = glf_asfloat((uint32_t)(r >> 32)); break;
        case 1:
            x = (float)((int32_t)(uint32_t)r) * 0x1p-28f;
            y = (float)((int32_t)(uint32_t)(r >> 32)) * 0x1p-28f;
            break;
        case 2:
            x = (float)(uint32_t)r * 0x1p-31f;
            y = (float)((int32_t)(uint32_t)(r >> 32)) * 0x1p-24f;
            break;
        default:
            x = (float)((uint32_t)r >> 8) * 0x1p-24f;
            y = (fn == F_POW) ? ((r >> 40) & 1 ? 0.25f : (float)((r >> 41) & 0xffff) * 0x1p-8f + 1.0f)
                              : (float)((int32_t)(uint32_t)(r >> 32)) * 0x1p-40f;
            break;
        }
        if (!same(ref1(fn, x, y), mine1(fn, x, y))) {
            ++bad;
#pragma omp critical
            if (nb < MAXB) { bx[nb] = x; by[nb] = y; ++nb; }
        }
    }
    return report(name, pairs, bad, bx, by, nb, fn);
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s fn [pairs]\n", argv[0]); return 2; }
    const char *f = argv[1];
    const long pairs = argc > 2 ? atol(argv[2]) : (1L << 28);
    long bad;
    if (!strcmp(f, "sincosf")) bad = check_unary(f, F_SIN, F_COS);
    else if (!strcmp(f, "expf")) bad = check_unary(f, F_EXP, -1);
    else if (!strcmp(f, "acosf")) bad = check_unary(f, F_ACOS, -1);
    else if (!strcmp(f, "atanf")) bad = check_unary(f, F_ATAN, -1);
    else if (!strcmp(f, "tanf")) bad = check_unary(f, F_TAN, -1);
    else if (!strcmp(f, "atan2f")) bad = check_binary(f, F_ATAN2, pairs);
    else if (!strcmp(f, "powf")) bad = check_binary(f, F_POW, pairs);
    else { fprintf(stderr, "unknown fn %s\n", f); return 2; }
    return bad ? 1 : 0;
}
