/* spectrum_rgb.c -- dev-time generator (not shipped, not on the GPU box):
 * RGB mode Spectrum::fromContinuousSpectrum of an InterpolatedSpectrum
 * (src/libcore/spectrum.cpp:171-190), restated in single precision:
 *   InterpolatedSpectrum::eval/average   spectrum.cpp:650-707
 *   ContinuousSpectrum::average           spectrum.cpp:546-567 (10000 evals, Epsilon, Epsilon)
 *   GaussLobattoIntegrator                libcore/quad.cpp:287-409
 *   Spectrum::fromXYZ (RGB build)         spectrum.cpp:222-227
 * stdin:  n_cie, then n_cie lines "lambda X Y Z"; then records
 *         "name n" followed by n lines "lambda value"
 * stdout: "name r g b" as C99 hex floats.
 * Build: gcc -O2 -ffp-contract=off -o spectrum_rgb spectrum_rgb.c -lm */
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int n; float *w, *v; } Interp;

static float smaxf(float a, float b) { return (a < b) ? b : a; }
static float sminf(float a, float b) { return (b < a) ? b : a; }
static float lerpf(float t, float v1, float v2) { return (1.0f - t) * v1 + t * v2; }   /* math.h:56-58 */

static float interp_eval(const Interp *s, float lambda) {   /* spectrum.cpp:685-707 */
    if (s->n < 2 || lambda < s->w[0] || lambda > s->w[s->n - 1]) return 0.0f;
    /* std::equal_range */
    int lo = 0, hi = s->n;
    while (lo < hi) { int mid = (lo + hi) / 2; if (s->w[mid] < lambda) lo = mid + 1; else hi = mid; }
    int idx1 = lo;
    lo = idx1; hi = s->n;
    while (lo < hi) { int mid = (lo + hi) / 2; if (lambda < s->w[mid]) hi = mid; else lo = mid + 1; }
    int idx2 = lo;
    if (idx1 == idx2) {
        float a = s->w[idx1 - 1], b = s->w[idx1], fa = s->v[idx1 - 1], fb = s->v[idx1];
        return lerpf((lambda - a) / (b - a), fb, fa);   /* argument order as in the reference */
    } else if (idx2 == idx1 + 1) {
        return s->v[idx1];
    }
    fprintf(stderr, "internal error\n");
    exit(1);
}

static float interp_average(const Interp *s, float lambdaMin, float lambdaMax) {   /* spectrum.cpp:650-683 */
    if (s->n < 2) return 0.0f;
    float rangeStart = smaxf(lambdaMin, s->w[0]);
    float rangeEnd = sminf(lambdaMax, s->w[s->n - 1]);
    if (rangeEnd <= rangeStart) return 0.0f;
    int lo = 0, hi = s->n;
    while (lo < hi) { int mid = (lo + hi) / 2; if (s->w[mid] < rangeStart) lo = mid + 1; else hi = mid; }
    size_t entry = (size_t)(lo > 1 ? lo : 1) - 1;
    float result = 0.0f;
    for (; entry + 1 < (size_t)s->n && rangeEnd >= s->w[entry]; ++entry) {
        float a = s->w[entry], b = s->w[entry + 1];
        float ca = smaxf(a, rangeStart), cb = sminf(b, rangeEnd);
        float fa = s->v[entry], fb = s->v[entry + 1], invAB = 1.0f / (b - a);
        if (cb <= ca) continue;
        float interpA = lerpf((ca - a) * invAB, fa, fb);
        float interpB = lerpf((cb - a) * invAB, fa, fb);
        result += 0.5f * (interpA + interpB) * (cb - ca);
    }
    return result / (lambdaMax - lambdaMin);
}

/* ProductSpectrum(smooth, cie).eval (spectrum.cpp:503-505) */
static const Interp *g_s1, *g_s2;
static float product_eval(float l) { return interp_eval(g_s1, l) * interp_eval(g_s2, l); }

/* GaussLobattoIntegrator (quad.cpp:287-409), useConvergenceEstimate = false */
static float g_alpha, g_beta;
static const float g_x1 = 0.94288241569547971906f, g_x2 = 0.64185334234578130578f, g_x3 = 0.23638319966214988028f;
static const size_t g_maxEvals = 10000;
static const float g_absError = 1e-4f, g_relError = 1e-4f;

static float abs_tolerance(float a, float b, size_t *evals) {
    const float m = (a + b) / 2, h = (b - a) / 2;
    const float y1 = product_eval(a), y3 = product_eval(m - g_alpha * h), y5 = product_eval(m - g_beta * h);
    const float y7 = product_eval(m), y9 = product_eval(m + g_beta * h), y11 = product_eval(m + g_alpha * h);
    const float y13 = product_eval(b);
    float acc = h * ((float)0.0158271919734801831 * (y1 + y13)
                   + (float)0.0942738402188500455 * (product_eval(m - g_x1 * h) + product_eval(m + g_x1 * h))
                   + (float)0.1550719873365853963 * (y3 + y11)
                   + (float)0.1888215739601824544 * (product_eval(m - g_x2 * h) + product_eval(m + g_x2 * h))
                   + (float)0.1997734052268585268 * (y5 + y9)
                   + (float)0.2249264653333395270 * (product_eval(m - g_x3 * h) + product_eval(m + g_x3 * h))
                   + (float)0.2426110719014077338 * y7);
    *evals += 13;
    float r = 1.0f;
    float result = INFINITY;
    if (g_relError != 0 && acc != 0) result = acc * smaxf(g_relError, FLT_EPSILON) / (r * FLT_EPSILON);
    if (g_absError != 0) result = sminf(result, g_absError / (r * FLT_EPSILON));
    return result;
}

static float gl_step(float a, float b, float fa, float fb, float acc, size_t *evals) {
    const float h = (b - a) / 2, m = (a + b) / 2;
    const float mll = m - g_alpha * h, ml = m - g_beta * h, mr = m + g_beta * h, mrr = m + g_alpha * h;
    const float fmll = product_eval(mll), fml = product_eval(ml), fm = product_eval(m), fmr = product_eval(mr),
                fmrr = product_eval(mrr);
    const float integral2 = (h / 6) * (fa + fb + 5 * (fml + fmr));
    const float integral1 = (h / 1470) * (77 * (fa + fb) + 432 * (fmll + fmrr) + 625 * (fml + fmr) + 672 * fm);
    *evals += 5;
    if (*evals >= g_maxEvals) return integral1;
    float dist = acc + (integral1 - integral2);
    if (dist == acc || mll <= a || b <= mrr) return integral1;
    float r = gl_step(a, mll, fa, fmll, acc, evals);
    r = r + gl_step(mll, ml, fmll, fml, acc, evals);
    r = r + gl_step(ml, m, fml, fm, acc, evals);
    r = r + gl_step(m, mr, fm, fmr, acc, evals);
    r = r + gl_step(mr, mrr, fmr, fmrr, acc, evals);
    r = r + gl_step(mrr, b, fmrr, fb, acc, evals);
    return r;
}

static float gl_integrate(float a, float b) {
    float factor = 1;
    size_t evals = 0;
    if (a == b) return 0;
    if (b < a) { float t = a; a = b; b = t; factor = -1; }
    const float absTolerance = abs_tolerance(a, b, &evals);
    evals += 2;
    return factor * gl_step(a, b, product_eval(a), product_eval(b), absTolerance, &evals);
}

static float continuous_average(float lambdaMin, float lambdaMax) {   /* spectrum.cpp:546-567 */
    if (lambdaMax <= lambdaMin) return 0.0f;
    float integral = 0;
    size_t nSteps = (size_t)ceilf((lambdaMax - lambdaMin) / 50);
    if (nSteps < 1) nSteps = 1;
    float stepSize = (lambdaMax - lambdaMin) / nSteps, pos = lambdaMin;
    for (size_t i = 0; i < nSteps; ++i) {
        integral += gl_integrate(pos, pos + stepSize);
        pos += stepSize;
    }
    return integral / (lambdaMax - lambdaMin);
}

static void read_interp(Interp *s, int n) {
    s->n = n;
    s->w = malloc(sizeof(float) * n);
    s->v = malloc(sizeof(float) * n);
    char a[64], b[64];
    for (int i = 0; i < n; ++i) {
        if (scanf("%63s %63s", a, b) != 2) { fprintf(stderr, "bad input\n"); exit(1); }
        s->w[i] = strtof(a, NULL);
        s->v[i] = strtof(b, NULL);
    }
}

int main(void) {
    g_alpha = (float)sqrt(2.0 / 3.0);
    g_beta = (float)(1.0 / sqrt(5.0));
    int ncie;
    if (scanf("%d", &ncie) != 1) return 1;
    Interp X, Y, Z;
    X.n = Y.n = Z.n = ncie;
    X.w = malloc(sizeof(float) * ncie); X.v = malloc(sizeof(float) * ncie);
    Y.w = X.w; Y.v = malloc(sizeof(float) * ncie);
    Z.w = X.w; Z.v = malloc(sizeof(float) * ncie);
    char l[64], x[64], y[64], z[64];
    for (int i = 0; i < ncie; ++i) {
        if (scanf("%63s %63s %63s %63s", l, x, y, z) != 4) return 1;
        X.w[i] = strtof(l, NULL); X.v[i] = strtof(x, NULL); Y.v[i] = strtof(y, NULL); Z.v[i] = strtof(z, NULL);
    }
    const float start = X.w[0], end = X.w[ncie - 1];
    char name[256];
    int n;
    while (scanf("%255s %d", name, &n) == 2) {
        Interp s;
        read_interp(&s, n);
        g_s1 = &s;
        g_s2 = &X; float Xv = continuous_average(start, end);
        g_s2 = &Y; float Yv = continuous_average(start, end);
        g_s2 = &Z; float Zv = continuous_average(start, end);
        float normalization = 1.0f / interp_average(&Y, start, end);
        Xv *= normalization; Yv *= normalization; Zv *= normalization;
        float r = 3.240479f * Xv + -1.537150f * Yv + -0.498535f * Zv;
        float g = -0.969256f * Xv + 1.875991f * Yv + 0.041556f * Zv;
        float b = 0.055648f * Xv + -0.204043f * Yv + 1.057311f * Zv;
        printf("%s %a %a %a\n", name, r, g, b);
        free(s.w); free(s.v);
    }
    return 0;
}
