/* rtrans_nd.c -- rough-transmittance tables as the reference computes them.
 *
 * Restates Mitsuba's table generator (src/utils/rdielprec.cpp:40-190) with
 * the reference's own integrator: NDIntegrator's adaptive cubature
 * (src/libcore/quad.cpp:489-1431) -- the degree-7/5 Genz-Malik rule in 2D
 * (:788-967), the 15-point Gauss-Kronrod rule in 1D (:973-1116), the
 * error-keyed region heap (:1123-1224) and the Gladwell "parallel" loop that
 * integrateVectorized selects (:1230-1322, :1423-1431).  The integrand is the
 * weight of roughdielectric's sample() restricted to ETransmission in
 * EImportance mode (src/bsdfs/roughdielectric.cpp:424-511), for alpha = 0
 * the smooth dielectric's 1 - F (src/bsdfs/dielectric.cpp), and the diffuse
 * term integrates 2 mu T(mu^(1/4)) over the theta table's cubic interpolant
 * (rdielprec.cpp:58-62, evalCubicInterp1D src/libcore/spline.cpp:23-60).
 *
 * Microfacet sampling restates src/bsdfs/microfacet.h (sampleAll :287-402,
 * sampleVisible :421-460, sampleVisible11 :573-670, eval :191-238, smithG1
 * :477-518) and util.cpp (fresnelDielectricExt :651-677, refract :767-771).
 *
 * The shipped data/microfacet/<distr>.dat predate two later changes to that code,
 * and the generator state that reproduces them (tests/test_roughplastic_host.py,
 * DESIGN.md 2) is, in double precision (rdielprec.cpp:209 recommends it):
 *   - microfacet normals drawn from D(m)cos(m) (sampleVisible = false), with
 *     the Walter et al. roughness scaling 1.2 - 0.2 sqrt|cos| for beckmann and
 *     ggx (roughdielectric.cpp:445-451) and without it for phong;
 *   - alpha not clamped to 1e-4 (microfacet.h:70-71, :135-136 came later).
 * Alternatives for experiments, by environment variable: RT_VISIBLE (visible-
 * normal sampling as roughdielectric.cpp stands), RT_WALTER / RT_NOWALTER,
 * RT_CLAMP, RT_SERIAL (NDIntegrator::integrate's one-region-at-a-time loop),
 * RT_MAXEVAL / RT_REL (integrator limits), RT_DEBUG=1|2 (per-integral stats |
 * integrand values); build with -DRT_DOUBLE=0 for a single-precision run.
 *
 * Grids: rdielprec.cpp:115-160 (ior = iorStart + (iorEnd - iorStart) t^4,
 * alpha likewise, cos(theta) = t^4 with t(0) = step/10); sizes and ranges as
 * the headers of the shipped files state them (ggx/beckmann 50 x 50 x 100 with
 * alpha in [0, 4]; phong 50 x 30 x 100 with alpha in [0, 0.5]).
 *
 * usage: rtrans_nd <beckmann|ggx|phong> <out.dat> [threads]
 *        rtrans_nd <distr> --cell <inverted> <iorIdx> <alphaIdx>
 *              prints the cell's 100 transmittances and diffuse term (%a)
 *        rtrans_nd <distr> --weights < "alpha eta wx wy wz sx sy walter" lines
 *              prints the integrand (the transmission weight) per line (%a)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <omp.h>

#ifndef RT_DOUBLE
#define RT_DOUBLE 1
#endif
#if RT_DOUBLE
typedef double Float;
#define FS(x) sin(x)
#define FC(x) cos(x)
#define FSQRT(x) sqrt(x)
#define FABS(x) fabs(x)
#define FTAN(x) tan(x)
#define FATAN(x) atan(x)
#define FATAN2(y, x) atan2(y, x)
#define FACOS(x) acos(x)
#define FPOW(x, y) pow(x, y)
#define FEXP(x) exp(x)
#define FFLOOR(x) floor(x)
#define FASTEXP(x) exp(x)
#define FASTLOG(x) log(x)
#define FCOPYSIGN(a, b) copysign(a, b)
#else
typedef float Float;
#define FS(x) sinf(x)
#define FC(x) cosf(x)
#define FSQRT(x) sqrtf(x)
#define FABS(x) fabsf(x)
#define FTAN(x) tanf(x)
#define FATAN(x) atanf(x)
#define FATAN2(y, x) atan2f(y, x)
#define FACOS(x) acosf(x)
#define FPOW(x, y) powf(x, y)
#define FEXP(x) expf(x)
#define FFLOOR(x) floorf(x)
#define FASTEXP(x) ((float)exp((double)(x)))   /* math::fastexp, math.h:185-199 */
#define FASTLOG(x) ((float)log((double)(x)))
#define FCOPYSIGN(a, b) copysignf(a, b)
#endif

#define M_PI_R ((Float)3.14159265358979323846)
#define INV_PI_R ((Float)0.31830988618379067154)
#define INV_TWOPI_R ((Float)0.15915494309189533577)
#define EPS_R ((Float)1e-4f)   /* Epsilon, constants.h:28 (float literal) */

enum { BECKMANN = 0, GGX = 1, PHONG = 2 };

/* generator switches (set in main from the distribution and the environment) */
static int g_parallel = 1, g_debug = 0, g_nowalter = 0, g_noclamp = 0;

static inline Float fmaxr(Float a, Float b) { return a > b ? a : b; }  /* std::max */
static inline Float safe_sqrt(Float v) { return FSQRT(fmaxr((Float)0, v)); }

typedef struct { Float x, y, z; } V;
static inline V v3(Float x, Float y, Float z) { V r = {x, y, z}; return r; }
static inline Float dotv(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

/* ---- math.cpp:25-72 -------------------------------------------------- */
static Float m_erfinv(Float x) {
    Float w = -FASTLOG(((Float)1 - x) * ((Float)1 + x)), p;
    if (w < (Float)5) {
        w = w - (Float)2.5;
        p = (Float)2.81022636e-08;
        p = (Float)3.43273939e-07 + p * w;
        p = (Float)-3.5233877e-06 + p * w;
        p = (Float)-4.39150654e-06 + p * w;
        p = (Float)0.00021858087 + p * w;
        p = (Float)-0.00125372503 + p * w;
        p = (Float)-0.00417768164 + p * w;
        p = (Float)0.246640727 + p * w;
        p = (Float)1.50140941 + p * w;
    } else {
        w = FSQRT(w) - (Float)3;
        p = (Float)-0.000200214257;
        p = (Float)0.000100950558 + p * w;
        p = (Float)0.00134934322 + p * w;
        p = (Float)-0.00367342844 + p * w;
        p = (Float)0.00573950773 + p * w;
        p = (Float)-0.0076224613 + p * w;
        p = (Float)0.00943887047 + p * w;
        p = (Float)1.00167406 + p * w;
        p = (Float)2.83297682 + p * w;
    }
    return p * x;
}
static Float m_erf(Float x) {
    Float a1 = (Float)0.254829592, a2 = (Float)-0.284496736, a3 = (Float)1.421413741;
    Float a4 = (Float)-1.453152027, a5 = (Float)1.061405429, p = (Float)0.3275911;
    Float sign = FCOPYSIGN((Float)1, x);
    x = FABS(x);
    Float t = (Float)1.0 / ((Float)1.0 + p * x);
    Float y = (Float)1.0 - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * FASTEXP(-x * x);
    return sign * y;
}
static Float m_hypot2(Float a, Float b) {
    Float r;
    if (FABS(a) > FABS(b)) { r = b / a; r = FABS(a) * FSQRT((Float)1 + r * r); }
    else if (b != 0) { r = a / b; r = FABS(b) * FSQRT((Float)1 + r * r); }
    else r = 0;
    return r;
}

/* ---- microfacet.h (isotropic instances only: alphaU == alphaV) ------- */
typedef struct { int type; Float alpha; int visible; Float exponent; } Distr;

static void distr_init(Distr *d, int type, Float alpha, int visible) { /* :67-74, :138-144 */
    d->type = type;
    d->alpha = g_noclamp ? alpha : fmaxr(alpha, (Float)1e-4f);
    d->visible = type == PHONG ? 0 : visible;
    d->exponent = 0;
    if (type == PHONG) d->exponent = fmaxr((Float)2 / (d->alpha * d->alpha) - (Float)2, (Float)0); /* :673-676 */
}
static void distr_scale_alpha(Distr *d, Float v) { /* :181-186 */
    d->alpha *= v;
    if (d->type == PHONG) d->exponent = fmaxr((Float)2 / (d->alpha * d->alpha) - (Float)2, (Float)0);
}
static Float distr_eval(const Distr *d, V m) { /* :191-238 */
    if (m.z <= 0) return 0;
    Float cosTheta2 = m.z * m.z;
    Float be = ((m.x * m.x) / (d->alpha * d->alpha) + (m.y * m.y) / (d->alpha * d->alpha)) / cosTheta2;
    Float result;
    if (d->type == BECKMANN) {
        result = FASTEXP(-be) / (M_PI_R * d->alpha * d->alpha * cosTheta2 * cosTheta2);
    } else if (d->type == GGX) {
        Float root = ((Float)1 + be) * cosTheta2;
        result = (Float)1 / (M_PI_R * d->alpha * d->alpha * root * root);
    } else {
        result = FSQRT((d->exponent + 2) * (d->exponent + 2)) * INV_TWOPI_R * FPOW(m.z, d->exponent);
    }
    if (result * m.z < (Float)1e-20f) result = 0;
    return result;
}
static Float distr_smithG1(const Distr *d, V v, V m) { /* :477-518 */
    if (dotv(v, m) * v.z <= 0) return 0;
    Float t2 = (Float)1 - v.z * v.z;                 /* Frame::tanTheta: sqrt(max(0, 1-cos^2))/cos */
    Float tanTheta = FABS(safe_sqrt(t2) / v.z);
    if (tanTheta == 0) return 1;
    Float alpha = d->alpha;                            /* projectRoughness, isotropic */
    if (d->type == GGX) {
        Float root = alpha * tanTheta;
        return (Float)2 / ((Float)1 + m_hypot2((Float)1, root));
    }
    Float a = (Float)1 / (alpha * tanTheta);
    if (a >= (Float)1.6f) return 1;
    Float aSqr = a * a;
    return ((Float)3.535f * a + (Float)2.181f * aSqr) / ((Float)1 + (Float)2.276f * a + (Float)2.577f * aSqr);
}
static V distr_sample_all(const Distr *d, Float sx, Float sy, Float *pdf) { /* :287-402, isotropic */
    Float cosThetaM, sinPhiM, cosPhiM;
    if (d->type == BECKMANN || d->type == GGX) {
        Float phi = ((Float)2 * M_PI_R) * sy;
        sinPhiM = FS(phi); cosPhiM = FC(phi);
        Float alphaSqr = d->alpha * d->alpha;
        if (d->type == BECKMANN) {
            Float tanThetaMSqr = alphaSqr * -FASTLOG((Float)1 - sx);
            cosThetaM = (Float)1 / FSQRT((Float)1 + tanThetaMSqr);
            *pdf = ((Float)1 - sx) / (M_PI_R * d->alpha * d->alpha * cosThetaM * cosThetaM * cosThetaM);
        } else {
            Float tanThetaMSqr = alphaSqr * sx / ((Float)1 - sx);
            cosThetaM = (Float)1 / FSQRT((Float)1 + tanThetaMSqr);
            Float temp = 1 + tanThetaMSqr / alphaSqr;
            *pdf = INV_PI_R / (d->alpha * d->alpha * cosThetaM * cosThetaM * cosThetaM * temp * temp);
        }
    } else {
        Float phiM = ((Float)2 * M_PI_R) * sy;
        sinPhiM = FS(phiM); cosPhiM = FC(phiM);
        cosThetaM = FPOW(sx, (Float)1 / (d->exponent + (Float)2));
        *pdf = FSQRT((d->exponent + 2) * (d->exponent + 2)) * INV_TWOPI_R * FPOW(cosThetaM, d->exponent + (Float)1);
    }
    if (*pdf < (Float)1e-20f) *pdf = 0;
    Float sinThetaM = FSQRT(fmaxr((Float)0, (Float)1 - cosThetaM * cosThetaM));
    return v3(sinThetaM * cosPhiM, sinThetaM * sinPhiM, cosThetaM);
}
static void distr_sample_visible11(const Distr *d, Float thetaI, Float sx, Float sy, Float *slx, Float *sly) { /* :573-670 */
    const Float SQRT_PI_INV = (Float)1 / FSQRT(M_PI_R);
    if (d->type == BECKMANN) {
        if (thetaI < (Float)1e-4f) {
            Float r = FSQRT(-FASTLOG((Float)1 - sx)), ph = (Float)2 * M_PI_R * sy;
            *slx = r * FC(ph); *sly = r * FS(ph);
            return;
        }
        Float tanThetaI = FTAN(thetaI), cotThetaI = (Float)1 / tanThetaI;
        Float a = -1, c = m_erf(cotThetaI);
        Float sample_x = fmaxr(sx, (Float)1e-6f);
        Float fit = 1 + thetaI * ((Float)-0.876f + thetaI * ((Float)0.4265f - (Float)0.0594f * thetaI));
        Float b = c - (1 + c) * FPOW(1 - sample_x, fit);
        Float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * FEXP(-cotThetaI * cotThetaI));
        int it = 0;
        while (++it < 10) {
            if (!(b >= a && b <= c)) b = (Float)0.5f * (a + c);
            Float invErf = m_erfinv(b);
            Float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * FEXP(-invErf * invErf)) - sample_x;
            Float derivative = normalization * (1 - invErf * tanThetaI);
            if (FABS(value) < (Float)1e-5f) break;
            if (value > 0) c = b; else a = b;
            b -= value / derivative;
        }
        *slx = m_erfinv(b);
        *sly = m_erfinv((Float)2 * fmaxr(sy, (Float)1e-6f) - (Float)1);
        return;
    }
    if (thetaI < (Float)1e-4f) {
        Float r = safe_sqrt(sx / (1 - sx)), ph = (Float)2 * M_PI_R * sy;
        *slx = r * FC(ph); *sly = r * FS(ph);
        return;
    }
    Float tanThetaI = FTAN(thetaI), a = 1 / tanThetaI;
    Float G1 = (Float)2 / ((Float)1 + safe_sqrt((Float)1 + (Float)1 / (a * a)));
    Float A = (Float)2 * sx / G1 - (Float)1;
    if (FABS(A) == 1) A -= FCOPYSIGN((Float)1, A) * EPS_R;
    Float tmp = (Float)1 / (A * A - (Float)1), B = tanThetaI;
    Float D = safe_sqrt(B * B * tmp * tmp - (A * A - B * B) * tmp);
    Float s1 = B * tmp - D, s2 = B * tmp + D;
    *slx = (A < 0 || s2 > (Float)1 / tanThetaI) ? s1 : s2;
    Float S;
    if (sy > (Float)0.5f) { S = 1; sy = (Float)2 * (sy - (Float)0.5f); }
    else { S = -1; sy = (Float)2 * ((Float)0.5f - sy); }
    Float z = (sy * (sy * (sy * (-(Float)0.365728915865723) + (Float)0.790235037209296) - (Float)0.424965825137544) + (Float)0.000152998850436920) /
              (sy * (sy * (sy * (sy * (Float)0.169507819808272 - (Float)0.397203533833404) - (Float)0.232500544458471) + (Float)1) - (Float)0.539825872510702);
    *sly = S * z * FSQRT((Float)1 + (*slx) * (*slx));
}
static V distr_sample_visible(const Distr *d, V _wi, Float sx, Float sy) { /* :421-460 */
    V wi = v3(d->alpha * _wi.x, d->alpha * _wi.y, _wi.z);
    Float inv = (Float)1 / FSQRT(dotv(wi, wi));
    wi = v3(wi.x * inv, wi.y * inv, wi.z * inv);
    Float theta = 0, phi = 0;
    if (wi.z < (Float)0.99999) { theta = FACOS(wi.z); phi = FATAN2(wi.y, wi.x); }
    Float sinPhi = FS(phi), cosPhi = FC(phi), slx, sly;
    distr_sample_visible11(d, theta, sx, sy, &slx, &sly);
    Float nx = cosPhi * slx - sinPhi * sly, ny = sinPhi * slx + cosPhi * sly;
    nx *= d->alpha; ny *= d->alpha;
    Float n = (Float)1 / FSQRT(nx * nx + ny * ny + (Float)1.0);
    return v3(-nx * n, -ny * n, n);
}

/* ---- util.cpp:651-677, 767-771 ---------------------------------------- */
static Float fresnel_ext(Float cosThetaI_, Float *cosThetaT_, Float eta) {
    if (eta == 1) { *cosThetaT_ = -cosThetaI_; return 0; }
    Float scale = (cosThetaI_ > 0) ? 1 / eta : eta,
          cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0) { *cosThetaT_ = 0; return 1; }
    Float cosThetaI = FABS(cosThetaI_), cosThetaT = FSQRT(cosThetaTSqr);
    Float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    Float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    *cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return (Float)0.5f * (Rs * Rs + Rp * Rp);
}

/* ---- the integrand: roughdielectric.cpp:424-511, ETransmission, EImportance */
typedef struct { int type, visible; Float alpha, eta; V wi; } Cell;

static Float trans_weight(const Cell *c, Float sx, Float sy) {
    if (sx == 1) sx = 1 - EPS_R;     /* rdielprec.cpp:48-51 */
    if (sy == 1) sy = 1 - EPS_R;
    V wi = c->wi;
    if (c->alpha == 0) {             /* "dielectric": smooth, transmission only */
        Float ct, F = fresnel_ext(wi.z, &ct, c->eta);   /* dielectric.cpp sample(): (1 - F), no TIR test */
        return 1 - F;
    }
    Distr distr, sd;
    /* m_alphaU->eval(its).average(): a ConstantFloatTexture's Spectrum(a), summed
       and scaled by (1.0f / 3) (spectrum.h:481-486; roughdielectric.cpp:206,440) */
    Float a = g_noclamp ? c->alpha : fmaxr(c->alpha, (Float)1e-4f);
    Float avg = ((a + a) + a) * (Float)(1.0f / 3);
    distr_init(&distr, c->type, avg, c->visible);
    sd = distr;
    if (!distr.visible && !g_nowalter) distr_scale_alpha(&sd, (Float)1.2f - (Float)0.2f * FSQRT(FABS(wi.z)));
    Float pdf;
    V m;
    Float sgn = FCOPYSIGN((Float)1, wi.z);
    if (sd.visible) {
        V w = v3(sgn * wi.x, sgn * wi.y, sgn * wi.z);
        m = distr_sample_visible(&sd, w, sx, sy);
        Float G1 = distr_smithG1(&sd, w, m);    /* pdfVisible :462-466 */
        pdf = w.z == 0 ? 0 : G1 * FABS(dotv(w, m)) * distr_eval(&sd, m) / FABS(w.z);
    } else {
        m = distr_sample_all(&sd, sx, sy, &pdf);
    }
    if (pdf == 0) return 0;
    Float ct, F = fresnel_ext(dotv(wi, m), &ct, c->eta);
    Float weight = 1 - F;
    if (ct == 0) return 0;
    Float e = ct < 0 ? 1 / c->eta : c->eta;          /* refract (util.cpp:767-771) */
    Float k = dotv(wi, m) * e + ct;
    V wo = v3(m.x * k - wi.x * e, m.y * k - wi.y * e, m.z * k - wi.z * e);
    if (wi.z * wo.z >= 0) return 0;
    if (distr.visible)
        weight *= distr_smithG1(&distr, wo, m);
    else
        weight *= FABS(distr_eval(&distr, m) * (distr_smithG1(&distr, wi, m) * distr_smithG1(&distr, wo, m))
                       * dotv(wi, m) / (pdf * wi.z));
    return weight;
}

/* ---- NDIntegrator (quad.cpp:489-1431) --------------------------------- */
typedef struct { Float val, err; } EstErr;
typedef struct { Float c[2], h[2], vol; unsigned split; EstErr ee; Float errmax; } Region;
typedef void (*Integrand)(void *ctx, size_t n, const Float *in, Float *out);

static Float rel_error(EstErr e) { return e.val == 0 ? (Float)INFINITY : FABS(e.err / e.val); }

typedef struct {
    unsigned dim, npts;
    Float *pts, *vals;
    size_t cap;
    Float w1, w3, w5, wE1, wE3;
} Rule;

static void rule_reserve(Rule *r, unsigned nR) { /* alloc_rule_pts :619-635 */
    if (nR <= r->cap) return;
    nR *= 2;
    free(r->pts);
    r->pts = (Float *)malloc(sizeof(Float) * nR * r->npts * (r->dim + 1));
    r->vals = r->pts + (size_t)nR * r->npts * r->dim;
    r->cap = nR;
}

static void gm_eval(Rule *r, Integrand f, void *ctx, unsigned nR, Region *R) { /* :813-931, dim = 2 */
    const Float lambda2 = (Float)0.3585685828003180919906451539079374954541;
    const Float lambda4 = (Float)0.9486832980505137995996680633298155601160;
    const Float lambda5 = (Float)0.6882472016116852977216287342936235251269;
    const Float weight2 = (Float)(980.0 / 6561.0), weight4 = (Float)(200.0 / 19683.0);
    const Float weightE2 = (Float)(245.0 / 486.0), weightE4 = (Float)(25.0 / 729.0);
    const Float ratio = (lambda2 * lambda2) / (lambda4 * lambda4);
    const unsigned dim = 2;
    rule_reserve(r, nR);
    Float *pts = r->pts, *vals = r->vals;
    unsigned np = 0;
    for (unsigned iR = 0; iR < nR; ++iR) {
        const Float *c = R[iR].c, *h = R[iR].h;
        Float p[2] = {c[0], c[1]}, wl2[2], wl[2];
        for (unsigned i = 0; i < dim; ++i) wl2[i] = h[i] * lambda2;
        for (unsigned i = 0; i < dim; ++i) wl[i] = h[i] * lambda4;
        /* evalR0_0fs4d (:757-771) */
        Float *q = pts + np * dim;
        q[0] = p[0]; q[1] = p[1]; q += 2;
        for (unsigned i = 0; i < dim; ++i) {
            p[i] = c[i] - wl2[i]; q[0] = p[0]; q[1] = p[1]; q += 2;
            p[i] = c[i] + wl2[i]; q[0] = p[0]; q[1] = p[1]; q += 2;
            p[i] = c[i] - wl[i];  q[0] = p[0]; q[1] = p[1]; q += 2;
            p[i] = c[i] + wl[i];  q[0] = p[0]; q[1] = p[1]; q += 2;
            p[i] = c[i];
        }
        np += 1 + 4 * dim;
        /* evalRR0_0fs (:739-755) */
        for (unsigned i = 0; i < dim - 1; ++i) {
            p[i] = c[i] - wl[i];
            for (unsigned j = i + 1; j < dim; ++j) {
                p[j] = c[j] - wl[j]; q[0] = p[0]; q[1] = p[1]; q += 2;
                p[i] = c[i] + wl[i]; q[0] = p[0]; q[1] = p[1]; q += 2;
                p[j] = c[j] + wl[j]; q[0] = p[0]; q[1] = p[1]; q += 2;
                p[i] = c[i] - wl[i]; q[0] = p[0]; q[1] = p[1]; q += 2;
                p[j] = c[j];
            }
            p[i] = c[i];
        }
        np += 2 * dim * (dim - 1);
        /* evalR_Rfs (:716-737), Gray-code order */
        for (unsigned i = 0; i < dim; ++i) wl[i] = h[i] * lambda5;
        unsigned signs = 0;
        for (unsigned i = 0; i < dim; ++i) p[i] = c[i] + wl[i];
        for (unsigned i = 0;; ++i) {
            q[0] = p[0]; q[1] = p[1]; q += 2;
            unsigned d = __builtin_ctz(~i);
            if (d >= dim) break;
            unsigned mask = 1U << d;
            signs ^= mask;
            p[d] = (signs & mask) ? c[d] - wl[d] : c[d] + wl[d];
        }
        np += 1U << dim;
    }
    f(ctx, np, pts, vals);
    Float diff[2 * 4096 * 2 + 2];   /* reuse of pts as diff in the reference; nR is bounded below */
    Float *df = nR <= 4096 ? diff : (Float *)malloc(sizeof(Float) * dim * nR);
    for (unsigned i = 0; i < dim * nR; ++i) df[i] = 0;
    for (unsigned iR = 0; iR < nR; ++iR) {
        Float val0 = vals[0], sum2 = 0, sum3 = 0, sum4 = 0, sum5 = 0;
        unsigned k, k0 = 1;
        for (k = 0; k < dim; ++k) {
            Float v0 = vals[k0 + 4 * k], v1 = vals[k0 + 4 * k + 1], v2 = vals[k0 + 4 * k + 2], v3_ = vals[k0 + 4 * k + 3];
            sum2 += v0 + v1;
            sum3 += v2 + v3_;
            df[iR * dim + k] += FABS(v0 + v1 - 2 * val0 - ratio * (v2 + v3_ - 2 * val0));
        }
        k0 += 4 * k;
        for (k = 0; k < 2 * dim * (dim - 1); ++k) sum4 += vals[k0 + k];
        k0 += k;
        for (k = 0; k < (1U << dim); ++k) sum5 += vals[k0 + k];
        Float result = R[iR].vol * (r->w1 * val0 + weight2 * sum2 + r->w3 * sum3 + weight4 * sum4 + r->w5 * sum5);
        Float res5th = R[iR].vol * (r->wE1 * val0 + weightE2 * sum2 + r->wE3 * sum3 + weightE4 * sum4);
        R[iR].ee.val = result;
        R[iR].ee.err = FABS(res5th - result);
        vals += r->npts;
    }
    for (unsigned iR = 0; iR < nR; ++iR) {
        Float maxdiff = 0;
        unsigned dm = 0;
        for (unsigned i = 0; i < dim; ++i)
            if (df[iR * dim + i] > maxdiff) { maxdiff = df[iR * dim + i]; dm = i; }
        R[iR].split = dm;
        R[iR].errmax = R[iR].ee.err;
    }
    if (df != diff) free(df);
}

static void gk15_eval(Rule *r, Integrand f, void *ctx, unsigned nR, Region *R) { /* :973-1110 */
    const unsigned n = 8;
    const Float xgk[8] = {(Float)0.991455371120812639206854697526329, (Float)0.949107912342758524526189684047851,
                          (Float)0.864864423359769072789712788640926, (Float)0.741531185599394439863864773280788,
                          (Float)0.586087235467691130294144838258730, (Float)0.405845151377397166906606412076961,
                          (Float)0.207784955007898467600689403773245, (Float)0.000000000000000000000000000000000};
    const Float wg[4] = {(Float)0.129484966168869693270611432679082, (Float)0.279705391489276667901467771423780,
                         (Float)0.381830050505118944950369775488975, (Float)0.417959183673469387755102040816327};
    const Float wgk[8] = {(Float)0.022935322010529224963732008058970, (Float)0.063092092629978553290700663189204,
                          (Float)0.104790010322250183839876322541518, (Float)0.140653259715525918745189590510238,
                          (Float)0.169004726639267902826583426598550, (Float)0.190350578064785409913256402421014,
                          (Float)0.204432940075298892414161999234649, (Float)0.209482141084727828012999174891714};
    rule_reserve(r, nR);
    Float *pts = r->pts, *vals = r->vals;
    unsigned np = 0;
    for (unsigned iR = 0; iR < nR; ++iR) {
        Float c = R[iR].c[0], h = R[iR].h[0];
        pts[np++] = c;
        for (unsigned j = 0; j < (n - 1) / 2; ++j) { Float w = h * xgk[2 * j + 1]; pts[np++] = c - w; pts[np++] = c + w; }
        for (unsigned j = 0; j < n / 2; ++j) { Float w = h * xgk[2 * j]; pts[np++] = c - w; pts[np++] = c + w; }
        R[iR].split = 0;
    }
    f(ctx, np, pts, vals);
    for (unsigned iR = 0; iR < nR; ++iR) {
        Float h = R[iR].h[0];
        Float rg = vals[0] * wg[n / 2 - 1], rk = vals[0] * wgk[n - 1], ra = FABS(rk), asc, mean, err;
        unsigned k = 1;
        for (unsigned j = 0; j < (n - 1) / 2; ++j) {
            Float v = vals[k] + vals[k + 1];
            rg += wg[j] * v; rk += wgk[2 * j + 1] * v;
            ra += wgk[2 * j + 1] * (FABS(vals[k]) + FABS(vals[k + 1]));
            k += 2;
        }
        for (unsigned j = 0; j < n / 2; ++j) {
            rk += wgk[2 * j] * (vals[k] + vals[k + 1]);
            ra += wgk[2 * j] * (FABS(vals[k]) + FABS(vals[k + 1]));
            k += 2;
        }
        R[iR].ee.val = rk * h;
        mean = rk * (Float)0.5f;
        asc = wgk[n - 1] * FABS(vals[0] - mean);
        k = 1;
        for (unsigned j = 0; j < (n - 1) / 2; ++j) { asc += wgk[2 * j + 1] * (FABS(vals[k] - mean) + FABS(vals[k + 1] - mean)); k += 2; }
        for (unsigned j = 0; j < n / 2; ++j) { asc += wgk[2 * j] * (FABS(vals[k] - mean) + FABS(vals[k + 1] - mean)); k += 2; }
        err = FABS(rk - rg) * h;
        ra *= h; asc *= h;
        if (asc != 0 && err != 0) {
            Float scale = FPOW((200 * err / asc), (Float)1.5);
            err = (scale < 1) ? asc * scale : asc;
        }
        R[iR].ee.err = err;
        R[iR].errmax = err;
        vals += 15;
    }
}

/* binary max-heap keyed by errmax (:1123-1224), fdim = 1 */
typedef struct { unsigned n, cap; Region *items; EstErr ee; } Heap;
static void heap_push(Heap *h, Region hi) {
    h->ee.val += hi.ee.val; h->ee.err += hi.ee.err;
    unsigned ins = h->n;
    if (++h->n > h->cap) { h->cap = h->n * 2; h->items = (Region *)realloc(h->items, sizeof(Region) * h->cap); }
    while (ins) {
        unsigned parent = (ins - 1) / 2;
        if (hi.errmax <= h->items[parent].errmax) break;
        h->items[ins] = h->items[parent];
        ins = parent;
    }
    h->items[ins] = hi;
}
static Region heap_pop(Heap *h) {
    Region ret = h->items[0];
    int i = 0, n = (int)--h->n, child;
    h->items[0] = h->items[n];
    while ((child = i * 2 + 1) < n) {
        int largest = h->items[child].errmax <= h->items[i].errmax ? i : child;
        if (++child < n && h->items[largest].errmax < h->items[child].errmax) largest = child;
        if (largest == i) break;
        Region s = h->items[i]; h->items[i] = h->items[largest]; h->items[i = largest] = s;
    }
    h->ee.val -= ret.ee.val; h->ee.err -= ret.ee.err;
    return ret;
}

static void cut_region(Region *R, Region *R2) { /* :579-591 */
    unsigned d = R->split;
    *R2 = *R;
    R->h[d] *= (Float)0.5f;
    R->vol *= (Float)0.5f;
    R2->h[d] = R->h[d]; R2->c[d] = R->c[d];
    R2->vol = R->vol;
    /* make_hypercube recomputes the volume from the halved widths (:522-536) */
    Float vol = 1;
    for (unsigned i = 0; i < 2; ++i) vol *= 2 * R2->h[i];
    R2->vol = vol;
    R->c[d] -= R->h[d];
    R2->c[d] += R->h[d];
}

static size_t g_maxeval = 50000;
static Float g_rel = (Float)1e-6f;   /* NDIntegrator(1, 2, 50000, 0, 1e-6f): rdielprec.cpp:84 */

/* ruleadapt_integrate with parallel = 1 (:1230-1346); returns the re-summed value */
static Float nd_integrate(unsigned dim, Integrand f, void *ctx, size_t maxEval, Float reqAbs, Float reqRel) {
    Rule r = {0};
    r.dim = dim;
    void (*eval)(Rule *, Integrand, void *, unsigned, Region *);
    if (dim == 1) { r.npts = 15; eval = gk15_eval; }
    else {
        r.npts = 1 + 2 * 2 * dim + 2 * dim * (dim - 1) + (1U << dim);
        r.w1 = (Float)(12824 - 9120 * (int)dim + 400 * (int)(dim * dim)) / (Float)19683;   /* :954-958 */
        r.w3 = (Float)(1820 - 400 * (int)dim) / (Float)19683;
        r.w5 = (Float)6859 / (Float)19683 / (Float)(1U << dim);
        r.wE1 = (Float)(729 - 950 * (int)dim + 50 * (int)(dim * dim)) / (Float)729;
        r.wE3 = (Float)(265 - 100 * (int)dim) / (Float)1458;
        eval = gm_eval;
    }
    Heap H = {0};
    H.cap = 1; H.items = (Region *)malloc(sizeof(Region));
    unsigned nRcap = 2;
    Region *R = (Region *)malloc(sizeof(Region) * nRcap);
    /* make_hypercube_range (:538-549) */
    for (unsigned i = 0; i < dim; ++i) { R[0].c[i] = (Float)0.5f * (0 + 1); R[0].h[i] = (Float)0.5f * (1 - 0); }
    Float vol = 1;
    for (unsigned i = 0; i < dim; ++i) vol *= 2 * R[0].h[i];
    R[0].vol = vol;
    R[0].split = 0;
    eval(&r, f, ctx, 1, R);
    heap_push(&H, R[0]);
    size_t numEval = r.npts;
    while (numEval < maxEval || !maxEval) {
        if (H.ee.err <= reqAbs || rel_error(H.ee) <= reqRel) break;
        if (!g_parallel) { /* minimise the number of evaluations (:1315-1321): NDIntegrator::integrate */
            R[0] = heap_pop(&H);
            cut_region(R, R + 1);
            eval(&r, f, ctx, 2, R);
            heap_push(&H, R[0]); heap_push(&H, R[1]);
            numEval += r.npts * 2;
            continue;
        }
        unsigned nR = 0;
        EstErr ee = H.ee;
        do {
            if (nR + 2 > nRcap) { nRcap = (nR + 2) * 2; R = (Region *)realloc(R, nRcap * sizeof(Region)); }
            R[nR] = heap_pop(&H);
            ee.err -= R[nR].ee.err;
            cut_region(R + nR, R + nR + 1);
            numEval += r.npts * 2;
            nR += 2;
            if (ee.err <= reqAbs || rel_error(ee) <= reqRel) break;
        } while (H.n > 0 && (numEval < maxEval || !maxEval));
        eval(&r, f, ctx, nR, R);
        for (unsigned i = 0; i < nR; ++i) heap_push(&H, R[i]);
    }
    Float val = 0, err = 0;
    for (unsigned i = 0; i < H.n; ++i) { val += H.items[i].ee.val; err += H.items[i].ee.err; }
    if (g_debug) fprintf(stderr, "dim %u evals %zu regions %u val %.9g err %.3g\n", dim, numEval, H.n, (double)val, (double)err);
    free(H.items); free(R); free(r.pts);
    return val;
}

static void trans_integrand(void *ctx, size_t n, const Float *in, Float *out) {
    const Cell *c = (const Cell *)ctx;
    for (size_t i = 0; i < n; ++i) {
        out[i] = trans_weight(c, in[2 * i], in[2 * i + 1]);
        if (g_debug > 1) fprintf(stderr, "  f(%.9g, %.9g) = %.9g\n", (double)in[2 * i], (double)in[2 * i + 1], (double)out[i]);
    }
}

typedef struct { const Float *data; size_t res; } DiffCtx;
static Float cubic1d(Float x, const Float *v, size_t size) { /* spline.cpp:23-60, min 0 max 1 */
    if (!(x >= 0 && x <= 1)) return 0;
    Float t = ((x - 0) * (Float)(size - 1)) / (1 - 0);
    size_t k = (size_t)t;
    if (k > size - 2) k = size - 2;
    Float f0 = v[k], f1 = v[k + 1], d0, d1;
    d0 = k > 0 ? (Float)0.5f * (v[k + 1] - v[k - 1]) : v[k + 1] - v[k];
    d1 = k + 2 < size ? (Float)0.5f * (v[k + 2] - v[k]) : v[k + 1] - v[k];
    t = t - (Float)k;
    Float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}
static void diff_integrand(void *ctx, size_t n, const Float *in, Float *out) {
    const DiffCtx *d = (const DiffCtx *)ctx;
    for (size_t i = 0; i < n; ++i) out[i] = 2 * in[i] * cubic1d(FPOW(in[i], (Float)0.25f), d->data, d->res);
}

/* computeTransmittance (rdielprec.cpp:66-112) */
static void compute_cell(int type, int visible, Float ior, Float alpha, int inverted, size_t res, float *outT, float *outDiff) {
    Cell c;
    c.type = type; c.visible = visible; c.alpha = alpha;
    c.eta = inverted ? (Float)1 / ior : ior;     /* intIOR/extIOR swap: m_eta = intIOR / extIOR */
    Float *T = (Float *)malloc(sizeof(Float) * res);
    Float stepSize = (Float)1.0f / (Float)(res - 1);
    for (size_t i = 0; i < res; ++i) {
        Float t = (Float)i * stepSize;
        if (i == 0) t = stepSize / 10;
        Float cosTheta = FPOW(t, (Float)4.0f);
        c.wi = v3(safe_sqrt(1 - cosTheta * cosTheta), 0, cosTheta);
        T[i] = nd_integrate(2, trans_integrand, &c, g_maxeval, 0, g_rel);
        outT[i] = (float)T[i];
    }
    DiffCtx d = {T, res};
    *outDiff = (float)nd_integrate(1, diff_integrand, &d, 50000, 0, (Float)1e-6f);
    free(T);
}

static int parse_type(const char *s) {
    return !strcmp(s, "beckmann") ? BECKMANN : !strcmp(s, "ggx") ? GGX : !strcmp(s, "phong") ? PHONG : -1;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <beckmann|ggx|phong> <out.dat> [threads]\n"
                        "       %s <distr> --cell <inverted> <iorIdx> <alphaIdx>\n", argv[0], argv[0]);
        return 2;
    }
    int type = parse_type(argv[1]);
    if (type < 0) { fprintf(stderr, "unknown distribution %s\n", argv[1]); return 2; }
    /* the shipped tables' generator state (header comment) */
    int visible = 0;
    g_nowalter = type == PHONG;
    g_noclamp = 1;
    if (getenv("RT_VISIBLE")) visible = 1;
    if (getenv("RT_WALTER")) g_nowalter = 0;
    if (getenv("RT_NOWALTER")) g_nowalter = 1;
    if (getenv("RT_CLAMP")) g_noclamp = 0;
    if (getenv("RT_SERIAL")) g_parallel = 0;
    if (getenv("RT_DEBUG")) g_debug = atoi(getenv("RT_DEBUG"));
    if (getenv("RT_MAXEVAL")) g_maxeval = strtoull(getenv("RT_MAXEVAL"), 0, 10);
    if (getenv("RT_REL")) g_rel = (Float)atof(getenv("RT_REL"));
    const uint64_t nEta = 50, nAlpha = type == PHONG ? 30 : 50, nTheta = 100;
    /* rdielprec.cpp:32-36, 119-122 (Float variables from double literals) */
    const Float iorStart = (Float)(1 + 1e-4), iorEnd = 4, alphaStart = 0, alphaEnd = type == PHONG ? (Float)0.5 : (Float)4;
    const Float iorStep = (Float)1.0f / (Float)(nEta - 1), alphaStep = (Float)1.0f / (Float)(nAlpha - 1);
    /* rdielprec.cpp:152-163: the grid in Float from the single-precision header values */
#define IOR_AT(i) ((Float)iorStart + ((Float)iorEnd - (Float)iorStart) * FPOW((Float)(i) * iorStep, (Float)4.0f))
#define ALPHA_AT(j) ((Float)alphaStart + ((Float)alphaEnd - (Float)alphaStart) * FPOW((Float)(j) * alphaStep, (Float)4.0f))
    if (!strcmp(argv[2], "--weights")) {
        /* the integrand itself, for the oracle pinning test: stdin lines
           "alpha eta wx wy wz sx sy walter" -> the transmission weight (%a) */
        double a, e, wx, wy, wz, sx, sy;
        int walter;
        while (scanf("%lf %lf %lf %lf %lf %lf %lf %d", &a, &e, &wx, &wy, &wz, &sx, &sy, &walter) == 8) {
            Cell c;
            c.type = type; c.visible = 0; c.alpha = (Float)a; c.eta = (Float)e;
            c.wi = v3((Float)wx, (Float)wy, (Float)wz);
            g_nowalter = !walter;
            printf("%a\n", (double)trans_weight(&c, (Float)sx, (Float)sy));
        }
        return 0;
    }
    if (!strcmp(argv[2], "--cell")) {
        if (argc < 6) return 2;
        int inv = atoi(argv[3]), i = atoi(argv[4]), j = atoi(argv[5]);
        float T[100], D;
        compute_cell(type, visible, IOR_AT(i), ALPHA_AT(j), inv, nTheta, T, &D);
        for (int k = 0; k < 100; ++k) printf("%a\n", T[k]);
        printf("%a\n", D);
        return 0;
    }
    if (argc > 3) omp_set_num_threads(atoi(argv[3]));
    float *trans = (float *)calloc(2 * nEta * nAlpha * nTheta, sizeof(float));
    float *diff = (float *)calloc(2 * nEta * nAlpha, sizeof(float));
    #pragma omp parallel for schedule(dynamic) collapse(3)
    for (int inv = 0; inv < 2; ++inv)
        for (int i = 0; i < (int)nEta; ++i)
            for (int j = 0; j < (int)nAlpha; ++j) {
                size_t cell = ((size_t)inv * nEta + i) * nAlpha + j;
                compute_cell(type, visible, IOR_AT(i), ALPHA_AT(j), inv, nTheta, trans + cell * nTheta, diff + cell);
            }
    FILE *f = fopen(argv[2], "wb");
    if (!f) { perror(argv[2]); return 1; }
    fwrite("MTS_TRANSMITTANCE", 1, 17, f);   /* rdielprec.cpp:141-150 */
    uint64_t sz[3] = {nEta, nAlpha, nTheta};
    fwrite(sz, 8, 3, f);
    float hdr[4] = {(float)iorStart, (float)iorEnd, (float)alphaStart, (float)alphaEnd};
    fwrite(hdr, 4, 4, f);
    for (uint64_t b = 0; b < 2 * nEta; ++b)
        for (uint64_t j = 0; j < nAlpha; ++j) {
            fwrite(trans + (b * nAlpha + j) * nTheta, 4, nTheta, f);
            fwrite(diff + b * nAlpha + j, 4, 1, f);
        }
    fclose(f);
    free(trans); free(diff);
    return 0;
}
