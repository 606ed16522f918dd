/* rtrans_gen.c -- generate rough-transmittance tables in the format of
 * Mitsuba's data/microfacet/<distribution>.dat (read by RoughTransmittance,
 * src/bsdfs/rtrans.h:46-150), for machines without the reference's data files.
 *
 * The quantity follows the reference's generator (src/utils/rdielprec.cpp):
 * for relative IOR eta, roughness alpha and incident cosine mu, the
 * transmittance of a rough dielectric boundary in importance mode,
 *   T = E_m[ (1 - F(wi.m)) G1(wi,m) G1(wo,m) |wi.m| / (cos(wi) cos(m)) ],
 * with m drawn from D(m) cos(m) and wo = refract(wi, m) below the surface
 * (the expectation of roughdielectric's sample() weight, roughdielectric.cpp:
 * 423-500); alpha = 0 is the smooth dielectric's 1 - F.  The diffuse
 * transmittance is int_0^1 2 mu T(mu) dmu over the cubic interpolant of the
 * theta table, as diffTransmittanceIntegrand does.  Grids (rdielprec.cpp:
 * 60-180): ior = iorStart + (iorEnd - iorStart) t^4, alpha likewise,
 * cos(theta) = t^4 with t(0) = step/10; the second block is the inverted
 * interface (intIOR 1, extIOR ior).  Ranges and sizes are those in the
 * headers of the reference's shipped files (ggx/beckmann: 50 x 50 x 100,
 * alpha in [0, 4]; phong: 50 x 30 x 100, alpha in [0, 0.5]).
 *
 * The reference integrates with adaptive cubature to 1e-6; this tool uses
 * Gauss-Legendre quadrature on panels graded geometrically toward both ends
 * of the D-sampling coordinate (the distributions' tails) and the trapezoid
 * rule in phi, in double precision, so its values agree with the shipped
 * files to the tolerance DESIGN.md states, not bit for bit.
 *
 * usage: rtrans_gen <beckmann|ggx|phong> <out.dat> [threads]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <omp.h>

enum { BECKMANN = 0, GGX = 1, PHONG = 2 };

#define NODES 4          /* Gauss-Legendre nodes per u1 panel */
#define NPHI 48          /* trapezoid nodes in phi (periodic: exponential convergence) */
#define GRADE 40         /* geometric panels toward u1 = 0 and u1 = 1 (the distributions' tails) */
static double gl_x[NODES], gl_w[NODES];
static double pan[2 * GRADE + 10];
static int npan = 0;

static void make_panels(void) { /* 0, 2^-40 .. 2^-2, 8 uniform on [1/4, 3/4], 1 - 2^-2 .. 1 - 2^-40, 1 */
    pan[npan++] = 0;
    for (int k = GRADE; k >= 3; --k) pan[npan++] = ldexp(1.0, -k);
    for (int k = 0; k <= 8; ++k) pan[npan++] = 0.25 + 0.5 * k / 8;
    for (int k = 3; k <= GRADE; ++k) pan[npan++] = 1 - ldexp(1.0, -k);
    pan[npan++] = 1;
}

static void gauss_legendre(void) { /* nodes/weights on [0,1] by Newton on P_n */
    for (int i = 0; i < NODES; ++i) {
        double x = cos(M_PI * (i + 0.75) / (NODES + 0.5)), dp = 0;
        for (int it = 0; it < 100; ++it) {
            double p0 = 1, p1 = x;
            for (int k = 2; k <= NODES; ++k) { double p2 = ((2 * k - 1) * x * p1 - (k - 1) * p0) / k; p0 = p1; p1 = p2; }
            dp = NODES * (x * p1 - p0) / (x * x - 1);
            double dx = p1 / dp;
            x -= dx;
            if (fabs(dx) < 1e-16) break;
        }
        gl_x[i] = 0.5 * (1 - x);
        gl_w[i] = 1.0 / ((1 - x * x) * dp * dp);
    }
}

typedef struct { double x, y, z; } V;
static double dotv(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

/* Smith G1 (microfacet.h:477-518), isotropic */
static double smith_g1(int type, double alpha, V v, V m) {
    if (dotv(v, m) * v.z <= 0) return 0.0;
    double t2 = 1 - v.z * v.z;
    if (t2 <= 0) return 1.0;
    double tanTheta = fabs(sqrt(t2) / v.z);
    if (tanTheta == 0) return 1.0;
    if (type == GGX) {
        double root = alpha * tanTheta;
        return 2.0 / (1.0 + sqrt(1.0 + root * root));
    }
    double a = 1.0 / (alpha * tanTheta);
    if (a >= 1.6) return 1.0;
    double a2 = a * a;
    return (3.535 * a + 2.181 * a2) / (1.0 + 2.276 * a + 2.577 * a2);
}

/* fresnelDielectricExt (util.cpp:651-677) */
static double fresnel(double cosThetaI_, double *cosThetaT_, double eta) {
    if (eta == 1) { *cosThetaT_ = -cosThetaI_; return 0.0; }
    double scale = (cosThetaI_ > 0) ? 1 / eta : eta, cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0) { *cosThetaT_ = 0.0; return 1.0; }
    double cosThetaI = fabs(cosThetaI_), cosThetaT = sqrt(cosThetaTSqr);
    double Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    double Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    *cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return 0.5 * (Rs * Rs + Rp * Rp);
}

/* transmittance for wi = (sqrt(1-mu^2), 0, mu) */
static double transmittance(int type, double eta, double alpha, double mu) {
    V wi = {sqrt(fmax(0.0, 1 - mu * mu)), 0, mu};
    if (alpha == 0) { double ct; return 1 - fresnel(mu, &ct, eta); }
    if (alpha < 1e-4) alpha = 1e-4;                       /* microfacet.h:89-90 */
    double expo = fmax(2.0 / (alpha * alpha) - 2.0, 0.0); /* computePhongExponent */
    double sum = 0;
    for (int pi = 0; pi + 1 < npan; ++pi)
        for (int i = 0; i < NODES; ++i) {
            double h = pan[pi + 1] - pan[pi];
            double u1 = pan[pi] + h * gl_x[i], w1 = gl_w[i] * h;
            double cosM, tan2;
            if (type == BECKMANN) { tan2 = -alpha * alpha * log(1 - u1); cosM = 1 / sqrt(1 + tan2); }
            else if (type == GGX) { tan2 = alpha * alpha * u1 / (1 - u1); cosM = 1 / sqrt(1 + tan2); }
            else { cosM = pow(u1, 1 / (expo + 2)); }
            double sinM = sqrt(fmax(0.0, 1 - cosM * cosM));
            for (int j = 0; j < NPHI; ++j) {
                    double w2 = 1.0 / NPHI;
                    double phi = 2 * M_PI * (j + 0.5) / NPHI;
                    V m = {sinM * cos(phi), sinM * sin(phi), cosM};
                    double wim = dotv(wi, m), ct;
                    double F = fresnel(wim, &ct, eta);
                    if (ct == 0) continue;
                    double e = ct < 0 ? 1 / eta : eta;      /* refract (util.cpp:767-771) */
                    double k = wim * e + ct;
                    V wo = {m.x * k - wi.x * e, m.y * k - wi.y * e, m.z * k - wi.z * e};
                    if (wi.z * wo.z >= 0) continue;
                    double G = smith_g1(type, alpha, wi, m) * smith_g1(type, alpha, wo, m);
                    sum += w1 * w2 * (1 - F) * G * fabs(wim) / (mu * cosM);
                }
        }
    return sum;
}

/* interpCubic1D = evalCubicInterp1D on [0,1] (spline.cpp:23-60), in double */
static double cubic1d(double x, const float *v, size_t n) {
    if (!(x >= 0 && x <= 1)) return 0;
    double t = x * (n - 1);
    size_t k = (size_t)t;
    if (k > n - 2) k = n - 2;
    double f0 = v[k], f1 = v[k + 1];
    double d0 = k > 0 ? 0.5 * (v[k + 1] - v[k - 1]) : v[k + 1] - v[k];
    double d1 = k + 2 < n ? 0.5 * (v[k + 2] - v[k]) : v[k + 1] - v[k];
    t -= k;
    double t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s <beckmann|ggx|phong> <out.dat> [threads]\n", argv[0]); return 2; }
    int type = !strcmp(argv[1], "beckmann") ? BECKMANN : !strcmp(argv[1], "ggx") ? GGX : !strcmp(argv[1], "phong") ? PHONG : -1;
    if (type < 0) { fprintf(stderr, "unknown distribution %s\n", argv[1]); return 2; }
    if (argc > 3) omp_set_num_threads(atoi(argv[3]));
    gauss_legendre();
    make_panels();
    const uint64_t nEta = 50, nAlpha = type == PHONG ? 30 : 50, nTheta = 100;
    const float iorStart = 1 + 1e-4f, iorEnd = 4, alphaStart = 0, alphaEnd = type == PHONG ? 0.5f : 4.0f;
    float *trans = (float *)calloc(2 * nEta * nAlpha * nTheta, sizeof(float));
    float *diff = (float *)calloc(2 * nEta * nAlpha, sizeof(float));
    #pragma omp parallel for schedule(dynamic) collapse(2)
    for (int inv = 0; inv < 2; ++inv)
        for (int i = 0; i < (int)nEta; ++i) {
            double t = (double)i / (nEta - 1);
            double ior = iorStart + (iorEnd - iorStart) * pow(t, 4.0);
            double eta = inv ? 1.0 / ior : ior;
            for (uint64_t j = 0; j < nAlpha; ++j) {
                double ta = (double)j / (nAlpha - 1);
                double alpha = alphaStart + (alphaEnd - alphaStart) * pow(ta, 4.0);
                float *row = trans + ((inv * nEta + i) * nAlpha + j) * nTheta;
                double step = 1.0 / (nTheta - 1);
                for (uint64_t k = 0; k < nTheta; ++k) {
                    double tt = k == 0 ? step / 10 : k * step;
                    row[k] = (float)transmittance(type, eta, alpha, pow(tt, 4.0));
                }
                double d = 0; /* int_0^1 2 x T(x^(1/4)-warped) dx */
                for (int p = 0; p < 64; ++p)
                    for (int q = 0; q < NODES; ++q) {
                        double x = (p + gl_x[q]) / 64;
                        d += gl_w[q] / 64 * 2 * x * cubic1d(pow(x, 0.25), row, nTheta);
                    }
                diff[(inv * nEta + i) * nAlpha + j] = (float)d;
            }
        }
    FILE *f = fopen(argv[2], "wb");
    if (!f) { perror(argv[2]); return 1; }
    fwrite("MTS_TRANSMITTANCE", 1, 17, f);
    uint64_t sz[3] = {nEta, nAlpha, nTheta};
    fwrite(sz, 8, 3, f);
    float r[4] = {iorStart, iorEnd, alphaStart, alphaEnd};
    fwrite(r, 4, 4, f);
    for (uint64_t b = 0; b < 2 * nEta; ++b)
        for (uint64_t j = 0; j < nAlpha; ++j) {
            fwrite(trans + (b * nAlpha + j) * nTheta, 4, nTheta, f);
            fwrite(diff + b * nAlpha + j, 4, 1, f);
        }
    fclose(f);
    free(trans); free(diff);
    return 0;
}
