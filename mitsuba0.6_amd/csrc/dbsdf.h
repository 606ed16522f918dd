// dbsdf.h -- device BSDFs of the path: diffuse, roughconductor, roughdielectric,
// roughplastic and the MicrofacetDistribution they share (Beckmann, GGX,
// Phong/AS), with checkerboard-textured reflectance / roughness.
//
//   src/bsdfs/diffuse.cpp:110-150        src/bsdfs/microfacet.h:67-670
//   src/bsdfs/roughconductor.cpp:257-410 src/bsdfs/roughdielectric.cpp:270-615
//   src/bsdfs/roughplastic.cpp:300-470   src/bsdfs/rtrans.h:179-260
//   src/bsdfs/conductor.cpp:216-283      src/bsdfs/dielectric.cpp:218-333
//   src/bsdfs/plastic.cpp:240-440        src/bsdfs/twosided.cpp:105-175
//   src/libcore/spline.cpp:23-60,236-304 src/textures/checkerboard.cpp
//   src/librender/texture.cpp:112-121
//   src/libcore/util.cpp:651-771 (Fresnel, reflect, refract)
//   src/libcore/math.cpp:25-95 (erf, erfinv, hypot2)
#pragma once
#include "dmath.h"
#include "layout.h"

enum { DISTR_BECKMANN = 0, DISTR_GGX = 1, DISTR_PHONG = 2 };

#ifdef MTSG_BSDF_INLINE
#define BSDF_CALL __device__ __forceinline__
#else
#define BSDF_CALL __device__ __noinline__
#endif
// out-of-line microfacet / Fresnel helpers of the generic BSDF set
// (MTSG_HELPER_INLINE: every set inlines them, an A/B knob)
#ifdef MTSG_HELPER_INLINE
#define HELPER_CALL __device__ __forceinline__
#else
#define HELPER_CALL __device__ __noinline__
#endif
enum { BSDF_DIFFUSE = 0, BSDF_ROUGHCONDUCTOR = 1, BSDF_ROUGHDIELECTRIC = 2, BSDF_ROUGHPLASTIC = 3,
       BSDF_CONDUCTOR = 4, BSDF_DIELECTRIC = 5, BSDF_PLASTIC = 6, BSDF_TWOSIDED = 7 };   // = MTSGPU_BSDF_*

__device__ __forceinline__ float tan_theta(f3 v) {           // frame.h:117-122
    float temp = 1 - v.z * v.z;
    if (temp <= 0.0f) return 0.0f;
    return dsqrt(temp) / v.z;
}
__device__ __forceinline__ float sin_theta2(f3 v) { return 1.0f - v.z * v.z; }

// ---- warps (warp.cpp:43-102) --------------------------------------------
__device__ __forceinline__ f3 square_to_cosine_hemisphere(float sx, float sy) {
    float r1 = 2.0f * sx - 1.0f;
    float r2 = 2.0f * sy - 1.0f;
    float phi, r;
    if (r1 == 0 && r2 == 0) {
        r = phi = 0;
    } else if (r1 * r1 > r2 * r2) {
        r = r1;
        phi = (D_PI / 4.0f) * (r2 / r1);
    } else {
        r = r2;
        phi = (D_PI / 2.0f) - (r1 / r2) * (D_PI / 4.0f);
    }
    float c, s;
    d_sincos(phi, &s, &c);
    float px = r * c, py = r * s;
    float z = safe_sqrt(1.0f - px * px - py * py);
    if (z == 0) z = 1e-10f;
    return mk(px, py, z);
}

// ---- math.cpp --------------------------------------------------------------
HELPER_CALL float m_erfinv(float x) {
    float w = -d_fastlog(((float)1 - x) * ((float)1 + x));
    float p;
    if (w < (float)5) {
        w = w - (float)2.5;
        p = (float)2.81022636e-08;
        p = (float)3.43273939e-07 + p * w;
        p = (float)-3.5233877e-06 + p * w;
        p = (float)-4.39150654e-06 + p * w;
        p = (float)0.00021858087 + p * w;
        p = (float)-0.00125372503 + p * w;
        p = (float)-0.00417768164 + p * w;
        p = (float)0.246640727 + p * w;
        p = (float)1.50140941 + p * w;
    } else {
        w = dsqrt(w) - (float)3;
        p = (float)-0.000200214257;
        p = (float)0.000100950558 + p * w;
        p = (float)0.00134934322 + p * w;
        p = (float)-0.00367342844 + p * w;
        p = (float)0.00573950773 + p * w;
        p = (float)-0.0076224613 + p * w;
        p = (float)0.00943887047 + p * w;
        p = (float)1.00167406 + p * w;
        p = (float)2.83297682 + p * w;
    }
    return p * x;
}
__device__ __forceinline__ float m_erf(float x) {
    float a1 = (float)0.254829592, a2 = (float)-0.284496736, a3 = (float)1.421413741;
    float a4 = (float)-1.453152027, a5 = (float)1.061405429, p = (float)0.3275911;
    float sign = signum(x);
    x = fabsf(x);
    float t = (float)1.0 / ((float)1.0 + p * x);
    float y = (float)1.0 - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * d_fastexp(-x * x);
    return sign * y;
}
__device__ __forceinline__ float m_hypot2(float a, float b) {
    float r;
    if (fabsf(a) > fabsf(b)) { r = b / a; r = fabsf(a) * dsqrt(1.0f + r * r); }
    else if (b != 0.0f) { r = a / b; r = fabsf(b) * dsqrt(1.0f + r * r); }
    else r = 0.0f;
    return r;
}

// ---- MicrofacetDistribution -----------------------------------------------
struct Distr { int type; float alphaU, alphaV; int sampleVisible; float expU, expV; };

// ---- the compile-time BSDF set of a kernel variant ------------------------
// BS = the variant's MTSG_FEAT_* bits that select BSDF code (BSET_BITS): EXT
// (roughplastic, textures, smooth BSDFs, twosided), DIFF (every BSDF diffuse),
// GGX (every rough BSDF of the scene uses the GGX distribution), NORC / NORD
// (no roughconductor / roughdielectric).  The reference dispatches per vertex
// through BSDF's virtual eval/sample (src/integrators/path/path.cpp:171-211);
// here the scene's set is known before the launch, so a specialised variant
// compiles only the lobes and the distribution the scene has, and inlines the
// microfacet helpers that the generic set calls out of line
// (profiles/r03_ab_spec_C*.log).
#define BSET_BITS (MTSG_FEAT_EXT | MTSG_FEAT_DIFF | MTSG_FEAT_GGX | MTSG_FEAT_NORC | MTSG_FEAT_NORD | MTSG_FEAT_INL)
template <int BS> struct BSet {
    static constexpr bool EXT = (BS & MTSG_FEAT_EXT) != 0, DIFF = (BS & MTSG_FEAT_DIFF) != 0;
    static constexpr bool GGX = (BS & MTSG_FEAT_GGX) != 0;
    static constexpr bool RC = (BS & MTSG_FEAT_NORC) == 0, RD = (BS & MTSG_FEAT_NORD) == 0;
    // helpers inline in specialised sets (GGX) and in the wavefront engine's per-type kernels (INL)
    static constexpr bool INL = GGX || (BS & MTSG_FEAT_INL) != 0;
};
// the distribution type as the variant knows it
template <int BS> __device__ __forceinline__ int dtype(const Distr &d) { return BSet<BS>::GGX ? (int)DISTR_GGX : d.type; }
// BSDF records are read straight from global memory (no generic/flat loads)
typedef const __attribute__((address_space(1))) MtsgBsdf GBsdf;

__device__ __forceinline__ void distr_phong_exp(Distr &d) {      // microfacet.h:673-676
    d.expU = smax(2.0f / (d.alphaU * d.alphaU) - 2.0f, 0.0f);
    d.expV = smax(2.0f / (d.alphaV * d.alphaV) - 2.0f, 0.0f);
}
__device__ __forceinline__ Distr distr_make(int type, float au, float av, int sv) {  // :89-97
    Distr d;
    d.type = type; d.alphaU = smax(au, 1e-4f); d.alphaV = smax(av, 1e-4f);
    d.sampleVisible = sv; d.expU = d.expV = 0.0f;
    if (type == DISTR_PHONG) distr_phong_exp(d);
    return d;
}
__device__ __forceinline__ bool distr_iso(const Distr &d) { return d.alphaU == d.alphaV; }

__device__ __forceinline__ float distr_interp_phong(const Distr &d, f3 v) {   // :538-549
    float st2 = sin_theta2(v);
    if (distr_iso(d) || st2 <= 0x1p-128f) return d.expU;
    float inv = 1 / st2;
    return d.expU * (v.x * v.x * inv) + d.expV * (v.y * v.y * inv);
}

template <int BS>
__device__ __forceinline__ float distr_eval_b(Distr d, f3 m) {   // :191-238
    if (m.z <= 0) return 0.0f;
    float cosTheta2 = m.z * m.z;
    float be = ((m.x * m.x) / (d.alphaU * d.alphaU) + (m.y * m.y) / (d.alphaV * d.alphaV)) / cosTheta2;
    float result;
    if (dtype<BS>(d) == DISTR_BECKMANN) {
        result = d_fastexp(-be) / (D_PI * d.alphaU * d.alphaV * cosTheta2 * cosTheta2);
    } else if (dtype<BS>(d) == DISTR_GGX) {
        float root = ((float)1 + be) * cosTheta2;
        result = (float)1 / (D_PI * d.alphaU * d.alphaV * root * root);
    } else {
        float exponent = distr_interp_phong(d, m);
        result = dsqrt((d.expU + 2) * (d.expV + 2)) * D_INV_TWOPI * d_powf(m.z, exponent);
    }
    if (result * m.z < 1e-20f) result = 0;
    return result;
}
template <int BS> HELPER_CALL float distr_eval_o(Distr d, f3 m) { return distr_eval_b<BS>(d, m); }
template <int BS> __device__ __forceinline__ float distr_eval(Distr d, f3 m) {
    if constexpr (BSet<BS>::INL) return distr_eval_b<BS>(d, m);
    else return distr_eval_o<BS>(d, m);
}

__device__ __forceinline__ float distr_project_roughness(const Distr &d, f3 v) {   // :526-536
    float invSinTheta2 = 1 / sin_theta2(v);
    if (distr_iso(d) || invSinTheta2 <= 0) return d.alphaU;
    float cosPhi2 = v.x * v.x * invSinTheta2;
    float sinPhi2 = v.y * v.y * invSinTheta2;
    return dsqrt(cosPhi2 * d.alphaU * d.alphaU + sinPhi2 * d.alphaV * d.alphaV);
}

template <int BS>
__device__ __forceinline__ float distr_smithG1_b(Distr d, f3 v, f3 m) {   // :477-518
    if (dot(v, m) * v.z <= 0) return 0.0f;
    float tanTheta = fabsf(tan_theta(v));
    if (tanTheta == 0.0f) return 1.0f;
    float alpha = distr_project_roughness(d, v);
    if (dtype<BS>(d) == DISTR_GGX) {
        float root = alpha * tanTheta;
        return 2.0f / (1.0f + m_hypot2((float)1.0f, root));
    }
    float a = 1.0f / (alpha * tanTheta);
    if (a >= 1.6f) return 1.0f;
    float aSqr = a * a;
    return (3.535f * a + 2.181f * aSqr) / (1.0f + 2.276f * a + 2.577f * aSqr);
}
template <int BS> HELPER_CALL float distr_smithG1_o(Distr d, f3 v, f3 m) { return distr_smithG1_b<BS>(d, v, m); }
template <int BS> __device__ __forceinline__ float distr_smithG1(Distr d, f3 v, f3 m) {
    if constexpr (BSet<BS>::INL) return distr_smithG1_b<BS>(d, v, m);
    else return distr_smithG1_o<BS>(d, v, m);
}

__device__ __forceinline__ void distr_first_quadrant(const Distr &d, float u1, float &phi, float &exponent) {
    float c, s;                                                           // :679-688
    phi = d_atan(dsqrt((d.expU + 2.0f) / (d.expV + 2.0f)) * d_tan(D_PI * u1 * 0.5f));
    d_sincos(phi, &s, &c);
    exponent = d.expU * c * c + d.expV * s * s;
}

template <int BS>
__device__ __forceinline__ f3 distr_sample_all_impl(Distr d, float sx, float sy, float &pdf) {  // :287-402
    float cosThetaM = 0.0f, sinPhiM, cosPhiM, alphaSqr;
    if (dtype<BS>(d) != DISTR_PHONG) {
        if (distr_iso(d)) {
            d_sincos((2.0f * D_PI) * sy, &sinPhiM, &cosPhiM);
            alphaSqr = d.alphaU * d.alphaU;
        } else {
            float phiM = d_atan(d.alphaV / d.alphaU * d_tan(D_PI + 2 * D_PI * sy)) + D_PI * floorf(2 * sy + 0.5f);
            d_sincos(phiM, &sinPhiM, &cosPhiM);
            float cosSc = cosPhiM / d.alphaU, sinSc = sinPhiM / d.alphaV;
            alphaSqr = 1.0f / (cosSc * cosSc + sinSc * sinSc);
        }
        if (dtype<BS>(d) == DISTR_BECKMANN) {
            float tanThetaMSqr = alphaSqr * -d_fastlog(1.0f - sx);
            cosThetaM = 1.0f / dsqrt(1.0f + tanThetaMSqr);
            pdf = (1.0f - sx) / (D_PI * d.alphaU * d.alphaV * cosThetaM * cosThetaM * cosThetaM);
        } else {
            float tanThetaMSqr = alphaSqr * sx / (1.0f - sx);
            cosThetaM = 1.0f / dsqrt(1.0f + tanThetaMSqr);
            float temp = 1 + tanThetaMSqr / alphaSqr;
            pdf = D_INV_PI / (d.alphaU * d.alphaV * cosThetaM * cosThetaM * cosThetaM * temp * temp);
        }
    } else {
        float phiM, exponent;
        if (distr_iso(d)) {
            phiM = (2.0f * D_PI) * sy;
            exponent = d.expU;
        } else {
            if (sy < 0.25f) {
                distr_first_quadrant(d, 4 * sy, phiM, exponent);
            } else if (sy < 0.5f) {
                distr_first_quadrant(d, 4 * (0.5f - sy), phiM, exponent);
                phiM = D_PI - phiM;
            } else if (sy < 0.75f) {
                distr_first_quadrant(d, 4 * (sy - 0.5f), phiM, exponent);
                phiM += D_PI;
            } else {
                distr_first_quadrant(d, 4 * (1 - sy), phiM, exponent);
                phiM = 2 * D_PI - phiM;
            }
        }
        d_sincos(phiM, &sinPhiM, &cosPhiM);
        cosThetaM = d_powf(sx, 1.0f / (exponent + 2.0f));
        pdf = dsqrt((d.expU + 2.0f) * (d.expV + 2.0f)) * D_INV_TWOPI * d_powf(cosThetaM, exponent + 1.0f);
    }
    if (pdf < 1e-20f) pdf = 0;
    float sinThetaM = dsqrt(smax((float)0, 1 - cosThetaM * cosThetaM));
    return mk(sinThetaM * cosPhiM, sinThetaM * sinPhiM, cosThetaM);
}

template <int BS>
__device__ __forceinline__ void distr_sample_visible11_impl(Distr d, float thetaI, float sx, float sy,
                                                           float &slx, float &sly) {   // :573-670
    const float SQRT_PI_INV = 1 / dsqrt(D_PI);
    if (dtype<BS>(d) == DISTR_BECKMANN) {
        if (thetaI < 1e-4f) {
            float s, c;
            float r = dsqrt(-d_fastlog(1.0f - sx));
            d_sincos(2 * D_PI * sy, &s, &c);
            slx = r * c; sly = r * s;
            return;
        }
        float tanThetaI = d_tan(thetaI);
        float cotThetaI = 1 / tanThetaI;
        float a = -1, c = m_erf(cotThetaI);
        float sample_x = smax(sx, (float)1e-6f);
        float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
        float b = c - (1 + c) * d_powf(1 - sample_x, fit);
        float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * d_expf(-cotThetaI * cotThetaI));
        int it = 0;
        while (++it < 10) {
            if (!(b >= a && b <= c)) b = 0.5f * (a + c);
            float invErf = m_erfinv(b);
            float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * d_expf(-invErf * invErf)) - sample_x;
            float derivative = normalization * (1 - invErf * tanThetaI);
            if (fabsf(value) < 1e-5f) break;
            if (value > 0) c = b; else a = b;
            b -= value / derivative;
        }
        slx = m_erfinv(b);
        sly = m_erfinv(2.0f * smax(sy, (float)1e-6f) - 1.0f);
        return;
    }
    if (thetaI < 1e-4f) {                                                       // GGX
        float s, c;
        float r = safe_sqrt(sx / (1 - sx));
        d_sincos(2 * D_PI * sy, &s, &c);
        slx = r * c; sly = r * s;
        return;
    }
    float tanThetaI = d_tan(thetaI);
    float a = 1 / tanThetaI;
    float G1 = 2.0f / (1.0f + safe_sqrt(1.0f + 1.0f / (a * a)));
    float A = 2.0f * sx / G1 - 1.0f;
    if (fabsf(A) == 1) A -= signum(A) * D_EPSILON;
    float tmp = 1.0f / (A * A - 1.0f);
    float B = tanThetaI;
    float D = safe_sqrt(B * B * tmp * tmp - (A * A - B * B) * tmp);
    float slope_x_1 = B * tmp - D;
    float slope_x_2 = B * tmp + D;
    slx = (A < 0.0f || slope_x_2 > 1.0f / tanThetaI) ? slope_x_1 : slope_x_2;
    float S;
    if (sy > 0.5f) { S = 1.0f; sy = 2.0f * (sy - 0.5f); }
    else { S = -1.0f; sy = 2.0f * (0.5f - sy); }
    float z = (sy * (sy * (sy * (-(float)0.365728915865723) + (float)0.790235037209296) - (float)0.424965825137544) + (float)0.000152998850436920) /
              (sy * (sy * (sy * (sy * (float)0.169507819808272 - (float)0.397203533833404) - (float)0.232500544458471) + (float)1) - (float)0.539825872510702);
    sly = S * z * dsqrt(1.0f + slx * slx);
}

// out-of-line entry points return their results by value (no stack round trip)
struct F2 { float x, y; };
struct MPdf { f3 m; float pdf; };
template <int BS> HELPER_CALL F2 distr_sample_visible11_o(Distr d, float thetaI, float sx, float sy) {
    F2 r;
    distr_sample_visible11_impl<BS>(d, thetaI, sx, sy, r.x, r.y);
    return r;
}
template <int BS> __device__ __forceinline__ F2 distr_sample_visible11(Distr d, float thetaI, float sx, float sy) {
    if constexpr (BSet<BS>::INL) {
        F2 r;
        distr_sample_visible11_impl<BS>(d, thetaI, sx, sy, r.x, r.y);
        return r;
    } else {
        return distr_sample_visible11_o<BS>(d, thetaI, sx, sy);
    }
}
template <int BS> HELPER_CALL MPdf distr_sample_all_o(Distr d, float sx, float sy) {
    MPdf r;
    r.m = distr_sample_all_impl<BS>(d, sx, sy, r.pdf);
    return r;
}
template <int BS> __device__ __forceinline__ MPdf distr_sample_all(Distr d, float sx, float sy) {
    if constexpr (BSet<BS>::INL) {
        MPdf r;
        r.m = distr_sample_all_impl<BS>(d, sx, sy, r.pdf);
        return r;
    } else {
        return distr_sample_all_o<BS>(d, sx, sy);
    }
}

template <int BS>
__device__ __forceinline__ f3 distr_sample_visible(const Distr &d, f3 _wi, float sx, float sy) {  // :421-460
    f3 wi = normalize(mk(d.alphaU * _wi.x, d.alphaV * _wi.y, _wi.z));
    float theta = 0, phi = 0;
    if (wi.z < (float)0.99999) {
        theta = d_acos(wi.z);
        phi = d_atan2(wi.y, wi.x);
    }
    float sinPhi, cosPhi;
    d_sincos(phi, &sinPhi, &cosPhi);
    const F2 sl = distr_sample_visible11<BS>(d, theta, sx, sy);
    const float slx = sl.x, sly = sl.y;
    float nx = cosPhi * slx - sinPhi * sly;
    float ny = sinPhi * slx + cosPhi * sly;
    nx *= d.alphaU;
    ny *= d.alphaV;
    float normalization = (float)1 / dsqrt(nx * nx + ny * ny + (float)1.0);
    return mk(-nx * normalization, -ny * normalization, normalization);
}

template <int BS>
__device__ __forceinline__ float distr_pdf_visible(const Distr &d, f3 wi, f3 m) {   // :462-466
    if (wi.z == 0) return 0.0f;
    return distr_smithG1<BS>(d, wi, m) * absdot(wi, m) * distr_eval<BS>(d, m) / fabsf(wi.z);
}
template <int BS>
__device__ __forceinline__ float distr_pdf(const Distr &d, f3 wi, f3 m) {           // :270-276
    if (d.sampleVisible) return distr_pdf_visible<BS>(d, wi, m);
    return distr_eval<BS>(d, m) * m.z;
}
template <int BS>
__device__ __forceinline__ f3 distr_sample(const Distr &d, f3 wi, float sx, float sy, float &pdf) {
    if (d.sampleVisible) {                                                          // :243-253
        f3 m = distr_sample_visible<BS>(d, wi, sx, sy);
        pdf = distr_pdf_visible<BS>(d, wi, m);
        return m;
    }
    const MPdf r = distr_sample_all<BS>(d, sx, sy);
    pdf = r.pdf;
    return r.m;
}
template <int BS>
__device__ __forceinline__ void distr_scale_alpha(Distr &d, float v) {              // :181-186
    d.alphaU *= v; d.alphaV *= v;
    if (dtype<BS>(d) == DISTR_PHONG) distr_phong_exp(d);
}

// ---- Fresnel (util.cpp) -------------------------------------------------
__device__ __forceinline__ float fresnel_dielectric_ext(float cosThetaI_, float &cosThetaT_, float eta) {
    if (eta == 1) { cosThetaT_ = -cosThetaI_; return 0.0f; }
    float scale = (cosThetaI_ > 0) ? 1 / eta : eta,
          cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) { cosThetaT_ = 0.0f; return 1.0f; }
    float cosThetaI = fabsf(cosThetaI_);
    float cosThetaT = dsqrt(cosThetaTSqr);
    float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return 0.5f * (Rs * Rs + Rp * Rp);
}
__device__ __forceinline__ f3 s_safe_sqrt(f3 a) { return mk(safe_sqrt(a.x), safe_sqrt(a.y), safe_sqrt(a.z)); }
__device__ __forceinline__ f3 fresnel_conductor_exact_b(float cosThetaI, f3 eta, f3 k) {   // util.cpp:739-761
    float cosThetaI2 = cosThetaI * cosThetaI, sinThetaI2 = 1 - cosThetaI2, sinThetaI4 = sinThetaI2 * sinThetaI2;
    f3 temp1 = sub(sub(mulv(eta, eta), mulv(k, k)), mk(sinThetaI2, sinThetaI2, sinThetaI2));
    f3 a2pb2 = s_safe_sqrt(add(mulv(temp1, temp1), mul(mulv(mulv(mulv(k, k), eta), eta), 4)));
    f3 a = s_safe_sqrt(mul(add(a2pb2, temp1), 0.5f));
    f3 term1 = add(a2pb2, mk(cosThetaI2, cosThetaI2, cosThetaI2));
    f3 term2 = mul(a, 2 * cosThetaI);
    f3 Rs2 = divv(sub(term1, term2), add(term1, term2));
    f3 term3 = add(mul(a2pb2, cosThetaI2), mk(sinThetaI4, sinThetaI4, sinThetaI4));
    f3 term4 = mul(term2, sinThetaI2);
    f3 Rp2 = divv(mulv(Rs2, sub(term3, term4)), add(term3, term4));
    return mul(add(Rp2, Rs2), 0.5f);
}
HELPER_CALL f3 fresnel_conductor_exact_o(float cosThetaI, f3 eta, f3 k) { return fresnel_conductor_exact_b(cosThetaI, eta, k); }
template <int BS> __device__ __forceinline__ f3 fresnel_conductor_exact(float cosThetaI, f3 eta, f3 k) {
    if constexpr (BSet<BS>::INL) return fresnel_conductor_exact_b(cosThetaI, eta, k);
    else return fresnel_conductor_exact_o(cosThetaI, eta, k);
}
__device__ __forceinline__ f3 reflect_v(f3 wi, f3 n) { return sub(mul(n, 2 * dot(wi, n)), wi); }
__device__ __forceinline__ f3 refract_v(f3 wi, f3 n, float eta, float cosThetaT) {
    if (cosThetaT < 0) eta = 1 / eta;
    return sub(mul(n, dot(wi, n) * eta + cosThetaT), mul(wi, eta));
}

__device__ __forceinline__ f3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ f3 ld3(const __attribute__((address_space(1))) float *p) { return mk(p[0], p[1], p[2]); }

struct BSample { f3 wo; f3 weight; float pdf; float eta; int sampledType; };

// ---- textures (Texture2D::eval, texture.cpp:112-121; checkerboard.cpp) -----
typedef const __attribute__((address_space(1))) MtsgTex GTex;
typedef const __attribute__((address_space(1))) float glb_f32;

// (int) of a float as x86-64 cvttss2si does it: out of range / NaN -> INT_MIN
__device__ __forceinline__ int x86_f2i(float f) {
    return (f > -2147483648.0f && f < 2147483648.0f) ? (int)f : (int)0x80000000u;
}
__device__ __forceinline__ int imodulo(int a, int b) { int r = a % b; return (r < 0) ? r + b : r; }   // math.h:42

__device__ __forceinline__ f3 tex_eval(GTex &t, float u, float v) {
    const float uu = u * t.uscale + t.uoff, vv = v * t.vscale + t.voff;
    const int x = 2 * imodulo(x86_f2i(uu * 2), 2) - 1, y = 2 * imodulo(x86_f2i(vv * 2), 2) - 1;
    return (x * y == 1) ? ld3(t.c0) : ld3(t.c1);
}
__device__ __forceinline__ float avg3(f3 s) { float r = 0.0f; r += s.x; r += s.y; r += s.z; return r * (1.0f / 3); }

// reflectance / diffuseReflectance at the hit (texture or constant)
template <int BS>
__device__ __forceinline__ f3 bsdf_refl(GBsdf &b, float u, float v) {
    if constexpr (BSet<BS>::EXT) { if (b.refl_tex.type) return tex_eval(b.refl_tex, u, v); }
    return ld3(b.refl);
}
// the rough BSDF's distribution at the hit: m_alpha->eval(its).average() for a
// textured alpha (MicrofacetDistribution(type, alpha, sampleVisible) clamps)
template <int BS>
__device__ __forceinline__ Distr bsdf_distr(GBsdf &b, float u, float v) {
    if constexpr (BSet<BS>::EXT) {
        if (b.alpha_tex.type) {
            const float a = avg3(tex_eval(b.alpha_tex, u, v));
            return distr_make(b.distr, a, a, b.sample_visible);
        }
    }
    return distr_make(b.distr, b.alpha_u, b.alpha_v, b.sample_visible);
}

// ---- RoughTransmittance on the eta-reduced tables (rtrans.h:179-260) -------
// evalCubicInterp1D / 2D (spline.cpp:23-60, 236-304), extrapolate = false
__device__ __forceinline__ float cubic1d(float x, glb_f32 *values, uint32_t size) {
    if (!(x >= 0.0f && x <= 1.0f)) return 0.0f;
    float t = ((x - 0.0f) * (float)(size - 1)) / (1.0f - 0.0f);
    uint32_t k = (uint32_t)t;
    if (k > size - 2) k = size - 2;
    const float f0 = values[k], f1 = values[k + 1];
    float d0, d1;
    if (k > 0) d0 = 0.5f * (values[k + 1] - values[k - 1]);
    else d0 = values[k + 1] - values[k];
    if (k + 2 < size) d1 = 0.5f * (values[k + 2] - values[k]);
    else d1 = values[k + 1] - values[k];
    t = t - (float)k;
    const float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}

struct KnotW { uint32_t knot; float w[4]; };
__device__ __forceinline__ bool cubic_weights(float p, uint32_t size, KnotW &k) {
    if (!(p >= 0.0f && p <= 1.0f)) return false;
    float t = ((p - 0.0f) * (float)(size - 1)) / (1.0f - 0.0f);
    uint32_t kn = (uint32_t)t;
    if (kn > size - 2) kn = size - 2;
    k.knot = kn;
    t = t - (float)kn;
    const float t2 = t * t, t3 = t2 * t;
    k.w[0] = 0.0f;
    k.w[1] = 2 * t3 - 3 * t2 + 1;
    k.w[2] = -2 * t3 + 3 * t2;
    k.w[3] = 0.0f;
    const float d0 = t3 - 2 * t2 + t, d1 = t3 - t2;
    if (kn > 0) { k.w[2] += 0.5f * d0; k.w[0] -= 0.5f * d0; }
    else { k.w[2] += d0; k.w[1] -= d0; }
    if (kn + 2 < size) { k.w[3] += 0.5f * d1; k.w[1] -= 0.5f * d1; }
    else { k.w[2] += d1; k.w[1] -= d1; }
    return true;
}

__device__ __noinline__
float cubic2d(float px, float py, glb_f32 *values, uint32_t sx, uint32_t sy) {
    KnotW kx, ky;
    if (!cubic_weights(px, sx, kx)) return 0.0f;
    if (!cubic_weights(py, sy, ky)) return 0.0f;
    float result = 0.0f;
    for (int y = -1; y <= 2; ++y) {
        const float wy = ky.w[y + 1];
        for (int x = -1; x <= 2; ++x) {
            const float wxy = kx.w[x + 1] * wy;
            if (wxy == 0) continue;
            const size_t pos = (size_t)(ky.knot + y) * sx + kx.knot + x;
            result += values[pos] * wxy;
        }
    }
    return result;
}

// warpedAlpha of eval() and evalDiffuse() (rtrans.h:197, 241): a function of the
// vertex's roughness only, so one powf serves every lookup at the vertex (RpPre)
__device__ __forceinline__ float rt_warp_alpha(GBsdf &b, float alpha) {
    return d_powf((alpha - b.rt_alpha_min) / (b.rt_alpha_max - b.rt_alpha_min), 0.25f);
}
// external table: eval(cosTheta, alpha) with m_etaFixed (rtrans.h:184-208), given
// warpedAlpha (unused when the table is reduced to a fixed alpha)
__device__ __forceinline__ float rt_eval_w(GBsdf &b, glb_f32 *rt, float cosTheta, float warpedAlpha) {
    const float warpedCosTheta = d_powf(fabsf(cosTheta), 0.25f);
    if (!(cosTheta >= 0)) return 0.f;
    float result;
    if (b.rt_alpha_fixed) {
        result = cubic1d(warpedCosTheta, rt + b.rt_ext, (uint32_t)b.rt_theta);
    } else {
        result = cubic2d(warpedCosTheta, warpedAlpha, rt + b.rt_ext, (uint32_t)b.rt_theta, (uint32_t)b.rt_alpha);
    }
    return smin(1.0f, smax(0.0f, result));
}
// internal table: evalDiffuse(alpha) with m_etaFixed (rtrans.h:236-247), given warpedAlpha
__device__ __forceinline__ float rt_eval_diffuse_w(GBsdf &b, glb_f32 *rt, float warpedAlpha) {
    const float result = cubic1d(warpedAlpha, rt + b.rt_int, (uint32_t)b.rt_alpha);
    return smin(1.0f, smax(0.0f, result));
}

// RoughPlastic's per-vertex rough-transmittance terms.  eval() forms T12 =
// m_externalRoughTransmittance->eval(cosTheta(wi), alpha) and Fdr = 1 -
// m_internalRoughTransmittance->evalDiffuse(alpha), pdf() and sample() form the
// same T12 for probSpecular (roughplastic.cpp:300-458; rtrans.h:184-208,
// 236-247): they depend only on the vertex (wi and the roughness at the hit),
// so the kernel forms them once per vertex and hands them to every query there
// -- the same values, from 2 instead of 7 table lookups per bounce
// walpha: rt_warp_alpha of the vertex's roughness, for eval()'s T21 lookups too
struct RpPre { float twi, fdr, walpha; };
template <int BS>
__device__ __forceinline__ RpPre rp_pre(GBsdf &b, glb_f32 *rt, f3 wi, float u, float v) {
    const Distr d = bsdf_distr<BS>(b, u, v);
    RpPre p;
    p.walpha = rt_warp_alpha(b, d.alphaU);
    p.twi = rt_eval_w(b, rt, wi.z, p.walpha);
    p.fdr = 1 - rt_eval_diffuse_w(b, rt, p.walpha);
    return p;
}

// the terms for the BSDF `b` queried with `wi` (zero for any other BSDF)
template <int BS>
__device__ __forceinline__ RpPre rp_pre_for(GBsdf &b, glb_f32 *rt, f3 wi, float u, float v) {
    RpPre p = {0.0f, 0.0f, 0.0f};
    if constexpr (BSet<BS>::EXT) {
        if (b.type == BSDF_ROUGHPLASTIC) p = rp_pre<BS>(b, rt, wi, u, v);
    }
    return p;
}

// probSpecular of roughplastic's pdf()/sample() (roughplastic.cpp:371-378, 424-431)
__device__ __forceinline__ float rp_prob_specular(GBsdf &b, float twi) {
    float probSpecular = 1 - twi;
    probSpecular = (probSpecular * b.spec_weight) /
                   (probSpecular * b.spec_weight + (1 - probSpecular) * (1 - b.spec_weight));
    return probSpecular;
}

// RoughPlastic::eval (roughplastic.cpp:300-345)
template <int BS>
__device__ __forceinline__ f3 rp_eval_body(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v, RpPre pre) {
    if (wi.z <= 0 || wo.z <= 0) return mk(0, 0, 0);
    const Distr d = bsdf_distr<BS>(b, u, v);
    f3 result = mk(0, 0, 0);
    {
        const f3 H = normalize(add(wo, wi));
        const float D = distr_eval<BS>(d, H);
        float ct;
        const float F = fresnel_dielectric_ext(dot(wi, H), ct, b.eta);
        const float G = distr_smithG1<BS>(d, wi, H) * distr_smithG1<BS>(d, wo, H);
        const float value = F * D * G / (4.0f * wi.z);
        result = add(result, mul(ld3(b.spec_r), value));
    }
    f3 diff = bsdf_refl<BS>(b, u, v);
    const float T12 = pre.twi;
    const float T21 = rt_eval_w(b, rt, wo.z, pre.walpha);
    const float Fdr = pre.fdr;
    if (b.nonlinear) diff = divv(diff, sub(mk(1.0f, 1.0f, 1.0f), mul(diff, Fdr)));
    else diff = divs(diff, 1 - Fdr);
    return add(result, mul(diff, D_INV_PI * wo.z * T12 * T21 * b.inv_eta2));
}

// RoughPlastic::pdf (roughplastic.cpp:347-393)
template <int BS>
__device__ __forceinline__ float rp_pdf_body(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v, RpPre pre) {
    if (wi.z <= 0 || wo.z <= 0) return 0.0f;
    const Distr d = bsdf_distr<BS>(b, u, v);
    const f3 H = normalize(add(wo, wi));
    const float probSpecular = rp_prob_specular(b, pre.twi);
    const float probDiffuse = 1 - probSpecular;
    const float dwh_dwo = 1.0f / (4.0f * dot(wo, H));
    const float prob = distr_pdf<BS>(d, wi, H);
    float result = prob * dwh_dwo * probSpecular;
    result += probDiffuse * (D_INV_PI * wo.z);
    return result;
}
template <int BS>
BSDF_CALL f3 rp_eval(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v, RpPre pre) {
    return rp_eval_body<BS>(b, rt, wi, wo, u, v, pre);
}
template <int BS>
BSDF_CALL float rp_pdf(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v, RpPre pre) {
    return rp_pdf_body<BS>(b, rt, wi, wo, u, v, pre);
}
struct EvalPdf { f3 val; float pdf; };
// eval, and pdf where the value is nonzero, of one query in one call (NEE)
template <int BS>
BSDF_CALL EvalPdf rp_eval_pdf(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v, RpPre pre) {
    EvalPdf r;
    r.val = rp_eval_body<BS>(b, rt, wi, wo, u, v, pre);
    r.pdf = is_zero(r.val) ? 0.0f : rp_pdf_body<BS>(b, rt, wi, wo, u, v, pre);
    return r;
}

// ---- smooth (delta) BSDFs: conductor, dielectric, plastic ------------------
// eval()/pdf() are only queried by the path's emitter sampling, i.e. with
// measure = ESolidAngle, where the delta lobes contribute nothing
// (conductor.cpp:216-245, dielectric.cpp:228-275): only plastic's diffuse base
// remains (plastic.cpp:245-310).
__device__ __forceinline__ float fresnel_dielectric_ext2(float cosThetaI, float eta) {   // util.cpp:680-683
    float ct;
    return fresnel_dielectric_ext(cosThetaI, ct, eta);
}
__device__ __forceinline__ f3 sp_diffuse(GBsdf &b, float u, float v) {   // diff /= ... (plastic.cpp:276-280)
    f3 diff = bsdf_refl<MTSG_FEAT_EXT>(b, u, v);
    if (b.nonlinear) diff = divv(diff, sub(mk(1.0f, 1.0f, 1.0f), mul(diff, b.fdr_int)));
    else diff = divs(diff, 1 - b.fdr_int);
    return diff;
}
__device__ __forceinline__ float sp_prob_specular(GBsdf &b, float Fi) {   // plastic.cpp:296-299
    return (Fi * b.spec_weight) / (Fi * b.spec_weight + (1 - Fi) * (1 - b.spec_weight));
}
__device__ __noinline__ f3 sm_eval(GBsdf &b, f3 wi, f3 wo, float u, float v) {
    if (b.type != BSDF_PLASTIC) return mk(0, 0, 0);
    if (wo.z <= 0 || wi.z <= 0) return mk(0, 0, 0);
    const float Fi = fresnel_dielectric_ext2(wi.z, b.eta);
    const float Fo = fresnel_dielectric_ext2(wo.z, b.eta);
    return mul(sp_diffuse(b, u, v), D_INV_PI * wo.z * b.inv_eta2 * (1 - Fi) * (1 - Fo));
}
__device__ __noinline__ float sm_pdf(GBsdf &b, f3 wi, f3 wo) {
    if (b.type != BSDF_PLASTIC) return 0.0f;
    if (wo.z <= 0 || wi.z <= 0) return 0.0f;
    const float probSpecular = sp_prob_specular(b, fresnel_dielectric_ext2(wi.z, b.eta));
    return (D_INV_PI * wo.z) * (1 - probSpecular);
}
// sample(bRec, pdf, sample) (conductor.cpp:269-283, dielectric.cpp:277-333, plastic.cpp:356-420)
__device__ __noinline__ BSample sm_sample(GBsdf &b, f3 wi, float sx, float sy, float u, float v) {
    BSample r;
    r.weight = mk(0, 0, 0); r.pdf = 0; r.eta = 1.0f; r.sampledType = 0; r.wo = mk(0, 0, 1);
    if (b.type == BSDF_CONDUCTOR) {
        if (wi.z <= 0) return r;
        r.sampledType = MTSG_F_DELTA_REFL;
        r.wo = mk(-wi.x, -wi.y, wi.z);
        r.eta = 1.0f;
        r.pdf = 1;
        r.weight = mulv(ld3(b.spec_r), fresnel_conductor_exact<0>(wi.z, ld3(b.eta3), ld3(b.k3)));
        return r;
    }
    if (b.type == BSDF_DIELECTRIC) {
        float cosThetaT;
        const float F = fresnel_dielectric_ext(wi.z, cosThetaT, b.eta);
        if (sx <= F) {
            r.sampledType = MTSG_F_DELTA_REFL;
            r.wo = mk(-wi.x, -wi.y, wi.z);
            r.eta = 1.0f;
            r.pdf = F;
            r.weight = ld3(b.spec_r);
        } else {
            const float scale = -(cosThetaT < 0 ? b.inv_eta : b.eta);
            r.sampledType = MTSG_F_DELTA_TRANS;
            r.wo = mk(scale * wi.x, scale * wi.y, cosThetaT);
            r.eta = cosThetaT < 0 ? b.eta : b.inv_eta;
            r.pdf = 1 - F;
            const float factor = cosThetaT < 0 ? b.inv_eta : b.eta;
            r.weight = mul(ld3(b.spec_t), factor * factor);
        }
        return r;
    }
    // plastic
    if (wi.z <= 0) return r;
    const float Fi = fresnel_dielectric_ext2(wi.z, b.eta);
    r.eta = 1.0f;
    const float probSpecular = sp_prob_specular(b, Fi);
    if (sx < probSpecular) {
        r.sampledType = MTSG_F_DELTA_REFL;
        r.wo = mk(-wi.x, -wi.y, wi.z);
        r.pdf = probSpecular;
        r.weight = divs(mul(ld3(b.spec_r), Fi), probSpecular);
    } else {
        r.sampledType = MTSG_F_DIFF_REFL;
        r.wo = square_to_cosine_hemisphere((sx - probSpecular) / (1 - probSpecular), sy);
        const float Fo = fresnel_dielectric_ext2(r.wo.z, b.eta);
        const f3 diff = sp_diffuse(b, u, v);
        r.pdf = (1 - probSpecular) * (D_INV_PI * r.wo.z);
        r.weight = mul(diff, b.inv_eta2 * (1 - Fi) * (1 - Fo) / (1 - probSpecular));
    }
    return r;
}

// ---- BSDF::eval / pdf / sample --------------------------------------------
// one BSDF type's eval / pdf / sample bodies (inlined into the dispatchers
// below, and on their own into the wavefront engine's per-type shade kernels)
template <int BS>
__device__ __forceinline__ f3 diff_eval_body(GBsdf &b, f3 wi, f3 wo, float u, float v) {   // diffuse.cpp:110-117
    if (wi.z <= 0 || wo.z <= 0) return mk(0, 0, 0);
    return mul(bsdf_refl<BS>(b, u, v), D_INV_PI * wo.z);
}
__device__ __forceinline__ float diff_pdf_body(f3 wi, f3 wo) {                            // diffuse.cpp:119-126
    if (wi.z <= 0 || wo.z <= 0) return 0.0f;
    return D_INV_PI * wo.z;
}
template <int BS>
__device__ __forceinline__ f3 rc_eval_body(GBsdf &b, f3 wi, f3 wo, float u, float v) {   // roughconductor.cpp:257-292
    const f3 zero = mk(0, 0, 0);
    if (wi.z <= 0 || wo.z <= 0) return zero;
    f3 H = normalize(add(wo, wi));
    Distr d = bsdf_distr<BS>(b, u, v);
    float D = distr_eval<BS>(d, H);
    if (D == 0) return zero;
    f3 F = mulv(fresnel_conductor_exact<BS>(dot(wi, H), ld3(b.eta3), ld3(b.k3)), ld3(b.spec_r));
    float G = distr_smithG1<BS>(d, wi, H) * distr_smithG1<BS>(d, wo, H);
    float model = D * G / (4.0f * wi.z);
    return mul(F, model);
}
template <int BS>
__device__ __forceinline__ f3 rd_eval_body(GBsdf &b, f3 wi, f3 wo, float u, float v) {   // roughdielectric.cpp:270-346
    const f3 zero = mk(0, 0, 0);
    if (wi.z == 0) return zero;
    bool reflect = wi.z * wo.z > 0;
    f3 H;
    if (reflect) {
        H = normalize(add(wo, wi));
    } else {
        float eta = wi.z > 0 ? b.eta : b.inv_eta;
        H = normalize(add(wi, mul(wo, eta)));
    }
    H = mul(H, signum(H.z));
    Distr d = bsdf_distr<BS>(b, u, v);
    float D = distr_eval<BS>(d, H);
    if (D == 0) return zero;
    float ct;
    float F = fresnel_dielectric_ext(dot(wi, H), ct, b.eta);
    float G = distr_smithG1<BS>(d, wi, H) * distr_smithG1<BS>(d, wo, H);
    if (reflect) {
        float value = F * D * G / (4.0f * fabsf(wi.z));
        return mul(ld3(b.spec_r), value);
    }
    float eta = wi.z > 0.0f ? b.eta : b.inv_eta;
    float sqrtDenom = dot(wi, H) + eta * dot(wo, H);
    float value = ((1 - F) * D * G * eta * eta * dot(wi, H) * dot(wo, H)) / (wi.z * sqrtDenom * sqrtDenom);
    float factor = (wi.z > 0 ? b.inv_eta : b.eta);
    return mul(ld3(b.spec_t), fabsf(value * factor * factor));
}

template <int BS>
__device__ __forceinline__ f3 bsdf_eval_body(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v) {
    if (b.type == BSDF_DIFFUSE) return diff_eval_body<BS>(b, wi, wo, u, v);
    if constexpr (BSet<BS>::EXT) {
        if (b.type == BSDF_ROUGHPLASTIC) return rp_eval<BS>(b, rt, wi, wo, u, v, rp_pre<BS>(b, rt, wi, u, v));
        if (b.type >= BSDF_CONDUCTOR) return sm_eval(b, wi, wo, u, v);
    }
    if (BSet<BS>::RC && (!BSet<BS>::RD || b.type == BSDF_ROUGHCONDUCTOR)) return rc_eval_body<BS>(b, wi, wo, u, v);
    if (!BSet<BS>::RD) return mk(0, 0, 0);
    return rd_eval_body<BS>(b, wi, wo, u, v);
}

template <int BS>
__device__ __forceinline__ float rc_pdf_body(GBsdf &b, f3 wi, f3 wo, float u, float v) {   // roughconductor.cpp:294-319
    if (wi.z <= 0 || wo.z <= 0) return 0.0f;
    f3 H = normalize(add(wo, wi));
    Distr d = bsdf_distr<BS>(b, u, v);
    if (b.sample_visible) return distr_eval<BS>(d, H) * distr_smithG1<BS>(d, wi, H) / (4.0f * wi.z);
    return distr_pdf<BS>(d, wi, H) / (4 * absdot(wo, H));
}
template <int BS>
__device__ __forceinline__ float rd_pdf_body(GBsdf &b, f3 wi, f3 wo, float u, float v) {   // roughdielectric.cpp:348-405
    bool reflect = wi.z * wo.z > 0;
    f3 H;
    float dwh_dwo;
    if (reflect) {
        H = normalize(add(wo, wi));
        dwh_dwo = 1.0f / (4.0f * dot(wo, H));
    } else {
        float eta = wi.z > 0 ? b.eta : b.inv_eta;
        H = normalize(add(wi, mul(wo, eta)));
        float sqrtDenom = dot(wi, H) + eta * dot(wo, H);
        dwh_dwo = (eta * eta * dot(wo, H)) / (sqrtDenom * sqrtDenom);
    }
    H = mul(H, signum(H.z));
    Distr d = bsdf_distr<BS>(b, u, v);
    if (!b.sample_visible) distr_scale_alpha<BS>(d, 1.2f - 0.2f * dsqrt(fabsf(wi.z)));
    float prob = distr_pdf<BS>(d, mul(wi, signum(wi.z)), H);
    float ct;
    float F = fresnel_dielectric_ext(dot(wi, H), ct, b.eta);
    prob *= reflect ? F : (1 - F);
    return fabsf(prob * dwh_dwo);
}

template <int BS>
__device__ __forceinline__ float bsdf_pdf_body(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v) {
    if (b.type == BSDF_DIFFUSE) return diff_pdf_body(wi, wo);
    if constexpr (BSet<BS>::EXT) {
        if (b.type == BSDF_ROUGHPLASTIC) return rp_pdf<BS>(b, rt, wi, wo, u, v, rp_pre<BS>(b, rt, wi, u, v));
        if (b.type >= BSDF_CONDUCTOR) return sm_pdf(b, wi, wo);
    }
    if (BSet<BS>::RC && (!BSet<BS>::RD || b.type == BSDF_ROUGHCONDUCTOR)) return rc_pdf_body<BS>(b, wi, wo, u, v);
    if (!BSet<BS>::RD) return 0.0f;
    return rd_pdf_body<BS>(b, wi, wo, u, v);
}

template <int BS>
BSDF_CALL f3 bsdf_eval(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v) {
    return bsdf_eval_body<BS>(b, rt, wi, wo, u, v);
}
template <int BS>
BSDF_CALL float bsdf_pdf(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v) {
    return bsdf_pdf_body<BS>(b, rt, wi, wo, u, v);
}

// BSDF::eval, then BSDF::pdf of the same query where the value is nonzero
// (the NEE estimate of path.cpp:176-199 needs both): one out-of-line call, so
// the caller's live registers are saved around one call instead of two
template <int BS>
BSDF_CALL EvalPdf bsdf_eval_pdf(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v, RpPre pre) {
    if constexpr (BSet<BS>::EXT) {
        if (b.type == BSDF_ROUGHPLASTIC) return rp_eval_pdf<BS>(b, rt, wi, wo, u, v, pre);
    }
    EvalPdf r;
    r.val = bsdf_eval_body<BS>(b, rt, wi, wo, u, v);
    r.pdf = is_zero(r.val) ? 0.0f : bsdf_pdf_body<BS>(b, rt, wi, wo, u, v);
    return r;
}

// BSDF::sample(bRec, pdf, sample): roughdielectric consumes one more 1D sample
// for the lobe choice (roughdielectric.cpp:554); it is passed in as `u1d` by
// the caller, which draws it from the sampler only for that BSDF.

// RoughPlastic::sample(bRec, pdf, sample) (roughplastic.cpp:395-458); INL:
// its pdf and eval inline (the per-type shade kernels), else the calls
template <int BS, bool INL>
__device__ __forceinline__ BSample rp_sample_body(GBsdf &b, glb_f32 *rt, f3 wi, float sx, float sy, float u, float v,
                                                  RpPre pre) {
    BSample r;
    r.weight = mk(0, 0, 0); r.pdf = 0; r.eta = 1.0f; r.sampledType = 0; r.wo = mk(0, 0, 1);
    if (wi.z <= 0) return r;
    bool choseSpecular = true;
    const Distr d = bsdf_distr<BS>(b, u, v);
    const float probSpecular = rp_prob_specular(b, pre.twi);
    if (sy < probSpecular) {
        sy /= probSpecular;
    } else {
        sy = (sy - probSpecular) / (1 - probSpecular);
        choseSpecular = false;
    }
    if (choseSpecular) {
        float mpdf;
        const f3 m = distr_sample<BS>(d, wi, sx, sy, mpdf);
        r.wo = reflect_v(wi, m);
        r.sampledType = MTSG_F_GLOSSY_REFL;
        if (r.wo.z <= 0) return r;
    } else {
        r.sampledType = MTSG_F_DIFF_REFL;
        r.wo = square_to_cosine_hemisphere(sx, sy);
    }
    r.eta = 1.0f;
    r.pdf = INL ? rp_pdf_body<BS>(b, rt, wi, r.wo, u, v, pre) : rp_pdf<BS>(b, rt, wi, r.wo, u, v, pre);
    if (r.pdf == 0) return r;
    r.weight = divs(INL ? rp_eval_body<BS>(b, rt, wi, r.wo, u, v, pre) : rp_eval<BS>(b, rt, wi, r.wo, u, v, pre),
                    r.pdf);
    return r;
}
template <int BS>
BSDF_CALL BSample rp_sample(GBsdf &b, glb_f32 *rt, f3 wi, float sx, float sy, float u, float v, RpPre pre) {
    return rp_sample_body<BS, false>(b, rt, wi, sx, sy, u, v, pre);
}

__device__ __forceinline__ BSample bsample_zero() {
    BSample r;
    r.weight = mk(0, 0, 0); r.pdf = 0; r.eta = 1.0f; r.sampledType = 0; r.wo = mk(0, 0, 1);
    return r;
}
template <int BS>
__device__ __forceinline__ BSample diff_sample_body(GBsdf &b, f3 wi, float sx, float sy, float u, float v) {
    BSample r = bsample_zero();                                            // diffuse.cpp:139-150
    if (wi.z <= 0) return r;
    r.wo = square_to_cosine_hemisphere(sx, sy);
    r.eta = 1.0f;
    r.sampledType = MTSG_F_DIFF_REFL;
    r.pdf = D_INV_PI * r.wo.z;
    r.weight = bsdf_refl<BS>(b, u, v);
    return r;
}
template <int BS>
__device__ __forceinline__ BSample rc_sample_body(GBsdf &b, f3 wi, float sx, float sy, float u, float v) {
    BSample r = bsample_zero();                                            // roughconductor.cpp:357-406
    if (wi.z < 0) return r;
    Distr d = bsdf_distr<BS>(b, u, v);
    float pdf;
    f3 m = distr_sample<BS>(d, wi, sx, sy, pdf);
    r.pdf = pdf;
    if (pdf == 0) return r;
    r.wo = reflect_v(wi, m);
    r.eta = 1.0f;
    r.sampledType = MTSG_F_GLOSSY_REFL;
    if (r.wo.z <= 0) return r;
    f3 F = mulv(fresnel_conductor_exact<BS>(dot(wi, m), ld3(b.eta3), ld3(b.k3)), ld3(b.spec_r));
    float weight;
    if (b.sample_visible) weight = distr_smithG1<BS>(d, r.wo, m);
    else weight = distr_eval<BS>(d, m) * (distr_smithG1<BS>(d, wi, m) * distr_smithG1<BS>(d, r.wo, m)) * dot(wi, m) / (pdf * wi.z);
    r.pdf = pdf / (4.0f * dot(r.wo, m));
    r.weight = mul(F, weight);
    return r;
}
template <int BS>
__device__ __forceinline__ BSample rd_sample_body(GBsdf &b, f3 wi, float sx, float sy, float u1d, float u, float v) {
    BSample r = bsample_zero();                                            // roughdielectric.cpp:525-615
    Distr d = bsdf_distr<BS>(b, u, v);
    Distr sd = d;
    if (!b.sample_visible) distr_scale_alpha<BS>(sd, 1.2f - 0.2f * dsqrt(fabsf(wi.z)));
    float microfacetPDF;
    f3 m = distr_sample<BS>(sd, mul(wi, signum(wi.z)), sx, sy, microfacetPDF);
    if (microfacetPDF == 0) return r;
    float pdf = microfacetPDF;
    float cosThetaT;
    float F = fresnel_dielectric_ext(dot(wi, m), cosThetaT, b.eta);
    f3 weight = mk(1.0f, 1.0f, 1.0f);
    bool sampleReflection = true;
    if (u1d > F) { sampleReflection = false; pdf *= 1 - F; }
    else pdf *= F;
    float dwh_dwo;
    if (sampleReflection) {
        r.wo = reflect_v(wi, m);
        r.eta = 1.0f;
        r.sampledType = MTSG_F_GLOSSY_REFL;
        if (wi.z * r.wo.z <= 0) { r.pdf = pdf; return r; }
        weight = mulv(weight, ld3(b.spec_r));
        dwh_dwo = 1.0f / (4.0f * dot(r.wo, m));
    } else {
        if (cosThetaT == 0) { r.pdf = pdf; return r; }
        r.wo = refract_v(wi, m, b.eta, cosThetaT);
        r.eta = cosThetaT < 0 ? b.eta : b.inv_eta;
        r.sampledType = MTSG_F_GLOSSY_TRANS;
        if (wi.z * r.wo.z >= 0) { r.pdf = pdf; return r; }
        float factor = cosThetaT < 0 ? b.inv_eta : b.eta;
        weight = mulv(weight, mul(ld3(b.spec_t), factor * factor));
        float sqrtDenom = dot(wi, m) + r.eta * dot(r.wo, m);
        dwh_dwo = (r.eta * r.eta * dot(r.wo, m)) / (sqrtDenom * sqrtDenom);
    }
    if (b.sample_visible) weight = mul(weight, distr_smithG1<BS>(d, r.wo, m));
    else weight = mul(weight, fabsf(distr_eval<BS>(d, m) * (distr_smithG1<BS>(d, wi, m) * distr_smithG1<BS>(d, r.wo, m)) * dot(wi, m) / (microfacetPDF * wi.z)));
    r.pdf = pdf * fabsf(dwh_dwo);
    r.weight = weight;
    return r;
}

template <int BS>
BSDF_CALL BSample bsdf_sample(GBsdf &b, glb_f32 *rt, f3 wi, float sx, float sy, float u1d, float u, float v,
                              RpPre pre) {
    if (b.type == BSDF_DIFFUSE) return diff_sample_body<BS>(b, wi, sx, sy, u, v);
    if constexpr (BSet<BS>::EXT) {
        if (b.type == BSDF_ROUGHPLASTIC) return rp_sample<BS>(b, rt, wi, sx, sy, u, v, pre);
        if (b.type >= BSDF_CONDUCTOR) return sm_sample(b, wi, sx, sy, u, v);
    }
    if (BSet<BS>::RC && (!BSet<BS>::RD || b.type == BSDF_ROUGHCONDUCTOR)) return rc_sample_body<BS>(b, wi, sx, sy, u, v);
    if (!BSet<BS>::RD) return bsample_zero();
    return rd_sample_body<BS>(b, wi, sx, sy, u1d, u, v);
}

// Call-site dispatch.  DIFF_ONLY (MTSG_FEAT_DIFF: every BSDF of the scene is
// diffuse, diffuse.cpp:110-150) evaluates the diffuse lobe inline, so the
// bounce loop makes no out-of-line calls and writes no callee-saved VGPRs to
// scratch around them; otherwise the out-of-line functions above are called.
// (Inlining the diffuse case in front of the calls for every scene cost C3-C5
// 2-4%: profiles/r02_ab_diffuse_fast.log.)
template <int BS>
__device__ __forceinline__ f3 bsdf_eval_fast(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v) {
    if constexpr (BSet<BS>::DIFF) {
        if (wi.z <= 0 || wo.z <= 0) return mk(0, 0, 0);
        return mul(bsdf_refl<BS>(b, u, v), D_INV_PI * wo.z);
    } else {
        return bsdf_eval<BS>(b, rt, wi, wo, u, v);
    }
}
template <int BS>
__device__ __forceinline__ float bsdf_pdf_fast(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v) {
    if constexpr (BSet<BS>::DIFF) {
        if (wi.z <= 0 || wo.z <= 0) return 0.0f;
        return D_INV_PI * wo.z;
    } else {
        return bsdf_pdf<BS>(b, rt, wi, wo, u, v);
    }
}
template <int BS>
__device__ __forceinline__ EvalPdf bsdf_eval_pdf_fast(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v,
                                                      RpPre pre) {
    if constexpr (BSet<BS>::DIFF) {
        EvalPdf r;
        r.val = bsdf_eval_fast<BS>(b, rt, wi, wo, u, v);
        r.pdf = bsdf_pdf_fast<BS>(b, rt, wi, wo, u, v);
        return r;
    } else {
        return bsdf_eval_pdf<BS>(b, rt, wi, wo, u, v, pre);
    }
}
template <int BS>
__device__ __forceinline__ BSample bsdf_sample_fast(GBsdf &b, glb_f32 *rt, f3 wi, float sx, float sy, float u1d,
                                                    float u, float v, RpPre pre) {
    if constexpr (BSet<BS>::DIFF) {
        BSample r;
        r.weight = mk(0, 0, 0); r.pdf = 0; r.eta = 1.0f; r.sampledType = 0; r.wo = mk(0, 0, 1);
        if (wi.z <= 0) return r;
        r.wo = square_to_cosine_hemisphere(sx, sy);
        r.sampledType = MTSG_F_DIFF_REFL;
        r.pdf = D_INV_PI * r.wo.z;
        r.weight = bsdf_refl<BS>(b, u, v);
        return r;
    } else {
        return bsdf_sample<BS>(b, rt, wi, sx, sy, u1d, u, v, pre);
    }
}

// The wavefront engine's per-type shade kernels know the BSDF type of the
// vertex at compile time (KIND = the BSDF_* type; -1: any, dispatched as
// above): one type's body inline, no type dispatch and no calls.
template <int BS, int KIND>
__device__ __forceinline__ EvalPdf bsdf_eval_pdf_k(GBsdf &b, glb_f32 *rt, f3 wi, f3 wo, float u, float v, RpPre pre) {
    EvalPdf r;
    if constexpr (KIND == BSDF_DIFFUSE) {
        r.val = diff_eval_body<BS>(b, wi, wo, u, v);
        r.pdf = is_zero(r.val) ? 0.0f : diff_pdf_body(wi, wo);
    } else if constexpr (KIND == BSDF_ROUGHCONDUCTOR) {
        r.val = rc_eval_body<BS>(b, wi, wo, u, v);
        r.pdf = is_zero(r.val) ? 0.0f : rc_pdf_body<BS>(b, wi, wo, u, v);
    } else if constexpr (KIND == BSDF_ROUGHDIELECTRIC) {
        r.val = rd_eval_body<BS>(b, wi, wo, u, v);
        r.pdf = is_zero(r.val) ? 0.0f : rd_pdf_body<BS>(b, wi, wo, u, v);
    } else if constexpr (KIND == BSDF_ROUGHPLASTIC) {
        r.val = rp_eval_body<BS>(b, rt, wi, wo, u, v, pre);
        r.pdf = is_zero(r.val) ? 0.0f : rp_pdf_body<BS>(b, rt, wi, wo, u, v, pre);
    } else {
        return bsdf_eval_pdf_fast<BS>(b, rt, wi, wo, u, v, pre);
    }
    return r;
}
template <int BS, int KIND>
__device__ __forceinline__ BSample bsdf_sample_k(GBsdf &b, glb_f32 *rt, f3 wi, float sx, float sy, float u1d, float u,
                                                 float v, RpPre pre) {
    if constexpr (KIND == BSDF_DIFFUSE) return diff_sample_body<BS>(b, wi, sx, sy, u, v);
    else if constexpr (KIND == BSDF_ROUGHCONDUCTOR) return rc_sample_body<BS>(b, wi, sx, sy, u, v);
    else if constexpr (KIND == BSDF_ROUGHDIELECTRIC) return rd_sample_body<BS>(b, wi, sx, sy, u1d, u, v);
    else if constexpr (KIND == BSDF_ROUGHPLASTIC) return rp_sample_body<BS, true>(b, rt, wi, sx, sy, u, v, pre);
    else return bsdf_sample_fast<BS>(b, rt, wi, sx, sy, u1d, u, v, pre);
}
