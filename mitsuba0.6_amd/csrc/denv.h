// denv.h -- device side of the `envmap` emitter (src/emitters/envmap.cpp) and
// of the TMIPMap lookups it makes (include/mitsuba/render/mipmap.h).
//
// The MIP pyramid is stored as RGB halves (+1 pad half) exactly as the
// reference's SpectrumHalf pyramid; texels are decoded with an exact
// half->float conversion.  All arithmetic follows the reference's expression
// order (dmath.h); libm calls go through the double-evaluated helpers.
#pragma once
#include "dmath.h"
#include "layout.h"

typedef __attribute__((address_space(1))) const MtsgEnv glb_env;
typedef __attribute__((address_space(1))) const float glb_f32;
typedef unsigned int env_u2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const env_u2 glb_u2;

// the envmap NEE's sampleDirect / pdfDirect: out-of-line calls (MTSG_ENV_INLINE: inlined, an A/B knob)
#ifdef MTSG_ENV_INLINE
#define ENV_CALL __device__ __forceinline__
#else
#define ENV_CALL __device__ __noinline__
#endif
__device__ __forceinline__ float half_bits_to_float(uint32_t h) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)h);
}

// TMIPMap::evalTexel with ERepeat (u) / EClamp (v) (mipmap.h:427-490)
__device__ __forceinline__ f3 env_texel(glb_env *E, int level, int x, int y) {
    const int w = E->lw[level], h = E->lh[level];
    if (x < 0 || x >= w) {
        x = x % w;
        if (x < 0) x += w;
    }
    if (y < 0 || y >= h) y = y < 0 ? 0 : (y > h - 1 ? h - 1 : y);
    const env_u2 raw = ((glb_u2 *)(uintptr_t)E->texels)[(size_t)E->loff[level] + (size_t)y * w + x];
    return mk(half_bits_to_float(raw.x & 0xffffu), half_bits_to_float(raw.x >> 16), half_bits_to_float(raw.y & 0xffffu));
}

__device__ __forceinline__ float env_lum(f3 c) { return c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f; }  // spectrum.h:638-640

// evalBox (mipmap.h:493-497)
__device__ __forceinline__ f3 env_eval_box(glb_env *E, int level, float u, float v) {
    return env_texel(E, level, (int)floorf(u * (float)E->lw[level]), (int)floorf(v * (float)E->lh[level]));
}

// evalBilinear (mipmap.h:500-522)
__device__ __noinline__ f3 env_eval_bilinear(glb_env *E, int level, float uvx, float uvy) {
    if (!isfinite(uvx) || !isfinite(uvy)) return mk(0, 0, 0);
    if (level >= E->levels) return env_eval_box(E, E->levels - 1, uvx, uvy);
    const float u = uvx * (float)E->lw[level] - 0.5f, v = uvy * (float)E->lh[level] - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(v);
    const float dx1 = u - (float)xPos, dx2 = 1.0f - dx1, dy1 = v - (float)yPos, dy2 = 1.0f - dy1;
    f3 r = mul(mul(env_texel(E, level, xPos, yPos), dx2), dy2);
    r = add(r, mul(mul(env_texel(E, level, xPos, yPos + 1), dx2), dy1));
    r = add(r, mul(mul(env_texel(E, level, xPos + 1, yPos), dx1), dy2));
    r = add(r, mul(mul(env_texel(E, level, xPos + 1, yPos + 1), dx1), dy1));
    return r;
}

// evalEWA (mipmap.h:760-836)
__device__ __noinline__ f3 env_eval_ewa(glb_env *E, int level, float uvx, float uvy, float A, float B, float C) {
    if (!isfinite(A + B + C + uvx + uvy)) return mk(0, 0, 0);
    if (level >= E->levels) return env_eval_box(E, E->levels - 1, uvx, uvy);
    const float u = uvx * (float)E->lw[level] - 0.5f;
    const float v = uvy * (float)E->lh[level] - 0.5f;
    const float rx = E->ratio_x[level], ry = E->ratio_y[level];
    A /= rx * rx;
    B /= rx * ry;
    C /= ry * ry;
    const float invDet = 1.0f / (-B * B + 4.0f * A * C);
    const float deltaU = 2.0f * dsqrt(C * invDet), deltaV = 2.0f * dsqrt(A * invDet);
    const int u0 = (int)ceilf(u - deltaU), u1 = (int)floorf(u + deltaU);
    const int v0 = (int)ceilf(v - deltaV), v1 = (int)floorf(v + deltaV);
    const float As = A * (float)MTSG_EWA_LUT, Bs = B * (float)MTSG_EWA_LUT, Cs = C * (float)MTSG_EWA_LUT;
    f3 result = mk(0, 0, 0);
    float denominator = 0.0f;
    const float ddq = 2 * As, uu0 = (float)u0 - u;
    for (int vt = v0; vt <= v1; ++vt) {
        const float vv = (float)vt - v;
        float q = As * uu0 * uu0 + (Bs * uu0 + Cs * vv) * vv;
        float dq = As * (2 * uu0 + 1) + Bs * vv;
        for (int ut = u0; ut <= u1; ++ut) {
            if (q < (float)MTSG_EWA_LUT) {
                // (uint32_t) q as the reference's x86-64 build converts it (cvttss2si, 64 bit)
                const uint32_t qi = (uint32_t)(long long)q;
                if (qi < MTSG_EWA_LUT) {
                    const float weight = E->lut[(int)q];
                    result = add(result, mul(env_texel(E, level, ut, vt), weight));
                    denominator += weight;
                }
            }
            q += dq;
            dq += ddq;
        }
    }
    if (denominator == 0) return env_eval_bilinear(E, level, uvx, uvy);
    return divs(result, denominator);
}

// math::hypot2 (libcore/math.cpp:74-86)
__device__ __forceinline__ float d_hypot2(float a, float b) {
    float r;
    if (fabsf(a) > fabsf(b)) {
        r = b / a;
        r = fabsf(a) * dsqrt(1.0f + r * r);
    } else if (b != 0.0f) {
        r = a / b;
        r = fabsf(b) * dsqrt(1.0f + r * r);
    } else {
        r = 0.0f;
    }
    return r;
}

// TMIPMap::eval with EEWA (mipmap.h:560-660)
__device__ __noinline__ f3 env_eval_filtered(glb_env *E, float uvx, float uvy, float d0x, float d0y, float d1x, float d1y) {
    const float w0 = (float)E->w0, h0 = (float)E->h0;
    const float du0 = d0x * w0, dv0 = d0y * h0, du1 = d1x * w0, dv1 = d1y * h0;
    float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1), C = du0 * du0 + du1 * du1;
    float F = A * C - B * B * 0.25f;
    const float root = d_hypot2(A - C, B), Aprime = 0.5f * (A + C - root), Cprime = 0.5f * (A + C + root);
    float majorRadius = Aprime != 0 ? dsqrt(F / Aprime) : 0;
    float minorRadius = Cprime != 0 ? dsqrt(F / Cprime) : 0;
    if (!(minorRadius > 0) || !(majorRadius > 0) || F < 0) {
        const float level = d_fastlog(smax(majorRadius, D_EPSILON)) * E->inv_ln2;
        const int ilevel = (int)floorf(level);
        if (ilevel < 0) return env_eval_bilinear(E, 0, uvx, uvy);
        const float a = level - (float)ilevel;
        return add(mul(env_eval_bilinear(E, ilevel, uvx, uvy), 1.0f - a), mul(env_eval_bilinear(E, ilevel + 1, uvx, uvy), a));
    }
    if (minorRadius * E->max_aniso < majorRadius) {
        minorRadius = majorRadius / E->max_aniso;
        const float theta = 0.5f * d_atan(B / (A - C));
        float sinTheta, cosTheta;
        d_sincos(theta, &sinTheta, &cosTheta);
        const float a2 = majorRadius * majorRadius, b2 = minorRadius * minorRadius, sinTheta2 = sinTheta * sinTheta,
                    cosTheta2 = cosTheta * cosTheta, sin2Theta = 2 * sinTheta * cosTheta;
        A = a2 * cosTheta2 + b2 * sinTheta2;
        B = (a2 - b2) * sin2Theta;
        C = a2 * sinTheta2 + b2 * cosTheta2;
        F = a2 * b2;
    }
    const float scale = 1.0f / F;
    A *= scale;
    B *= scale;
    C *= scale;
    const float level = smax(0.0f, d_fastlog(minorRadius) * E->inv_ln2);
    const int ilevel = (int)level;
    const float a = level - (float)ilevel;
    if (majorRadius < 1 || !(A > 0 && C > 0)) return env_eval_bilinear(E, ilevel, uvx, uvy);
    return add(mul(env_eval_ewa(E, ilevel, uvx, uvy, A, B, C), 1.0f - a), mul(env_eval_ewa(E, ilevel + 1, uvx, uvy, A, B, C), a));
}

__device__ __forceinline__ f3 env_xf(const float *m, f3 v) {   // Transform::operator()(Vector) (transform.h:175-183)
    return mk(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z, m[6] * v.x + m[7] * v.y + m[8] * v.z);
}
__device__ __forceinline__ f3 env_to_local(glb_env *E, f3 v) {
    return mk(E->to_local[0] * v.x + E->to_local[1] * v.y + E->to_local[2] * v.z,
              E->to_local[3] * v.x + E->to_local[4] * v.y + E->to_local[5] * v.z,
              E->to_local[6] * v.x + E->to_local[7] * v.y + E->to_local[8] * v.z);
}
__device__ __forceinline__ f3 env_to_world(glb_env *E, f3 v) {
    return mk(E->to_world[0] * v.x + E->to_world[1] * v.y + E->to_world[2] * v.z,
              E->to_world[3] * v.x + E->to_world[4] * v.y + E->to_world[5] * v.z,
              E->to_world[6] * v.x + E->to_world[7] * v.y + E->to_world[8] * v.z);
}

// A world direction's spherical coordinates in the map (envmap.cpp:384-386, 612-614):
// evalEnvironment and internalPdfDirection form the same (u, v) from the same
// local direction, so a miss that needs both forms them once
struct EnvUV { float u, v, ly; };   // ly: the local direction's y (pdf's sinTheta)
__device__ __forceinline__ EnvUV env_uv(glb_env *E, f3 d) {
    const f3 v = env_to_local(E, d);
    EnvUV r;
    r.u = d_atan2(v.x, -v.z) * D_INV_TWOPI;
    r.v = d_acos(smin(1.0f, smax(-1.0f, v.y))) * D_INV_PI;
    r.ly = v.y;
    return r;
}
// EnvironmentMap::evalEnvironment without differentials (envmap.cpp:380-393)
__device__ __forceinline__ f3 env_eval_at(glb_env *E, EnvUV c) { return mul(env_eval_bilinear(E, 0, c.u, c.v), E->scale); }
__device__ __forceinline__ f3 env_eval(glb_env *E, f3 d) { return env_eval_at(E, env_uv(E, d)); }

// EnvironmentMap::evalEnvironment with ray differentials (envmap.cpp:380-410)
__device__ __forceinline__ f3 env_eval_diff(glb_env *E, f3 d, f3 rxd, f3 ryd) {
    const f3 v = env_to_local(E, d);
    const float u = d_atan2(v.x, -v.z) * D_INV_TWOPI, w = d_acos(smin(1.0f, smax(-1.0f, v.y))) * D_INV_PI;
    const f3 dvdx = sub(env_to_local(E, rxd), v), dvdy = sub(env_to_local(E, ryd), v);
    const float t1 = D_INV_TWOPI / (v.x * v.x + v.z * v.z);
    const float t2 = -D_INV_PI / smax(safe_sqrt(1.0f - v.y * v.y), D_EPSILON);
    const float dudx_x = t1 * (dvdx.z * v.x - dvdx.x * v.z), dudx_y = t2 * dvdx.y;
    const float dudy_x = t1 * (dvdy.z * v.x - dvdy.x * v.z), dudy_y = t2 * dvdy.y;
    return mul(env_eval_filtered(E, u, w, dudx_x, dudx_y, dudy_x, dudy_y), E->scale);
}

// BSphere::rayIntersect + solveQuadratic (bsphere.h:88-95, libcore/util.cpp:447-485)
__device__ __forceinline__ bool env_bsphere(glb_env *E, f3 ro, f3 d, float &nearT, float &farT) {
    const f3 o = sub(ro, mk(E->center[0], E->center[1], E->center[2]));
    const float a = len2(d), b = 2 * dot(o, d), c = len2(o) - E->radius * E->radius;
    if (a == 0) {
        if (b != 0) { nearT = farT = -c / b; return true; }
        return false;
    }
    const float discrim = b * b - 4.0f * a * c;
    if (discrim < 0) return false;
    const float sq = dsqrt(discrim);
    const float temp = b < 0 ? -0.5f * (b - sq) : -0.5f * (b + sq);
    float x0 = temp / a, x1 = c / temp;
    if (x0 > x1) { const float t = x0; x0 = x1; x1 = t; }
    nearT = x0;
    farT = x1;
    return true;
}

// sampleReuse of the envmap's float CDFs (envmap.cpp:687-692): std::lower_bound
// over [lo, hi), narrowed by the guide table when there is one (MtsgEnv::guide_*:
// the same index as the full-range search)
typedef __attribute__((address_space(1))) const uint16_t glb_u16;
__device__ __forceinline__ uint32_t env_sample_reuse(glb_f32 *__restrict__ cdf, glb_u16 *guide, uint32_t gbits,
                                                     uint32_t size, float &sample) {
    uint32_t lo = 0, hi = size + 1;
    if (guide) {
        const uint32_t k = (uint32_t)(sample * (float)(1u << gbits));   // exact scaling, floor
        if (k < (1u << gbits)) { lo = guide[k]; hi = guide[k + 1]; }
    }
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] < sample) lo = mid + 1; else hi = mid;
    }
    const int e = (int)lo - 1;
    uint32_t index = (uint32_t)(e < 0 ? 0 : e);
    if (index > size - 1) index = size - 1;
    sample = (sample - cdf[index]) / (cdf[index + 1] - cdf[index]);
    return index;
}

__device__ __forceinline__ float interval_to_tent(float s) {   // warp.cpp:143-155
    float sign;
    if (s < 0.5f) { sign = 1; s *= 2; } else { sign = -1; s = 2 * (s - 0.5f); }
    return sign * (1 - dsqrt(s));
}

// EnvironmentMap::sampleDirect (envmap.cpp:516-543) + internalSampleDirection
// (envmap.cpp:567-603): returns value/pdf; pdf = 0 on failure
__device__ __forceinline__ f3 env_sample_direct_impl(glb_env *E, f3 ref, float sx, float sy, f3 &dOut, float &dist, float &pdfOut) {
    const uint32_t W = (uint32_t)E->w0, H = (uint32_t)E->h0;
    glb_u16 *gr = (glb_u16 *)(uintptr_t)E->guide_rows, *gc = (glb_u16 *)(uintptr_t)E->guide_cols;
    const uint32_t row = env_sample_reuse((glb_f32 *)(uintptr_t)E->cdf_rows, gr, E->guide_rbits, H, sy);
    const uint32_t col = env_sample_reuse((glb_f32 *)(uintptr_t)E->cdf_cols + (size_t)row * (W + 1),
                                          gc ? gc + (size_t)row * ((1u << E->guide_cbits) + 1) : nullptr,
                                          E->guide_cbits, W, sx);
    const float posx = (float)col + interval_to_tent(sx), posy = (float)row + interval_to_tent(sy);
    const int xPos = (int)floorf(posx), yPos = (int)floorf(posy);
    const float dx1 = posx - (float)xPos, dx2 = 1.0f - dx1, dy1 = posy - (float)yPos, dy2 = 1.0f - dy1;
    const f3 value1 = add(mul(mul(env_texel(E, 0, xPos, yPos), dx2), dy2), mul(mul(env_texel(E, 0, xPos + 1, yPos), dx1), dy2));
    const f3 value2 = add(mul(mul(env_texel(E, 0, xPos, yPos + 1), dx2), dy1), mul(mul(env_texel(E, 0, xPos + 1, yPos + 1), dx1), dy1));
    const f3 value = mul(add(value1, value2), E->scale);
    const int y0c = yPos < 0 ? 0 : (yPos > (int)H - 1 ? (int)H - 1 : yPos);
    const int y1c = yPos + 1 < 0 ? 0 : (yPos + 1 > (int)H - 1 ? (int)H - 1 : yPos + 1);
    float pdf = (env_lum(value1) * ((glb_f32 *)(uintptr_t)E->row_weights)[y0c] + env_lum(value2) * ((glb_f32 *)(uintptr_t)E->row_weights)[y1c]) * E->normalization;
    float sinPhi, cosPhi, sinTheta, cosTheta;
    d_sincos(E->pixel_x * (posx + 0.5f), &sinPhi, &cosPhi);
    d_sincos(E->pixel_y * (posy + 0.5f), &sinTheta, &cosTheta);
    const f3 dl = mk(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
    pdf /= smax(fabsf(sinTheta), D_EPSILON);
    const f3 d = env_to_world(E, dl);
    float nearT, farT;
    if (is_zero(value) || pdf == 0 || !env_bsphere(E, ref, d, nearT, farT) || nearT >= 0 || farT <= 0) {
        pdfOut = 0.0f;
        return mk(0, 0, 0);
    }
    pdfOut = pdf;
    dist = farT;
    dOut = d;
    return divs(value, pdf);
}

// internalPdfDirection (envmap.cpp:606-633), solid angle, at the direction's env_uv
ENV_CALL float env_pdf_at(glb_env *E, EnvUV c) {
    const float uvx = c.u, uvy = c.v;
    if (!isfinite(uvx) || !isfinite(uvy)) return 0.0f;
    const int W = E->w0, H = E->h0;
    const float u = uvx * (float)W - 0.5f, v = uvy * (float)H - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(v);
    const float dx1 = u - (float)xPos, dx2 = 1.0f - dx1, dy1 = v - (float)yPos, dy2 = 1.0f - dy1;
    const f3 value1 = add(mul(mul(env_texel(E, 0, xPos, yPos), dx2), dy2), mul(mul(env_texel(E, 0, xPos + 1, yPos), dx1), dy2));
    const f3 value2 = add(mul(mul(env_texel(E, 0, xPos, yPos + 1), dx2), dy1), mul(mul(env_texel(E, 0, xPos + 1, yPos + 1), dx1), dy1));
    const float sinTheta = safe_sqrt(1 - c.ly * c.ly);
    const int y0c = yPos < 0 ? 0 : (yPos > H - 1 ? H - 1 : yPos);
    const int y1c = yPos + 1 < 0 ? 0 : (yPos + 1 > H - 1 ? H - 1 : yPos + 1);
    return (env_lum(value1) * ((glb_f32 *)(uintptr_t)E->row_weights)[y0c] + env_lum(value2) * ((glb_f32 *)(uintptr_t)E->row_weights)[y1c]) * E->normalization /
           smax(fabsf(sinTheta), D_EPSILON);
}
__device__ __forceinline__ float env_pdf_direction(glb_env *E, f3 d) { return env_pdf_at(E, env_uv(E, d)); }

// A miss's evalEnvironment value (evalBilinear at level 0, mipmap.h:500-522) and
// its internalPdfDirection (envmap.cpp:606-633) at the same (u, v), in one call:
// both read the same four texels (level 0 is w0 x h0, scene_build.cpp), and each
// result keeps its own summation order
struct EnvValPdf { f3 value; float pdf; };
ENV_CALL EnvValPdf env_eval_pdf_at(glb_env *E, EnvUV c) {
    EnvValPdf r;
    r.value = mk(0, 0, 0);
    r.pdf = 0.0f;
    if (!isfinite(c.u) || !isfinite(c.v)) return r;
    const int W = E->w0, H = E->h0;
    const float u = c.u * (float)W - 0.5f, v = c.v * (float)H - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(v);
    const float dx1 = u - (float)xPos, dx2 = 1.0f - dx1, dy1 = v - (float)yPos, dy2 = 1.0f - dy1;
    const f3 t00 = env_texel(E, 0, xPos, yPos), t01 = env_texel(E, 0, xPos, yPos + 1);
    const f3 t10 = env_texel(E, 0, xPos + 1, yPos), t11 = env_texel(E, 0, xPos + 1, yPos + 1);
    f3 e = mul(mul(t00, dx2), dy2);   // evalBilinear's order
    e = add(e, mul(mul(t01, dx2), dy1));
    e = add(e, mul(mul(t10, dx1), dy2));
    e = add(e, mul(mul(t11, dx1), dy1));
    r.value = mul(e, E->scale);
    const f3 value1 = add(mul(mul(t00, dx2), dy2), mul(mul(t10, dx1), dy2));   // internalPdfDirection's
    const f3 value2 = add(mul(mul(t01, dx2), dy1), mul(mul(t11, dx1), dy1));
    const float sinTheta = safe_sqrt(1 - c.ly * c.ly);
    const int y0c = yPos < 0 ? 0 : (yPos > H - 1 ? H - 1 : yPos);
    const int y1c = yPos + 1 < 0 ? 0 : (yPos + 1 > H - 1 ? H - 1 : yPos + 1);
    r.pdf = (env_lum(value1) * ((glb_f32 *)(uintptr_t)E->row_weights)[y0c] +
             env_lum(value2) * ((glb_f32 *)(uintptr_t)E->row_weights)[y1c]) * E->normalization /
            smax(fabsf(sinTheta), D_EPSILON);
    return r;
}

struct EnvSample { f3 value, d; float dist, pdf; };
ENV_CALL EnvSample env_sample_direct(glb_env *E, f3 ref, float sx, float sy) {
    EnvSample r;
    r.d = mk(0, 0, 1);
    r.dist = 0.0f;
    r.value = env_sample_direct_impl(E, ref, sx, sy, r.d, r.dist, r.pdf);
    return r;
}
