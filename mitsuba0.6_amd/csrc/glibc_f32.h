// glibc_f32.h -- glibc's single-precision transcendentals, restated.
//
// The reference calls glibc for sincosf, acosf, atanf, atan2f, tanf, expf and
// powf (include/mitsuba/core/math.h:218-221 math::sincos; std::acos/atan/atan2/
// tan/exp/pow on floats in src/bsdfs/microfacet.h:203-711, src/libcore/warp.cpp:
// 29-140, src/emitters/envmap.cpp:386-607, src/shapes/sphere.cpp:219-220,
// src/bsdfs/rtrans.h:184-365, include/mitsuba/render/mipmap.h:680).  This header
// computes each of them bit for bit as glibc 2.35 (Ubuntu GLIBC 2.35-0ubuntu3.11,
// x86_64) does on a CPU with FMA and AVX2, where libm's ifuncs select the
// -mfma -mavx2 builds of the double-internal routines:
//   sincosf  sysdeps/ieee754/flt-32/s_sincosf.c + s_sincosf.h (FMA build)
//   expf     sysdeps/ieee754/flt-32/e_expf.c + e_exp2f_data.c (FMA build)
//   powf     sysdeps/ieee754/flt-32/e_powf.c + e_powf_log2_data.c (FMA build)
//   acosf    sysdeps/ieee754/flt-32/e_acosf.c (fdlibm, float arithmetic)
//   atanf    sysdeps/ieee754/flt-32/s_atanf.c (fdlibm)
//   atan2f   sysdeps/ieee754/flt-32/e_atan2f.c (fdlibm, calls atanf)
//   tanf     sysdeps/ieee754/flt-32/s_tanf.c (sincosf's range reduction
//            without FMA, then the fdlibm __kernel_tanf of k_tanf.c)
// Where the FMA build contracts `a + b*c` the restatement writes fma(b, c, a);
// everything else is one IEEE operation per source operation (the library is
// built with -ffp-contract=off).  tests/test_glibc_f32.py checks the host build
// of this header against the container's libm.so.6 on all 2^32 inputs of each
// unary function and on dense grids for atan2f/powf; tests/test_gpu_libm.py
// checks the device build the same way.
//
// Results differ from glibc only in NaN payloads (x86's default NaN has the
// sign bit set; the tests compare NaNs as a class) and in the floating-point
// exception flags and errno, which the path never reads.
//
// One source for two compilers: hipcc (device functions, tables in constant
// memory) and gcc/g++ (host functions, for the exhaustive CPU check).
#pragma once
#include <stdint.h>
#include <string.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define GLF_FN __device__ __forceinline__
#define GLF_TABLE static __constant__ const
#define GLF_FMA(a, b, c) __builtin_fma((a), (b), (c))
#define GLF_SQRTF(x) __builtin_sqrtf(x)
// A double polynomial / reduction constant, materialised by two s_mov_b32 where
// it is used.  As a plain literal, LICM hoisted the constants out of the
// persistent megakernel's loop into VGPR pairs, and register pressure then put
// them in scratch: every powf reloaded three of them from memory.  Without
// the SLP vectoriser, C2 107 instead of 123 VGPRs, C4 106 instead of 112, C5
// 96 instead of 112 B of scratch per lane (tools/gpu_runs/r05/spills.sh).  Volatile asm is not hoisted; the value is the same.
template <uint64_t B> __device__ __forceinline__ double glf_kd_bits() {
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "n"((uint32_t)(B & 0xffffffffu)));
    asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "n"((uint32_t)(B >> 32)));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
#define GLF_KD(c) glf_kd_bits<__builtin_bit_cast(uint64_t, (double)(c))>()
#else
#define GLF_KD(c) (c)
#include <math.h>
#define GLF_FN static inline
#define GLF_TABLE static const
#define GLF_FMA(a, b, c) fma((a), (b), (c))
#define GLF_SQRTF(x) sqrtf(x)
#endif

GLF_FN uint32_t glf_asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
GLF_FN float glf_asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
GLF_FN uint64_t glf_asuint64(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }
GLF_FN double glf_asdouble(uint64_t u) { double f; memcpy(&f, &u, 8); return f; }
GLF_FN float glf_fabsf(float x) { return glf_asfloat(glf_asuint(x) & 0x7fffffffu); }
// top 12 bits of a float's double-format exponent field (abstop12 / top12)
GLF_FN uint32_t glf_abstop12(float x) { return (glf_asuint(x) >> 20) & 0x7ff; }
// a quiet NaN for invalid operations (glibc returns x86's default NaN)
GLF_FN float glf_nan(void) { return glf_asfloat(0x7fc00000u); }

// ---------------------------------------------------------------------------
// sincosf (s_sincosf.c, s_sincosf.h, FMA build)
// ---------------------------------------------------------------------------
// __sincosf_table[2]: sign[4], 2/pi * 2^24, pi/2, then the cosine polynomial
// c0..c4 and the sine polynomial s1..s3.  Entry 1 computes -cos for the odd
// quadrants' swap (c0..c4 negated).
#define GLF_HPI_INV GLF_KD(0x1.45f306dc9c883p+23)
#define GLF_HPI GLF_KD(0x1.921fb54442d18p+0)
#define GLF_PI63 GLF_KD(0x1.921fb54442d18p-62)
#define GLF_S1 GLF_KD(-0x1.555545995a603p-3)
#define GLF_S2 GLF_KD(0x1.1107605230bc4p-7)
#define GLF_S3 GLF_KD(-0x1.994eb3774cf24p-13)
#define GLF_C1 GLF_KD(-0x1.ffffffd0c621cp-2)
#define GLF_C2 GLF_KD(0x1.55553e1068f19p-5)
#define GLF_C3 GLF_KD(-0x1.6c087e89a359dp-10)
#define GLF_C4 GLF_KD(0x1.99343027bf8c3p-16)

// 4/pi to 192 bits; 8 new bits per entry (__inv_pio4)
GLF_TABLE uint32_t glf_inv_pio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};

// sincosf_poly: the polynomials for quadrant n with table sign `neg` (entry 1)
GLF_FN void glf_sincosf_poly(double x, double x2, int neg, int n, float *sinp, float *cosp) {
    const double c0 = neg ? -1.0 : 1.0;
    const double c1 = neg ? -GLF_C1 : GLF_C1, c2 = neg ? -GLF_C2 : GLF_C2;
    const double c3 = neg ? -GLF_C3 : GLF_C3, c4 = neg ? -GLF_C4 : GLF_C4;
    const double x4 = x2 * x2;
    const double x3 = x2 * x;
    const double cc2 = GLF_FMA(x2, c4, c3);
    const double ss1 = GLF_FMA(x2, GLF_S3, GLF_S2);
    const double cc1 = GLF_FMA(x2, c1, c0);
    const double x5 = x3 * x2;
    const double x6 = x4 * x2;
    const double s = GLF_FMA(x3, GLF_S1, x);
    const double c = GLF_FMA(x4, c2, cc1);
    const float so = (float)GLF_FMA(x5, ss1, s);
    const float co = (float)GLF_FMA(x6, cc2, c);
    if (n & 1) { *sinp = co; *cosp = so; }
    else { *sinp = so; *cosp = co; }
}

// reduce_fast with the FMA build's contraction: x - n*pi/2 as one fma
GLF_FN double glf_reduce_fast_fma(double x, int *np) {
    const double r = x * GLF_HPI_INV;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return GLF_FMA(-(double)n, GLF_HPI, x);
}

// reduce_fast as the non-FMA build (tanf) evaluates it
GLF_FN double glf_reduce_fast(double x, int *np) {
    const double r = x * GLF_HPI_INV;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return x - (double)n * GLF_HPI;
}

// reduce_large: 32x96-bit product with 4/pi (|x| >= 120, sign ignored)
GLF_FN double glf_reduce_large(uint32_t xi, int *np) {
    const uint32_t *arr = &glf_inv_pio4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = (uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * GLF_PI63;
}

GLF_FN void glf_sincosf(float y, float *sinp, float *cosp) {
    double x = y;
    int n;
    if (glf_abstop12(y) < glf_abstop12(0x1.921fb6p-1f)) {          // |y| < pi/4
        const double x2 = x * x;
        if (glf_abstop12(y) < glf_abstop12(0x1p-12f)) { *sinp = y; *cosp = 1.0f; return; }
        glf_sincosf_poly(x, x2, 0, 0, sinp, cosp);
    } else if (glf_abstop12(y) < glf_abstop12(120.0f)) {
        x = glf_reduce_fast_fma(x, &n);
        const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;   // sign[n & 3]
        glf_sincosf_poly(x * s, x * x, (n & 2) != 0, n, sinp, cosp);
    } else if (glf_abstop12(y) < glf_abstop12(__builtin_inff())) {
        const uint32_t xi = glf_asuint(y);
        const int sign = xi >> 31;
        x = glf_reduce_large(xi, &n);
        const int q = (n + sign) & 3;
        const double s = (q == 1 || q == 2) ? -1.0 : 1.0;
        glf_sincosf_poly(x * s, x * x, (q & 2) != 0, n, sinp, cosp);
    } else {
        *sinp = *cosp = glf_nan();                                    // y - y: Inf or NaN
    }
}

// ---------------------------------------------------------------------------
// expf / powf (e_expf.c, e_powf.c, e_exp2f_data.c, e_powf_log2_data.c; FMA build)
// ---------------------------------------------------------------------------
// __exp2f_data.tab[i] = asuint64(2^(i/32)) - (i << 47)
GLF_TABLE uint64_t glf_exp2f_tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
#define GLF_EXP2F_SHIFT GLF_KD(0x1.8p+52)
#define GLF_EXP2F_SHIFT_SCALED GLF_KD(0x1.8p+47)
#define GLF_EXP2F_C0 GLF_KD(0x1.c6af84b912394p-5)
#define GLF_EXP2F_C1 GLF_KD(0x1.ebfce50fac4f3p-3)
#define GLF_EXP2F_C2 GLF_KD(0x1.62e42ff0c52d6p-1)
#define GLF_EXPF_INVLN2N GLF_KD(0x1.71547652b82fep+5)
#define GLF_EXPF_C0 GLF_KD(0x1.c6af84b912394p-20)
#define GLF_EXPF_C1 GLF_KD(0x1.ebfce50fac4f3p-13)
#define GLF_EXPF_C2 GLF_KD(0x1.62e42ff0c52d6p-6)

// __math_oflowf / __math_uflowf / __math_may_uflowf (math_errf.c): the
// product of two same-signed constants, rounded
GLF_FN float glf_xflowf(uint32_t sign, float y) { return (sign ? -y : y) * y; }

GLF_FN float glf_expf(float x) {
    const double xd = (double)x;
    const uint32_t abstop = glf_abstop12(x);
    if (abstop >= glf_abstop12(88.0f)) {
        if (glf_asuint(x) == glf_asuint(-__builtin_inff())) return 0.0f;
        if (abstop >= glf_abstop12(__builtin_inff())) return x + x;
        if (x > 0x1.62e42ep6f) return glf_xflowf(0, 0x1p97f);
        if (x < -0x1.9fe368p6f) return glf_xflowf(0, 0x1p-95f);
        if (x < -0x1.9d1d9ep6f) return glf_xflowf(0, 0x1.4p-75f);
    }
    // z = x*N/ln2; kd = z + shift and r = z - kd, both contracted
    double kd = GLF_FMA(GLF_EXPF_INVLN2N, xd, GLF_EXP2F_SHIFT);
    const uint64_t ki = glf_asuint64(kd);
    kd -= GLF_EXP2F_SHIFT;
    const double r = GLF_FMA(GLF_EXPF_INVLN2N, xd, -kd);
    uint64_t t = glf_exp2f_tab[ki % 32];
    t += ki << 47;
    const double s = glf_asdouble(t);
    const double z = GLF_FMA(r, GLF_EXPF_C0, GLF_EXPF_C1);
    const double r2 = r * r;
    double y = GLF_FMA(r, GLF_EXPF_C2, 1.0);
    y = GLF_FMA(z, r2, y);
    y = y * s;
    return (float)y;
}

// __powf_log2_data: {1/c, log2(c)} per subinterval, and the log2 polynomial
GLF_TABLE double glf_powf_log2_tab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4},  {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2},  {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}};
#define GLF_POWF_A0 GLF_KD(0x1.27616c9496e0bp-2)
#define GLF_POWF_A1 GLF_KD(-0x1.71969a075c67ap-2)
#define GLF_POWF_A2 GLF_KD(0x1.ec70a6ca7baddp-2)
#define GLF_POWF_A3 GLF_KD(-0x1.7154748bef6c8p-1)
#define GLF_POWF_A4 GLF_KD(0x1.71547652ab82bp+0)

// log2_inline: x = 2^k z with z in [0x3f330000, 2*0x3f330000)
GLF_FN double glf_powf_log2(uint32_t ix) {
    const uint32_t tmp = ix - 0x3f330000;
    const int i = (tmp >> 19) % 16;
    const uint32_t top = tmp & 0xff800000;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double invc = glf_powf_log2_tab[i][0], logc = glf_powf_log2_tab[i][1];
    const double z = (double)glf_asfloat(iz);
    const double r = GLF_FMA(z, invc, -1.0);
    const double y0 = logc + (double)k;
    const double r2 = r * r;
    double y = GLF_FMA(GLF_POWF_A0, r, GLF_POWF_A1);
    const double p = GLF_FMA(GLF_POWF_A2, r, GLF_POWF_A3);
    const double r4 = r2 * r2;
    double q = GLF_FMA(GLF_POWF_A4, r, y0);
    q = GLF_FMA(p, r2, q);
    y = GLF_FMA(y, r4, q);
    return y;
}

// exp2_inline (TOINT_INTRINSICS == 0 on x86_64): sign_bias sets the sign
GLF_FN double glf_powf_exp2(double xd, uint32_t sign_bias) {
    double kd = xd + GLF_EXP2F_SHIFT_SCALED;
    const uint64_t ki = glf_asuint64(kd);
    kd -= GLF_EXP2F_SHIFT_SCALED;
    const double r = xd - kd;
    uint64_t t = glf_exp2f_tab[ki % 32];
    const uint64_t ski = ki + sign_bias;
    t += ski << 47;
    const double s = glf_asdouble(t);
    const double z = GLF_FMA(GLF_EXP2F_C0, r, GLF_EXP2F_C1);
    const double r2 = r * r;
    double y = GLF_FMA(GLF_EXP2F_C2, r, 1.0);
    y = GLF_FMA(z, r2, y);
    return y * s;
}

// 0: not an integer, 1: odd integer, 2: even integer
GLF_FN int glf_checkint(uint32_t iy) {
    const int e = iy >> 23 & 0xff;
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}

GLF_FN int glf_zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000 - 1; }

GLF_FN float glf_powf(float x, float y) {
    uint32_t sign_bias = 0;
    uint32_t ix = glf_asuint(x), iy = glf_asuint(y);
    if (ix - 0x00800000 >= 0x7f800000 - 0x00800000 || glf_zeroinfnan(iy)) {
        if (glf_zeroinfnan(iy)) {
            if (2 * iy == 0) return 1.0f;                      // (signalling NaNs aside)
            if (ix == 0x3f800000) return 1.0f;
            if (2 * ix > 2u * 0x7f800000 || 2 * iy > 2u * 0x7f800000) return x + y;
            if (2 * ix == 2 * 0x3f800000) return 1.0f;
            if ((2 * ix < 2 * 0x3f800000) == !(iy & 0x80000000)) return 0.0f;
            return y * y;
        }
        if (glf_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000) && glf_checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000) ? 1 / x2 : x2;
        }
        // x and y are non-zero finite
        if (ix & 0x80000000) {
            const int yint = glf_checkint(iy);
            if (yint == 0) return glf_nan();                   // __math_invalidf
            if (yint == 1) sign_bias = 1 << 16;                 // SIGN_BIAS
            ix &= 0x7fffffff;
        }
        if (ix < 0x00800000) {                                  // subnormal x
            ix = glf_asuint(x * 0x1p23f);
            ix &= 0x7fffffff;
            ix -= 23 << 23;
        }
    }
    const double logx = glf_powf_log2(ix);
    const double ylogx = (double)y * logx;
    if (((glf_asuint64(ylogx) >> 47) & 0xffff) >= (glf_asuint64(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return glf_xflowf(sign_bias, 0x1p97f);
        if (ylogx <= -150.0) return glf_xflowf(sign_bias, 0x1p-95f);
        if (ylogx < -149.0) return glf_xflowf(sign_bias, 0x1.4p-75f);
    }
    return (float)glf_powf_exp2(ylogx, sign_bias);
}

// ---------------------------------------------------------------------------
// acosf (e_acosf.c)
// ---------------------------------------------------------------------------
#define GLF_ACOS_PI 0x1.921fb4p+1f        // 0x40490fda
#define GLF_PIO2_HI 0x1.921fb4p+0f        // 0x3fc90fda
#define GLF_PIO2_LO 0x1.4442d0p-24f       // 0x33a22168
#define GLF_PS0 0x1.555556p-3f            // 0x3e2aaaab
#define GLF_PS1 -0x1.4d6120p-2f           // 0xbea6b090
#define GLF_PS2 0x1.9c1550p-3f            // 0x3e4e0aa8
#define GLF_PS3 -0x1.48228cp-5f           // 0xbd241146
#define GLF_PS4 0x1.9efe08p-11f           // 0x3a4f7f04
#define GLF_PS5 0x1.23de10p-15f           // 0x3811ef08
#define GLF_QS1 -0x1.33a272p+1f           // 0xc019d139
#define GLF_QS2 0x1.02ae5ap+1f            // 0x4001572d
#define GLF_QS3 -0x1.6066c2p-1f           // 0xbf303361
#define GLF_QS4 0x1.3b8c5cp-4f            // 0x3d9dc62e

GLF_FN float glf_acosf(float x) {
    const int32_t hx = (int32_t)glf_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    float z, p, q, r, w, s, c, df;
    if (ix == 0x3f800000) {
        if (hx > 0) return 0.0f;
        return GLF_ACOS_PI + 0x1.4442d0p-23f;              // pi + 2*pio2_lo
    } else if (ix > 0x3f800000) {
        return glf_nan();                                    // (x-x)/(x-x)
    }
    if (ix < 0x3f000000) {                                   // |x| < 0.5
        if (ix <= 0x32800000) return GLF_PIO2_HI + GLF_PIO2_LO;
        z = x * x;
        p = z * (GLF_PS0 + z * (GLF_PS1 + z * (GLF_PS2 + z * (GLF_PS3 + z * (GLF_PS4 + z * GLF_PS5)))));
        q = 1.0f + z * (GLF_QS1 + z * (GLF_QS2 + z * (GLF_QS3 + z * GLF_QS4)));
        r = p / q;
        return GLF_PIO2_HI - (x - (GLF_PIO2_LO - x * r));
    } else if (hx < 0) {                                     // x < -0.5
        z = (1.0f + x) * 0.5f;
        p = z * (GLF_PS0 + z * (GLF_PS1 + z * (GLF_PS2 + z * (GLF_PS3 + z * (GLF_PS4 + z * GLF_PS5)))));
        q = 1.0f + z * (GLF_QS1 + z * (GLF_QS2 + z * (GLF_QS3 + z * GLF_QS4)));
        s = GLF_SQRTF(z);
        r = p / q;
        w = r * s - GLF_PIO2_LO;
        return GLF_ACOS_PI - 2.0f * (s + w);
    } else {                                                 // x > 0.5
        z = (1.0f - x) * 0.5f;
        s = GLF_SQRTF(z);
        df = glf_asfloat(glf_asuint(s) & 0xfffff000);
        c = (z - df * df) / (s + df);
        p = z * (GLF_PS0 + z * (GLF_PS1 + z * (GLF_PS2 + z * (GLF_PS3 + z * (GLF_PS4 + z * GLF_PS5)))));
        q = 1.0f + z * (GLF_QS1 + z * (GLF_QS2 + z * (GLF_QS3 + z * GLF_QS4)));
        r = p / q;
        w = r * s + c;
        return 2.0f * (df + w);
    }
}

// ---------------------------------------------------------------------------
// atanf (s_atanf.c), atan2f (e_atan2f.c)
// ---------------------------------------------------------------------------
GLF_TABLE float glf_atanhi[4] = {0x1.dac670p-2f, 0x1.921fb4p-1f, 0x1.f730bcp-1f, 0x1.921fb4p+0f};
GLF_TABLE float glf_atanlo[4] = {0x1.586ed2p-28f, 0x1.4442d0p-25f, 0x1.281f68p-25f, 0x1.4442d0p-24f};
#define GLF_AT0 0x1.555556p-2f            // 0x3eaaaaab
#define GLF_AT1 -0x1.99999ap-3f           // 0xbe4ccccd
#define GLF_AT2 0x1.24924ap-3f            // 0x3e124925
#define GLF_AT3 -0x1.c71c70p-4f           // 0xbde38e38
#define GLF_AT4 0x1.745cdcp-4f            // 0x3dba2e6e
#define GLF_AT5 -0x1.3b0f2ap-4f           // 0xbd9d8795
#define GLF_AT6 0x1.10d66ap-4f            // 0x3d886b35
#define GLF_AT7 -0x1.dde2d6p-5f           // 0xbd6ef16b
#define GLF_AT8 0x1.97b4b2p-5f            // 0x3d4bda59
#define GLF_AT9 -0x1.2b4442p-5f           // 0xbd15a221
#define GLF_AT10 0x1.0ad3aep-6f           // 0x3c8569d7

GLF_FN float glf_atanf(float x) {
    const int32_t hx = (int32_t)glf_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {                                  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        if (hx > 0) return glf_atanhi[3] + glf_atanlo[3];
        return -glf_atanhi[3] - glf_atanlo[3];
    }
    if (ix < 0x3ee00000) {                                   // |x| < 0.4375
        if (ix < 0x31000000) return x;                       // |x| < 2^-29 (huge+x > one)
        id = -1;
    } else {
        x = glf_fabsf(x);
        if (ix < 0x3f980000) {                               // |x| < 1.1875
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (GLF_AT0 + w * (GLF_AT2 + w * (GLF_AT4 + w * (GLF_AT6 + w * (GLF_AT8 + w * GLF_AT10)))));
    const float s2 = w * (GLF_AT1 + w * (GLF_AT3 + w * (GLF_AT5 + w * (GLF_AT7 + w * GLF_AT9))));
    if (id < 0) return x - x * (s1 + s2);
    const float zz = glf_atanhi[id] - ((x * (s1 + s2) - glf_atanlo[id]) - x);
    return (hx < 0) ? -zz : zz;
}

#define GLF_TINY 1.0e-30f
#define GLF_PI_O_4 0x1.921fb6p-1f         // 0x3f490fdb
#define GLF_PI_O_2 0x1.921fb6p+0f         // 0x3fc90fdb
#define GLF_PI 0x1.921fb6p+1f             // 0x40490fdb
#define GLF_PI_LO -0x1.777a5cp-24f        // 0xb3bbbd2e

GLF_FN float glf_atan2f(float y, float x) {
    const int32_t hx = (int32_t)glf_asuint(x), hy = (int32_t)glf_asuint(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    float z;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;   // NaN
    if (hx == 0x3f800000) return glf_atanf(y);               // x = 1.0
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);       // 2*sign(x)+sign(y)
    if (iy == 0) {
        switch (m) {
        case 0:
        case 1: return y;
        case 2: return GLF_PI + GLF_TINY;
        default: return -GLF_PI - GLF_TINY;
        }
    }
    if (ix == 0) return (hy < 0) ? -GLF_PI_O_2 - GLF_TINY : GLF_PI_O_2 + GLF_TINY;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
            case 0: return GLF_PI_O_4 + GLF_TINY;
            case 1: return -GLF_PI_O_4 - GLF_TINY;
            case 2: return 3.0f * GLF_PI_O_4 + GLF_TINY;
            default: return -3.0f * GLF_PI_O_4 - GLF_TINY;
            }
        } else {
            switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return GLF_PI + GLF_TINY;
            default: return -GLF_PI - GLF_TINY;
            }
        }
    }
    if (iy == 0x7f800000) return (hy < 0) ? -GLF_PI_O_2 - GLF_TINY : GLF_PI_O_2 + GLF_TINY;
    const int32_t k = (iy - ix) >> 23;
    if (k > 60) z = GLF_PI_O_2 + 0.5f * GLF_PI_LO;          // |y/x| > 2^60
    else if (hx < 0 && k < -60) z = 0.0f;                    // |y|/x < -2^60
    else z = glf_atanf(glf_fabsf(y / x));
    switch (m) {
    case 0: return z;
    case 1: return glf_asfloat(glf_asuint(z) ^ 0x80000000u);
    case 2: return GLF_PI - (z - GLF_PI_LO);
    default: return (z - GLF_PI_LO) - GLF_PI;
    }
}

// ---------------------------------------------------------------------------
// tanf (s_tanf.c, k_tanf.c)
// ---------------------------------------------------------------------------
#define GLF_PIO4 0x1.921fb4p-1f           // 0x3f490fda
#define GLF_PIO4LO 0x1.4442d0p-25f        // 0x33222168
#define GLF_T0 0x1.555556p-2f             // 0x3eaaaaab
#define GLF_T1 0x1.111112p-3f             // 0x3e088889
#define GLF_T2 0x1.ba1ba2p-5f             // 0x3d5d0dd1
#define GLF_T3 0x1.664f48p-6f             // 0x3cb327a4
#define GLF_T4 0x1.226e3ep-7f             // 0x3c11371f
#define GLF_T5 0x1.d6d22cp-9f             // 0x3b6b6916
#define GLF_T6 0x1.7dbc90p-10f            // 0x3abede48
#define GLF_T7 0x1.344d90p-11f            // 0x3a1a26c8
#define GLF_T8 0x1.026f72p-12f            // 0x398137b9
#define GLF_T9 0x1.47e88ap-14f            // 0x38a3f445
#define GLF_T10 0x1.2b80f4p-14f           // 0x3895c07a
#define GLF_T11 -0x1.375cbep-16f          // 0xb79bae5f
#define GLF_T12 0x1.b2a708p-16f           // 0x37d95384

GLF_FN float glf_kernel_tanf(float x, float y, int iy) {
    float z, r, v, w, s;
    const int32_t hx = (int32_t)glf_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix < 0x39000000) {                                   // |x| < 2^-13
        if ((int)x == 0) {
            if ((ix | (iy + 1)) == 0) return 1.0f / glf_fabsf(x);
            else if (iy == 1) return x;
            else return -1.0f / x;
        }
    }
    if (ix >= 0x3f2ca140) {                                  // |x| >= 0.6744
        if (hx < 0) { x = -x; y = -y; }
        z = GLF_PIO4 - x;
        w = GLF_PIO4LO - y;
        x = z + w;
        y = 0.0f;
        if (glf_fabsf(x) < 0x1p-13f)
            return (float)((1 - ((hx >> 30) & 2)) * iy) * (1.0f - (float)(2 * iy) * x);
    }
    z = x * x;
    w = z * z;
    r = GLF_T1 + w * (GLF_T3 + w * (GLF_T5 + w * (GLF_T7 + w * (GLF_T9 + w * GLF_T11))));
    v = z * (GLF_T2 + w * (GLF_T4 + w * (GLF_T6 + w * (GLF_T8 + w * (GLF_T10 + w * GLF_T12)))));
    s = z * x;
    r = y + z * (s * (r + v) + y);
    r += GLF_T0 * s;
    w = x + r;
    if (ix >= 0x3f2ca140) {
        v = (float)iy;
        return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
    }
    if (iy == 1) return w;
    // -1/(x+r) accurately
    z = glf_asfloat(glf_asuint(w) & 0xfffff000);
    v = r - (z - x);
    const float a = -1.0f / w;
    const float t = glf_asfloat(glf_asuint(a) & 0xfffff000);
    s = 1.0f + t * z;
    return t + a * (s + t * v);
}

GLF_FN float glf_tanf(float x) {
    const int32_t ix = (int32_t)(glf_asuint(x) & 0x7fffffff);
    if (ix <= 0x3f490fda) return glf_kernel_tanf(x, 0.0f, 1);
    if (ix >= 0x7f800000) return glf_nan();                  // x - x
    double xd = (double)x;
    int n;
    if (glf_abstop12(x) < glf_abstop12(120.0f)) {
        xd = glf_reduce_fast(xd, &n);
    } else {
        xd = glf_reduce_large(glf_asuint(x), &n);
        if (glf_asuint(x) >> 31) xd = -xd;
    }
    const float y0 = (float)xd;
    const float y1 = (float)(xd - (double)y0);
    return glf_kernel_tanf(y0, y1, 1 - ((n & 1) << 1));
}
