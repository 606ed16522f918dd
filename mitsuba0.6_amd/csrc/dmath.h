// dmath.h -- device-side arithmetic of the path (gfx950).
//
// Single-precision, evaluated in the reference's expression order (the whole
// library is built with -ffp-contract=off: the reference's x86 SSE build has
// no FMA).  Division and sqrt are IEEE correctly rounded
// (-fhip-fp32-correctly-rounded-divide-sqrt).  The transcendentals the
// reference takes from glibc are glibc's own algorithms (glibc_f32.h);
// math::fastexp/fastlog are double precision in the reference too
// (include/mitsuba/core/math.h:175-216).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glibc_f32.h"

#define D_EPSILON 1e-4f            // constants.h:28
#define D_SHADOW_EPSILON 1e-3f     // constants.h:29
#define D_PI 3.14159265358979323846f
#define D_INV_PI 0.31830988618379067154f
#define D_INV_TWOPI 0.15915494309189533577f
#define D_ONE_MINUS_EPS 0x1.fffffep-1f

struct f3 { float x, y, z; };

__device__ __forceinline__ f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mul(f3 a, float f) { return mk(a.x * f, a.y * f, a.z * f); }
__device__ __forceinline__ f3 mulv(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 divv(f3 a, f3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
__device__ __forceinline__ f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ f3 divs(f3 a, float f) { float r = 1.0f / f; return mul(a, r); }  // vector.h:535-541
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float absdot(f3 a, f3 b) { return fabsf(dot(a, b)); }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x));
}
__device__ __forceinline__ float len2(f3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ float dsqrt(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ float len(f3 a) { return dsqrt(len2(a)); }
__device__ __forceinline__ f3 normalize(f3 a) { return divs(a, len(a)); }
__device__ __forceinline__ bool is_zero(f3 a) { return a.x == 0 && a.y == 0 && a.z == 0; }
__device__ __forceinline__ float comp(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// std::max / std::min semantics
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float safe_sqrt(float v) { return dsqrt(smax(0.0f, v)); }   // math.h:260
__device__ __forceinline__ float signum(float v) { return copysignf(1.0f, v); }         // math.h:270
__device__ __forceinline__ float smaxc(f3 s) { float r = s.x; r = smax(r, s.y); r = smax(r, s.z); return r; }

// libm: glibc's float routines restated bit for bit (glibc_f32.h);
// math::fastexp/fastlog are double exp/log in the reference (math.h:185-199)
__device__ __forceinline__ void d_sincos(float x, float *s, float *c) { glf_sincosf(x, s, c); }
__device__ __forceinline__ float d_acos(float x) { return glf_acosf(x); }
__device__ __forceinline__ float d_atan2(float y, float x) { return glf_atan2f(y, x); }
__device__ __forceinline__ float d_tan(float x) { return glf_tanf(x); }
__device__ __forceinline__ float d_atan(float x) { return glf_atanf(x); }
__device__ __forceinline__ float d_expf(float x) { return glf_expf(x); }
__device__ __forceinline__ float d_powf(float x, float y) { return glf_powf(x, y); }
__device__ __forceinline__ float d_fastexp(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float d_fastlog(float x) { return (float)log((double)x); }

struct Frame { f3 s, t, n; };
__device__ __forceinline__ f3 to_local(const Frame &f, f3 v) { return mk(dot(v, f.s), dot(v, f.t), dot(v, f.n)); }
__device__ __forceinline__ f3 to_world(const Frame &f, f3 v) {
    return add(add(mul(f.s, v.x), mul(f.t, v.y)), mul(f.n, v.z));
}
// A hit record's shading frame (computeShadingFrame, util.cpp:603-608) keeps s and
// n: its t is cross(n, s) by construction, re-formed where it is used (the same
// products, so the same bits) instead of held in three more registers across
// the BSDF calls
struct ShFrame {
    f3 s, n;
    __device__ __forceinline__ f3 t() const { return cross(n, s); }
};
__device__ __forceinline__ f3 to_local(const ShFrame &f, f3 v) { return mk(dot(v, f.s), dot(v, f.t()), dot(v, f.n)); }
__device__ __forceinline__ f3 to_world(const ShFrame &f, f3 v) {
    return add(add(mul(f.s, v.x), mul(f.t(), v.y)), mul(f.n, v.z));
}
