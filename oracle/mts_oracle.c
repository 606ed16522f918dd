/*
 * mts_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C restatement of Mitsuba 0.6's unidirectional path tracer hot path
 * (/root/reference = Yujie-G/mitsuba0.6).  Every function cites the reference
 * lines it follows.  Arithmetic is single precision, evaluated in the same
 * order as the reference expressions, compiled with -ffp-contract=off (the
 * reference's x86 SSE build has no FMA).
 *
 * Pinning: the reference cannot be built here (every header includes boost,
 * absent from the image), so this restatement is pinned by
 *   - the reference's own known-answer test for the intersection record
 *     (src/tests/test_dgeom.cpp:35-80) -> tests/test_oracle_kat.py;
 *   - golden vectors computed from the reference's vendored Sobol tables
 *     (src/samplers/sobolseq.cpp) -> tests/golden/sobol_golden.json;
 *   - the reference's chi^2 / sample-vs-pdf consistency criteria
 *     (src/tests/test_chisquare.cpp:94-215) -> tests/test_oracle_bsdf.py.
 * Whole-path Li() output is "parity unpinned" against the reference binary
 * (no reference test pins it); it is pinned against this
 * restatement, which follows the reference line by line.
 *
 * libm: mode 0 calls the glibc float functions the reference calls
 * (sincosf, acosf, atan2f, tanf, expf, powf, atanf) and double exp/log for
 * math::fastexp/fastlog (include/mitsuba/core/math.h:175-216).  The product's
 * device code computes glibc's own algorithms (csrc/glibc_f32.h, checked bit
 * for bit against libm.so.6 by tests/test_glibc_f32.py), so the parity tests
 * run mode 0.  Mode 1 rounds the correctly rounded double result to float
 * (the device's libm before round 3); DESIGN.md reports its difference to
 * mode 0 as the former libm noise floor.
 */
#define _GNU_SOURCE
#include "mts_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* constants (include/mitsuba/core/constants.h:28-31,53-66)                  */
/* ------------------------------------------------------------------------ */
#define EPSILON 1e-4f
#define SHADOW_EPSILON 1e-3f
#define M_PI_F 3.14159265358979323846f
#define INV_PI_F 0.31830988618379067154f
#define INV_TWOPI_F 0.15915494309189533577f
#define ONE_MINUS_EPS_F 0x1.fffffep-1f
#define FILTER_RES 31 /* MTS_FILTER_RESOLUTION, rfilter.h:28 */
#define BLOCK_SIZE 32 /* scene.cpp:24 */

static int g_cr = 0; /* libm mode */
/* oracle_set_kdtree: traverse this kd-tree (KDNode words, primitive lists) in
   Scene::rayIntersect / isOccluded instead of the BVH (NULL: the BVH) */
static const uint32_t *g_kd_nodes = NULL, *g_kd_indices = NULL;
/* diagnostics (tools/diag_bench_kernel.py): ORACLE_TRACE="px,py,j" prints every ray query
   of that one sample with its exact bits and answer to stderr (render threads = 1) */
static int g_trace_px = -1, g_trace_py = -1, g_trace_j = -1;
static _Thread_local int g_trace_on = 0;

/* std::max / std::min semantics (NaN handling matters) */
static inline float smax(float a, float b) { return (a < b) ? b : a; }
static inline float smin(float a, float b) { return (b < a) ? b : a; }

/* ---- libm as called by the reference ---------------------------------- */
static inline void o_sincos(float x, float *s, float *c) {
    if (g_cr) { *s = (float)sin((double)x); *c = (float)cos((double)x); }
    else sincosf(x, s, c);
}
static inline float o_acos(float x) { return g_cr ? (float)acos((double)x) : acosf(x); }
static inline float o_atan2(float y, float x) { return g_cr ? (float)atan2((double)y, (double)x) : atan2f(y, x); }
static inline float o_tan(float x) { return g_cr ? (float)tan((double)x) : tanf(x); }
static inline float o_atan(float x) { return g_cr ? (float)atan((double)x) : atanf(x); }
static inline float o_exp(float x) { return g_cr ? (float)exp((double)x) : expf(x); }
static inline float o_pow(float x, float y) { return g_cr ? (float)pow((double)x, (double)y) : powf(x, y); }
/* math::fastexp/fastlog (math.h:185-200): double precision in both modes */
static inline float o_fastexp(float x) { return (float)exp((double)x); }
static inline float o_fastlog(float x) { return (float)log((double)x); }
/* math::safe_sqrt (math.h:260-262) */
static inline float safe_sqrt(float v) { return sqrtf(smax(0.0f, v)); }
/* math::signum (math.h:270-279) */
static inline float signumf(float v) { return copysignf(1.0f, v); }

/* ------------------------------------------------------------------------ */
/* vectors, spectra, frames (core/vector.h, spectrum.h, frame.h)             */
/* ------------------------------------------------------------------------ */
typedef struct { float x, y, z; } V3;
static inline V3 v3(float x, float y, float z) { V3 r = {x, y, z}; return r; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 vmul(V3 a, float f) { return v3(a.x * f, a.y * f, a.z * f); }
static inline V3 vmulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 vdivv(V3 a, V3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
/* operator/(T f): recip = 1/f (vector.h:535-541, spectrum.h:415-423) */
static inline V3 vdiv(V3 a, float f) { float r = 1.0f / f; return vmul(a, r); }
static inline float vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float vabsdot(V3 a, V3 b) { return fabsf(vdot(a, b)); }
static inline V3 vcross(V3 a, V3 b) {
    return v3((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x));
}
static inline float vlen2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline float vlen(V3 a) { return sqrtf(vlen2(a)); }
static inline V3 vnormalize(V3 a) { return vdiv(a, vlen(a)); }
static inline int vzero(V3 a) { return a.x == 0 && a.y == 0 && a.z == 0; }
static inline float vget(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline void vset(V3 *a, int i, float f) { if (i == 0) a->x = f; else if (i == 1) a->y = f; else a->z = f; }
/* Spectrum::max (spectrum.h:543-548) */
static inline float smaxc(V3 s) { float r = s.x; r = smax(r, s.y); r = smax(r, s.z); return r; }
/* Spectrum::average (spectrum.h:481-486) */
static inline float savg(V3 s) { float r = 0.0f; r += s.x; r += s.y; r += s.z; return r * (1.0f / 3); }

typedef struct { V3 s, t, n; } Frame;
static inline V3 to_local(const Frame *f, V3 v) { return v3(vdot(v, f->s), vdot(v, f->t), vdot(v, f->n)); }
static inline V3 to_world(const Frame *f, V3 v) {
    return vadd(vadd(vmul(f->s, v.x), vmul(f->t, v.y)), vmul(f->n, v.z));
}
/* Frame::tanTheta (frame.h:117-122), sinTheta2 (:103-105) */
static inline float tan_theta(V3 v) {
    float temp = 1 - v.z * v.z;
    if (temp <= 0.0f) return 0.0f;
    return sqrtf(temp) / v.z;
}
static inline float sin_theta2(V3 v) { return 1.0f - v.z * v.z; }

/* coordinateSystem (util.cpp:592-601) */
static void coordinate_system(V3 a, V3 *b, V3 *c) {
    if (fabsf(a.x) > fabsf(a.y)) {
        float invLen = 1.0f / sqrtf(a.x * a.x + a.z * a.z);
        *c = v3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / sqrtf(a.y * a.y + a.z * a.z);
        *c = v3(0.0f, a.z * invLen, -a.y * invLen);
    }
    *b = vcross(*c, a);
}

/* computeShadingFrame (util.cpp:603-608) */
static void compute_shading_frame(V3 n, V3 dpdu, Frame *f) {
    f->n = n;
    f->s = vnormalize(vsub(dpdu, vmul(f->n, vdot(f->n, dpdu))));
    f->t = vcross(f->n, f->s);
}

/* ------------------------------------------------------------------------ */
/* 4x4 transforms (core/transform.h, transform.cpp, matrix.h/.inl)           */
/* ------------------------------------------------------------------------ */
typedef struct { float m[4][4]; } M4;
typedef struct { M4 t, inv; } Xform;

static M4 m4_mul(const M4 *a, const M4 *b) { /* matrix.h:744-756 */
    M4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float sum = 0;
            for (int k = 0; k < 4; ++k) sum += a->m[i][k] * b->m[k][j];
            r.m[i][j] = sum;
        }
    return r;
}

static int m4_invert(const M4 *src, M4 *target) { /* matrix.inl:138-193 */
    int indxc[4], indxr[4], ipiv[4] = {0, 0, 0, 0};
    *target = *src;
    for (int i = 0; i < 4; i++) {
        int irow = -1, icol = -1;
        float big = 0;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] != 1) {
                for (int k = 0; k < 4; k++) {
                    if (ipiv[k] == 0) {
                        if (fabsf(target->m[j][k]) >= big) {
                            big = fabsf(target->m[j][k]);
                            irow = j; icol = k;
                        }
                    } else if (ipiv[k] > 1) return 0;
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) { float t = target->m[irow][k]; target->m[irow][k] = target->m[icol][k]; target->m[icol][k] = t; }
        indxr[i] = irow; indxc[i] = icol;
        if (target->m[icol][icol] == 0) return 0;
        float pivinv = 1.f / target->m[icol][icol];
        target->m[icol][icol] = 1.f;
        for (int j = 0; j < 4; j++) target->m[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j != icol) {
                float save = target->m[j][icol];
                target->m[j][icol] = 0;
                for (int k = 0; k < 4; k++) target->m[j][k] -= target->m[icol][k] * save;
            }
        }
    }
    for (int j = 3; j >= 0; j--) {
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) {
                float t = target->m[k][indxr[j]]; target->m[k][indxr[j]] = target->m[k][indxc[j]]; target->m[k][indxc[j]] = t;
            }
    }
    return 1;
}

static M4 m4_diag(float a, float b, float c, float d) {
    M4 r; memset(&r, 0, sizeof r);
    r.m[0][0] = a; r.m[1][1] = b; r.m[2][2] = c; r.m[3][3] = d;
    return r;
}
static Xform xf_compose(const Xform *a, const Xform *b) { /* transform.cpp:28-31 */
    Xform r; r.t = m4_mul(&a->t, &b->t); r.inv = m4_mul(&b->inv, &a->inv); return r;
}
static Xform xf_scale(float x, float y, float z) { /* transform.cpp:49-63 */
    Xform r; r.t = m4_diag(x, y, z, 1); r.inv = m4_diag(1.0f / x, 1.0f / y, 1.0f / z, 1); return r;
}
static Xform xf_translate(float x, float y, float z) { /* transform.cpp:33-47 */
    Xform r; r.t = m4_diag(1, 1, 1, 1); r.inv = r.t;
    r.t.m[0][3] = x; r.t.m[1][3] = y; r.t.m[2][3] = z;
    r.inv.m[0][3] = -x; r.inv.m[1][3] = -y; r.inv.m[2][3] = -z;
    return r;
}
static inline float deg_to_rad(float v) { return v * (M_PI_F / 180.0f); } /* util.h:297 */
static inline float rad_to_deg(float v) { return v * (180.0f / M_PI_F); } /* util.h:294 */
static int xf_perspective(float fov, float clipNear, float clipFar, Xform *out) { /* transform.cpp:99-123 */
    float recip = 1.0f / (clipFar - clipNear);
    float cot = 1.0f / tanf(deg_to_rad(fov / 2.0f));
    M4 t; memset(&t, 0, sizeof t);
    t.m[0][0] = cot; t.m[1][1] = cot;
    t.m[2][2] = clipFar * recip; t.m[2][3] = -clipNear * clipFar * recip;
    t.m[3][2] = 1;
    out->t = t;
    return m4_invert(&t, &out->inv);
}
/* Transform::operator()(Point) (transform.h:108-125) */
static V3 xf_point(const M4 *m, V3 p) {
    float x = m->m[0][0] * p.x + m->m[0][1] * p.y + m->m[0][2] * p.z + m->m[0][3];
    float y = m->m[1][0] * p.x + m->m[1][1] * p.y + m->m[1][2] * p.z + m->m[1][3];
    float z = m->m[2][0] * p.x + m->m[2][1] * p.y + m->m[2][2] * p.z + m->m[2][3];
    float w = m->m[3][0] * p.x + m->m[3][1] * p.y + m->m[3][2] * p.z + m->m[3][3];
    if (w == 1.0f) return v3(x, y, z);
    return vdiv(v3(x, y, z), w);
}
static V3 xf_point_affine(const M4 *m, V3 p) { /* transform.h:128-136 */
    float x = m->m[0][0] * p.x + m->m[0][1] * p.y + m->m[0][2] * p.z + m->m[0][3];
    float y = m->m[1][0] * p.x + m->m[1][1] * p.y + m->m[1][2] * p.z + m->m[1][3];
    float z = m->m[2][0] * p.x + m->m[2][1] * p.y + m->m[2][2] * p.z + m->m[2][3];
    return v3(x, y, z);
}
static V3 xf_vector(const M4 *m, V3 v) { /* transform.h:175-183 */
    float x = m->m[0][0] * v.x + m->m[0][1] * v.y + m->m[0][2] * v.z;
    float y = m->m[1][0] * v.x + m->m[1][1] * v.y + m->m[1][2] * v.z;
    float z = m->m[2][0] * v.x + m->m[2][1] * v.y + m->m[2][2] * v.z;
    return v3(x, y, z);
}

/* ------------------------------------------------------------------------ */
/* perspective camera (perspective.cpp:126-163,271-298; sensor.cpp:95-107,   */
/* 239-305)                                                                  */
/* ------------------------------------------------------------------------ */
typedef struct {
    M4 sampleToCamera, toWorld;
    float invResX, invResY, nearClip, farClip;
    V3 dx, dy;
} Camera;

static int camera_configure(const mtsgpu_sensor_desc *s, Camera *cam) {
    if (s->film_width == 0 || s->film_height == 0) return MTSGPU_EINVAL;
    float aspect = (float)s->film_width / (float)s->film_height;
    float xfov = s->fov;
    int axis = s->fov_axis;
    if (axis == MTSGPU_FOV_SMALLER) axis = aspect > 1 ? MTSGPU_FOV_Y : MTSGPU_FOV_X;
    else if (axis == MTSGPU_FOV_LARGER) axis = aspect > 1 ? MTSGPU_FOV_X : MTSGPU_FOV_Y;
    if (axis == MTSGPU_FOV_Y) {
        xfov = rad_to_deg(2 * atanf(tanf(0.5f * deg_to_rad(s->fov)) * aspect));
    } else if (axis == MTSGPU_FOV_DIAGONAL) {
        float diagonal = 2 * tanf(0.5f * deg_to_rad(s->fov));
        float width = diagonal / sqrtf(1.0f + 1.0f / (aspect * aspect));
        xfov = rad_to_deg(2 * atanf(width * 0.5f));
    }
    if (!(xfov > 0 && xfov < 180)) return MTSGPU_EINVAL;
    if (!(s->near_clip > 0) || !(s->near_clip < s->far_clip)) return MTSGPU_EINVAL;
    /* crop = film: relSize = 1, relOffset = 0 */
    Xform a = xf_scale(1.0f / 1.0f, 1.0f / 1.0f, 1.0f);
    Xform b = xf_translate(-0.0f, -0.0f, 0.0f);
    Xform c = xf_scale(-0.5f, -0.5f * aspect, 1.0f);
    Xform d = xf_translate(-1.0f, -1.0f / aspect, 0.0f);
    Xform p;
    if (!xf_perspective(xfov, s->near_clip, s->far_clip, &p)) return MTSGPU_EINVAL;
    Xform ab = xf_compose(&a, &b);
    Xform abc = xf_compose(&ab, &c);
    Xform abcd = xf_compose(&abc, &d);
    Xform camToSample = xf_compose(&abcd, &p);
    cam->sampleToCamera = camToSample.inv;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) cam->toWorld.m[i][j] = s->to_world[i * 4 + j];
    cam->invResX = (float)1 / (float)s->film_width;
    cam->invResY = (float)1 / (float)s->film_height;
    cam->nearClip = s->near_clip;
    cam->farClip = s->far_clip;
    V3 o0 = xf_point(&cam->sampleToCamera, v3(0.0f, 0.0f, 0.0f));
    cam->dx = vsub(xf_point(&cam->sampleToCamera, v3(cam->invResX, 0.0f, 0.0f)), o0);
    cam->dy = vsub(xf_point(&cam->sampleToCamera, v3(0.0f, cam->invResY, 0.0f)), o0);
    return MTSGPU_OK;
}

typedef struct {
    V3 o, d, dRcp;
    float mint, maxt;
    int hasDiff;
    V3 rxO, ryO, rxD, ryD;
} Ray;

static inline void ray_set_dir(Ray *r, V3 d) {
    r->d = d;
    r->dRcp = v3((float)1 / d.x, (float)1 / d.y, (float)1 / d.z);
}
static inline V3 ray_at(const Ray *r, float t) { return vadd(r->o, vmul(r->d, t)); }

/* PerspectiveCameraImpl::sampleRayDifferential (perspective.cpp:271-298) */
static void camera_sample_ray(const Camera *cam, float sx, float sy, Ray *ray) {
    V3 nearP = xf_point(&cam->sampleToCamera, v3(sx * cam->invResX, sy * cam->invResY, 0.0f));
    V3 d = vnormalize(nearP);
    float invZ = 1.0f / d.z;
    ray->mint = cam->nearClip * invZ;
    ray->maxt = cam->farClip * invZ;
    ray->o = xf_point_affine(&cam->toWorld, v3(0.0f, 0.0f, 0.0f));
    ray_set_dir(ray, xf_vector(&cam->toWorld, d));
    ray->rxO = ray->ryO = ray->o;
    ray->rxD = xf_vector(&cam->toWorld, vnormalize(vadd(nearP, cam->dx)));
    ray->ryD = xf_vector(&cam->toWorld, vnormalize(vadd(nearP, cam->dy)));
    ray->hasDiff = 1;
}

/* ------------------------------------------------------------------------ */
/* Sobol sampler (samplers/sobol.cpp:147-258, samplers/sobolseq.h:43-130)    */
/* Direction numbers: Joe & Kuo (sobolseq.cpp:21-27), regenerated here from  */
/* the published parameters with the Sobol' recurrence.                      */
/* ------------------------------------------------------------------------ */
#define SOBOL_DIMS 1024
#define SOBOL_SIZE 52
static uint32_t g_sobol[SOBOL_DIMS * SOBOL_SIZE];
static int g_sobol_ready = 0;

int oracle_sobol_init(const char *path) {
    FILE *f = fopen(path, "r");
    if (!f) return MTSGPU_EINVAL;
    uint64_t m[SOBOL_SIZE];
    for (int k = 0; k < SOBOL_SIZE; ++k) g_sobol[k] = (uint32_t)(((uint64_t)1 << (SOBOL_SIZE - 1 - k)) >> 20);
    char line[1024];
    int dims = 1;
    while (fgets(line, sizeof line, f)) {
        if (line[0] == '#' || line[0] == '\n') continue;
        char *p = line;
        long d = strtol(p, &p, 10), s = strtol(p, &p, 10), a = strtol(p, &p, 10);
        if (d < 2 || d > SOBOL_DIMS || s < 1 || s > 20) { fclose(f); return MTSGPU_EINVAL; }
        for (int i = 0; i < s; ++i) m[i] = (uint64_t)strtoull(p, &p, 10);
        for (int k = (int)s; k < SOBOL_SIZE; ++k) {
            uint64_t v = m[k - s] ^ (m[k - s] << s);
            for (int i = 1; i < s; ++i)
                if ((a >> (s - 1 - i)) & 1) v ^= m[k - i] << i;
            m[k] = v;
        }
        for (int k = 0; k < SOBOL_SIZE; ++k)
            g_sobol[(d - 1) * SOBOL_SIZE + k] = (uint32_t)((m[k] << (SOBOL_SIZE - 1 - k)) >> 20);
        dims++;
    }
    fclose(f);
    if (dims != SOBOL_DIMS) return MTSGPU_EINVAL;
    g_sobol_ready = 1;
    return MTSGPU_OK;
}

uint32_t oracle_sobol_matrix(uint32_t dim, uint32_t col) { return g_sobol[dim * SOBOL_SIZE + col]; }

/* sobol::sampleSingle (sobolseq.h:43-57) */
float oracle_sobol_sample(uint64_t index, uint32_t dim, uint32_t scramble) {
    uint32_t result = scramble;
    for (uint32_t i = dim * SOBOL_SIZE; index; index >>= 1, ++i)
        if (index & 1) result ^= g_sobol[i];
    return smin(result * (1.0f / (float)(1ULL << 32)), ONE_MINUS_EPS_F);
}

/* sobol::look_up (sobolseq.h:93-125): the index of the frame-th sample of the
 * (0,2)-sequence in pixel (px,py) at resolution 2^m.  Restated as the GF(2)
 * solve it encodes: the van der Corput coordinate fixes the low m index bits,
 * the second Sobol coordinate fixes bits m..2m-1 through an m x m system. */
typedef struct { uint32_t m; uint32_t inv[32]; uint32_t ycol[64]; } LookupTable;
static LookupTable g_lut[32];
static int g_lut_ready[32];

static void lookup_prepare(uint32_t m) {
    LookupTable *L = &g_lut[m];
    L->m = m;
    for (int b = 0; b < 64; ++b) L->ycol[b] = (b < SOBOL_SIZE) ? (g_sobol[SOBOL_SIZE + b] >> (32 - m)) : 0;
    /* rows: A[r] bit t = bit r of ycol[m+t]; invert with [A | I] */
    uint32_t A[32], I[32];
    for (uint32_t r = 0; r < m; ++r) {
        A[r] = 0; I[r] = 1u << r;
        for (uint32_t t = 0; t < m; ++t) A[r] |= ((L->ycol[m + t] >> r) & 1u) << t;
    }
    for (uint32_t c = 0; c < m; ++c) {
        uint32_t piv = c;
        while (piv < m && !((A[piv] >> c) & 1u)) ++piv;
        if (piv == m) { fprintf(stderr, "sobol look_up: singular system m=%u\n", m); abort(); }
        uint32_t ta = A[c]; A[c] = A[piv]; A[piv] = ta;
        uint32_t ti = I[c]; I[c] = I[piv]; I[piv] = ti;
        for (uint32_t r = 0; r < m; ++r)
            if (r != c && ((A[r] >> c) & 1u)) { A[r] ^= A[c]; I[r] ^= I[c]; }
    }
    /* now A = I, so x = Ainv*rhs: bit t of x = parity(I[t] & rhs) */
    for (uint32_t t = 0; t < m; ++t) L->inv[t] = I[t];
}

uint64_t oracle_sobol_lookup(uint32_t m, uint32_t frame, uint32_t px, uint32_t py, uint64_t scramble) {
    if (m == 0 || m > 31) return (uint64_t)frame;
    if (!g_lut_ready[m]) { lookup_prepare(m); g_lut_ready[m] = 1; }
    const LookupTable *L = &g_lut[m];
    uint32_t s = (uint32_t)((scramble & 0xFFFFFFFFull) >> (32 - m));
    uint32_t sx = px ^ s, sy = py ^ s;
    uint32_t mask = (m == 32) ? 0xFFFFFFFFu : ((1u << m) - 1u);
    sx &= mask; sy &= mask;
    uint64_t jlo = 0;
    for (uint32_t t = 0; t < m; ++t) jlo |= (uint64_t)((sx >> (m - 1 - t)) & 1u) << t;
    uint64_t index = ((uint64_t)frame << (2 * m)) | jlo;
    uint32_t K = 0;
    for (uint32_t b = 0; b < 64; ++b)
        if ((index >> b) & 1) K ^= L->ycol[b];
    uint32_t rhs = (sy ^ K) & mask;
    uint64_t jhi = 0;
    for (uint32_t t = 0; t < m; ++t) jhi |= (uint64_t)(__builtin_parity(L->inv[t] & rhs)) << t;
    return index | (jhi << m);
}

/* sampleTEA (core/qmc.h:146-156) */
static uint64_t sample_tea(uint32_t v0, uint32_t v1, int rounds) {
    uint32_t sum = 0;
    for (int i = 0; i < rounds; ++i) {
        sum += 0x9e3779b9;
        v0 += ((v1 << 4) + 0xA341316C) ^ (v1 + sum) ^ ((v1 >> 5) + 0xC8013EA4);
        v1 += ((v0 << 4) + 0xAD90777D) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7E95761E);
    }
    return ((uint64_t)v1 << 32) + v0;
}

typedef struct {
    uint64_t scramble;
    float resolution;
    uint32_t logRes;
    int px, py;
    uint64_t sampleIndex, sobolIndex;
    uint32_t dim;
    uint32_t arrayEnd; /* m_arrayEndDim: dims [5, arrayEnd) hold the requested 2D arrays */
    int err;
    int indep;         /* the `independent` sampler (independent.cpp) instead of `sobol` */
    struct SfmtState *rng;   /* SFMT replay: Random::nextFloat draws of the worker's stream */
} Sampler;

/* The independent sampler's stream (independent.cpp:82-104).  The reference
 * draws from one SFMT19937 generator per worker thread, so its values depend on
 * the block schedule and are not reproducible.  Here every
 * (pixel, sample) owns a counter-based stream: a splitmix64-finalised key and
 * one finalised draw per dimension; Random::nextFloat's [1,2) - 1 conversion
 * of the low 32 bits (random.cpp:630-639).  Same function as the kernel's. */
static uint64_t indep_mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint64_t indep_key(uint32_t px, uint32_t py, uint32_t frame) {
    return indep_mix64((((uint64_t)px << 48) | ((uint64_t)py << 32) | frame) ^ 0x6A09E667F3BCC909ull);
}
static float indep_float(uint64_t key, uint32_t dim) {
    const uint32_t u = (uint32_t)indep_mix64(key + (uint64_t)(dim + 1) * 0x9E3779B97F4A7C15ull);
    union { uint32_t u; float f; } x;
    x.u = (u >> 9) | 0x3f800000u;
    return x.f - 1.0f;
}
static float smp_value(const Sampler *s, uint64_t idx, uint32_t dim) {
    return s->indep ? indep_float(idx, dim) : oracle_sobol_sample(idx, dim, (uint32_t)s->scramble);
}

static void sampler_init(Sampler *s, uint64_t scramble, uint32_t w, uint32_t h) {
    memset(s, 0, sizeof *s);
    s->scramble = scramble;
    if (scramble) s->scramble = sample_tea((uint32_t)scramble, (uint32_t)(scramble >> 32), 4);
    /* setFilmResolution(cropSize, bucketed = true) (sobol.cpp:147-158, integrator.cpp:38-41) */
    uint32_t v = w > h ? w : h;
    uint32_t r = v - 1; r |= r >> 1; r |= r >> 2; r |= r >> 4; r |= r >> 8; r |= r >> 16; r += 1;
    s->resolution = (float)r;
    uint32_t lg = 0; while ((1u << lg) < r) ++lg;
    s->logRes = lg;
    s->arrayEnd = 5;
}

static void sampler_set_index(Sampler *s, uint64_t idx) { /* sobol.cpp:204-217 */
    s->dim = 0;
    s->sampleIndex = idx;
    if (s->indep)
        s->sobolIndex = indep_key((uint32_t)s->px, (uint32_t)s->py, (uint32_t)idx);
    else if (s->logRes > 1 && s->px >= 0)
        s->sobolIndex = oracle_sobol_lookup(s->logRes, (uint32_t)idx, (uint32_t)s->px, (uint32_t)s->py, s->scramble);
    else
        s->sobolIndex = idx;
}
static void sampler_generate(Sampler *s, int px, int py) { s->px = px; s->py = py; sampler_set_index(s, 0); }

static float sfmt_next_float(struct SfmtState *s);
static float next1d(Sampler *s) { /* sobol.cpp:219-229; dims [5, arrayEnd) are the arrays' */
    if (s->rng) { s->dim++; return sfmt_next_float(s->rng); }   /* independent.cpp:97-99 */
    if (s->dim >= 5 && s->dim < s->arrayEnd) s->dim = s->arrayEnd;
    if (s->dim >= SOBOL_DIMS && !s->indep) { s->err = 1; return 0.0f; }
    return smp_value(s, s->sobolIndex, s->dim++);
}
static void next2d(Sampler *s, float *u, float *v) { /* sobol.cpp:231-250 */
    if (s->rng) {   /* independent.cpp:101-105: value1 then value2 */
        *u = sfmt_next_float(s->rng);
        *v = sfmt_next_float(s->rng);
        s->dim += 2;
        return;
    }
    if (s->dim + 1 >= 5 && s->dim < s->arrayEnd) s->dim = s->arrayEnd;
    if (s->dim + 1 >= SOBOL_DIMS && !s->indep) { s->err = 1; *u = *v = 0.0f; return; }
    if (s->indep) {
        *u = indep_float(s->sobolIndex, s->dim++);
        *v = indep_float(s->sobolIndex, s->dim++);
    } else if (s->dim == 0 && s->sobolIndex != s->sampleIndex) {
        *u = oracle_sobol_sample(s->sobolIndex, s->dim++, (uint32_t)s->scramble) * s->resolution - (float)s->px;
        *v = oracle_sobol_sample(s->sobolIndex, s->dim++, (uint32_t)s->scramble) * s->resolution - (float)s->py;
    } else {
        *u = oracle_sobol_sample(s->sobolIndex, s->dim++, (uint32_t)s->scramble);
        *v = oracle_sobol_sample(s->sobolIndex, s->dim++, (uint32_t)s->scramble);
    }
}

/* element k of this sample's requested 2D array of `size` points starting at
 * dimension `dim`: Sampler::next2DArray (sampler.cpp:82-92) over the arrays
 * SobolSampler::generate fills (sobol.cpp:171-197) */
static void sampler_array2d(const Sampler *s, uint32_t dim, uint32_t size, uint32_t k, float *u, float *v) {
    uint32_t j = (uint32_t)(s->sampleIndex * size + k);
    uint64_t idx = s->indep ? indep_key((uint32_t)s->px, (uint32_t)s->py, j)
                            : oracle_sobol_lookup(s->logRes, j, (uint32_t)s->px, (uint32_t)s->py, s->scramble);
    *u = smp_value(s, idx, dim);
    *v = smp_value(s, idx, dim + 1);
}

/* ------------------------------------------------------------------------ */
/* SFMT19937 (libcore/random.cpp:68-471, the generic (non-SSE) recursion,     */
/* which the SSE path reproduces) and Random::nextULong / nextFloat /         */
/* seed(Random *) (random.cpp:524-553, 630-639).  Pinned by the reference's   */
/* own output vectors (src/tests/test_random.cpp:433-508).                    */
/* ------------------------------------------------------------------------ */
#define SFMT_N 156
#define SFMT_N32 624
#define SFMT_N64 312
#define SFMT_POS1 122
#define SFMT_SL1 18
#define SFMT_SL2 1
#define SFMT_SR1 11
#define SFMT_SR2 1
static const uint32_t SFMT_MSK[4] = {0xdfffffefu, 0xddfecb7fu, 0xbffaffffu, 0xbffffff6u};
static const uint32_t SFMT_PARITY[4] = {0x00000001u, 0x00000000u, 0x00000000u, 0x13c9e684u};

typedef struct SfmtState { uint32_t w[SFMT_N32]; int idx; } Sfmt;

/* 128-bit little-endian shifts by `bytes` (random.cpp:139-171) */
static void sfmt_shift_left(uint32_t out[4], const uint32_t in[4], int bytes) {
    const uint64_t lo = (uint64_t)in[0] | ((uint64_t)in[1] << 32), hi = (uint64_t)in[2] | ((uint64_t)in[3] << 32);
    const uint64_t ohi = (hi << (bytes * 8)) | (lo >> (64 - bytes * 8)), olo = lo << (bytes * 8);
    out[0] = (uint32_t)olo; out[1] = (uint32_t)(olo >> 32); out[2] = (uint32_t)ohi; out[3] = (uint32_t)(ohi >> 32);
}
static void sfmt_shift_right(uint32_t out[4], const uint32_t in[4], int bytes) {
    const uint64_t lo = (uint64_t)in[0] | ((uint64_t)in[1] << 32), hi = (uint64_t)in[2] | ((uint64_t)in[3] << 32);
    const uint64_t olo = (lo >> (bytes * 8)) | (hi << (64 - bytes * 8)), ohi = hi >> (bytes * 8);
    out[0] = (uint32_t)olo; out[1] = (uint32_t)(olo >> 32); out[2] = (uint32_t)ohi; out[3] = (uint32_t)(ohi >> 32);
}
/* do_recursion (random.cpp:204-219): r = a ^ (a << 8) ^ ((b >> 11) & MSK) ^ (c >> 8) ^ (d << 18) */
static void sfmt_recursion(uint32_t *r, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
    uint32_t x[4], y[4];
    sfmt_shift_left(x, a, SFMT_SL2);
    sfmt_shift_right(y, c, SFMT_SR2);
    for (int k = 0; k < 4; ++k) r[k] = a[k] ^ x[k] ^ ((b[k] >> SFMT_SR1) & SFMT_MSK[k]) ^ y[k] ^ (d[k] << SFMT_SL1);
}
static void sfmt_gen_all(Sfmt *s) {   /* gen_rand_all (random.cpp:353-390) */
    uint32_t *r1 = &s->w[4 * (SFMT_N - 2)], *r2 = &s->w[4 * (SFMT_N - 1)];
    int i;
    for (i = 0; i < SFMT_N - SFMT_POS1; ++i) {
        uint32_t r[4];
        sfmt_recursion(r, &s->w[4 * i], &s->w[4 * (i + SFMT_POS1)], r1, r2);
        memcpy(&s->w[4 * i], r, sizeof r);
        r1 = r2; r2 = &s->w[4 * i];
    }
    for (; i < SFMT_N; ++i) {
        uint32_t r[4];
        sfmt_recursion(r, &s->w[4 * i], &s->w[4 * (i + SFMT_POS1 - SFMT_N)], r1, r2);
        memcpy(&s->w[4 * i], r, sizeof r);
        r1 = r2; r2 = &s->w[4 * i];
    }
}
static void sfmt_period_certification(Sfmt *s) {   /* random.cpp:322-347 */
    uint32_t inner = 0;
    for (int i = 0; i < 4; ++i) inner ^= s->w[i] & SFMT_PARITY[i];
    for (int i = 16; i > 0; i >>= 1) inner ^= inner >> i;
    if (inner & 1) return;
    for (int i = 0; i < 4; ++i) {
        uint32_t work = 1;
        for (int j = 0; j < 32; ++j) {
            if (work & SFMT_PARITY[i]) { s->w[i] ^= work; return; }
            work <<= 1;
        }
    }
}
static void sfmt_init_gen_rand(Sfmt *s, uint64_t seed) {   /* random.cpp:397-406 */
    uint64_t v = seed;
    s->w[0] = (uint32_t)v; s->w[1] = (uint32_t)(v >> 32);
    for (int i = 1; i < SFMT_N64; ++i) {
        v = 6364136223846793005ull * (v ^ (v >> 62)) + (uint64_t)i;
        s->w[2 * i] = (uint32_t)v; s->w[2 * i + 1] = (uint32_t)(v >> 32);
    }
    s->idx = SFMT_N32;
    sfmt_period_certification(s);
}
static uint32_t sfmt_func1(uint32_t x) { return (x ^ (x >> 27)) * 1664525u; }
static uint32_t sfmt_func2(uint32_t x) { return (x ^ (x >> 27)) * 1566083941u; }
static void sfmt_init_by_array(Sfmt *s, const uint32_t *key, int len) {   /* random.cpp:408-471 */
    const int size = SFMT_N32, lag = 11, mid = (size - lag) / 2;
    uint32_t *p = s->w;
    memset(p, 0x8b, sizeof s->w);
    int count = len + 1 > SFMT_N32 ? len + 1 : SFMT_N32;
    uint32_t r = sfmt_func1(p[0] ^ p[mid] ^ p[SFMT_N32 - 1]);
    p[mid] += r;
    r += (uint32_t)len;
    p[mid + lag] += r;
    p[0] = r;
    count--;
    int i = 1, j = 0;
    for (; j < count && j < len; j++) {
        r = sfmt_func1(p[i] ^ p[(i + mid) % SFMT_N32] ^ p[(i + SFMT_N32 - 1) % SFMT_N32]);
        p[(i + mid) % SFMT_N32] += r;
        r += key[j] + (uint32_t)i;
        p[(i + mid + lag) % SFMT_N32] += r;
        p[i] = r;
        i = (i + 1) % SFMT_N32;
    }
    for (; j < count; j++) {
        r = sfmt_func1(p[i] ^ p[(i + mid) % SFMT_N32] ^ p[(i + SFMT_N32 - 1) % SFMT_N32]);
        p[(i + mid) % SFMT_N32] += r;
        r += (uint32_t)i;
        p[(i + mid + lag) % SFMT_N32] += r;
        p[i] = r;
        i = (i + 1) % SFMT_N32;
    }
    for (j = 0; j < SFMT_N32; j++) {
        r = sfmt_func2(p[i] + p[(i + mid) % SFMT_N32] + p[(i + SFMT_N32 - 1) % SFMT_N32]);
        p[(i + mid) % SFMT_N32] ^= r;
        r -= (uint32_t)i;
        p[(i + mid + lag) % SFMT_N32] ^= r;
        p[i] = r;
        i = (i + 1) % SFMT_N32;
    }
    s->idx = SFMT_N32;
    sfmt_period_certification(s);
}
static uint64_t sfmt_next64(Sfmt *s) {   /* gen_rand64 (random.cpp:288-297) */
    if (s->idx >= SFMT_N32) { sfmt_gen_all(s); s->idx = 0; }
    const uint64_t r = (uint64_t)s->w[s->idx] | ((uint64_t)s->w[s->idx + 1] << 32);
    s->idx += 2;
    return r;
}
static float sfmt_next_float(struct SfmtState *s) {   /* Random::nextFloat, SINGLE_PRECISION (random.cpp:630-639) */
    union { uint32_t u; float f; } x;
    x.u = ((uint32_t)(sfmt_next64(s) & 0xFFFFFFFFull) >> 9) | 0x3f800000u;
    return x.f - 1.0f;
}
/* Random(Random *parent) = seed(parent): 312 of the parent's outputs as the
 * init_by_array key, little-endian 32-bit words (random.cpp:528-548) */
static void sfmt_clone(Sfmt *child, Sfmt *parent) {
    uint32_t key[SFMT_N32];
    for (int i = 0; i < SFMT_N64; ++i) {
        const uint64_t v = sfmt_next64(parent);
        key[2 * i] = (uint32_t)v; key[2 * i + 1] = (uint32_t)(v >> 32);
    }
    sfmt_init_by_array(child, key, SFMT_N32);
}

/* test access: the first n outputs of Random(seed), or (clone >= 1) of the
   clone-th Random(&master) clone of it */
int oracle_sfmt_u64(uint64_t seed, uint64_t *out, int n, int clone) {
    Sfmt s, c;
    sfmt_init_gen_rand(&s, seed);
    for (int k = 0; k < clone; ++k) sfmt_clone(&c, &s);
    Sfmt *g = clone > 0 ? &c : &s;
    for (int i = 0; i < n; ++i) out[i] = sfmt_next64(g);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* The reference's render order, for the SFMT replay samplers:               */
/* BlockedImageProcess's spiral over blocks (librender/imageproc.cpp:28-80)   */
/* and each block's pixels along HilbertCurve2D<uint8_t> (core/sfcurve.h,     */
/* renderproc.cpp:79-81).  out: (x, y) pairs relative to the crop window;     */
/* block_start[b] = index of block b's first pixel, block_start[total] = n.  */
/* ------------------------------------------------------------------------ */
static void hilbert_gen(int order, int front, int right, int back, int left, uint8_t *pos, uint8_t w, uint8_t h,
                        int bx, int by, int *out, int *n) {
    if (order == 0) {
        if (pos[0] < w && pos[1] < h) { out[2 * *n] = bx + pos[0]; out[2 * *n + 1] = by + pos[1]; ++*n; }
        return;
    }
    /* move(dir) in uint8_t arithmetic: ENorth y--, EEast x++, ESouth y++, EWest x-- */
#define HMOVE(d) do { if ((d) == 0) pos[1]--; else if ((d) == 1) pos[0]++; else if ((d) == 2) pos[1]++; else pos[0]--; } while (0)
    hilbert_gen(order - 1, left, back, right, front, pos, w, h, bx, by, out, n); HMOVE(right);
    hilbert_gen(order - 1, front, right, back, left, pos, w, h, bx, by, out, n); HMOVE(back);
    hilbert_gen(order - 1, front, right, back, left, pos, w, h, bx, by, out, n); HMOVE(left);
    hilbert_gen(order - 1, right, front, left, back, pos, w, h, bx, by, out, n);
#undef HMOVE
}
int oracle_render_order(int width, int height, int blockSize, int *out, int *block_start, int *num_blocks) {
    const int nbx = (int)ceilf((float)width / (float)blockSize), nby = (int)ceilf((float)height / (float)blockSize);
    const int total = nbx * nby;
    /* EDirection {ERight = 0, EDown, ELeft, EUp} (render/imageproc.h:65-70) */
    int cx = nbx / 2, cy = nby / 2, dir = 0, stepsLeft = 1, numSteps = 1, n = 0;
    const float invLog2 = 1.0f / (float)log((double)2.0f);   /* math::fastlog in double (math.h:193-195) */
    for (int b = 0; b < total; ++b) {
        const int bw = width - cx * blockSize < blockSize ? width - cx * blockSize : blockSize;
        const int bh = height - cy * blockSize < blockSize ? height - cy * blockSize : blockSize;
        block_start[b] = n;
        const int mx = bw > bh ? bw : bh;
        const int order = (int)ceilf(invLog2 * (float)log((double)(float)mx));
        uint8_t pos[2] = {0, 0};
        /* generate(order, ENorth, EEast, ESouth, EWest): N = 0, E = 1, S = 2, W = 3 */
        hilbert_gen(order, 0, 1, 2, 3, pos, (uint8_t)bw, (uint8_t)bh, cx * blockSize, cy * blockSize, out, &n);
        if (b + 1 == total) break;
        do {
            if (dir == 0) ++cx; else if (dir == 1) ++cy; else if (dir == 2) --cx; else --cy;
            if (--stepsLeft == 0) {
                dir = (dir + 1) % 4;
                if (dir == 2 || dir == 0) ++numSteps;
                stepsLeft = numSteps;
            }
        } while (cx < 0 || cy < 0 || cx >= nbx || cy >= nby);
    }
    block_start[total] = n;
    *num_blocks = total;
    return n;
}

/* ------------------------------------------------------------------------ */
/* warps (libcore/warp.cpp:43-102, include/mitsuba/core/warp.h:55-56)        */
/* ------------------------------------------------------------------------ */
static void square_to_disk_concentric(float sx, float sy, float *px, float *py) {
    float r1 = 2.0f * sx - 1.0f;
    float r2 = 2.0f * sy - 1.0f;
    float phi, r;
    if (r1 == 0 && r2 == 0) {
        r = phi = 0;
    } else if (r1 * r1 > r2 * r2) {
        r = r1;
        phi = (M_PI_F / 4.0f) * (r2 / r1);
    } else {
        r = r2;
        phi = (M_PI_F / 2.0f) - (r1 / r2) * (M_PI_F / 4.0f);
    }
    float c, s;
    o_sincos(phi, &s, &c);
    *px = r * c;
    *py = r * s;
}
static V3 square_to_cosine_hemisphere(float sx, float sy) {
    float px, py;
    square_to_disk_concentric(sx, sy, &px, &py);
    float z = safe_sqrt(1.0f - px * px - py * py);
    if (z == 0) z = 1e-10f;
    return v3(px, py, z);
}
static inline float cosine_hemisphere_pdf(V3 d) { return INV_PI_F * d.z; }

/* ------------------------------------------------------------------------ */
/* math::erf / erfinv / hypot2 (libcore/math.cpp:25-95)                       */
/* ------------------------------------------------------------------------ */
static float m_erfinv(float x) {
    float w = -o_fastlog(((float)1 - x) * ((float)1 + x));
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
        w = sqrtf(w) - (float)3;
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
static float m_erf(float x) {
    float a1 = (float)0.254829592, a2 = (float)-0.284496736, a3 = (float)1.421413741;
    float a4 = (float)-1.453152027, a5 = (float)1.061405429, p = (float)0.3275911;
    float sign = signumf(x);
    x = fabsf(x);
    float t = (float)1.0 / ((float)1.0 + p * x);
    float y = (float)1.0 - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * o_fastexp(-x * x);
    return sign * y;
}
static float m_hypot2(float a, float b) {
    float r;
    if (fabsf(a) > fabsf(b)) { r = b / a; r = fabsf(a) * sqrtf(1.0f + r * r); }
    else if (b != 0.0f) { r = a / b; r = fabsf(b) * sqrtf(1.0f + r * r); }
    else r = 0.0f;
    return r;
}

/* ------------------------------------------------------------------------ */
/* MicrofacetDistribution (bsdfs/microfacet.h)                               */
/* ------------------------------------------------------------------------ */
typedef struct { int type; float alphaU, alphaV; int sampleVisible; float expU, expV; } Distr;

static void distr_init(Distr *d, int type, float au, float av, int sv) { /* microfacet.h:89-97 */
    d->type = type; d->alphaU = smax(au, 1e-4f); d->alphaV = smax(av, 1e-4f);
    d->sampleVisible = sv; d->expU = d->expV = 0.0f;
    if (type == MTSGPU_DISTR_PHONG) { /* computePhongExponent (:673-676) */
        d->expU = smax(2.0f / (d->alphaU * d->alphaU) - 2.0f, 0.0f);
        d->expV = smax(2.0f / (d->alphaV * d->alphaV) - 2.0f, 0.0f);
    }
}
static inline int distr_iso(const Distr *d) { return d->alphaU == d->alphaV; }

static float distr_interp_phong(const Distr *d, V3 v) { /* :538-549 */
    float st2 = sin_theta2(v);
    if (distr_iso(d) || st2 <= 0x1p-128f) return d->expU;
    float inv = 1 / st2;
    return d->expU * (v.x * v.x * inv) + d->expV * (v.y * v.y * inv);
}

static float distr_eval(const Distr *d, V3 m) { /* :191-238 */
    if (m.z <= 0) return 0.0f;
    float cosTheta2 = m.z * m.z;
    float beckmannExponent = ((m.x * m.x) / (d->alphaU * d->alphaU) + (m.y * m.y) / (d->alphaV * d->alphaV)) / cosTheta2;
    float result;
    if (d->type == MTSGPU_DISTR_BECKMANN) {
        result = o_fastexp(-beckmannExponent) / (M_PI_F * d->alphaU * d->alphaV * cosTheta2 * cosTheta2);
    } else if (d->type == MTSGPU_DISTR_GGX) {
        float root = ((float)1 + beckmannExponent) * cosTheta2;
        result = (float)1 / (M_PI_F * d->alphaU * d->alphaV * root * root);
    } else {
        float exponent = distr_interp_phong(d, m);
        result = sqrtf((d->expU + 2) * (d->expV + 2)) * INV_TWOPI_F * o_pow(m.z, exponent);
    }
    if (result * m.z < 1e-20f) result = 0;
    return result;
}

static float distr_project_roughness(const Distr *d, V3 v) { /* :526-536 */
    float invSinTheta2 = 1 / sin_theta2(v);
    if (distr_iso(d) || invSinTheta2 <= 0) return d->alphaU;
    float cosPhi2 = v.x * v.x * invSinTheta2;
    float sinPhi2 = v.y * v.y * invSinTheta2;
    return sqrtf(cosPhi2 * d->alphaU * d->alphaU + sinPhi2 * d->alphaV * d->alphaV);
}

static float distr_smithG1(const Distr *d, V3 v, V3 m) { /* :477-518 */
    if (vdot(v, m) * v.z <= 0) return 0.0f;
    float tanTheta = fabsf(tan_theta(v));
    if (tanTheta == 0.0f) return 1.0f;
    float alpha = distr_project_roughness(d, v);
    if (d->type == MTSGPU_DISTR_GGX) {
        float root = alpha * tanTheta;
        return 2.0f / (1.0f + m_hypot2((float)1.0f, root));
    }
    float a = 1.0f / (alpha * tanTheta);
    if (a >= 1.6f) return 1.0f;
    float aSqr = a * a;
    return (3.535f * a + 2.181f * aSqr) / (1.0f + 2.276f * a + 2.577f * aSqr);
}
static inline float distr_G(const Distr *d, V3 wi, V3 wo, V3 m) { return distr_smithG1(d, wi, m) * distr_smithG1(d, wo, m); }

static void distr_sample_first_quadrant(const Distr *d, float u1, float *phi, float *exponent) { /* :679-688 */
    float c, s;
    *phi = o_atan(sqrtf((d->expU + 2.0f) / (d->expV + 2.0f)) * o_tan(M_PI_F * u1 * 0.5f));
    o_sincos(*phi, &s, &c);
    *exponent = d->expU * c * c + d->expV * s * s;
}

static V3 distr_sample_all(const Distr *d, float sx, float sy, float *pdf) { /* :287-402 */
    float cosThetaM = 0.0f, sinPhiM, cosPhiM, alphaSqr;
    if (d->type == MTSGPU_DISTR_BECKMANN || d->type == MTSGPU_DISTR_GGX) {
        if (distr_iso(d)) {
            o_sincos((2.0f * M_PI_F) * sy, &sinPhiM, &cosPhiM);
            alphaSqr = d->alphaU * d->alphaU;
        } else {
            float phiM = o_atan(d->alphaV / d->alphaU * o_tan(M_PI_F + 2 * M_PI_F * sy)) + M_PI_F * floorf(2 * sy + 0.5f);
            o_sincos(phiM, &sinPhiM, &cosPhiM);
            float cosSc = cosPhiM / d->alphaU, sinSc = sinPhiM / d->alphaV;
            alphaSqr = 1.0f / (cosSc * cosSc + sinSc * sinSc);
        }
        if (d->type == MTSGPU_DISTR_BECKMANN) {
            float tanThetaMSqr = alphaSqr * -o_fastlog(1.0f - sx);
            cosThetaM = 1.0f / sqrtf(1.0f + tanThetaMSqr);
            *pdf = (1.0f - sx) / (M_PI_F * d->alphaU * d->alphaV * cosThetaM * cosThetaM * cosThetaM);
        } else {
            float tanThetaMSqr = alphaSqr * sx / (1.0f - sx);
            cosThetaM = 1.0f / sqrtf(1.0f + tanThetaMSqr);
            float temp = 1 + tanThetaMSqr / alphaSqr;
            *pdf = INV_PI_F / (d->alphaU * d->alphaV * cosThetaM * cosThetaM * cosThetaM * temp * temp);
        }
    } else {
        float phiM, exponent;
        if (distr_iso(d)) {
            phiM = (2.0f * M_PI_F) * sy;
            exponent = d->expU;
        } else {
            if (sy < 0.25f) {
                distr_sample_first_quadrant(d, 4 * sy, &phiM, &exponent);
            } else if (sy < 0.5f) {
                distr_sample_first_quadrant(d, 4 * (0.5f - sy), &phiM, &exponent);
                phiM = M_PI_F - phiM;
            } else if (sy < 0.75f) {
                distr_sample_first_quadrant(d, 4 * (sy - 0.5f), &phiM, &exponent);
                phiM += M_PI_F;
            } else {
                distr_sample_first_quadrant(d, 4 * (1 - sy), &phiM, &exponent);
                phiM = 2 * M_PI_F - phiM;
            }
        }
        o_sincos(phiM, &sinPhiM, &cosPhiM);
        cosThetaM = o_pow(sx, 1.0f / (exponent + 2.0f));
        *pdf = sqrtf((d->expU + 2.0f) * (d->expV + 2.0f)) * INV_TWOPI_F * o_pow(cosThetaM, exponent + 1.0f);
    }
    if (*pdf < 1e-20f) *pdf = 0;
    float sinThetaM = sqrtf(smax((float)0, 1 - cosThetaM * cosThetaM));
    return v3(sinThetaM * cosPhiM, sinThetaM * sinPhiM, cosThetaM);
}

static void distr_sample_visible11(const Distr *d, float thetaI, float sx, float sy, float *slx, float *sly) { /* :573-670 */
    const float SQRT_PI_INV = 1 / sqrtf(M_PI_F);
    if (d->type == MTSGPU_DISTR_BECKMANN) {
        if (thetaI < 1e-4f) {
            float s, c;
            float r = sqrtf(-o_fastlog(1.0f - sx));
            o_sincos(2 * M_PI_F * sy, &s, &c);
            *slx = r * c; *sly = r * s;
            return;
        }
        float tanThetaI = o_tan(thetaI);
        float cotThetaI = 1 / tanThetaI;
        float a = -1, c = m_erf(cotThetaI);
        float sample_x = smax(sx, (float)1e-6f);
        float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
        float b = c - (1 + c) * o_pow(1 - sample_x, fit);
        float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * o_exp(-cotThetaI * cotThetaI));
        int it = 0;
        while (++it < 10) {
            if (!(b >= a && b <= c)) b = 0.5f * (a + c);
            float invErf = m_erfinv(b);
            float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * o_exp(-invErf * invErf)) - sample_x;
            float derivative = normalization * (1 - invErf * tanThetaI);
            if (fabsf(value) < 1e-5f) break;
            if (value > 0) c = b; else a = b;
            b -= value / derivative;
        }
        *slx = m_erfinv(b);
        *sly = m_erfinv(2.0f * smax(sy, (float)1e-6f) - 1.0f);
        return;
    }
    /* GGX */
    if (thetaI < 1e-4f) {
        float s, c;
        float r = safe_sqrt(sx / (1 - sx));
        o_sincos(2 * M_PI_F * sy, &s, &c);
        *slx = r * c; *sly = r * s;
        return;
    }
    float tanThetaI = o_tan(thetaI);
    float a = 1 / tanThetaI;
    float G1 = 2.0f / (1.0f + safe_sqrt(1.0f + 1.0f / (a * a)));
    float A = 2.0f * sx / G1 - 1.0f;
    if (fabsf(A) == 1) A -= signumf(A) * EPSILON;
    float tmp = 1.0f / (A * A - 1.0f);
    float B = tanThetaI;
    float D = safe_sqrt(B * B * tmp * tmp - (A * A - B * B) * tmp);
    float slope_x_1 = B * tmp - D;
    float slope_x_2 = B * tmp + D;
    *slx = (A < 0.0f || slope_x_2 > 1.0f / tanThetaI) ? slope_x_1 : slope_x_2;
    float S;
    if (sy > 0.5f) { S = 1.0f; sy = 2.0f * (sy - 0.5f); }
    else { S = -1.0f; sy = 2.0f * (0.5f - sy); }
    float z = (sy * (sy * (sy * (-(float)0.365728915865723) + (float)0.790235037209296) - (float)0.424965825137544) + (float)0.000152998850436920) /
              (sy * (sy * (sy * (sy * (float)0.169507819808272 - (float)0.397203533833404) - (float)0.232500544458471) + (float)1) - (float)0.539825872510702);
    *sly = S * z * sqrtf(1.0f + (*slx) * (*slx));
}

static V3 distr_sample_visible(const Distr *d, V3 _wi, float sx, float sy) { /* :421-460 */
    V3 wi = vnormalize(v3(d->alphaU * _wi.x, d->alphaV * _wi.y, _wi.z));
    float theta = 0, phi = 0;
    if (wi.z < (float)0.99999) {
        theta = o_acos(wi.z);
        phi = o_atan2(wi.y, wi.x);
    }
    float sinPhi, cosPhi;
    o_sincos(phi, &sinPhi, &cosPhi);
    float slx, sly;
    distr_sample_visible11(d, theta, sx, sy, &slx, &sly);
    float nx = cosPhi * slx - sinPhi * sly;
    float ny = sinPhi * slx + cosPhi * sly;
    nx *= d->alphaU;
    ny *= d->alphaV;
    float normalization = (float)1 / sqrtf(nx * nx + ny * ny + (float)1.0);
    return v3(-nx * normalization, -ny * normalization, normalization);
}

static float distr_pdf_visible(const Distr *d, V3 wi, V3 m) { /* :462-466 */
    if (wi.z == 0) return 0.0f;
    return distr_smithG1(d, wi, m) * vabsdot(wi, m) * distr_eval(d, m) / fabsf(wi.z);
}
static float distr_pdf(const Distr *d, V3 wi, V3 m) { /* :270-276 */
    if (d->sampleVisible) return distr_pdf_visible(d, wi, m);
    return distr_eval(d, m) * m.z;
}
static V3 distr_sample(const Distr *d, V3 wi, float sx, float sy, float *pdf) { /* :243-253 */
    if (d->sampleVisible) {
        V3 m = distr_sample_visible(d, wi, sx, sy);
        *pdf = distr_pdf_visible(d, wi, m);
        return m;
    }
    return distr_sample_all(d, sx, sy, pdf);
}
static void distr_scale_alpha(Distr *d, float v) { /* :181-186 */
    d->alphaU *= v; d->alphaV *= v;
    if (d->type == MTSGPU_DISTR_PHONG) {
        d->expU = smax(2.0f / (d->alphaU * d->alphaU) - 2.0f, 0.0f);
        d->expV = smax(2.0f / (d->alphaV * d->alphaV) - 2.0f, 0.0f);
    }
}

/* ------------------------------------------------------------------------ */
/* Fresnel (libcore/util.cpp:651-771)                                        */
/* ------------------------------------------------------------------------ */
static float fresnel_dielectric_ext(float cosThetaI_, float *cosThetaT_, float eta) {
    if (eta == 1) { *cosThetaT_ = -cosThetaI_; return 0.0f; }
    float scale = (cosThetaI_ > 0) ? 1 / eta : eta,
          cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) { *cosThetaT_ = 0.0f; return 1.0f; }
    float cosThetaI = fabsf(cosThetaI_);
    float cosThetaT = sqrtf(cosThetaTSqr);
    float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    *cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return 0.5f * (Rs * Rs + Rp * Rp);
}
static V3 s_safe_sqrt(V3 a) { return v3(safe_sqrt(a.x), safe_sqrt(a.y), safe_sqrt(a.z)); }
static V3 fresnel_conductor_exact(float cosThetaI, V3 eta, V3 k) { /* util.cpp:739-761 */
    float cosThetaI2 = cosThetaI * cosThetaI, sinThetaI2 = 1 - cosThetaI2, sinThetaI4 = sinThetaI2 * sinThetaI2;
    V3 temp1 = vsub(vsub(vmulv(eta, eta), vmulv(k, k)), v3(sinThetaI2, sinThetaI2, sinThetaI2));
    V3 a2pb2 = s_safe_sqrt(vadd(vmulv(temp1, temp1), vmul(vmulv(vmulv(vmulv(k, k), eta), eta), 4)));
    V3 a = s_safe_sqrt(vmul(vadd(a2pb2, temp1), 0.5f));
    V3 term1 = vadd(a2pb2, v3(cosThetaI2, cosThetaI2, cosThetaI2));
    V3 term2 = vmul(a, 2 * cosThetaI);
    V3 Rs2 = vdivv(vsub(term1, term2), vadd(term1, term2));
    V3 term3 = vadd(vmul(a2pb2, cosThetaI2), v3(sinThetaI4, sinThetaI4, sinThetaI4));
    V3 term4 = vmul(term2, sinThetaI2);
    V3 Rp2 = vdivv(vmulv(Rs2, vsub(term3, term4)), vadd(term3, term4));
    return vmul(vadd(Rp2, Rs2), 0.5f);
}
static inline V3 reflect_v(V3 wi, V3 n) { return vsub(vmul(n, 2 * vdot(wi, n)), wi); } /* util.cpp:763-765 */
static inline V3 refract_v(V3 wi, V3 n, float eta, float cosThetaT) { /* util.cpp:767-771 */
    if (cosThetaT < 0) eta = 1 / eta;
    return vsub(vmul(n, vdot(wi, n) * eta + cosThetaT), vmul(wi, eta));
}

/* ------------------------------------------------------------------------ */
/* BSDFs (bsdfs/diffuse.cpp, roughconductor.cpp, roughdielectric.cpp)        */
/* ------------------------------------------------------------------------ */
enum { /* BSDF::EBSDFType (include/mitsuba/render/bsdf.h) */
    E_NULL = 0x00001, E_DIFF_REFL = 0x00002, E_DIFF_TRANS = 0x00004, E_GLOSSY_REFL = 0x00008,
    E_GLOSSY_TRANS = 0x00010, E_DELTA_REFL = 0x00020, E_DELTA_TRANS = 0x00040,
    E_FRONT = 0x01000, E_BACK = 0x02000
};
#define E_SMOOTH (E_DIFF_REFL | E_DIFF_TRANS | E_GLOSSY_REFL | E_GLOSSY_TRANS)
#define E_TRANSMISSION (E_DIFF_TRANS | E_GLOSSY_TRANS | E_DELTA_TRANS | E_NULL)
#define E_DELTA (E_NULL | E_DELTA_REFL | E_DELTA_TRANS)

/* Texture2D + checkerboard (librender/texture.cpp:81-121, textures/checkerboard.cpp) */
typedef struct { int type; V3 c0, c1; float uoff, voff, us, vs; } Tex;

/* RoughTransmittance (bsdfs/rtrans.h:46-448) */
typedef struct {
    size_t eta, alpha, theta;
    float etaMin, etaMax, alphaMin, alphaMax;
    int etaFixed, alphaFixed;
    float *trans, *diff;
} RTab;

typedef struct {
    int type, distr, sampleVisible, flags;
    float alpha; /* texture average, isotropic */
    float alphaU, alphaV;
    V3 refl, specR, specT, eta3, k3;
    float eta, invEta;
    /* roughplastic (roughplastic.cpp:197-300); refl = diffuseReflectance */
    float specWeight, invEta2;
    int nonlinear;
    RTab ext, in;
    Tex reflTex, alphaTex;
    /* plastic (plastic.cpp:186-216) */
    float fdrInt, fdrExt;
    /* twosided (twosided.cpp:63-103): m_nestedBRDF[2] */
    const void *nested[2];
} Bsdf;

/* (int) of a float the way x86-64 cvttss2si converts it: out of range / NaN -> INT_MIN */
static inline int x86_f2i(float f) { return (f > -2147483648.0f && f < 2147483648.0f) ? (int)f : INT_MIN; }
static inline int imodulo(int a, int b) { int r = a % b; return (r < 0) ? r + b : r; } /* math.h:42 */

static V3 tex_eval(const Tex *t, float u, float v) { /* Texture2D::eval + Checkerboard::eval */
    float uu = u * t->us + t->uoff, vv = v * t->vs + t->voff;
    int x = 2 * imodulo(x86_f2i(uu * 2), 2) - 1, y = 2 * imodulo(x86_f2i(vv * 2), 2) - 1;
    return (x * y == 1) ? t->c0 : t->c1;
}

/* spline.cpp:23-60 */
static float o_cubic1d(float x, const float *values, size_t size, float min, float max) {
    if (!(x >= min && x <= max)) return 0.0f;
    float t = ((x - min) * (float)(size - 1)) / (max - min);
    size_t k = (size_t)t;
    if (k > size - 2) k = size - 2;
    float f0 = values[k], f1 = values[k + 1], d0, d1;
    if (k > 0) d0 = 0.5f * (values[k + 1] - values[k - 1]);
    else d0 = values[k + 1] - values[k];
    if (k + 2 < size) d1 = 0.5f * (values[k + 2] - values[k]);
    else d1 = values[k + 1] - values[k];
    t = t - (float)k;
    float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}
/* per-dimension knot weights of evalCubicInterp2D/3D (spline.cpp:241-283) */
static int o_cubic_w(float p, size_t size, size_t *knot, float w[4]) {
    if (!(p >= 0.0f && p <= 1.0f)) return 0;
    float t = ((p - 0.0f) * (float)(size - 1)) / (1.0f - 0.0f);
    size_t k = (size_t)t;
    if (k > size - 2) k = size - 2;
    *knot = k;
    t = t - (float)k;
    float t2 = t * t, t3 = t2 * t;
    w[0] = 0.0f; w[1] = 2 * t3 - 3 * t2 + 1; w[2] = -2 * t3 + 3 * t2; w[3] = 0.0f;
    float d0 = t3 - 2 * t2 + t, d1 = t3 - t2;
    if (k > 0) { w[2] += 0.5f * d0; w[0] -= 0.5f * d0; } else { w[2] += d0; w[1] -= d0; }
    if (k + 2 < size) { w[3] += 0.5f * d1; w[1] -= 0.5f * d1; } else { w[2] += d1; w[1] -= d1; }
    return 1;
}
static float o_cubic2d(float px, float py, const float *values, size_t sx, size_t sy) { /* spline.cpp:236-304 */
    size_t kx, ky; float wx[4], wy[4];
    if (!o_cubic_w(px, sx, &kx, wx) || !o_cubic_w(py, sy, &ky, wy)) return 0.0f;
    float result = 0.0f;
    for (int y = -1; y <= 2; ++y) {
        float w = wy[y + 1];
        for (int x = -1; x <= 2; ++x) {
            float wxy = wx[x + 1] * w;
            if (wxy == 0) continue;
            result += values[(ky + y) * sx + kx + x] * wxy;
        }
    }
    return result;
}
static float o_cubic3d(float px, float py, float pz, const float *values, size_t sx, size_t sy, size_t sz) {
    size_t kx, ky, kz; float wx[4], wy[4], wz[4]; /* spline.cpp:379-451 */
    if (!o_cubic_w(px, sx, &kx, wx) || !o_cubic_w(py, sy, &ky, wy) || !o_cubic_w(pz, sz, &kz, wz)) return 0.0f;
    float result = 0.0f;
    for (int z = -1; z <= 2; ++z) {
        float w = wz[z + 1];
        for (int y = -1; y <= 2; ++y) {
            float wyz = wy[y + 1] * w;
            for (int x = -1; x <= 2; ++x) {
                float wxyz = wx[x + 1] * wyz;
                if (wxyz == 0) continue;
                result += values[((kz + z) * sy + (ky + y)) * sx + kx + x] * wxyz;
            }
        }
    }
    return result;
}

static void rtab_free(RTab *t) { free(t->trans); free(t->diff); t->trans = t->diff = NULL; }

static int rtab_load(const void *data, size_t bytes, RTab *t) { /* rtrans.h:46-150 */
    const size_t hl = 17, fixed = hl + 24 + 16;
    const unsigned char *p = (const unsigned char *)data;
    memset(t, 0, sizeof *t);
    if (!data || bytes < fixed || memcmp(p, "MTS_TRANSMITTANCE", hl) != 0) return MTSGPU_EINVAL;
    uint64_t sz[3]; float r[4];
    memcpy(sz, p + hl, 24); memcpy(r, p + hl + 24, 16);
    t->eta = (size_t)sz[0]; t->alpha = (size_t)sz[1]; t->theta = (size_t)sz[2];
    t->etaMin = r[0]; t->etaMax = r[1]; t->alphaMin = r[2]; t->alphaMax = r[3];
    if (t->eta < 2 || t->alpha < 2 || t->theta < 2 || t->eta > 4096 || t->alpha > 4096 || t->theta > 4096)
        return MTSGPU_EINVAL;
    size_t ts = 2 * t->eta * t->alpha * t->theta, ds = 2 * t->eta * t->alpha;
    if (bytes != fixed + (ts + ds) * 4) return MTSGPU_EINVAL;
    t->trans = (float *)malloc(ts * 4); t->diff = (float *)malloc(ds * 4);
    const unsigned char *f = p + fixed;
    size_t a = 0, b = 0;
    for (size_t i = 0; i < 2 * t->eta; ++i)
        for (size_t j = 0; j < t->alpha; ++j) {
            for (size_t k = 0; k < t->theta; ++k) { memcpy(&t->trans[a++], f, 4); f += 4; }
            memcpy(&t->diff[b++], f, 4); f += 4;
        }
    return MTSGPU_OK;
}
static void rtab_clone(const RTab *s, RTab *d) {
    *d = *s;
    size_t ts = 2 * s->eta * s->alpha * s->theta, ds = 2 * s->eta * s->alpha;
    d->trans = (float *)malloc(ts * 4); memcpy(d->trans, s->trans, ts * 4);
    d->diff = (float *)malloc(ds * 4); memcpy(d->diff, s->diff, ds * 4);
}
/* setEta / setAlpha (rtrans.h:262-360): configure-time, glibc powf as the reference */
static void rtab_set_eta(RTab *t, float eta) {
    if (t->etaFixed) return;
    const float *trans = t->trans, *diffTrans = t->diff;
    if (eta < 1) { trans += t->eta * t->alpha * t->theta; diffTrans += t->eta * t->alpha; eta = 1.0f / eta; }
    if (eta < t->etaMin) eta = t->etaMin;
    float warpedEta = powf((eta - t->etaMin) / (t->etaMax - t->etaMin), 0.25f);
    float *nt = (float *)malloc(t->alpha * t->theta * 4), *nd = (float *)malloc(t->alpha * 4);
    float dAlpha = 1.0f / (t->alpha - 1), dTheta = 1.0f / (t->theta - 1);
    for (size_t i = 0; i < t->alpha; ++i) {
        for (size_t j = 0; j < t->theta; ++j)
            nt[i * t->theta + j] = o_cubic3d(j * dTheta, i * dAlpha, warpedEta, trans, t->theta, t->alpha, t->eta);
        nd[i] = o_cubic2d(i * dAlpha, warpedEta, diffTrans, t->alpha, t->eta);
    }
    free(t->trans); free(t->diff);
    t->trans = nt; t->diff = nd; t->etaFixed = 1;
}
static void rtab_set_alpha(RTab *t, float alpha) {
    if (t->alphaFixed) return;
    float warpedAlpha = powf((alpha - t->alphaMin) / (t->alphaMax - t->alphaMin), 0.25f);
    float *nt = (float *)malloc(t->theta * 4), *nd = (float *)malloc(4);
    float dTheta = 1.0f / (t->theta - 1);
    for (size_t i = 0; i < t->theta; ++i) nt[i] = o_cubic2d(i * dTheta, warpedAlpha, t->trans, t->theta, t->alpha);
    nd[0] = o_cubic1d(warpedAlpha, t->diff, t->alpha, 0.0f, 1.0f);
    free(t->trans); free(t->diff);
    t->trans = nt; t->diff = nd; t->alphaFixed = 1;
}
/* eval / evalDiffuse on an eta-reduced table (rtrans.h:179-247); render-time pow */
static float rtab_eval(const RTab *t, float cosTheta, float alpha) {
    float warpedCosTheta = o_pow(fabsf(cosTheta), 0.25f), result;
    if (!(cosTheta >= 0)) return 0.f;
    if (t->alphaFixed) {
        result = o_cubic1d(warpedCosTheta, t->trans, t->theta, 0.0f, 1.0f);
    } else {
        float warpedAlpha = o_pow((alpha - t->alphaMin) / (t->alphaMax - t->alphaMin), 0.25f);
        result = o_cubic2d(warpedCosTheta, warpedAlpha, t->trans, t->theta, t->alpha);
    }
    return smin(1.0f, smax(0.0f, result));
}
static float rtab_eval_diffuse(const RTab *t, float alpha) {
    float result;
    if (t->alphaFixed) {
        result = t->diff[0];
    } else {
        float warpedAlpha = o_pow((alpha - t->alphaMin) / (t->alphaMax - t->alphaMin), 0.25f);
        result = o_cubic1d(warpedAlpha, t->diff, t->alpha, 0.0f, 1.0f);
    }
    return smin(1.0f, smax(0.0f, result));
}

static float tex_scale_for_energy(V3 v, int ensure) { /* bsdf.cpp:88-112 */
    if (!ensure) return 1.0f;
    float actualMax = smaxc(v);
    if (actualMax > 1.0f) return 0.99f * (1.0f / actualMax);
    return 1.0f;
}

static V3 d3(const float *f) { return v3(f[0], f[1], f[2]); }
/* getMaximum / getMinimum / getAverage of a constant or checkerboard texture */
static V3 tdesc_max(const mtsgpu_texture_desc *t, V3 c) {
    return t->type ? v3(smax(t->color0[0], t->color1[0]), smax(t->color0[1], t->color1[1]), smax(t->color0[2], t->color1[2])) : c;
}
static V3 tdesc_min(const mtsgpu_texture_desc *t, V3 c) {
    return t->type ? v3(smin(t->color0[0], t->color1[0]), smin(t->color0[1], t->color1[1]), smin(t->color0[2], t->color1[2])) : c;
}
static V3 tdesc_avg(const mtsgpu_texture_desc *t, V3 c) {
    return t->type ? vmul(vadd(d3(t->color0), d3(t->color1)), 0.5f) : c;
}
static float luminance3(V3 s) { return s.x * 0.212671f + s.y * 0.715160f + s.z * 0.072169f; } /* spectrum.h:725 */
/* the texture as configured, ScaleTexture (scale.cpp:85-87) folded into its colours */
static int tex_configure(const mtsgpu_texture_desc *t, float scale, Tex *o) {
    memset(o, 0, sizeof *o);
    if (t->type == MTSGPU_TEX_NONE) return MTSGPU_OK;
    if (t->type != MTSGPU_TEX_CHECKERBOARD) return MTSGPU_EINVAL;
    o->type = t->type;
    o->c0 = d3(t->color0); o->c1 = d3(t->color1);
    if (scale != 1.0f) { o->c0 = vmul(o->c0, scale); o->c1 = vmul(o->c1, scale); }
    o->uoff = t->uoffset; o->voff = t->voffset; o->us = t->uscale; o->vs = t->vscale;
    return MTSGPU_OK;
}

static void bsdf_free(Bsdf *b) { rtab_free(&b->ext); rtab_free(&b->in); }

/* RoughPlastic ctor + configure (roughplastic.cpp:197-300) */
static int roughplastic_configure(const mtsgpu_bsdf_desc *d, Bsdf *b) {
    if (d->int_ior < 0 || d->ext_ior < 0 || d->int_ior == d->ext_ior) return MTSGPU_EINVAL;
    b->eta = d->int_ior / d->ext_ior;
    b->nonlinear = d->nonlinear != 0;
    if (d->distribution < 0 || d->distribution > 2) return MTSGPU_EINVAL;
    b->distr = d->distribution;
    b->sampleVisible = d->distribution == MTSGPU_DISTR_PHONG ? 0 : d->sample_visible;
    float au = smax(d->alpha_u, 1e-4f), av = smax(d->alpha_v, 1e-4f);
    if (d->alpha_tex.type == MTSGPU_TEX_NONE && au != av) return MTSGPU_EINVAL; /* anisotropic */
    b->alphaU = b->alphaV = savg(v3(au, au, au));
    V3 dr = d3(d->diffuse_reflectance), sr = d3(d->specular_reflectance);
    float sd = tex_scale_for_energy(tdesc_max(&d->reflectance_tex, dr), d->ensure_energy_conservation);
    float ss = tex_scale_for_energy(sr, d->ensure_energy_conservation);
    b->refl = sd != 1.0f ? vmul(dr, sd) : dr;
    b->specR = ss != 1.0f ? vmul(sr, ss) : sr;
    int rc;
    if ((rc = tex_configure(&d->reflectance_tex, sd, &b->reflTex))) return rc;
    if ((rc = tex_configure(&d->alpha_tex, 1.0f, &b->alphaTex))) return rc;
    V3 davg = tdesc_avg(&d->reflectance_tex, dr);
    if (sd != 1.0f) davg = vmul(davg, sd);
    float dAvg = luminance3(davg), sAvg = luminance3(b->specR);
    b->specWeight = sAvg / (dAvg + sAvg);
    b->invEta2 = 1.0f / (b->eta * b->eta);
    b->flags = E_GLOSSY_REFL | E_DIFF_REFL | E_FRONT;
    if ((rc = rtab_load(d->rtrans_data, (size_t)d->rtrans_bytes, &b->ext))) return rc;
    /* checkEta / checkAlpha (rtrans.h:371-388) */
    float e = b->eta < 1 ? 1 / b->eta : b->eta;
    V3 a3 = v3(au, au, au);
    float amin = savg(tdesc_min(&d->alpha_tex, a3)), amax = savg(tdesc_max(&d->alpha_tex, a3));
    if (e < b->ext.etaMin || e > b->ext.etaMax || amin < b->ext.alphaMin || amin > b->ext.alphaMax ||
        amax < b->ext.alphaMin || amax > b->ext.alphaMax) { bsdf_free(b); return MTSGPU_EINVAL; }
    rtab_clone(&b->ext, &b->in);
    rtab_set_eta(&b->ext, b->eta);
    rtab_set_eta(&b->in, 1 / b->eta);
    if (d->alpha_tex.type == MTSGPU_TEX_NONE) rtab_set_alpha(&b->ext, b->alphaU);
    return MTSGPU_OK;
}

/* fresnelDielectricExt(cosThetaI, eta) (util.cpp:680-683) */
static float fresnel_dielectric_ext2(float cosThetaI, float eta) {
    float ct;
    return fresnel_dielectric_ext(cosThetaI, &ct, eta);
}

/* GaussLobattoIntegrator(1024, 0, 1e-5f, useConvergenceEstimate = true)
 * (quad.cpp:287-409) on fresnelDiffuseIntegrand (util.cpp:808-811), i.e.
 * fresnelDiffuseReflectance(eta, false) (util.cpp:814-860).  The six
 * recursive steps are summed left to right. */
typedef struct { float eta; size_t evals; } GLQuad;
static float gl_alpha(void) { return (float)sqrt(2.0 / 3.0); }
static float gl_beta(void) { return (float)(1.0 / sqrt(5.0)); }
static float gl_f(const GLQuad *q, float xi) { return fresnel_dielectric_ext2(sqrtf(xi), q->eta); }
static float gl_abs_tolerance(GLQuad *q, float a, float b) {
    const float al = gl_alpha(), be = gl_beta();
    const float x1 = (float)0.94288241569547971906, x2 = (float)0.64185334234578130578, x3 = (float)0.23638319966214988028;
    const float m = (a + b) / 2, h = (b - a) / 2;
    const float y1 = gl_f(q, a), y3 = gl_f(q, m - al * h), y5 = gl_f(q, m - be * h), y7 = gl_f(q, m);
    const float y9 = gl_f(q, m + be * h), y11 = gl_f(q, m + al * h), y13 = gl_f(q, b);
    const float acc = h * ((float)0.0158271919734801831 * (y1 + y13)
                         + (float)0.0942738402188500455 * (gl_f(q, m - x1 * h) + gl_f(q, m + x1 * h))
                         + (float)0.1550719873365853963 * (y3 + y11)
                         + (float)0.1888215739601824544 * (gl_f(q, m - x2 * h) + gl_f(q, m + x2 * h))
                         + (float)0.1997734052268585268 * (y5 + y9)
                         + (float)0.2249264653333395270 * (gl_f(q, m - x3 * h) + gl_f(q, m + x3 * h))
                         + (float)0.2426110719014077338 * y7);
    q->evals += 13;
    float r = 1.0f;
    const float integral2 = (h / 6) * (y1 + y13 + 5 * (y5 + y9));
    const float integral1 = (h / 1470) * (77 * (y1 + y13) + 432 * (y3 + y11) + 625 * (y5 + y9) + 672 * y7);
    if (fabsf(integral2 - acc) != 0.0f) r = fabsf(integral1 - acc) / fabsf(integral2 - acc);
    if (r == 0.0f || r > 1.0f) r = 1.0f;
    float result = INFINITY;
    if (acc != 0) result = acc * smax(1e-5f, FLT_EPSILON) / (r * FLT_EPSILON);
    return result;
}
static float gl_step(GLQuad *q, float a, float b, float fa, float fb, float acc) {
    const float al = gl_alpha(), be = gl_beta();
    const float h = (b - a) / 2, m = (a + b) / 2;
    const float mll = m - al * h, ml = m - be * h, mr = m + be * h, mrr = m + al * h;
    const float fmll = gl_f(q, mll), fml = gl_f(q, ml), fm = gl_f(q, m), fmr = gl_f(q, mr), fmrr = gl_f(q, mrr);
    const float integral2 = (h / 6) * (fa + fb + 5 * (fml + fmr));
    const float integral1 = (h / 1470) * (77 * (fa + fb) + 432 * (fmll + fmrr) + 625 * (fml + fmr) + 672 * fm);
    q->evals += 5;
    if (q->evals >= 1024) return integral1;
    const float dist = acc + (integral1 - integral2);
    if (dist == acc || mll <= a || b <= mrr) return integral1;
    float r = gl_step(q, a, mll, fa, fmll, acc);
    r = r + gl_step(q, mll, ml, fmll, fml, acc);
    r = r + gl_step(q, ml, m, fml, fm, acc);
    r = r + gl_step(q, m, mr, fm, fmr, acc);
    r = r + gl_step(q, mr, mrr, fmr, fmrr, acc);
    r = r + gl_step(q, mrr, b, fmrr, fb, acc);
    return r;
}
float oracle_fresnel_diffuse_reflectance(float eta) {
    GLQuad q = {eta, 0};
    const float tol = gl_abs_tolerance(&q, 0.0f, 1.0f);
    q.evals += 2;
    return gl_step(&q, 0.0f, 1.0f, gl_f(&q, 0.0f), gl_f(&q, 1.0f), tol);
}

/* SmoothConductor / SmoothDielectric / SmoothPlastic ctor + configure
 * (conductor.cpp:164-212, dielectric.cpp:146-201, plastic.cpp:144-216) */
static int smooth_configure(const mtsgpu_bsdf_desc *d, Bsdf *b) {
    V3 sr = d3(d->specular_reflectance);
    float ss = tex_scale_for_energy(sr, d->ensure_energy_conservation);
    b->specR = ss != 1.0f ? vmul(sr, ss) : sr;
    if (d->type == MTSGPU_BSDF_CONDUCTOR) {
        float r = 1.0f / d->ext_eta;
        b->eta3 = vmul(d3(d->eta), r);
        b->k3 = vmul(d3(d->k), r);
        b->flags = E_DELTA_REFL | E_FRONT;
        return MTSGPU_OK;
    }
    if (d->int_ior < 0 || d->ext_ior < 0) return MTSGPU_EINVAL;
    b->eta = d->int_ior / d->ext_ior;
    if (d->type == MTSGPU_BSDF_DIELECTRIC) {
        b->invEta = 1 / b->eta;
        V3 st = d3(d->specular_transmittance);
        float sct = tex_scale_for_energy(st, d->ensure_energy_conservation);
        b->specT = sct != 1.0f ? vmul(st, sct) : st;
        b->flags = E_DELTA_REFL | E_DELTA_TRANS | E_FRONT | E_BACK;
        return MTSGPU_OK;
    }
    b->nonlinear = d->nonlinear != 0;
    V3 dr = d3(d->diffuse_reflectance);
    float sd = tex_scale_for_energy(tdesc_max(&d->reflectance_tex, dr), d->ensure_energy_conservation);
    b->refl = sd != 1.0f ? vmul(dr, sd) : dr;
    int rc;
    if ((rc = tex_configure(&d->reflectance_tex, sd, &b->reflTex))) return rc;
    b->fdrInt = oracle_fresnel_diffuse_reflectance(1 / b->eta);
    b->fdrExt = oracle_fresnel_diffuse_reflectance(b->eta);
    V3 davg = tdesc_avg(&d->reflectance_tex, dr);
    if (sd != 1.0f) davg = vmul(davg, sd);
    float dAvg = luminance3(davg), sAvg = luminance3(b->specR);
    b->specWeight = sAvg / (dAvg + sAvg);
    b->invEta2 = 1 / (b->eta * b->eta);
    b->flags = E_DELTA_REFL | E_DIFF_REFL | E_FRONT;
    return MTSGPU_OK;
}

/* TwoSidedBRDF::configure (twosided.cpp:82-103); `all` = the scene's BSDFs */
static int twosided_configure(const mtsgpu_bsdf_desc *d, Bsdf *b, const Bsdf *all, uint32_t n) {
    if (d->nested[0] < 0 || d->nested[0] >= (int)n) return MTSGPU_EINVAL;
    int n1 = d->nested[1] < 0 ? d->nested[0] : d->nested[1];
    if (n1 >= (int)n) return MTSGPU_EINVAL;
    b->nested[0] = &all[d->nested[0]];
    b->nested[1] = &all[n1];
    int flags = 0;
    for (int k = 0; k < 2; ++k) {
        const Bsdf *c = (const Bsdf *)b->nested[k];
        if (c->type == MTSGPU_BSDF_TWOSIDED) return MTSGPU_EINVAL;
        int lobes = c->flags & ~(E_FRONT | E_BACK);
        if (lobes) flags |= lobes | (k == 0 ? E_FRONT : E_BACK);
    }
    if (flags & E_TRANSMISSION) return MTSGPU_EINVAL;
    b->flags = flags;
    return MTSGPU_OK;
}

static int bsdf_configure(const mtsgpu_bsdf_desc *d, Bsdf *b) {
    memset(b, 0, sizeof *b);
    b->type = d->type;
    if (d->type == MTSGPU_BSDF_TWOSIDED) return MTSGPU_OK; /* twosided_configure, once all are built */
    if (d->type == MTSGPU_BSDF_CONDUCTOR || d->type == MTSGPU_BSDF_DIELECTRIC || d->type == MTSGPU_BSDF_PLASTIC)
        return smooth_configure(d, b);
    if (d->type == MTSGPU_BSDF_DIFFUSE) {
        V3 r = d3(d->reflectance);
        float sc = tex_scale_for_energy(tdesc_max(&d->reflectance_tex, r), d->ensure_energy_conservation);
        if (sc != 1.0f) r = vmul(r, sc);
        b->refl = r;
        int rc = tex_configure(&d->reflectance_tex, sc, &b->reflTex);
        if (rc) return rc;
        V3 mx = b->reflTex.type ? v3(smax(b->reflTex.c0.x, b->reflTex.c1.x), smax(b->reflTex.c0.y, b->reflTex.c1.y),
                                     smax(b->reflTex.c0.z, b->reflTex.c1.z)) : r;
        b->flags = (smaxc(mx) > 0) ? (E_DIFF_REFL | E_FRONT) : 0; /* diffuse.cpp:93-101 */
        return MTSGPU_OK;
    }
    if (d->type == MTSGPU_BSDF_ROUGHPLASTIC) return roughplastic_configure(d, b);
    if (d->type != MTSGPU_BSDF_ROUGHCONDUCTOR && d->type != MTSGPU_BSDF_ROUGHDIELECTRIC) return MTSGPU_EINVAL;
    if (d->alpha_tex.type != MTSGPU_TEX_NONE) {
        int rc = tex_configure(&d->alpha_tex, 1.0f, &b->alphaTex);
        if (rc) return rc;
    }
    if (d->distribution < 0 || d->distribution > 2) return MTSGPU_EINVAL;
    b->distr = d->distribution;
    /* MicrofacetDistribution(props) (microfacet.h:105-150) */
    float au = smax(d->alpha_u, 1e-4f), av = smax(d->alpha_v, 1e-4f);
    b->sampleVisible = d->distribution == MTSGPU_DISTR_PHONG ? 0 : d->sample_visible;
    /* ConstantFloatTexture(alpha)->eval(its).average() (hw/basicshader.h:105) */
    b->alphaU = savg(v3(au, au, au));
    b->alphaV = savg(v3(av, av, av));
    V3 sr = v3(d->specular_reflectance[0], d->specular_reflectance[1], d->specular_reflectance[2]);
    float sc = tex_scale_for_energy(sr, d->ensure_energy_conservation);
    if (sc != 1.0f) sr = vmul(sr, sc);
    b->specR = sr;
    if (d->type == MTSGPU_BSDF_ROUGHCONDUCTOR) {
        /* roughconductor.cpp:168-199: m_eta = eta / extEta */
        float r = 1.0f / d->ext_eta;
        b->eta3 = vmul(v3(d->eta[0], d->eta[1], d->eta[2]), r);
        b->k3 = vmul(v3(d->k[0], d->k[1], d->k[2]), r);
        b->flags = E_GLOSSY_REFL | E_FRONT;
    } else {
        if (d->int_ior < 0 || d->ext_ior < 0 || d->int_ior == d->ext_ior) return MTSGPU_EINVAL;
        b->eta = d->int_ior / d->ext_ior; /* roughdielectric.cpp:198-199 */
        b->invEta = 1 / b->eta;
        V3 st = v3(d->specular_transmittance[0], d->specular_transmittance[1], d->specular_transmittance[2]);
        float sct = tex_scale_for_energy(st, d->ensure_energy_conservation);
        if (sct != 1.0f) st = vmul(st, sct);
        b->specT = st;
        b->flags = E_GLOSSY_REFL | E_GLOSSY_TRANS | E_FRONT | E_BACK;
    }
    return MTSGPU_OK;
}

typedef struct { V3 wi, wo; float eta; int sampledType; float u, v; /* its.uv */ } BRec;

static V3 bsdf_refl(const Bsdf *b, const BRec *r) { /* m_reflectance->eval(bRec.its) */
    return b->reflTex.type ? tex_eval(&b->reflTex, r->u, r->v) : b->refl;
}
/* MicrofacetDistribution at the hit: m_alpha->eval(its).average() for a texture */
static void bsdf_distr(const Bsdf *b, const BRec *r, Distr *d) {
    if (b->alphaTex.type) {
        float a = savg(tex_eval(&b->alphaTex, r->u, r->v));
        distr_init(d, b->distr, a, a, b->sampleVisible);
    } else {
        distr_init(d, b->distr, b->alphaU, b->alphaV, b->sampleVisible);
    }
}

static float rp_prob_specular(const Bsdf *b, float cosThetaI, float alpha) { /* roughplastic.cpp:371-378 */
    float probSpecular = 1 - rtab_eval(&b->ext, cosThetaI, alpha);
    probSpecular = (probSpecular * b->specWeight) /
                   (probSpecular * b->specWeight + (1 - probSpecular) * (1 - b->specWeight));
    return probSpecular;
}
static V3 rp_eval(const Bsdf *b, const BRec *r) { /* RoughPlastic::eval (roughplastic.cpp:300-345) */
    if (r->wi.z <= 0 || r->wo.z <= 0) return v3(0, 0, 0);
    Distr d; bsdf_distr(b, r, &d);
    V3 result = v3(0, 0, 0);
    V3 H = vnormalize(vadd(r->wo, r->wi));
    float D = distr_eval(&d, H);
    float ct;
    float F = fresnel_dielectric_ext(vdot(r->wi, H), &ct, b->eta);
    float G = distr_G(&d, r->wi, r->wo, H);
    float value = F * D * G / (4.0f * r->wi.z);
    result = vadd(result, vmul(b->specR, value));
    V3 diff = bsdf_refl(b, r);
    float T12 = rtab_eval(&b->ext, r->wi.z, d.alphaU);
    float T21 = rtab_eval(&b->ext, r->wo.z, d.alphaU);
    float Fdr = 1 - rtab_eval_diffuse(&b->in, d.alphaU);
    if (b->nonlinear) diff = vdivv(diff, vsub(v3(1.0f, 1.0f, 1.0f), vmul(diff, Fdr)));
    else diff = vdiv(diff, 1 - Fdr);
    return vadd(result, vmul(diff, INV_PI_F * r->wo.z * T12 * T21 * b->invEta2));
}
static float rp_pdf(const Bsdf *b, const BRec *r) { /* RoughPlastic::pdf (roughplastic.cpp:347-393) */
    if (r->wi.z <= 0 || r->wo.z <= 0) return 0.0f;
    Distr d; bsdf_distr(b, r, &d);
    V3 H = vnormalize(vadd(r->wo, r->wi));
    float probSpecular = rp_prob_specular(b, r->wi.z, d.alphaU), probDiffuse = 1 - probSpecular;
    float dwh_dwo = 1.0f / (4.0f * vdot(r->wo, H));
    float prob = distr_pdf(&d, r->wi, H);
    float result = prob * dwh_dwo * probSpecular;
    result += probDiffuse * cosine_hemisphere_pdf(r->wo);
    return result;
}

/* SmoothPlastic's diffuse term (plastic.cpp:270-280) */
static V3 sp_diffuse(const Bsdf *b, const BRec *r) {
    V3 diff = bsdf_refl(b, r);
    if (b->nonlinear) diff = vdivv(diff, vsub(v3(1.0f, 1.0f, 1.0f), vmul(diff, b->fdrInt)));
    else diff = vdiv(diff, 1 - b->fdrInt);
    return diff;
}
static float sp_prob_specular(const Bsdf *b, float Fi) { /* plastic.cpp:296-299 */
    return (Fi * b->specWeight) / (Fi * b->specWeight + (1 - Fi) * (1 - b->specWeight));
}

/* eval()/pdf() with measure = ESolidAngle, the only measure Li() queries
 * (path.cpp:185,195): delta lobes contribute nothing there
 * (conductor.cpp:216-245, dielectric.cpp:228-275, plastic.cpp:245-311) */
static V3 sm_eval(const Bsdf *b, const BRec *r) {
    if (b->type != MTSGPU_BSDF_PLASTIC) return v3(0, 0, 0);
    if (r->wo.z <= 0 || r->wi.z <= 0) return v3(0, 0, 0);
    float Fi = fresnel_dielectric_ext2(r->wi.z, b->eta);
    float Fo = fresnel_dielectric_ext2(r->wo.z, b->eta);
    V3 diff = sp_diffuse(b, r);
    return vmul(diff, cosine_hemisphere_pdf(r->wo) * b->invEta2 * (1 - Fi) * (1 - Fo));
}
static float sm_pdf(const Bsdf *b, const BRec *r) {
    if (b->type != MTSGPU_BSDF_PLASTIC) return 0.0f;
    if (r->wo.z <= 0 || r->wi.z <= 0) return 0.0f;
    float Fi = fresnel_dielectric_ext2(r->wi.z, b->eta);
    float probSpecular = sp_prob_specular(b, Fi);
    return cosine_hemisphere_pdf(r->wo) * (1 - probSpecular);
}
/* sample(bRec, pdf, sample) (conductor.cpp:269-283, dielectric.cpp:277-333, plastic.cpp:356-420) */
static V3 sm_sample(const Bsdf *b, BRec *r, float *pdf, float sx, float sy) {
    V3 zero = v3(0, 0, 0);
    if (b->type == MTSGPU_BSDF_CONDUCTOR) {
        if (r->wi.z <= 0) return zero;
        r->sampledType = E_DELTA_REFL;
        r->wo = v3(-r->wi.x, -r->wi.y, r->wi.z);
        r->eta = 1.0f;
        *pdf = 1;
        return vmulv(b->specR, fresnel_conductor_exact(r->wi.z, b->eta3, b->k3));
    }
    if (b->type == MTSGPU_BSDF_DIELECTRIC) {
        float cosThetaT;
        float F = fresnel_dielectric_ext(r->wi.z, &cosThetaT, b->eta);
        if (sx <= F) {
            r->sampledType = E_DELTA_REFL;
            r->wo = v3(-r->wi.x, -r->wi.y, r->wi.z);
            r->eta = 1.0f;
            *pdf = F;
            return b->specR;
        }
        float scale = -(cosThetaT < 0 ? b->invEta : b->eta);
        r->sampledType = E_DELTA_TRANS;
        r->wo = v3(scale * r->wi.x, scale * r->wi.y, cosThetaT);
        r->eta = cosThetaT < 0 ? b->eta : b->invEta;
        *pdf = 1 - F;
        float factor = cosThetaT < 0 ? b->invEta : b->eta; /* mode == ERadiance */
        return vmul(b->specT, factor * factor);
    }
    /* plastic */
    if (r->wi.z <= 0) return zero;
    float Fi = fresnel_dielectric_ext2(r->wi.z, b->eta);
    r->eta = 1.0f;
    float probSpecular = sp_prob_specular(b, Fi);
    if (sx < probSpecular) {
        r->sampledType = E_DELTA_REFL;
        r->wo = v3(-r->wi.x, -r->wi.y, r->wi.z);
        *pdf = probSpecular;
        return vdiv(vmul(b->specR, Fi), probSpecular);
    }
    r->sampledType = E_DIFF_REFL;
    r->wo = square_to_cosine_hemisphere((sx - probSpecular) / (1 - probSpecular), sy);
    float Fo = fresnel_dielectric_ext2(r->wo.z, b->eta);
    V3 diff = sp_diffuse(b, r);
    *pdf = (1 - probSpecular) * cosine_hemisphere_pdf(r->wo);
    return vmul(diff, b->invEta2 * (1 - Fi) * (1 - Fo) / (1 - probSpecular));
}

static V3 bsdf_eval(const Bsdf *b, const BRec *r) {
    V3 zero = v3(0, 0, 0);
    if (b->type == MTSGPU_BSDF_TWOSIDED) { /* twosided.cpp:105-117 */
        BRec q = *r;
        if (q.wi.z > 0) return bsdf_eval((const Bsdf *)b->nested[0], &q);
        q.wi.z *= -1;
        q.wo.z *= -1;
        return bsdf_eval((const Bsdf *)b->nested[1], &q);
    }
    if (b->type >= MTSGPU_BSDF_CONDUCTOR) return sm_eval(b, r);
    if (b->type == MTSGPU_BSDF_DIFFUSE) { /* diffuse.cpp:110-117 */
        /* bRec.typeMask = EAll, so only the cosine tests can reject */
        if (r->wi.z <= 0 || r->wo.z <= 0) return zero;
        return vmul(bsdf_refl(b, r), INV_PI_F * r->wo.z);
    }
    if (b->type == MTSGPU_BSDF_ROUGHPLASTIC) return rp_eval(b, r);
    Distr d;
    if (b->type == MTSGPU_BSDF_ROUGHCONDUCTOR) { /* roughconductor.cpp:257-292 */
        if (r->wi.z <= 0 || r->wo.z <= 0) return zero;
        V3 H = vnormalize(vadd(r->wo, r->wi));
        bsdf_distr(b, r, &d);
        float D = distr_eval(&d, H);
        if (D == 0) return zero;
        V3 F = vmulv(fresnel_conductor_exact(vdot(r->wi, H), b->eta3, b->k3), b->specR);
        float G = distr_G(&d, r->wi, r->wo, H);
        float model = D * G / (4.0f * r->wi.z);
        return vmul(F, model);
    }
    /* roughdielectric.cpp:270-346 */
    if (r->wi.z == 0) return zero;
    int reflect = r->wi.z * r->wo.z > 0;
    V3 H;
    if (reflect) {
        H = vnormalize(vadd(r->wo, r->wi));
    } else {
        float eta = r->wi.z > 0 ? b->eta : b->invEta;
        H = vnormalize(vadd(r->wi, vmul(r->wo, eta)));
    }
    H = vmul(H, signumf(H.z));
    bsdf_distr(b, r, &d);
    float D = distr_eval(&d, H);
    if (D == 0) return zero;
    float ct;
    float F = fresnel_dielectric_ext(vdot(r->wi, H), &ct, b->eta);
    float G = distr_G(&d, r->wi, r->wo, H);
    if (reflect) {
        float value = F * D * G / (4.0f * fabsf(r->wi.z));
        return vmul(b->specR, value);
    }
    float eta = r->wi.z > 0.0f ? b->eta : b->invEta;
    float sqrtDenom = vdot(r->wi, H) + eta * vdot(r->wo, H);
    float value = ((1 - F) * D * G * eta * eta * vdot(r->wi, H) * vdot(r->wo, H)) /
                  (r->wi.z * sqrtDenom * sqrtDenom);
    float factor = (r->wi.z > 0 ? b->invEta : b->eta); /* mode == ERadiance */
    return vmul(b->specT, fabsf(value * factor * factor));
}

static float bsdf_pdf(const Bsdf *b, const BRec *r) {
    if (b->type == MTSGPU_BSDF_TWOSIDED) { /* twosided.cpp:119-131 */
        BRec q = *r;
        if (q.wi.z > 0) return bsdf_pdf((const Bsdf *)b->nested[0], &q);
        q.wi.z *= -1;
        q.wo.z *= -1;
        return bsdf_pdf((const Bsdf *)b->nested[1], &q);
    }
    if (b->type >= MTSGPU_BSDF_CONDUCTOR) return sm_pdf(b, r);
    if (b->type == MTSGPU_BSDF_DIFFUSE) { /* diffuse.cpp:119-126 */
        if (r->wi.z <= 0 || r->wo.z <= 0) return 0.0f;
        return cosine_hemisphere_pdf(r->wo);
    }
    if (b->type == MTSGPU_BSDF_ROUGHPLASTIC) return rp_pdf(b, r);
    Distr d;
    if (b->type == MTSGPU_BSDF_ROUGHCONDUCTOR) { /* roughconductor.cpp:294-319 */
        if (r->wi.z <= 0 || r->wo.z <= 0) return 0.0f;
        V3 H = vnormalize(vadd(r->wo, r->wi));
        bsdf_distr(b, r, &d);
        if (b->sampleVisible)
            return distr_eval(&d, H) * distr_smithG1(&d, r->wi, H) / (4.0f * r->wi.z);
        return distr_pdf(&d, r->wi, H) / (4 * vabsdot(r->wo, H));
    }
    /* roughdielectric.cpp:348-405 */
    int reflect = r->wi.z * r->wo.z > 0;
    V3 H;
    float dwh_dwo;
    if (reflect) {
        H = vnormalize(vadd(r->wo, r->wi));
        dwh_dwo = 1.0f / (4.0f * vdot(r->wo, H));
    } else {
        float eta = r->wi.z > 0 ? b->eta : b->invEta;
        H = vnormalize(vadd(r->wi, vmul(r->wo, eta)));
        float sqrtDenom = vdot(r->wi, H) + eta * vdot(r->wo, H);
        dwh_dwo = (eta * eta * vdot(r->wo, H)) / (sqrtDenom * sqrtDenom);
    }
    H = vmul(H, signumf(H.z));
    bsdf_distr(b, r, &d);
    if (!b->sampleVisible) distr_scale_alpha(&d, 1.2f - 0.2f * sqrtf(fabsf(r->wi.z)));
    float prob = distr_pdf(&d, vmul(r->wi, signumf(r->wi.z)), H);
    float ct;
    float F = fresnel_dielectric_ext(vdot(r->wi, H), &ct, b->eta);
    prob *= reflect ? F : (1 - F);
    return fabsf(prob * dwh_dwo);
}

/* sample(bRec, pdf, sample) of each BSDF; consumes sampler->next1D() for the
 * roughdielectric lobe choice (roughdielectric.cpp:554) */
static V3 bsdf_sample(const Bsdf *b, BRec *r, float *pdf, float sx, float sy, Sampler *smp) {
    V3 zero = v3(0, 0, 0);
    if (b->type == MTSGPU_BSDF_TWOSIDED) { /* twosided.cpp:151-172 */
        int flipped = 0;
        if (r->wi.z < 0) { r->wi.z *= -1; flipped = 1; }
        V3 result = bsdf_sample((const Bsdf *)b->nested[flipped], r, pdf, sx, sy, smp);
        if (flipped) {
            r->wi.z *= -1;
            if (!vzero(result) && *pdf != 0) r->wo.z *= -1;
        }
        return result;
    }
    if (b->type >= MTSGPU_BSDF_CONDUCTOR) return sm_sample(b, r, pdf, sx, sy);
    if (b->type == MTSGPU_BSDF_DIFFUSE) { /* diffuse.cpp:139-150 */
        if (r->wi.z <= 0) return zero;
        r->wo = square_to_cosine_hemisphere(sx, sy);
        r->eta = 1.0f;
        r->sampledType = E_DIFF_REFL;
        *pdf = cosine_hemisphere_pdf(r->wo);
        return bsdf_refl(b, r);
    }
    if (b->type == MTSGPU_BSDF_ROUGHPLASTIC) { /* RoughPlastic::sample (roughplastic.cpp:395-458) */
        if (r->wi.z <= 0) return zero;
        int choseSpecular = 1;
        Distr dd; bsdf_distr(b, r, &dd);
        float probSpecular = rp_prob_specular(b, r->wi.z, dd.alphaU);
        if (sy < probSpecular) {
            sy /= probSpecular;
        } else {
            sy = (sy - probSpecular) / (1 - probSpecular);
            choseSpecular = 0;
        }
        if (choseSpecular) {
            float mpdf;
            V3 m = distr_sample(&dd, r->wi, sx, sy, &mpdf);
            r->wo = reflect_v(r->wi, m);
            r->sampledType = E_GLOSSY_REFL;
            if (r->wo.z <= 0) return zero;
        } else {
            r->sampledType = E_DIFF_REFL;
            r->wo = square_to_cosine_hemisphere(sx, sy);
        }
        r->eta = 1.0f;
        *pdf = rp_pdf(b, r);
        if (*pdf == 0) return zero;
        return vdiv(rp_eval(b, r), *pdf);
    }
    Distr d;
    if (b->type == MTSGPU_BSDF_ROUGHCONDUCTOR) { /* roughconductor.cpp:357-406 */
        if (r->wi.z < 0) return zero;
        bsdf_distr(b, r, &d);
        V3 m = distr_sample(&d, r->wi, sx, sy, pdf);
        if (*pdf == 0) return zero;
        r->wo = reflect_v(r->wi, m);
        r->eta = 1.0f;
        r->sampledType = E_GLOSSY_REFL;
        if (r->wo.z <= 0) return zero;
        V3 F = vmulv(fresnel_conductor_exact(vdot(r->wi, m), b->eta3, b->k3), b->specR);
        float weight;
        if (b->sampleVisible) weight = distr_smithG1(&d, r->wo, m);
        else weight = distr_eval(&d, m) * distr_G(&d, r->wi, r->wo, m) * vdot(r->wi, m) / (*pdf * r->wi.z);
        *pdf /= 4.0f * vdot(r->wo, m);
        return vmul(F, weight);
    }
    /* roughdielectric.cpp:525-615 */
    bsdf_distr(b, r, &d);
    Distr sd = d;
    if (!b->sampleVisible) distr_scale_alpha(&sd, 1.2f - 0.2f * sqrtf(fabsf(r->wi.z)));
    float microfacetPDF;
    V3 m = distr_sample(&sd, vmul(r->wi, signumf(r->wi.z)), sx, sy, &microfacetPDF);
    if (microfacetPDF == 0) return zero;
    *pdf = microfacetPDF;
    float cosThetaT;
    float F = fresnel_dielectric_ext(vdot(r->wi, m), &cosThetaT, b->eta);
    V3 weight = v3(1.0f, 1.0f, 1.0f);
    int sampleReflection = 1;
    if (next1d(smp) > F) { sampleReflection = 0; *pdf *= 1 - F; }
    else *pdf *= F;
    float dwh_dwo;
    if (sampleReflection) {
        r->wo = reflect_v(r->wi, m);
        r->eta = 1.0f;
        r->sampledType = E_GLOSSY_REFL;
        if (r->wi.z * r->wo.z <= 0) return zero;
        weight = vmulv(weight, b->specR);
        dwh_dwo = 1.0f / (4.0f * vdot(r->wo, m));
    } else {
        if (cosThetaT == 0) return zero;
        r->wo = refract_v(r->wi, m, b->eta, cosThetaT);
        r->eta = cosThetaT < 0 ? b->eta : b->invEta;
        r->sampledType = E_GLOSSY_TRANS;
        if (r->wi.z * r->wo.z >= 0) return zero;
        float factor = cosThetaT < 0 ? b->invEta : b->eta;
        weight = vmulv(weight, vmul(b->specT, factor * factor));
        float sqrtDenom = vdot(r->wi, m) + r->eta * vdot(r->wo, m);
        dwh_dwo = (r->eta * r->eta * vdot(r->wo, m)) / (sqrtDenom * sqrtDenom);
    }
    if (b->sampleVisible) weight = vmul(weight, distr_smithG1(&d, r->wo, m));
    else weight = vmul(weight, fabsf(distr_eval(&d, m) * distr_G(&d, r->wi, r->wo, m) * vdot(r->wi, m) / (microfacetPDF * r->wi.z)));
    *pdf *= fabsf(dwh_dwo);
    return weight;
}

/* ------------------------------------------------------------------------ */
/* TriAccel (render/triaccel.h:58-160)                                       */
/* ------------------------------------------------------------------------ */
typedef struct { uint32_t k; float n_u, n_v, n_d, a_u, a_v, b_nu, b_nv, c_nu, c_nv; } TriAccel;

static int triaccel_load(TriAccel *ta, V3 A, V3 B, V3 C) {
    static const int waldModulo[4] = {1, 2, 0, 1};
    V3 b = vsub(C, A), c = vsub(B, A), N = vcross(c, b);
    ta->k = 0;
    for (int j = 0; j < 3; j++)
        if (fabsf(vget(N, j)) > fabsf(vget(N, (int)ta->k))) ta->k = (uint32_t)j;
    uint32_t u = (uint32_t)waldModulo[ta->k], v = (uint32_t)waldModulo[ta->k + 1];
    const float n_k = vget(N, (int)ta->k), denom = vget(b, (int)u) * vget(c, (int)v) - vget(b, (int)v) * vget(c, (int)u);
    if (denom == 0) { ta->k = 3; return 1; }
    ta->n_u = vget(N, (int)u) / n_k;
    ta->n_v = vget(N, (int)v) / n_k;
    ta->n_d = vdot(A, N) / n_k;
    ta->b_nu = vget(b, (int)u) / denom;
    ta->b_nv = -vget(b, (int)v) / denom;
    ta->a_u = vget(A, (int)u);
    ta->a_v = vget(A, (int)v);
    ta->c_nu = vget(c, (int)v) / denom;
    ta->c_nv = -vget(c, (int)u) / denom;
    return 0;
}

static inline int triaccel_intersect(const TriAccel *ta, const Ray *ray, float mint, float maxt,
                                     float *u, float *v, float *t) {
    float o_u, o_v, o_k, d_u, d_v, d_k;
    switch (ta->k) {
        case 0: o_u = ray->o.y; o_v = ray->o.z; o_k = ray->o.x; d_u = ray->d.y; d_v = ray->d.z; d_k = ray->d.x; break;
        case 1: o_u = ray->o.z; o_v = ray->o.x; o_k = ray->o.y; d_u = ray->d.z; d_v = ray->d.x; d_k = ray->d.y; break;
        case 2: o_u = ray->o.x; o_v = ray->o.y; o_k = ray->o.z; d_u = ray->d.x; d_v = ray->d.y; d_k = ray->d.z; break;
        default: return 0;
    }
    *t = (ta->n_d - o_u * ta->n_u - o_v * ta->n_v - o_k) / (d_u * ta->n_u + d_v * ta->n_v + d_k);
    if (*t < mint || *t > maxt) return 0;
    const float hu = o_u + *t * d_u - ta->a_u;
    const float hv = o_v + *t * d_v - ta->a_v;
    *u = hv * ta->b_nu + hu * ta->b_nv;
    *v = hu * ta->c_nu + hv * ta->c_nv;
    return *u >= 0 && *v >= 0 && *u + *v <= 1.0f;
}

/* ------------------------------------------------------------------------ */
/* analytic shapes: rectangle.cpp, disk.cpp, sphere.cpp                      */
/* ------------------------------------------------------------------------ */
typedef struct {
    int type, flip;
    Xform o2w;            /* m_objectToWorld with its carried inverse (m_worldToObject) */
    V3 center, n, fs, ft, dpdu, dpdv;
    float radius, invArea;
    float bmin[3], bmax[3];  /* getAABB() */
} Ana;

static V3 xf_normal(const M4 *inv, V3 v) { /* Transform::operator()(Normal) (transform.h:203-211) */
    return v3(inv->m[0][0] * v.x + inv->m[1][0] * v.y + inv->m[2][0] * v.z,
              inv->m[0][1] * v.x + inv->m[1][1] * v.y + inv->m[2][1] * v.z,
              inv->m[0][2] * v.x + inv->m[1][2] * v.y + inv->m[2][2] * v.z);
}
static void ana_grow(Ana *a, V3 p) {
    for (int i = 0; i < 3; ++i) {
        float x = vget(p, i);
        if (x < a->bmin[i]) a->bmin[i] = x;
        if (x > a->bmax[i]) a->bmax[i] = x;
    }
}
static int desc_xform(const float *t16, const float *inv16, Xform *out) {
    memcpy(&out->t.m[0][0], t16, 16 * sizeof(float));
    int have = 0;
    for (int i = 0; i < 16; ++i) have |= inv16[i] != 0.0f;
    if (have) { memcpy(&out->inv.m[0][0], inv16, 16 * sizeof(float)); return MTSGPU_OK; }
    return m4_invert(&out->t, &out->inv) ? MTSGPU_OK : MTSGPU_EINVAL;
}

/* constructors + configure() + getAABB() (rectangle.cpp:80-119, disk.cpp:83-130, sphere.cpp:108-157) */
static int ana_configure(const mtsgpu_mesh_desc *md, Ana *a) {
    memset(a, 0, sizeof *a);
    a->type = md->shape_type;
    for (int i = 0; i < 3; ++i) { a->bmin[i] = FLT_MAX; a->bmax[i] = -FLT_MAX; }
    if (md->shape_type == MTSGPU_SHAPE_RECTANGLE || md->shape_type == MTSGPU_SHAPE_DISK) {
        if (desc_xform(md->to_world, md->to_world_inv, &a->o2w)) return MTSGPU_EINVAL;
        if (md->flip_normals) { Xform sc = xf_scale(1, 1, -1); a->o2w = xf_compose(&a->o2w, &sc); }
        const M4 *T = &a->o2w.t;
        if (md->shape_type == MTSGPU_SHAPE_RECTANGLE) {
            a->dpdu = xf_vector(T, v3(2, 0, 0));
            a->dpdv = xf_vector(T, v3(0, 2, 0));
            a->n = vnormalize(xf_normal(&a->o2w.inv, v3(0, 0, 1)));
            a->fs = vnormalize(a->dpdu);
            a->ft = vnormalize(a->dpdv);
            a->invArea = 1.0f / (vlen(a->dpdu) * vlen(a->dpdv));
            if (fabsf(vdot(vnormalize(a->dpdu), vnormalize(a->dpdv))) > EPSILON) return MTSGPU_EINVAL; /* shear */
            ana_grow(a, xf_point(T, v3(-1, -1, 0))); ana_grow(a, xf_point(T, v3(1, -1, 0)));
            ana_grow(a, xf_point(T, v3(1, 1, 0))); ana_grow(a, xf_point(T, v3(-1, 1, 0)));
        } else {
            V3 dpdu = xf_vector(T, v3(1, 0, 0)), dpdv = xf_vector(T, v3(0, 1, 0));
            if (fabsf(vdot(vnormalize(dpdu), vnormalize(dpdv))) > 1e-3f) return MTSGPU_EINVAL;
            if (fabsf(vlen(dpdu) / vlen(dpdv) - 1) > 1e-3f) return MTSGPU_EINVAL;
            a->invArea = 1.0f / (M_PI_F * vlen(dpdu) * vlen(dpdu));
            a->n = vnormalize(xf_normal(&a->o2w.inv, v3(0, 0, 1)));
            ana_grow(a, xf_point(T, v3(1, 0, 0))); ana_grow(a, xf_point(T, v3(-1, 0, 0)));
            ana_grow(a, xf_point(T, v3(0, 1, 0))); ana_grow(a, xf_point(T, v3(0, -1, 0)));
        }
        return MTSGPU_OK;
    }
    if (md->shape_type != MTSGPU_SHAPE_SPHERE) return MTSGPU_EINVAL;
    a->o2w = xf_translate(md->center[0], md->center[1], md->center[2]);
    float radius = md->radius;
    if (md->has_to_world) {
        Xform T;
        if (desc_xform(md->to_world, md->to_world_inv, &T)) return MTSGPU_EINVAL;
        float r = vlen(xf_vector(&T.t, v3(1, 0, 0)));
        float ir = 1 / r;
        Xform sc = xf_scale(ir, ir, ir);
        Xform ts = xf_compose(&T, &sc);
        a->o2w = xf_compose(&ts, &a->o2w);
        radius *= r;
    }
    a->flip = md->flip_normals != 0;
    a->center = xf_point(&a->o2w.t, v3(0, 0, 0));
    a->radius = radius;
    a->invArea = 1 / (4 * M_PI_F * radius * radius);
    if (radius <= 0) return MTSGPU_EINVAL;
    ana_grow(a, vsub(a->center, v3(radius, radius, radius)));
    ana_grow(a, vadd(a->center, v3(radius, radius, radius)));
    return MTSGPU_OK;
}

/* solveQuadraticDouble / solveQuadratic (util.cpp:447-525) */
static int solve_quadratic_d(double a, double b, double c, double *x0, double *x1) {
    if (a == 0) {
        if (b != 0) { *x0 = *x1 = -c / b; return 1; }
        return 0;
    }
    double discrim = b * b - 4.0f * a * c;
    if (discrim < 0) return 0;
    double temp, sqrtDiscrim = sqrt(discrim);
    if (b < 0) temp = -0.5f * (b - sqrtDiscrim);
    else temp = -0.5f * (b + sqrtDiscrim);
    *x0 = temp / a;
    *x1 = c / temp;
    if (*x0 > *x1) { double t = *x0; *x0 = *x1; *x1 = t; }
    return 1;
}
static int solve_quadratic_f(float a, float b, float c, float *x0, float *x1) {
    if (a == 0) {
        if (b != 0) { *x0 = *x1 = -c / b; return 1; }
        return 0;
    }
    float discrim = b * b - 4.0f * a * c;
    if (discrim < 0) return 0;
    float temp, sqrtDiscrim = sqrtf(discrim);
    if (b < 0) temp = -0.5f * (b - sqrtDiscrim);
    else temp = -0.5f * (b + sqrtDiscrim);
    *x0 = temp / a;
    *x1 = c / temp;
    if (*x0 > *x1) { float t = *x0; *x0 = *x1; *x1 = t; }
    return 1;
}

/* Shape::rayIntersect(ray, mint, maxt, t, temp) (rectangle.cpp:125-148, disk.cpp:139-162,
 * sphere.cpp:163-187); shadow = the (ray, mint, maxt) overload (sphere.cpp:189-207).
 * (*lx, *ly) = the object-space hit kept in `temp` by rectangle/disk */
static int ana_intersect(const Ana *a, const Ray *ray, float mint, float maxt, int shadow,
                         float *t, float *lx, float *ly) {
    if (a->type == MTSGPU_SHAPE_SPHERE) {
        double ox = (double)ray->o.x - (double)a->center.x, oy = (double)ray->o.y - (double)a->center.y,
               oz = (double)ray->o.z - (double)a->center.z;
        double dx = ray->d.x, dy = ray->d.y, dz = ray->d.z;
        double A = dx * dx + dy * dy + dz * dz;
        double B = 2 * (ox * dx + oy * dy + oz * dz);
        double C = (ox * ox + oy * oy + oz * oz) - a->radius * a->radius;
        double nearT, farT;
        if (!solve_quadratic_d(A, B, C, &nearT, &farT)) return 0;
        if (shadow) {
            if (nearT > maxt || farT < mint) return 0;
            if (nearT < mint && farT > maxt) return 0;
            return 1;
        }
        if (!(nearT <= maxt && farT >= mint)) return 0;
        if (nearT < mint) {
            if (farT > maxt) return 0;
            *t = (float)farT;
        } else {
            *t = (float)nearT;
        }
        *lx = *ly = 0.0f;
        return 1;
    }
    /* m_worldToObject.transformAffine(_ray, ray) (transform.h:292-307) */
    V3 o = xf_point_affine(&a->o2w.inv, ray->o), d = xf_vector(&a->o2w.inv, ray->d);
    float hit = -o.z / d.z;
    if (!(hit >= mint && hit <= maxt)) return 0;
    float px = o.x + d.x * hit, py = o.y + d.y * hit;
    if (a->type == MTSGPU_SHAPE_RECTANGLE) { if (!(fabsf(px) <= 1 && fabsf(py) <= 1)) return 0; }
    else if (!(px * px + py * py <= 1)) return 0;
    *t = hit; *lx = px; *ly = py;
    return 1;
}

/* fillIntersectionRecord (rectangle.cpp:155-167, disk.cpp:169-200, sphere.cpp:209-255):
 * p, geometric normal, shading normal (before computeShadingFrame), dpdu, uv.  The
 * disk sets only shFrame.n and leaves geoFrame as the record held it: the
 * oracle (like the product) uses the shading normal there. */
static void ana_fill(const Ana *a, const Ray *ray, float t, float lx, float ly,
                     V3 *p, V3 *geoN, V3 *shN, V3 *dpdu, float *u, float *v) {
    *p = vadd(ray->o, vmul(ray->d, t));
    if (a->type == MTSGPU_SHAPE_RECTANGLE) {
        *geoN = *shN = a->n;
        *dpdu = a->dpdu;
        *u = 0.5f * (lx + 1); *v = 0.5f * (ly + 1);
    } else if (a->type == MTSGPU_SHAPE_DISK) {
        float r = sqrtf(lx * lx + ly * ly), invR = (r == 0) ? 0.0f : (1.0f / r);
        float phi = o_atan2(ly, lx);
        if (phi < 0) phi += 2 * M_PI_F;
        float cosPhi = lx * invR, sinPhi = ly * invR;
        *dpdu = r != 0 ? xf_vector(&a->o2w.t, v3(cosPhi, sinPhi, 0)) : xf_vector(&a->o2w.t, v3(1, 0, 0));
        *geoN = *shN = a->n;
        *u = r; *v = phi * INV_TWOPI_F;
    } else {
        *p = vadd(a->center, vmul(vnormalize(vsub(*p, a->center)), a->radius));
        V3 local = xf_vector(&a->o2w.inv, vsub(*p, a->center));
        float theta = o_acos(smin(1.0f, smax(-1.0f, local.z / a->radius))); /* math::safe_acos */
        float phi = o_atan2(local.y, local.x);
        if (phi < 0) phi += 2 * M_PI_F;
        *u = phi * (0.5f * INV_PI_F);
        *v = theta * INV_PI_F;
        float tp = 2 * M_PI_F;
        *dpdu = xf_vector(&a->o2w.t, v3(-local.y * tp, local.x * tp, 0 * tp));
        V3 n = vnormalize(vsub(*p, a->center));
        if (a->flip) n = vmul(n, -1.0f);
        *geoN = *shN = n;
    }
}

/* m_shape->sampleDirect(dRec, sample) of an analytic area light: samplePosition
 * (rectangle.cpp:210-216, disk.cpp:247-255) + Shape::sampleDirect (shape.cpp:102-115),
 * or Sphere::sampleDirect (sphere.cpp:286-355) */
static void ana_sample_direct(const Ana *a, V3 ref, float sx, float sy, V3 *p, V3 *n, V3 *d, float *dist, float *pdf) {
    if (a->type == MTSGPU_SHAPE_SPHERE) {
        V3 refToCenter = vsub(a->center, ref);
        float refDist2 = vlen2(refToCenter);
        float invRefDist = (float)1 / sqrtf(refDist2);
        float sinAlpha = a->radius * invRefDist;
        if (sinAlpha < 1 - EPSILON) {
            float cosAlpha = safe_sqrt(1.0f - sinAlpha * sinAlpha);
            Frame F;
            F.n = vmul(refToCenter, invRefDist);
            coordinate_system(F.n, &F.s, &F.t);
            float cosTheta = (1 - sx) + sx * cosAlpha; /* warp::squareToUniformCone (warp.cpp:54-63) */
            float sinTheta = safe_sqrt(1.0f - cosTheta * cosTheta);
            float sinPhi, cosPhi;
            o_sincos(2.0f * M_PI_F * sy, &sinPhi, &cosPhi);
            *d = to_world(&F, v3(cosPhi * sinTheta, sinPhi * sinTheta, cosTheta));
            *pdf = INV_TWOPI_F / (1 - cosAlpha);
            float projDist = vdot(refToCenter, *d);
            float baseT = refDist2 / projDist;
            V3 query = vadd(ref, vmul(*d, baseT));
            V3 queryToCenter = vsub(a->center, query);
            float queryDist2 = vlen2(queryToCenter);
            float queryProjDist = vdot(queryToCenter, *d);
            float A = 1.0f, B = -2 * queryProjDist, C = queryDist2 - a->radius * a->radius;
            float nearT, farT;
            if (!solve_quadratic_f(A, B, C, &nearT, &farT)) nearT = queryProjDist;
            *dist = baseT + nearT;
            *n = vnormalize(vsub(vmul(*d, nearT), queryToCenter));
            *p = vadd(a->center, vmul(*n, a->radius));
        } else {
            float z = 1.0f - 2.0f * sy; /* warp::squareToUniformSphere (warp.cpp:25-31) */
            float r = safe_sqrt(1.0f - z * z);
            float sinPhi, cosPhi;
            o_sincos(2.0f * M_PI_F * sx, &sinPhi, &cosPhi);
            V3 dv = v3(r * cosPhi, r * sinPhi, z);
            *p = vadd(a->center, vmul(dv, a->radius));
            *n = dv;
            *d = vsub(*p, ref);
            float dist2 = vlen2(*d);
            *dist = sqrtf(dist2);
            *d = vdiv(*d, *dist);
            *pdf = a->invArea * dist2 / vabsdot(*d, *n);
        }
        if (a->flip) *n = vmul(*n, -1.0f);
        return;
    }
    if (a->type == MTSGPU_SHAPE_RECTANGLE) {
        *p = xf_point(&a->o2w.t, v3(sx * 2 - 1, sy * 2 - 1, 0));
    } else {
        float px, py;
        square_to_disk_concentric(sx, sy, &px, &py);
        *p = xf_point(&a->o2w.t, v3(px, py, 0));
    }
    *n = a->n;
    *pdf = a->invArea;
    *d = vsub(*p, ref);
    float distSquared = vlen2(*d);
    *dist = sqrtf(distSquared);
    *d = vdiv(*d, *dist);
    float dp = vabsdot(*d, *n);
    *pdf *= dp != 0 ? (distSquared / dp) : 0.0f;
}

/* pdfDirect in solid angle (shape.cpp:117-126; sphere.cpp:357-387) */
static float ana_pdf_direct(const Ana *a, V3 ref, V3 d, V3 n, float dist) {
    if (a->type == MTSGPU_SHAPE_SPHERE) {
        V3 refToCenter = vsub(a->center, ref);
        float invRefDist = (float)1.0f / vlen(refToCenter);
        float sinAlpha = a->radius * invRefDist;
        if (sinAlpha < 1 - EPSILON) {
            float cosAlpha = safe_sqrt(1 - sinAlpha * sinAlpha);
            return INV_TWOPI_F / (1 - cosAlpha);
        }
        return a->invArea * dist * dist / vabsdot(d, n);
    }
    return a->invArea * (dist * dist) / vabsdot(d, n);
}

/* ------------------------------------------------------------------------ */
/* scene (configure): meshes, emitters, acceleration                          */
/* ------------------------------------------------------------------------ */
/* ------------------------------------------------------------------------ */
/* environment emitter (emitters/envmap.cpp) and its MIP map                  */
/* (render/mipmap.h, core/rfilter.h Resampler, rfilters/lanczos.cpp)          */
/* ------------------------------------------------------------------------ */
#define ENV_MAX_LEVELS 18
#define EWA_LUT 64 /* MTS_MIPMAP_LUT_SIZE, mipmap.h:37 */

typedef struct Env {
    int constant;  /* ConstantBackgroundEmitter (constant.cpp): radiance only */
    V3 radiance;
    int levels, w0, h0;
    int lw[ENV_MAX_LEVELS], lh[ENV_MAX_LEVELS];
    float ratioX[ENV_MAX_LEVELS], ratioY[ENV_MAX_LEVELS];
    uint16_t *lv[ENV_MAX_LEVELS]; /* RGB halves per texel (SpectrumHalf) */
    float *cdfRows, *cdfCols, *rowWeights;
    float normalization, pixelX, pixelY, scale;
    V3 center; float radius;
    M4 toWorld, toLocal;
    float lut[EWA_LUT];
    float maxAniso;
} Env;

/* half::half(float) (core/half.h:434-488, libcore/half.cpp:78-200) */
static uint16_t o_float_to_half(float f) {
    uint32_t i; memcpy(&i, &f, 4);
    const int s = (i >> 16) & 0x00008000;
    int e = ((i >> 23) & 0x000000ff) - (127 - 15);
    int m = i & 0x007fffff;
    if (e <= 0) {
        if (e < -10) return (uint16_t)s;
        m = m | 0x00800000;
        int t = 14 - e;
        int a = (1 << (t - 1)) - 1;
        int b = (m >> t) & 1;
        m = (m + a + b) >> t;
        return (uint16_t)(s | m);
    } else if (e == 0xff - (127 - 15)) {
        if (m == 0) return (uint16_t)(s | 0x7c00);
        m >>= 13;
        return (uint16_t)(s | 0x7c00 | m | (m == 0));
    } else {
        m = m + 0x00000fff + ((m >> 13) & 1);
        if (m & 0x00800000) { m = 0; e += 1; }
        if (e > 30) return (uint16_t)(s | 0x7c00);
        return (uint16_t)(s | (e << 10) | (m >> 13));
    }
}
/* half::operator float (exact) */
static float o_half_to_float(uint16_t h) {
    int s = (h >> 15) & 1, e = (h >> 10) & 0x1f, m = h & 0x3ff;
    float r;
    if (e == 0) r = ldexpf((float)m, -24);
    else if (e == 31) r = m ? NAN : INFINITY;
    else r = ldexpf((float)(m | 0x400), e - 25);
    return s ? -r : r;
}
static inline float lum3(V3 c) { return c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f; } /* spectrum.h:638-640 */

/* LanczosSincFilter::eval, lobes = 2 (lanczos.cpp:43-55); glibc sinf as the reference */
static float lanczos2(float x) {
    x = fabsf(x);
    if (x < EPSILON) return 1.0f;
    else if (x > 2.0f) return 0.0f;
    float x1 = M_PI_F * x; /* M_PI = M_PI_FLT under SINGLE_PRECISION (constants.h:80-83) */
    float x2 = x1 / 2.0f;
    return (sinf(x1) * sinf(x2)) / (x1 * x2);
}

/* one pass of Bitmap::resample (bitmap.cpp:2258-2329) with Resampler<float>
   (rfilter.h:123-198) and resampleAndClamp(0, +inf) (rfilter.h:232-280) */
static void resample_pass(const float *src, int srcRes, size_t sStride, float *dst, int dstRes, size_t tStride,
                          int nlines, size_t sLine, size_t tLine, int repeat) {
    float filterRadius = 2.0f, scale = 1.0f, invScale = 1.0f;
    if (dstRes < srcRes) { scale = (float)srcRes / (float)dstRes; invScale = 1 / scale; filterRadius *= scale; }
    int taps = (int)ceilf(filterRadius * 2);
    int *start = (int *)malloc(sizeof(int) * dstRes);
    float *w = (float *)malloc(sizeof(float) * (size_t)taps * dstRes);
    for (int i = 0; i < dstRes; i++) {
        float center = (i + 0.5f) / dstRes * srcRes;
        start[i] = (int)floorf(center - filterRadius + 0.5f);
        float sum = 0;
        for (int j = 0; j < taps; j++) {
            float pos = start[i] + j + 0.5f - center;
            float weight = lanczos2(pos * invScale);
            w[i * taps + j] = weight;
            sum += weight;
        }
        float normalization = 1.0f / sum;
        for (int j = 0; j < taps; j++) w[i * taps + j] = w[i * taps + j] * normalization;
    }
    for (int line = 0; line < nlines; ++line) {
        const float *s = src + line * sLine;
        float *t = dst + line * tLine;
        for (int i = 0; i < dstRes; ++i)
            for (int ch = 0; ch < 3; ++ch) {
                float result = 0;
                for (int j = 0; j < taps; ++j) {
                    int pos = start[i] + j;
                    if (pos < 0 || pos >= srcRes) {
                        if (repeat) { pos = pos % srcRes; if (pos < 0) pos += srcRes; }
                        else pos = pos < 0 ? 0 : (pos > srcRes - 1 ? srcRes - 1 : pos);
                    }
                    result += s[sStride * 3 * pos + ch] * w[i * taps + j];
                }
                float r = smax(0.0f, result);
                t[tStride * 3 * i + ch] = smin(INFINITY, r);
            }
    }
    free(start); free(w);
}

static void env_free(Env *E) {
    for (int l = 0; l < ENV_MAX_LEVELS; ++l) free(E->lv[l]);
    free(E->cdfRows); free(E->cdfCols); free(E->rowWeights);
}

static V3 env_texel(const Env *E, int level, int x, int y) { /* evalTexel, mipmap.h:427-490 */
    int w = E->lw[level], h = E->lh[level];
    if (x < 0 || x >= w) { x = x % w; if (x < 0) x += w; }          /* ERepeat */
    if (y < 0 || y >= h) y = y < 0 ? 0 : (y > h - 1 ? h - 1 : y);   /* EClamp */
    const uint16_t *t = E->lv[level] + 3 * ((size_t)y * w + x);
    return v3(o_half_to_float(t[0]), o_half_to_float(t[1]), o_half_to_float(t[2]));
}

/* EnvironmentMap ctor + configure (envmap.cpp:105-185,261-321), TMIPMap ctor (mipmap.h:155-301) */
static int env_configure(const mtsgpu_emitter_desc *e, Env *E) {
    memset(E, 0, sizeof *E);
    int W = (int)e->env_width, H = (int)e->env_height;
    if (!e->env_rgb || W <= 0 || H <= 0 || W > 0xFFFF || H > 0xFFFF) return MTSGPU_EINVAL;
    E->w0 = W; E->h0 = H; E->scale = e->env_scale; E->maxAniso = 10.0f;
    size_t n = (size_t)W * H * 3;
    float *cur = (float *)malloc(sizeof(float) * n);
    memcpy(cur, e->env_rgb, sizeof(float) * n);
    float mn = INFINITY;
    for (size_t i = 0; i < n; ++i) mn = smin(mn, cur[i]);
    if (mn < 0) for (size_t i = 0; i < n; ++i) cur[i] = smax(0.0f, cur[i]);   /* clampNegative */
    int w = W, h = H, level = 0;
    for (;;) {
        E->lw[level] = w; E->lh[level] = h;
        E->ratioX[level] = (float)w / (float)W; E->ratioY[level] = (float)h / (float)H;
        E->lv[level] = (uint16_t *)malloc(sizeof(uint16_t) * 3 * (size_t)w * h);
        for (size_t i = 0; i < (size_t)w * h * 3; ++i) E->lv[level][i] = o_float_to_half(cur[i]);
        ++level;
        if (!(w > 1 || h > 1)) break;
        if (level >= ENV_MAX_LEVELS) { free(cur); return MTSGPU_EINVAL; }
        int nw = (w + 1) / 2, nh = (h + 1) / 2;   /* std::max(1, (size + 1) / 2) */
        if (nw < 1) nw = 1;
        if (nh < 1) nh = 1;
        float *tmp = cur;
        if (nw != w) {
            float *t = (float *)malloc(sizeof(float) * 3 * (size_t)nw * h);
            resample_pass(tmp, w, 1, t, nw, 1, h, (size_t)w * 3, (size_t)nw * 3, 1);
            free(tmp); tmp = t;
        }
        if (nh != h) {
            float *t = (float *)malloc(sizeof(float) * 3 * (size_t)nw * nh);
            resample_pass(tmp, h, nw, t, nh, nw, nw, 3, 3, 0);
            free(tmp); tmp = t;
        }
        cur = tmp; w = nw; h = nh;
    }
    free(cur);
    E->levels = level;
    for (int i = 0; i < EWA_LUT; ++i) {
        float r2 = (float)i / (float)(EWA_LUT - 1);
        E->lut[i] = o_fastexp(-2.0f * r2) - o_fastexp(-2.0f);
    }
    E->cdfCols = (float *)malloc(sizeof(float) * (size_t)(W + 1) * H);
    E->cdfRows = (float *)malloc(sizeof(float) * (H + 1));
    E->rowWeights = (float *)malloc(sizeof(float) * H);
    size_t colPos = 0, rowPos = 0;
    float rowSum = 0.0f;
    E->cdfRows[rowPos++] = 0;
    for (int y = 0; y < H; ++y) {
        float colSum = 0;
        E->cdfCols[colPos++] = 0;
        for (int x = 0; x < W; ++x) {
            colSum += lum3(env_texel(E, 0, x, y));
            E->cdfCols[colPos++] = colSum;
        }
        float normalization = 1.0f / colSum;
        for (int x = 1; x < W; ++x) E->cdfCols[colPos - x - 1] *= normalization;
        E->cdfCols[colPos - 1] = 1.0f;
        float weight = sinf((y + 0.5f) * M_PI_F / H);
        E->rowWeights[y] = weight;
        rowSum += colSum * weight;
        E->cdfRows[rowPos++] = rowSum;
    }
    float normalization = 1.0f / rowSum;
    for (int y = 1; y < H; ++y) E->cdfRows[rowPos - y - 1] *= normalization;
    E->cdfRows[rowPos - 1] = 1.0f;
    if (rowSum == 0 || !isfinite(rowSum)) return MTSGPU_EINVAL;
    E->normalization = 1.0f / (rowSum * (2 * M_PI_F / W) * (M_PI_F / H));
    E->pixelX = 2 * M_PI_F / W;
    E->pixelY = M_PI_F / H;
    int haveInv = 0;
    for (int i = 0; i < 16; ++i) {
        E->toWorld.m[i / 4][i % 4] = e->env_to_world[i];
        E->toLocal.m[i / 4][i % 4] = e->env_to_world_inv[i];
        haveInv |= e->env_to_world_inv[i] != 0.0f;
    }
    if (!haveInv && !m4_invert(&E->toWorld, &E->toLocal)) return MTSGPU_EINVAL;
    return MTSGPU_OK;
}

static V3 env_eval_box(const Env *E, int level, float u, float v) { /* mipmap.h:493-497 */
    return env_texel(E, level, (int)floorf(u * E->lw[level]), (int)floorf(v * E->lh[level]));
}
static V3 env_eval_bilinear(const Env *E, int level, float uvx, float uvy) { /* mipmap.h:500-522 */
    if (!isfinite(uvx) || !isfinite(uvy)) return v3(0, 0, 0);
    if (level >= E->levels) return env_eval_box(E, E->levels - 1, uvx, uvy);
    float u = uvx * E->lw[level] - 0.5f, v = uvy * E->lh[level] - 0.5f;
    int xPos = (int)floorf(u), yPos = (int)floorf(v);
    float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
    V3 r = vmul(vmul(env_texel(E, level, xPos, yPos), dx2), dy2);
    r = vadd(r, vmul(vmul(env_texel(E, level, xPos, yPos + 1), dx2), dy1));
    r = vadd(r, vmul(vmul(env_texel(E, level, xPos + 1, yPos), dx1), dy2));
    r = vadd(r, vmul(vmul(env_texel(E, level, xPos + 1, yPos + 1), dx1), dy1));
    return r;
}
static V3 env_eval_ewa(const Env *E, int level, float uvx, float uvy, float A, float B, float C) { /* mipmap.h:760-836 */
    if (!isfinite(A + B + C + uvx + uvy)) return v3(0, 0, 0);
    if (level >= E->levels) return env_eval_box(E, E->levels - 1, uvx, uvy);
    float u = uvx * E->lw[level] - 0.5f;
    float v = uvy * E->lh[level] - 0.5f;
    A /= E->ratioX[level] * E->ratioX[level];
    B /= E->ratioX[level] * E->ratioY[level];
    C /= E->ratioY[level] * E->ratioY[level];
    float invDet = 1.0f / (-B * B + 4.0f * A * C), deltaU = 2.0f * sqrtf(C * invDet), deltaV = 2.0f * sqrtf(A * invDet);
    int u0 = (int)ceilf(u - deltaU), u1 = (int)floorf(u + deltaU);
    int v0 = (int)ceilf(v - deltaV), v1 = (int)floorf(v + deltaV);
    float As = A * EWA_LUT, Bs = B * EWA_LUT, Cs = C * EWA_LUT;
    V3 result = v3(0, 0, 0);
    float denominator = 0.0f;
    float ddq = 2 * As, uu0 = (float)u0 - u;
    for (int vt = v0; vt <= v1; ++vt) {
        const float vv = (float)vt - v;
        float q = As * uu0 * uu0 + (Bs * uu0 + Cs * vv) * vv;
        float dq = As * (2 * uu0 + 1) + Bs * vv;
        for (int ut = u0; ut <= u1; ++ut) {
            if (q < (float)EWA_LUT) {
                uint32_t qi = (uint32_t)(long long)q;
                if (qi < EWA_LUT) {
                    const float weight = E->lut[(int)q];
                    result = vadd(result, vmul(env_texel(E, level, ut, vt), weight));
                    denominator += weight;
                }
            }
            q += dq;
            dq += ddq;
        }
    }
    if (denominator == 0) return env_eval_bilinear(E, level, uvx, uvy);
    return vdiv(result, denominator);
}
static float o_hypot2(float a, float b) { /* math.cpp:74-86 */
    float r;
    if (fabsf(a) > fabsf(b)) { r = b / a; r = fabsf(a) * sqrtf(1.0f + r * r); }
    else if (b != 0.0f) { r = a / b; r = fabsf(b) * sqrtf(1.0f + r * r); }
    else r = 0.0f;
    return r;
}
static inline float o_log2(float v) { /* math.cpp:103-106 */
    const float invLn2 = 1.0f / logf(2.0f);
    return o_fastlog(v) * invLn2;
}
static V3 env_eval_filtered(const Env *E, float uvx, float uvy, float d0x, float d0y, float d1x, float d1y) { /* mipmap.h:560-660 */
    float du0 = d0x * E->w0, dv0 = d0y * E->h0, du1 = d1x * E->w0, dv1 = d1y * E->h0;
    float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1), C = du0 * du0 + du1 * du1, F = A * C - B * B * 0.25f;
    float root = o_hypot2(A - C, B), Aprime = 0.5f * (A + C - root), Cprime = 0.5f * (A + C + root);
    float majorRadius = Aprime != 0 ? sqrtf(F / Aprime) : 0, minorRadius = Cprime != 0 ? sqrtf(F / Cprime) : 0;
    if (!(minorRadius > 0) || !(majorRadius > 0) || F < 0) {
        float level = o_log2(smax(majorRadius, EPSILON));
        int ilevel = (int)floorf(level);
        if (ilevel < 0) return env_eval_bilinear(E, 0, uvx, uvy);
        float a = level - ilevel;
        return vadd(vmul(env_eval_bilinear(E, ilevel, uvx, uvy), 1.0f - a), vmul(env_eval_bilinear(E, ilevel + 1, uvx, uvy), a));
    }
    if (minorRadius * E->maxAniso < majorRadius) {
        minorRadius = majorRadius / E->maxAniso;
        float theta = 0.5f * o_atan(B / (A - C)), sinTheta, cosTheta;
        o_sincos(theta, &sinTheta, &cosTheta);
        float a2 = majorRadius * majorRadius, b2 = minorRadius * minorRadius, sinTheta2 = sinTheta * sinTheta,
              cosTheta2 = cosTheta * cosTheta, sin2Theta = 2 * sinTheta * cosTheta;
        A = a2 * cosTheta2 + b2 * sinTheta2;
        B = (a2 - b2) * sin2Theta;
        C = a2 * sinTheta2 + b2 * cosTheta2;
        F = a2 * b2;
    }
    float scale = 1.0f / F;
    A *= scale; B *= scale; C *= scale;
    float level = smax(0.0f, o_log2(minorRadius));
    int ilevel = (int)level;
    float a = level - ilevel;
    if (majorRadius < 1 || !(A > 0 && C > 0)) return env_eval_bilinear(E, ilevel, uvx, uvy);
    return vadd(vmul(env_eval_ewa(E, ilevel, uvx, uvy, A, B, C), 1.0f - a), vmul(env_eval_ewa(E, ilevel + 1, uvx, uvy, A, B, C), a));
}
static inline float safe_acosf(float v) { return o_acos(smin(1.0f, smax(-1.0f, v))); } /* math.h:250-252 */

/* EnvironmentMap::evalEnvironment (envmap.cpp:380-410); constant.cpp:241-243 */
static V3 env_eval(const Env *E, const Ray *ray) {
    if (E->constant) return E->radiance;
    V3 v = xf_vector(&E->toLocal, ray->d);
    float uvx = o_atan2(v.x, -v.z) * INV_TWOPI_F, uvy = safe_acosf(v.y) * INV_PI_F;
    V3 value;
    if (!ray->hasDiff) {
        value = env_eval_bilinear(E, 0, uvx, uvy);
    } else {
        V3 dvdx = vsub(xf_vector(&E->toLocal, ray->rxD), v), dvdy = vsub(xf_vector(&E->toLocal, ray->ryD), v);
        float t1 = INV_TWOPI_F / (v.x * v.x + v.z * v.z), t2 = -INV_PI_F / smax(safe_sqrt(1.0f - v.y * v.y), EPSILON);
        value = env_eval_filtered(E, uvx, uvy, t1 * (dvdx.z * v.x - dvdx.x * v.z), t2 * dvdx.y,
                                  t1 * (dvdy.z * v.x - dvdy.x * v.z), t2 * dvdy.y);
    }
    return vmul(value, E->scale);
}

/* solveQuadratic (util.cpp:447-485), BSphere::rayIntersect (bsphere.h:88-95) */
static int solve_quadratic(float a, float b, float c, float *x0, float *x1) {
    if (a == 0) {
        if (b != 0) { *x0 = *x1 = -c / b; return 1; }
        return 0;
    }
    float discrim = b * b - 4.0f * a * c;
    if (discrim < 0) return 0;
    float temp, sqrtDiscrim = sqrtf(discrim);
    if (b < 0) temp = -0.5f * (b - sqrtDiscrim);
    else temp = -0.5f * (b + sqrtDiscrim);
    *x0 = temp / a;
    *x1 = c / temp;
    if (*x0 > *x1) { float t = *x0; *x0 = *x1; *x1 = t; }
    return 1;
}
static int env_bsphere(const Env *E, V3 ro, V3 d, float *nearT, float *farT) {
    V3 o = vsub(ro, E->center);
    float A = vlen2(d), B = 2 * vdot(o, d), C = vlen2(o) - E->radius * E->radius;
    return solve_quadratic(A, B, C, nearT, farT);
}

/* sampleReuse over the envmap CDFs (envmap.cpp:687-692) */
static uint32_t env_sample_reuse(const float *cdf, uint32_t size, float *sample) {
    uint32_t lo = 0, hi = size + 1;
    while (lo < hi) { uint32_t mid = (lo + hi) / 2; if (cdf[mid] < *sample) lo = mid + 1; else hi = mid; }
    long e = (long)lo - 1;
    uint32_t index = (uint32_t)(e < 0 ? 0 : e);
    if (index > size - 1) index = size - 1;
    *sample = (*sample - cdf[index]) / (cdf[index + 1] - cdf[index]);
    return index;
}
static float interval_to_tent(float sample) { /* warp.cpp:143-155 */
    float sign;
    if (sample < 0.5f) { sign = 1; sample *= 2; }
    else { sign = -1; sample = 2 * (sample - 0.5f); }
    return sign * (1 - sqrtf(sample));
}
static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }


typedef struct {
    V3 *pos, *nrm;        /* nrm NULL: face normals */
    float *uv;
    uint32_t *idx;
    V3 *dpdu;             /* per-triangle UV tangent (trimesh.cpp:683-739) or NULL */
    uint32_t nv, nt, primOffset;
    int bsdf, emitter;
    float *areaCdf;       /* nt+1 */
    float invArea;
    int kind;             /* MTSGPU_SHAPE_* (analytic: nt = 1, no vertices) */
    Ana ana;
} Mesh;

typedef struct { int type; V3 radiance; float weight; int mesh; } Emitter;

typedef struct { float bmin[3], bmax[3]; uint32_t left, right, first, count; } BNode;

typedef struct {
    Mesh *meshes; uint32_t nmeshes;
    Bsdf *bsdfs; uint32_t nbsdfs; /* + defaults appended */
    Emitter *emitters; uint32_t nemitters;
    float *emCdf; float emNorm;
    TriAccel *ta; uint32_t *taMesh, *taTri; uint32_t nprims;
    BNode *nodes; uint32_t nnodes; uint32_t *order;
    float aabbMin[3], aabbMax[3];
    Camera cam;
    int envIndex;
    Env *env;
} Scene;

/* unitAngle (core/util.h:309-314) -- uses float asin */
static float unit_angle(V3 u, V3 v) {
    if (vdot(u, v) < 0) return M_PI_F - 2 * asinf(0.5f * vlen(vadd(v, u)));
    return 2 * asinf(0.5f * vlen(vsub(v, u)));
}

/* DiscreteDistribution (core/pmf.h:35-169) */
static float dd_normalize(float *cdf, uint32_t n, float *normalization) {
    float sum = cdf[n];
    if (sum > 0) {
        *normalization = 1.0f / sum;
        for (uint32_t i = 1; i < n + 1; ++i) cdf[i] *= *normalization;
        cdf[n] = 1.0f;
    } else {
        *normalization = 0.0f;
    }
    return sum;
}
static uint32_t dd_sample(const float *cdf, uint32_t n, float value) {
    /* std::lower_bound over cdf[0..n] */
    uint32_t lo = 0, hi = n + 1;
    while (lo < hi) { uint32_t mid = (lo + hi) / 2; if (cdf[mid] < value) lo = mid + 1; else hi = mid; }
    long idx = (long)lo - 1; if (idx < 0) idx = 0;
    uint32_t index = (uint32_t)idx; if (index > n - 1) index = n - 1;
    while (cdf[index + 1] - cdf[index] == 0 && index < n - 1) ++index; /* guarded variant of :133-134 */
    return index;
}
static uint32_t dd_sample_reuse(const float *cdf, uint32_t n, float *value, float *pdf) {
    uint32_t index = dd_sample(cdf, n, *value);
    if (pdf) *pdf = cdf[index + 1] - cdf[index];
    *value = (*value - cdf[index]) / (cdf[index + 1] - cdf[index]);
    return index;
}

static void compute_normals(Mesh *m, int face, int flip, const float *nin) { /* trimesh.cpp:608-681 */
    if (face) {
        m->nrm = NULL;
        if (flip)
            for (uint32_t i = 0; i < m->nt; ++i) { uint32_t t = m->idx[3 * i]; m->idx[3 * i] = m->idx[3 * i + 1]; m->idx[3 * i + 1] = t; }
        return;
    }
    m->nrm = (V3 *)calloc(m->nv, sizeof(V3));
    if (nin) {
        for (uint32_t i = 0; i < m->nv; ++i) {
            m->nrm[i] = v3(nin[3 * i], nin[3 * i + 1], nin[3 * i + 2]);
            if (flip) m->nrm[i] = vmul(m->nrm[i], -1);
        }
        return;
    }
    for (uint32_t i = 0; i < m->nt; i++) {
        V3 n = v3(0, 0, 0);
        for (int j = 0; j < 3; ++j) {
            V3 v0 = m->pos[m->idx[3 * i + j]], v1 = m->pos[m->idx[3 * i + (j + 1) % 3]], v2 = m->pos[m->idx[3 * i + (j + 2) % 3]];
            V3 sideA = vsub(v1, v0), sideB = vsub(v2, v0);
            if (j == 0) {
                n = vcross(sideA, sideB);
                float length = vlen(n);
                if (length == 0) break;
                n = vdiv(n, length);
            }
            float angle = unit_angle(vnormalize(sideA), vnormalize(sideB));
            V3 *dst = &m->nrm[m->idx[3 * i + j]];
            *dst = vadd(*dst, vmul(n, angle));
        }
    }
    for (uint32_t i = 0; i < m->nv; i++) {
        V3 n = m->nrm[i];
        float length = vlen(n);
        if (flip) length *= -1;
        if (length != 0) m->nrm[i] = vdiv(n, length);
        else m->nrm[i] = v3(1, 0, 0);
    }
}

static void compute_uv_tangents(Mesh *m) { /* trimesh.cpp:683-739 */
    if (!m->uv) { m->dpdu = NULL; return; }
    m->dpdu = (V3 *)calloc(m->nt, sizeof(V3));
    for (uint32_t i = 0; i < m->nt; i++) {
        uint32_t i0 = m->idx[3 * i], i1 = m->idx[3 * i + 1], i2 = m->idx[3 * i + 2];
        V3 v0 = m->pos[i0], v1 = m->pos[i1], v2 = m->pos[i2];
        float u0 = m->uv[2 * i0], w0 = m->uv[2 * i0 + 1], u1 = m->uv[2 * i1], w1 = m->uv[2 * i1 + 1], u2 = m->uv[2 * i2], w2 = m->uv[2 * i2 + 1];
        V3 dP1 = vsub(v1, v0), dP2 = vsub(v2, v0);
        float dUV1x = u1 - u0, dUV1y = w1 - w0, dUV2x = u2 - u0, dUV2y = w2 - w0;
        V3 n = vcross(dP1, dP2);
        float length = vlen(n);
        if (length == 0) continue;
        float determinant = dUV1x * dUV2y - dUV1y * dUV2x;
        if (determinant == 0) {
            V3 b, c;
            coordinate_system(vdiv(n, length), &b, &c);
            m->dpdu[i] = b;
        } else {
            float invDet = 1.0f / determinant;
            m->dpdu[i] = vmul(vsub(vmul(dP1, dUV2y), vmul(dP2, dUV1y)), invDet);
        }
    }
}

/* --- oracle BVH (median split; any exact closest-hit structure gives the same
 * result as the reference kd-tree up to exact-t ties, which both the oracle
 * and the product break towards the larger primitive index) -------------- */
typedef struct { float c[3]; float bmin[3], bmax[3]; } PrimBox;

/* absolute part of the node boxes' conservative inflation: 1e-7 of the scene diagonal (as
   scene_build.cpp's Builder::absEps).  A box of zero extent at coordinate 0 -- a floor at
   y = 0 -- gets no relative inflation at all, and its slab t can round one ulp beyond the
   TriAccel t of a triangle it holds: without this the traversal could cull an exact-t tie
   partner (C4's coplanar hall and floor meshes), and the closest hit would depend on the
   traversal order instead of the (t, larger primitive) rule */
static float g_bvh_abs_eps = 1e-30f;
static uint32_t bvh_build(Scene *S, PrimBox *pb, uint32_t *order, uint32_t first, uint32_t count, uint32_t *nnodes) {
    uint32_t id = (*nnodes)++;
    BNode *n = &S->nodes[id];
    float bmin[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, bmax[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    float cmin[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, cmax[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (uint32_t i = first; i < first + count; ++i) {
        PrimBox *p = &pb[order[i]];
        for (int a = 0; a < 3; ++a) {
            if (p->bmin[a] < bmin[a]) bmin[a] = p->bmin[a];
            if (p->bmax[a] > bmax[a]) bmax[a] = p->bmax[a];
            if (p->c[a] < cmin[a]) cmin[a] = p->c[a];
            if (p->c[a] > cmax[a]) cmax[a] = p->c[a];
        }
    }
    for (int a = 0; a < 3; ++a) { /* conservative inflation: never loses a hit */
        float e = (bmax[a] - bmin[a]) * 1e-4f + 1e-6f * (fabsf(bmin[a]) + fabsf(bmax[a])) + g_bvh_abs_eps;
        n->bmin[a] = bmin[a] - e; n->bmax[a] = bmax[a] + e;
    }
    if (count <= 4) { n->first = first; n->count = count; n->left = n->right = 0; return id; }
    int axis = 0;
    float ext = cmax[0] - cmin[0];
    for (int a = 1; a < 3; ++a) if (cmax[a] - cmin[a] > ext) { ext = cmax[a] - cmin[a]; axis = a; }
    /* nth_element by centroid on axis (simple sort of the range) */
    uint32_t mid = first + count / 2;
    /* insertion-free quickselect */
    uint32_t lo = first, hi = first + count - 1;
    while (lo < hi) {
        float pivot = pb[order[(lo + hi) / 2]].c[axis];
        uint32_t i = lo, j = hi;
        while (i <= j) {
            while (pb[order[i]].c[axis] < pivot) i++;
            while (pb[order[j]].c[axis] > pivot) { if (j == 0) break; j--; }
            if (i <= j) { uint32_t t = order[i]; order[i] = order[j]; order[j] = t; i++; if (j == 0) break; j--; }
        }
        if (mid <= j) hi = j; else if (mid >= i) lo = i; else break;
    }
    n->count = 0;
    uint32_t l = bvh_build(S, pb, order, first, mid - first, nnodes);
    uint32_t r = bvh_build(S, pb, order, mid, first + count - mid, nnodes);
    S->nodes[id].left = l; S->nodes[id].right = r; S->nodes[id].count = 0;
    return id;
}

static void scene_free(Scene *S) {
    for (uint32_t i = 0; i < S->nmeshes; ++i) {
        Mesh *m = &S->meshes[i];
        free(m->pos); free(m->nrm); free(m->uv); free(m->idx); free(m->dpdu); free(m->areaCdf);
    }
    if (S->bsdfs) for (uint32_t i = 0; i < S->nbsdfs + 2; ++i) bsdf_free(&S->bsdfs[i]);
    free(S->meshes); free(S->bsdfs); free(S->emitters); free(S->emCdf);
    free(S->ta); free(S->taMesh); free(S->taTri); free(S->nodes); free(S->order);
    if (S->env) { env_free(S->env); free(S->env); }
    memset(S, 0, sizeof *S);
}

static int scene_configure(const mtsgpu_scene_desc *D, Scene *S) {
    memset(S, 0, sizeof *S);
    S->envIndex = -1;
    int rc = camera_configure(&D->sensor, &S->cam);
    if (rc) return rc;
    S->nbsdfs = D->num_bsdfs;
    S->bsdfs = (Bsdf *)calloc(D->num_bsdfs + 2, sizeof(Bsdf));
    for (uint32_t i = 0; i < D->num_bsdfs; ++i)
        if ((rc = bsdf_configure(&D->bsdfs[i], &S->bsdfs[i]))) return rc;
    for (uint32_t i = 0; i < D->num_bsdfs; ++i)
        if (D->bsdfs[i].type == MTSGPU_BSDF_TWOSIDED &&
            (rc = twosided_configure(&D->bsdfs[i], &S->bsdfs[i], S->bsdfs, D->num_bsdfs))) return rc;
    /* Shape::configure default BSDFs (shape.cpp:48-70) */
    mtsgpu_bsdf_desc dd; memset(&dd, 0, sizeof dd);
    dd.type = MTSGPU_BSDF_DIFFUSE; dd.ensure_energy_conservation = 1;
    bsdf_configure(&dd, &S->bsdfs[D->num_bsdfs]);           /* black, emitters */
    dd.reflectance[0] = dd.reflectance[1] = dd.reflectance[2] = 0.5f;
    bsdf_configure(&dd, &S->bsdfs[D->num_bsdfs + 1]);       /* 0.5 gray */

    S->nemitters = D->num_emitters;
    S->emitters = (Emitter *)calloc(D->num_emitters + 1, sizeof(Emitter));
    for (uint32_t i = 0; i < D->num_emitters; ++i) {
        const mtsgpu_emitter_desc *e = &D->emitters[i];
        S->emitters[i].type = e->type;
        S->emitters[i].radiance = v3(e->radiance[0], e->radiance[1], e->radiance[2]);
        S->emitters[i].weight = e->sampling_weight;
        S->emitters[i].mesh = -1;
        if (e->type == MTSGPU_EMITTER_ENVMAP) {
            if (S->env) return MTSGPU_EINVAL; /* one environment emitter per scene (scene.cpp:510-513) */
            S->env = (Env *)calloc(1, sizeof(Env));
            S->envIndex = (int)i;
            if ((rc = env_configure(e, S->env))) return rc;
        } else if (e->type == MTSGPU_EMITTER_CONSTANT) { /* constant.cpp:44-96 */
            if (S->env) return MTSGPU_EINVAL;
            S->env = (Env *)calloc(1, sizeof(Env));
            S->envIndex = (int)i;
            S->env->constant = 1;
            S->env->radiance = v3(e->radiance[0], e->radiance[1], e->radiance[2]);
        } else if (e->type != MTSGPU_EMITTER_AREA) {
            return MTSGPU_EINVAL;
        }
    }
    if (D->num_emitters == 0) return MTSGPU_EINVAL; /* sunsky fallback is out of scope */

    S->nmeshes = D->num_meshes;
    S->meshes = (Mesh *)calloc(D->num_meshes, sizeof(Mesh));
    uint32_t prims = 0;
    for (uint32_t i = 0; i < D->num_meshes; ++i) {
        const mtsgpu_mesh_desc *md = &D->meshes[i];
        Mesh *m = &S->meshes[i];
        if (md->shape_type != MTSGPU_SHAPE_TRIMESH) { /* one primitive */
            m->kind = md->shape_type;
            if ((rc = ana_configure(md, &m->ana))) return rc;
            m->nt = 1; m->primOffset = prims; prims += 1;
            m->emitter = md->emitter;
            if (md->emitter >= (int)D->num_emitters) return MTSGPU_EINVAL;
            if (md->bsdf >= 0) { if (md->bsdf >= (int)D->num_bsdfs) return MTSGPU_EINVAL; m->bsdf = md->bsdf; }
            else m->bsdf = (md->emitter >= 0) ? (int)D->num_bsdfs : (int)D->num_bsdfs + 1;
            if (md->emitter >= 0) {
                if (S->emitters[md->emitter].mesh >= 0) return MTSGPU_EINVAL;
                S->emitters[md->emitter].mesh = (int)i;
                m->invArea = m->ana.invArea;
            }
            continue;
        }
        if (md->num_triangles == 0 || !md->positions || !md->indices) return MTSGPU_EINVAL;
        m->nv = md->num_vertices; m->nt = md->num_triangles; m->primOffset = prims;
        prims += m->nt;
        m->pos = (V3 *)malloc(sizeof(V3) * m->nv);
        for (uint32_t v = 0; v < m->nv; ++v) m->pos[v] = v3(md->positions[3 * v], md->positions[3 * v + 1], md->positions[3 * v + 2]);
        m->idx = (uint32_t *)malloc(sizeof(uint32_t) * 3 * m->nt);
        memcpy(m->idx, md->indices, sizeof(uint32_t) * 3 * m->nt);
        for (uint32_t t = 0; t < 3 * m->nt; ++t) if (m->idx[t] >= m->nv) return MTSGPU_EINVAL;
        if (md->texcoords) { m->uv = (float *)malloc(sizeof(float) * 2 * m->nv); memcpy(m->uv, md->texcoords, sizeof(float) * 2 * m->nv); }
        m->emitter = md->emitter;
        if (md->emitter >= (int)D->num_emitters) return MTSGPU_EINVAL;
        if (md->bsdf >= 0) { if (md->bsdf >= (int)D->num_bsdfs) return MTSGPU_EINVAL; m->bsdf = md->bsdf; }
        else m->bsdf = (md->emitter >= 0) ? (int)D->num_bsdfs : (int)D->num_bsdfs + 1;
        if (md->emitter >= 0) {
            if (S->emitters[md->emitter].mesh >= 0) return MTSGPU_EINVAL;
            S->emitters[md->emitter].mesh = (int)i;
        }
        compute_normals(m, md->face_normals, md->flip_normals, md->normals);
        compute_uv_tangents(m);
        if (md->emitter >= 0) { /* TriMesh::prepareSamplingTable (trimesh.cpp:389-404) */
            m->areaCdf = (float *)malloc(sizeof(float) * (m->nt + 1));
            m->areaCdf[0] = 0.0f;
            for (uint32_t t = 0; t < m->nt; ++t) {
                V3 p0 = m->pos[m->idx[3 * t]], p1 = m->pos[m->idx[3 * t + 1]], p2 = m->pos[m->idx[3 * t + 2]];
                float area = 0.5f * vlen(vcross(vsub(p1, p0), vsub(p2, p0))); /* triangle.cpp:60-66 */
                m->areaCdf[t + 1] = m->areaCdf[t] + area;
            }
            float norm;
            float surfaceArea = dd_normalize(m->areaCdf, m->nt, &norm);
            m->invArea = 1.0f / surfaceArea;
        }
    }
    for (uint32_t i = 0; i < S->nemitters; ++i)
        if (S->emitters[i].type == MTSGPU_EMITTER_AREA && S->emitters[i].mesh < 0) return MTSGPU_EINVAL;
    /* Scene::initialize emitter PDF (scene.cpp:376-381) */
    S->emCdf = (float *)malloc(sizeof(float) * (S->nemitters + 1));
    S->emCdf[0] = 0.0f;
    for (uint32_t i = 0; i < S->nemitters; ++i) S->emCdf[i + 1] = S->emCdf[i] + S->emitters[i].weight;
    dd_normalize(S->emCdf, S->nemitters, &S->emNorm);

    /* TriAccel precompute (skdtree.cpp:74-109) + scene bounds (gkdtree.h:996-1001,1211-1217) */
    S->nprims = prims;
    S->ta = (TriAccel *)malloc(sizeof(TriAccel) * prims);
    S->taMesh = (uint32_t *)malloc(sizeof(uint32_t) * prims);
    S->taTri = (uint32_t *)malloc(sizeof(uint32_t) * prims);
    PrimBox *pb = (PrimBox *)malloc(sizeof(PrimBox) * prims);
    float amin[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, amax[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (uint32_t i = 0; i < S->nmeshes; ++i) {
        Mesh *m = &S->meshes[i];
        if (m->kind != MTSGPU_SHAPE_TRIMESH) { /* k = KNoTriangleFlag (skdtree.cpp:74-109) */
            uint32_t p = m->primOffset;
            memset(&S->ta[p], 0, sizeof(TriAccel));
            S->ta[p].k = 0xFFFFFFFFu;
            S->taMesh[p] = i; S->taTri[p] = 0;
            for (int a = 0; a < 3; ++a) {
                pb[p].bmin[a] = m->ana.bmin[a]; pb[p].bmax[a] = m->ana.bmax[a];
                pb[p].c[a] = 0.5f * (m->ana.bmin[a] + m->ana.bmax[a]);
                if (m->ana.bmin[a] < amin[a]) amin[a] = m->ana.bmin[a];
                if (m->ana.bmax[a] > amax[a]) amax[a] = m->ana.bmax[a];
            }
            continue;
        }
        for (uint32_t t = 0; t < m->nt; ++t) {
            uint32_t p = m->primOffset + t;
            V3 A = m->pos[m->idx[3 * t]], B = m->pos[m->idx[3 * t + 1]], C = m->pos[m->idx[3 * t + 2]];
            triaccel_load(&S->ta[p], A, B, C);
            S->taMesh[p] = i; S->taTri[p] = t;
            for (int a = 0; a < 3; ++a) {
                float x0 = vget(A, a), x1 = vget(B, a), x2 = vget(C, a);
                float lo = x0, hi = x0;
                if (x1 < lo) lo = x1;
                if (x1 > hi) hi = x1;
                if (x2 < lo) lo = x2;
                if (x2 > hi) hi = x2;
                pb[p].bmin[a] = lo; pb[p].bmax[a] = hi;
                pb[p].c[a] = 0.5f * (lo + hi);
                if (lo < amin[a]) amin[a] = lo;
                if (hi > amax[a]) amax[a] = hi;
            }
        }
    }
    const float eps = 1e-3f; /* MTS_KD_AABB_EPSILON */
    for (int a = 0; a < 3; ++a) {
        amin[a] -= (amax[a] - amin[a]) * eps + eps;
        amax[a] += (amax[a] - amin[a]) * eps + eps;
        S->aabbMin[a] = amin[a]; S->aabbMax[a] = amax[a];
    }
    if (S->env) { /* EnvironmentMap::createShape (envmap.cpp:331-345) via scene.cpp:385-413 */
        V3 cp = xf_point(&S->cam.toWorld, v3(0.0f, 0.0f, 0.0f));
        float mn[3], mx[3];
        for (int a = 0; a < 3; ++a) { mn[a] = smin(S->aabbMin[a], vget(cp, a)); mx[a] = smax(S->aabbMax[a], vget(cp, a)); }
        V3 mxv = v3(mx[0], mx[1], mx[2]);
        S->env->center = vmul(vadd(mxv, v3(mn[0], mn[1], mn[2])), 0.5f);
        S->env->radius = smax(EPSILON, vlen(vsub(S->env->center, mxv)) * 1.5f);
    }
    S->order = (uint32_t *)malloc(sizeof(uint32_t) * prims);
    for (uint32_t i = 0; i < prims; ++i) S->order[i] = i;
    S->nodes = (BNode *)malloc(sizeof(BNode) * (2 * prims + 1));
    uint32_t nn = 0;
    float diag = 0;
    for (int a = 0; a < 3; ++a) diag += (S->aabbMax[a] - S->aabbMin[a]) * (S->aabbMax[a] - S->aabbMin[a]);
    g_bvh_abs_eps = 1e-7f * sqrtf(diag) + 1e-30f;   /* read by bvh_build only (scene setup is single-threaded) */
    bvh_build(S, pb, S->order, 0, prims, &nn);
    S->nnodes = nn;
    free(pb);
    return MTSGPU_OK;
}

/* AABB::rayIntersect (core/aabb.h:308-338) on the scene bounds */
static int aabb_ray(const float *mn, const float *mx, const Ray *ray, float *nearT, float *farT) {
    *nearT = -INFINITY; *farT = INFINITY;
    for (int i = 0; i < 3; i++) {
        const float origin = vget(ray->o, i);
        const float minVal = mn[i], maxVal = mx[i];
        if (vget(ray->d, i) == 0) {
            if (origin < minVal || origin > maxVal) return 0;
        } else {
            float t1 = (minVal - origin) * vget(ray->dRcp, i);
            float t2 = (maxVal - origin) * vget(ray->dRcp, i);
            if (t1 > t2) { float t = t1; t1 = t2; t2 = t; }
            *nearT = smax(t1, *nearT);
            *farT = smin(t2, *farT);
            if (!(*nearT <= *farT)) return 0;
        }
    }
    return 1;
}

static inline int node_hit(const BNode *n, const Ray *r, float tmin, float tmax) {
    float t0 = tmin, t1 = tmax;
    for (int a = 0; a < 3; ++a) {
        float o = vget(r->o, a), inv = vget(r->dRcp, a);
        float ta = (n->bmin[a] - o) * inv, tb = (n->bmax[a] - o) * inv;
        if (ta != ta || tb != tb) { /* 0*inf: origin on the slab plane */
            if (o < n->bmin[a] || o > n->bmax[a]) return 0;
            continue;
        }
        if (ta > tb) { float t = ta; ta = tb; tb = t; }
        if (ta > t0) t0 = ta;
        if (tb < t1) t1 = tb;
        if (t0 > t1) return 0;
    }
    return 1;
}

typedef struct { uint64_t rays, shadow, tests, nodes; } Counters;

/* ShapeKDTree::intersect (skdtree.h:248-338): TriAccel or Shape::rayIntersect */
static inline int prim_intersect(const Scene *S, uint32_t p, const Ray *ray, float mint, float maxt, int shadow,
                                 float *u, float *v, float *t) {
    if (S->ta[p].k == 0xFFFFFFFFu)
        return ana_intersect(&S->meshes[S->taMesh[p]].ana, ray, mint, maxt, shadow, t, u, v);
    return triaccel_intersect(&S->ta[p], ray, mint, maxt, u, v, t);
}

/* closest hit over [mint, maxt] (the clipped interval ShapeKDTree passes to
 * rayIntersectHavran, sahkdtree3.h:178-308); ties -> larger prim index */
static int trace_closest(const Scene *S, const Ray *ray, float mint, float maxt,
                         uint32_t *prim, float *tu, float *tv, float *tt, Counters *C) {
    uint32_t stack[128]; int sp = 0;
    stack[sp++] = 0;
    int found = 0; uint32_t best = 0; float bt = maxt, bu = 0, bv = 0;
    while (sp) {
        const BNode *n = &S->nodes[stack[--sp]];
        C->nodes++;
        if (!node_hit(n, ray, mint, bt)) continue;
        if (n->count) {
            for (uint32_t i = n->first; i < n->first + n->count; ++i) {
                uint32_t p = S->order[i];
                float u, v, t;
                C->tests++;
                if (prim_intersect(S, p, ray, mint, bt, 0, &u, &v, &t)) {
                    if (!found || t < bt || p > best) { found = 1; best = p; bt = t; bu = u; bv = v; }
                }
            }
        } else {
            stack[sp++] = n->right; stack[sp++] = n->left;
        }
    }
    if (found) { *prim = best; *tu = bu; *tv = bv; *tt = bt; }
    return found;
}
static int trace_any(const Scene *S, const Ray *ray, float mint, float maxt, Counters *C) {
    uint32_t stack[128]; int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const BNode *n = &S->nodes[stack[--sp]];
        C->nodes++;
        if (!node_hit(n, ray, mint, maxt)) continue;
        if (n->count) {
            for (uint32_t i = n->first; i < n->first + n->count; ++i) {
                float u, v, t;
                C->tests++;
                if (prim_intersect(S, S->order[i], ray, mint, maxt, 1, &u, &v, &t)) return 1;
            }
        } else {
            stack[sp++] = n->right; stack[sp++] = n->left;
        }
    }
    return 0;
}

typedef struct {
    int valid;
    float t;
    V3 p, geoN, wi;
    Frame sh;
    int mesh; uint32_t tri;
    float u, v;   /* its.uv */
    float bu, bv; /* TriAccel barycentrics of the hit */
} Its;

/* ShapeKDTree::rayIntersect(ray, its) (skdtree.cpp:112-142) + fillIntersectionRecord<true>
 * (skdtree.h:343-429) */
static int kd_havran(const Scene *S, const uint32_t *nodes, const uint32_t *indices, const Ray *ray, float mint,
                     float maxt, int shadow, uint32_t *prim, float *tu, float *tv, float *tt);
static void scene_intersect(const Scene *S, const Ray *ray, Its *its, Counters *C) {
    float mint, maxt;
    its->valid = 0;
    its->t = INFINITY;
    C->rays++;
    if (!aabb_ray(S->aabbMin, S->aabbMax, ray, &mint, &maxt)) return;
    float rayMinT = ray->mint;
    if (rayMinT == EPSILON)
        rayMinT *= smax(smax(smax(fabsf(ray->o.x), fabsf(ray->o.y)), fabsf(ray->o.z)), EPSILON);
    if (rayMinT > mint) mint = rayMinT;
    if (ray->maxt < maxt) maxt = ray->maxt;
    if (!(maxt > mint)) return;
    uint32_t prim; float u, v, t;
    const int hit = g_kd_nodes ? kd_havran(S, g_kd_nodes, g_kd_indices, ray, mint, maxt, 0, &prim, &u, &v, &t)
                               : trace_closest(S, ray, mint, maxt, &prim, &u, &v, &t, C);
    if (g_trace_on)
        fprintf(stderr, "ORACLE_TRACE closest o %a %a %a d %a %a %a mint %a maxt %a (ray %a %a) -> %s prim %u t %a u %a v %a\n",
                ray->o.x, ray->o.y, ray->o.z, ray->d.x, ray->d.y, ray->d.z, mint, maxt, ray->mint, ray->maxt,
                hit ? "hit" : "miss", hit ? prim : 0u, hit ? t : 0.0f, hit ? u : 0.0f, hit ? v : 0.0f);
    if (!hit) return;
    const Mesh *m = &S->meshes[S->taMesh[prim]];
    uint32_t tri = S->taTri[prim];
    its->valid = 1; its->t = t; its->mesh = (int)S->taMesh[prim]; its->tri = tri;
    its->bu = u; its->bv = v;
    if (m->kind != MTSGPU_SHAPE_TRIMESH) { /* Shape::fillIntersectionRecord + skdtree.h:425-427 */
        V3 shN, dpdu;
        ana_fill(&m->ana, ray, t, u, v, &its->p, &its->geoN, &shN, &dpdu, &its->u, &its->v);
        compute_shading_frame(shN, dpdu, &its->sh);
        its->wi = to_local(&its->sh, vneg(ray->d));
        return;
    }
    const float bx = 1 - u - v, by = u, bz = v;
    const uint32_t i0 = m->idx[3 * tri], i1 = m->idx[3 * tri + 1], i2 = m->idx[3 * tri + 2];
    V3 p0 = m->pos[i0], p1 = m->pos[i1], p2 = m->pos[i2];
    its->p = vadd(vadd(vmul(p0, bx), vmul(p1, by)), vmul(p2, bz));
    V3 side1 = vsub(p1, p0), side2 = vsub(p2, p0);
    V3 faceNormal = vcross(side1, side2);
    float length = vlen(faceNormal);
    if (!vzero(faceNormal)) faceNormal = vdiv(faceNormal, length);
    V3 dpdu = m->dpdu ? m->dpdu[tri] : side1;
    V3 shN;
    if (m->nrm) {
        shN = vnormalize(vadd(vadd(vmul(m->nrm[i0], bx), vmul(m->nrm[i1], by)), vmul(m->nrm[i2], bz)));
        if (vdot(faceNormal, shN) < 0) faceNormal = vneg(faceNormal);
    } else {
        shN = faceNormal;
    }
    its->geoN = faceNormal;
    compute_shading_frame(shN, dpdu, &its->sh);
    its->wi = to_local(&its->sh, vneg(ray->d));
    if (m->uv) { /* skdtree.h:398-405 */
        its->u = m->uv[2 * i0] * bx + m->uv[2 * i1] * by + m->uv[2 * i2] * bz;
        its->v = m->uv[2 * i0 + 1] * bx + m->uv[2 * i1 + 1] * by + m->uv[2 * i2 + 1] * bz;
    } else {
        its->u = by; its->v = bz;
    }
}

/* ShapeKDTree::rayIntersect(ray) shadow variant (skdtree.cpp:207-226) */
static int scene_occluded(const Scene *S, const Ray *ray, Counters *C) {
    float mint, maxt;
    C->shadow++;
    if (!aabb_ray(S->aabbMin, S->aabbMax, ray, &mint, &maxt)) return 0;
    float rayMinT = ray->mint;
    if (rayMinT == EPSILON)
        rayMinT *= smax(smax(fabsf(ray->o.x), fabsf(ray->o.y)), fabsf(ray->o.z));
    if (rayMinT > mint) mint = rayMinT;
    if (ray->maxt < maxt) maxt = ray->maxt;
    if (!(maxt > mint)) return 0;
    if (g_kd_nodes) {
        uint32_t prim; float u, v, t;
        return kd_havran(S, g_kd_nodes, g_kd_indices, ray, mint, maxt, 1, &prim, &u, &v, &t);
    }
    const int occ = trace_any(S, ray, mint, maxt, C);
    if (g_trace_on)
        fprintf(stderr, "ORACLE_TRACE shadow o %a %a %a d %a %a %a mint %a maxt %a (ray %a %a) -> %d\n", ray->o.x, ray->o.y,
                ray->o.z, ray->d.x, ray->d.y, ray->d.z, mint, maxt, ray->mint, ray->maxt, occ);
    return occ;
}

/* ------------------------------------------------------------------------ */
/* direct emitter sampling                                                   */
/* ------------------------------------------------------------------------ */
typedef struct {
    V3 ref, refN, p, n, d;
    float dist, pdf;
    int measureSolidAngle;
    int emitter;
} DRec;

/* EnvironmentMap::sampleDirect (envmap.cpp:516-543) + internalSampleDirection (:567-603) */
/* ConstantBackgroundEmitter::sampleDirect (constant.cpp:167-214) */
static V3 const_sample_direct(const Env *E, DRec *dRec, float sx, float sy) {
    V3 d;
    float pdf;
    if (!vzero(dRec->refN)) {
        d = square_to_cosine_hemisphere(sx, sy);
        pdf = cosine_hemisphere_pdf(d);
        Frame F;
        F.n = dRec->refN;
        coordinate_system(F.n, &F.s, &F.t);
        d = to_world(&F, d);
    } else {
        float z = 1.0f - 2.0f * sy; /* warp::squareToUniformSphere (warp.cpp:25-31) */
        float r = safe_sqrt(1.0f - z * z);
        float sinPhi, cosPhi;
        o_sincos(2.0f * M_PI_F * sx, &sinPhi, &cosPhi);
        d = v3(r * cosPhi, r * sinPhi, z);
        pdf = 0.07957747154594766788f; /* INV_FOURPI */
    }
    float nearT, farT;
    dRec->pdf = 0.0f;
    if (!env_bsphere(E, dRec->ref, d, &nearT, &farT)) return v3(0, 0, 0);
    if (!(nearT < 0 && farT > 0)) return v3(0, 0, 0);
    dRec->p = vadd(dRec->ref, vmul(d, farT));
    dRec->n = vnormalize(vsub(E->center, dRec->p));
    dRec->measureSolidAngle = 1;
    dRec->d = d;
    dRec->dist = farT;
    dRec->pdf = pdf;
    if (!vzero(dRec->refN) && vdot(dRec->d, dRec->refN) <= 0) return v3(0, 0, 0);
    return vdiv(E->radiance, pdf);
}

static V3 env_sample_direct(const Env *E, DRec *dRec, float sx, float sy) {
    uint32_t row = env_sample_reuse(E->cdfRows, (uint32_t)E->h0, &sy);
    uint32_t col = env_sample_reuse(E->cdfCols + (size_t)row * (E->w0 + 1), (uint32_t)E->w0, &sx);
    float posx = (float)col + interval_to_tent(sx), posy = (float)row + interval_to_tent(sy);
    int xPos = (int)floorf(posx), yPos = (int)floorf(posy);
    float dx1 = posx - xPos, dx2 = 1.0f - dx1, dy1 = posy - yPos, dy2 = 1.0f - dy1;
    V3 value1 = vadd(vmul(vmul(env_texel(E, 0, xPos, yPos), dx2), dy2), vmul(vmul(env_texel(E, 0, xPos + 1, yPos), dx1), dy2));
    V3 value2 = vadd(vmul(vmul(env_texel(E, 0, xPos, yPos + 1), dx2), dy1), vmul(vmul(env_texel(E, 0, xPos + 1, yPos + 1), dx1), dy1));
    V3 value = vmul(vadd(value1, value2), E->scale);
    float pdf = (lum3(value1) * E->rowWeights[clampi(yPos, 0, E->h0 - 1)] +
                 lum3(value2) * E->rowWeights[clampi(yPos + 1, 0, E->h0 - 1)]) * E->normalization;
    float sinPhi, cosPhi, sinTheta, cosTheta;
    o_sincos(E->pixelX * (posx + 0.5f), &sinPhi, &cosPhi);
    o_sincos(E->pixelY * (posy + 0.5f), &sinTheta, &cosTheta);
    V3 d = v3(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
    pdf /= smax(fabsf(sinTheta), EPSILON);
    V3 dw = xf_vector(&E->toWorld, d);
    float nearT, farT;
    if (vzero(value) || pdf == 0 || !env_bsphere(E, dRec->ref, dw, &nearT, &farT) || nearT >= 0 || farT <= 0) {
        dRec->pdf = 0.0f;
        return v3(0, 0, 0);
    }
    dRec->pdf = pdf;
    dRec->p = vadd(dRec->ref, vmul(dw, farT));
    dRec->n = vnormalize(vsub(E->center, dRec->p));
    dRec->dist = farT;
    dRec->d = dw;
    dRec->measureSolidAngle = 1;
    return vdiv(value, pdf);
}

/* internalPdfDirection (envmap.cpp:606-633), called with trafo.inverse()(d) by pdfDirect (:545-556) */
static float env_pdf_direction(const Env *E, V3 dw) {
    V3 d = xf_vector(&E->toLocal, dw);
    float uvx = o_atan2(d.x, -d.z) * INV_TWOPI_F, uvy = safe_acosf(d.y) * INV_PI_F;
    if (!isfinite(uvx) || !isfinite(uvy)) return 0.0f;
    float u = uvx * E->w0 - 0.5f, v = uvy * E->h0 - 0.5f;
    int xPos = (int)floorf(u), yPos = (int)floorf(v);
    float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
    V3 value1 = vadd(vmul(vmul(env_texel(E, 0, xPos, yPos), dx2), dy2), vmul(vmul(env_texel(E, 0, xPos + 1, yPos), dx1), dy2));
    V3 value2 = vadd(vmul(vmul(env_texel(E, 0, xPos, yPos + 1), dx2), dy1), vmul(vmul(env_texel(E, 0, xPos + 1, yPos + 1), dx1), dy1));
    float sinTheta = safe_sqrt(1 - d.y * d.y);
    return (lum3(value1) * E->rowWeights[clampi(yPos, 0, E->h0 - 1)] + lum3(value2) * E->rowWeights[clampi(yPos + 1, 0, E->h0 - 1)])
           * E->normalization / smax(fabsf(sinTheta), EPSILON);
}

/* AreaLight::eval (area.cpp:104-109) */
static V3 its_Le(const Scene *S, const Its *its, V3 d) {
    const Emitter *e = &S->emitters[S->meshes[its->mesh].emitter];
    if (vdot(its->sh.n, d) <= 0) return v3(0, 0, 0);
    return e->radiance;
}

/* Scene::sampleEmitterDirect (scene.cpp:828-852) -> AreaLight::sampleDirect
 * (area.cpp:158-173) -> Shape::sampleDirect (shape.cpp:102-115) ->
 * TriMesh::samplePosition (trimesh.cpp:412-425) -> Triangle::sample (triangle.cpp:24-58) */
static V3 sample_emitter_direct(const Scene *S, DRec *dRec, float sx, float sy, Counters *C, int volpath) {
    V3 zero = v3(0, 0, 0);
    float emPdf;
    uint32_t index = dd_sample_reuse(S->emCdf, S->nemitters, &sx, &emPdf);
    const Emitter *e = &S->emitters[index];
    V3 value;
    if (e->type == MTSGPU_EMITTER_ENVMAP) {
        value = env_sample_direct(S->env, dRec, sx, sy);
    } else if (e->type == MTSGPU_EMITTER_CONSTANT) {
        value = const_sample_direct(S->env, dRec, sx, sy);
    } else if (S->meshes[e->mesh].kind != MTSGPU_SHAPE_TRIMESH) {
        ana_sample_direct(&S->meshes[e->mesh].ana, dRec->ref, sx, sy, &dRec->p, &dRec->n, &dRec->d, &dRec->dist,
                          &dRec->pdf);
        dRec->measureSolidAngle = 1;
        if (vdot(dRec->d, dRec->refN) >= 0 && vdot(dRec->d, dRec->n) < 0 && dRec->pdf != 0) { /* area.cpp:158-173 */
            value = vdiv(e->radiance, dRec->pdf);
        } else {
            dRec->pdf = 0.0f;
            value = zero;
        }
    } else {
    const Mesh *m = &S->meshes[e->mesh];
    /* samplePosition */
    float py = sy;
    uint32_t tri = dd_sample_reuse(m->areaCdf, m->nt, &py, NULL);
    V3 p0 = m->pos[m->idx[3 * tri]], p1 = m->pos[m->idx[3 * tri + 1]], p2 = m->pos[m->idx[3 * tri + 2]];
    float a = safe_sqrt(1.0f - sx);              /* warp::squareToUniformTriangle (warp.cpp:76-79) */
    float bx = 1 - a, by = a * py;
    V3 sideA = vsub(p1, p0), sideB = vsub(p2, p0);
    dRec->p = vadd(vadd(p0, vmul(sideA, bx)), vmul(sideB, by));
    if (m->nrm) {
        V3 n0 = m->nrm[m->idx[3 * tri]], n1 = m->nrm[m->idx[3 * tri + 1]], n2 = m->nrm[m->idx[3 * tri + 2]];
        dRec->n = vnormalize(vadd(vadd(vmul(n0, 1.0f - bx - by), vmul(n1, bx)), vmul(n2, by)));
    } else {
        dRec->n = vnormalize(vcross(sideA, sideB));
    }
    dRec->pdf = m->invArea;
    /* Shape::sampleDirect */
    dRec->d = vsub(dRec->p, dRec->ref);
    float distSquared = vlen2(dRec->d);
    dRec->dist = sqrtf(distSquared);
    dRec->d = vdiv(dRec->d, dRec->dist);
    float dp = vabsdot(dRec->d, dRec->n);
    dRec->pdf *= dp != 0 ? (distSquared / dp) : 0.0f;
    dRec->measureSolidAngle = 1;
    if (vdot(dRec->d, dRec->refN) >= 0 && vdot(dRec->d, dRec->n) < 0 && dRec->pdf != 0) {
        value = vdiv(e->radiance, dRec->pdf);
    } else {
        dRec->pdf = 0.0f;
        value = zero;
    }
    }
    if (dRec->pdf != 0) {
        Ray sray;
        sray.o = dRec->ref;
        ray_set_dir(&sray, dRec->d);
        sray.mint = EPSILON;
        sray.maxt = dRec->dist * (1 - SHADOW_EPSILON);
        sray.hasDiff = 0;
        const int env = e->type == MTSGPU_EMITTER_ENVMAP || e->type == MTSGPU_EMITTER_CONSTANT;
        if (volpath && (env || S->meshes[e->mesh].kind != MTSGPU_SHAPE_TRIMESH)) {
            /* Scene::sampleAttenuatedEmitterDirect -> evalTransmittance (scene.cpp:619-679, 876-898):
             * the segment to dRec.p (= ray(farT) for the environment, envmap.cpp:536, constant.cpp:254),
             * re-normalised; every supported emitter is EOnSurface (area.cpp, envmap.cpp:107,
             * constant.cpp:48), so lengthFactor = 1 - ShadowEpsilon on every segment (scene.cpp:624) */
            const V3 lp = env ? vadd(dRec->ref, vmul(dRec->d, dRec->dist)) : dRec->p;
            const V3 v = vsub(lp, dRec->ref);
            const float rem = sqrtf(vlen2(v));
            ray_set_dir(&sray, vdiv(v, rem));
            sray.maxt = rem * (1 - SHADOW_EPSILON);
        }
        if (scene_occluded(S, &sray, C)) return zero;
        dRec->emitter = (int)index;
        dRec->pdf *= emPdf;
        value = vdiv(value, emPdf);
        return value;
    }
    return zero;
}

/* Scene::pdfEmitterDirect (scene.cpp:949-952) -> AreaLight::pdfDirect (area.cpp:175-181)
 * -> Shape::pdfDirect (shape.cpp:117-126); pdfEmitterDiscrete (scene.h:848-850) */
static float pdf_emitter_direct(const Scene *S, const DRec *dRec) {
    const Emitter *e = &S->emitters[dRec->emitter];
    float pdf = 0.0f;
    if (e->type == MTSGPU_EMITTER_ENVMAP) {
        pdf = env_pdf_direction(S->env, dRec->d);
    } else if (e->type == MTSGPU_EMITTER_CONSTANT) { /* constant.cpp:216-231, solid angle */
        pdf = !vzero(dRec->refN) ? INV_PI_F * smax(0.0f, vdot(dRec->d, dRec->refN)) : 0.07957747154594766788f;
    } else if (vdot(dRec->d, dRec->refN) >= 0 && vdot(dRec->d, dRec->n) < 0) {
        const Mesh *m = &S->meshes[e->mesh];
        if (m->kind != MTSGPU_SHAPE_TRIMESH) {
            pdf = ana_pdf_direct(&m->ana, dRec->ref, dRec->d, dRec->n, dRec->dist);
        } else {
            float pdfPos = m->invArea;
            pdf = pdfPos * (dRec->dist * dRec->dist) / vabsdot(dRec->d, dRec->n);
        }
    }
    return pdf * (e->weight * S->emNorm);
}

static inline float mi_weight(float pdfA, float pdfB) { /* path.cpp:296-300 */
    pdfA *= pdfA; pdfB *= pdfB;
    return pdfA / (pdfA + pdfB);
}

/* ------------------------------------------------------------------------ */
/* MIPathTracer::Li (integrators/path/path.cpp:119-294)                      */
/* ------------------------------------------------------------------------ */
typedef struct { int maxDepth, rrDepth, strict, hide, hasAlpha, volpath; } PathParams;

static V3 Li(const Scene *S, const PathParams *P, Ray ray, Sampler *smp, float *alpha, int *depthOut, Counters *C) {
    Its its;
    V3 L = v3(0, 0, 0);
    int scattered = 0;
    int emitted = 1; /* RadianceQueryRecord::EEmittedRadiance, cleared after the first bounce */
    int depth = 1;
    scene_intersect(S, &ray, &its, C);       /* rRec.rayIntersect(ray) (records.inl:117-144) */
    *alpha = P->hasAlpha ? (its.valid ? 1.0f : 0.0f) : 1.0f;
    ray.mint = EPSILON;
    V3 throughput = v3(1.0f, 1.0f, 1.0f);
    float eta = 1.0f;
    while (depth <= P->maxDepth || P->maxDepth < 0) {
        if (!its.valid) {
            /* Scene::evalEnvironment (scene.h:910-913) with the camera ray's differentials */
            if (S->env && emitted && (!P->hide || scattered))
                L = vadd(L, vmulv(throughput, env_eval(S->env, &ray)));
            break;
        }
        const Bsdf *bsdf = &S->bsdfs[S->meshes[its.mesh].bsdf];
        int isEmitter = S->meshes[its.mesh].emitter >= 0;
        if (isEmitter && emitted && (!P->hide || scattered))
            L = vadd(L, vmulv(throughput, its_Le(S, &its, vneg(ray.d))));
        /* volpath.cpp:214-221 stops only for a strictly negative -dot(geoN, d) * cosTheta(wi) */
        const float snp = vdot(ray.d, its.geoN) * its.wi.z;
        if ((depth >= P->maxDepth && P->maxDepth > 0) || (P->strict && (P->volpath ? snp > 0 : snp >= 0)))
            break;

        DRec dRec;
        memset(&dRec, 0, sizeof dRec);
        dRec.ref = its.p;
        dRec.refN = (bsdf->flags & (E_TRANSMISSION | E_BACK)) == 0 ? its.sh.n : v3(0, 0, 0);
        if (bsdf->flags & E_SMOOTH) {
            float nx, ny;
            next2d(smp, &nx, &ny);
            V3 value = sample_emitter_direct(S, &dRec, nx, ny, C, P->volpath);
            if (!vzero(value)) {
                BRec bRec;
                bRec.wi = its.wi;
                bRec.wo = to_local(&its.sh, dRec.d);
                bRec.u = its.u; bRec.v = its.v;
                V3 bsdfVal = bsdf_eval(bsdf, &bRec);
                if (!vzero(bsdfVal) && (!P->strict || vdot(its.geoN, dRec.d) * bRec.wo.z > 0)) {
                    float bsdfPdf = dRec.measureSolidAngle ? bsdf_pdf(bsdf, &bRec) : 0;
                    float weight = mi_weight(dRec.pdf, bsdfPdf);
                    L = vadd(L, vmul(vmulv(vmulv(throughput, value), bsdfVal), weight));
                }
            }
        }

        float bsdfPdf;
        BRec bRec;
        bRec.wi = its.wi; bRec.eta = 1.0f; bRec.sampledType = 0; bRec.u = its.u; bRec.v = its.v;
        float bx, by;
        next2d(smp, &bx, &by);
        V3 bsdfWeight = bsdf_sample(bsdf, &bRec, &bsdfPdf, bx, by, smp);
        if (vzero(bsdfWeight)) break;
        scattered |= bRec.sampledType != E_NULL;
        const V3 wo = to_world(&its.sh, bRec.wo);
        float woDotGeoN = vdot(its.geoN, wo);
        if (P->strict && woDotGeoN * bRec.wo.z <= 0) break;

        int hitEmitter = 0;
        V3 value = v3(0, 0, 0);
        Ray nray;
        nray.o = its.p; ray_set_dir(&nray, wo); nray.mint = EPSILON; nray.maxt = INFINITY; nray.hasDiff = 0;
        ray = nray;
        scene_intersect(S, &ray, &its, C);
        if (its.valid) {
            if (S->meshes[its.mesh].emitter >= 0) {
                value = its_Le(S, &its, vneg(ray.d));
                /* DirectSamplingRecord::setQuery (records.inl:168-176) */
                dRec.p = its.p; dRec.n = its.sh.n; dRec.measureSolidAngle = 1;
                dRec.emitter = S->meshes[its.mesh].emitter; dRec.d = ray.d; dRec.dist = its.t;
                hitEmitter = 1;
            }
        } else {
            /* path.cpp:233-247; EnvironmentMap::fillDirectSamplingRecord (envmap.cpp:358-374) */
            float nearT, farT;
            if (!S->env || (P->hide && !scattered) || !env_bsphere(S->env, ray.o, ray.d, &nearT, &farT) ||
                nearT > 0 || farT < 0) {
                /* volpath.cpp:326-336: the miss still passes the RR step before the loop ends */
                if (P->volpath && depth++ >= P->rrDepth) (void)next1d(smp);
                break;
            }
            value = env_eval(S->env, &ray);
            dRec.p = ray_at(&ray, farT);
            dRec.n = vnormalize(vsub(S->env->center, dRec.p));
            dRec.measureSolidAngle = 1;
            dRec.emitter = S->envIndex;
            dRec.d = ray.d;
            dRec.dist = farT;
            hitEmitter = 1;
        }
        throughput = vmulv(throughput, bsdfWeight);
        eta *= bRec.eta;
        if (hitEmitter) {
            float lumPdf = !(bRec.sampledType & E_DELTA) ? pdf_emitter_direct(S, &dRec) : 0;
            L = vadd(L, vmul(vmulv(throughput, value), mi_weight(bsdfPdf, lumPdf)));
        }
        if (!its.valid) {
            if (P->volpath && depth++ >= P->rrDepth) (void)next1d(smp);
            break;
        }
        emitted = 0;
        if (depth++ >= P->rrDepth) {
            float q = smin(smaxc(throughput) * eta * eta, (float)0.95f);
            if (next1d(smp) >= q) break;
            throughput = vdiv(throughput, q);
        }
        if (smp->err) break;
    }
    *depthOut = depth;
    return L;
}

/* ------------------------------------------------------------------------ */
/* MIDirectIntegrator::Li (integrators/direct/direct.cpp:144-306), rRec.depth = 1 */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint32_t nLum, nBSDF;          /* m_emitterSamples, m_bsdfSamples */
    float weightLum, weightBSDF, fracLum, fracBSDF;
    uint32_t lumDim, bsdfDim;      /* first dimension of each requested 2D array */
} DirectParams;

static void direct_configure(uint32_t nLum, uint32_t nBSDF, DirectParams *D, Sampler *smp) { /* :128-143 */
    size_t sum = nLum + nBSDF;
    D->nLum = nLum; D->nBSDF = nBSDF;
    D->weightBSDF = 1 / (float)nBSDF;
    D->weightLum = 1 / (float)nLum;
    D->fracBSDF = nBSDF / (float)sum;
    D->fracLum = nLum / (float)sum;
    uint32_t dim = 5;
    if (nLum > 1) { D->lumDim = dim; dim += 2; }
    if (nBSDF > 1) { D->bsdfDim = dim; dim += 2; }
    smp->arrayEnd = dim;
}

static V3 Li_direct(const Scene *S, const PathParams *P, const DirectParams *D, Ray ray, Sampler *smp, float *alpha,
                    Counters *C) {
    Its its;
    V3 L = v3(0, 0, 0);
    scene_intersect(S, &ray, &its, C);
    *alpha = P->hasAlpha ? (its.valid ? 1.0f : 0.0f) : 1.0f;
    if (!its.valid) {
        if (S->env && !P->hide) return env_eval(S->env, &ray);
        return L;
    }
    if (S->meshes[its.mesh].emitter >= 0 && !P->hide) L = vadd(L, its_Le(S, &its, vneg(ray.d)));
    const Bsdf *bsdf = &S->bsdfs[S->meshes[its.mesh].bsdf];
    if (P->strict && vdot(ray.d, its.geoN) * its.wi.z >= 0) return L;

    /* emitter sampling */
    float u2[2];
    if (D->nLum <= 1) next2d(smp, &u2[0], &u2[1]);
    DRec dRec;
    memset(&dRec, 0, sizeof dRec);
    dRec.ref = its.p;
    dRec.refN = (bsdf->flags & (E_TRANSMISSION | E_BACK)) == 0 ? its.sh.n : v3(0, 0, 0);
    if (bsdf->flags & E_SMOOTH) {
        for (uint32_t i = 0; i < D->nLum; ++i) {
            float nx = u2[0], ny = u2[1];
            if (D->nLum > 1) sampler_array2d(smp, D->lumDim, D->nLum, i, &nx, &ny);
            V3 value = sample_emitter_direct(S, &dRec, nx, ny, C, 0);
            if (!vzero(value)) {
                BRec bRec;
                bRec.wi = its.wi;
                bRec.wo = to_local(&its.sh, dRec.d);
                bRec.u = its.u; bRec.v = its.v;
                V3 bsdfVal = bsdf_eval(bsdf, &bRec);
                if (!vzero(bsdfVal) && (!P->strict || vdot(its.geoN, dRec.d) * bRec.wo.z > 0)) {
                    float bsdfPdf = bsdf_pdf(bsdf, &bRec); /* emitter->isOnSurface(): all of ours */
                    float weight = mi_weight(dRec.pdf * D->fracLum, bsdfPdf * D->fracBSDF) * D->weightLum;
                    L = vadd(L, vmul(vmulv(value, bsdfVal), weight));
                }
            }
        }
    }

    /* BSDF sampling */
    if (D->nBSDF <= 1) next2d(smp, &u2[0], &u2[1]);
    for (uint32_t i = 0; i < D->nBSDF; ++i) {
        float bx = u2[0], by = u2[1];
        if (D->nBSDF > 1) sampler_array2d(smp, D->bsdfDim, D->nBSDF, i, &bx, &by);
        float bsdfPdf;
        BRec bRec;
        bRec.wi = its.wi; bRec.eta = 1.0f; bRec.sampledType = 0; bRec.u = its.u; bRec.v = its.v;
        V3 bsdfVal = bsdf_sample(bsdf, &bRec, &bsdfPdf, bx, by, smp);
        if (vzero(bsdfVal)) continue;
        const V3 wo = to_world(&its.sh, bRec.wo);
        float woDotGeoN = vdot(its.geoN, wo);
        if (P->strict && woDotGeoN * bRec.wo.z <= 0) continue;
        Ray bray;
        bray.o = its.p; ray_set_dir(&bray, wo); bray.mint = EPSILON; bray.maxt = INFINITY; bray.hasDiff = 0;
        Its bits;
        V3 value;
        scene_intersect(S, &bray, &bits, C);
        if (bits.valid) {
            if (S->meshes[bits.mesh].emitter < 0) continue;
            value = its_Le(S, &bits, vneg(bray.d));
            dRec.p = bits.p; dRec.n = bits.sh.n; dRec.measureSolidAngle = 1;
            dRec.emitter = S->meshes[bits.mesh].emitter; dRec.d = bray.d; dRec.dist = bits.t;
        } else {
            if (!S->env || (P->hide && bRec.sampledType == E_NULL)) continue;
            value = env_eval(S->env, &bray);
            float nearT, farT;
            if (!env_bsphere(S->env, bray.o, bray.d, &nearT, &farT) || nearT > 0 || farT < 0) continue;
            dRec.p = ray_at(&bray, farT);
            dRec.n = vnormalize(vsub(S->env->center, dRec.p));
            dRec.measureSolidAngle = 1;
            dRec.emitter = S->envIndex;
            dRec.d = bray.d;
            dRec.dist = farT;
        }
        float lumPdf = !(bRec.sampledType & E_DELTA) ? pdf_emitter_direct(S, &dRec) : 0;
        float weight = mi_weight(bsdfPdf * D->fracBSDF, lumPdf * D->fracLum) * D->weightBSDF;
        L = vadd(L, vmul(vmulv(value, bsdfVal), weight));
    }
    return L;
}

/* ------------------------------------------------------------------------ */
/* film: ImageBlock::put (render/imageblock.h:124-204) + rfilter LUT          */
/* (libcore/rfilter.cpp:37-55, rfilters/box.cpp, rfilters/gaussian.cpp)       */
/* ------------------------------------------------------------------------ */
typedef struct { float radius, scale; float values[FILTER_RES + 1]; int border; } Filter;

static int filter_configure(int type, float param, Filter *f) {
    float stddev = 0;
    if (type == MTSGPU_RFILTER_BOX) f->radius = param + 1e-5f;
    else if (type == MTSGPU_RFILTER_GAUSSIAN) { stddev = param; f->radius = 4 * stddev; }
    else return MTSGPU_EINVAL;
    if (!(f->radius > 0)) return MTSGPU_EINVAL;
    float sum = 0.0f;
    for (int i = 0; i < FILTER_RES; ++i) {
        float x = (f->radius * i) / FILTER_RES, value;
        if (type == MTSGPU_RFILTER_BOX) value = fabsf(x) <= f->radius ? 1.0f : 0.0f;
        else {
            float alpha = -1.0f / (2.0f * stddev * stddev);
            value = smax((float)0.0f, o_fastexp(alpha * x * x) - o_fastexp(alpha * f->radius * f->radius));
        }
        f->values[i] = value;
        sum += value;
    }
    f->values[FILTER_RES] = 0.0f;
    f->scale = FILTER_RES / f->radius;
    f->border = (int)ceilf(f->radius - 0.5f);
    sum *= 2 * f->radius / FILTER_RES;
    float normalization = 1.0f / sum;
    for (int i = 0; i < FILTER_RES; ++i) f->values[i] *= normalization;
    return MTSGPU_OK;
}
static inline float filter_eval_disc(const Filter *f, float x) {
    int i = (int)fabsf(x * f->scale);
    if (FILTER_RES < i) i = FILTER_RES;
    return f->values[i];
}

/* splat into the 32x32 block that renders pixel (px,py); own-pixel weight goes
 * to `own`, every other touched pixel to `spill` (film layout, border b) */
static int film_put(const Filter *f, int W, int H, int px, int py, float sx, float sy,
                    const float *val5, float *own, double *spill, int fw, int fh) {
    for (int i = 0; i < 5; ++i)
        if (!isfinite(val5[i]) || val5[i] < 0) return 0;
    const int b = f->border;
    const int bx = (px / BLOCK_SIZE) * BLOCK_SIZE, by = (py / BLOCK_SIZE) * BLOCK_SIZE;
    /* the block bitmap is allocated at blockSize + 2b even for partial blocks
       (renderproc.cpp:68-86 only resets the logical size) */
    const int bw = BLOCK_SIZE + 2 * b, bh = BLOCK_SIZE + 2 * b;
    (void)W; (void)H;
    const float posx = sx - 0.5f - (float)(bx - b), posy = sy - 0.5f - (float)(by - b);
    int minx = (int)ceilf(posx - f->radius), miny = (int)ceilf(posy - f->radius);
    int maxx = (int)floorf(posx + f->radius), maxy = (int)floorf(posy + f->radius);
    if (minx < 0) minx = 0;
    if (miny < 0) miny = 0;
    if (maxx > bw - 1) maxx = bw - 1;
    if (maxy > bh - 1) maxy = bh - 1;
    float wx[64], wy[64];
    for (int x = minx, i = 0; x <= maxx; ++x) wx[i++] = filter_eval_disc(f, x - posx);
    for (int y = miny, i = 0; y <= maxy; ++y) wy[i++] = filter_eval_disc(f, y - posy);
    for (int y = miny, yr = 0; y <= maxy; ++y, ++yr) {
        for (int x = minx, xr = 0; x <= maxx; ++x, ++xr) {
            const float weight = wx[xr] * wy[yr];
            int gx = x + bx, gy = y + by; /* film coordinates (border included) */
            if (gx >= fw || gy >= fh) continue; /* Bitmap::accumulate clips to the film */
            const int isOwn = gx == px + b && gy == py + b;
            if (isOwn) {
                float *dst = own + ((size_t)gy * fw + gx) * 5;
                for (int k = 0; k < 5; ++k) dst[k] += weight * val5[k];
            } else {
                /* pixels of other tasks: shared between OpenMP threads.  Summed in double
                   (the GPU's film_splat): exact, so independent of the order threads land */
                double *dst = spill + ((size_t)gy * fw + gx) * 5;
                for (int k = 0; k < 5; ++k) {
                    const double add = (double)(weight * val5[k]);
#ifdef _OPENMP
#pragma omp atomic
#endif
                    dst[k] += add;
                }
            }
        }
    }
    return 1;
}

/* ------------------------------------------------------------------------ */
/* gather mode (filters whose footprint covers neighbours: gaussian).  The    */
/* reference sums a pixel's splats in its block schedule's order (ImageBlock  */
/* ::put per block, Film::put as blocks finish, renderproc.cpp:142-149); the  */
/* GPU's film_gather (path_kernel.hip) and this restatement use one fixed     */
/* order instead: per film pixel, for each sample index j ascending, the      */
/* source pixels of the (2H+1)^2 neighbourhood in row-major order, each       */
/* adding weight * value[k] with film_put's footprint and weights.            */
/* ------------------------------------------------------------------------ */
#define GATHER_HMAX 4 /* the GPU's MTSG_GATHER_HMAX */
typedef struct { float v[4]; float sx, sy; int valid; } GatherRec;

static int gather_h(int rfilter, const Filter *f) {
    if (rfilter == MTSGPU_RFILTER_BOX) return 0;
    int H = (int)floorf(f->radius + 0.5f);
    if (H < f->border) H = f->border;
    return (H >= 1 && H <= GATHER_HMAX) ? H : 0;
}

/* the render loop's pixel predicate: window, row blocks or 8x8 tiles of this shard */
static int pixel_rendered(const mtsgpu_render_params *P, int qx, int qy) {
    const int lx = qx - (int)P->x0, ly = qy - (int)P->y0;
    if (lx < 0 || ly < 0 || lx >= (int)P->width || ly >= (int)P->height) return 0;
    const uint32_t rb = P->row_block ? P->row_block : 1, rs = P->row_stride ? P->row_stride : 1;
    if (P->flags & MTSGPU_FLAG_TILE_SHARD) {
        const uint32_t t = (uint32_t)(ly / 8) * ((P->width + 7) / 8) + (uint32_t)(lx / 8);
        return t % rs == P->row_phase;
    }
    return ((uint32_t)ly / rb) % rs == P->row_phase;
}

static void film_gather(const Filter *f, const mtsgpu_render_params *P, int fw, int fh, int H, const GatherRec *recs,
                        float *film) {
    const int b = f->border, bw = BLOCK_SIZE + 2 * b, bh = BLOCK_SIZE + 2 * b;
    const int gx0 = (int)P->x0 + b - H < 0 ? 0 : (int)P->x0 + b - H;
    const int gy0 = (int)P->y0 + b - H < 0 ? 0 : (int)P->y0 + b - H;
    const int gx1 = (int)(P->x0 + P->width) + b + H > fw ? fw : (int)(P->x0 + P->width) + b + H;
    const int gy1 = (int)(P->y0 + P->height) + b + H > fh ? fh : (int)(P->y0 + P->height) + b + H;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int gy = gy0; gy < gy1; ++gy) {
        for (int gx = gx0; gx < gx1; ++gx) {
            float *dst = film + ((size_t)gy * fw + gx) * 5;
            for (uint32_t j = 0; j < P->spp; ++j) {
                for (int dy = -H; dy <= H; ++dy) {
                    for (int dx = -H; dx <= H; ++dx) {
                        const int qx = gx - b + dx, qy = gy - b + dy;
                        if (!pixel_rendered(P, qx, qy)) continue;
                        const GatherRec *r = recs + (((size_t)(qy - (int)P->y0) * P->width + (size_t)(qx - (int)P->x0)) * P->spp + j);
                        if (!r->valid) continue;
                        /* film_put's footprint in the block bitmap of q's block */
                        const int bx = (qx / BLOCK_SIZE) * BLOCK_SIZE, by = (qy / BLOCK_SIZE) * BLOCK_SIZE;
                        const float posx = r->sx - 0.5f - (float)(bx - b), posy = r->sy - 0.5f - (float)(by - b);
                        int minx = (int)ceilf(posx - f->radius), miny = (int)ceilf(posy - f->radius);
                        int maxx = (int)floorf(posx + f->radius), maxy = (int)floorf(posy + f->radius);
                        if (minx < 0) minx = 0;
                        if (miny < 0) miny = 0;
                        if (maxx > bw - 1) maxx = bw - 1;
                        if (maxy > bh - 1) maxy = bh - 1;
                        const int x = gx - bx, y = gy - by;
                        if (x < minx || x > maxx || y < miny || y > maxy) continue;
                        const float weight = filter_eval_disc(f, x - posx) * filter_eval_disc(f, y - posy);
                        const float val5[5] = {r->v[0], r->v[1], r->v[2], r->v[3], 1.0f};
                        for (int k = 0; k < 5; ++k) dst[k] += weight * val5[k];
                    }
                }
            }
        }
    }
}

/* ------------------------------------------------------------------------ */
/* SamplingIntegrator::renderBlock (librender/integrator.cpp:140-188)        */
/* ------------------------------------------------------------------------ */
typedef struct {
    Scene *S;
    const PathParams *PP;
    const mtsgpu_render_params *P;
    int direct;
    float diffScale;
    const Filter *F;
    int W, H, fw, fh;
    float *film;
    double *spill;   /* neighbour splats, summed in double (film_put) */
    float *samples;
    GatherRec *recs; /* gather mode: each sample's value and position instead of a splat */
} RenderCtx;

/* one pixel's sampleCount samples: sampler->generate(offset), then per sample
 * next2D + sampleRayDifferential + Li + block->put + advance (integrator.cpp:
 * 165-186); rng: the SFMT replay stream (NULL: sobol / counter-based streams) */
static void render_pixel(const RenderCtx *R, long pi, int px, int py, Sfmt *rng, Counters *tot, uint64_t *pathLen,
                         uint64_t *nsamples, int *err) {
    const mtsgpu_render_params *P = R->P;
    Sampler smp;
    sampler_init(&smp, P->scramble, P->width, P->height);   /* crop size (integrator.cpp:37-41) */
    smp.indep = P->sampler != MTSGPU_SAMPLER_SOBOL;
    smp.rng = rng;
    DirectParams DP;
    memset(&DP, 0, sizeof DP);
    if (R->direct) direct_configure(P->emitter_samples, P->bsdf_samples, &DP, &smp); /* configureSampler */
    sampler_generate(&smp, px, py);
    Counters C = {0, 0, 0, 0};
    for (uint32_t j = 0; j < P->spp; ++j) {
        float ux, uy;
        next2d(&smp, &ux, &uy);
        const float sx = (float)px + ux, sy = (float)py + uy;
        Ray ray;
        camera_sample_ray(&R->S->cam, sx, sy, &ray);
        /* sensorRay.scaleDifferential(diffScaleFactor) (integrator.cpp:181, ray.h:163-168) */
        ray.rxO = vadd(ray.o, vmul(vsub(ray.rxO, ray.o), R->diffScale));
        ray.ryO = vadd(ray.o, vmul(vsub(ray.ryO, ray.o), R->diffScale));
        ray.rxD = vadd(ray.d, vmul(vsub(ray.rxD, ray.d), R->diffScale));
        ray.ryD = vadd(ray.d, vmul(vsub(ray.ryD, ray.d), R->diffScale));
        float alpha; int depth = 1;
        g_trace_on = px == g_trace_px && py == g_trace_py && (int)j == g_trace_j;
        if (g_trace_on) fprintf(stderr, "ORACLE_TRACE sample px %d py %d j %u\n", px, py, j);
        V3 L = R->direct ? Li_direct(R->S, R->PP, &DP, ray, &smp, &alpha, &C) : Li(R->S, R->PP, ray, &smp, &alpha, &depth, &C);
        if (smp.err) *err = 1;
        *pathLen += (uint64_t)depth; ++*nsamples;
        float val5[5] = {L.x, L.y, L.z, alpha, 1.0f};
        if (R->recs) {
            GatherRec *g = R->recs + ((size_t)pi * P->spp + j);
            g->valid = 1;
            for (int i = 0; i < 5; ++i)
                if (!isfinite(val5[i]) || val5[i] < 0) g->valid = 0;
            for (int i = 0; i < 4; ++i) g->v[i] = val5[i];
            g->sx = sx; g->sy = sy;
        } else {
            film_put(R->F, R->W, R->H, px, py, sx, sy, val5, R->film, R->spill, R->fw, R->fh);
        }
        if (R->samples) {
            float *rec = R->samples + ((size_t)pi * P->spp + j) * MTSGPU_SAMPLE_RECORD_FLOATS;
            rec[0] = L.x; rec[1] = L.y; rec[2] = L.z; rec[3] = alpha;
            rec[4] = sx; rec[5] = sy; rec[6] = (float)depth; rec[7] = smp.err ? 1.0f : 0.0f;
        }
        sampler_set_index(&smp, smp.sampleIndex + 1);
    }
#ifdef _OPENMP
#pragma omp atomic
#endif
    tot->rays += C.rays;
#ifdef _OPENMP
#pragma omp atomic
#endif
    tot->shadow += C.shadow;
#ifdef _OPENMP
#pragma omp atomic
#endif
    tot->tests += C.tests;
#ifdef _OPENMP
#pragma omp atomic
#endif
    tot->nodes += C.nodes;
}

int oracle_render(const mtsgpu_scene_desc *scene, const mtsgpu_render_params *P,
                  float *film, float *samples, mtsgpu_stats *stats, int libm_mode, int threads) {
    if (!g_sobol_ready) return MTSGPU_ESTATE;
    if (!scene || !P || !film) return MTSGPU_EINVAL;
    const int direct = P->integrator == MTSGPU_INTEGRATOR_DIRECT;
    if (P->integrator != MTSGPU_INTEGRATOR_PATH && P->integrator != MTSGPU_INTEGRATOR_VOLPATH && !direct) return MTSGPU_EINVAL;
    if (P->spp == 0 || (!direct && (P->rr_depth <= 0 || (P->max_depth <= 0 && P->max_depth != -1)))) return MTSGPU_EINVAL;
    if (direct && P->emitter_samples + P->bsdf_samples == 0) return MTSGPU_EINVAL;
    const int replay = P->sampler == MTSGPU_SAMPLER_SFMT_REPLAY || P->sampler == MTSGPU_SAMPLER_SFMT_BLOCKS;
    if (P->sampler < MTSGPU_SAMPLER_SOBOL || P->sampler > MTSGPU_SAMPLER_SFMT_BLOCKS) return MTSGPU_EINVAL;
    /* replay: the whole crop in the reference's block order; no sample arrays
       (IndependentSampler::generate would draw them per pixel first) */
    if (replay && (P->row_stride > 1 || direct))   /* path / volpath, as the GPU */
        return MTSGPU_EINVAL;
    g_cr = libm_mode;
    {
        const char *tr = getenv("ORACLE_TRACE");
        if (!tr || sscanf(tr, "%d,%d,%d", &g_trace_px, &g_trace_py, &g_trace_j) != 3) g_trace_px = g_trace_py = g_trace_j = -1;
    }
    Scene S;
    int rc = scene_configure(scene, &S);
    if (rc) { scene_free(&S); return rc; }
    Filter F;
    if ((rc = filter_configure(P->rfilter, P->rfilter_param, &F))) { scene_free(&S); return rc; }
    const int W = (int)scene->sensor.film_width, H = (int)scene->sensor.film_height;
    if (P->x0 + P->width > (uint32_t)W || P->y0 + P->height > (uint32_t)H) { scene_free(&S); return MTSGPU_EINVAL; }
    const int b = F.border, fw = W + 2 * b, fh = H + 2 * b;
    const size_t filmFloats = (size_t)fw * fh * 5;
    double *spill = (double *)calloc(filmFloats, sizeof(double));
    memset(film, 0, filmFloats * sizeof(float));
    PathParams PP = {P->max_depth, P->rr_depth, P->strict_normals, P->hide_emitters, P->has_alpha,
                     P->integrator == MTSGPU_INTEGRATOR_VOLPATH};
    const uint32_t rb = P->row_block ? P->row_block : 1, rs = P->row_stride ? P->row_stride : 1;
    Counters tot = {0, 0, 0, 0};
    uint64_t pathLen = 0, nsamples = 0;
    int err = 0;
    const int gh = gather_h(P->rfilter, &F);
    GatherRec *recs = gh ? (GatherRec *)calloc((size_t)P->width * P->height * P->spp, sizeof(GatherRec)) : NULL;
    if (gh && !recs) { free(spill); scene_free(&S); return MTSGPU_ENOMEM; }
    RenderCtx R = {&S, &PP, P, direct, 1.0f / sqrtf((float)P->spp), &F, W, H, fw, fh, film, spill, samples, recs};
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    if (replay) {
        /* the scene's IndependentSampler holds Random() = seed(5489) (random.cpp:473-489,
           random.h:113); RenderJob clones it once per worker in core order (renderjob.cpp:
           58-66), each clone seeded from the master's next 312 outputs.  SFMT_REPLAY: one
           worker (`mitsuba -p 1`) renders every block in order; SFMT_BLOCKS: block k of
           the spiral is rendered by clone k */
        const int bs = BLOCK_SIZE;
        const int nb = ((int)P->width + bs - 1) / bs * (((int)P->height + bs - 1) / bs);
        int *ord = (int *)malloc(sizeof(int) * 2 * (size_t)P->width * P->height);
        int *bstart = (int *)malloc(sizeof(int) * ((size_t)nb + 1));
        int nblocks = 0;
        oracle_render_order((int)P->width, (int)P->height, bs, ord, bstart, &nblocks);
        const int units = P->sampler == MTSGPU_SAMPLER_SFMT_BLOCKS ? nblocks : 1;
        Sfmt master;
        sfmt_init_gen_rand(&master, 5489ull);
        Sfmt *rngs = (Sfmt *)malloc(sizeof(Sfmt) * (size_t)units);
        for (int u = 0; u < units; ++u) sfmt_clone(&rngs[u], &master);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : pathLen, nsamples) reduction(| : err)
#endif
        for (int u = 0; u < units; ++u) {
            const int k0 = units == 1 ? 0 : bstart[u], k1 = units == 1 ? bstart[nblocks] : bstart[u + 1];
            for (int k = k0; k < k1; ++k) {
                const int lx = ord[2 * k], ly = ord[2 * k + 1];
                render_pixel(&R, (long)ly * P->width + lx, (int)P->x0 + lx, (int)P->y0 + ly, &rngs[u], &tot, &pathLen,
                             &nsamples, &err);
            }
        }
        free(rngs);
        free(bstart);
        free(ord);
    } else {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : pathLen, nsamples) reduction(| : err)
#endif
        for (long pi = 0; pi < (long)P->width * P->height; ++pi) {
            const int lx = (int)(pi % P->width), ly = (int)(pi / P->width);
            const int px = (int)P->x0 + lx, py = (int)P->y0 + ly;
            if (P->flags & MTSGPU_FLAG_TILE_SHARD) {   /* 8x8 tiles t % row_stride == row_phase */
                const uint32_t t = (uint32_t)(ly / 8) * ((P->width + 7) / 8) + (uint32_t)(lx / 8);
                if (t % rs != P->row_phase) continue;
            } else if (((uint32_t)(py - (int)P->y0) / rb) % rs != P->row_phase) continue;
            render_pixel(&R, pi, px, py, NULL, &tot, &pathLen, &nsamples, &err);
        }
    }
    if (recs) {
        film_gather(&F, P, fw, fh, gh, recs, film);
        free(recs);
    }
    for (size_t i = 0; i < filmFloats; ++i) film[i] += (float)spill[i];
    free(spill);
    if (stats) {
        memset(stats, 0, sizeof *stats);
        stats->samples = nsamples; stats->rays = tot.rays; stats->shadow_rays = tot.shadow;
        stats->path_length_sum = pathLen; stats->node_visits = tot.nodes; stats->tri_tests = tot.tests;
    }
    scene_free(&S);
    return err ? MTSGPU_EDIM : MTSGPU_OK;
}

/* ------------------------------------------------------------------------ */
/* unit-level probes                                                          */
/* ------------------------------------------------------------------------ */
/* the configured reconstruction filter (filter_configure): out = {radius, scale,
   border, values[0..FILTER_RES]} (tests restate the film's gather order with it) */
int oracle_filter(int type, float param, float *out) {
    Filter f;
    int rc = filter_configure(type, param, &f);
    if (rc) return rc;
    out[0] = f.radius; out[1] = f.scale; out[2] = (float)f.border;
    for (int i = 0; i <= FILTER_RES; ++i) out[3 + i] = f.values[i];
    return MTSGPU_OK;
}

int oracle_triaccel_load(const float *A, const float *B, const float *C, float *out10) {
    TriAccel ta;
    int r = triaccel_load(&ta, v3(A[0], A[1], A[2]), v3(B[0], B[1], B[2]), v3(C[0], C[1], C[2]));
    uint32_t k = ta.k; memcpy(&out10[0], &k, 4);
    out10[1] = ta.n_u; out10[2] = ta.n_v; out10[3] = ta.n_d; out10[4] = ta.a_u; out10[5] = ta.a_v;
    out10[6] = ta.b_nu; out10[7] = ta.b_nv; out10[8] = ta.c_nu; out10[9] = ta.c_nv;
    return r;
}
int oracle_triaccel_intersect(const float *t10, const float *o, const float *d, float mint, float maxt, float *uvt) {
    TriAccel ta; memcpy(&ta.k, &t10[0], 4);
    ta.n_u = t10[1]; ta.n_v = t10[2]; ta.n_d = t10[3]; ta.a_u = t10[4]; ta.a_v = t10[5];
    ta.b_nu = t10[6]; ta.b_nv = t10[7]; ta.c_nu = t10[8]; ta.c_nv = t10[9];
    Ray r; r.o = v3(o[0], o[1], o[2]); ray_set_dir(&r, v3(d[0], d[1], d[2]));
    return triaccel_intersect(&ta, &r, mint, maxt, &uvt[0], &uvt[1], &uvt[2]);
}
int oracle_camera(const mtsgpu_sensor_desc *s, float *m16, float *dxdy6) {
    Camera c;
    int rc = camera_configure(s, &c);
    if (rc) return rc;
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) m16[i * 4 + j] = c.sampleToCamera.m[i][j];
    dxdy6[0] = c.dx.x; dxdy6[1] = c.dx.y; dxdy6[2] = c.dx.z;
    dxdy6[3] = c.dy.x; dxdy6[4] = c.dy.y; dxdy6[5] = c.dy.z;
    return MTSGPU_OK;
}

/* one BSDF::sample(bRec, pdf, sample) with a replayable 1D sample u3[2]
 * (the FakeSampler of test_chisquare.cpp:58-88) */
/* the probes configure a BSDF once per distinct description (roughplastic
 * reduces its transmittance tables in configure) */
static mtsgpu_bsdf_desc g_probe_desc;
static Bsdf g_probe_bsdf;
static int g_probe_valid = 0;
static int probe_bsdf(const mtsgpu_bsdf_desc *bd, Bsdf *out) {
    if (bd->type == MTSGPU_BSDF_TWOSIDED) return MTSGPU_EINVAL; /* needs the scene's nested BSDFs */
    if (!g_probe_valid || memcmp(bd, &g_probe_desc, sizeof *bd) != 0) {
        if (g_probe_valid) bsdf_free(&g_probe_bsdf);
        g_probe_valid = 0;
        int rc = bsdf_configure(bd, &g_probe_bsdf);
        if (rc) return rc;
        g_probe_desc = *bd;
        g_probe_valid = 1;
    }
    *out = g_probe_bsdf;
    return MTSGPU_OK;
}

int oracle_bsdf_sample(const mtsgpu_bsdf_desc *bd, const float *wi3, const float *u3,
                       float *wo3, float *weight3, float *pdf, float *eta, int libm_mode) {
    g_cr = libm_mode;
    Bsdf b;
    int rc = probe_bsdf(bd, &b);
    if (rc) return rc;
    /* replay: a one-dimension Sobol index that returns u3[2] is not available,
     * so next1D is served from a tiny stub sampler */
    Sampler s; memset(&s, 0, sizeof s);
    BRec r; r.wi = v3(wi3[0], wi3[1], wi3[2]); r.eta = 1.0f; r.sampledType = 0; r.u = r.v = 0;
    V3 w;
    if (b.type == MTSGPU_BSDF_ROUGHDIELECTRIC) {
        /* emulate next1D() = u3[2] by sampling dimension 0 of index 0 -> 0.0 is
         * not general; instead evaluate the lobe choice explicitly */
        Distr d; distr_init(&d, b.distr, b.alphaU, b.alphaV, b.sampleVisible);
        (void)d;
        /* run the shared code with a sampler whose next1D returns u3[2]:
         * use a Sobol index 0 with scramble = u3[2] bits */
        uint32_t bits = (uint32_t)((double)u3[2] * 4294967296.0);
        s.scramble = bits; s.sobolIndex = 0; s.sampleIndex = 0; s.dim = 6; s.logRes = 0;
        w = bsdf_sample(&b, &r, pdf, u3[0], u3[1], &s);
    } else {
        w = bsdf_sample(&b, &r, pdf, u3[0], u3[1], &s);
    }
    wo3[0] = r.wo.x; wo3[1] = r.wo.y; wo3[2] = r.wo.z;
    weight3[0] = w.x; weight3[1] = w.y; weight3[2] = w.z;
    *eta = r.eta;
    return (int)r.sampledType;
}
/* The rough-transmittance integrand the reference's generator integrates
 * (rdielprec.cpp:40-56: roughdielectric's sample(bRec, sample) restricted to
 * ETransmission in EImportance mode, roughdielectric.cpp:424-511), computed
 * with this oracle's own microfacet, Fresnel and refraction functions, with
 * D(m)cos(m) sampling (sampleVisible = false) and optionally without Walter's
 * roughness scaling (the state the shipped tables were generated in).  Test
 * hook: tests/test_rtrans_pinning.py compares it with tools/rtrans_nd.c, whose
 * integrals reproduce the reference's data/microfacet/<distr>.dat. */
float oracle_rdiel_trans_weight(int type, float alpha, float eta, const float *wi3, float sx, float sy, int walter) {
    g_cr = 1;
    if (sx == 1) sx = 1 - EPSILON;
    if (sy == 1) sy = 1 - EPSILON;
    const V3 wi = v3(wi3[0], wi3[1], wi3[2]);
    const float a = smax(alpha, 1e-4f);
    const float avg = ((a + a) + a) * (1.0f / 3);   /* Spectrum::average of the constant texture */
    Distr d, sd;
    distr_init(&d, type, avg, avg, 0);
    sd = d;
    if (walter) distr_scale_alpha(&sd, 1.2f - 0.2f * sqrtf(fabsf(wi.z)));
    float pdf;
    const V3 m = distr_sample(&sd, vmul(wi, signumf(wi.z)), sx, sy, &pdf);
    if (pdf == 0) return 0.0f;
    float cosThetaT;
    const float F = fresnel_dielectric_ext(vdot(wi, m), &cosThetaT, eta);
    if (cosThetaT == 0) return 0.0f;
    const V3 wo = refract_v(wi, m, eta, cosThetaT);
    if (wi.z * wo.z >= 0) return 0.0f;
    return (1 - F) * fabsf(distr_eval(&d, m) * distr_G(&d, wi, wo, m) * vdot(wi, m) / (pdf * wi.z));
}

int oracle_bsdf_eval(const mtsgpu_bsdf_desc *bd, const float *wi3, const float *wo3,
                     float *value3, float *pdf, int libm_mode) {
    g_cr = libm_mode;
    Bsdf b;
    int rc = probe_bsdf(bd, &b);
    if (rc) return rc;
    BRec r; r.wi = v3(wi3[0], wi3[1], wi3[2]); r.wo = v3(wo3[0], wo3[1], wo3[2]); r.eta = 1; r.sampledType = 0;
    r.u = r.v = 0;
    V3 v = bsdf_eval(&b, &r);
    value3[0] = v.x; value3[1] = v.y; value3[2] = v.z;
    *pdf = bsdf_pdf(&b, &r);
    return MTSGPU_OK;
}

int oracle_configure(const mtsgpu_scene_desc *scene) {
    Scene S;
    int rc = scene_configure(scene, &S);
    scene_free(&S);
    return rc;
}

int oracle_env_tables(const mtsgpu_scene_desc *scene, float *params, uint16_t *texels, size_t texel_cap,
                      float *rows, float *cols, float *weights) {
    Scene S;
    int rc = scene_configure(scene, &S);
    if (rc || !S.env) { scene_free(&S); return rc ? rc : MTSGPU_EINVAL; }
    const Env *E = S.env;
    size_t total = 0;
    for (int l = 0; l < E->levels; ++l) total += (size_t)E->lw[l] * E->lh[l];
    if (params) {
        memset(params, 0, 64 * sizeof(float));
        params[0] = (float)E->levels; params[1] = (float)E->w0; params[2] = (float)E->h0;
        params[3] = E->normalization; params[4] = E->pixelX; params[5] = E->pixelY; params[6] = E->scale;
        params[7] = E->center.x; params[8] = E->center.y; params[9] = E->center.z; params[10] = E->radius;
        params[11] = (float)total;
        for (int l = 0; l < E->levels; ++l) { params[16 + l] = (float)E->lw[l]; params[34 + l] = (float)E->lh[l]; }
    }
    if (texels) {
        if (texel_cap < 4 * total) { scene_free(&S); return MTSGPU_EINVAL; }
        size_t k = 0;
        for (int l = 0; l < E->levels; ++l)
            for (size_t t = 0; t < (size_t)E->lw[l] * E->lh[l]; ++t) {
                texels[k++] = E->lv[l][3 * t]; texels[k++] = E->lv[l][3 * t + 1]; texels[k++] = E->lv[l][3 * t + 2]; texels[k++] = 0;
            }
    }
    if (rows) memcpy(rows, E->cdfRows, sizeof(float) * (E->h0 + 1));
    if (cols) memcpy(cols, E->cdfCols, sizeof(float) * (size_t)E->h0 * (E->w0 + 1));
    if (weights) memcpy(weights, E->rowWeights, sizeof(float) * E->h0);
    scene_free(&S);
    return MTSGPU_OK;
}

/* ShapeKDTree::rayIntersect(ray, its) probe (tests/test_oracle_kat.py, after
 * src/tests/test_dgeom.cpp:35-176): out16 = {valid, t, p[3], geoN[3], shN[3], shS[3], mesh, tri} */
/* the batch query of mtsgpu_trace_rays: rays n x {o, mint, d, maxt} -> n x {t, u, v, prim bits} */
int oracle_trace_rays(const mtsgpu_scene_desc *scene, const float *rays, uint32_t n, int shadow, float *hits) {
    Scene S;
    int rc = scene_configure(scene, &S);
    if (rc) { scene_free(&S); return rc; }
    #pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        const float *r = rays + 8 * i;
        Ray ray;
        memset(&ray, 0, sizeof ray);
        ray.o = v3(r[0], r[1], r[2]);
        ray_set_dir(&ray, v3(r[4], r[5], r[6]));
        ray.mint = r[3]; ray.maxt = r[7];
        Counters C = {0, 0, 0, 0};
        float *h = hits + 4 * i;
        if (shadow) {
            h[0] = scene_occluded(&S, &ray, &C) ? 1.0f : 0.0f; h[1] = h[2] = 0.0f; h[3] = 0.0f;
            uint32_t none = 0xffffffffu; memcpy(&h[3], &none, 4);
            continue;
        }
        Its its;
        scene_intersect(&S, &ray, &its, &C);
        uint32_t prim = 0xffffffffu;
        if (its.valid) {
            prim = S.meshes[its.mesh].primOffset + its.tri;
            h[0] = its.t; h[1] = its.bu; h[2] = its.bv;
        } else {
            h[0] = INFINITY; h[1] = h[2] = 0.0f;
        }
        memcpy(&h[3], &prim, 4);
    }
    scene_free(&S);
    return MTSGPU_OK;
}

/* SAHKDTree3D::rayIntersectHavran (sahkdtree3.h:178-308) over a given kd-tree
 * (KDNode words, gkdtree.h:453-601; the product's builder exports it through
 * mtsgpu_debug_kdtree), with the 8-entry hashed mailbox (:138-152) and
 * ShapeKDTree::intersect's TriAccel test on the global [mint, maxt] (a hit at
 * t == maxt is kept: the last of exactly tied triangles wins). */
static int kd_havran(const Scene *S, const uint32_t *nodes, const uint32_t *indices, const Ray *ray, float mint,
                     float maxt, int shadow, uint32_t *prim, float *tu, float *tv, float *tt) {
    typedef struct { uint32_t node; float t; uint32_t prev; float p[3]; } Ent;
    Ent stack[48];
    uint32_t mbox[8];
    memset(mbox, 0xFF, sizeof mbox);
    const float oa[3] = {ray->o.x, ray->o.y, ray->o.z}, da[3] = {ray->d.x, ray->d.y, ray->d.z};
    const float rcp[3] = {ray->dRcp.x, ray->dRcp.y, ray->dRcp.z};
    uint32_t enPt = 0, exPt = 1;
    stack[0].t = mint;
    for (int k = 0; k < 3; ++k) stack[0].p[k] = oa[k] + da[k] * mint;
    stack[1].t = maxt;
    for (int k = 0; k < 3; ++k) stack[1].p[k] = oa[k] + da[k] * maxt;
    stack[1].node = 0xffffffffu;
    int found = 0;
    uint32_t node = 0;
    while (node != 0xffffffffu) {
        while (!(nodes[2 * node] & 0x80000000u)) {
            const uint32_t comb = nodes[2 * node];
            float split;
            memcpy(&split, &nodes[2 * node + 1], 4);
            const int axis = (int)(comb & 3u);
            const uint32_t left = node + ((comb & ~(3u | 0x40000000u)) >> 2);
            uint32_t farChild;
            if (stack[enPt].p[axis] <= split) {
                if (stack[exPt].p[axis] <= split) { node = left; continue; }
                if (stack[enPt].p[axis] == split) { node = left + 1; continue; }
                node = left;
                farChild = left + 1;
            } else {
                if (split < stack[exPt].p[axis]) { node = left + 1; continue; }
                farChild = left;
                node = left + 1;
            }
            const float distToSplit = (split - oa[axis]) * rcp[axis];
            const uint32_t tmp = exPt++;
            if (exPt == enPt) ++exPt;
            if (exPt >= 48) return found;
            stack[exPt].prev = tmp;
            stack[exPt].t = distToSplit;
            stack[exPt].node = farChild;
            for (int k = 0; k < 3; ++k) stack[exPt].p[k] = oa[k] + da[k] * distToSplit;
            stack[exPt].p[axis] = split;
        }
        for (uint32_t e = nodes[2 * node] & 0x7fffffffu; e != nodes[2 * node + 1]; ++e) {
            const uint32_t p = indices[e];
            if (mbox[p & 7u] == p) continue;
            float u, v, t;
            if (triaccel_intersect(&S->ta[p], ray, mint, maxt, &u, &v, &t)) {
                if (shadow) return 1;
                maxt = t;
                found = 1;
                *prim = p; *tu = u; *tv = v; *tt = t;
            }
            mbox[p & 7u] = p;
        }
        if (stack[exPt].t > maxt) break;
        enPt = exPt;
        node = stack[exPt].node;
        exPt = stack[enPt].prev;
    }
    return found;
}

void oracle_set_kdtree(const uint32_t *nodes, const uint32_t *indices) {
    g_kd_nodes = nodes;
    g_kd_indices = indices;
}

/* oracle_trace_rays over a given kd-tree (ShapeKDTree::rayIntersect: scene
 * clip + adaptive epsilon as scene_intersect / scene_occluded, then Havran) */
int oracle_trace_rays_kd(const mtsgpu_scene_desc *scene, const uint32_t *nodes, const uint32_t *indices,
                         const float *rays, uint32_t n, int shadow, float *hits) {
    Scene S;
    int rc = scene_configure(scene, &S);
    if (rc) { scene_free(&S); return rc; }
    #pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        const float *r = rays + 8 * i;
        Ray ray;
        memset(&ray, 0, sizeof ray);
        ray.o = v3(r[0], r[1], r[2]);
        ray_set_dir(&ray, v3(r[4], r[5], r[6]));
        ray.mint = r[3]; ray.maxt = r[7];
        float *h = hits + 4 * i;
        uint32_t prim = 0xffffffffu;
        float mint, maxt, u = 0, v = 0, t = INFINITY;
        int hit = 0;
        if (aabb_ray(S.aabbMin, S.aabbMax, &ray, &mint, &maxt)) {
            float rayMinT = ray.mint;
            if (rayMinT == EPSILON)
                rayMinT *= shadow ? smax(smax(fabsf(ray.o.x), fabsf(ray.o.y)), fabsf(ray.o.z))
                                  : smax(smax(smax(fabsf(ray.o.x), fabsf(ray.o.y)), fabsf(ray.o.z)), EPSILON);
            if (rayMinT > mint) mint = rayMinT;
            if (ray.maxt < maxt) maxt = ray.maxt;
            if (maxt > mint) hit = kd_havran(&S, nodes, indices, &ray, mint, maxt, shadow, &prim, &u, &v, &t);
        }
        if (shadow) {
            h[0] = hit ? 1.0f : 0.0f; h[1] = h[2] = 0.0f;
            prim = 0xffffffffu;
        } else if (hit) {
            h[0] = t; h[1] = u; h[2] = v;
        } else {
            h[0] = INFINITY; h[1] = h[2] = 0.0f;
            prim = 0xffffffffu;
        }
        memcpy(&h[3], &prim, 4);
    }
    scene_free(&S);
    return MTSGPU_OK;
}

int oracle_intersect(const mtsgpu_scene_desc *scene, const float *o, const float *d, float *out16) {
    Scene S;
    int rc = scene_configure(scene, &S);
    if (rc) { scene_free(&S); return rc; }
    Ray ray;
    memset(&ray, 0, sizeof ray);
    ray.o = v3(o[0], o[1], o[2]);
    ray_set_dir(&ray, v3(d[0], d[1], d[2]));
    ray.mint = EPSILON; ray.maxt = INFINITY;
    Its its;
    Counters C = {0, 0, 0, 0};
    scene_intersect(&S, &ray, &its, &C);
    memset(out16, 0, 16 * sizeof(float));
    out16[0] = (float)its.valid;
    if (its.valid) {
        out16[1] = its.t;
        out16[2] = its.p.x; out16[3] = its.p.y; out16[4] = its.p.z;
        out16[5] = its.geoN.x; out16[6] = its.geoN.y; out16[7] = its.geoN.z;
        out16[8] = its.sh.n.x; out16[9] = its.sh.n.y; out16[10] = its.sh.n.z;
        out16[11] = its.sh.s.x; out16[12] = its.sh.s.y; out16[13] = its.sh.s.z;
        out16[14] = (float)its.mesh; out16[15] = (float)its.tri;
    }
    scene_free(&S);
    return MTSGPU_OK;
}
