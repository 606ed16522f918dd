// danalytic.h -- device side of the analytic shapes: rectangle, disk, sphere.
//
//   intersection   rectangle.cpp:125-153, disk.cpp:139-167, sphere.cpp:163-207
//                  (solveQuadraticDouble, util.cpp:487-525)
//   hit record     rectangle.cpp:155-167, disk.cpp:169-200, sphere.cpp:209-255,
//                  then ShapeKDTree::fillIntersectionRecord's shading frame
//                  (skdtree.h:425-427)
//   emitter        Shape::sampleDirect/pdfDirect (shape.cpp:102-126) over
//                  rectangle.cpp:210-220 / disk.cpp:247-259 samplePosition;
//                  Sphere::sampleDirect/pdfDirect (sphere.cpp:286-387)
//
// Per-shape constants (transforms, frame, 1/area) come from the host
// (scene_build.cpp:configure_analytic) in an MtsgAnalytic record.
#pragma once
#include "dmath.h"
#include "layout.h"

typedef const __attribute__((address_space(1))) MtsgAnalytic GAna;
typedef const __attribute__((address_space(1))) float gf32;

__device__ __forceinline__ f3 ana_ld3(gf32 *p) { return mk(p[0], p[1], p[2]); }

// Transform::transformAffine(const Point &) / operator()(const Vector &) / operator()(const Point &)
__device__ __forceinline__ f3 m_affine(gf32 *m, f3 p) {
    return mk(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3], m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
              m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]);
}
__device__ __forceinline__ f3 m_vec(gf32 *m, f3 v) {
    return mk(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z);
}
__device__ __forceinline__ f3 m_point(gf32 *m, f3 p) {
    const f3 r = m_affine(m, p);
    const float w = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (w == 1.0f) return r;
    return divs(r, w);
}

// coordinateSystem (util.cpp:592-601)
__device__ __forceinline__ void coordinate_system(f3 a, f3 &b, f3 &c) {
    if (fabsf(a.x) > fabsf(a.y)) {
        const float invLen = 1.0f / dsqrt(a.x * a.x + a.z * a.z);
        c = mk(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        const float invLen = 1.0f / dsqrt(a.y * a.y + a.z * a.z);
        c = mk(0.0f, a.z * invLen, -a.y * invLen);
    }
    b = cross(c, a);
}

// warp::squareToUniformDiskConcentric (warp.cpp:81-102)
__device__ __forceinline__ void square_to_disk_concentric(float sx, float sy, float &px, float &py) {
    const float r1 = 2.0f * sx - 1.0f, r2 = 2.0f * sy - 1.0f;
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
    px = r * c;
    py = r * s;
}

// solveQuadraticDouble (util.cpp:487-525)
__device__ __forceinline__ bool solve_quadratic_d(double a, double b, double c, double &x0, double &x1) {
    if (a == 0) {
        if (b != 0) { x0 = x1 = -c / b; return true; }
        return false;
    }
    const double discrim = b * b - 4.0f * a * c;
    if (discrim < 0) return false;
    const double sqrtDiscrim = __builtin_sqrt(discrim);
    const double temp = (b < 0) ? -0.5f * (b - sqrtDiscrim) : -0.5f * (b + sqrtDiscrim);
    x0 = temp / a;
    x1 = c / temp;
    if (x0 > x1) { const double t = x0; x0 = x1; x1 = t; }
    return true;
}
// solveQuadratic (util.cpp:447-485), single precision
__device__ __forceinline__ bool solve_quadratic_f(float a, float b, float c, float &x0, float &x1) {
    if (a == 0) {
        if (b != 0) { x0 = x1 = -c / b; return true; }
        return false;
    }
    const float discrim = b * b - 4.0f * a * c;
    if (discrim < 0) return false;
    const float sqrtDiscrim = dsqrt(discrim);
    const float temp = (b < 0) ? -0.5f * (b - sqrtDiscrim) : -0.5f * (b + sqrtDiscrim);
    x0 = temp / a;
    x1 = c / temp;
    if (x0 > x1) { const float t = x0; x0 = x1; x1 = t; }
    return true;
}


// Shape::rayIntersect(ray, mint, maxt, t, temp) (closest) / rayIntersect(ray, mint, maxt)
// (ANY); (lx, ly) = the rectangle's / disk's object-space hit (the `temp` data)
template <bool ANY>
__device__ __forceinline__ bool ana_intersect(GAna &a, f3 o, f3 d, float mint, float maxt, float &t, float &lx,
                                              float &ly) {
    if (a.type == MTSG_SHAPE_SPHERE) {
        const double ox = (double)o.x - (double)a.center[0], oy = (double)o.y - (double)a.center[1],
                     oz = (double)o.z - (double)a.center[2];
        const double dx = d.x, dy = d.y, dz = d.z;
        const double A = dx * dx + dy * dy + dz * dz;
        const double B = 2 * (ox * dx + oy * dy + oz * dz);
        const float r2 = a.radius * a.radius;
        const double C = (ox * ox + oy * oy + oz * oz) - (double)r2;
        double nearT, farT;
        if (!solve_quadratic_d(A, B, C, nearT, farT)) return false;
        if (ANY) {   // sphere.cpp:189-207
            if (nearT > maxt || farT < mint) return false;
            if (nearT < mint && farT > maxt) return false;
            return true;
        }
        if (!(nearT <= maxt && farT >= mint)) return false;
        if (nearT < mint) {
            if (farT > maxt) return false;
            t = (float)farT;
        } else {
            t = (float)nearT;
        }
        lx = ly = 0.0f;
        return true;
    }
    // rectangle / disk: m_worldToObject.transformAffine(ray), plane z = 0
    gf32 *W = a.to_obj;
    const f3 ro = m_affine(W, o), rd = m_vec(W, d);
    const float hit = -ro.z / rd.z;
    if (!(hit >= mint && hit <= maxt)) return false;
    const float px = ro.x + rd.x * hit, py = ro.y + rd.y * hit;
    const bool inside = (a.type == MTSG_SHAPE_RECTANGLE) ? (fabsf(px) <= 1 && fabsf(py) <= 1)
                                                           : (px * px + py * py <= 1);
    if (!inside) return false;
    t = hit;
    lx = px;
    ly = py;
    return true;
}

// the plugin's fillIntersectionRecord + the kd-tree's shading frame: position,
// geometric / shading normal, dpdu and uv of a hit at distance t
struct AnaHit { f3 p, geoN, shN, dpdu; float u, v; };
__device__ __forceinline__ AnaHit ana_fill(GAna &a, f3 o, f3 d, float t, float lx, float ly) {
    AnaHit h;
    h.p = add(o, mul(d, t));   // ray(its.t)
    if (a.type == MTSG_SHAPE_RECTANGLE) {
        h.geoN = h.shN = ana_ld3(a.n);
        h.dpdu = ana_ld3(a.dpdu);
        h.u = 0.5f * (lx + 1);
        h.v = 0.5f * (ly + 1);
    } else if (a.type == MTSG_SHAPE_DISK) {
        const float r = dsqrt(lx * lx + ly * ly), invR = (r == 0) ? 0.0f : (1.0f / r);
        float phi = d_atan2(ly, lx);
        if (phi < 0) phi += 2 * D_PI;
        const float cosPhi = lx * invR, sinPhi = ly * invR;
        h.dpdu = (r != 0) ? m_vec(a.to_world, mk(cosPhi, sinPhi, 0)) : m_vec(a.to_world, mk(1, 0, 0));
        // the plugin sets only shFrame.n; its geometric frame keeps the record's previous
        // contents (disk.cpp:186-198): the shading normal stands in for it
        h.geoN = h.shN = ana_ld3(a.n);
        h.u = r;
        h.v = phi * D_INV_TWOPI;
    } else {
        const f3 c = ana_ld3(a.center);
        h.p = add(c, mul(normalize(sub(h.p, c)), a.radius));   // SINGLE_PRECISION re-projection
        const f3 local = m_vec(a.to_obj, sub(h.p, c));
        const float theta = d_acos(smin(1.0f, smax(-1.0f, local.z / a.radius)));   // math::safe_acos
        float phi = d_atan2(local.y, local.x);
        if (phi < 0) phi += 2 * D_PI;
        h.u = phi * (0.5f * D_INV_PI);
        h.v = theta * D_INV_PI;
        const float tp = 2 * D_PI;
        h.dpdu = m_vec(a.to_world, mk(-local.y * tp, local.x * tp, 0 * tp));
        f3 n = normalize(sub(h.p, c));
        if (a.flip) n = mul(n, -1.0f);
        h.geoN = h.shN = n;
        (void)theta;
    }
    return h;
}

struct AnaSample { f3 p, n, d; float dist, pdf; };

// AreaLight::sampleDirect's m_shape->sampleDirect(dRec, sample) for an analytic shape
__device__ __forceinline__ AnaSample ana_sample_direct(GAna &a, f3 ref, float sx, float sy) {
    AnaSample r;
    if (a.type == MTSG_SHAPE_SPHERE) {   // sphere.cpp:286-355
        const f3 c = ana_ld3(a.center);
        const f3 refToCenter = sub(c, ref);
        const float refDist2 = len2(refToCenter);
        const float invRefDist = 1.0f / dsqrt(refDist2);
        const float sinAlpha = a.radius * invRefDist;
        if (sinAlpha < 1 - D_EPSILON) {
            const float cosAlpha = safe_sqrt(1.0f - sinAlpha * sinAlpha);
            Frame F;
            F.n = mul(refToCenter, invRefDist);
            coordinate_system(F.n, F.s, F.t);
            // warp::squareToUniformCone (warp.cpp:54-63)
            const float cosTheta = (1 - sx) + sx * cosAlpha;
            const float sinTheta = safe_sqrt(1.0f - cosTheta * cosTheta);
            float sinPhi, cosPhi;
            d_sincos(2.0f * D_PI * sy, &sinPhi, &cosPhi);
            r.d = to_world(F, mk(cosPhi * sinTheta, sinPhi * sinTheta, cosTheta));
            r.pdf = D_INV_TWOPI / (1 - cosAlpha);
            const float projDist = dot(refToCenter, r.d);
            const float baseT = refDist2 / projDist;
            const f3 query = add(ref, mul(r.d, baseT));
            const f3 queryToCenter = sub(c, query);
            const float queryDist2 = len2(queryToCenter);
            const float queryProjDist = dot(queryToCenter, r.d);
            const float A = 1.0f, B = -2 * queryProjDist, C = queryDist2 - a.radius * a.radius;
            float nearT, farT;
            if (!solve_quadratic_f(A, B, C, nearT, farT)) nearT = queryProjDist;
            r.dist = baseT + nearT;
            r.n = normalize(sub(mul(r.d, nearT), queryToCenter));
            r.p = add(c, mul(r.n, a.radius));
        } else {
            // warp::squareToUniformSphere (warp.cpp:25-31)
            const float z = 1.0f - 2.0f * sy;
            const float rr = safe_sqrt(1.0f - z * z);
            float sinPhi, cosPhi;
            d_sincos(2.0f * D_PI * sx, &sinPhi, &cosPhi);
            const f3 dv = mk(rr * cosPhi, rr * sinPhi, z);
            r.p = add(c, mul(dv, a.radius));
            r.n = dv;
            r.d = sub(r.p, ref);
            const float dist2 = len2(r.d);
            r.dist = dsqrt(dist2);
            r.d = divs(r.d, r.dist);
            r.pdf = a.inv_area * dist2 / absdot(r.d, r.n);
        }
        if (a.flip) r.n = mul(r.n, -1.0f);
        return r;
    }
    // samplePosition (rectangle.cpp:210-216, disk.cpp:247-255), then Shape::sampleDirect (shape.cpp:102-115)
    if (a.type == MTSG_SHAPE_RECTANGLE) {
        r.p = m_point(a.to_world, mk(sx * 2 - 1, sy * 2 - 1, 0));
    } else {
        float px, py;
        square_to_disk_concentric(sx, sy, px, py);
        r.p = m_point(a.to_world, mk(px, py, 0));
    }
    r.n = ana_ld3(a.n);
    r.pdf = a.inv_area;
    r.d = sub(r.p, ref);
    const float distSquared = len2(r.d);
    r.dist = dsqrt(distSquared);
    r.d = divs(r.d, r.dist);
    const float dp = absdot(r.d, r.n);
    r.pdf *= dp != 0 ? (distSquared / dp) : 0.0f;
    return r;
}

// Shape::pdfDirect in solid angle (shape.cpp:117-126; Sphere: sphere.cpp:357-387)
// for the emitter hit at distance `dist` along d with normal n, seen from `ref`
__device__ __forceinline__ float ana_pdf_direct(GAna &a, f3 ref, f3 d, f3 n, float dist) {
    if (a.type == MTSG_SHAPE_SPHERE) {
        const f3 refToCenter = sub(ana_ld3(a.center), ref);
        const float invRefDist = (float)1.0f / len(refToCenter);
        const float sinAlpha = a.radius * invRefDist;
        if (sinAlpha < 1 - D_EPSILON) {
            const float cosAlpha = safe_sqrt(1 - sinAlpha * sinAlpha);
            return D_INV_TWOPI / (1 - cosAlpha);
        }
        return a.inv_area * dist * dist / absdot(d, n);
    }
    return a.inv_area * (dist * dist) / absdot(d, n);
}
