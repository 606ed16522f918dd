// scene_build.cpp -- host configure() for the MI355X path integrator.
//
// Derives, from the scene description of include/mtsgpu.h, everything the
// reference computes in its configure()/initialize() steps, then lays it out
// for HBM (layout.h):
//   camera        librender/sensor.cpp:95-107,239-305, sensors/perspective.cpp:126-163
//   BSDFs         bsdfs/diffuse.cpp:75-101, roughconductor.cpp:168-240,
//                 roughdielectric.cpp:183-256, librender/bsdf.cpp:88-113
//   meshes        TriMesh::configure / computeNormals / computeUVTangents /
//                 prepareSamplingTable (librender/trimesh.cpp:361-739)
//   default BSDFs Shape::configure (librender/shape.cpp:48-75)
//   emitter PDF   Scene::initialize (librender/scene.cpp:376-381)
//   TriAccel      skdtree.cpp:74-109, render/triaccel.h:58-90
//   scene bounds  gkdtree.h:996-1001,1211-1217 (MTS_KD_AABB_EPSILON)
// The acceleration structure is a binned-SAH BVH2 instead of the reference's
// SAH kd-tree: traversal returns the same closest hit.
#include "scene_build.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "sobol_params.inc"

namespace {

inline float fmax_std(float a, float b) { return (a < b) ? b : a; }   // std::max
inline float fmin_std(float a, float b) { return (b < a) ? b : a; }   // std::min

struct V { float x, y, z; };
inline V v(float x, float y, float z) { V r = {x, y, z}; return r; }
inline V operator+(V a, V b) { return v(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V operator-(V a, V b) { return v(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V operator*(V a, float f) { return v(a.x * f, a.y * f, a.z * f); }
inline V vdiv(V a, float f) { float r = 1.0f / f; return a * r; }
inline float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V cross(V a, V b) { return v((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)); }
inline float length(V a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline V normalize(V a) { return vdiv(a, length(a)); }
inline float at(V a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
inline float avg3(float a) { float r = 0.0f; r += a; r += a; r += a; return r * (1.0f / 3); }   // Spectrum::average

const float kPi = 3.14159265358979323846f;

// ---- 4x4 transforms (core/matrix.h:744-756, matrix.inl:138-193, transform.cpp) ----
struct M4 { float m[4][4]; };
M4 mul(const M4 &a, const M4 &b) {
    M4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float sum = 0;
            for (int k = 0; k < 4; ++k) sum += a.m[i][k] * b.m[k][j];
            r.m[i][j] = sum;
        }
    return r;
}
bool invert(const M4 &src, M4 &t) {
    int indxc[4], indxr[4], ipiv[4] = {0, 0, 0, 0};
    t = src;
    for (int i = 0; i < 4; i++) {
        int irow = -1, icol = -1;
        float big = 0;
        for (int j = 0; j < 4; j++)
            if (ipiv[j] != 1)
                for (int k = 0; k < 4; k++) {
                    if (ipiv[k] == 0) {
                        if (std::fabs(t.m[j][k]) >= big) { big = std::fabs(t.m[j][k]); irow = j; icol = k; }
                    } else if (ipiv[k] > 1) {
                        return false;
                    }
                }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) std::swap(t.m[irow][k], t.m[icol][k]);
        indxr[i] = irow; indxc[i] = icol;
        if (t.m[icol][icol] == 0) return false;
        float pivinv = 1.f / t.m[icol][icol];
        t.m[icol][icol] = 1.f;
        for (int j = 0; j < 4; j++) t.m[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++)
            if (j != icol) {
                float save = t.m[j][icol];
                t.m[j][icol] = 0;
                for (int k = 0; k < 4; k++) t.m[j][k] -= t.m[icol][k] * save;
            }
    }
    for (int j = 3; j >= 0; j--)
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) std::swap(t.m[k][indxr[j]], t.m[k][indxc[j]]);
    return true;
}
struct Xf { M4 t, inv; };
M4 diag(float a, float b, float c, float d) {
    M4 r; std::memset(&r, 0, sizeof r);
    r.m[0][0] = a; r.m[1][1] = b; r.m[2][2] = c; r.m[3][3] = d;
    return r;
}
Xf compose(const Xf &a, const Xf &b) { return Xf{mul(a.t, b.t), mul(b.inv, a.inv)}; }
Xf scale(float x, float y, float z) { return Xf{diag(x, y, z, 1), diag(1.0f / x, 1.0f / y, 1.0f / z, 1)}; }
Xf translate(float x, float y, float z) {
    Xf r{diag(1, 1, 1, 1), diag(1, 1, 1, 1)};
    r.t.m[0][3] = x; r.t.m[1][3] = y; r.t.m[2][3] = z;
    r.inv.m[0][3] = -x; r.inv.m[1][3] = -y; r.inv.m[2][3] = -z;
    return r;
}
inline float deg2rad(float x) { return x * (kPi / 180.0f); }
inline float rad2deg(float x) { return x * (180.0f / kPi); }
V xf_point(const M4 &m, V p) {
    float x = m.m[0][0] * p.x + m.m[0][1] * p.y + m.m[0][2] * p.z + m.m[0][3];
    float y = m.m[1][0] * p.x + m.m[1][1] * p.y + m.m[1][2] * p.z + m.m[1][3];
    float z = m.m[2][0] * p.x + m.m[2][1] * p.y + m.m[2][2] * p.z + m.m[2][3];
    float w = m.m[3][0] * p.x + m.m[3][1] * p.y + m.m[3][2] * p.z + m.m[3][3];
    if (w == 1.0f) return v(x, y, z);
    return vdiv(v(x, y, z), w);
}

V xf_vec(const M4 &m, V a) {          // Transform::operator()(const Vector &) (transform.h:175-183)
    return v(m.m[0][0] * a.x + m.m[0][1] * a.y + m.m[0][2] * a.z, m.m[1][0] * a.x + m.m[1][1] * a.y + m.m[1][2] * a.z,
             m.m[2][0] * a.x + m.m[2][1] * a.y + m.m[2][2] * a.z);
}
V xf_normal(const M4 &inv, V a) {     // Transform::operator()(const Normal &) (transform.h:203-211)
    return v(inv.m[0][0] * a.x + inv.m[1][0] * a.y + inv.m[2][0] * a.z,
             inv.m[0][1] * a.x + inv.m[1][1] * a.y + inv.m[2][1] * a.z,
             inv.m[0][2] * a.x + inv.m[1][2] * a.y + inv.m[2][2] * a.z);
}
void put3(float *d, V a) { d[0] = a.x; d[1] = a.y; d[2] = a.z; }
void put16(float *d, const M4 &m) { std::memcpy(d, &m.m[0][0], 16 * sizeof(float)); }

// 'toWorld' of a shape desc as the reference's Transform (matrix + carried inverse)
int desc_transform(const float *t16, const float *inv16, Xf &out, std::string &err) {
    std::memcpy(&out.t.m[0][0], t16, 16 * sizeof(float));
    bool haveInv = false;
    for (int i = 0; i < 16; ++i) haveInv |= inv16[i] != 0.0f;
    if (haveInv) std::memcpy(&out.inv.m[0][0], inv16, 16 * sizeof(float));
    else if (!invert(out.t, out.inv)) { err = "Singular matrix in Matrix::invert"; return MTSGPU_EINVAL; }
    return MTSGPU_OK;
}

// Rectangle / Disk / Sphere constructors + configure() (rectangle.cpp:80-119,
// disk.cpp:83-130, sphere.cpp:108-133) and getAABB()
int configure_analytic(const mtsgpu_mesh_desc &m, MtsgAnalytic &a, float lo[3], float hi[3], std::string &err) {
    std::memset(&a, 0, sizeof a);
    a.type = m.shape_type;
    Xf o2w;
    int rc;
    auto grow = [&](V p) {
        const float q[3] = {p.x, p.y, p.z};
        for (int i = 0; i < 3; ++i) { lo[i] = std::min(lo[i], q[i]); hi[i] = std::max(hi[i], q[i]); }
    };
    for (int i = 0; i < 3; ++i) { lo[i] = FLT_MAX; hi[i] = -FLT_MAX; }
    if (m.shape_type == MTSGPU_SHAPE_RECTANGLE || m.shape_type == MTSGPU_SHAPE_DISK) {
        if ((rc = desc_transform(m.to_world, m.to_world_inv, o2w, err))) return rc;
        if (m.flip_normals) o2w = compose(o2w, scale(1, 1, -1));   // (prependScale: m_transform * scale)
        if (m.shape_type == MTSGPU_SHAPE_RECTANGLE) {
            const V dpdu = xf_vec(o2w.t, v(2, 0, 0)), dpdv = xf_vec(o2w.t, v(0, 2, 0));
            const V n = normalize(xf_normal(o2w.inv, v(0, 0, 1)));
            put3(a.dpdu, dpdu); put3(a.dpdv, dpdv); put3(a.n, n);
            put3(a.fs, normalize(dpdu)); put3(a.ft, normalize(dpdv));
            a.inv_area = 1.0f / (length(dpdu) * length(dpdv));
            if (std::fabs(dot(normalize(dpdu), normalize(dpdv))) > 1e-4f) {
                err = "Error: 'toWorld' transformation contains shear!"; return MTSGPU_EINVAL;
            }
            grow(xf_point(o2w.t, v(-1, -1, 0))); grow(xf_point(o2w.t, v(1, -1, 0)));
            grow(xf_point(o2w.t, v(1, 1, 0))); grow(xf_point(o2w.t, v(-1, 1, 0)));
        } else {
            const V dpdu = xf_vec(o2w.t, v(1, 0, 0)), dpdv = xf_vec(o2w.t, v(0, 1, 0));
            if (std::fabs(dot(normalize(dpdu), normalize(dpdv))) > 1e-3f) {
                err = "Error: 'toWorld' transformation contains shear!"; return MTSGPU_EINVAL;
            }
            if (std::fabs(length(dpdu) / length(dpdv) - 1) > 1e-3f) {
                err = "Error: 'toWorld' transformation contains a non-uniform scale!"; return MTSGPU_EINVAL;
            }
            a.inv_area = 1.0f / (kPi * length(dpdu) * length(dpdu));
            put3(a.n, normalize(xf_normal(o2w.inv, v(0, 0, 1))));
            grow(xf_point(o2w.t, v(1, 0, 0))); grow(xf_point(o2w.t, v(-1, 0, 0)));
            grow(xf_point(o2w.t, v(0, 1, 0))); grow(xf_point(o2w.t, v(0, -1, 0)));
        }
    } else if (m.shape_type == MTSGPU_SHAPE_SPHERE) {
        o2w = translate(m.center[0], m.center[1], m.center[2]);
        float radius = m.radius;
        if (m.has_to_world) {
            Xf T;
            if ((rc = desc_transform(m.to_world, m.to_world_inv, T, err))) return rc;
            const float r = length(xf_vec(T.t, v(1, 0, 0)));
            const float ir = 1 / r;
            o2w = compose(compose(T, scale(ir, ir, ir)), o2w);
            radius *= r;
        }
        a.flip = m.flip_normals ? 1 : 0;
        const V c = xf_point(o2w.t, v(0, 0, 0));
        put3(a.center, c);
        a.radius = radius;
        a.inv_area = 1 / (4 * kPi * radius * radius);
        if (radius <= 0) { err = "Cannot create spheres of radius <= 0"; return MTSGPU_EINVAL; }
        grow(c - v(radius, radius, radius));
        grow(c + v(radius, radius, radius));
    } else {
        err = "unsupported shape type"; return MTSGPU_EINVAL;
    }
    put16(a.to_world, o2w.t);
    put16(a.to_obj, o2w.inv);
    return MTSGPU_OK;
}

int configure_camera(const mtsgpu_sensor_desc &s, MtsgCamera &cam, std::string &err) {
    if (s.film_width == 0 || s.film_height == 0) { err = "film size must be positive"; return MTSGPU_EINVAL; }
    const float aspect = (float)s.film_width / (float)s.film_height;
    float xfov = s.fov;
    int axis = s.fov_axis;
    if (axis == MTSGPU_FOV_SMALLER) axis = aspect > 1 ? MTSGPU_FOV_Y : MTSGPU_FOV_X;
    else if (axis == MTSGPU_FOV_LARGER) axis = aspect > 1 ? MTSGPU_FOV_X : MTSGPU_FOV_Y;
    if (axis == MTSGPU_FOV_Y) {
        xfov = rad2deg(2 * std::atan(std::tan(0.5f * deg2rad(s.fov)) * aspect));
    } else if (axis == MTSGPU_FOV_DIAGONAL) {
        float diagonal = 2 * std::tan(0.5f * deg2rad(s.fov));
        float width = diagonal / std::sqrt(1.0f + 1.0f / (aspect * aspect));
        xfov = rad2deg(2 * std::atan(width * 0.5f));
    } else if (axis != MTSGPU_FOV_X) {
        err = "The 'fovAxis' parameter must be set to one of 'smaller', 'larger', 'diagonal', 'x', or 'y'!";
        return MTSGPU_EINVAL;
    }
    if (!(xfov > 0 && xfov < 180)) { err = "The horizontal field of view must be in the interval (0, 180)!"; return MTSGPU_EINVAL; }
    if (!(s.near_clip > 0)) { err = "The 'nearClip' parameter must be greater than zero!"; return MTSGPU_EINVAL; }
    if (!(s.near_clip < s.far_clip)) { err = "The 'nearClip' parameter must be less than 'farClip'!"; return MTSGPU_EINVAL; }
    // Transform::perspective (transform.cpp:99-123)
    float recip = 1.0f / (s.far_clip - s.near_clip);
    float cot = 1.0f / std::tan(deg2rad(xfov / 2.0f));
    M4 P; std::memset(&P, 0, sizeof P);
    P.m[0][0] = cot; P.m[1][1] = cot;
    P.m[2][2] = s.far_clip * recip; P.m[2][3] = -s.near_clip * s.far_clip * recip;
    P.m[3][2] = 1;
    Xf persp;
    persp.t = P;
    if (!invert(P, persp.inv)) { err = "Unable to invert singular matrix"; return MTSGPU_EINVAL; }
    // perspective.cpp:146-151 (crop = film)
    Xf a = scale(1.0f / 1.0f, 1.0f / 1.0f, 1.0f);
    Xf b = translate(-0.0f, -0.0f, 0.0f);
    Xf c = scale(-0.5f, -0.5f * aspect, 1.0f);
    Xf d = translate(-1.0f, -1.0f / aspect, 0.0f);
    Xf camToSample = compose(compose(compose(compose(a, b), c), d), persp);
    const M4 &s2c = camToSample.inv;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            cam.sample_to_camera[i * 4 + j] = s2c.m[i][j];
            cam.to_world[i * 4 + j] = s.to_world[i * 4 + j];
        }
    cam.inv_res_x = (float)1 / (float)s.film_width;
    cam.inv_res_y = (float)1 / (float)s.film_height;
    cam.near_clip = s.near_clip;
    cam.far_clip = s.far_clip;
    V o0 = xf_point(s2c, v(0.0f, 0.0f, 0.0f));
    V dx = xf_point(s2c, v(cam.inv_res_x, 0.0f, 0.0f)) - o0;
    V dy = xf_point(s2c, v(0.0f, cam.inv_res_y, 0.0f)) - o0;
    cam.dx[0] = dx.x; cam.dx[1] = dx.y; cam.dx[2] = dx.z;
    cam.dy[0] = dy.x; cam.dy[1] = dy.y; cam.dy[2] = dy.z;
    return MTSGPU_OK;
}

float energy_scale(const float *s, int ensure) {   // BSDF::ensureEnergyConservation (bsdf.cpp:88-113)
    if (!ensure) return 1.0f;
    float mx = s[0];
    mx = fmax_std(mx, s[1]);
    mx = fmax_std(mx, s[2]);
    if (mx > 1.0f) return 0.99f * (1.0f / mx);
    return 1.0f;
}

// Texture getMaximum/getMinimum/getAverage (checkerboard.cpp, texture.cpp ConstantSpectrumTexture)
void tex_max(const mtsgpu_texture_desc &t, const float *c, float out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = t.type ? fmax_std(t.color0[i], t.color1[i]) : c[i];
}
void tex_min(const mtsgpu_texture_desc &t, const float *c, float out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = t.type ? fmin_std(t.color0[i], t.color1[i]) : c[i];
}
void tex_avg(const mtsgpu_texture_desc &t, const float *c, float out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = t.type ? (t.color0[i] + t.color1[i]) * 0.5f : c[i];
}
float avg_spec(const float s[3]) { float r = 0.0f; r += s[0]; r += s[1]; r += s[2]; return r * (1.0f / 3); }
float luminance(const float s[3]) { return s[0] * 0.212671f + s[1] * 0.715160f + s[2] * 0.072169f; }   // spectrum.h:725

// a textured parameter into the device record; `scale` = ensureEnergyConservation's
// ScaleTexture factor (eval = nested eval * scale, scale.cpp:85-87)
int set_tex(const mtsgpu_texture_desc &t, float scale, MtsgTex &o, std::string &err) {
    std::memset(&o, 0, sizeof o);
    if (t.type == MTSGPU_TEX_NONE) return MTSGPU_OK;
    if (t.type != MTSGPU_TEX_CHECKERBOARD) { err = "unsupported texture type"; return MTSGPU_EINVAL; }
    o.type = t.type;
    for (int i = 0; i < 3; ++i) {
        o.c0[i] = scale != 1.0f ? t.color0[i] * scale : t.color0[i];
        o.c1[i] = scale != 1.0f ? t.color1[i] * scale : t.color1[i];
    }
    o.uoff = t.uoffset; o.voff = t.voffset; o.uscale = t.uscale; o.vscale = t.vscale;
    return MTSGPU_OK;
}

// RoughPlastic ctor + configure (roughplastic.cpp:197-300)
int configure_roughplastic(const mtsgpu_bsdf_desc &d, MtsgBsdf &b, std::vector<float> &rt, std::string &err) {
    if (d.int_ior < 0 || d.ext_ior < 0 || d.int_ior == d.ext_ior) {
        err = "The interior and exterior indices of refraction must be positive and differ!";
        return MTSGPU_EINVAL;
    }
    b.eta = d.int_ior / d.ext_ior;
    b.nonlinear = d.nonlinear ? 1 : 0;
    if (d.distribution < 0 || d.distribution > 2) {
        err = "Specified an invalid distribution, must be \"beckmann\", \"ggx\", or \"phong\"/\"as\"!";
        return MTSGPU_EINVAL;
    }
    b.distr = d.distribution;
    b.sample_visible = d.distribution == MTSGPU_DISTR_PHONG ? 0 : d.sample_visible;
    const float au = fmax_std(d.alpha_u, 1e-4f), av = fmax_std(d.alpha_v, 1e-4f);
    if (d.alpha_tex.type == MTSGPU_TEX_NONE && au != av) {
        err = "The 'roughplastic' plugin currently does not support anisotropic microfacet distributions!";
        return MTSGPU_EINVAL;
    }
    // m_alpha = ConstantFloatTexture(distr.getAlpha()) unless a texture was added
    float alpha3[3] = {au, au, au};
    b.alpha_u = b.alpha_v = avg3(au);
    int rc;
    // ensureEnergyConservation of both reflectances (bsdf.cpp:88-113)
    float mx[3];
    tex_max(d.reflectance_tex, d.diffuse_reflectance, mx);
    const float sd = energy_scale(mx, d.ensure_energy_conservation);
    const float ss = energy_scale(d.specular_reflectance, d.ensure_energy_conservation);
    for (int i = 0; i < 3; ++i) {
        b.refl[i] = sd != 1.0f ? d.diffuse_reflectance[i] * sd : d.diffuse_reflectance[i];
        b.spec_r[i] = ss != 1.0f ? d.specular_reflectance[i] * ss : d.specular_reflectance[i];
    }
    if ((rc = set_tex(d.reflectance_tex, sd, b.refl_tex, err))) return rc;
    if ((rc = set_tex(d.alpha_tex, 1.0f, b.alpha_tex, err))) return rc;
    // m_specularSamplingWeight = sAvg / (dAvg + sAvg) of the (scaled) textures' averages
    float davg[3], savg[3];
    tex_avg(d.reflectance_tex, d.diffuse_reflectance, davg);
    for (int i = 0; i < 3; ++i) {
        if (sd != 1.0f) davg[i] = davg[i] * sd;
        savg[i] = b.spec_r[i];
    }
    const float dAvg = luminance(davg), sAvg = luminance(savg);
    b.spec_weight = sAvg / (dAvg + sAvg);
    b.inv_eta2 = 1.0f / (b.eta * b.eta);
    b.flags = MTSG_F_GLOSSY_REFL | MTSG_F_DIFF_REFL | MTSG_F_FRONT;
    // RoughTransmittance(m_type): the distribution's table, checked and reduced
    MtsgRTrans ext;
    if ((rc = mtsg_rtrans_load(d.rtrans_data, (size_t)d.rtrans_bytes, ext, err))) {
        if (!d.rtrans_data) err = "roughplastic: no rough transmittance table (data/microfacet/<distribution>.dat)";
        return rc;
    }
    float amin[3], amax[3];
    tex_min(d.alpha_tex, alpha3, amin);
    tex_max(d.alpha_tex, alpha3, amax);
    if ((rc = mtsg_rtrans_check(ext, b.eta, avg_spec(amin), avg_spec(amax), err))) return rc;
    MtsgRTrans in = ext;
    mtsg_rtrans_set_eta(ext, b.eta);
    mtsg_rtrans_set_eta(in, 1 / b.eta);
    if (d.alpha_tex.type == MTSGPU_TEX_NONE) mtsg_rtrans_set_alpha(ext, b.alpha_u);
    b.rt_theta = (int32_t)ext.theta;
    b.rt_alpha = (int32_t)ext.alpha;
    b.rt_alpha_fixed = ext.alphaFixed ? 1 : 0;
    b.rt_alpha_min = ext.alphaMin;
    b.rt_alpha_max = ext.alphaMax;
    b.rt_ext = (int32_t)rt.size();
    rt.insert(rt.end(), ext.trans.begin(), ext.trans.end());
    b.rt_int = (int32_t)rt.size();
    rt.insert(rt.end(), in.diff.begin(), in.diff.end());
    return MTSGPU_OK;
}

// fresnelDielectricExt(cosThetaI, eta) (util.cpp:651-677)
float fresnel_dielectric_ext_h(float cosThetaI_, float eta) {
    if (eta == 1) return 0.0f;
    const float scale = (cosThetaI_ > 0) ? 1 / eta : eta,
                cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) return 1.0f;
    const float cosThetaI = std::fabs(cosThetaI_), cosThetaT = std::sqrt(cosThetaTSqr);
    const float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    const float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    return 0.5f * (Rs * Rs + Rp * Rp);
}

// GaussLobattoIntegrator(1024, 0, 1e-5f) with the convergence estimate
// (quad.cpp:287-409) over fresnelDiffuseIntegrand (util.cpp:808-811): the
// accurate branch of fresnelDiffuseReflectance(eta, false) (util.cpp:814-860).
// The six sub-steps are summed (and their evaluations counted) left to right.
struct FdrQuad {
    float eta;
    size_t evals = 0;
    static constexpr size_t kMaxEvals = 1024;
    static constexpr float kRelError = 1e-5f;
    const float alpha = (float)std::sqrt(2.0 / 3.0), beta = (float)(1.0 / std::sqrt(5.0));
    const float x1 = (float)0.94288241569547971906, x2 = (float)0.64185334234578130578,
                x3 = (float)0.23638319966214988028;
    float f(float xi) const { return fresnel_dielectric_ext_h(std::sqrt(xi), eta); }
    float abs_tolerance(float a, float b) {
        const float m = (a + b) / 2, h = (b - a) / 2;
        const float y1 = f(a), y3 = f(m - alpha * h), y5 = f(m - beta * h), y7 = f(m), y9 = f(m + beta * h),
                    y11 = f(m + alpha * h), y13 = f(b);
        const float acc = h * ((float)0.0158271919734801831 * (y1 + y13)
                             + (float)0.0942738402188500455 * (f(m - x1 * h) + f(m + x1 * h))
                             + (float)0.1550719873365853963 * (y3 + y11)
                             + (float)0.1888215739601824544 * (f(m - x2 * h) + f(m + x2 * h))
                             + (float)0.1997734052268585268 * (y5 + y9)
                             + (float)0.2249264653333395270 * (f(m - x3 * h) + f(m + x3 * h))
                             + (float)0.2426110719014077338 * y7);
        evals += 13;
        float r = 1.0f;
        const float integral2 = (h / 6) * (y1 + y13 + 5 * (y5 + y9));
        const float integral1 = (h / 1470) * (77 * (y1 + y13) + 432 * (y3 + y11) + 625 * (y5 + y9) + 672 * y7);
        if (std::fabs(integral2 - acc) != 0.0f) r = std::fabs(integral1 - acc) / std::fabs(integral2 - acc);
        if (r == 0.0f || r > 1.0f) r = 1.0f;
        float result = INFINITY;
        if (acc != 0) result = acc * fmax_std(kRelError, FLT_EPSILON) / (r * FLT_EPSILON);
        return result;
    }
    float step(float a, float b, float fa, float fb, float acc) {
        const float h = (b - a) / 2, m = (a + b) / 2;
        const float mll = m - alpha * h, ml = m - beta * h, mr = m + beta * h, mrr = m + alpha * h;
        const float fmll = f(mll), fml = f(ml), fm = f(m), fmr = f(mr), fmrr = f(mrr);
        const float integral2 = (h / 6) * (fa + fb + 5 * (fml + fmr));
        const float integral1 = (h / 1470) * (77 * (fa + fb) + 432 * (fmll + fmrr) + 625 * (fml + fmr) + 672 * fm);
        evals += 5;
        if (evals >= kMaxEvals) return integral1;
        const float dist = acc + (integral1 - integral2);
        if (dist == acc || mll <= a || b <= mrr) return integral1;
        float r = step(a, mll, fa, fmll, acc);
        r = r + step(mll, ml, fmll, fml, acc);
        r = r + step(ml, m, fml, fm, acc);
        r = r + step(m, mr, fm, fmr, acc);
        r = r + step(mr, mrr, fmr, fmrr, acc);
        r = r + step(mrr, b, fmrr, fb, acc);
        return r;
    }
    float integrate() {   // over [0, 1]
        const float tol = abs_tolerance(0.0f, 1.0f);
        evals += 2;
        return step(0.0f, 1.0f, f(0.0f), f(1.0f), tol);
    }
};

float fresnel_diffuse_reflectance(float eta) {
    FdrQuad q;
    q.eta = eta;
    return q.integrate();
}

// SmoothConductor / SmoothDielectric / SmoothPlastic ctor + configure
// (conductor.cpp:164-212, dielectric.cpp:146-201, plastic.cpp:144-216)
int configure_smooth(const mtsgpu_bsdf_desc &d, MtsgBsdf &b, std::string &err) {
    const float ss = energy_scale(d.specular_reflectance, d.ensure_energy_conservation);
    for (int i = 0; i < 3; ++i) b.spec_r[i] = ss != 1.0f ? d.specular_reflectance[i] * ss : d.specular_reflectance[i];
    if (d.type == MTSGPU_BSDF_CONDUCTOR) {
        const float r = 1.0f / d.ext_eta;   // m_eta = eta / extEta (Spectrum / Float: reciprocal multiply)
        for (int i = 0; i < 3; ++i) { b.eta3[i] = d.eta[i] * r; b.k3[i] = d.k[i] * r; }
        b.flags = MTSG_F_DELTA_REFL | MTSG_F_FRONT;
        return MTSGPU_OK;
    }
    if (d.int_ior < 0 || d.ext_ior < 0) {
        err = "The interior and exterior indices of refraction must be positive!";
        return MTSGPU_EINVAL;
    }
    b.eta = d.int_ior / d.ext_ior;
    if (d.type == MTSGPU_BSDF_DIELECTRIC) {
        b.inv_eta = 1 / b.eta;
        const float st = energy_scale(d.specular_transmittance, d.ensure_energy_conservation);
        for (int i = 0; i < 3; ++i)
            b.spec_t[i] = st != 1.0f ? d.specular_transmittance[i] * st : d.specular_transmittance[i];
        b.flags = MTSG_F_DELTA_REFL | MTSG_F_DELTA_TRANS | MTSG_F_FRONT | MTSG_F_BACK;
        return MTSGPU_OK;
    }
    // plastic
    b.nonlinear = d.nonlinear ? 1 : 0;
    float mx[3];
    tex_max(d.reflectance_tex, d.diffuse_reflectance, mx);
    const float sd = energy_scale(mx, d.ensure_energy_conservation);
    for (int i = 0; i < 3; ++i) b.refl[i] = sd != 1.0f ? d.diffuse_reflectance[i] * sd : d.diffuse_reflectance[i];
    int rc;
    if ((rc = set_tex(d.reflectance_tex, sd, b.refl_tex, err))) return rc;
    b.fdr_int = fresnel_diffuse_reflectance(1 / b.eta);
    b.fdr_ext = fresnel_diffuse_reflectance(b.eta);
    float davg[3], savg[3];
    tex_avg(d.reflectance_tex, d.diffuse_reflectance, davg);
    for (int i = 0; i < 3; ++i) {
        if (sd != 1.0f) davg[i] = davg[i] * sd;
        savg[i] = b.spec_r[i];
    }
    const float dAvg = luminance(davg), sAvg = luminance(savg);
    b.spec_weight = sAvg / (dAvg + sAvg);
    b.inv_eta2 = 1 / (b.eta * b.eta);
    b.flags = MTSG_F_DELTA_REFL | MTSG_F_DIFF_REFL | MTSG_F_FRONT;
    return MTSGPU_OK;
}

int configure_bsdf(const mtsgpu_bsdf_desc &d, MtsgBsdf &b, std::vector<float> &rt, std::string &err) {
    std::memset(&b, 0, sizeof b);
    b.type = d.type;
    b.nested[0] = b.nested[1] = -1;
    if (d.type == MTSGPU_BSDF_TWOSIDED) return MTSGPU_OK;   // resolved by configure_twosided
    if (d.type == MTSGPU_BSDF_CONDUCTOR || d.type == MTSGPU_BSDF_DIELECTRIC || d.type == MTSGPU_BSDF_PLASTIC)
        return configure_smooth(d, b, err);
    if (d.type == MTSGPU_BSDF_DIFFUSE) {
        float mx[3];
        tex_max(d.reflectance_tex, d.reflectance, mx);
        float sc = energy_scale(mx, d.ensure_energy_conservation);
        for (int i = 0; i < 3; ++i) b.refl[i] = sc != 1.0f ? d.reflectance[i] * sc : d.reflectance[i];
        int rc = set_tex(d.reflectance_tex, sc, b.refl_tex, err);
        if (rc) return rc;
        float m2[3];
        tex_max(d.reflectance_tex, b.refl, m2);
        if (d.reflectance_tex.type) for (int i = 0; i < 3; ++i) m2[i] = fmax_std(b.refl_tex.c0[i], b.refl_tex.c1[i]);
        float mxs = fmax_std(fmax_std(m2[0], m2[1]), m2[2]);
        b.flags = mxs > 0 ? (MTSG_F_DIFF_REFL | MTSG_F_FRONT) : 0;
        return MTSGPU_OK;
    }
    if (d.type == MTSGPU_BSDF_ROUGHPLASTIC) return configure_roughplastic(d, b, rt, err);
    if (d.type != MTSGPU_BSDF_ROUGHCONDUCTOR && d.type != MTSGPU_BSDF_ROUGHDIELECTRIC) {
        err = "unsupported BSDF type"; return MTSGPU_EINVAL;
    }
    if (d.alpha_tex.type != MTSGPU_TEX_NONE) {
        int rc = set_tex(d.alpha_tex, 1.0f, b.alpha_tex, err);
        if (rc) return rc;
    }
    if (d.distribution < 0 || d.distribution > 2) {
        err = "Specified an invalid distribution, must be \"beckmann\", \"ggx\", or \"phong\"/\"as\"!";
        return MTSGPU_EINVAL;
    }
    b.distr = d.distribution;
    b.sample_visible = d.distribution == MTSGPU_DISTR_PHONG ? 0 : d.sample_visible;
    const float au = fmax_std(d.alpha_u, 1e-4f), av = fmax_std(d.alpha_v, 1e-4f);
    b.alpha_u = avg3(au);
    b.alpha_v = avg3(av);
    float sc = energy_scale(d.specular_reflectance, d.ensure_energy_conservation);
    for (int i = 0; i < 3; ++i) b.spec_r[i] = sc != 1.0f ? d.specular_reflectance[i] * sc : d.specular_reflectance[i];
    if (d.type == MTSGPU_BSDF_ROUGHCONDUCTOR) {
        const float r = 1.0f / d.ext_eta;
        for (int i = 0; i < 3; ++i) { b.eta3[i] = d.eta[i] * r; b.k3[i] = d.k[i] * r; }
        b.flags = MTSG_F_GLOSSY_REFL | MTSG_F_FRONT;
    } else {
        if (d.int_ior < 0 || d.ext_ior < 0 || d.int_ior == d.ext_ior) {
            err = "The interior and exterior indices of refraction must be positive and differ!";
            return MTSGPU_EINVAL;
        }
        b.eta = d.int_ior / d.ext_ior;
        b.inv_eta = 1 / b.eta;
        float st = energy_scale(d.specular_transmittance, d.ensure_energy_conservation);
        for (int i = 0; i < 3; ++i) b.spec_t[i] = st != 1.0f ? d.specular_transmittance[i] * st : d.specular_transmittance[i];
        b.flags = MTSG_F_GLOSSY_REFL | MTSG_F_GLOSSY_TRANS | MTSG_F_FRONT | MTSG_F_BACK;
    }
    return MTSGPU_OK;
}

// unitAngle (core/util.h:309-314)
float unit_angle(V a, V b) {
    if (dot(a, b) < 0) return kPi - 2 * std::asin(0.5f * length(b + a));
    return 2 * std::asin(0.5f * length(b - a));
}

// coordinateSystem (util.cpp:592-601)
void coordinate_system(V a, V &b, V &c) {
    if (std::fabs(a.x) > std::fabs(a.y)) {
        float invLen = 1.0f / std::sqrt(a.x * a.x + a.z * a.z);
        c = v(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / std::sqrt(a.y * a.y + a.z * a.z);
        c = v(0.0f, a.z * invLen, -a.y * invLen);
    }
    b = cross(c, a);
}

// ---- BVH2 (binned SAH) ------------------------------------------------------
struct BBox {
    float lo[3], hi[3];
    void reset() { for (int a = 0; a < 3; ++a) { lo[a] = FLT_MAX; hi[a] = -FLT_MAX; } }
    void grow(const BBox &b) { for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); } }
    void growp(const float *p) { for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], p[a]); hi[a] = std::max(hi[a], p[a]); } }
    float area() const {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (dx < 0) return 0;
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};

struct BuildPrim { BBox box; float c[3]; uint32_t id; };

const uint32_t kMaxDepth = 28;   // traversal stack (LDS) holds < 32 entries

// SAH knobs (A/B only; results never depend on them): MTSGPU_SAH_BINS (128: C3 +3.4%,
// C4 +0.7% over 32, profiles/r03_ab_sah_C*.log),
// MTSGPU_SAH_CI (cost of a triangle test per node visit, 1), MTSGPU_LEAF_MAX (8, <= 15)
static int env_int(const char *k, int def, int lo, int hi) {
    const char *v = std::getenv(k);
    return v ? std::max(lo, std::min(hi, std::atoi(v))) : def;
}
static float env_float(const char *k, float def) {
    const char *v = std::getenv(k);
    return v ? (float)std::atof(v) : def;
}

struct Builder {
    std::vector<BuildPrim> &prims;
    std::vector<MtsgNode> &nodes;
    std::vector<uint32_t> order;
    float absEps;
    uint32_t maxDepth = 0;
    const int nbins = env_int("MTSGPU_SAH_BINS", 128, 4, 1024);
    const float ci = env_float("MTSGPU_SAH_CI", 1.0f);
    const uint32_t leafMax = (uint32_t)env_int("MTSGPU_LEAF_MAX", MTSG_LEAF_MAX, 1, 15);
    // the binned SAH's scratch, sized once and reused by every build() call
    std::vector<BBox> bb, lb;
    std::vector<uint32_t> bc, lc;
    explicit Builder(std::vector<BuildPrim> &p, std::vector<MtsgNode> &n)
        : prims(p), nodes(n), bb(nbins), lb(nbins), bc(nbins), lc(nbins) {}

    void inflate(BBox &b) const {
        for (int a = 0; a < 3; ++a) {
            float e = (b.hi[a] - b.lo[a]) * 1e-4f + 1e-6f * (std::fabs(b.lo[a]) + std::fabs(b.hi[a])) + absEps;
            b.lo[a] -= e; b.hi[a] += e;
        }
    }
    BBox bounds(uint32_t first, uint32_t count) const {
        BBox b; b.reset();
        for (uint32_t i = first; i < first + count; ++i) b.grow(prims[order[i]].box);
        return b;
    }
    // returns child reference for the range
    int32_t build(uint32_t first, uint32_t count, uint32_t depth) {
        maxDepth = std::max(maxDepth, depth);
        if (count <= 2 || (count <= leafMax && depth >= kMaxDepth - 1))
            return mtsg_leaf_ref(first, count);
        // switch to median splits early enough that depth stays <= kMaxDepth
        uint32_t lg = 0;
        while ((2u << lg) * 2 < count) ++lg;   // ~log2(count / 2)
        const bool forceMedian = depth + lg + 2 >= kMaxDepth;
        BBox cb; cb.reset();
        for (uint32_t i = first; i < first + count; ++i) cb.growp(prims[order[i]].c);
        const int NB = nbins;
        float bestCost = FLT_MAX; int bestAxis = -1, bestSplit = -1;
        const BBox nb = bounds(first, count);
        const float leafCost = ci * (float)count;
        for (int axis = 0; axis < 3; ++axis) {
            const float ext = cb.hi[axis] - cb.lo[axis];
            if (!(ext > 0)) continue;
            std::fill(bc.begin(), bc.end(), 0u);
            for (int i = 0; i < NB; ++i) bb[i].reset();
            const float k = NB / ext;
            for (uint32_t i = first; i < first + count; ++i) {
                const BuildPrim &p = prims[order[i]];
                int bi = std::min(NB - 1, (int)((p.c[axis] - cb.lo[axis]) * k));
                bb[bi].grow(p.box); bc[bi]++;
            }
            BBox acc; acc.reset(); uint32_t n = 0;
            for (int i = 0; i < NB; ++i) { acc.grow(bb[i]); n += bc[i]; lb[i] = acc; lc[i] = n; }
            acc.reset(); n = 0;
            for (int i = NB - 1; i > 0; --i) {
                acc.grow(bb[i]); n += bc[i];
                if (lc[i - 1] == 0 || n == 0) continue;
                const float cost = 1.0f + ci * (lb[i - 1].area() * lc[i - 1] + acc.area() * n) / std::max(nb.area(), 1e-30f);
                if (cost < bestCost) { bestCost = cost; bestAxis = axis; bestSplit = i; }
            }
        }
        uint32_t mid;
        if (bestAxis < 0 || (count <= leafMax && bestCost >= leafCost)) {
            if (count <= leafMax) return mtsg_leaf_ref(first, count);
            // degenerate centroids: median split on index order
            mid = first + count / 2;
        } else {
            const float ext = cb.hi[bestAxis] - cb.lo[bestAxis];
            const float k = NB / ext;
            auto it = std::partition(order.begin() + first, order.begin() + first + count, [&](uint32_t id) {
                int bi = std::min(NB - 1, (int)((prims[id].c[bestAxis] - cb.lo[bestAxis]) * k));
                return bi < bestSplit;
            });
            mid = (uint32_t)(it - order.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        if (forceMedian) {
            // keep the tree shallow: median split on the widest centroid axis
            int axis = 0;
            for (int a = 1; a < 3; ++a) if (cb.hi[a] - cb.lo[a] > cb.hi[axis] - cb.lo[axis]) axis = a;
            mid = first + count / 2;
            std::nth_element(order.begin() + first, order.begin() + mid, order.begin() + first + count,
                             [&](uint32_t x, uint32_t y) { return prims[x].c[axis] < prims[y].c[axis]; });
        }
        const uint32_t id = (uint32_t)nodes.size();
        nodes.push_back(MtsgNode());
        BBox b0 = bounds(first, mid - first), b1 = bounds(mid, first + count - mid);
        inflate(b0); inflate(b1);
        const int32_t c0 = build(first, mid - first, depth + 1);
        const int32_t c1 = build(mid, first + count - mid, depth + 1);
        MtsgNode &n = nodes[id];
        n.c0lox = b0.lo[0]; n.c0hix = b0.hi[0]; n.c0loy = b0.lo[1]; n.c0hiy = b0.hi[1];
        n.c1lox = b1.lo[0]; n.c1hix = b1.hi[0]; n.c1loy = b1.lo[1]; n.c1hiy = b1.hi[1];
        n.c0loz = b0.lo[2]; n.c0hiz = b0.hi[2]; n.c1loz = b1.lo[2]; n.c1hiz = b1.hi[2];
        n.c0 = c0; n.c1 = c1; n.pad0 = n.pad1 = 0;
        return (int32_t)id;
    }
};

// ---- environment emitter (emitters/envmap.cpp, render/mipmap.h) ------------
// half::half(float) (core/half.h:434-488, libcore/half.cpp:78-200): round to
// nearest even, overflow to infinity, NaN payload kept
uint16_t float_to_half(float f) {
    uint32_t i;
    std::memcpy(&i, &f, 4);
    const uint32_t s = (i >> 16) & 0x8000u;
    int e = (int)((i >> 23) & 0xff) - (127 - 15);
    uint32_t m = i & 0x7fffffu;
    if (e <= 0) {
        if (e < -10) return (uint16_t)s;
        m |= 0x800000u;
        const int t = 14 - e;
        const uint32_t a = (1u << (t - 1)) - 1u, b = (m >> t) & 1u;
        m = (m + a + b) >> t;
        return (uint16_t)(s | m);
    }
    if (e == 0xff - (127 - 15)) {
        if (m == 0) return (uint16_t)(s | 0x7c00u);
        m >>= 13;
        return (uint16_t)(s | 0x7c00u | m | (m == 0));
    }
    m = m + 0xfffu + ((m >> 13) & 1u);
    if (m & 0x800000u) { m = 0; e += 1; }
    if (e > 30) return (uint16_t)(s | 0x7c00u);
    return (uint16_t)(s | ((uint32_t)e << 10) | (m >> 13));
}
float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ffu, bits;
    if (e == 0) {
        if (m == 0) bits = s;
        else {
            e = 127 - 15 + 1;
            while (!(m & 0x400u)) { m <<= 1; --e; }
            bits = s | (e << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        bits = s | 0x7f800000u | (m << 13);
    } else {
        bits = s | ((e + 127 - 15) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

// x as a half rounded toward +inf (up) or -inf (down): BVH box bounds that never shrink
static uint16_t half_outward(float x, bool up) {
    const uint16_t h = float_to_half(x);
    const float y = half_to_float(h);
    if (up ? !(y < x) : !(y > x)) return h;
    const bool neg = (h & 0x8000u) != 0;
    if (up) return neg ? (uint16_t)(h - 1) : (uint16_t)(h + 1);   // toward +inf (0x7bff + 1 = +inf)
    if ((h & 0x7fffu) == 0) return 0x8001u;                        // +0 -> the negative subnormal
    return neg ? (uint16_t)(h + 1) : (uint16_t)(h - 1);
}

// MtsgNode -> MtsgHNode (layout.h): same children, half boxes rounded outward
static MtsgHNode half_node(const MtsgNode &n) {
    const float lo[6] = {n.c0lox, n.c0loy, n.c1lox, n.c1loy, n.c0loz, n.c1loz};
    const float hi[6] = {n.c0hix, n.c0hiy, n.c1hix, n.c1hiy, n.c0hiz, n.c1hiz};
    MtsgHNode h;
    for (int k = 0; k < 6; ++k)
        h.box[k] = (uint32_t)half_outward(lo[k], false) | ((uint32_t)half_outward(hi[k], true) << 16);
    h.c0 = n.c0;
    h.c1 = n.c1;
    return h;
}

// the BVH2 `n2` collapsed to 4-wide nodes (layout.h MtsgQNode), depth-first
// with the root at 0: an inner BVH2 child is replaced by its two children
struct QCollapse {
    const std::vector<MtsgNode> &n2;
    std::vector<MtsgQNode> &q;
    uint32_t depth = 0;
    int32_t emit(int32_t ref, uint32_t level) {
        if (ref < 0) return ref;
        depth = std::max(depth, level);
        struct Kid { float lo[3], hi[3]; int32_t ref; } kids[4];
        int nk = 0;
        auto box = [](const MtsgNode &n, int c, Kid &k) {
            if (c == 0) {
                k.lo[0] = n.c0lox; k.hi[0] = n.c0hix; k.lo[1] = n.c0loy; k.hi[1] = n.c0hiy; k.lo[2] = n.c0loz; k.hi[2] = n.c0hiz;
                k.ref = n.c0;
            } else {
                k.lo[0] = n.c1lox; k.hi[0] = n.c1hix; k.lo[1] = n.c1loy; k.hi[1] = n.c1hiy; k.lo[2] = n.c1loz; k.hi[2] = n.c1hiz;
                k.ref = n.c1;
            }
        };
        const MtsgNode &n = n2[ref];
        for (int c = 0; c < 2; ++c) {
            Kid k;
            box(n, c, k);
            if (k.ref >= 0) {
                box(n2[k.ref], 0, kids[nk++]);
                box(n2[k.ref], 1, kids[nk++]);
            } else {
                kids[nk++] = k;
            }
        }
        const int32_t id = (int32_t)q.size();
        q.push_back(MtsgQNode());
        int32_t refs[4] = {0, 0, 0, 0};
        for (int j = 0; j < nk; ++j) refs[j] = emit(kids[j].ref, level + 1);
        MtsgQNode &out = q[id];
        for (int j = 0; j < 4; ++j) {
            for (int a = 0; a < 3; ++a)
                out.box[3 * j + a] = j < nk ? (uint32_t)half_outward(kids[j].lo[a], false) |
                                                  ((uint32_t)half_outward(kids[j].hi[a], true) << 16)
                                            : 0u;
            out.child[j] = refs[j];
        }
        return id;
    }
};

// LanczosSincFilter::eval with lobes = 2 (rfilters/lanczos.cpp:43-55)
float lanczos2(float x) {
    x = std::fabs(x);
    if (x < 1e-4f) return 1.0f;
    if (x > 2.0f) return 0.0f;
    const float x1 = kPi * x;   // M_PI is M_PI_FLT in the SINGLE_PRECISION build (constants.h:80-83)
    const float x2 = x1 / 2.0f;
    return (std::sin(x1) * std::sin(x2)) / (x1 * x2);
}

// Resampler<float> in resampling mode (core/rfilter.h:107-198) +
// resampleAndClamp(min 0, max inf) (rfilter.h:232-280); repeat or clamp boundary
struct Resampler1D {
    int src, dst, taps;
    bool repeat;
    std::vector<int> start;
    std::vector<float> w;
    Resampler1D(int sourceRes, int targetRes, bool rep) : src(sourceRes), dst(targetRes), repeat(rep) {
        float filterRadius = 2.0f, scale = 1.0f, invScale = 1.0f;
        if (targetRes < sourceRes) {
            scale = (float)sourceRes / (float)targetRes;
            invScale = 1 / scale;
            filterRadius *= scale;
        }
        taps = (int)std::ceil(filterRadius * 2);
        start.resize(targetRes);
        w.resize((size_t)taps * targetRes);
        for (int i = 0; i < targetRes; i++) {
            const float center = ((float)i + 0.5f) / (float)targetRes * (float)sourceRes;
            start[i] = (int)std::floor(center - filterRadius + 0.5f);
            float sum = 0;
            for (int j = 0; j < taps; j++) {
                const float pos = (float)(start[i] + j) + 0.5f - center;
                const float weight = lanczos2(pos * invScale);
                w[(size_t)i * taps + j] = weight;
                sum += weight;
            }
            const float normalization = 1.0f / sum;
            for (int j = 0; j < taps; j++) w[(size_t)i * taps + j] = w[(size_t)i * taps + j] * normalization;
        }
    }
    // source/target: `channels` interleaved floats per sample, sample stride in samples
    void run(const float *source, size_t sstride, float *target, size_t tstride, int channels) const {
        for (int i = 0; i < dst; ++i) {
            for (int ch = 0; ch < channels; ++ch) {
                float result = 0;
                for (int j = 0; j < taps; ++j) {
                    int pos = start[i] + j;
                    if (pos < 0 || pos >= src) {
                        if (repeat) { pos %= src; if (pos < 0) pos += src; }
                        else pos = std::min(std::max(pos, 0), src - 1);
                    }
                    result += source[sstride * channels * (size_t)pos + ch] * w[(size_t)i * taps + j];
                }
                const float lo = (0.0f < result) ? result : 0.0f;              // std::max(min, result)
                target[tstride * channels * (size_t)i + ch] = (lo < INFINITY) ? lo : INFINITY;
            }
        }
    }
};

// Bitmap::resample with the MIP map's lanczos-2 filter, ERepeat (u) / EClamp (v)
// (libcore/bitmap.cpp:2230-2329): an x pass then a y pass, each only if the size changes
std::vector<float> resample_level(const std::vector<float> &src, int w, int h, int nw, int nh) {
    std::vector<float> cur = src;
    if (w != nw) {
        Resampler1D r(w, nw, true);
        std::vector<float> tmp((size_t)nw * h * 3);
        for (int y = 0; y < h; ++y) r.run(cur.data() + (size_t)y * w * 3, 1, tmp.data() + (size_t)y * nw * 3, 1, 3);
        cur.swap(tmp);
    }
    if (h != nh) {
        Resampler1D r(h, nh, false);
        std::vector<float> tmp((size_t)nw * nh * 3);
        for (int x = 0; x < nw; ++x) r.run(cur.data() + (size_t)x * 3, nw, tmp.data() + (size_t)x * 3, nw, 3);
        cur.swap(tmp);
    }
    return cur;
}

// EnvironmentMap ctor (envmap.cpp:105-185: TMIPMap with EEWA, anisotropy 10,
// mipmap.h:155-301) and configure() (envmap.cpp:261-321)
// Guide tables for the envmap's two CDF searches (the cutpoint method): with
// G = 2^bits buckets, guide[k] = lower_bound(cdf, k / G).  For u in [k/G,
// (k+1)/G) the reference's std::lower_bound(cdf, u) (envmap.cpp:687-692) lies
// in [guide[k], guide[k+1]] because the CDF is non-decreasing, so the device
// searches that range only and lands on the same index.  A CDF that is not
// non-decreasing (negative or NaN texels) keeps the full-range search: its
// lower_bound depends on the search path.
static uint32_t guide_bits(uint32_t size) {
    uint32_t b = 0;
    while ((1u << b) < size && b < 12) ++b;
    return b;
}
static void build_guide(const float *cdf, uint32_t size, uint32_t bits, uint16_t *g) {
    const uint32_t G = 1u << bits;
    bool mono = true;
    for (uint32_t i = 0; i < size; ++i) mono &= cdf[i] <= cdf[i + 1];
    for (uint32_t k = 0; k <= G; ++k) {
        if (!mono) { g[k] = (uint16_t)(k == 0 ? 0 : size + 1); continue; }
        const float u = (float)k * (1.0f / (float)G);   // exact: G is a power of two
        g[k] = (uint16_t)(std::lower_bound(cdf, cdf + size + 1, u) - cdf);
    }
}
static void build_env_guides(HostScene &S, int W, int H) {
    S.env_guide_rows.clear();
    S.env_guide_cols.clear();
    MtsgEnv &E = S.env;
    E.guide_rbits = E.guide_cbits = 0;
    if (W + 1 > 65535 || H + 1 > 65535 || std::getenv("MTSGPU_NO_ENV_GUIDE")) return;
    E.guide_rbits = guide_bits((uint32_t)H);
    E.guide_cbits = guide_bits((uint32_t)W);
    const uint32_t gr = (1u << E.guide_rbits) + 1, gc = (1u << E.guide_cbits) + 1;
    S.env_guide_rows.assign(gr, 0);
    S.env_guide_cols.assign((size_t)gc * H, 0);
    build_guide(S.env_cdf_rows.data(), (uint32_t)H, E.guide_rbits, S.env_guide_rows.data());
    for (int y = 0; y < H; ++y)
        build_guide(S.env_cdf_cols.data() + (size_t)y * (W + 1), (uint32_t)W, E.guide_cbits,
                    S.env_guide_cols.data() + (size_t)y * gc);
}

int build_envmap(const mtsgpu_emitter_desc &e, int index, HostScene &S, std::string &err) {
    const int W = (int)e.env_width, H = (int)e.env_height;
    if (!e.env_rgb || W <= 0 || H <= 0) { err = "envmap: missing image data"; return MTSGPU_EINVAL; }
    if (std::max(W, H) > 0xFFFF) {
        err = "Environment maps images must be smaller than 65536  pixels in width and height";
        return MTSGPU_EINVAL;
    }
    MtsgEnv &E = S.env;
    std::memset(&E, 0, sizeof E);
    E.emitter = index;
    E.w0 = W; E.h0 = H;
    E.scale = e.env_scale;
    E.max_aniso = 10.0f;
    E.inv_ln2 = 1.0f / std::log(2.0f);
    // level 0: BlockedArray::init (barray.h:103-126) -> clampNegative if min < 0 (mipmap.h:226-236)
    std::vector<float> cur(e.env_rgb, e.env_rgb + (size_t)W * H * 3);
    bool negative = false;
    for (float x : cur) negative |= x < 0;
    if (negative)
        for (float &x : cur) x = (0.0f < x) ? x : 0.0f;
    S.env_texels.clear();
    auto quantize = [&](const std::vector<float> &lv, int w, int h, int level) {
        E.lw[level] = w; E.lh[level] = h;
        E.loff[level] = (uint32_t)(S.env_texels.size() / 4);
        E.ratio_x[level] = (float)w / (float)W;
        E.ratio_y[level] = (float)h / (float)H;
        for (size_t t = 0; t < (size_t)w * h; ++t) {
            S.env_texels.push_back(float_to_half(lv[3 * t]));
            S.env_texels.push_back(float_to_half(lv[3 * t + 1]));
            S.env_texels.push_back(float_to_half(lv[3 * t + 2]));
            S.env_texels.push_back(0);
        }
    };
    quantize(cur, W, H, 0);
    int levels = 1, w = W, h = H;
    while (w > 1 || h > 1) {   // mipmap.h:241-263
        const int nw = std::max(1, (w + 1) / 2), nh = std::max(1, (h + 1) / 2);
        cur = resample_level(cur, w, h, nw, nh);
        if (levels >= MTSG_ENV_MAX_LEVELS) { err = "envmap: too many MIP levels"; return MTSGPU_EINVAL; }
        quantize(cur, nw, nh, levels);
        ++levels;
        w = nw; h = nh;
    }
    E.levels = levels;
    for (int i = 0; i < MTSG_EWA_LUT; ++i) {   // mipmap.h:296-301
        const float r2 = (float)i / (float)(MTSG_EWA_LUT - 1);
        E.lut[i] = (float)std::exp((double)(-2.0f * r2)) - (float)std::exp((double)-2.0f);
    }
    // sampling CDFs over sin(theta)-weighted luminance of level 0
    S.env_cdf_cols.assign((size_t)(W + 1) * H, 0.0f);
    S.env_cdf_rows.assign((size_t)H + 1, 0.0f);
    S.env_row_weights.assign((size_t)H, 0.0f);
    size_t colPos = 0, rowPos = 0;
    float rowSum = 0.0f;
    S.env_cdf_rows[rowPos++] = 0;
    for (int y = 0; y < H; ++y) {
        float colSum = 0;
        S.env_cdf_cols[colPos++] = 0;
        for (int x = 0; x < W; ++x) {
            const uint16_t *t = &S.env_texels[((size_t)y * W + x) * 4];
            const float c[3] = {half_to_float(t[0]), half_to_float(t[1]), half_to_float(t[2])};
            colSum += luminance(c);
            S.env_cdf_cols[colPos++] = colSum;
        }
        const float normalization = 1.0f / colSum;
        for (int x = 1; x < W; ++x) S.env_cdf_cols[colPos - x - 1] *= normalization;
        S.env_cdf_cols[colPos - 1] = 1.0f;
        const float weight = std::sin(((float)y + 0.5f) * kPi / (float)H);
        S.env_row_weights[y] = weight;
        rowSum += colSum * weight;
        S.env_cdf_rows[rowPos++] = rowSum;
    }
    const float normalization = 1.0f / rowSum;
    for (int y = 1; y < H; ++y) S.env_cdf_rows[rowPos - y - 1] *= normalization;
    S.env_cdf_rows[rowPos - 1] = 1.0f;
    if (rowSum == 0) { err = "The environment map is completely black -- this is not allowed."; return MTSGPU_EINVAL; }
    if (!std::isfinite(rowSum)) {
        err = "The environment map contains an invalid floating point value (nan/inf) -- giving up.";
        return MTSGPU_EINVAL;
    }
    build_env_guides(S, W, H);
    E.normalization = 1.0f / (rowSum * (2 * kPi / (float)W) * (kPi / (float)H));
    E.pixel_x = 2 * kPi / (float)W;
    E.pixel_y = kPi / (float)H;
    // toWorld and the inverse the reference's Transform carries
    M4 T, Ti;
    bool haveInv = false;
    for (int i = 0; i < 16; ++i) {
        T.m[i / 4][i % 4] = e.env_to_world[i];
        Ti.m[i / 4][i % 4] = e.env_to_world_inv[i];
        haveInv |= e.env_to_world_inv[i] != 0.0f;
    }
    if (!haveInv && !invert(T, Ti)) { err = "envmap: singular 'toWorld'"; return MTSGPU_EINVAL; }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) { E.to_world[3 * r + c] = T.m[r][c]; E.to_local[3 * r + c] = Ti.m[r][c]; }
    return MTSGPU_OK;
}

// EnvironmentMap::createShape (envmap.cpp:331-345) as called by
// Scene::initializeBidirectional (scene.cpp:385-413): bounding sphere of the
// kd-tree bounds grown by the sensor position, radius x1.5
void envmap_bsphere(HostScene &S, const mtsgpu_sensor_desc &sensor) {
    M4 C;
    for (int i = 0; i < 16; ++i) C.m[i / 4][i % 4] = sensor.to_world[i];
    const V cp = xf_point(C, v(0.0f, 0.0f, 0.0f));   // AnimatedTransform::getTranslationBounds (track.cpp:79-83)
    float mn[3], mx[3];
    const float p[3] = {cp.x, cp.y, cp.z};
    for (int a = 0; a < 3; ++a) {
        mn[a] = fmin_std(S.aabb_min[a], p[a]);
        mx[a] = fmax_std(S.aabb_max[a], p[a]);
    }
    const V center = v((mx[0] + mn[0]) * 0.5f, (mx[1] + mn[1]) * 0.5f, (mx[2] + mn[2]) * 0.5f);
    const float radius = length(center - v(mx[0], mx[1], mx[2]));
    S.env.center[0] = center.x; S.env.center[1] = center.y; S.env.center[2] = center.z;
    S.env.radius = fmax_std(1e-4f, radius * 1.5f);
}

}  // namespace

// ---- Sobol ------------------------------------------------------------------
// Built once by a function-local static's initialiser, which C++11 runs
// exactly once even when several group members upload concurrently.
static std::vector<uint32_t> build_sobol_matrices() {
    std::vector<uint32_t> M((size_t)MTSG_SOBOL_DIMS * MTSG_SOBOL_SIZE, 0u);
    for (int k = 0; k < MTSG_SOBOL_SIZE; ++k) M[k] = (uint32_t)(((uint64_t)1 << (MTSG_SOBOL_SIZE - 1 - k)) >> 20);
    const size_t n = sizeof(kJoeKuoParams) / sizeof(kJoeKuoParams[0]);
    size_t i = 0;
    uint64_t m[MTSG_SOBOL_SIZE];
    while (i < n) {
        const uint32_t d = kJoeKuoParams[i], s = kJoeKuoParams[i + 1], a = kJoeKuoParams[i + 2];
        for (uint32_t t = 0; t < s; ++t) m[t] = kJoeKuoParams[i + 3 + t];
        i += 3 + s;
        // Sobol' recurrence: m_k = 2a_1 m_{k-1} ^ ... ^ 2^{s-1} a_{s-1} m_{k-s+1} ^ 2^s m_{k-s} ^ m_{k-s}
        for (uint32_t k = s; k < MTSG_SOBOL_SIZE; ++k) {
            uint64_t val = m[k - s] ^ (m[k - s] << s);
            for (uint32_t t = 1; t < s; ++t)
                if ((a >> (s - 1 - t)) & 1) val ^= m[k - t] << t;
            m[k] = val;
        }
        for (int k = 0; k < MTSG_SOBOL_SIZE; ++k)
            M[(size_t)(d - 1) * MTSG_SOBOL_SIZE + k] = (uint32_t)((m[k] << (MTSG_SOBOL_SIZE - 1 - k)) >> 20);
    }
    return M;
}

const std::vector<uint32_t> &mtsg_sobol_matrices() {
    static const std::vector<uint32_t> M = build_sobol_matrices();
    return M;
}

void mtsg_sobol_lookup_table(uint32_t m, MtsgLookup &L) {
    std::memset(&L, 0, sizeof L);
    L.m = m;
    if (m <= 1 || m > 31) return;
    const std::vector<uint32_t> &M = mtsg_sobol_matrices();
    for (int b = 0; b < 64; ++b) L.ycol[b] = b < MTSG_SOBOL_SIZE ? (M[MTSG_SOBOL_SIZE + b] >> (32 - m)) : 0u;
    uint32_t A[32], I[32];
    for (uint32_t r = 0; r < m; ++r) {
        A[r] = 0; I[r] = 1u << r;
        for (uint32_t t = 0; t < m; ++t) A[r] |= ((L.ycol[m + t] >> r) & 1u) << t;
    }
    for (uint32_t c = 0; c < m; ++c) {
        uint32_t piv = c;
        while (piv < m && !((A[piv] >> c) & 1u)) ++piv;
        if (piv == m) continue;   // cannot happen for a (0,2)-sequence
        std::swap(A[c], A[piv]); std::swap(I[c], I[piv]);
        for (uint32_t r = 0; r < m; ++r)
            if (r != c && ((A[r] >> c) & 1u)) { A[r] ^= A[c]; I[r] ^= I[c]; }
    }
    for (uint32_t t = 0; t < m; ++t) L.inv[t] = I[t];
}

uint64_t mtsg_sample_tea(uint32_t v0, uint32_t v1, int rounds) {   // core/qmc.h:146-156
    uint32_t sum = 0;
    for (int i = 0; i < rounds; ++i) {
        sum += 0x9e3779b9;
        v0 += ((v1 << 4) + 0xA341316C) ^ (v1 + sum) ^ ((v1 >> 5) + 0xC8013EA4);
        v1 += ((v0 << 4) + 0xAD90777D) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7E95761E);
    }
    return ((uint64_t)v1 << 32) + v0;
}

// ---- reconstruction filter (libcore/rfilter.cpp:37-55, rfilters/box.cpp, gaussian.cpp) ----
int mtsg_configure_filter(int32_t type, float param, MtsgFilter &f, std::string &err) {
    float stddev = 0;
    std::memset(&f, 0, sizeof f);
    f.type = type;
    if (type == MTSGPU_RFILTER_BOX) f.radius = param + 1e-5f;
    else if (type == MTSGPU_RFILTER_GAUSSIAN) { stddev = param; f.radius = 4 * stddev; }
    else { err = "unknown reconstruction filter"; return MTSGPU_EINVAL; }
    if (!(f.radius > 0)) { err = "filter radius must be positive"; return MTSGPU_EINVAL; }
    float sum = 0.0f;
    for (int i = 0; i < MTSG_FILTER_RES; ++i) {
        float x = (f.radius * i) / MTSG_FILTER_RES, value;
        if (type == MTSGPU_RFILTER_BOX) {
            value = std::fabs(x) <= f.radius ? 1.0f : 0.0f;
        } else {
            float alpha = -1.0f / (2.0f * stddev * stddev);
            value = fmax_std(0.0f, (float)std::exp((double)(alpha * x * x)) -
                                       (float)std::exp((double)(alpha * f.radius * f.radius)));
        }
        f.values[i] = value;
        sum += value;
    }
    f.values[MTSG_FILTER_RES] = 0.0f;
    f.scale = MTSG_FILTER_RES / f.radius;
    f.border = (int)std::ceil(f.radius - 0.5f);
    sum *= 2 * f.radius / MTSG_FILTER_RES;
    float normalization = 1.0f / sum;
    for (int i = 0; i < MTSG_FILTER_RES; ++i) f.values[i] *= normalization;
    return MTSGPU_OK;
}

// ---- scene ---------------------------------------------------------------
int mtsg_configure_scene(const mtsgpu_scene_desc *D, HostScene &S, std::string &err) {
    if (!D) { err = "null scene"; return MTSGPU_EINVAL; }
    S = HostScene();
    std::memset(&S.env, 0, sizeof S.env);
    S.env.emitter = -1;
    int rc = configure_camera(D->sensor, S.cam, err);
    if (rc) return rc;
    S.film_w = D->sensor.film_width;
    S.film_h = D->sensor.film_height;
    const uint32_t nb = D->num_bsdfs;
    S.bsdfs.resize(nb + 2);
    for (uint32_t i = 0; i < nb; ++i)
        if ((rc = configure_bsdf(D->bsdfs[i], S.bsdfs[i], S.rtrans, err))) return rc;
    // TwoSidedBRDF::configure (twosided.cpp:82-103): nested[1] defaults to
    // nested[0]; components = front ones | back ones; no transmission allowed
    for (uint32_t i = 0; i < nb; ++i) {
        const mtsgpu_bsdf_desc &d = D->bsdfs[i];
        if (d.type != MTSGPU_BSDF_TWOSIDED) continue;
        MtsgBsdf &b = S.bsdfs[i];
        if (d.nested[0] < 0 || d.nested[0] >= (int)nb) { err = "A nested one-sided material is required!"; return MTSGPU_EINVAL; }
        const int n1 = d.nested[1] < 0 ? d.nested[0] : d.nested[1];
        if (n1 >= (int)nb) { err = "twosided: nested BSDF index out of range"; return MTSGPU_EINVAL; }
        const int n[2] = {d.nested[0], n1};
        uint32_t flags = 0;
        for (int k = 0; k < 2; ++k) {
            const MtsgBsdf &c = S.bsdfs[n[k]];
            if (c.type == MTSGPU_BSDF_TWOSIDED) { err = "twosided: nesting a twosided BSDF is not supported"; return MTSGPU_EINVAL; }
            const uint32_t lobes = (uint32_t)c.flags & ~(uint32_t)(MTSG_F_FRONT | MTSG_F_BACK);
            if (lobes) flags |= lobes | (k == 0 ? MTSG_F_FRONT : MTSG_F_BACK);
        }
        if (flags & MTSG_F_TRANSMISSION) { err = "Only materials without a transmission component can be nested!"; return MTSGPU_EINVAL; }
        b.flags = (int32_t)flags;
        b.nested[0] = n[0];
        b.nested[1] = n[1];
    }
    for (uint32_t i = 0; i < nb; ++i) {
        const MtsgBsdf &b = S.bsdfs[i];
        if (b.type >= MTSGPU_BSDF_ROUGHPLASTIC || b.refl_tex.type || b.alpha_tex.type) S.ext = true;
    }
    for (uint32_t i = 0; i < D->num_meshes; ++i)   // analytic shapes run the EXT | ANA variant
        if (D->meshes[i].shape_type != MTSGPU_SHAPE_TRIMESH) S.ext = true;
    {   // Shape::configure defaults (shape.cpp:48-70): black for emitters, 0.5 otherwise
        mtsgpu_bsdf_desc dd; std::memset(&dd, 0, sizeof dd);
        dd.type = MTSGPU_BSDF_DIFFUSE; dd.ensure_energy_conservation = 1;
        configure_bsdf(dd, S.bsdfs[nb], S.rtrans, err);
        dd.reflectance[0] = dd.reflectance[1] = dd.reflectance[2] = 0.5f;
        configure_bsdf(dd, S.bsdfs[nb + 1], S.rtrans, err);
    }
    if (D->num_emitters == 0) { err = "scene has no emitters (the sunsky fallback is out of scope)"; return MTSGPU_EINVAL; }
    S.emitters.resize(D->num_emitters);
    for (uint32_t i = 0; i < D->num_emitters; ++i) {
        const mtsgpu_emitter_desc &e = D->emitters[i];
        MtsgEmitter &o = S.emitters[i];
        std::memset(&o, 0, sizeof o);
        o.type = e.type;
        o.shape = -1;
        o.weight = e.sampling_weight;
        for (int k = 0; k < 3; ++k) o.radiance[k] = e.radiance[k];
        if (e.type == MTSGPU_EMITTER_ENVMAP) {
            if (S.env.emitter >= 0) {   // scene.cpp:510-513
                err = "Only one environment emitter can be specified per scene.";
                return MTSGPU_EINVAL;
            }
            if ((rc = build_envmap(e, (int)i, S, err))) return rc;
        } else if (e.type == MTSGPU_EMITTER_CONSTANT) {
            // ConstantBackgroundEmitter (constant.cpp:44-96): a uniform environment on the
            // scene's bounding sphere (createShape, :67-91, as envmap_bsphere below)
            if (S.env.emitter >= 0) {
                err = "Only one environment emitter can be specified per scene.";
                return MTSGPU_EINVAL;
            }
            S.env.emitter = (int)i;
            S.env.constant = 1;
            for (int k = 0; k < 3; ++k) S.env.radiance[k] = e.radiance[k];
        } else if (e.type != MTSGPU_EMITTER_AREA) {
            err = "unsupported emitter type";
            return MTSGPU_EINVAL;
        }
    }
    // meshes
    uint32_t prims = 0, verts = 0;
    for (uint32_t i = 0; i < D->num_meshes; ++i) {
        const mtsgpu_mesh_desc &m = D->meshes[i];
        if (m.shape_type != MTSGPU_SHAPE_TRIMESH) { prims += 1; continue; }
        if (m.num_triangles == 0 || !m.positions || !m.indices) { err = "Encountered an empty triangle mesh!"; return MTSGPU_EINVAL; }
        prims += m.num_triangles; verts += m.num_vertices;
    }
    S.positions.resize((size_t)verts * 3);
    S.normals.assign((size_t)verts * 3, 0.0f);
    S.prim_vtx.resize((size_t)prims * 4);
    S.dpdu.resize((size_t)prims * 3);
    S.shapes.resize(D->num_meshes);
    std::vector<BuildPrim> bp(prims);
    std::vector<MtsgTri> tacc(prims);
    float amin[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, amax[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    uint32_t voff = 0, poff = 0;
    for (uint32_t si = 0; si < D->num_meshes; ++si) {
        const mtsgpu_mesh_desc &m = D->meshes[si];
        if (m.shape_type != MTSGPU_SHAPE_TRIMESH) {
            // one analytic primitive (ShapeKDTree: k = KNoTriangleFlag, skdtree.cpp:74-109)
            MtsgShape &sh = S.shapes[si];
            std::memset(&sh, 0, sizeof sh);
            if (m.emitter >= (int)D->num_emitters) { err = "emitter index out of range"; return MTSGPU_EINVAL; }
            if (m.bsdf >= (int)nb) { err = "bsdf index out of range"; return MTSGPU_EINVAL; }
            sh.emitter = m.emitter;
            sh.bsdf = m.bsdf >= 0 ? m.bsdf : (m.emitter >= 0 ? (int)nb : (int)nb + 1);
            sh.kind = m.shape_type;
            sh.has_uv = 1;
            sh.analytic = (int32_t)S.analytic.size();
            MtsgAnalytic a;
            float lo[3], hi[3];
            if ((rc = configure_analytic(m, a, lo, hi, err))) return rc;
            S.analytic.push_back(a);
            const uint32_t p = poff;
            S.prim_vtx[4 * p] = S.prim_vtx[4 * p + 1] = S.prim_vtx[4 * p + 2] = 0;
            S.prim_vtx[4 * p + 3] = si;
            S.dpdu[3 * p] = S.dpdu[3 * p + 1] = S.dpdu[3 * p + 2] = 0.0f;
            MtsgTri &ta = tacc[p];
            std::memset(&ta, 0, sizeof ta);
            ta.k = MTSG_K_ANALYTIC;
            std::memcpy(&ta.n_u, &sh.analytic, sizeof(float));
            ta.prim = p;
            ta.shape = si;
            BuildPrim &q = bp[p];
            q.id = p;
            for (int ax = 0; ax < 3; ++ax) {
                q.box.lo[ax] = lo[ax]; q.box.hi[ax] = hi[ax];
                q.c[ax] = 0.5f * (lo[ax] + hi[ax]);
                amin[ax] = std::min(amin[ax], lo[ax]);
                amax[ax] = std::max(amax[ax], hi[ax]);
            }
            if (m.emitter >= 0) {
                MtsgEmitter &e = S.emitters[m.emitter];
                if (e.shape >= 0) { err = "Tried to attach multiple emitters to a shape!"; return MTSGPU_EINVAL; }
                e.shape = (int)si;
                e.tri_first = p;
                e.tri_count = 1;
                e.cdf_offset = 0;
                e.inv_area = a.inv_area;
            }
            poff += 1;
            continue;
        }
        const uint32_t nv = m.num_vertices, nt = m.num_triangles;
        std::vector<V> P(nv), N;
        for (uint32_t k = 0; k < nv; ++k) P[k] = v(m.positions[3 * k], m.positions[3 * k + 1], m.positions[3 * k + 2]);
        std::vector<uint32_t> idx(m.indices, m.indices + 3 * (size_t)nt);
        for (uint32_t k = 0; k < 3 * nt; ++k)
            if (idx[k] >= nv) { err = "triangle index out of range"; return MTSGPU_EINVAL; }
        MtsgShape &sh = S.shapes[si];
        sh.emitter = m.emitter;
        sh.kind = MTSGPU_SHAPE_TRIMESH;
        sh.analytic = -1;
        if (m.emitter >= (int)D->num_emitters) { err = "emitter index out of range"; return MTSGPU_EINVAL; }
        if (m.bsdf >= (int)nb) { err = "bsdf index out of range"; return MTSGPU_EINVAL; }
        sh.bsdf = m.bsdf >= 0 ? m.bsdf : (m.emitter >= 0 ? (int)nb : (int)nb + 1);
        {   // EAnisotropic (roughconductor.cpp:229-231) without texcoords: computeUVTangents error (trimesh.cpp:685-691)
            // (through twosided: its combined type carries the nested EAnisotropic)
            bool aniso = false;
            if (m.bsdf >= 0) {
                const mtsgpu_bsdf_desc *ub = &D->bsdfs[m.bsdf];
                const int cand[2] = {ub->type == MTSGPU_BSDF_TWOSIDED ? S.bsdfs[m.bsdf].nested[0] : m.bsdf,
                                     ub->type == MTSGPU_BSDF_TWOSIDED ? S.bsdfs[m.bsdf].nested[1] : m.bsdf};
                for (int c : cand) {
                    const mtsgpu_bsdf_desc &cb = D->bsdfs[c];
                    if ((cb.type == MTSGPU_BSDF_ROUGHCONDUCTOR || cb.type == MTSGPU_BSDF_ROUGHDIELECTRIC) &&
                        fmax_std(cb.alpha_u, 1e-4f) != fmax_std(cb.alpha_v, 1e-4f))
                        aniso = true;
                }
            }
            if (!m.texcoords && aniso) {
                err = "computeUVTangents(): texture coordinates are required to generate tangent vectors. If you "
                      "want to render with an anisotropic material, please make sure that all associated shapes "
                      "have valid texture coordinates.";
                return MTSGPU_EINVAL;
            }
        }
        // TriMesh::computeNormals (trimesh.cpp:608-681)
        bool hasNormals = false;
        if (m.face_normals) {
            if (m.flip_normals)
                for (uint32_t t = 0; t < nt; ++t) std::swap(idx[3 * t], idx[3 * t + 1]);
        } else if (m.normals) {
            hasNormals = true;
            N.resize(nv);
            for (uint32_t k = 0; k < nv; ++k) {
                N[k] = v(m.normals[3 * k], m.normals[3 * k + 1], m.normals[3 * k + 2]);
                if (m.flip_normals) N[k] = N[k] * -1;
            }
        } else {
            hasNormals = true;
            N.assign(nv, v(0, 0, 0));
            for (uint32_t t = 0; t < nt; t++) {
                V n = v(0, 0, 0);
                for (int j = 0; j < 3; ++j) {
                    const V v0 = P[idx[3 * t + j]], v1 = P[idx[3 * t + (j + 1) % 3]], v2 = P[idx[3 * t + (j + 2) % 3]];
                    const V sideA = v1 - v0, sideB = v2 - v0;
                    if (j == 0) {
                        n = cross(sideA, sideB);
                        float len = length(n);
                        if (len == 0) break;
                        n = vdiv(n, len);
                    }
                    float angle = unit_angle(normalize(sideA), normalize(sideB));
                    N[idx[3 * t + j]] = N[idx[3 * t + j]] + n * angle;
                }
            }
            for (uint32_t k = 0; k < nv; k++) {
                float len = length(N[k]);
                if (m.flip_normals) len *= -1;
                if (len != 0) N[k] = vdiv(N[k], len);
                else N[k] = v(1, 0, 0);
            }
        }
        sh.has_normals = hasNormals ? 1 : 0;
        sh.has_uv = (S.ext && m.texcoords) ? 1 : 0;
        if (sh.has_uv) {
            if (S.texcoords.empty()) S.texcoords.assign((size_t)verts * 2, 0.0f);
            std::memcpy(&S.texcoords[2 * (size_t)voff], m.texcoords, sizeof(float) * 2 * (size_t)nv);
        }
        for (uint32_t k = 0; k < nv; ++k) {
            S.positions[3 * (voff + k)] = P[k].x; S.positions[3 * (voff + k) + 1] = P[k].y; S.positions[3 * (voff + k) + 2] = P[k].z;
            if (hasNormals) {
                S.normals[3 * (voff + k)] = N[k].x; S.normals[3 * (voff + k) + 1] = N[k].y; S.normals[3 * (voff + k) + 2] = N[k].z;
            }
        }
        // TriMesh::computeUVTangents (trimesh.cpp:683-739); dpdu = p1 - p0 without texcoords (skdtree.h:376-382)
        for (uint32_t t = 0; t < nt; ++t) {
            const uint32_t i0 = idx[3 * t], i1 = idx[3 * t + 1], i2 = idx[3 * t + 2];
            const V v0 = P[i0], v1 = P[i1], v2 = P[i2];
            V dp = v1 - v0;
            if (m.texcoords) {
                dp = v(0, 0, 0);
                const float *uv = m.texcoords;
                const V dP1 = v1 - v0, dP2 = v2 - v0;
                const float du1 = uv[2 * i1] - uv[2 * i0], dv1 = uv[2 * i1 + 1] - uv[2 * i0 + 1];
                const float du2 = uv[2 * i2] - uv[2 * i0], dv2 = uv[2 * i2 + 1] - uv[2 * i0 + 1];
                const V n = cross(dP1, dP2);
                const float len = length(n);
                if (len != 0) {
                    const float det = du1 * dv2 - dv1 * du2;
                    if (det == 0) {
                        V b, c;
                        coordinate_system(vdiv(n, len), b, c);
                        dp = b;
                    } else {
                        const float invDet = 1.0f / det;
                        dp = (dP1 * dv2 - dP2 * dv1) * invDet;
                    }
                }
            }
            const uint32_t p = poff + t;
            S.dpdu[3 * p] = dp.x; S.dpdu[3 * p + 1] = dp.y; S.dpdu[3 * p + 2] = dp.z;
            S.prim_vtx[4 * p] = voff + i0; S.prim_vtx[4 * p + 1] = voff + i1; S.prim_vtx[4 * p + 2] = voff + i2;
            S.prim_vtx[4 * p + 3] = si;
            // TriAccel::load (triaccel.h:58-90)
            MtsgTri &ta = tacc[p];
            std::memset(&ta, 0, sizeof ta);
            static const int waldModulo[4] = {1, 2, 0, 1};
            const V A = v0, B = v1, C = v2;
            const V b = C - A, c = B - A, Nn = cross(c, b);
            ta.k = 0;
            for (int j = 0; j < 3; j++)
                if (std::fabs(at(Nn, j)) > std::fabs(at(Nn, (int)ta.k))) ta.k = (uint32_t)j;
            const int u = waldModulo[ta.k], w = waldModulo[ta.k + 1];
            const float n_k = at(Nn, (int)ta.k), denom = at(b, u) * at(c, w) - at(b, w) * at(c, u);
            if (denom == 0) {
                ta.k = 3;
            } else {
                ta.n_u = at(Nn, u) / n_k;
                ta.n_v = at(Nn, w) / n_k;
                ta.n_d = dot(A, Nn) / n_k;
                ta.b_nu = at(b, u) / denom;
                ta.b_nv = -at(b, w) / denom;
                ta.a_u = at(A, u);
                ta.a_v = at(A, w);
                ta.c_nu = at(c, w) / denom;
                ta.c_nv = -at(c, u) / denom;
            }
            ta.prim = p;
            ta.shape = si;
            BuildPrim &q = bp[p];
            q.id = p;
            q.box.reset();
            const float pa[3] = {A.x, A.y, A.z}, pb[3] = {B.x, B.y, B.z}, pc[3] = {C.x, C.y, C.z};
            q.box.growp(pa); q.box.growp(pb); q.box.growp(pc);
            for (int a = 0; a < 3; ++a) {
                q.c[a] = 0.5f * (q.box.lo[a] + q.box.hi[a]);
                amin[a] = std::min(amin[a], q.box.lo[a]);
                amax[a] = std::max(amax[a], q.box.hi[a]);
            }
        }
        if (m.emitter >= 0) {
            MtsgEmitter &e = S.emitters[m.emitter];
            if (e.shape >= 0) { err = "Tried to attach multiple emitters to a shape!"; return MTSGPU_EINVAL; }
            e.shape = (int)si;
            e.tri_first = poff;
            e.tri_count = nt;
            e.cdf_offset = (uint32_t)S.area_cdf.size();
            // TriMesh::prepareSamplingTable (trimesh.cpp:389-404), DiscreteDistribution (pmf.h)
            std::vector<float> cdf(nt + 1);
            cdf[0] = 0.0f;
            for (uint32_t t = 0; t < nt; ++t) {
                const V p0 = P[idx[3 * t]], p1 = P[idx[3 * t + 1]], p2 = P[idx[3 * t + 2]];
                cdf[t + 1] = cdf[t] + 0.5f * length(cross(p1 - p0, p2 - p0));   // Triangle::surfaceArea
            }
            const float sum = cdf[nt];
            if (sum > 0) {
                const float norm = 1.0f / sum;
                for (uint32_t t = 1; t < nt + 1; ++t) cdf[t] *= norm;
                cdf[nt] = 1.0f;
            }
            e.inv_area = 1.0f / sum;
            S.area_cdf.insert(S.area_cdf.end(), cdf.begin(), cdf.end());
        }
        voff += nv;
        poff += nt;
    }
    for (const MtsgEmitter &e : S.emitters)
        if (e.type == MTSGPU_EMITTER_AREA && e.shape < 0) { err = "area emitter without a shape"; return MTSGPU_EINVAL; }
    // emitter PDF (scene.cpp:376-381)
    S.em_cdf.assign(S.emitters.size() + 1, 0.0f);
    for (size_t i = 0; i < S.emitters.size(); ++i) S.em_cdf[i + 1] = S.em_cdf[i] + S.emitters[i].weight;
    {
        const size_t n = S.emitters.size();
        const float sum = S.em_cdf[n];
        if (sum > 0) {
            S.em_norm = 1.0f / sum;
            for (size_t i = 1; i < n + 1; ++i) S.em_cdf[i] *= S.em_norm;
            S.em_cdf[n] = 1.0f;
        } else {
            S.em_norm = 0.0f;
        }
    }
    // scene bounds, slightly enlarged (gkdtree.h:1211-1217)
    const float eps = 1e-3f;
    for (int a = 0; a < 3; ++a) {
        amin[a] -= (amax[a] - amin[a]) * eps + eps;
        amax[a] += (amax[a] - amin[a]) * eps + eps;
        S.aabb_min[a] = amin[a]; S.aabb_max[a] = amax[a];
    }
    if (S.env.emitter >= 0) envmap_bsphere(S, D->sensor);
    // BVH
    Builder B(bp, S.nodes);
    B.order.resize(prims);
    for (uint32_t i = 0; i < prims; ++i) B.order[i] = i;
    float diag = 0;
    for (int a = 0; a < 3; ++a) diag += (amax[a] - amin[a]) * (amax[a] - amin[a]);
    B.absEps = 1e-7f * std::sqrt(diag) + 1e-30f;
    S.nodes.reserve(prims + 2);
    const int32_t rootRef = B.build(0, prims, 0);   // the first inner node created is node 0
    if (rootRef < 0) {
        // whole scene in one leaf: a root node holding that leaf and an empty one
        BBox b = B.bounds(0, prims);
        B.inflate(b);
        MtsgNode n;
        n.c0lox = b.lo[0]; n.c0hix = b.hi[0]; n.c0loy = b.lo[1]; n.c0hiy = b.hi[1]; n.c0loz = b.lo[2]; n.c0hiz = b.hi[2];
        n.c1lox = n.c1hix = n.c1loy = n.c1hiy = n.c1loz = n.c1hiz = 0;
        n.c0 = rootRef; n.c1 = mtsg_leaf_ref(0, 0); n.pad0 = n.pad1 = 0;
        S.nodes.push_back(n);
    }
    S.bvh_depth = B.maxDepth;
    if (B.maxDepth + 1 >= 32) { err = "BVH too deep for the traversal stack"; return MTSGPU_EINVAL; }
    S.hnodes.resize(S.nodes.size());
    for (size_t i = 0; i < S.nodes.size(); ++i) S.hnodes[i] = half_node(S.nodes[i]);
    // triangles in leaf order
    S.tris.resize(prims);
    for (uint32_t i = 0; i < prims; ++i) S.tris[i] = tacc[B.order[i]];
    return MTSGPU_OK;
}

// the 4-wide collapse of the BVH2 for mtsgpu_bvh_host only (the device traverses
// the BVH2: the 4-wide traversal lost 5-6%)
void mtsg_build_qnodes(HostScene &S) {
    S.qnodes.clear();
    S.qnodes.reserve(S.nodes.size() / 2 + 2);
    QCollapse qc{S.nodes, S.qnodes};
    qc.emit(0, 1);
    S.qnode_depth = qc.depth;
}
