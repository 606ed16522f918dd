// rtrans_host.cpp -- roughplastic's rough-transmittance tables on the host.
//
// RoughTransmittance (src/bsdfs/rtrans.h:46-150) reads
// data/microfacet/<distribution>.dat: "MTS_TRANSMITTANCE", three uint64 sizes
// (eta, alpha, theta), four floats (etaMin, etaMax, alphaMin, alphaMax), then
// for each of 2*eta IOR samples and each alpha sample: theta transmittances
// and one diffuse transmittance.  RoughPlastic::configure
// (roughplastic.cpp:263-300) checks the IOR / roughness ranges, clones the
// table, reduces one copy to eta (external) and one to 1/eta (internal) with
// tricubic interpolation (setEta, rtrans.h:262-318), and for a constant
// roughness the external one further to 1D (setAlpha, rtrans.h:327-360).
// These reductions run here in float, in the reference's operation order, with
// the host's glibc powf (the reference's std::pow(float, float)).
#include <cmath>
#include <cstdio>
#include <cstring>

#include "scene_build.h"

namespace {

inline float fmax_std(float a, float b) { return (a < b) ? b : a; }
inline float fmin_std(float a, float b) { return (b < a) ? b : a; }

// spline.cpp:23-60 (extrapolate = false)
float cubic1d(float x, const float *values, size_t size, float min, float max) {
    if (!(x >= min && x <= max)) return 0.0f;
    float t = ((x - min) * (float)(size - 1)) / (max - min);
    size_t k = std::min((size_t)t, size - 2);
    float f0 = values[k], f1 = values[k + 1], d0, d1;
    if (k > 0) d0 = 0.5f * (values[k + 1] - values[k - 1]);
    else d0 = values[k + 1] - values[k];
    if (k + 2 < size) d1 = 0.5f * (values[k + 2] - values[k]);
    else d1 = values[k + 1] - values[k];
    t = t - (float)k;
    float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}

// node weights of one dimension (spline.cpp:241-283 / 384-426)
bool cubic_weights(float p, size_t size, float min, float max, size_t &knot, float w[4]) {
    if (!(p >= min && p <= max)) return false;
    float t = ((p - min) * (float)(size - 1)) / (max - min);
    knot = std::min((size_t)t, size - 2);
    t = t - (float)knot;
    float t2 = t * t, t3 = t2 * t;
    w[0] = 0.0f;
    w[1] = 2 * t3 - 3 * t2 + 1;
    w[2] = -2 * t3 + 3 * t2;
    w[3] = 0.0f;
    float d0 = t3 - 2 * t2 + t, d1 = t3 - t2;
    if (knot > 0) { w[2] += 0.5f * d0; w[0] -= 0.5f * d0; }
    else { w[2] += d0; w[1] -= d0; }
    if (knot + 2 < size) { w[3] += 0.5f * d1; w[1] -= 0.5f * d1; }
    else { w[2] += d1; w[1] -= d1; }
    return true;
}

// spline.cpp:236-304
float cubic2d(float px, float py, const float *values, size_t sx, size_t sy) {
    size_t kx, ky;
    float wx[4], wy[4];
    if (!cubic_weights(px, sx, 0.0f, 1.0f, kx, wx)) return 0.0f;
    if (!cubic_weights(py, sy, 0.0f, 1.0f, ky, wy)) return 0.0f;
    float result = 0.0f;
    for (int y = -1; y <= 2; ++y) {
        float w = wy[y + 1];
        for (int x = -1; x <= 2; ++x) {
            float wxy = wx[x + 1] * w;
            if (wxy == 0) continue;
            size_t pos = (ky + y) * sx + kx + x;
            result += values[pos] * wxy;
        }
    }
    return result;
}

// spline.cpp:379-451
float cubic3d(float px, float py, float pz, const float *values, size_t sx, size_t sy, size_t sz) {
    size_t kx, ky, kz;
    float wx[4], wy[4], wz[4];
    if (!cubic_weights(px, sx, 0.0f, 1.0f, kx, wx)) return 0.0f;
    if (!cubic_weights(py, sy, 0.0f, 1.0f, ky, wy)) return 0.0f;
    if (!cubic_weights(pz, sz, 0.0f, 1.0f, kz, wz)) return 0.0f;
    float result = 0.0f;
    for (int z = -1; z <= 2; ++z) {
        float w = wz[z + 1];
        for (int y = -1; y <= 2; ++y) {
            float wyz = wy[y + 1] * w;
            for (int x = -1; x <= 2; ++x) {
                float wxyz = wx[x + 1] * wyz;
                if (wxyz == 0) continue;
                size_t pos = ((kz + z) * sy + (ky + y)) * sx + kx + x;
                result += values[pos] * wxyz;
            }
        }
    }
    return result;
}

}  // namespace

int mtsg_rtrans_load(const void *data, size_t bytes, MtsgRTrans &t, std::string &err) {
    const char header[] = "MTS_TRANSMITTANCE";
    const size_t hl = sizeof(header) - 1, fixed = hl + 3 * 8 + 4 * 4;
    const unsigned char *p = (const unsigned char *)data;
    if (!data || bytes < fixed || std::memcmp(p, header, hl) != 0) {
        err = "Encountered an invalid transmittance data file!";
        return MTSGPU_EINVAL;
    }
    uint64_t sz[3];
    std::memcpy(sz, p + hl, 24);   // little endian (the file is written with ELittleEndian)
    float r[4];
    std::memcpy(r, p + hl + 24, 16);
    t.eta = (size_t)sz[0]; t.alpha = (size_t)sz[1]; t.theta = (size_t)sz[2];
    t.etaMin = r[0]; t.etaMax = r[1]; t.alphaMin = r[2]; t.alphaMax = r[3];
    if (t.eta < 2 || t.alpha < 2 || t.theta < 2 || t.eta > 4096 || t.alpha > 4096 || t.theta > 4096) {
        err = "Encountered an invalid transmittance data file!";
        return MTSGPU_EINVAL;
    }
    const size_t transSize = 2 * t.eta * t.alpha * t.theta, diffSize = 2 * t.eta * t.alpha;
    if (bytes != fixed + (transSize + diffSize) * 4) {   // SAssert(getPos() == getSize()) (rtrans.h:148)
        err = "RoughTransmittance: data file size does not match its header";
        return MTSGPU_EINVAL;
    }
    t.trans.resize(transSize);
    t.diff.resize(diffSize);
    const float *f = (const float *)(p + fixed);   // rtrans.h:136-145
    size_t fdr = 0, dat = 0;
    for (size_t i = 0; i < 2 * t.eta; ++i)
        for (size_t j = 0; j < t.alpha; ++j) {
            for (size_t k = 0; k < t.theta; ++k) std::memcpy(&t.trans[dat++], f++, 4);
            std::memcpy(&t.diff[fdr++], f++, 4);
        }
    t.etaFixed = t.alphaFixed = false;
    return MTSGPU_OK;
}

void mtsg_rtrans_set_eta(MtsgRTrans &t, float eta) {   // rtrans.h:262-318
    if (t.etaFixed) return;
    const float *trans = t.trans.data(), *diffTrans = t.diff.data();
    if (eta < 1) {
        trans += t.eta * t.alpha * t.theta;
        diffTrans += t.eta * t.alpha;
        eta = 1.0f / eta;
    }
    if (eta < t.etaMin) eta = t.etaMin;
    const float warpedEta = std::pow((eta - t.etaMin) / (t.etaMax - t.etaMin), 0.25f);
    std::vector<float> nt(t.alpha * t.theta), nd(t.alpha);
    const float dAlpha = 1.0f / (t.alpha - 1), dTheta = 1.0f / (t.theta - 1);
    for (size_t i = 0; i < t.alpha; ++i) {
        for (size_t j = 0; j < t.theta; ++j)
            nt[i * t.theta + j] = cubic3d(j * dTheta, i * dAlpha, warpedEta, trans, t.theta, t.alpha, t.eta);
        nd[i] = cubic2d(i * dAlpha, warpedEta, diffTrans, t.alpha, t.eta);
    }
    t.trans.swap(nt);
    t.diff.swap(nd);
    t.etaFixed = true;
}

void mtsg_rtrans_set_alpha(MtsgRTrans &t, float alpha) {   // rtrans.h:327-360
    if (t.alphaFixed) return;
    const float warpedAlpha = std::pow((alpha - t.alphaMin) / (t.alphaMax - t.alphaMin), 0.25f);
    std::vector<float> nt(t.theta), nd(1);
    const float dTheta = 1.0f / (t.theta - 1);
    for (size_t i = 0; i < t.theta; ++i) nt[i] = cubic2d(i * dTheta, warpedAlpha, t.trans.data(), t.theta, t.alpha);
    nd[0] = cubic1d(warpedAlpha, t.diff.data(), t.alpha, 0.0f, 1.0f);
    t.trans.swap(nt);
    t.diff.swap(nd);
    t.alphaFixed = true;
}

// RoughTransmittance::eval / evalDiffuse on a table reduced by setEta (rtrans.h:179-247)
float mtsg_rtrans_eval(const MtsgRTrans &t, float cosTheta, float alpha) {
    const float warpedCosTheta = std::pow(std::fabs(cosTheta), 0.25f);
    if (!(cosTheta >= 0)) return 0.f;
    float result;
    if (t.alphaFixed) {
        result = cubic1d(warpedCosTheta, t.trans.data(), t.theta, 0.0f, 1.0f);
    } else {
        const float warpedAlpha = std::pow((alpha - t.alphaMin) / (t.alphaMax - t.alphaMin), 0.25f);
        result = cubic2d(warpedCosTheta, warpedAlpha, t.trans.data(), t.theta, t.alpha);
    }
    return fmin_std(1.0f, fmax_std(0.0f, result));
}

float mtsg_rtrans_eval_diffuse(const MtsgRTrans &t, float alpha) {
    float result;
    if (t.alphaFixed) {
        result = t.diff[0];
    } else {
        const float warpedAlpha = std::pow((alpha - t.alphaMin) / (t.alphaMax - t.alphaMin), 0.25f);
        result = cubic1d(warpedAlpha, t.diff.data(), t.alpha, 0.0f, 1.0f);
    }
    return fmin_std(1.0f, fmax_std(0.0f, result));
}

int mtsg_rtrans_check(const MtsgRTrans &t, float eta, float alphaMin, float alphaMax, std::string &err) {
    char buf[320];
    float e = eta < 1 ? 1 / eta : eta;   // checkEta (rtrans.h:380-388)
    if (e < t.etaMin || e > t.etaMax) {
        std::snprintf(buf, sizeof buf, "Error: the requested relative index of refraction eta=%f is outside of the "
                      "supported range [%f, %f]! Please update your  scene so that it uses realistic IOR values.",
                      e, t.etaMin, t.etaMax);
        err = buf;
        return MTSGPU_EINVAL;
    }
    for (float a : {alphaMin, alphaMax}) {   // checkAlpha (rtrans.h:371-378)
        if (a < t.alphaMin || a > t.alphaMax) {
            std::snprintf(buf, sizeof buf, "Error: the requested roughness value alpha=%f is outside of the "
                          "supported range [%f, %f]! Please scale  your roughness value/texture to lie within "
                          "this range.", a, t.alphaMin, t.alphaMax);
            err = buf;
            return MTSGPU_EINVAL;
        }
    }
    return MTSGPU_OK;
}
