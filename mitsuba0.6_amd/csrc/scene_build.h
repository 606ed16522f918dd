// scene_build.h -- host-side configure() of a Mitsuba scene description into
// the HBM layout of layout.h (normals, tangents, TriAccel, emitter CDFs,
// camera matrices, filter LUT, Sobol tables, BVH).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/mtsgpu.h"
#include "layout.h"

// RoughTransmittance table (rtrans.h) and its eta/alpha reductions (rtrans_host.cpp)
struct MtsgRTrans {
    size_t eta = 0, alpha = 0, theta = 0;
    float etaMin = 0, etaMax = 0, alphaMin = 0, alphaMax = 0;
    bool etaFixed = false, alphaFixed = false;
    std::vector<float> trans, diff;
};
int mtsg_rtrans_load(const void *data, size_t bytes, MtsgRTrans &t, std::string &err);
void mtsg_rtrans_set_eta(MtsgRTrans &t, float eta);
void mtsg_rtrans_set_alpha(MtsgRTrans &t, float alpha);
float mtsg_rtrans_eval(const MtsgRTrans &t, float cosTheta, float alpha);
float mtsg_rtrans_eval_diffuse(const MtsgRTrans &t, float alpha);
int mtsg_rtrans_check(const MtsgRTrans &t, float eta, float alphaMin, float alphaMax, std::string &err);

struct HostScene {
    std::vector<MtsgNode> nodes;
    std::vector<MtsgHNode> hnodes;   // the same BVH, half-float boxes
    std::vector<MtsgQNode> qnodes;   // the same BVH collapsed to 4-wide nodes (mtsg_build_qnodes, host export only)
    uint32_t qnode_depth = 0;        // inner-node levels of qnodes
    std::vector<MtsgTri> tris;
    std::vector<uint32_t> prim_vtx;
    std::vector<float> dpdu, positions, normals;
    std::vector<MtsgShape> shapes;
    std::vector<MtsgBsdf> bsdfs;
    std::vector<MtsgEmitter> emitters;
    std::vector<float> area_cdf, em_cdf;
    float em_norm = 0;
    float aabb_min[3], aabb_max[3];
    MtsgCamera cam;
    uint32_t film_w = 0, film_h = 0;
    uint32_t bvh_depth = 0;
    // environment emitter (env.emitter < 0: none); pointers in `env` are set at upload
    MtsgEnv env;
    std::vector<uint16_t> env_texels;
    std::vector<float> env_cdf_rows, env_cdf_cols, env_row_weights;
    std::vector<uint16_t> env_guide_rows, env_guide_cols;   // MtsgEnv::guide_* (empty: no guide)
    // roughplastic tables (MtsgBsdf::rt_ext / rt_int offsets) and per-vertex UVs
    std::vector<float> rtrans, texcoords;
    bool ext = false;   // roughplastic or textured BSDFs: the MTSG_FEAT_EXT kernel variant
    std::vector<MtsgAnalytic> analytic;   // rectangle / disk / sphere records (MTSG_FEAT_ANA variant)
};

// Returns MTSGPU_OK or an error code; `err` receives the message.
int mtsg_configure_scene(const mtsgpu_scene_desc *desc, HostScene &out, std::string &err);
void mtsg_build_qnodes(HostScene &S);   // host export only (mtsgpu_bvh_host)
int mtsg_configure_filter(int32_t type, float param, MtsgFilter &f, std::string &err);
// Sobol: 1024 x 52 matrices regenerated from the Joe-Kuo parameters, and the
// look_up GF(2) tables for resolution 2^m.
const std::vector<uint32_t> &mtsg_sobol_matrices();
void mtsg_sobol_lookup_table(uint32_t m, MtsgLookup &lut);
uint64_t mtsg_sample_tea(uint32_t v0, uint32_t v1, int rounds);
