// scene_build.h -- host-side configure() of a Mitsuba scene description into
// the HBM layout of layout.h (normals, tangents, TriAccel, emitter CDFs,
// camera matrices, filter LUT, Sobol tables, BVH).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/mtsgpu.h"
#include "layout.h"

struct HostScene {
    std::vector<MtsgNode> nodes;
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
};

// Returns MTSGPU_OK or an error code; `err` receives the message.
int mtsg_configure_scene(const mtsgpu_scene_desc *desc, HostScene &out, std::string &err);
int mtsg_configure_filter(int32_t type, float param, MtsgFilter &f, std::string &err);
// Sobol: 1024 x 52 matrices regenerated from the Joe-Kuo parameters, and the
// look_up GF(2) tables for resolution 2^m.
const std::vector<uint32_t> &mtsg_sobol_matrices();
void mtsg_sobol_lookup_table(uint32_t m, MtsgLookup &lut);
uint64_t mtsg_sample_tea(uint32_t v0, uint32_t v1, int rounds);
