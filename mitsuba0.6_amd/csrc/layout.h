// layout.h -- HBM layout of a configured scene, shared by the host builder
// (scene_build.cpp) and the gfx950 kernels (path_kernel.hip).
//
// Everything is flat SoA/AoS arrays addressed by 32-bit indices:
//   nodes     BVH2, 64 B per node, both children's boxes in one node (one
//             node fetch = 4 x 16 B loads, tests two boxes)
//   tris      48 B per primitive in BVH leaf order: the reference's TriAccel
//             (triaccel.h:36-51) with {shapeIndex, primIndex} replaced by the
//             global primitive id (tie-break key) and the shape id
//   prim_vtx  per global primitive: vertex ids (global) + shape id
//   dpdu      per global primitive: UV tangent (trimesh.cpp:683-739) or p1-p0
//   vertices  positions / shading normals (zero-filled where a shape has none)
#pragma once
#include <stdint.h>
#include <hip/hip_vector_types.h>   // float4 of MtsgWave (host and device)

#define MTSG_MAX_STACK 64     // BVH builder keeps depth < MTSG_MAX_STACK
#define MTSG_LEAF_MAX 8       // primitives per leaf
#define MTSG_SOBOL_DIMS 1024
#define MTSG_SOBOL_SIZE 52
#define MTSG_FILTER_RES 31
#define MTSG_BLOCK_SIZE 32
#define MTSG_GATHER_HMAX 4   // film_gather<H> instantiations: footprints up to 9x9 pixels
#define MTSG_SCAN_MAX 64      // primitives up to which SCENE_LDS scenes scan instead of traversing

// node child reference: >= 0 inner node index; < 0 leaf: ~ref = first << 4 | count
static inline int32_t mtsg_leaf_ref(uint32_t first, uint32_t count) {
    return ~(int32_t)((first << 4) | count);
}

struct MtsgNode {            // 64 B (Aila-Laine layout)
    float c0lox, c0hix, c0loy, c0hiy;
    float c1lox, c1hix, c1loy, c1hiy;
    float c0loz, c0hiz, c1loz, c1hiz;
    int32_t c0, c1, pad0, pad1;
};

// The same BVH2 node with its child boxes as IEEE half floats rounded outward
// (lo toward -inf, hi toward +inf), so a box never shrinks and every exact
// triangle / shape test, hence every hit, is unchanged; 32 B, two 16 B loads.
// box[k] packs two halves (low half first) in MtsgNode's order:
// {c0lox c0hix}{c0loy c0hiy}{c1lox c1hix}{c1loy c1hiy}{c0loz c0hiz}{c1loz c1hiz}
struct MtsgHNode {
    uint32_t box[6];
    int32_t c0, c1;
};

// The BVH2 collapsed to a 4-wide BVH (each node's children are its BVH2
// node's grandchildren where those are inner nodes), child boxes as halves
// rounded outward like MtsgHNode: 64 B, four 16 B loads, half the node levels.
// box[3j .. 3j+2] = child j's {lox hix}{loy hiy}{loz hiz}; child[j]: a node
// index (> 0), a leaf reference (< 0, mtsg_leaf_ref) or 0 (no child).  Host
// export only (mtsgpu_bvh_host): the device traverses the BVH2
struct MtsgQNode {
    uint32_t box[12];
    int32_t child[4];
};

struct MtsgTri {             // 48 B
    uint32_t k;
    float n_u, n_v, n_d;
    float a_u, a_v, b_nu, b_nv;
    float c_nu, c_nv;
    uint32_t prim;           // global primitive index (shape order, triangle order)
    uint32_t shape;
};

enum {
    MTSG_F_NULL = 0x00001, MTSG_F_DIFF_REFL = 0x00002, MTSG_F_DIFF_TRANS = 0x00004,
    MTSG_F_GLOSSY_REFL = 0x00008, MTSG_F_GLOSSY_TRANS = 0x00010, MTSG_F_DELTA_REFL = 0x00020,
    MTSG_F_DELTA_TRANS = 0x00040, MTSG_F_FRONT = 0x01000, MTSG_F_BACK = 0x02000
};
#define MTSG_F_SMOOTH (MTSG_F_DIFF_REFL | MTSG_F_DIFF_TRANS | MTSG_F_GLOSSY_REFL | MTSG_F_GLOSSY_TRANS)
#define MTSG_F_TRANSMISSION (MTSG_F_DIFF_TRANS | MTSG_F_GLOSSY_TRANS | MTSG_F_DELTA_TRANS | MTSG_F_NULL)
#define MTSG_F_DELTA (MTSG_F_NULL | MTSG_F_DELTA_REFL | MTSG_F_DELTA_TRANS)

struct MtsgTex {             // Texture2D + checkerboard (texture.cpp:112-121, checkerboard.cpp)
    int32_t type;            // MTSGPU_TEX_*: 0 = the BSDF's constant value
    float c0[3], c1[3];
    float uoff, voff, uscale, vscale;
};

struct MtsgBsdf {            // configured BSDF (after ctor + configure)
    int32_t type, flags, distr, sample_visible;
    float alpha_u, alpha_v;  // texture average, clamped (microfacet.h:89-97)
    float eta, inv_eta;      // roughdielectric / roughplastic
    float refl[3], spec_r[3], spec_t[3], eta3[3], k3[3];
    float pad;
    // roughplastic (roughplastic.cpp:255-300): refl = diffuseReflectance
    float inv_eta2, spec_weight;
    int32_t nonlinear;
    int32_t rt_ext, rt_int;          // offsets (floats) into MtsgDeviceScene::rtrans
    int32_t rt_theta, rt_alpha;      // table sizes
    int32_t rt_alpha_fixed;          // external table reduced to 1D (constant alpha)
    float rt_alpha_min, rt_alpha_max;
    MtsgTex refl_tex, alpha_tex;     // textured reflectance / alpha (type 0: constant)
    // plastic (plastic.cpp:186-216): m_fdrInt, m_fdrExt (fresnelDiffuseReflectance)
    float fdr_int, fdr_ext;
    // twosided (twosided.cpp): record indices of the front / back nested BSDFs
    int32_t nested[2];
};

enum { MTSG_EMITTER_AREA = 0, MTSG_EMITTER_ENVMAP = 1, MTSG_EMITTER_CONSTANT = 2 };
enum { MTSG_FEAT_ENV = 1, MTSG_FEAT_EXT = 2, MTSG_FEAT_ANA = 4,
       MTSG_FEAT_DIFF = 8,     // DIFF: every BSDF is diffuse (path megakernel, FEAT 0 scenes only)
       // BSDF-set specialisation of the megakernel (dbsdf.h BSet): every rough
       // BSDF uses GGX / no roughdielectric / no roughconductor in the scene
       MTSG_FEAT_GGX = 16, MTSG_FEAT_NORD = 32, MTSG_FEAT_NORC = 64,
       MTSG_FEAT_INL = 128,     // microfacet / Fresnel helpers inline (the wavefront per-type kernels)
       MTSG_FEAT_NOSTRICT = 256,     // megakernel BSDF-set variants: strictNormals off (capi.cpp picks the generic kernel otherwise)
       MTSG_FEAT_NOREFN = 512 };     // BSDF-set variants of scenes lit by a (non-constant) envmap alone: no area
                                     // light and no constant emitter, so DirectSamplingRecord::refN is never read
enum { MTSG_INTEGRATOR_PATH = 0, MTSG_INTEGRATOR_DIRECT = 1, MTSG_INTEGRATOR_VOLPATH = 2 };   // = MTSGPU_INTEGRATOR_*
enum { MTSG_SAMPLER_SOBOL = 0, MTSG_SAMPLER_INDEPENDENT = 1, MTSG_SAMPLER_SFMT_REPLAY = 2,
       MTSG_SAMPLER_SFMT_BLOCKS = 3 };    // = MTSGPU_SAMPLER_*

struct MtsgShape {
    int32_t bsdf, emitter, has_normals, has_uv;
    int32_t kind;            // MTSGPU_SHAPE_* (0: triangle mesh)
    int32_t analytic;        // index into MtsgDeviceScene::analytic, -1: triangle mesh
};

// Analytic shapes (shapes/rectangle.cpp, disk.cpp, sphere.cpp): one primitive
// each; its TriAccel slot carries k = MTSG_K_ANALYTIC and the record index in
// the n_u bits.  Static per-shape quantities the plugins derive in their
// constructors / configure() are precomputed on the host.
#define MTSG_K_ANALYTIC 4u
enum { MTSG_SHAPE_TRIMESH = 0, MTSG_SHAPE_RECTANGLE = 1, MTSG_SHAPE_DISK = 2, MTSG_SHAPE_SPHERE = 3 };   // = MTSGPU_SHAPE_*
struct MtsgAnalytic {        // 240 B
    int32_t type;            // MTSGPU_SHAPE_RECTANGLE / _DISK / _SPHERE
    int32_t flip;            // sphere m_flipNormals
    float radius;            // sphere m_radius
    float inv_area;          // m_invSurfaceArea
    float to_world[16];      // m_objectToWorld (row-major)
    float to_obj[16];        // m_worldToObject = its inverse as the Transform carries it
    float center[3];         // sphere m_center
    float n[3];              // rectangle m_frame.n; disk normalize(trafo(Normal(0,0,1)))
    float fs[3], ft[3];      // rectangle m_frame.s, m_frame.t
    float dpdu[3], dpdv[3];  // rectangle m_dpdu, m_dpdv
};

struct MtsgEmitter {
    int32_t type, shape;
    uint32_t tri_first, tri_count;   // global prim range of the emitting mesh
    uint32_t cdf_offset;             // into area_cdf (tri_count + 1 entries)
    float inv_area, weight, pad;
    float radiance[3], pad2;
};

struct MtsgCamera {
    float sample_to_camera[16];
    float to_world[16];
    float inv_res_x, inv_res_y, near_clip, far_clip;
    float dx[3], dy[3];
};

struct MtsgFilter {
    float radius, scale;
    int32_t border, type;
    float values[MTSG_FILTER_RES + 1];
};

// Environment emitter (emitters/envmap.cpp): the reference's TMIPMap<Spectrum,
// SpectrumHalf> pyramid (render/mipmap.h) with every level stored as RGB halves
// (+1 pad half: one 8-byte load per texel), levels concatenated; the
// marginal/conditional luminance CDFs of configure() (envmap.cpp:261-321).
#define MTSG_ENV_MAX_LEVELS 18      // sides < 65536 (envmap.cpp:160-162)
#define MTSG_EWA_LUT 64             // MTS_MIPMAP_LUT_SIZE (mipmap.h:37)
struct MtsgEnv {
    int32_t emitter;                // index into the emitter list
    int32_t constant;               // 1: ConstantBackgroundEmitter (constant.cpp): `radiance` only
    float radiance[3];
    int32_t levels;
    int32_t w0, h0;
    float normalization;            // m_normalization
    float pixel_x, pixel_y;         // m_pixelSize
    float scale;                    // m_scale
    float center[3], radius;        // m_sceneBSphere
    float to_world[9], to_local[9]; // vector part of toWorld and of its inverse
    float inv_ln2;                  // math::log2 (math.cpp:103-106)
    float max_aniso;                // 10 (envmap.cpp:142)
    int32_t lw[MTSG_ENV_MAX_LEVELS], lh[MTSG_ENV_MAX_LEVELS];
    uint32_t loff[MTSG_ENV_MAX_LEVELS];
    float ratio_x[MTSG_ENV_MAX_LEVELS], ratio_y[MTSG_ENV_MAX_LEVELS];
    float lut[MTSG_EWA_LUT];
    const uint16_t *texels;         // 4 halves per texel
    const float *cdf_rows;          // h0 + 1
    const float *cdf_cols;          // h0 * (w0 + 1)
    const float *row_weights;       // h0
    // guide tables of the two CDF searches (cutpoint method): for u in [k/G, (k+1)/G)
    // std::lower_bound(cdf, u) lies in [guide[k], guide[k+1]]; null: full-range search
    const uint16_t *guide_rows;     // (1 << guide_rbits) + 1
    const uint16_t *guide_cols;     // h0 * ((1 << guide_cbits) + 1)
    uint32_t guide_rbits, guide_cbits;
};

struct MtsgDeviceScene {
    const MtsgNode *nodes;
    const MtsgHNode *hnodes;    // the same nodes, half-float boxes (large scenes)
    const MtsgTri *tris;
    const uint32_t *prim_vtx;   // 4 per primitive: v0, v1, v2, shape
    const float *dpdu;          // 3 per primitive
    const float *positions;     // 3 per vertex
    const float *normals;       // 3 per vertex
    const MtsgShape *shapes;
    const MtsgBsdf *bsdfs;
    const MtsgEmitter *emitters;
    const float *area_cdf;
    const float *em_cdf;        // num_emitters + 1
    const uint32_t *sobol;      // MTSG_SOBOL_DIMS * MTSG_SOBOL_SIZE
    const MtsgEnv *env;         // device copy, or null without an environment emitter
    const float *rtrans;        // roughplastic rough-transmittance slices (rtrans.h)
    const float *texcoords;     // 2 per vertex (textured scenes), else null
    const MtsgAnalytic *analytic;   // analytic shape records, or null
    uint32_t num_emitters, num_prims;
    float em_norm;
    int32_t env_emitter;        // index of the environment emitter, -1: none
    float aabb_min[3], aabb_max[3];
    MtsgCamera cam;
};

// look_up tables for one film resolution (host-precomputed GF(2) inverse)
struct MtsgLookup {
    uint32_t m;                 // log2 resolution (0: identity enumeration)
    uint32_t inv[32];
    uint32_t ycol[64];
};

// The wavefront engine (wf_kernel.hip).  One bounce = the
// per-type shade kernels, each over its queue of path slots (the slots whose
// closest-hit ray hit a shape whose BSDF is of that type, or missed: kind
// MISS), then one trace kernel over the two ray queues the shade kernels
// appended to, which writes the hit records by slot and sorts the slots into
// the next bounce's per-type queues.  Every queue is split into
// MTSG_WF_REGIONS regions (appender block b uses region b % regions), each of
// capacity `cap` = slots, so one wave's append is one atomic on one of 8
// counters and a region can never overflow; consumers walk the concatenation.
#define MTSG_WF_STATE_VECS 8          // float4 state vectors per slot (AoS: one slot = 128 B)
#define MTSG_WF_HIT_VECS 6            // float4 per precomputed hit record (dpath.h hit_store)
#define MTSG_WF_NONE 0xffffffffu      // hit record prim: no hit
#define MTSG_WF_REGIONS 8
#ifndef MTSG_WF_LDS_STACK
#define MTSG_WF_LDS_STACK 12          // trace kernel: traversal stack entries per lane in LDS (deeper: HBM)
#endif
// shade kinds: the BSDF type at the vertex (wf_kernel.hip specialises each)
enum { MTSG_WK_MISS = 0, MTSG_WK_DIFF = 1, MTSG_WK_RC = 2, MTSG_WK_RD = 3, MTSG_WK_RP = 4, MTSG_WK_GEN = 5,
       MTSG_WK_KINDS = 6 };
#define MTSG_WF_QUEUES (2 + MTSG_WK_KINDS)   // closest rays, shadow rays, the kinds' slot queues
struct MtsgWave {
    float4 *state;                    // [slots][MTSG_WF_STATE_VECS]
    float4 *ray[2];                   // [parity][2 (closest, shadow)][regions][cap][2] {o, mint}, {d, maxt}
    uint32_t *rslot[2];               // [parity][2][regions][cap] the slot of each ray
    uint32_t *cls[2];                 // [parity][kinds][regions][cap] slot queues
    uint32_t *cnt;                    // [parity][MTSG_WF_QUEUES][regions] entries
    float4 *hit;                      // [slots] {t, u, v, prim (TriAccel slot with analytic shapes) | MTSG_WF_NONE}
    uint32_t *occl;                   // [slots] shadow results
    uint32_t *live;                   // [2 parities] live slots after the bounce's shade kernels
    uint2 *ovf;                       // trace stack overflow: [trace lanes][ovf_depth]
    const uint32_t *shape_kind;       // [shapes] MTSG_WK_* of the shape's BSDF
    uint32_t slots;
    uint32_t cap, cap_cls;            // entries per region of a ray queue / of a kind queue (capi.cpp wf_caps)
    uint32_t parity;                  // bounce index & 1
    uint32_t seed;                    // first bounce: the MISS kernel takes every slot (identity queue)
    uint32_t ovf_depth;
    float4 *hitrec;                   // [slots][MTSG_WF_HIT_VECS] hit records formed by wf_trace, or null
    uint32_t hitrec_uv;               // textured scene: the records carry UVs
};

struct MtsgLaunch {
    MtsgDeviceScene scene;
    MtsgFilter filter;
    MtsgLookup lut;
    float resolution;           // sobol m_resolution
    float diff_scale;           // 1/sqrt(sampleCount): ray differential scale (integrator.cpp:144-145)
    uint32_t scramble;          // sobol m_scramble (after TEA), low 32 bits used by sampleSingle
    uint64_t scramble64;
    uint32_t spp;
    int32_t max_depth, rr_depth, strict_normals, hide_emitters, has_alpha;
    int32_t film_w, film_h, fw, fh;   // image size and film size incl. borders
    uint32_t x0, y0, width, height;
    uint32_t row_block, row_stride, row_phase;
    uint32_t tile_shard;              // MTSGPU_FLAG_TILE_SHARD: row_stride/row_phase interleave 8x8 tiles
    // work decomposition: items = (sample j in [j0, j0 + chunk_spp)) x (compact pixel p in [0, num_pixels))
    uint32_t tiles_x;                 // 8x8 pixel tiles across the window
    uint32_t num_pixels;              // compact pixels incl. padding of partial tiles
    uint32_t j0, chunk_spp;
    uint32_t round_shift;             // megakernel: a lane renders 2^round_shift samples of a pixel in a row (dmega.h, capi.cpp run_shift)
    uint64_t num_items;
    // Sobol direction numbers as 4-bit lookup tables: nib[dim][c][v] = XOR of the
    // columns 4c..4c+3 selected by v (same product as sobolseq.h:43-57)
    const uint32_t *sobol_nib;        // MTSG_SOBOL_DIMS * MTSG_NIBBLES * 16 words
    uint32_t lds_dims;                // dims [0, lds_dims) staged in LDS
    uint32_t nibbles;                 // 8 (index < 2^32) or MTSG_NIBBLES
    uint32_t stack_depth;             // LDS traversal stack entries per lane
    uint32_t num_nodes;               // BVH2 inner nodes
    uint32_t scene_lds;               // 1: nodes + TriAccel staged in LDS (small scenes)
    uint32_t waves;                   // kernel variant: waves per SIMD it is compiled for (3 or 4)
    uint32_t ext;                     // kernel variant: roughplastic / textured BSDFs present
    uint32_t ana;                     // kernel variant: analytic shapes present (implies ext)
    uint32_t all_diffuse;             // kernel variant: every BSDF is diffuse (MTSG_FEAT_DIFF)
    uint32_t bset;                    // the scene's MTSG_FEAT_GGX / NORD / NORC bits (capi.cpp)
    uint32_t xcds;                    // XCDs the device's CUs span (workgroup -> XCD remap; 1: none)
    // MTSGPU_FLAG_KDTREE (wavefront engine): wf_trace traverses the reference's kd-tree
    const uint32_t *kd_nodes;         // KDNode words (2 per node), null: the BVH
    const uint32_t *kd_indices;
    const MtsgTri *kd_tris;           // TriAccel records in leaf-list order (kd_tris[e]: primitive kd_indices[e])
    uint32_t scan;                    // tiny scene: linear TriAccel scan instead of the BVH (SCENE_LDS only)
    const MtsgTri *scan_tris;         // the scan's TriAccel records grouped by projection axis k = 0, 1, 2
    uint32_t scan_n[6];               // and within k by n_u = n_v = 0 (2k: general, 2k+1: axis-aligned plane);
                                      // degenerate k = 3 records dropped; counts per group
    uint32_t num_verts, num_shapes;   // sizes of the triangle data SCENE_LDS kernels stage in LDS
    int32_t integrator;               // MTSGPU_INTEGRATOR_*
    uint32_t sampler;                 // MTSGPU_SAMPLER_*
    // the `direct` integrator (direct.cpp:128-143): sample counts, MIS fractions and
    // weights, and the sampler's 2D arrays (dims [5, array_end))
    uint32_t lum_samples, bsdf_samples;
    float weight_lum, weight_bsdf, frac_lum, frac_bsdf;
    uint32_t lum_dim, bsdf_dim, array_end;
    // the SFMT replay samplers (MTSGPU_SAMPLER_SFMT_*): lane u renders unit u's pixels
    // order[unit_start[u] .. unit_start[u + 1]) (x | y << 16, crop-relative), all
    // samples of a pixel in turn, drawing from stream sfmt[u * MTSG_SFMT_WORDS ..]
    uint32_t replay, units;
    const uint32_t *order, *unit_start;
    uint32_t *sfmt;
    float *contrib;                   // the samples' splat records, slot (j - j0) * num_pixels + pix (film_slot):
                                      // box filter one float4 {L.rgb, own-pixel weight, alpha in its sign};
                                      // gather mode two, one 32 B sector: {L.rgb, sx (alpha in its sign)},
                                      // {sy (negative: an invalid sample), 0, 0, 0}
    float *film_own;                  // fw*fh*5: own-pixel sums (ordered reduction), or the gathered film
    double *film_spill;               // fw*fh*5: splats into other pixels (box filter only), double atomics:
                                      // a pixel's few neighbour splats sum exactly, in any order (dpath.h film_splat)
    // gather mode (filters whose footprint covers neighbours, e.g. gaussian): the kernels store
    // each sample's value and position; film_gather<H> forms every pixel's sum in a fixed order
    uint32_t gather;                  // 1: gather mode
    uint32_t gather_h;                // largest footprint offset from a sample's pixel (<= MTSG_GATHER_HMAX)
    float *samples;                   // optional per-sample records
    unsigned long long *counters;     // [0] samples [1] rays [2] shadow [3] pathlen [4] nodes [5] tests
                                      // [6] dim errors [7] hits [9] nee [10] sobol words
};

#ifndef MTSG_MIN_RUNS
#define MTSG_MIN_RUNS 100   // sample runs per lane the megakernel's run length leaves (capi.cpp run_shift)
#endif

#define MTSG_NIBBLES 13
