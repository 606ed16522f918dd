/*
 * mtsgpu.h -- C-ABI of the MI355X-native `path` integrator (libmtsgpu.so).
 *
 * This is the drop-in boundary for Mitsuba 0.6's unidirectional path tracer.
 * The reference renders through the Integrator plugin API:
 *
 *   SamplingIntegrator::render      src/librender/integrator.cpp:95-129
 *   SamplingIntegrator::renderBlock src/librender/integrator.cpp:140-188
 *   MIPathTracer::Li                src/integrators/path/path.cpp:119-294
 *
 * and a plugin is loaded through `extern "C" CreateInstance/GetDescription`
 * (include/mitsuba/core/cobject.h:99-107, src/libcore/plugin.cpp:62-123).
 * A `gpupath` plugin shim overrides render() and calls
 * the entry points below with plain pointers and sizes: no C++ or torch types
 * cross this boundary, every call returns an int status, nothing throws.
 *
 * Ownership: the caller owns every host buffer; the library copies what it
 * needs during mtsgpu_upload_scene.  One context per host thread.
 *
 * The scene description is the reference's scene *after plugin construction
 * and before configure()*: world-space triangle meshes (the TriMesh the
 * shape plugins produce), BSDF/emitter parameters, sensor, film and sampler
 * properties.  Everything the reference derives in configure() (vertex
 * normals, UV tangents, TriAccel, emitter CDFs, camera matrices, filter LUT)
 * is derived by the library itself, following the cited reference code.
 */
#ifndef MTSGPU_H
#define MTSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTSGPU_ABI_VERSION 8

/* ---- status codes ------------------------------------------------------ */
enum {
    MTSGPU_OK = 0,
    MTSGPU_EINVAL = -1,   /* bad argument / inconsistent scene (reference: Log(EError)) */
    MTSGPU_EHIP = -2,     /* HIP runtime error                                      */
    MTSGPU_ENOMEM = -3,   /* device or host allocation failed                        */
    MTSGPU_ESTATE = -4,   /* call out of order (e.g. render before upload)           */
    MTSGPU_EDIM = -5,     /* Sobol dimension table exhausted (sobol.cpp:224,238)     */
    MTSGPU_ECANCEL = -6,  /* *cancel flag was set (Integrator::cancel)               */
    MTSGPU_ENODEV = -7,   /* no usable gfx950 device                                 */
    MTSGPU_ENOENT = -8    /* mtsgpu_xml_bsdf_ex: the id is not in the scene file     */
};

/* ---- scene description (POD) ------------------------------------------- */
enum { /* BSDF plugins on the path (src/bsdfs) */
    MTSGPU_BSDF_DIFFUSE = 0,         /* diffuse.cpp         */
    MTSGPU_BSDF_ROUGHCONDUCTOR = 1,  /* roughconductor.cpp  */
    MTSGPU_BSDF_ROUGHDIELECTRIC = 2, /* roughdielectric.cpp */
    MTSGPU_BSDF_ROUGHPLASTIC = 3,    /* roughplastic.cpp + rtrans.h */
    MTSGPU_BSDF_CONDUCTOR = 4,       /* conductor.cpp  (smooth, delta reflection)        */
    MTSGPU_BSDF_DIELECTRIC = 5,      /* dielectric.cpp (smooth, delta refl. + transm.)   */
    MTSGPU_BSDF_PLASTIC = 6,         /* plastic.cpp    (delta coating + diffuse base)    */
    MTSGPU_BSDF_TWOSIDED = 7         /* twosided.cpp   (wraps nested[0], nested[1])      */
};

enum { /* MicrofacetDistribution::EType (src/bsdfs/microfacet.h:48-57) */
    MTSGPU_DISTR_BECKMANN = 0,
    MTSGPU_DISTR_GGX = 1,
    MTSGPU_DISTR_PHONG = 2
};

enum { /* Texture plugins a BSDF parameter may hold (src/textures) */
    MTSGPU_TEX_NONE = 0,             /* the constant value of the parameter         */
    MTSGPU_TEX_CHECKERBOARD = 1      /* checkerboard.cpp (Texture2D uv transform)   */
};

typedef struct {                    /* Texture2D (librender/texture.cpp:81-121)    */
    int32_t type;                   /* MTSGPU_TEX_*                                */
    float color0[3], color1[3];     /* checkerboard 'color0' (.4), 'color1' (.2)   */
    float uoffset, voffset;         /* 'uoffset', 'voffset' (0)                    */
    float uscale, vscale;           /* 'uscale'/'vscale' (default 'uvscale' = 1)   */
} mtsgpu_texture_desc;

typedef struct {
    int32_t type;                   /* MTSGPU_BSDF_*                               */
    int32_t distribution;           /* MTSGPU_DISTR_* (rough BSDFs)                */
    int32_t sample_visible;         /* 'sampleVisible' (default 1)                 */
    int32_t ensure_energy_conservation; /* 'ensureEnergyConservation' (default 1)   */
    float alpha_u, alpha_v;         /* 'alpha' / 'alphaU','alphaV' as given        */
    float reflectance[3];           /* diffuse 'reflectance'                       */
    float specular_reflectance[3];  /* all but diffuse: 'specularReflectance' (1)  */
    float specular_transmittance[3];/* roughdielectric (default 1)                 */
    float eta[3], k[3];             /* (rough)conductor: RGB eta/k, before /extEta */
    float ext_eta;                  /* roughconductor 'extEta' (air = 1.000277)    */
    float int_ior, ext_ior;         /* (rough)dielectric (bk7 = 1.5046, air);      */
                                    /* (rough)plastic (polypropylene = 1.49, air)  */
    /* (rough)plastic (roughplastic.cpp:197-300, plastic.cpp:144-216) */
    float diffuse_reflectance[3];   /* 'diffuseReflectance' (default 0.5)          */
    int32_t nonlinear;              /* 'nonlinear' (default 0)                     */
    const void *rtrans_data;        /* the bytes of data/microfacet/<distr>.dat    */
    uint64_t rtrans_bytes;          /* (RoughTransmittance, rtrans.h:46-150)       */
    /* textured parameters; type NONE -> the constant field above is used */
    mtsgpu_texture_desc reflectance_tex;   /* diffuse 'reflectance' / roughplastic 'diffuseReflectance' */
    mtsgpu_texture_desc alpha_tex;         /* rough*: isotropic 'alpha' (value = texture average)       */
    /* twosided (twosided.cpp:63-110): indices into the scene's bsdfs of the
       front-side BSDF and of the back-side one (-1: the front one is reused);
       nested BSDFs must be one-sided reflectors (diffuse, roughconductor,
       roughplastic, conductor, plastic): TwoSidedBRDF::configure raises otherwise */
    int32_t nested[2];
} mtsgpu_bsdf_desc;

enum { MTSGPU_EMITTER_AREA = 0,      /* area.cpp: on a shape (mesh_desc.emitter)          */
       MTSGPU_EMITTER_ENVMAP = 1,    /* envmap.cpp: lat-long image (env_* fields)          */
       MTSGPU_EMITTER_CONSTANT = 2   /* constant.cpp: uniform 'radiance' environment       */
};

typedef struct {
    int32_t type;                   /* MTSGPU_EMITTER_*                            */
    float radiance[3];              /* area.cpp 'radiance'                         */
    float sampling_weight;          /* 'samplingWeight' (emitter.cpp:103)          */
    /* envmap (envmap.cpp): linear RGB lat-long image, row-major, top row first  */
    const float *env_rgb;           /* 3*env_width*env_height floats, or NULL      */
    uint32_t env_width, env_height;
    float env_scale;                /* 'scale'                                     */
    float env_to_world[16];         /* row-major 4x4 'toWorld'                     */
    float env_to_world_inv[16];     /* its inverse as the reference's Transform    */
                                    /* carries it (transform.cpp); all zero: the   */
                                    /* library inverts env_to_world (Gauss-Jordan) */
} mtsgpu_emitter_desc;

enum { /* shape plugins (src/shapes) */
    MTSGPU_SHAPE_TRIMESH = 0,        /* obj / ply / serialized / cube: world-space triangles */
    MTSGPU_SHAPE_RECTANGLE = 1,      /* rectangle.cpp: [-1,1]^2 x {0} under 'toWorld'        */
    MTSGPU_SHAPE_DISK = 2,           /* disk.cpp: unit disk in z = 0 under 'toWorld'         */
    MTSGPU_SHAPE_SPHERE = 3          /* sphere.cpp: 'center', 'radius', optional 'toWorld'   */
};

typedef struct {
    const float *positions;         /* 3*num_vertices, world space                 */
    const float *normals;           /* 3*num_vertices or NULL                      */
    const float *texcoords;         /* 2*num_vertices or NULL                      */
    const uint32_t *indices;        /* 3*num_triangles                             */
    uint32_t num_vertices, num_triangles;
    int32_t bsdf;                   /* index into bsdfs, -1: Shape::configure default */
    int32_t emitter;                /* index into emitters (area), -1: none        */
    int32_t face_normals;           /* 'faceNormals'                               */
    int32_t flip_normals;           /* 'flipNormals'                               */
    /* analytic shapes (shape_type != TRIMESH) are one primitive each, intersected
       exactly as the plugin's rayIntersect does; positions/indices are unused */
    int32_t shape_type;             /* MTSGPU_SHAPE_*                              */
    int32_t has_to_world;           /* 'toWorld' given (sphere.cpp:113-121)        */
    float to_world[16];             /* row-major 'toWorld' (identity if absent)    */
    float to_world_inv[16];         /* its inverse as the reference's Transform    */
                                    /* carries it; all zero: the library inverts   */
    float center[3];                /* sphere 'center' (default 0)                 */
    float radius;                   /* sphere 'radius' (default 1)                 */
} mtsgpu_mesh_desc;

enum { MTSGPU_FOV_X = 0, MTSGPU_FOV_Y = 1, MTSGPU_FOV_DIAGONAL = 2,
       MTSGPU_FOV_SMALLER = 3, MTSGPU_FOV_LARGER = 4 };

typedef struct {                    /* perspective.cpp + librender/sensor.cpp      */
    float fov;                      /* degrees                                     */
    int32_t fov_axis;               /* MTSGPU_FOV_*                                */
    float near_clip, far_clip;      /* defaults 1e-2, 1e4                          */
    float to_world[16];             /* row-major camera-to-world                   */
    uint32_t film_width, film_height;
} mtsgpu_sensor_desc;

typedef struct {
    const mtsgpu_mesh_desc *meshes;       uint32_t num_meshes;
    const mtsgpu_bsdf_desc *bsdfs;        uint32_t num_bsdfs;
    const mtsgpu_emitter_desc *emitters;  uint32_t num_emitters; /* scene order */
    mtsgpu_sensor_desc sensor;
} mtsgpu_scene_desc;

/* ---- render parameters ------------------------------------------------- */
enum { MTSGPU_RFILTER_BOX = 0, MTSGPU_RFILTER_GAUSSIAN = 1 };

typedef struct {
    uint32_t spp;                   /* sampler 'sampleCount'                       */
    uint64_t scramble;              /* sobol 'scramble' (0: none)                  */
    int32_t max_depth;              /* 'maxDepth' (-1 = infinite)                  */
    int32_t rr_depth;               /* 'rrDepth' (5)                               */
    int32_t strict_normals;         /* 'strictNormals'                             */
    int32_t hide_emitters;          /* 'hideEmitters'                              */
    int32_t has_alpha;              /* film has an alpha channel (EOpacity)        */
    int32_t rfilter;                /* MTSGPU_RFILTER_*                            */
    float rfilter_param;            /* box: radius (0.5); gaussian: stddev (0.5)   */
    /* the film's crop window (hdrfilm cropOffsetX/Y, cropWidth/Height; film.cpp:
       35-43), image coordinates: the pixels rendered, and max(width, height)
       sets the Sobol resolution (Integrator::configureSampler, integrator.cpp:37-41) */
    uint32_t x0, y0, width, height;
    /* row interleave for tile sharding: render rows y with
       ((y - y0) / row_block) % row_stride == row_phase (stride 1 = all rows) */
    uint32_t row_block, row_stride, row_phase;
    const volatile int32_t *cancel; /* polled between launches, may be NULL        */
    uint32_t flags;                 /* MTSGPU_FLAG_*                               */
    /* the integrator plugin: MTSGPU_INTEGRATOR_PATH (path.cpp; max_depth, rr_depth)
       or MTSGPU_INTEGRATOR_DIRECT (direct.cpp:90-306): 'emitterSamples' and
       'bsdfSamples' (both default to 'shadingSamples' = 1); strict_normals and
       hide_emitters apply to both; MTSGPU_INTEGRATOR_VOLPATH (volpath.cpp) for
       scenes without participating media: path's parameters, with volpath's
       shadow segments (Scene::evalTransmittance), strictNormals test and
       path-length accounting */
    int32_t integrator;
    uint32_t emitter_samples, bsdf_samples;
    /* the sampler plugin: MTSGPU_SAMPLER_SOBOL (sobol.cpp; 'scramble') or
       MTSGPU_SAMPLER_INDEPENDENT (independent.cpp:51-116): uniform [0,1) draws
       from a per-(pixel, sample) counter-based stream in place of the
       reference's per-thread SFMT19937, whose values depend on the thread
       schedule; the film x/y must be below 65536 */
    int32_t sampler;
} mtsgpu_render_params;

enum { MTSGPU_INTEGRATOR_PATH = 0, MTSGPU_INTEGRATOR_DIRECT = 1, MTSGPU_INTEGRATOR_VOLPATH = 2 };
enum { MTSGPU_SAMPLER_SOBOL = 0, MTSGPU_SAMPLER_INDEPENDENT = 1,
       /* the reference's own independent sampler, replayed: SFMT19937 streams
          (random.cpp) cloned from Random(5489) as RenderJob does
          (renderjob.cpp:58-66), the crop's 32x32 blocks in BlockedImageProcess's
          spiral order (imageproc.cpp:43-80) and each block's pixels on its Hilbert
          curve (sfcurve.h, renderproc.cpp:79-81).  SFMT_REPLAY: one worker renders
          every block (`mitsuba -p 1`, sequential: for parity, not speed);
          SFMT_BLOCKS: block k is rendered by clone k (blocks in parallel).
          Whole crop only (row_stride 1); no direct-integrator sample arrays */
       MTSGPU_SAMPLER_SFMT_REPLAY = 2, MTSGPU_SAMPLER_SFMT_BLOCKS = 3 };

/* render flags */
#define MTSGPU_FLAG_TRAVERSAL_STATS 1u  /* count BVH node visits / TriAccel tests   */
/* execution engine of the path / volpath integrators (same per-sample results):
   the persistent megakernel or the wavefront pipeline (per-bounce ray queues);
   neither flag: the library's per-scene default */
#define MTSGPU_FLAG_WAVEFRONT 2u
#define MTSGPU_FLAG_MEGAKERNEL 4u
/* trace every ray through the reference's own SAH kd-tree (see
   mtsgpu_trace_rays_ex) instead of the BVH: exact-t ties then resolve as in
   the reference (the triangle tested last wins); runs in the wavefront engine,
   path / volpath, triangle scenes only */
#define MTSGPU_FLAG_KDTREE 8u
/* shard by 8x8 pixel tiles instead of row blocks: render the tiles t of the
   window's 8x8 tile grid (row-major, t = (ly / 8) * ceil(width / 8) + lx / 8)
   with t % row_stride == row_phase (row_block ignored).  Every rank then keeps
   whole 8x8 tiles at any rank count (the multi-GPU bench's unit) */
#define MTSGPU_FLAG_TILE_SHARD 16u

/* Film layout produced by mtsgpu_render: an ImageBlock of the full crop
 * (film_width+2b) x (film_height+2b) pixels, 5 floats each {R,G,B,alpha,w},
 * b = reconstruction-filter border (rfilter.cpp:50).  The buffer is
 * overwritten (zeroed first).  Summing the films of disjoint windows gives
 * the film of the union (the multi-GPU reduction). */

/* Optional per-sample record (parity / debugging), one per (pixel, sample) of
 * the window in row-major pixel order, sample-minor:
 * {Li.r, Li.g, Li.b, alpha, samplePos.x, samplePos.y, depth, flags}. */
#define MTSGPU_SAMPLE_RECORD_FLOATS 8

typedef struct {
    uint64_t samples;               /* Li() evaluations                            */
    uint64_t rays;                  /* closest-hit rays traced                     */
    uint64_t shadow_rays;           /* shadow rays traced                          */
    uint64_t path_length_sum;       /* sum of rRec.depth at exit (path.cpp:290)    */
    uint64_t node_visits;           /* BVH nodes visited (stats builds)            */
    uint64_t tri_tests;             /* TriAccel tests (stats builds)               */
    uint64_t hits;                  /* intersection records filled (stats builds)  */
    uint64_t nee_samples;           /* emitter samples drawn (stats builds)        */
    uint64_t sobol_reads;           /* direction-number words read, approx. (stats) */
    double kernel_ms;               /* device time of the render launches          */
} mtsgpu_stats;

typedef struct mtsgpu_ctx mtsgpu_ctx;

/* Create a context on HIP device `device` (-1: current). */
int mtsgpu_create(int device, mtsgpu_ctx **out);
/* Configure + upload a scene (copies everything; replaces any previous one). */
int mtsgpu_upload_scene(mtsgpu_ctx *ctx, const mtsgpu_scene_desc *scene);
/* Host-only (no device needed): run the configure() steps of upload_scene on
 * `scene` and report the first error as the reference would raise it
 * (Log(EError) message into msg[cap]).  Returns MTSGPU_OK or the error code. */
int mtsgpu_check_scene(const mtsgpu_scene_desc *scene, char *msg, size_t cap);

/* ---- the BSDF subtrees of a scene file (for the plugin shim) --------------
 * Host-only.  Inside Mitsuba, twosided's nested BSDFs and every BSDF's
 * textures are private children (src/bsdfs/twosided.cpp:198-210): a plugin
 * cannot reach them, but the scene's source file can
 * (Scene::getSourceFile, include/mitsuba/render/scene.h:1107).
 * mtsgpu_xml_bsdf_ex reads that file as SceneHandler does
 * (src/librender/scenehandler.cpp: $parameter substitution in every
 * attribute, <default>, <alias>, <include>, duplicate ids rejected) and
 * returns the tree below one <bsdf>:
 *   lookup MTSGPU_XML_BY_ID:    the <bsdf> with id `id`;
 *   lookup MTSGPU_XML_BY_SHAPE: the <bsdf> child (inline or <ref>) of the
 *                               <shape> with id `id` (a BSDF declared inline
 *                               has no id of its own).
 * Node 0 is that BSDF, every other node a nested <bsdf> or <texture> (a <ref>
 * child resolved by id) with its parent's index and the parameter name it
 * fills ('name' attribute); each node owns num_props property elements from
 * first_prop on (tag float/integer/boolean/string/rgb/srgb/spectrum/point/
 * vector, name, value after substitution, flags).  param_names/values are the
 * loader's parameters (`mitsuba -D name=value`, src/mitsuba/mitsuba.cpp:
 * 168-173); as in the loader they take precedence over the file's <default>s
 * (scenehandler.cpp:684-687).  A property's flags say whether its value went
 * through a substitution (MTSGPU_XML_PROP_PARAM) and whether a <default>
 * supplied it (MTSGPU_XML_PROP_DEFAULT).  A property element this reader
 * does not turn into a value -- one without a value attribute (<spectrum
 * filename=...>, <blackbody ...>) or a sampled spectrum ("400:0.1, 500:0.2")
 * -- is returned with MTSGPU_XML_PROP_UNSUPPORTED and its attributes as
 * "key=value ..." in value: the shim takes such a value from the plugin's own
 * Properties, which the loader has parsed.  The parse of a file (with its
 * includes and parameters) is cached while the files are unchanged, so the
 * shim's one call per BSDF reads the scene once.  The shim rebuilds a Properties
 * object per node.  Returns MTSGPU_OK, MTSGPU_ENOENT (the id is not in the
 * file), MTSGPU_EINVAL (unreadable file, syntax error, undefined parameter,
 * duplicate id, wrong element kind; message in err), or MTSGPU_ENOMEM when a
 * capacity is too small (the counts are still returned).
 * mtsgpu_xml_bsdf is the BY_ID lookup without loader parameters. */
enum { MTSGPU_XML_BSDF = 0, MTSGPU_XML_TEXTURE = 1 };
enum { MTSGPU_XML_BY_ID = 0, MTSGPU_XML_BY_SHAPE = 1 };
enum { MTSGPU_XML_PROP_PARAM = 1, MTSGPU_XML_PROP_DEFAULT = 2, MTSGPU_XML_PROP_UNSUPPORTED = 4 };
typedef struct {
    int32_t kind;                   /* MTSGPU_XML_BSDF / MTSGPU_XML_TEXTURE        */
    int32_t parent;                 /* parent node index, -1 for node 0            */
    char plugin[32];                /* the 'type' attribute (lower case)           */
    char name[64];                  /* parameter name under the parent ('' if none)*/
    char id[64];                    /* the element's 'id' ('' if none)             */
    int32_t first_prop, num_props;
} mtsgpu_xml_node;
typedef struct {
    char tag[16];                   /* float, integer, boolean, string, rgb, ...   */
    char name[64];
    char value[128];
    int32_t flags;                  /* MTSGPU_XML_PROP_*                           */
} mtsgpu_xml_prop;
int mtsgpu_xml_bsdf_ex(const char *xml_path, const char *id, int32_t lookup, const char *const *param_names,
                       const char *const *param_values, int32_t num_params, mtsgpu_xml_node *nodes, int node_cap,
                       mtsgpu_xml_prop *props, int prop_cap, int *num_nodes, int *num_props, char *err,
                       size_t err_cap);
int mtsgpu_xml_bsdf(const char *xml_path, const char *bsdf_id, mtsgpu_xml_node *nodes, int node_cap,
                    mtsgpu_xml_prop *props, int prop_cap, int *num_nodes, int *num_props, char *err,
                    size_t err_cap);
/* Border size b of the film for the given filter parameters. */
int mtsgpu_film_border(int32_t rfilter, float rfilter_param);
/* Render the window into `film` (host memory, layout above).  `samples` may be
 * NULL; otherwise it receives width*height*spp records.  Blocking. */
int mtsgpu_render(mtsgpu_ctx *ctx, const mtsgpu_render_params *params,
                  float *film, float *samples, mtsgpu_stats *stats);
/* Same, but `film` is a device pointer (HBM-resident, no PCIe copy); used by
 * the multi-GPU path to reduce films over RCCL.  `stream` is a hipStream_t
 * (NULL: the context's stream); the call returns after the work is enqueued
 * and the stream has been synchronised. */
int mtsgpu_render_device(mtsgpu_ctx *ctx, const mtsgpu_render_params *params,
                         float *film_device, void *stream, mtsgpu_stats *stats);
/* hdrfilm develop (HDRFilm::develop, src/films/hdrfilm.cpp:481-495 ->
 * Bitmap::convert, src/libcore/fmtconv.cpp:955-1030, 1137-1160): divides the
 * film interior by its weights (invWeight = w != 0 ? 1/w : w) and converts it
 * to `pixel_format` / `component_format`.  Output: (film_height-2*border) rows
 * of (film_width-2*border) pixels, channels interleaved in the order the
 * pixel format names them, components of 2 (float16) or 4 bytes.
 * `multiplier` = 1 for Film::develop (Bitmap::convert's argument). */
enum { MTSGPU_PIX_LUMINANCE = 0, MTSGPU_PIX_LUMINANCE_ALPHA = 1, MTSGPU_PIX_RGB = 2, MTSGPU_PIX_RGBA = 3,
       MTSGPU_PIX_XYZ = 4, MTSGPU_PIX_XYZA = 5 };
enum { MTSGPU_COMP_FLOAT16 = 0, MTSGPU_COMP_FLOAT32 = 1, MTSGPU_COMP_UINT32 = 2 };
typedef struct {
    uint32_t film_width, film_height;   /* the rendered film incl. borders (W+2b, H+2b) */
    uint32_t border;                    /* b                                             */
    int32_t pixel_format;               /* MTSGPU_PIX_*                                  */
    int32_t component_format;           /* MTSGPU_COMP_*                                 */
    float multiplier;
} mtsgpu_develop_params;
/* `film_device` / `out_device` are device pointers; `stream` a hipStream_t
 * (NULL: the context's stream).  Returns after the stream is synchronised. */
int mtsgpu_develop_device(mtsgpu_ctx *ctx, const mtsgpu_develop_params *params, const float *film_device,
                          void *out_device, void *stream);
/* Same from and to host memory (stages both through the context's buffers). */
int mtsgpu_develop(mtsgpu_ctx *ctx, const mtsgpu_develop_params *params, const float *film, void *out);
/* Batch ray queries on the uploaded scene, one GPU lane per ray:
 * Scene::rayIntersect (closest hit, shadow = 0) or the occlusion test
 * (shadow = 1) of ShapeKDTree::rayIntersect (src/librender/skdtree.cpp:
 * 112-142, 207-226), including the scene-bounds clip and the adaptive ray
 * epsilon.  rays: n x 8 floats {o.xyz, mint, d.xyz, maxt}; hits: n x 4
 * floats {t, u, v, prim} where prim is the global triangle index (mesh order,
 * then triangle order) as uint32 bits, 0xffffffff and t = inf on a miss;
 * shadow queries write t = 1 (occluded) or 0.  Host buffers; the kernel's
 * device time goes to *kernel_ms if non-NULL. */
int mtsgpu_trace_rays(mtsgpu_ctx *ctx, const float *rays, uint32_t n, int shadow, float *hits, double *kernel_ms);
/* The same with flags: MTSGPU_TRACE_SHADOW (the occlusion test) and
 * MTSGPU_TRACE_KDTREE: traverse the reference's own SAH kd-tree, built on the
 * host as GenericKDTree::buildInternal builds it (gkdtree.h:959-1264; min-max
 * binning above 65536 primitives, O(n log n) SAH sweep with perfect splits,
 * retraction) on first use, with SAHKDTree3D::rayIntersectHavran and its
 * mailbox (sahkdtree3.h:178-308): among exactly tied triangles the one the
 * reference tests last wins, where the BVH path takes the larger primitive
 * number.  Triangle scenes only. */
enum { MTSGPU_TRACE_SHADOW = 1u, MTSGPU_TRACE_KDTREE = 2u };
int mtsgpu_trace_rays_ex(mtsgpu_ctx *ctx, const float *rays, uint32_t n, uint32_t flags, float *hits,
                         double *kernel_ms);
/* The kd-tree of the uploaded scene (built if needed): info8 = {nodes, indices,
 * inner nodes, leaves, non-empty leaves, retracted splits, pruned primitives,
 * depth limit}; nodes (2 words each, KDNode layout gkdtree.h:453-601) and
 * indices are copied when their capacities (in words) suffice. */
int mtsgpu_debug_kdtree(mtsgpu_ctx *ctx, uint32_t *nodes, size_t node_cap, uint32_t *indices, size_t index_cap,
                        uint32_t *info8);
/* Host-only (no device needed): configure `scene` and build its kd-tree, as above. */
int mtsgpu_kdtree_host(const mtsgpu_scene_desc *scene, uint32_t *nodes, size_t node_cap, uint32_t *indices,
                       size_t index_cap, uint32_t *info8, char *msg, size_t cap);
/* Host-only (no device needed): configure `scene` and export the BVH the
 * kernels traverse: info4 = {BVH2 nodes, half-box nodes,
 * 4-wide nodes, 4-wide inner-node levels}; `nodes` (MtsgNode, 16 words each),
 * `hnodes` (MtsgHNode, 8 words: child boxes as IEEE halves rounded outward)
 * and `qnodes` (MtsgQNode, 16 words: the BVH2 collapsed to 4-wide nodes) are
 * copied when their capacities (in words) suffice.  Replaces no reference
 * interface: it is the checker's view of ShapeKDTree's acceleration structure
 * (src/librender/skdtree.cpp) as rebuilt here. */
int mtsgpu_bvh_host(const mtsgpu_scene_desc *scene, uint32_t *nodes, size_t node_cap, uint32_t *hnodes,
                    size_t hnode_cap, uint32_t *qnodes, size_t qnode_cap, uint32_t *info4, char *msg, size_t cap);
/* Diagnostics (tests): device arithmetic probe -- for each i, out[8i..8i+7] =
 * {a/b, sqrt|a|, sin a, cos a, acos(clamp a), atan2(a,b), exp(-|a|), a*b+a}
 * computed by the kernels' own routines; scene info = {nodes, prims, depth, CUs}. */
int mtsgpu_debug_arith(mtsgpu_ctx *ctx, const float *a, const float *b, float *out, int n);
int mtsgpu_debug_scene_info(mtsgpu_ctx *ctx, uint32_t *info4);
/* Diagnostics (tests/test_gpu_libm.py): out[i] = f(a[i], b[i]) by the kernels'
 * own transcendentals (glibc's float libm restated, glibc_f32.h; double exp/log
 * for math::fastexp/fastlog, include/mitsuba/core/math.h:185-199).  fn: 0 sin and
 * 1 cos (of sincosf), 2 expf, 3 acosf, 4 atanf, 5 tanf, 6 atan2f(a, b),
 * 7 powf(a, b), 8 fastexp, 9 fastlog.  With a == NULL, a[i] is the float whose
 * bits are first + i (b may be NULL for the unary functions).  Host buffers. */
int mtsgpu_debug_libm(mtsgpu_ctx *ctx, int fn, const float *a, const float *b, float *out, size_t n,
                      uint32_t first);
/* the 16 raw device counters of the last render (samples, rays, shadow rays,
   path lengths, node visits, TriAccel tests, dimension errors, hits, -, NEE
   samples, Sobol HBM words, diagnostic section cycles 11-14), and in 15 the
   kernel that ran: the megakernel's feature set (MTSG_FEAT_* bits of
   csrc/layout.h, BSDF-set bits included) | waves/SIMD << 8 | scene in LDS << 12,
   or 1 << 16 for the wavefront engine */
int mtsgpu_debug_counters(mtsgpu_ctx *ctx, uint64_t *out16);
/* n nextULong draws of the device's SFMT19937 (the SFMT replay samplers' generator)
   from Random(seed), or from the clone-th Random(&master) clone of it */
int mtsgpu_debug_sfmt(mtsgpu_ctx *ctx, uint64_t seed, int clone, uint64_t *out, int n);
/* Host-only (no device needed): configure `scene` and return its environment
 * emitter's tables -- params[64] = {levels, w0, h0, normalization, pixel_x,
 * pixel_y, scale, center xyz, radius, total texels, .., lw[l] at 16+l, lh[l] at
 * 34+l}; texels: 4 halves per texel (RGB + pad), all levels (capacity in
 * halves); rows h0+1, cols h0*(w0+1), weights h0 floats (any may be NULL). */
int mtsgpu_debug_env_tables(const mtsgpu_scene_desc *scene, float *params, uint16_t *texels, size_t texel_cap,
                            float *rows, float *cols, float *weights);
/* ---- device groups: one render over several GPUs ------------------------
 * SURVEY.md 8(b)'s `mtsgpu_create(const int *devices, int n, ...)`: a group
 * holds one context per listed device (a device may be listed twice: two
 * contexts on one GPU).  mtsgpu_group_render shards the crop window's 8x8
 * tiles over the members -- member k renders the tiles t with t % n == k
 * (MTSGPU_FLAG_TILE_SHARD, the multi-GPU bench's decomposition; the
 * interleaved blocks of BlockedImageProcess, src/librender/imageproc.cpp:28-80,
 * params->row_block is ignored) -- one host thread
 * per member, each into its own HBM film, and merges the films on the first
 * member's device (peer copies over xGMI, then dst += src in member order:
 * renderproc.cpp:142-149's Film::put sum; disjoint tiles make it exact for the
 * box filter).  params->row_stride must be 0 or 1 (the group owns the
 * sharding).  The SFMT replay samplers render on the first member alone (their
 * streams follow one block order).  Stats are summed, kernel_ms is the
 * slowest member's. */
typedef struct mtsgpu_group mtsgpu_group;
int mtsgpu_group_create(const int *devices, int n, mtsgpu_group **out);
int mtsgpu_group_size(const mtsgpu_group *group);
/* Upload the scene to every member (configured once per member, in parallel). */
int mtsgpu_group_upload_scene(mtsgpu_group *group, const mtsgpu_scene_desc *scene);
/* Render into `film` (host memory, the mtsgpu_render layout).  Blocking. */
int mtsgpu_group_render(mtsgpu_group *group, const mtsgpu_render_params *params, float *film, mtsgpu_stats *stats);
/* The same with the merged film left in HBM on the first member's device
 * (`film_device`, (W+2b)(H+2b)x5 floats). */
int mtsgpu_group_render_device(mtsgpu_group *group, const mtsgpu_render_params *params, float *film_device,
                               mtsgpu_stats *stats);
/* Host-only (no device): member k's render params in an n-member group render
 * (the tile decomposition above), and the number of window pixels a render
 * with the given params covers (the kernels' item -> pixel rule). */
int mtsgpu_group_member_params(const mtsgpu_render_params *params, int n, int k, mtsgpu_render_params *out);
uint64_t mtsgpu_render_pixels(const mtsgpu_render_params *params);
/* Member k's context (borrowed; for develop / trace_rays on one device). */
mtsgpu_ctx *mtsgpu_group_member(mtsgpu_group *group, int k);
const char *mtsgpu_group_last_error(mtsgpu_group *group);
void mtsgpu_group_destroy(mtsgpu_group *group);

/* Last error message of this context (or of the last failed create). */
const char *mtsgpu_last_error(mtsgpu_ctx *ctx);
void mtsgpu_destroy(mtsgpu_ctx *ctx);
int mtsgpu_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MTSGPU_H */
