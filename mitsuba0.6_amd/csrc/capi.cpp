// capi.cpp -- the C-ABI of libmtsgpu.so (include/mtsgpu.h).
//
// Replaces, for the `path` integrator, SamplingIntegrator::render ->
// BlockedRenderProcess -> BlockRenderer::process -> renderBlock
// (src/librender/integrator.cpp:95-188, renderproc.cpp:68-149): one call
// renders a pixel window with a persistent kernel and returns the ImageBlock
// (full crop + filter border) that Film::put would have accumulated.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mtsgpu.h"
#include "layout.h"
#include "scene_build.h"
#include "sfmt.h"
#include "kdtree.h"

hipError_t mtsg_launch_path(const MtsgLaunch &L, int grid, bool samples, bool stats, hipStream_t stream);
hipError_t mtsg_launch_gather(const MtsgLaunch &L, hipStream_t stream);
hipError_t mtsg_launch_reduce(const MtsgLaunch &L, hipStream_t stream);
hipError_t mtsg_launch_finalize(float *own, const double *spill, size_t n, hipStream_t stream);
hipError_t mtsg_launch_arith_probe(const float *a, const float *b, float *out, int n, hipStream_t stream);
hipError_t mtsg_launch_libm_probe(int fn, const float *a, const float *b, float *out, size_t n, uint32_t first,
                                  hipStream_t s);
hipError_t mtsg_launch_trace(const MtsgDeviceScene &S, const float *rays, uint32_t n, float *out, bool shadow,
                             uint32_t stackDepth, int numCUs, hipStream_t stream);
hipError_t mtsg_launch_trace_kd(const MtsgDeviceScene &S, const uint32_t *kdNodes, const uint32_t *kdIndices,
                                const MtsgTri *kdTris, const float *rays, uint32_t n, float *out, bool shadow,
                                int numCUs, hipStream_t stream);
int mtsg_path_kernel_occupancy(const MtsgLaunch &L, int *blocksPerCU);
int mtsg_path_variant(const MtsgLaunch &L);
hipError_t mtsg_launch_wf_shade(const MtsgLaunch &L, const MtsgWave &W, unsigned long long *part, int grid, int wk,
                                bool ggx, bool instr, hipStream_t s);
hipError_t mtsg_launch_wf_trace(const MtsgLaunch &L, const MtsgWave &W, unsigned long long *part, int grid,
                                bool stats, hipStream_t s);
hipError_t mtsg_launch_wf_flush(const unsigned long long *part, uint32_t blocks, unsigned long long *counters,
                                hipStream_t s);
int mtsg_wf_occupancy(const MtsgLaunch &L, int wk, bool ggx, int *shadeBpc, int *traceBpc);
int mtsg_path_features(const MtsgLaunch &L);
// the wavefront's trace kernel forms the whole hit record (MTSGPU_WF_HITREC=1; A/B in DESIGN.md 4)
static bool wf_hitrec_on() {
    const char *e = std::getenv("MTSGPU_WF_HITREC");
    return e && e[0] == '1';
}
hipError_t mtsg_launch_sfmt_probe(uint32_t *w, unsigned long long *out, int n, hipStream_t s);
hipError_t mtsg_launch_develop(const mtsgpu_develop_params &P, const float *film, void *out, int num_cus,
                               hipStream_t s);
int mtsg_develop_channels(int pixel_format);

namespace {

thread_local std::string g_create_error;
constexpr size_t BLOCK_THREADS = 256;   // = BLOCK in path_kernel.hip

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    hipError_t ensure(size_t n) {
        if (n <= bytes && p) return hipSuccess;
        release();
        hipError_t e = hipMalloc(&p, std::max<size_t>(n, 16));
        if (e == hipSuccess) bytes = std::max<size_t>(n, 16);
        return e;
    }
};

}  // namespace

struct mtsgpu_ctx {
    int device = 0;
    int num_cus = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    bool have_scene = false;
    HostScene host;
    MtsgDeviceScene dscene;
    DevBuf scan_tris;   // k-grouped TriAccel records of scan-sized scenes
    uint32_t scan_n[6] = {0, 0, 0, 0, 0, 0};
    DevBuf nodes, hnodes, tris, prim_vtx, dpdu, positions, normals, shapes, bsdfs, emitters, area_cdf, em_cdf, sobol;
    DevBuf env, env_texels, env_rows, env_cols, env_weights, env_grows, env_gcols;
    DevBuf rtrans, texcoords, analytic;
    DevBuf qrays, qhits;      // mtsgpu_trace_rays staging
    DevBuf film_own, film_spill, samples, counters, contrib;
    DevBuf dev_in, dev_out;   // staging of mtsgpu_develop (host film -> developed image)
    // wavefront pipeline: path slots, ray queues and results, counters
    DevBuf wf_state, wf_ray, wf_rslot, wf_cls, wf_cnt, wf_hit, wf_hitrec, wf_occl, wf_live, wf_ovf, wf_part, wf_kind;
    DevBuf rp_order, rp_start, rp_sfmt;   // SFMT replay: render order, unit starts, streams
    // the reference's SAH kd-tree (kdtree_build.cpp), built on first use
    bool kd_built = false;
    KdTree kd;
    DevBuf kd_nodes, kd_indices, kd_tris;
    uint32_t *wf_live_host = nullptr;   // pinned: live-slot counts read back while the pipeline runs
    hipEvent_t wf_ev[8] = {};
    std::vector<uint32_t> wf_kind_host;   // shape -> shade kind (wf_kinds)
    unsigned long long last_counters[16] = {};
};

namespace {

int ensure_kdtree(mtsgpu_ctx *ctx);   // the reference's SAH kd-tree, built on first use (below)

int fail(mtsgpu_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return code;
}

int hip_fail(mtsgpu_ctx *ctx, hipError_t e, const char *what) {
    return fail(ctx, e == hipErrorOutOfMemory ? MTSGPU_ENOMEM : MTSGPU_EHIP,
                std::string(what) + ": " + hipGetErrorString(e));
}

// Sobol direction numbers as 4-bit XOR tables: [dim][c][v] = XOR of columns
// 4c..4c+3 of the dimension selected by the bits of v (sobolseq.h:43-57)
// (thread-safe: a static initialised once, group members upload concurrently)
std::vector<uint32_t> build_sobol_nibble_tables() {
    const std::vector<uint32_t> &M = mtsg_sobol_matrices();
    std::vector<uint32_t> T((size_t)MTSG_SOBOL_DIMS * MTSG_NIBBLES * 16, 0u);
    for (int d = 0; d < MTSG_SOBOL_DIMS; ++d)
        for (int c = 0; c < MTSG_NIBBLES; ++c)
            for (int v = 0; v < 16; ++v) {
                uint32_t r = 0;
                for (int b = 0; b < 4; ++b)
                    if ((v >> b) & 1) r ^= M[(size_t)d * MTSG_SOBOL_SIZE + 4 * c + b];
                T[((size_t)d * MTSG_NIBBLES + c) * 16 + v] = r;
            }
    return T;
}

const std::vector<uint32_t> &sobol_nibble_tables() {
    static const std::vector<uint32_t> T = build_sobol_nibble_tables();
    return T;
}

template <class T>
hipError_t upload(DevBuf &b, const std::vector<T> &v, hipStream_t s) {
    hipError_t e = b.ensure(v.size() * sizeof(T));
    if (e != hipSuccess) return e;
    if (v.empty()) return hipSuccess;
    return hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
}

}  // namespace

extern "C" {

int mtsgpu_abi_version(void) { return MTSGPU_ABI_VERSION; }

int mtsgpu_create(int device, mtsgpu_ctx **out) {
    if (!out) return MTSGPU_EINVAL;
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) {
        g_create_error = std::string("no HIP device: ") + hipGetErrorString(e);
        return MTSGPU_ENODEV;
    }
    if (device < 0) {
        e = hipGetDevice(&device);
        if (e != hipSuccess) device = 0;
    }
    if (device >= count) { g_create_error = "device index out of range"; return MTSGPU_ENODEV; }
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) {
        g_create_error = std::string("hipGetDeviceProperties: ") + hipGetErrorString(e);
        return MTSGPU_EHIP;
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        g_create_error = std::string("libmtsgpu.so is built for gfx950, device is ") + prop.gcnArchName;
        return MTSGPU_ENODEV;
    }
    mtsgpu_ctx *ctx = new mtsgpu_ctx();
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount;
    if ((e = hipSetDevice(device)) != hipSuccess || (e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreate(&ctx->ev0)) != hipSuccess || (e = hipEventCreate(&ctx->ev1)) != hipSuccess) {
        g_create_error = std::string("HIP init: ") + hipGetErrorString(e);
        delete ctx;
        return MTSGPU_EHIP;
    }
    *out = ctx;
    return MTSGPU_OK;
}

int mtsgpu_upload_scene(mtsgpu_ctx *ctx, const mtsgpu_scene_desc *scene) {
    if (!ctx || !scene) return MTSGPU_EINVAL;
    ctx->have_scene = false;
    ctx->kd_built = false;
    std::string err;
    int rc = mtsg_configure_scene(scene, ctx->host, err);
    if (rc) return fail(ctx, rc, err);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    HostScene &H = ctx->host;
    hipStream_t s = ctx->stream;
    if ((e = upload(ctx->nodes, H.nodes, s)) != hipSuccess || (e = upload(ctx->hnodes, H.hnodes, s)) != hipSuccess ||
        (e = upload(ctx->tris, H.tris, s)) != hipSuccess ||
        (e = upload(ctx->prim_vtx, H.prim_vtx, s)) != hipSuccess || (e = upload(ctx->dpdu, H.dpdu, s)) != hipSuccess ||
        (e = upload(ctx->positions, H.positions, s)) != hipSuccess || (e = upload(ctx->normals, H.normals, s)) != hipSuccess ||
        (e = upload(ctx->shapes, H.shapes, s)) != hipSuccess || (e = upload(ctx->bsdfs, H.bsdfs, s)) != hipSuccess ||
        (e = upload(ctx->emitters, H.emitters, s)) != hipSuccess || (e = upload(ctx->area_cdf, H.area_cdf, s)) != hipSuccess ||
        (e = upload(ctx->em_cdf, H.em_cdf, s)) != hipSuccess || (e = upload(ctx->sobol, sobol_nibble_tables(), s)) != hipSuccess)
        return hip_fail(ctx, e, "scene upload");
    // tiny scenes: the TriAccel records grouped by projection axis and, within
    // an axis, planes normal to it (n_u = n_v = 0: the Cornell box's walls)
    // last, so the scan runs six branch-free loops, the aligned ones without
    // the numerator's and denominator's n_u/n_v terms (the closest hit and its
    // tie rule do not depend on the order the records are tested in)
    for (uint32_t &c : ctx->scan_n) c = 0;
    if (H.tris.size() <= MTSG_SCAN_MAX && H.analytic.empty()) {
        std::vector<MtsgTri> g;
        for (uint32_t k = 0; k < 3; ++k)
            for (uint32_t al = 0; al < 2; ++al)
                for (const MtsgTri &t : H.tris)
                    if (t.k == k && (uint32_t)(t.n_u == 0.0f && t.n_v == 0.0f) == al) { g.push_back(t); ctx->scan_n[2 * k + al]++; }
        if (g.empty()) g.push_back(MtsgTri{});
        if ((e = upload(ctx->scan_tris, g, s)) != hipSuccess) return hip_fail(ctx, e, "scene upload");
    }
    const MtsgEnv *denv = nullptr;
    if (H.env.emitter >= 0) {
        if ((e = upload(ctx->env_texels, H.env_texels, s)) != hipSuccess || (e = upload(ctx->env_rows, H.env_cdf_rows, s)) != hipSuccess ||
            (e = upload(ctx->env_cols, H.env_cdf_cols, s)) != hipSuccess || (e = upload(ctx->env_weights, H.env_row_weights, s)) != hipSuccess)
            return hip_fail(ctx, e, "envmap upload");
        H.env.texels = (const uint16_t *)ctx->env_texels.p;
        H.env.cdf_rows = (const float *)ctx->env_rows.p;
        H.env.cdf_cols = (const float *)ctx->env_cols.p;
        H.env.row_weights = (const float *)ctx->env_weights.p;
        H.env.guide_rows = H.env.guide_cols = nullptr;
        if (!H.env_guide_rows.empty()) {
            if ((e = upload(ctx->env_grows, H.env_guide_rows, s)) != hipSuccess ||
                (e = upload(ctx->env_gcols, H.env_guide_cols, s)) != hipSuccess)
                return hip_fail(ctx, e, "envmap upload");
            H.env.guide_rows = (const uint16_t *)ctx->env_grows.p;
            H.env.guide_cols = (const uint16_t *)ctx->env_gcols.p;
        }
        if ((e = ctx->env.ensure(sizeof(MtsgEnv))) != hipSuccess ||
            (e = hipMemcpyAsync(ctx->env.p, &H.env, sizeof(MtsgEnv), hipMemcpyHostToDevice, s)) != hipSuccess)
            return hip_fail(ctx, e, "envmap upload");
        denv = (const MtsgEnv *)ctx->env.p;
    }
    if ((!H.rtrans.empty() && (e = upload(ctx->rtrans, H.rtrans, s)) != hipSuccess) ||
        (!H.texcoords.empty() && (e = upload(ctx->texcoords, H.texcoords, s)) != hipSuccess) ||
        (!H.analytic.empty() && (e = upload(ctx->analytic, H.analytic, s)) != hipSuccess))
        return hip_fail(ctx, e, "texture/table upload");
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "scene upload sync");
    MtsgDeviceScene &D = ctx->dscene;
    std::memset(&D, 0, sizeof D);
    D.nodes = (const MtsgNode *)ctx->nodes.p;
    D.hnodes = (const MtsgHNode *)ctx->hnodes.p;
    D.tris = (const MtsgTri *)ctx->tris.p;
    D.prim_vtx = (const uint32_t *)ctx->prim_vtx.p;
    D.dpdu = (const float *)ctx->dpdu.p;
    D.positions = (const float *)ctx->positions.p;
    D.normals = (const float *)ctx->normals.p;
    D.shapes = (const MtsgShape *)ctx->shapes.p;
    D.bsdfs = (const MtsgBsdf *)ctx->bsdfs.p;
    D.emitters = (const MtsgEmitter *)ctx->emitters.p;
    D.area_cdf = (const float *)ctx->area_cdf.p;
    D.em_cdf = (const float *)ctx->em_cdf.p;
    D.sobol = nullptr;
    D.num_emitters = (uint32_t)H.emitters.size();
    D.num_prims = (uint32_t)H.tris.size();
    D.em_norm = H.em_norm;
    D.env = denv;
    D.env_emitter = H.env.emitter;
    D.rtrans = H.rtrans.empty() ? nullptr : (const float *)ctx->rtrans.p;
    D.texcoords = H.texcoords.empty() ? nullptr : (const float *)ctx->texcoords.p;
    D.analytic = H.analytic.empty() ? nullptr : (const MtsgAnalytic *)ctx->analytic.p;
    for (int a = 0; a < 3; ++a) { D.aabb_min[a] = H.aabb_min[a]; D.aabb_max[a] = H.aabb_max[a]; }
    D.cam = H.cam;
    ctx->have_scene = true;
    return MTSGPU_OK;
}

int mtsgpu_check_scene(const mtsgpu_scene_desc *scene, char *msg, size_t cap) {
    if (!scene) return MTSGPU_EINVAL;
    HostScene H;
    std::string err;
    int rc = mtsg_configure_scene(scene, H, err);
    if (msg && cap) {
        std::strncpy(msg, err.c_str(), cap - 1);
        msg[cap - 1] = 0;
    }
    return rc;
}

int mtsgpu_film_border(int32_t rfilter, float rfilter_param) {
    MtsgFilter f;
    std::string err;
    if (mtsg_configure_filter(rfilter, rfilter_param, f, err)) return MTSGPU_EINVAL;
    return f.border;
}

// The wavefront engine's launch plan: the shade kinds the scene's shapes can
// reach (the MISS kind always), each kernel's grid, the trace grid, the slots
struct WfPlan {
    bool kinds[MTSG_WK_KINDS] = {};
    bool ggx[MTSG_WK_KINDS] = {};
    int shadeGrid[MTSG_WK_KINDS] = {};
    int traceGrid = 0;
    uint32_t slots = 0;
    bool hitrec = false;   // wf_trace forms the hit records (MtsgWave::hitrec)
};

// The wavefront engine for one chunk of samples (wf_kernel.hip): the MISS
// kernel starts every slot's first path, then bounce after bounce the shade
// kernel of each kind, then the trace kernel, until no path slot is live.  The
// live count of every POLL-th bounce is read back asynchronously; the host
// stays at most LAG polls ahead of the GPU, so the queues never drain and the
// overshoot (empty bounces) stays small.
// Entries per region of the wavefront queues.  A kernel's block b appends to
// region b % R, at most BLOCK entries per block.  Ray queues are filled by the
// shade kernels, one per kind over n_k <= slots entries in all: a region gets at
// most sum_k ceil(ceil(n_k / BLOCK) / R) <= ceil((slots / BLOCK + K) / R) + K
// blocks.  A kind queue gets the trace kernel's closest-hit entries (its first
// nc <= slots entries: ceil((slots / BLOCK + 1) / R) + 1 blocks per region), and
// the miss queue the shade kernels' appends as well.  Round 4 sized every
// region for all slots: 8x the ray-queue bytes that can be live.
static void wf_caps(size_t slots, size_t &capRay, size_t &capCls) {
    const size_t B = BLOCK_THREADS, R = MTSG_WF_REGIONS, K = MTSG_WK_KINDS, nb = (slots + B - 1) / B;
    const size_t shade = (nb + K + R - 1) / R + K, trace = (nb + 1 + R - 1) / R + 1;
    capRay = std::min(slots, B * shade);
    capCls = std::min(slots, B * (shade + trace));
}

static int wf_render_chunk(mtsgpu_ctx *ctx, const MtsgLaunch &L, bool instr, bool stats, hipStream_t stream,
                           const WfPlan &plan, const volatile int *cancel) {
    hipError_t e;
    const uint32_t slots = plan.slots;
    const size_t R = MTSG_WF_REGIONS;
    size_t cap, capCls;
    wf_caps(slots, cap, capCls);
    // the shade kernels' launch record: their blocks are short-lived (one queue entry
    // per thread), so the Sobol dimensions they stage in LDS are a per-block cost;
    // MTSGPU_WF_SHADE_LDS_DIMS caps them (0: every dimension from HBM/L2)
    MtsgLaunch Ls = L;
    if (const char *env = std::getenv("MTSGPU_WF_SHADE_LDS_DIMS"))
        Ls.lds_dims = std::min<uint32_t>(Ls.lds_dims, (uint32_t)std::strtoul(env, nullptr, 10));
    MtsgWave W;
    std::memset(&W, 0, sizeof W);
    W.state = (float4 *)ctx->wf_state.p;
    for (int p = 0; p < 2; ++p) {
        W.ray[p] = (float4 *)ctx->wf_ray.p + (size_t)p * 2 * R * cap * 2;
        W.rslot[p] = (uint32_t *)ctx->wf_rslot.p + (size_t)p * 2 * R * cap;
        W.cls[p] = (uint32_t *)ctx->wf_cls.p + (size_t)p * MTSG_WK_KINDS * R * capCls;
    }
    W.cnt = (uint32_t *)ctx->wf_cnt.p;
    W.hit = (float4 *)ctx->wf_hit.p;
    W.occl = (uint32_t *)ctx->wf_occl.p;
    W.live = (uint32_t *)ctx->wf_live.p;
    W.ovf = (uint2 *)ctx->wf_ovf.p;
    W.shape_kind = (const uint32_t *)ctx->wf_kind.p;
    W.slots = slots;
    W.cap = (uint32_t)cap;
    W.cap_cls = (uint32_t)capCls;
    W.ovf_depth = L.stack_depth > MTSG_WF_LDS_STACK ? L.stack_depth - MTSG_WF_LDS_STACK : 0;
    if (plan.hitrec) {
        W.hitrec = (float4 *)ctx->wf_hitrec.p;
        W.hitrec_uv = (mtsg_path_features(L) & MTSG_FEAT_EXT) ? 1u : 0u;
    }
    unsigned long long *part = (unsigned long long *)ctx->wf_part.p;
    int partBlocks = plan.traceGrid;
    for (int k = 0; k < MTSG_WK_KINDS; ++k) partBlocks = std::max(partBlocks, plan.shadeGrid[k]);
    if ((e = hipMemsetAsync(ctx->wf_cnt.p, 0, (size_t)2 * MTSG_WF_QUEUES * R * 4, stream)) != hipSuccess ||
        (e = hipMemsetAsync(ctx->wf_live.p, 0, 2 * 4, stream)) != hipSuccess ||
        (e = hipMemsetAsync(part, 0, (size_t)partBlocks * 16 * 8, stream)) != hipSuccess)
        return hip_fail(ctx, e, "wavefront reset");
    constexpr int POLL = 4, LAG = 2, RING = 8;
    int polls = 0, checked = 0;
    const uint64_t maxBounces = (uint64_t)1 << 24;
    for (uint64_t it = 0;; ++it) {
        if (it >= maxBounces) return fail(ctx, MTSGPU_EHIP, "wavefront: no convergence");
        W.parity = (uint32_t)(it & 1);
        W.seed = it == 0 ? 1u : 0u;
        for (int k = 0; k < MTSG_WK_KINDS; ++k) {
            if (!plan.kinds[k] || (it == 0 && k != MTSG_WK_MISS)) continue;
            if ((e = mtsg_launch_wf_shade(Ls, W, part, plan.shadeGrid[k], k, plan.ggx[k], instr, stream)) != hipSuccess)
                return hip_fail(ctx, e, "wf_shade launch");
        }
        W.seed = 0;
        if (it % POLL == 0) {
            const int r = polls % RING;
            if ((e = hipMemcpyAsync(ctx->wf_live_host + r, W.live + W.parity, 4, hipMemcpyDeviceToHost,
                                    stream)) != hipSuccess ||
                (e = hipEventRecord(ctx->wf_ev[r], stream)) != hipSuccess)
                return hip_fail(ctx, e, "wavefront poll");
            ++polls;
        }
        if ((e = mtsg_launch_wf_trace(L, W, part, plan.traceGrid, stats, stream)) != hipSuccess)
            return hip_fail(ctx, e, "wf_trace launch");
        bool finished = false;
        while (!finished && polls > checked) {
            const int r = checked % RING;
            if (polls - checked <= LAG && hipEventQuery(ctx->wf_ev[r]) != hipSuccess) break;   // not yet, and not far ahead
            if ((e = hipEventSynchronize(ctx->wf_ev[r])) != hipSuccess) return hip_fail(ctx, e, "wavefront");
            ++checked;
            finished = ctx->wf_live_host[r] == 0;
        }
        if (finished) break;
        if (cancel && *cancel) break;
    }
    if ((e = mtsg_launch_wf_flush(part, (uint32_t)partBlocks, L.counters, stream)) != hipSuccess)
        return hip_fail(ctx, e, "wf_flush launch");
    return MTSGPU_OK;
}

// shape -> shade kind (wf_kernel.hip) from the shape's BSDF type; per kind,
// whether every BSDF of that kind uses the GGX distribution
static void wf_kinds(const HostScene &H, std::vector<uint32_t> &shapeKind, WfPlan &plan) {
    bool any[MTSG_WK_KINDS] = {}, nonGgx[MTSG_WK_KINDS] = {};
    shapeKind.assign(std::max<size_t>(1, H.shapes.size()), (uint32_t)MTSG_WK_GEN);
    for (size_t i = 0; i < H.shapes.size(); ++i) {
        const MtsgBsdf &b = H.bsdfs[H.shapes[i].bsdf];
        int k = MTSG_WK_GEN;
        switch (b.type) {
            case MTSGPU_BSDF_DIFFUSE: k = MTSG_WK_DIFF; break;
            case MTSGPU_BSDF_ROUGHCONDUCTOR: k = MTSG_WK_RC; break;
            case MTSGPU_BSDF_ROUGHDIELECTRIC: k = MTSG_WK_RD; break;
            case MTSGPU_BSDF_ROUGHPLASTIC: k = MTSG_WK_RP; break;
            default: break;
        }
        if (std::getenv("MTSGPU_WF_GENERIC")) k = MTSG_WK_GEN;   // A/B: every hit through the generic kernel
        shapeKind[i] = (uint32_t)k;
        any[k] = true;
        if (b.distr != MTSGPU_DISTR_GGX) nonGgx[k] = true;
    }
    for (int k = 0; k < MTSG_WK_KINDS; ++k) {
        plan.kinds[k] = any[k] || k == MTSG_WK_MISS;
        plan.ggx[k] = any[k] && !nonGgx[k];
    }
}

// ---------------------------------------------------------------------------
// The `independent` sampler replay (MTSGPU_SAMPLER_SFMT_*): stream seeding and
// the reference's render order
// ---------------------------------------------------------------------------
static void sfmt_period_certification(uint32_t *w) {   // random.cpp:322-347
    const uint32_t parity[4] = {0x00000001u, 0x00000000u, 0x00000000u, 0x13c9e684u};
    uint32_t inner = 0;
    for (int i = 0; i < 4; ++i) inner ^= w[i] & parity[i];
    for (int i = 16; i > 0; i >>= 1) inner ^= inner >> i;
    if (inner & 1) return;
    for (int i = 0; i < 4; ++i)
        for (uint32_t work = 1, j = 0; j < 32; ++j, work <<= 1)
            if (work & parity[i]) { w[i] ^= work; return; }
}

static void mtsg_sfmt_seed(uint32_t *w, uint64_t seed) {   // init_gen_rand (random.cpp:397-406)
    uint64_t v = seed;
    w[0] = (uint32_t)v;
    w[1] = (uint32_t)(v >> 32);
    for (int i = 1; i < MTSG_SFMT_N64; ++i) {
        v = 6364136223846793005ull * (v ^ (v >> 62)) + (uint64_t)i;
        w[2 * i] = (uint32_t)v;
        w[2 * i + 1] = (uint32_t)(v >> 32);
    }
    w[MTSG_SFMT_N32] = MTSG_SFMT_N32;
    sfmt_period_certification(w);
}

// Random(Random *parent): init_by_array over 312 of the parent's outputs as
// 624 little-endian words (random.cpp:408-471, 528-548)
static void mtsg_sfmt_clone(uint32_t *w, uint32_t *parent) {
    uint32_t key[MTSG_SFMT_N32];
    for (int i = 0; i < MTSG_SFMT_N64; ++i) {
        const uint64_t v = sfmt_next_ulong(parent);
        key[2 * i] = (uint32_t)v;
        key[2 * i + 1] = (uint32_t)(v >> 32);
    }
    const int n = MTSG_SFMT_N32, lag = 11, mid = (n - lag) / 2, len = MTSG_SFMT_N32;
    auto f1 = [](uint32_t x) { return (x ^ (x >> 27)) * 1664525u; };
    auto f2 = [](uint32_t x) { return (x ^ (x >> 27)) * 1566083941u; };
    std::memset(w, 0x8b, MTSG_SFMT_N32 * 4);
    int count = std::max(len + 1, n);
    uint32_t r = f1(w[0] ^ w[mid] ^ w[n - 1]);
    w[mid] += r;
    r += (uint32_t)len;
    w[mid + lag] += r;
    w[0] = r;
    --count;
    int i = 1, j = 0;
    for (; j < count && j < len; ++j, i = (i + 1) % n) {
        r = f1(w[i] ^ w[(i + mid) % n] ^ w[(i + n - 1) % n]);
        w[(i + mid) % n] += r;
        r += key[j] + (uint32_t)i;
        w[(i + mid + lag) % n] += r;
        w[i] = r;
    }
    for (; j < count; ++j, i = (i + 1) % n) {
        r = f1(w[i] ^ w[(i + mid) % n] ^ w[(i + n - 1) % n]);
        w[(i + mid) % n] += r;
        r += (uint32_t)i;
        w[(i + mid + lag) % n] += r;
        w[i] = r;
    }
    for (j = 0; j < n; ++j, i = (i + 1) % n) {
        r = f2(w[i] + w[(i + mid) % n] + w[(i + n - 1) % n]);
        w[(i + mid) % n] ^= r;
        r -= (uint32_t)i;
        w[(i + mid + lag) % n] ^= r;
        w[i] = r;
    }
    w[MTSG_SFMT_N32] = MTSG_SFMT_N32;
    sfmt_period_certification(w);
}

namespace {
// HilbertCurve2D<uint8_t>::generate (core/sfcurve.h): ENorth 0, EEast 1, ESouth 2, EWest 3
void hilbert(int order, int front, int right, int back, int left, uint8_t pos[2], uint8_t w, uint8_t h, uint32_t bx,
             uint32_t by, std::vector<uint32_t> &out) {
    if (order == 0) {
        if (pos[0] < w && pos[1] < h) out.push_back((bx + pos[0]) | ((by + pos[1]) << 16));
        return;
    }
    auto move = [&](int d) {
        if (d == 0) pos[1]--; else if (d == 1) pos[0]++; else if (d == 2) pos[1]++; else pos[0]--;
    };
    hilbert(order - 1, left, back, right, front, pos, w, h, bx, by, out); move(right);
    hilbert(order - 1, front, right, back, left, pos, w, h, bx, by, out); move(back);
    hilbert(order - 1, front, right, back, left, pos, w, h, bx, by, out); move(left);
    hilbert(order - 1, right, front, left, back, pos, w, h, bx, by, out);
}
}  // namespace

// the crop's pixels (x | y << 16, crop-relative) in the reference's order:
// BlockedImageProcess's spiral (imageproc.cpp:28-80), HilbertCurve2D per block
// (renderproc.cpp:79-81); blockStart: first pixel of each block, then the count
static void mtsg_render_order(uint32_t width, uint32_t height, uint32_t bs, std::vector<uint32_t> &order,
                       std::vector<uint32_t> &blockStart) {
    const int nbx = (int)std::ceil((float)width / (float)bs), nby = (int)std::ceil((float)height / (float)bs);
    const int total = nbx * nby;
    int cx = nbx / 2, cy = nby / 2, dir = 0 /* ERight */, stepsLeft = 1, numSteps = 1;
    const float invLog2 = 1.0f / (float)std::log((double)2.0f);   // math::fastlog (math.h:193-195)
    order.clear();
    blockStart.clear();
    for (int b = 0; b < total; ++b) {
        const int bw = std::min<int>((int)width - cx * (int)bs, (int)bs), bh = std::min<int>((int)height - cy * (int)bs, (int)bs);
        blockStart.push_back((uint32_t)order.size());
        const int order2 = (int)std::ceil(invLog2 * (float)std::log((double)(float)std::max(bw, bh)));
        uint8_t pos[2] = {0, 0};
        hilbert(order2, 0, 1, 2, 3, pos, (uint8_t)bw, (uint8_t)bh, (uint32_t)(cx * (int)bs), (uint32_t)(cy * (int)bs),
                order);
        if (b + 1 == total) break;
        do {
            if (dir == 0) ++cx; else if (dir == 1) ++cy; else if (dir == 2) --cx; else --cy;
            if (--stepsLeft == 0) {
                dir = (dir + 1) % 4;
                if (dir == 2 || dir == 0) ++numSteps;   // ELeft, ERight
                stepsLeft = numSteps;
            }
        } while (cx < 0 || cy < 0 || cx >= nbx || cy >= nby);
    }
    blockStart.push_back((uint32_t)order.size());
}

// megakernel sample runs (dmega.h): a lane renders 2^s consecutive samples of one pixel, so
// its wave keeps the same 64 pixels for 2^s paths.  Large scenes: the longest runs that leave
// every lane MTSG_MIN_RUNS of them (full frame: C3 s = 4 +13%, C5 s = 5 +14% over s = 0; longer
// runs leave a tail, profiles/r06_rounds/).  Tiny LDS scenes gain nothing: pairs, whose box
// records share a 32 B sector (film_slot).  MTSGPU_ROUND_SHIFT=s overrides (A/B)
static uint32_t run_shift(const MtsgLaunch &L, uint64_t lanes) {
    if (const char *env = std::getenv("MTSGPU_ROUND_SHIFT")) return (uint32_t)std::min(6, std::max(0, std::atoi(env)));
    uint32_t s = L.scene_lds ? 1u : 6u;
    const uint64_t perLane = L.num_items / std::max<uint64_t>(1, lanes);
    while (s > 0 && ((1u << s) > L.chunk_spp || (perLane >> s) < MTSG_MIN_RUNS)) --s;
    return s;
}

static int render_impl(mtsgpu_ctx *ctx, const mtsgpu_render_params *P, float *film_host, float *film_dev,
                       float *samples_host, hipStream_t stream, mtsgpu_stats *stats) {
    if (!ctx || !P) return MTSGPU_EINVAL;
    if (!ctx->have_scene) return fail(ctx, MTSGPU_ESTATE, "render called before a successful upload_scene");
    if (P->spp == 0) return fail(ctx, MTSGPU_EINVAL, "sampleCount must be positive");
    const bool pathLike = P->integrator == MTSGPU_INTEGRATOR_PATH || P->integrator == MTSGPU_INTEGRATOR_VOLPATH;
    if (pathLike && P->rr_depth <= 0)
        return fail(ctx, MTSGPU_EINVAL, "'rrDepth' must be set to a value greater than zero!");
    if (pathLike && P->max_depth <= 0 && P->max_depth != -1)
        return fail(ctx, MTSGPU_EINVAL, "'maxDepth' must be set to -1 (infinite) or a value greater than zero!");
    const HostScene &H = ctx->host;
    if ((uint64_t)P->x0 + P->width > H.film_w || (uint64_t)P->y0 + P->height > H.film_h)
        return fail(ctx, MTSGPU_EINVAL, "render window exceeds the film");
    if (P->cancel && *P->cancel) return fail(ctx, MTSGPU_ECANCEL, "cancelled");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    if (!stream) stream = ctx->stream;

    MtsgLaunch L;
    std::memset(&L, 0, sizeof L);
    L.scene = ctx->dscene;
    std::string err;
    if (mtsg_configure_filter(P->rfilter, P->rfilter_param, L.filter, err)) return fail(ctx, MTSGPU_EINVAL, err);
    // SobolSampler::setFilmResolution(cropSize, bucketed = true) (sobol.cpp:147-158)
    // the render window is the film's crop window: cropSize drives the sampler
    // (Integrator::configureSampler, integrator.cpp:37-41)
    const uint32_t mx = std::max(P->width, P->height);
    uint32_t r = mx - 1;
    r |= r >> 1; r |= r >> 2; r |= r >> 4; r |= r >> 8; r |= r >> 16; r += 1;
    uint32_t m = 0;
    while ((1u << m) < r) ++m;
    L.resolution = (float)r;
    L.diff_scale = 1.0f / std::sqrt((float)P->spp);   // integrator.cpp:144-145
    mtsg_sobol_lookup_table(m, L.lut);
    uint64_t scr = P->scramble;
    if (scr) scr = mtsg_sample_tea((uint32_t)scr, (uint32_t)(scr >> 32), 4);   // sobol.cpp:93-101
    L.scramble = (uint32_t)scr;
    L.scramble64 = scr;
    L.spp = P->spp;
    L.max_depth = P->max_depth;
    L.rr_depth = P->rr_depth;
    L.strict_normals = P->strict_normals;
    L.hide_emitters = P->hide_emitters;
    L.has_alpha = P->has_alpha;
    L.film_w = (int)H.film_w;
    L.film_h = (int)H.film_h;
    L.fw = (int)H.film_w + 2 * L.filter.border;
    L.fh = (int)H.film_h + 2 * L.filter.border;
    L.x0 = P->x0; L.y0 = P->y0; L.width = P->width; L.height = P->height;
    L.row_block = P->row_block ? P->row_block : 1;
    L.row_stride = P->row_stride ? P->row_stride : 1;
    L.row_phase = P->row_phase % L.row_stride;
    // work decomposition: compact rows (interleave) x columns in 8x8 tiles, or
    // (MTSGPU_FLAG_TILE_SHARD) every row_stride-th 8x8 tile of the window
    L.tile_shard = (P->flags & MTSGPU_FLAG_TILE_SHARD) ? 1u : 0u;
    L.tiles_x = (P->width + 7) / 8;
    if (L.tile_shard) {
        const uint64_t tiles = (uint64_t)L.tiles_x * ((P->height + 7) / 8);
        L.num_pixels = (uint32_t)((tiles + L.row_stride - 1) / L.row_stride * 64);
    } else {
        const uint32_t rowsCompact =
            ((P->height + L.row_block - 1) / L.row_block + L.row_stride - 1) / L.row_stride * L.row_block;
        const uint32_t tilesY = (rowsCompact + 7) / 8;
        L.num_pixels = L.tiles_x * tilesY * 64;
    }
    // Sobol index width: frame << 2m | 2m bits (sobolseq.h:93-125); 52 columns per dimension
    // the direct integrator's 2D sample arrays index the Sobol sequence at spp x count
    const bool direct = P->integrator == MTSGPU_INTEGRATOR_DIRECT;
    if (!pathLike && !direct) return fail(ctx, MTSGPU_EINVAL, "unknown integrator");
    if (direct && P->emitter_samples + P->bsdf_samples == 0)
        return fail(ctx, MTSGPU_EINVAL, "direct: emitterSamples + bsdfSamples must be positive");
    if (P->sampler < MTSGPU_SAMPLER_SOBOL || P->sampler > MTSGPU_SAMPLER_SFMT_BLOCKS)
        return fail(ctx, MTSGPU_EINVAL, "unknown sampler");
    const bool replay = P->sampler == MTSGPU_SAMPLER_SFMT_REPLAY || P->sampler == MTSGPU_SAMPLER_SFMT_BLOCKS;
    if (replay && (!pathLike || L.row_stride > 1 || P->width > 65535 || P->height > 65535))
        return fail(ctx, MTSGPU_EINVAL, "SFMT replay: path/volpath over a whole crop window (no row shards)");
    L.sampler = (uint32_t)P->sampler;
    const uint64_t perSampleIdx = direct ? std::max<uint64_t>(1, std::max(P->emitter_samples, P->bsdf_samples)) : 1;
    uint32_t sppBits = 0;
    while ((1ull << sppBits) < (uint64_t)P->spp * perSampleIdx) ++sppBits;
    const uint32_t indexBits = (m > 1 ? 2 * m : 0) + sppBits;
    if (L.sampler == MTSGPU_SAMPLER_SOBOL && indexBits > 52)
        return fail(ctx, MTSGPU_EINVAL, "sample index exceeds the 52-bit Sobol direction numbers");
    // independent streams are keyed by (x, y, sample): 16 + 16 + 32 bits
    if (L.sampler == MTSGPU_SAMPLER_INDEPENDENT && (H.film_w > 65536 || H.film_h > 65536 ||
                                                   (uint64_t)P->spp * perSampleIdx > 0xFFFFFFFFull))
        return fail(ctx, MTSGPU_EINVAL, "independent sampler: film or sample count too large for the stream key");
    L.nibbles = indexBits <= 32 ? 8 : MTSG_NIBBLES;
    L.lds_dims = 32;
    L.sobol_nib = (const uint32_t *)ctx->sobol.p;
    L.stack_depth = H.bvh_depth + 2;
    L.num_nodes = (uint32_t)H.nodes.size();
    // small scenes: stage the whole BVH + TriAccel array in LDS (<= 32 KiB)
    L.num_verts = (uint32_t)(H.positions.size() / 3);
    L.num_shapes = (uint32_t)H.shapes.size();
    const size_t sceneBytes = H.nodes.size() * sizeof(MtsgNode) + H.tris.size() * sizeof(MtsgTri) +
                              H.prim_vtx.size() * 4 + H.dpdu.size() * 4 + H.positions.size() * 4 +
                              H.normals.size() * 4 + H.shapes.size() * sizeof(MtsgShape);
    L.scene_lds = (sceneBytes <= (32u << 10) && !std::getenv("MTSGPU_NO_SCENE_LDS")) ? 1u : 0u;
    L.scan = (L.scene_lds && H.tris.size() <= MTSG_SCAN_MAX && H.analytic.empty() && !std::getenv("MTSGPU_NO_SCAN"))
                 ? 1u : 0u;
    L.scan_tris = (const MtsgTri *)ctx->scan_tris.p;
    for (int k = 0; k < 6; ++k) L.scan_n[k] = ctx->scan_n[k];
    // large scenes are latency-bound: run 4 waves/SIMD when 4 blocks' traversal
    // stacks + look_up tables fit the 160 KiB LDS, with as many Sobol dims in
    // LDS as the rest allows (the others are read through L1/L2)
    L.ext = H.ext ? 1u : 0u;
    L.ana = H.analytic.empty() ? 0u : 1u;
    // gfx950 has 32 CUs per XCD; the hardware deals workgroups round-robin over
    // the XCDs of the device (a CPX partition is one XCD: no remap).  A CU count
    // that is not a multiple of 32 is not a whole-XCD partition: no remap either.
    L.xcds = (ctx->num_cus % 32 == 0) ? (uint32_t)std::max(1, ctx->num_cus / 32) : 1u;
    L.all_diffuse = std::getenv("MTSGPU_NO_DIFF_VARIANT") ? 0u : 1u;
    for (const MtsgBsdf &b : H.bsdfs) L.all_diffuse &= b.type == MTSGPU_BSDF_DIFFUSE ? 1u : 0u;
    // the scene's BSDF set, for the specialised megakernel variants (dbsdf.h BSet)
    {
        bool ggx = true, rc = false, rd = false;
        for (const MtsgBsdf &b : H.bsdfs) {
            const bool rough = b.type == MTSGPU_BSDF_ROUGHCONDUCTOR || b.type == MTSGPU_BSDF_ROUGHDIELECTRIC ||
                               b.type == MTSGPU_BSDF_ROUGHPLASTIC;
            if (rough && b.distr != MTSGPU_DISTR_GGX) ggx = false;
            rc |= b.type == MTSGPU_BSDF_ROUGHCONDUCTOR;
            rd |= b.type == MTSGPU_BSDF_ROUGHDIELECTRIC;
        }
        // the set variants traverse half-float node boxes (layout.h MtsgHNode): a
        // scene beyond half range would get infinite (still exact, but useless) boxes
        float extent = 0.0f;
        for (int a = 0; a < 3; ++a) extent = std::max(extent, std::max(std::fabs(H.aabb_min[a]), std::fabs(H.aabb_max[a])));
        // (the set kernels are built without strictNormals: MTSG_FEAT_NOSTRICT)
        L.bset = (std::getenv("MTSGPU_NO_BSDF_SETS") || !(extent < 32768.0f) || P->strict_normals) ? 0u
                 : (ggx ? (uint32_t)MTSG_FEAT_GGX : 0u) | (rc ? 0u : (uint32_t)MTSG_FEAT_NORC) |
                       (rd ? 0u : (uint32_t)MTSG_FEAT_NORD);
        // envmap-only scenes (no area light, no constant emitter): the set kernels without
        // refN (MTSG_FEAT_NOREFN, dpath.h PathShader::REFN)
        bool envOnly = H.env.emitter >= 0 && !H.env.constant && !std::getenv("MTSGPU_NO_REFN_SPEC");
        for (const MtsgEmitter &em : H.emitters) envOnly &= em.type == MTSG_EMITTER_ENVMAP;
        if (L.bset && envOnly) L.bset |= (uint32_t)MTSG_FEAT_NOREFN;
    }
    // MIDirectIntegrator::configure / configureSampler (direct.cpp:128-143)
    L.integrator = P->integrator;
    L.array_end = 5;
    if (direct) {
        const uint32_t nl = P->emitter_samples, nb = P->bsdf_samples;
        const size_t sum = (size_t)nl + nb;
        L.lum_samples = nl;
        L.bsdf_samples = nb;
        L.weight_bsdf = 1 / (float)nb;
        L.weight_lum = 1 / (float)nl;
        L.frac_bsdf = nb / (float)sum;
        L.frac_lum = nl / (float)sum;
        if (nl > 1) { L.lum_dim = L.array_end; L.array_end += 2; }
        if (nb > 1) { L.bsdf_dim = L.array_end; L.array_end += 2; }
    }
    L.waves = 3;
    if (!L.scene_lds) {
        const size_t perBlock = (160u << 10) / 4;
        const size_t fixed = ((size_t)L.stack_depth * 3 * BLOCK_THREADS + 1) / 2 * 4 + 16 * 16 * 4;
        if (fixed < perBlock) {
            L.waves = 4;
            L.lds_dims = (uint32_t)std::min<size_t>(32, (perBlock - fixed) / ((size_t)L.nibbles * 16 * 4));
        }
    }
    // the all-diffuse variant makes no calls: 4 waves/SIMD (128 VGPRs) beat 3 (C2 +8.3%)
    // and 5 (-15%) (profiles/r02_ab_c2_waves4.log, r02_ab_c2_waves45.log)
    if (L.scene_lds && L.all_diffuse) L.waves = 4;
    if (const char *env = std::getenv("MTSGPU_WAVES")) {
        const int w = std::atoi(env);
        L.waves = w == 4 ? 4u : 3u;
    }
    L.round_shift = 0;   // set per chunk (run_shift)
    // gather mode (film_gather, path_kernel.hip): filters whose footprint covers the
    // neighbours (gaussian) -- every film pixel sums its neighbourhood's sample records in
    // a fixed order instead of taking atomic splats.  H = the largest footprint offset from a
    // sample's pixel: |x - px| <= floor(radius + 1/2) (film_splat's ceil/floor bounds)
    L.gather = 0;
    L.gather_h = 0;
    if (P->rfilter != MTSGPU_RFILTER_BOX) {
        const int H = std::max(L.filter.border, (int)std::floor(L.filter.radius + 0.5f));
        if (H >= 1 && H <= MTSG_GATHER_HMAX && !std::getenv("MTSGPU_NO_GATHER")) {
            L.gather = 1;
            L.gather_h = (uint32_t)H;
        }
    }
    if (const char *env = std::getenv("MTSGPU_SOBOL_LDS_DIMS"))
        L.lds_dims = (uint32_t)std::min(1024l, std::max(0l, std::strtol(env, nullptr, 10)));
    // own-pixel splat buffer [chunk][pixels] of float4; spp processed in chunks
    // that fit the budget: a quarter of the device's free HBM, at most 32 GiB
    // (C5's 1280x720x1024 splats, 15 GB, then run as one launch, one tail)
    size_t budget = (size_t)8 << 30;
    {
        size_t freeB = 0, totalB = 0;
        if (hipMemGetInfo(&freeB, &totalB) == hipSuccess && freeB / 4 > budget)
            budget = std::min<size_t>(freeB / 4 + ctx->contrib.bytes, (size_t)32 << 30);
    }
    if (const char *env = std::getenv("MTSGPU_CONTRIB_BYTES")) budget = std::max<size_t>(std::strtoull(env, nullptr, 10), 1 << 20);
    const size_t perSample = (size_t)L.num_pixels * (L.gather ? 32 : 16);   // one (gather mode: two) float4 per sample
    const uint32_t chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(P->spp, budget / perSample));
    const size_t filmFloats = (size_t)L.fw * L.fh * 5;
    if ((e = ctx->film_own.ensure(filmFloats * 4)) != hipSuccess || (e = ctx->film_spill.ensure(filmFloats * 8)) != hipSuccess ||
        (e = ctx->counters.ensure(16 * 8)) != hipSuccess || (e = ctx->contrib.ensure(perSample * (chunk + (chunk & 1)))) != hipSuccess)
        return hip_fail(ctx, e, "film allocation");
    float *own = film_dev ? film_dev : (float *)ctx->film_own.p;
    const size_t nsamp = samples_host ? (size_t)P->width * P->height * P->spp * MTSGPU_SAMPLE_RECORD_FLOATS : 0;
    if (nsamp) {
        if ((e = ctx->samples.ensure(nsamp * 4)) != hipSuccess) return hip_fail(ctx, e, "sample buffer");
        if ((e = hipMemsetAsync(ctx->samples.p, 0, nsamp * 4, stream)) != hipSuccess) return hip_fail(ctx, e, "memset");
    }
    if ((e = hipMemsetAsync(own, 0, filmFloats * 4, stream)) != hipSuccess ||
        (e = hipMemsetAsync(ctx->film_spill.p, 0, filmFloats * 8, stream)) != hipSuccess ||
        (e = hipMemsetAsync(ctx->counters.p, 0, 16 * 8, stream)) != hipSuccess)
        return hip_fail(ctx, e, "memset");
    L.film_own = own;
    L.film_spill = (double *)ctx->film_spill.p;
    L.samples = nsamp ? (float *)ctx->samples.p : nullptr;
    L.contrib = (float *)ctx->contrib.p;
    unsigned long long *cnt = (unsigned long long *)ctx->counters.p;
    L.counters = cnt;

    int bpc = 0;
    mtsg_path_kernel_occupancy(L, &bpc);
    if (bpc <= 0) bpc = 1;
    const bool stats_mode = (P->flags & MTSGPU_FLAG_TRAVERSAL_STATS) != 0;
    if (replay) {
        // IndependentSampler's Random() = seed(5489); RenderJob clones it per worker in
        // order (renderjob.cpp:58-66).  Units: one worker over all blocks, or one per block
        if (chunk < P->spp) return fail(ctx, MTSGPU_EINVAL, "SFMT replay: sampleCount exceeds one chunk");
        std::vector<uint32_t> order, blockStart;
        mtsg_render_order(P->width, P->height, MTSG_BLOCK_SIZE, order, blockStart);
        std::vector<uint32_t> unitStart;
        if (P->sampler == MTSGPU_SAMPLER_SFMT_BLOCKS) unitStart = blockStart;
        else unitStart = {0u, (uint32_t)order.size()};
        const uint32_t units = (uint32_t)unitStart.size() - 1;
        std::vector<uint32_t> streams((size_t)units * MTSG_SFMT_WORDS, 0u), master(MTSG_SFMT_WORDS, 0u);
        mtsg_sfmt_seed(master.data(), 5489ull);
        for (uint32_t u = 0; u < units; ++u) mtsg_sfmt_clone(streams.data() + (size_t)u * MTSG_SFMT_WORDS, master.data());
        if ((e = upload(ctx->rp_order, order, stream)) != hipSuccess || (e = upload(ctx->rp_start, unitStart, stream)) != hipSuccess ||
            (e = upload(ctx->rp_sfmt, streams, stream)) != hipSuccess ||
            (e = hipStreamSynchronize(stream)) != hipSuccess)   // the host vectors go out of scope
            return hip_fail(ctx, e, "replay upload");
        L.replay = 1;
        L.units = units;
        L.order = (const uint32_t *)ctx->rp_order.p;
        L.unit_start = (const uint32_t *)ctx->rp_start.p;
        L.sfmt = (uint32_t *)ctx->rp_sfmt.p;
    }
    // execution engine (same per-sample results): the wavefront pipeline or the megakernel
    bool wave = false;   // default: the megakernel (DESIGN.md 4 has the engine A/B)
    if (const char *env = std::getenv("MTSGPU_ENGINE")) wave = pathLike && std::strcmp(env, "wavefront") == 0;
    if (P->flags & MTSGPU_FLAG_WAVEFRONT) wave = pathLike;
    if (P->flags & MTSGPU_FLAG_MEGAKERNEL) wave = false;
    if (replay) wave = false;   // one lane per replay unit
    if (P->flags & MTSGPU_FLAG_KDTREE) {
        // the reference's own kd-tree: the wavefront engine with wf_trace_kd
        if (!pathLike || replay)
            return fail(ctx, MTSGPU_EINVAL, "kd-tree traversal: path / volpath with the sobol or independent sampler");
        if (P->flags & MTSGPU_FLAG_MEGAKERNEL) return fail(ctx, MTSGPU_EINVAL, "kd-tree traversal runs in the wavefront engine");
        const int rc = ensure_kdtree(ctx);
        if (rc) return rc;
        wave = true;
        L.kd_nodes = (const uint32_t *)ctx->kd_nodes.p;
        L.kd_indices = (const uint32_t *)ctx->kd_indices.p;
        L.kd_tris = (const MtsgTri *)ctx->kd_tris.p;
    }
    WfPlan plan;
    if (wave) {
        std::vector<uint32_t> &shapeKind = ctx->wf_kind_host;   // kept alive for the async upload
        wf_kinds(ctx->host, shapeKind, plan);
        const size_t R = MTSG_WF_REGIONS;
        for (int k = 0; k < MTSG_WK_KINDS; ++k) {
            if (!plan.kinds[k]) continue;
            int sb = 0, tb = 0;
            mtsg_wf_occupancy(L, k, plan.ggx[k], &sb, &tb);
            if (sb <= 0 || tb <= 0) return fail(ctx, MTSGPU_EHIP, "wavefront kernels do not fit the device");
        }
        // path slots: about 2M (MTSGPU_WF_SLOTS), whole blocks; the kernels run one queue
        // entry per thread, so each grid covers the largest its queues can be (slots;
        // 2 x slots for the trace kernel's two ray queues) and surplus blocks exit at once
        uint64_t target = (uint64_t)1 << 21;
        if (const char *env = std::getenv("MTSGPU_WF_SLOTS")) target = std::max<uint64_t>(1, std::strtoull(env, nullptr, 10));
        const uint64_t items = (uint64_t)std::min(chunk, P->spp) * L.num_pixels;
        target = std::min(target, items);
        plan.slots = (uint32_t)((std::max<uint64_t>(1, target) + BLOCK_THREADS - 1) / BLOCK_THREADS * BLOCK_THREADS);
        for (int k = 0; k < MTSG_WK_KINDS; ++k)
            if (plan.kinds[k]) plan.shadeGrid[k] = (int)(plan.slots / BLOCK_THREADS);
        plan.traceGrid = (int)(2 * (uint64_t)plan.slots / BLOCK_THREADS);
        plan.hitrec = wf_hitrec_on();
        const size_t slots = plan.slots;
        size_t cap, capCls;
        wf_caps(slots, cap, capCls);
        const size_t ovfDepth = L.stack_depth > MTSG_WF_LDS_STACK ? L.stack_depth - MTSG_WF_LDS_STACK : 0;
        int partBlocks = plan.traceGrid;
        for (int k = 0; k < MTSG_WK_KINDS; ++k) partBlocks = std::max(partBlocks, plan.shadeGrid[k]);
        if ((e = ctx->wf_state.ensure((size_t)MTSG_WF_STATE_VECS * slots * 16)) != hipSuccess ||
            (e = ctx->wf_ray.ensure((size_t)2 * 2 * R * cap * 32)) != hipSuccess ||
            (e = ctx->wf_rslot.ensure((size_t)2 * 2 * R * cap * 4)) != hipSuccess ||
            (e = ctx->wf_cls.ensure((size_t)2 * MTSG_WK_KINDS * R * capCls * 4)) != hipSuccess ||
            (e = ctx->wf_cnt.ensure((size_t)2 * MTSG_WF_QUEUES * R * 4)) != hipSuccess ||
            (e = ctx->wf_hit.ensure(slots * 16)) != hipSuccess ||
            (plan.hitrec && (e = ctx->wf_hitrec.ensure(slots * MTSG_WF_HIT_VECS * 16)) != hipSuccess) ||
            (e = ctx->wf_occl.ensure(slots * 4)) != hipSuccess ||
            (e = ctx->wf_live.ensure(2 * 4)) != hipSuccess ||
            (e = ctx->wf_ovf.ensure((size_t)plan.traceGrid * BLOCK_THREADS * ovfDepth * 8)) != hipSuccess ||
            (e = ctx->wf_part.ensure((size_t)partBlocks * 16 * 8)) != hipSuccess ||
            (e = upload(ctx->wf_kind, shapeKind, stream)) != hipSuccess)
            return hip_fail(ctx, e, "wavefront buffers");
        if (!ctx->wf_live_host) {
            if ((e = hipHostMalloc((void **)&ctx->wf_live_host, 8 * sizeof(uint32_t))) != hipSuccess)
                return hip_fail(ctx, e, "wavefront pinned buffer");
            for (hipEvent_t &ev : ctx->wf_ev)
                if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return hip_fail(ctx, e, "event");
        }
    }
    if ((e = hipEventRecord(ctx->ev0, stream)) != hipSuccess) return hip_fail(ctx, e, "event");
    for (uint32_t j0 = 0; j0 < P->spp; j0 += chunk) {
        if (P->cancel && *P->cancel) break;
        L.j0 = j0;
        L.chunk_spp = std::min(chunk, P->spp - j0);
        L.num_items = (uint64_t)L.chunk_spp * L.num_pixels;
        if (wave) {
            const int rc = wf_render_chunk(ctx, L, nsamp != 0 || stats_mode, stats_mode, stream, plan, P->cancel);
            if (rc != MTSGPU_OK) return rc;
        } else {
            const uint64_t blocksNeeded = replay ? (L.units + 255) / 256 : (L.num_items + 255) / 256;
            const int grid = (int)std::min<uint64_t>((uint64_t)ctx->num_cus * bpc, std::max<uint64_t>(1, blocksNeeded));
            // the replay renders one unit per lane (its own SFMT stream): every unit needs a resident lane
            if (replay && (uint64_t)grid * 256 < L.units)
                return fail(ctx, MTSGPU_EINVAL, "SFMT replay: more 32x32 blocks than resident lanes (crop too large)");
            L.round_shift = run_shift(L, (uint64_t)grid * BLOCK_THREADS);
            if ((e = mtsg_launch_path(L, grid, nsamp != 0, stats_mode, stream)) != hipSuccess) return hip_fail(ctx, e, "path kernel launch");
        }
        if ((e = L.gather ? mtsg_launch_gather(L, stream) : mtsg_launch_reduce(L, stream)) != hipSuccess)
            return hip_fail(ctx, e, "film reduce launch");
    }
    if ((e = hipEventRecord(ctx->ev1, stream)) != hipSuccess) return hip_fail(ctx, e, "event");
    if ((e = mtsg_launch_finalize(own, L.film_spill, filmFloats, stream)) != hipSuccess) return hip_fail(ctx, e, "finalize launch");
    unsigned long long hc[16];
    if ((e = hipMemcpyAsync(hc, cnt, sizeof hc, hipMemcpyDeviceToHost, stream)) != hipSuccess) return hip_fail(ctx, e, "counters");
    if (film_host && (e = hipMemcpyAsync(film_host, own, filmFloats * 4, hipMemcpyDeviceToHost, stream)) != hipSuccess)
        return hip_fail(ctx, e, "film copy");
    if (nsamp && (e = hipMemcpyAsync(samples_host, ctx->samples.p, nsamp * 4, hipMemcpyDeviceToHost, stream)) != hipSuccess)
        return hip_fail(ctx, e, "sample copy");
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(ctx, e, "path kernel");
    std::memcpy(ctx->last_counters, hc, sizeof hc);
    // counter 15: which kernel ran -- for the megakernel path_kernel<INSTR, SCENE_LDS, FEAT, WAVES>:
    // FEAT's low 8 bits | WAVES << 8 | SCENE_LDS << 12 | INSTR << 13 | (FEAT & NOSTRICT) << 14 (the
    // set kernels' strictNormals-free build) | (FEAT & NOREFN) << 15; 1 << 16 for the wavefront engine
    // (tests and A/B logs read it)
    if (wave) {
        ctx->last_counters[15] = 1ull << 16;
    } else {
        const int v = mtsg_path_variant(L);
        ctx->last_counters[15] = (unsigned long long)((v & 0xff) | (int)(L.waves << 8) | (int)(L.scene_lds << 12) |
                                                      ((nsamp != 0 || stats_mode) ? 1 << 13 : 0) |
                                                      ((v & MTSG_FEAT_NOSTRICT) ? 1 << 14 : 0) |
                                                      ((v & MTSG_FEAT_NOREFN) ? 1 << 15 : 0));
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
    if (stats) {
        stats->samples = hc[0];
        stats->rays = hc[1];
        stats->shadow_rays = hc[2];
        stats->path_length_sum = hc[3];
        stats->node_visits = stats_mode ? hc[4] : 0;
        stats->tri_tests = stats_mode ? hc[5] : 0;
        stats->hits = stats_mode ? hc[7] : 0;
        stats->nee_samples = stats_mode ? hc[9] : 0;
        stats->sobol_reads = stats_mode ? hc[10] : 0;
        stats->kernel_ms = ms;
    }
    if (hc[6]) return fail(ctx, MTSGPU_EDIM, "Lookup dimension exceeds the direction number table size! You may have to "
                                             "reduce the 'maxDepth' parameter of your integrator.");
    if (P->cancel && *P->cancel) return fail(ctx, MTSGPU_ECANCEL, "cancelled");
    return MTSGPU_OK;
}

int mtsgpu_render(mtsgpu_ctx *ctx, const mtsgpu_render_params *params, float *film, float *samples, mtsgpu_stats *stats) {
    if (!film) return fail(ctx, MTSGPU_EINVAL, "film buffer is NULL");
    return render_impl(ctx, params, film, nullptr, samples, nullptr, stats);
}

int mtsgpu_render_device(mtsgpu_ctx *ctx, const mtsgpu_render_params *params, float *film_device, void *stream,
                         mtsgpu_stats *stats) {
    if (!film_device) return fail(ctx, MTSGPU_EINVAL, "film buffer is NULL");
    return render_impl(ctx, params, nullptr, film_device, nullptr, (hipStream_t)stream, stats);
}

// hdrfilm develop (film_kernel.hip)
namespace {
int develop_check(mtsgpu_ctx *ctx, const mtsgpu_develop_params *P, size_t *out_bytes) {
    if (!ctx) return MTSGPU_EINVAL;
    if (!P) return fail(ctx, MTSGPU_EINVAL, "develop params are NULL");
    const int ch = mtsg_develop_channels(P->pixel_format);
    if (!ch) return fail(ctx, MTSGPU_EINVAL, "develop: unknown pixel format");
    if (P->component_format < MTSGPU_COMP_FLOAT16 || P->component_format > MTSGPU_COMP_UINT32)
        return fail(ctx, MTSGPU_EINVAL, "develop: unknown component format");
    if (P->film_width <= 2 * P->border || P->film_height <= 2 * P->border)
        return fail(ctx, MTSGPU_EINVAL, "develop: film smaller than its borders");
    const size_t n = (size_t)(P->film_width - 2 * P->border) * (P->film_height - 2 * P->border);
    *out_bytes = n * ch * (P->component_format == MTSGPU_COMP_FLOAT16 ? 2 : 4);
    return MTSGPU_OK;
}
}  // namespace

int mtsgpu_develop_device(mtsgpu_ctx *ctx, const mtsgpu_develop_params *P, const float *film_device,
                          void *out_device, void *stream) {
    size_t ob = 0;
    int rc = develop_check(ctx, P, &ob);
    if (rc != MTSGPU_OK) return rc;
    if (!film_device || !out_device) return fail(ctx, MTSGPU_EINVAL, "develop: NULL buffer");
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    hipError_t e = mtsg_launch_develop(*P, film_device, out_device, ctx->num_cus, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e == hipSuccess ? MTSGPU_OK : hip_fail(ctx, e, "develop");
}

int mtsgpu_develop(mtsgpu_ctx *ctx, const mtsgpu_develop_params *P, const float *film, void *out) {
    size_t ob = 0;
    int rc = develop_check(ctx, P, &ob);
    if (rc != MTSGPU_OK) return rc;
    if (!film || !out) return fail(ctx, MTSGPU_EINVAL, "develop: NULL buffer");
    (void)hipSetDevice(ctx->device);
    const size_t ib = (size_t)P->film_width * P->film_height * 5 * sizeof(float);
    hipError_t e;
    if ((e = ctx->dev_in.ensure(ib)) != hipSuccess || (e = ctx->dev_out.ensure(ob)) != hipSuccess)
        return hip_fail(ctx, e, "develop buffers");
    hipStream_t s = ctx->stream;
    if ((e = hipMemcpyAsync(ctx->dev_in.p, film, ib, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = mtsg_launch_develop(*P, (const float *)ctx->dev_in.p, ctx->dev_out.p, ctx->num_cus, s)) != hipSuccess ||
        (e = hipMemcpyAsync(out, ctx->dev_out.p, ob, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return hip_fail(ctx, e, "develop");
    return MTSGPU_OK;
}

const char *mtsgpu_last_error(mtsgpu_ctx *ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

void mtsgpu_destroy(mtsgpu_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    DevBuf *bufs[] = {&ctx->scan_tris, &ctx->kd_nodes, &ctx->kd_indices, &ctx->kd_tris, &ctx->nodes, &ctx->hnodes, &ctx->tris, &ctx->prim_vtx, &ctx->dpdu, &ctx->positions, &ctx->normals,
                      &ctx->shapes, &ctx->bsdfs, &ctx->emitters, &ctx->area_cdf, &ctx->em_cdf, &ctx->sobol,
                      &ctx->film_own, &ctx->film_spill, &ctx->samples, &ctx->counters, &ctx->contrib,
                      &ctx->env, &ctx->env_texels, &ctx->env_rows, &ctx->env_cols, &ctx->env_weights, &ctx->env_grows, &ctx->env_gcols,
                      &ctx->rtrans, &ctx->texcoords, &ctx->qrays, &ctx->qhits,
                      &ctx->dev_in, &ctx->dev_out, &ctx->wf_state, &ctx->wf_ray, &ctx->wf_rslot, &ctx->wf_cls,
                      &ctx->wf_cnt, &ctx->wf_hit, &ctx->wf_hitrec, &ctx->wf_occl, &ctx->wf_live, &ctx->wf_ovf, &ctx->wf_part, &ctx->wf_kind, &ctx->rp_order, &ctx->rp_start, &ctx->rp_sfmt, &ctx->env_grows, &ctx->env_gcols};
    for (DevBuf *b : bufs) b->release();
    for (hipEvent_t &e : ctx->wf_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->wf_live_host) (void)hipHostFree(ctx->wf_live_host);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

namespace {
// the kd-tree over the uploaded scene's triangles (global primitive order: the
// TriAccel slots carry their primitive number), uploaded with TriAccel records
// in that order; scenes with analytic shapes are not supported here
// host part: the tree over the configured scene's triangles in global order
int build_kd_host(const HostScene &H, KdTree &kd, std::vector<MtsgTri> *tg, std::string &err) {
    if (!H.analytic.empty()) { err = "kd-tree: scenes with analytic shapes are not supported"; return MTSGPU_EINVAL; }
    const size_t prims = H.tris.size();
    std::vector<float> P(prims * 9);
    if (tg) tg->assign(prims, MtsgTri());
    for (size_t s = 0; s < prims; ++s) {
        const uint32_t prim = H.tris[s].prim;
        if (prim >= prims) { err = "kd-tree: primitive numbering"; return MTSGPU_EINVAL; }
        if (tg) (*tg)[prim] = H.tris[s];
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k)   // prim_vtx is in global primitive order (only the TriAccel slots are in leaf order)
                P[9 * (size_t)prim + 3 * v + k] = H.positions[3 * (size_t)H.prim_vtx[4 * (size_t)prim + v] + k];
    }
    if (!mtsg_build_kdtree(P.data(), (uint32_t)prims, kd, true)) {
        err = "kd-tree: a child offset exceeds KDNode's 28-bit relative field (indirection nodes are not supported)";
        return MTSGPU_EINVAL;
    }
    return MTSGPU_OK;
}

void kd_export(const KdTree &K, uint32_t *nodes, size_t node_cap, uint32_t *indices, size_t index_cap, uint32_t *info8) {
    const uint32_t v[8] = {(uint32_t)(K.nodes.size() / 2), (uint32_t)K.indices.size(), K.stats.inner, K.stats.leaves,
                           K.stats.nonempty_leaves, K.stats.retracted, K.stats.pruned, K.stats.max_depth};
    std::memcpy(info8, v, sizeof v);
    if (nodes && node_cap >= K.nodes.size()) std::memcpy(nodes, K.nodes.data(), K.nodes.size() * 4);
    if (indices && index_cap >= K.indices.size()) std::memcpy(indices, K.indices.data(), K.indices.size() * 4);
}

int ensure_kdtree(mtsgpu_ctx *ctx) {
    if (ctx->kd_built) return MTSGPU_OK;
    std::vector<MtsgTri> tg;
    std::string err;
    int rc = build_kd_host(ctx->host, ctx->kd, &tg, err);
    if (rc) return fail(ctx, rc, err);
    (void)hipSetDevice(ctx->device);
    hipError_t e;
    // the TriAccel records in leaf-list order (one per primitive reference), so a
    // leaf's records are read without the indices[e] -> record dependence
    if (ctx->kd.nodes.size() / 2 >= (1u << 30)) return fail(ctx, MTSGPU_EINVAL, "kd-tree: more than 2^30 nodes");
    std::vector<MtsgTri> lt(ctx->kd.indices.size());
    for (size_t i = 0; i < lt.size(); ++i) lt[i] = tg[ctx->kd.indices[i]];
    lt.push_back(MtsgTri{});   // one record past the last entry (reading ahead in the leaf loop lost 1-3%, r05)
    if ((e = upload(ctx->kd_nodes, ctx->kd.nodes, ctx->stream)) != hipSuccess ||
        (e = upload(ctx->kd_indices, ctx->kd.indices, ctx->stream)) != hipSuccess ||
        (e = upload(ctx->kd_tris, lt, ctx->stream)) != hipSuccess || (e = hipStreamSynchronize(ctx->stream)) != hipSuccess)
        return hip_fail(ctx, e, "kd-tree upload");
    ctx->kd_built = true;
    return MTSGPU_OK;
}
}  // namespace

int mtsgpu_trace_rays(mtsgpu_ctx *ctx, const float *rays, uint32_t n, int shadow, float *hits, double *kernel_ms) {
    return mtsgpu_trace_rays_ex(ctx, rays, n, shadow ? MTSGPU_TRACE_SHADOW : 0u, hits, kernel_ms);
}

int mtsgpu_debug_kdtree(mtsgpu_ctx *ctx, uint32_t *nodes, size_t node_cap, uint32_t *indices, size_t index_cap,
                        uint32_t *info8) {
    if (!ctx || !info8) return MTSGPU_EINVAL;
    if (!ctx->have_scene) return fail(ctx, MTSGPU_ESTATE, "debug_kdtree before upload_scene");
    int rc = ensure_kdtree(ctx);
    if (rc) return rc;
    kd_export(ctx->kd, nodes, node_cap, indices, index_cap, info8);
    return MTSGPU_OK;
}

int mtsgpu_bvh_host(const mtsgpu_scene_desc *scene, uint32_t *nodes, size_t node_cap, uint32_t *hnodes,
                    size_t hnode_cap, uint32_t *qnodes, size_t qnode_cap, uint32_t *info4, char *msg, size_t cap) {
    if (!scene || !info4) return MTSGPU_EINVAL;
    HostScene H;
    std::string err;
    const int rc = mtsg_configure_scene(scene, H, err);
    if (msg && cap) {
        std::strncpy(msg, err.c_str(), cap - 1);
        msg[cap - 1] = 0;
    }
    if (rc) return rc;
    mtsg_build_qnodes(H);
    info4[0] = (uint32_t)H.nodes.size();
    info4[1] = (uint32_t)H.hnodes.size();
    info4[2] = (uint32_t)H.qnodes.size();
    info4[3] = H.qnode_depth;
    if (nodes && node_cap >= H.nodes.size() * 16) std::memcpy(nodes, H.nodes.data(), H.nodes.size() * 64);
    if (hnodes && hnode_cap >= H.hnodes.size() * 8) std::memcpy(hnodes, H.hnodes.data(), H.hnodes.size() * 32);
    if (qnodes && qnode_cap >= H.qnodes.size() * 16) std::memcpy(qnodes, H.qnodes.data(), H.qnodes.size() * 64);
    return MTSGPU_OK;
}

int mtsgpu_kdtree_host(const mtsgpu_scene_desc *scene, uint32_t *nodes, size_t node_cap, uint32_t *indices,
                       size_t index_cap, uint32_t *info8, char *msg, size_t cap) {
    if (!scene || !info8) return MTSGPU_EINVAL;
    HostScene H;
    KdTree K;
    std::string err;
    int rc = mtsg_configure_scene(scene, H, err);
    if (!rc) rc = build_kd_host(H, K, nullptr, err);
    if (msg && cap) {
        std::strncpy(msg, err.c_str(), cap - 1);
        msg[cap - 1] = 0;
    }
    if (!rc) kd_export(K, nodes, node_cap, indices, index_cap, info8);
    return rc;
}

int mtsgpu_trace_rays_ex(mtsgpu_ctx *ctx, const float *rays, uint32_t n, uint32_t flags, float *hits,
                         double *kernel_ms) {
    const int shadow = (flags & MTSGPU_TRACE_SHADOW) ? 1 : 0;
    if (!ctx) return MTSGPU_EINVAL;
    if (!ctx->have_scene) return fail(ctx, MTSGPU_ESTATE, "trace_rays before upload_scene");
    if (!rays || !hits) return fail(ctx, MTSGPU_EINVAL, "trace_rays: NULL buffer");
    if (n == 0) return MTSGPU_OK;
    if (flags & MTSGPU_TRACE_KDTREE) {
        int rc = ensure_kdtree(ctx);
        if (rc) return rc;
    }
    (void)hipSetDevice(ctx->device);
    hipError_t e;
    if ((e = ctx->qrays.ensure((size_t)n * 32)) != hipSuccess || (e = ctx->qhits.ensure((size_t)n * 16)) != hipSuccess)
        return hip_fail(ctx, e, "trace buffers");
    hipStream_t s = ctx->stream;
    if ((e = hipMemcpyAsync(ctx->qrays.p, rays, (size_t)n * 32, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipEventRecord(ctx->ev0, s)) != hipSuccess ||
        (e = (flags & MTSGPU_TRACE_KDTREE)
                 ? mtsg_launch_trace_kd(ctx->dscene, (const uint32_t *)ctx->kd_nodes.p, (const uint32_t *)ctx->kd_indices.p,
                                        (const MtsgTri *)ctx->kd_tris.p, (const float *)ctx->qrays.p, n,
                                        (float *)ctx->qhits.p, shadow != 0, ctx->num_cus, s)
                 : mtsg_launch_trace(ctx->dscene, (const float *)ctx->qrays.p, n, (float *)ctx->qhits.p, shadow != 0,
                                     ctx->host.bvh_depth + 2, ctx->num_cus, s)) != hipSuccess ||
        (e = hipEventRecord(ctx->ev1, s)) != hipSuccess ||
        (e = hipMemcpyAsync(hits, ctx->qhits.p, (size_t)n * 16, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return hip_fail(ctx, e, "trace_rays");
    if (kernel_ms) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
        *kernel_ms = ms;
    }
    return MTSGPU_OK;
}

// diagnostics: device arithmetic probe (tests/test_gpu_arith.py)
int mtsgpu_debug_arith(mtsgpu_ctx *ctx, const float *a, const float *b, float *out, int n) {
    if (!ctx || n <= 0) return MTSGPU_EINVAL;
    float *da = nullptr, *db = nullptr, *dout = nullptr;
    hipError_t e;
    if ((e = hipMalloc(&da, n * 4)) != hipSuccess || (e = hipMalloc(&db, n * 4)) != hipSuccess ||
        (e = hipMalloc(&dout, (size_t)n * 32)) != hipSuccess)
        return hip_fail(ctx, e, "malloc");
    (void)hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, b, n * 4, hipMemcpyHostToDevice);
    e = mtsg_launch_arith_probe(da, db, dout, n, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 32, hipMemcpyDeviceToHost);
    (void)hipFree(da); (void)hipFree(db); (void)hipFree(dout);
    return e == hipSuccess ? MTSGPU_OK : hip_fail(ctx, e, "arith probe");
}

// diagnostics: the device's transcendentals over inputs (tests/test_gpu_libm.py)
int mtsgpu_debug_libm(mtsgpu_ctx *ctx, int fn, const float *a, const float *b, float *out, size_t n,
                      uint32_t first) {
    if (!ctx || !out || n == 0 || fn < 0 || fn > 9 || ((fn == 6 || fn == 7) && a && !b)) return MTSGPU_EINVAL;
    (void)hipSetDevice(ctx->device);
    float *da = nullptr, *db = nullptr, *dout = nullptr;
    hipError_t e = hipMalloc(&dout, n * 4);
    if (e == hipSuccess && a) e = hipMalloc(&da, n * 4);
    if (e == hipSuccess && b) e = hipMalloc(&db, n * 4);
    if (e == hipSuccess && a) e = hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && b) e = hipMemcpy(db, b, n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = mtsg_launch_libm_probe(fn, da, db, dout, n, first, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost);
    if (da) (void)hipFree(da);
    if (db) (void)hipFree(db);
    if (dout) (void)hipFree(dout);
    return e == hipSuccess ? MTSGPU_OK : hip_fail(ctx, e, "libm probe");
}

// diagnostics: n nextULong draws of the device's SFMT19937 from Random(seed), or
// from its clone-th Random(&master) clone (host seeding, device generation)
int mtsgpu_debug_sfmt(mtsgpu_ctx *ctx, uint64_t seed, int clone, uint64_t *out, int n) {
    if (!ctx || !out || n <= 0 || clone < 0) return MTSGPU_EINVAL;
    std::vector<uint32_t> master(MTSG_SFMT_WORDS, 0u), child(MTSG_SFMT_WORDS, 0u);
    mtsg_sfmt_seed(master.data(), seed);
    for (int k = 0; k < clone; ++k) mtsg_sfmt_clone(child.data(), master.data());
    const std::vector<uint32_t> &st = clone > 0 ? child : master;
    uint32_t *dw = nullptr;
    unsigned long long *dout = nullptr;
    hipError_t e;
    (void)hipSetDevice(ctx->device);
    if ((e = hipMalloc(&dw, MTSG_SFMT_WORDS * 4)) != hipSuccess || (e = hipMalloc(&dout, (size_t)n * 8)) != hipSuccess) {
        if (dw) (void)hipFree(dw);
        return hip_fail(ctx, e, "malloc");
    }
    e = hipMemcpy(dw, st.data(), MTSG_SFMT_WORDS * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = mtsg_launch_sfmt_probe(dw, dout, n, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 8, hipMemcpyDeviceToHost);
    (void)hipFree(dw);
    (void)hipFree(dout);
    return e == hipSuccess ? MTSGPU_OK : hip_fail(ctx, e, "sfmt probe");
}

int mtsgpu_debug_counters(mtsgpu_ctx *ctx, uint64_t *out16) {
    if (!ctx || !out16) return MTSGPU_EINVAL;
    for (int k = 0; k < 16; ++k) out16[k] = ctx->last_counters[k];
    return MTSGPU_OK;
}

// diagnostics: BVH statistics of the uploaded scene
int mtsgpu_debug_scene_info(mtsgpu_ctx *ctx, uint32_t *info4) {
    if (!ctx || !ctx->have_scene || !info4) return MTSGPU_EINVAL;
    info4[0] = (uint32_t)ctx->host.nodes.size();
    info4[1] = (uint32_t)ctx->host.tris.size();
    info4[2] = ctx->host.bvh_depth;
    info4[3] = (uint32_t)ctx->num_cus;
    return MTSGPU_OK;
}

// diagnostics: host-side environment tables (tests/test_host_configure.py)
int mtsgpu_debug_env_tables(const mtsgpu_scene_desc *scene, float *params, uint16_t *texels, size_t texel_cap,
                            float *rows, float *cols, float *weights) {
    HostScene H;
    std::string err;
    const int rc = mtsg_configure_scene(scene, H, err);
    if (rc) { g_create_error = err; return rc; }
    const MtsgEnv &E = H.env;
    if (E.emitter < 0) { g_create_error = "scene has no environment emitter"; return MTSGPU_EINVAL; }
    if (params) {
        std::memset(params, 0, 64 * sizeof(float));
        params[0] = (float)E.levels; params[1] = (float)E.w0; params[2] = (float)E.h0;
        params[3] = E.normalization; params[4] = E.pixel_x; params[5] = E.pixel_y; params[6] = E.scale;
        params[7] = E.center[0]; params[8] = E.center[1]; params[9] = E.center[2]; params[10] = E.radius;
        params[11] = (float)(H.env_texels.size() / 4);
        for (int l = 0; l < E.levels && l < MTSG_ENV_MAX_LEVELS; ++l) { params[16 + l] = (float)E.lw[l]; params[34 + l] = (float)E.lh[l]; }
    }
    if (texels) {
        if (texel_cap < H.env_texels.size()) return MTSGPU_EINVAL;
        std::memcpy(texels, H.env_texels.data(), H.env_texels.size() * sizeof(uint16_t));
    }
    if (rows) std::memcpy(rows, H.env_cdf_rows.data(), H.env_cdf_rows.size() * sizeof(float));
    if (cols) std::memcpy(cols, H.env_cdf_cols.data(), H.env_cdf_cols.size() * sizeof(float));
    if (weights) std::memcpy(weights, H.env_row_weights.data(), H.env_row_weights.size() * sizeof(float));
    return MTSGPU_OK;
}

}  // extern "C"
