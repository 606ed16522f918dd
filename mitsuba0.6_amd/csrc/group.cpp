// Device groups: one render call over several GPUs of a node (SURVEY.md 8(b):
// "Multi-GPU happens inside render").  The reference parallelises a render
// over 32x32 blocks handed to worker threads and sums their ImageBlocks into
// the film (BlockedImageProcess, src/librender/imageproc.cpp:28-80;
// BlockedRenderProcess::processResult -> Film::put, renderproc.cpp:142-149).
// Here each GPU is a worker with a fixed share of interleaved 8x8 tiles; it
// renders them into a film of its own in HBM, and the films are merged on the
// first member's device: a peer copy over xGMI, then dst += src, in member
// order, so the merged film does not depend on which member finished first.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mtsgpu.h"

hipError_t mtsg_launch_film_accumulate(float *dst, const float *src, size_t n, int num_cus, hipStream_t s);

namespace {
thread_local std::string g_group_create_error;

struct Member {
    int device = 0;
    int num_cus = 0;
    mtsgpu_ctx *ctx = nullptr;
    float *film = nullptr;       // this member's film in its own HBM
    size_t film_bytes = 0;
    int rc = MTSGPU_OK;
    std::string err;
    mtsgpu_stats stats{};
};
}  // namespace

struct mtsgpu_group {
    std::vector<Member> m;
    hipStream_t stream = nullptr;    // merge stream on member 0's device
    float *stage = nullptr;          // peer-copy landing buffer on member 0's device
    size_t stage_bytes = 0;
    uint32_t film_w = 0, film_h = 0;
    bool have_scene = false;
    std::string err;
};

namespace {

int gfail(mtsgpu_group *g, int code, const std::string &msg) {
    g->err = msg;
    return code;
}

int ghip(mtsgpu_group *g, hipError_t e, const char *what) {
    return gfail(g, e == hipErrorOutOfMemory ? MTSGPU_ENOMEM : MTSGPU_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

hipError_t ensure(float *&p, size_t &have, size_t want) {
    if (want <= have && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    have = 0;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) have = want;
    return e;
}

// runs f(k) on one host thread per member and returns the first failing member's index (or -1)
template <class F>
int for_members(mtsgpu_group *g, F f) {
    std::vector<std::thread> th;
    th.reserve(g->m.size());
    for (size_t k = 0; k < g->m.size(); ++k) th.emplace_back([&, k] { f(g->m[k], (int)k); });
    for (auto &t : th) t.join();
    for (size_t k = 0; k < g->m.size(); ++k)
        if (g->m[k].rc != MTSGPU_OK) return (int)k;
    return -1;
}

void add_stats(mtsgpu_stats &a, const mtsgpu_stats &b) {
    a.samples += b.samples; a.rays += b.rays; a.shadow_rays += b.shadow_rays;
    a.path_length_sum += b.path_length_sum; a.node_visits += b.node_visits; a.tri_tests += b.tri_tests;
    a.hits += b.hits; a.nee_samples += b.nee_samples; a.sobol_reads += b.sobol_reads;
    a.kernel_ms = std::max(a.kernel_ms, b.kernel_ms);
}

}  // namespace

extern "C" {

// member k's share of an n-member render: the bench's decomposition
// (MTSGPU_FLAG_TILE_SHARD), the window's 8x8 tiles t with t % n == k, so the
// members' pixel counts differ by at most one tile (the reference deals its
// 32x32 blocks to workers: BlockedImageProcess, imageproc.cpp:28-80)
int mtsgpu_group_member_params(const mtsgpu_render_params *params, int n, int k, mtsgpu_render_params *out) {
    if (!params || !out || n <= 0 || k < 0 || k >= n) return MTSGPU_EINVAL;
    *out = *params;
    out->flags |= MTSGPU_FLAG_TILE_SHARD;
    out->row_block = 8;
    out->row_stride = (uint32_t)n;
    out->row_phase = (uint32_t)k;
    return MTSGPU_OK;
}

// the pixels of the crop window a render with these params covers: the
// kernels' item -> pixel rule (dpath.h pixel_of) counted on the host
uint64_t mtsgpu_render_pixels(const mtsgpu_render_params *P) {
    if (!P || P->width == 0 || P->height == 0) return 0;
    const uint64_t stride = P->row_stride ? P->row_stride : 1, phase = P->row_phase % stride;
    const uint64_t tx = (P->width + 7) / 8, ty = (P->height + 7) / 8;
    uint64_t n = 0;
    if (P->flags & MTSGPU_FLAG_TILE_SHARD) {
        for (uint64_t t = phase; t < tx * ty; t += stride) {
            const uint64_t x0 = (t % tx) * 8, y0 = (t / tx) * 8;
            n += std::min<uint64_t>(8, P->width - x0) * std::min<uint64_t>(8, P->height - y0);
        }
        return n;
    }
    const uint64_t rb = P->row_block ? P->row_block : 1;
    for (uint64_t y = 0; y < P->height; ++y)
        if ((y / rb) % stride == phase) n += P->width;
    return n;
}

int mtsgpu_group_create(const int *devices, int n, mtsgpu_group **out) {
    if (!out) return MTSGPU_EINVAL;
    *out = nullptr;
    if (!devices || n <= 0) { g_group_create_error = "a device group needs at least one device"; return MTSGPU_EINVAL; }
    mtsgpu_group *g = new mtsgpu_group();
    g->m.resize((size_t)n);
    for (int k = 0; k < n; ++k) {
        Member &M = g->m[(size_t)k];
        int rc = mtsgpu_create(devices[k], &M.ctx);
        if (rc != MTSGPU_OK) {
            g_group_create_error = std::string("device ") + std::to_string(devices[k]) + ": " + mtsgpu_last_error(nullptr);
            mtsgpu_group_destroy(g);
            return rc;
        }
        M.device = devices[k] < 0 ? 0 : devices[k];
        if (devices[k] < 0) (void)hipGetDevice(&M.device);
        (void)hipDeviceGetAttribute(&M.num_cus, hipDeviceAttributeMultiprocessorCount, M.device);
    }
    // the merge runs on member 0's device and reads the other members' films over xGMI
    const int d0 = g->m[0].device;
    hipError_t e = hipSetDevice(d0);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking);
    for (int k = 1; k < n && e == hipSuccess; ++k) {
        const int dk = g->m[(size_t)k].device;
        if (dk == d0) continue;
        int can = 0;
        (void)hipDeviceCanAccessPeer(&can, d0, dk);
        if (!can) continue;   // hipMemcpyPeerAsync stages through the host then
        hipError_t pe = hipDeviceEnablePeerAccess(dk, 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) e = pe;
        (void)hipGetLastError();
    }
    if (e != hipSuccess) {
        g_group_create_error = std::string("device group init: ") + hipGetErrorString(e);
        mtsgpu_group_destroy(g);
        return MTSGPU_EHIP;
    }
    *out = g;
    return MTSGPU_OK;
}

int mtsgpu_group_size(const mtsgpu_group *g) { return g ? (int)g->m.size() : 0; }

mtsgpu_ctx *mtsgpu_group_member(mtsgpu_group *g, int k) {
    return (g && k >= 0 && k < (int)g->m.size()) ? g->m[(size_t)k].ctx : nullptr;
}

int mtsgpu_group_upload_scene(mtsgpu_group *g, const mtsgpu_scene_desc *scene) {
    if (!g || !scene) return MTSGPU_EINVAL;
    g->have_scene = false;
    const int bad = for_members(g, [&](Member &M, int) {
        M.rc = mtsgpu_upload_scene(M.ctx, scene);
        if (M.rc != MTSGPU_OK) M.err = mtsgpu_last_error(M.ctx);
    });
    if (bad >= 0) return gfail(g, g->m[(size_t)bad].rc, g->m[(size_t)bad].err);
    g->film_w = scene->sensor.film_width;
    g->film_h = scene->sensor.film_height;
    g->have_scene = true;
    return MTSGPU_OK;
}

int mtsgpu_group_render_device(mtsgpu_group *g, const mtsgpu_render_params *params, float *film_device,
                               mtsgpu_stats *stats) {
    if (!g || !params || !film_device) return MTSGPU_EINVAL;
    if (!g->have_scene) return gfail(g, MTSGPU_ESTATE, "render before upload_scene");
    if (params->row_stride > 1) return gfail(g, MTSGPU_EINVAL, "a device group shards the rows itself: row_stride must be 0 or 1");
    const int border = mtsgpu_film_border(params->rfilter, params->rfilter_param);
    if (border < 0) return gfail(g, MTSGPU_EINVAL, "invalid reconstruction filter");
    const size_t floats = (size_t)(g->film_w + 2 * border) * (g->film_h + 2 * border) * 5;
    const size_t bytes = floats * sizeof(float);
    const bool replay = params->sampler == MTSGPU_SAMPLER_SFMT_REPLAY || params->sampler == MTSGPU_SAMPLER_SFMT_BLOCKS;
    const int n = replay ? 1 : (int)g->m.size();
    for (auto &M : g->m) { M.rc = MTSGPU_OK; M.err.clear(); M.stats = mtsgpu_stats{}; }

    // member 0 renders straight into the caller's buffer; the others into their own HBM films
    std::vector<std::thread> th;
    for (int k = 0; k < n; ++k)
        th.emplace_back([&, k] {
            Member &M = g->m[(size_t)k];
            hipError_t e = hipSetDevice(M.device);
            if (e == hipSuccess && k > 0) e = ensure(M.film, M.film_bytes, bytes);
            if (e != hipSuccess) { M.rc = MTSGPU_EHIP; M.err = std::string("member film: ") + hipGetErrorString(e); return; }
            mtsgpu_render_params P;
            mtsgpu_group_member_params(params, n, k, &P);
            M.rc = mtsgpu_render_device(M.ctx, &P, k == 0 ? film_device : M.film, nullptr, &M.stats);
            if (M.rc != MTSGPU_OK) M.err = mtsgpu_last_error(M.ctx);
        });
    for (auto &t : th) t.join();
    for (int k = 0; k < n; ++k)
        if (g->m[(size_t)k].rc != MTSGPU_OK)
            return gfail(g, g->m[(size_t)k].rc, "member " + std::to_string(k) + ": " + g->m[(size_t)k].err);

    // merge on member 0's device in member order
    const Member &M0 = g->m[0];
    hipError_t e = hipSetDevice(M0.device);
    if (e != hipSuccess) return ghip(g, e, "hipSetDevice");
    if (n > 1 && (e = ensure(g->stage, g->stage_bytes, bytes)) != hipSuccess) return ghip(g, e, "merge buffer");
    for (int k = 1; k < n; ++k) {
        const Member &M = g->m[(size_t)k];
        e = M.device == M0.device ? hipMemcpyAsync(g->stage, M.film, bytes, hipMemcpyDeviceToDevice, g->stream)
                                  : hipMemcpyPeerAsync(g->stage, M0.device, M.film, M.device, bytes, g->stream);
        if (e != hipSuccess) return ghip(g, e, "peer copy");
        if ((e = mtsg_launch_film_accumulate(film_device, g->stage, floats, M0.num_cus, g->stream)) != hipSuccess)
            return ghip(g, e, "film merge");
    }
    if ((e = hipStreamSynchronize(g->stream)) != hipSuccess) return ghip(g, e, "film merge");
    if (stats) {
        *stats = mtsgpu_stats{};
        for (int k = 0; k < n; ++k) add_stats(*stats, g->m[(size_t)k].stats);
    }
    return MTSGPU_OK;
}

int mtsgpu_group_render(mtsgpu_group *g, const mtsgpu_render_params *params, float *film, mtsgpu_stats *stats) {
    if (!g || !params || !film) return MTSGPU_EINVAL;
    if (!g->have_scene) return gfail(g, MTSGPU_ESTATE, "render before upload_scene");
    const int border = mtsgpu_film_border(params->rfilter, params->rfilter_param);
    if (border < 0) return gfail(g, MTSGPU_EINVAL, "invalid reconstruction filter");
    const size_t bytes = (size_t)(g->film_w + 2 * border) * (g->film_h + 2 * border) * 5 * sizeof(float);
    Member &M0 = g->m[0];
    hipError_t e = hipSetDevice(M0.device);
    if (e == hipSuccess) e = ensure(M0.film, M0.film_bytes, bytes);
    if (e != hipSuccess) return ghip(g, e, "film");
    int rc = mtsgpu_group_render_device(g, params, M0.film, stats);
    if (rc != MTSGPU_OK) return rc;
    (void)hipSetDevice(M0.device);
    if ((e = hipMemcpy(film, M0.film, bytes, hipMemcpyDeviceToHost)) != hipSuccess) return ghip(g, e, "film download");
    return MTSGPU_OK;
}

const char *mtsgpu_group_last_error(mtsgpu_group *g) { return g ? g->err.c_str() : g_group_create_error.c_str(); }

void mtsgpu_group_destroy(mtsgpu_group *g) {
    if (!g) return;
    for (auto &M : g->m) {
        if (M.film) { (void)hipSetDevice(M.device); (void)hipFree(M.film); }
        if (M.ctx) mtsgpu_destroy(M.ctx);
    }
    if (!g->m.empty()) (void)hipSetDevice(g->m[0].device);
    if (g->stage) (void)hipFree(g->stage);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

}  // extern "C"
