// wf_kernel.hip -- the wavefront engine's trace kernel and host-side
// launchers (the engine: wf_impl.h; its shade kernels are compiled per scene
// feature set in wf_shade_f.hip, one object per set, so they build in parallel)
#include "wf_impl.h"

#include <cstdlib>

int mtsg_path_features(const MtsgLaunch &L);   // path_kernel.hip
#define MTSG_WF_PICK_DECL(N) WfShadeFn mtsg_wf_pick_##N(int wk, bool instr, bool ggx);
MTSG_WF_PICK_DECL(0) MTSG_WF_PICK_DECL(1) MTSG_WF_PICK_DECL(2) MTSG_WF_PICK_DECL(3) MTSG_WF_PICK_DECL(6)
MTSG_WF_PICK_DECL(7)
#undef MTSG_WF_PICK_DECL

// the per-block partial counters of a chunk -> MtsgLaunch::counters
__global__ void wf_flush(const unsigned long long *part, uint32_t blocks, unsigned long long *counters) {
    const uint32_t k = threadIdx.x & 15u;   // 256 threads: counter k, blocks b = threadIdx / 16 (mod 16)
    unsigned long long t = 0;
    for (uint32_t b = threadIdx.x >> 4; b < blocks; b += 16) t += part[(size_t)b * 16 + k];
    if (t) atomicAdd(counters + k, t);
}

// ---------------------------------------------------------------------------
// host-side launchers (capi.cpp)
// ---------------------------------------------------------------------------
size_t mtsg_wf_shade_lds_bytes(const MtsgLaunch &L) { return ((size_t)L.lds_dims * L.nibbles * 16 + 16 * 16) * 4; }
// The kd trace kernel: its mailbox in LDS at 8 waves/SIMD, the stack in scratch
// (round 5, profiles/r05_ab_kd_mailbox_lds.log: C4 65.8 -> 76.9, C3 370 -> 398
// Msamples/s; with the first 3 stack entries in LDS as well 75.1 / 371; the
// scratch-only kernel capped at 4 waves through its LDS 54.0 / 278).  Round 4's
// mailbox plus 8 entries at 4 waves: C4 62.2 -> 65.0, C3 356.8 -> 330.2
// (profiles/r04_ab_kd_lds.log)
size_t mtsg_wf_trace_lds_bytes(const MtsgLaunch &L) {
    if (L.kd_nodes) return (size_t)wf_kd_lds_lane_bytes(MTSG_WF_KD_LDSK, MTSG_WF_KD_MBL) * BLOCK + 16;
    const bool scan = L.scene_lds && L.scan;
    const size_t scene = (L.scene_lds && !L.scan) ? ((size_t)L.num_nodes * 16 + (size_t)L.scene.num_prims * 12) : 0;
    const size_t K = std::min<size_t>(L.stack_depth, MTSG_WF_LDS_STACK);
    const size_t stack = scan ? 0 : (K * 3 * BLOCK + 1) / 2;
    return (scene + stack) * 4 + 16;
}

static WfShadeFn wf_shade_pick(const MtsgLaunch &L, int wk, bool instr, bool ggx) {
    switch (mtsg_path_features(L)) {   // = MTSG_FEAT_ENV | EXT | ANA bits
        case 0: return mtsg_wf_pick_0(wk, instr, ggx);
        case 1: return mtsg_wf_pick_1(wk, instr, ggx);
        case 2: return mtsg_wf_pick_2(wk, instr, ggx);
        case 3: return mtsg_wf_pick_3(wk, instr, ggx);
        case 6: return mtsg_wf_pick_6(wk, instr, ggx);
        default: return mtsg_wf_pick_7(wk, instr, ggx);
    }
}

typedef void (*WfTraceFn)(MtsgLaunch, MtsgWave, unsigned long long *);
static WfTraceFn wf_trace_pick(const MtsgLaunch &L, bool stats) {
    const bool ana = L.ana != 0;
    constexpr int KDK = MTSG_WF_KD_LDSK;
    constexpr bool KDMB = MTSG_WF_KD_MBL;
    if (L.kd_nodes) return stats ? wf_trace<true, false, false, true, KDK, KDMB> : wf_trace<false, false, false, true, KDK, KDMB>;
    if (stats) {
        if (L.scene_lds) return ana ? wf_trace<true, true, true, false> : wf_trace<true, true, false, false>;
        return ana ? wf_trace<true, false, true, false> : wf_trace<true, false, false, false>;
    }
    if (L.scene_lds) return ana ? wf_trace<false, true, true, false> : wf_trace<false, true, false, false>;
    return ana ? wf_trace<false, false, true, false> : wf_trace<false, false, false, false>;
}

hipError_t mtsg_launch_wf_shade(const MtsgLaunch &L, const MtsgWave &W, unsigned long long *part, int grid, int wk,
                                bool ggx, bool instr, hipStream_t s) {
    WfShadeFn f = wf_shade_pick(L, wk, instr, ggx);
    if (!f) return hipErrorInvalidValue;
    hipLaunchKernelGGL(f, dim3(grid), dim3(BLOCK), mtsg_wf_shade_lds_bytes(L), s, L, W, part, (uint32_t)wk);
    return hipGetLastError();
}

hipError_t mtsg_launch_wf_trace(const MtsgLaunch &L, const MtsgWave &W, unsigned long long *part, int grid,
                                bool stats, hipStream_t s) {
    hipLaunchKernelGGL(wf_trace_pick(L, stats), dim3(grid), dim3(BLOCK), mtsg_wf_trace_lds_bytes(L), s, L, W, part);
    return hipGetLastError();
}

hipError_t mtsg_launch_wf_flush(const unsigned long long *part, uint32_t blocks, unsigned long long *counters,
                                hipStream_t s) {
    hipLaunchKernelGGL(wf_flush, dim3(1), dim3(256), 0, s, part, blocks, counters);
    return hipGetLastError();
}

// resident blocks per CU of a shade kind's kernel and of the trace kernel (their grids)
int mtsg_wf_occupancy(const MtsgLaunch &L, int wk, bool ggx, int *shadeBpc, int *traceBpc) {
    *shadeBpc = *traceBpc = 0;
    int r = 0;
    if (wk >= 0) {
        WfShadeFn f = wf_shade_pick(L, wk, false, ggx);
        if (!f) return (int)hipErrorInvalidValue;
        r = (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(shadeBpc, f, BLOCK, mtsg_wf_shade_lds_bytes(L));
        if (r) return r;
    }
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(traceBpc, wf_trace_pick(L, false), BLOCK,
                                                             mtsg_wf_trace_lds_bytes(L));
}
