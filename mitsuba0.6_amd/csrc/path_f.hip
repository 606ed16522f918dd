// path_f.hip -- the megakernel variants (dmega.h) of one scene feature set
// PATH_FEAT (MTSG_FEAT_ENV | EXT | ANA bits), built once per set by the
// Makefile (-DPATH_FEAT=n -> path_f<n>.o), so the sets compile in parallel.
//
// Per set: the generic kernel (every BSDF, virtual-dispatch order of
// path.cpp:171-211), for all-diffuse small scenes (PATH_FEAT 0) the DIFF
// kernel, and the 7 BSDF-set specialisations of large scenes (dbsdf.h BSet):
// bits = {every rough BSDF is GGX, no roughdielectric, no roughconductor};
// with an environment emitter also the 7 sets of envmap-only scenes (bit 3,
// MTSG_FEAT_NOREFN: no area light, no constant emitter).
// The set kernels are compiled without strictNormals (MTSG_FEAT_NOSTRICT).
#include "dmega.h"

#define PF_NAME2(a, N) a##N
#define PF_NAME(a, N) PF_NAME2(a, N)

namespace {
constexpr int spec_feat(int bits) {
    return PATH_FEAT | (int)MTSG_FEAT_NOSTRICT | ((bits & 1) ? (int)MTSG_FEAT_GGX : 0) |
           ((bits & 2) ? (int)MTSG_FEAT_NORD : 0) | ((bits & 4) ? (int)MTSG_FEAT_NORC : 0) |
           ((bits & 8) ? (int)MTSG_FEAT_NOREFN : 0);
}

// variants: small scenes (BVH in LDS) run 3 waves/SIMD with 32 Sobol dims in
// LDS (all-diffuse ones 4: no calls in their bounce loop); large scenes run 4
// waves/SIMD (128 VGPRs) when the traversal stacks fit 4 blocks per CU, else 3
// (capi.cpp picks L.waves and L.lds_dims)
template <int FEAT>
void launch_v(const MtsgLaunch &L, int grid, bool instr, hipStream_t stream) {
    if constexpr ((FEAT & (MTSG_FEAT_GGX | MTSG_FEAT_NORD | MTSG_FEAT_NORC)) != 0) {   // large scenes only
        if (L.waves == 4) launch_path_w<false, FEAT, 4>(L, grid, instr, stream);
        else launch_path_w<false, FEAT, MTSG_WAVES_PER_EU>(L, grid, instr, stream);
    } else {
        if (L.scene_lds) {
            if constexpr ((FEAT & MTSG_FEAT_DIFF) != 0) {
                if (L.waves == 4) { launch_path_w<true, FEAT, 4>(L, grid, instr, stream); return; }
            }
            launch_path_w<true, FEAT, MTSG_WAVES_PER_EU>(L, grid, instr, stream);
        }
        else if (L.waves == 4) launch_path_w<false, FEAT, 4>(L, grid, instr, stream);
        else launch_path_w<false, FEAT, MTSG_WAVES_PER_EU>(L, grid, instr, stream);
    }
}
template <int FEAT>
int occupancy_v(const MtsgLaunch &L, int *bpc) {
    if constexpr ((FEAT & (MTSG_FEAT_GGX | MTSG_FEAT_NORD | MTSG_FEAT_NORC)) != 0) {
        if (L.waves == 4) return occupancy_w<false, FEAT, 4>(L, bpc);
        return occupancy_w<false, FEAT, MTSG_WAVES_PER_EU>(L, bpc);
    } else {
        if (L.scene_lds) {
            if constexpr ((FEAT & MTSG_FEAT_DIFF) != 0) {
                if (L.waves == 4) return occupancy_w<true, FEAT, 4>(L, bpc);
            }
            return occupancy_w<true, FEAT, MTSG_WAVES_PER_EU>(L, bpc);
        }
        if (L.waves == 4) return occupancy_w<false, FEAT, 4>(L, bpc);
        return occupancy_w<false, FEAT, MTSG_WAVES_PER_EU>(L, bpc);
    }
}
}  // namespace

hipError_t PF_NAME(mtsg_launch_path_f, PATH_FEAT)(const MtsgLaunch &L, int grid, bool instr, hipStream_t s, int bits) {
    switch (bits) {
        case 1: launch_v<spec_feat(1)>(L, grid, instr, s); break;
        case 2: launch_v<spec_feat(2)>(L, grid, instr, s); break;
        case 3: launch_v<spec_feat(3)>(L, grid, instr, s); break;
        case 4: launch_v<spec_feat(4)>(L, grid, instr, s); break;
        case 5: launch_v<spec_feat(5)>(L, grid, instr, s); break;
        case 6: launch_v<spec_feat(6)>(L, grid, instr, s); break;
        case 7: launch_v<spec_feat(7)>(L, grid, instr, s); break;
#if PATH_FEAT & 1   // envmap-only scenes (MTSG_FEAT_NOREFN): feature sets with an environment emitter
        case 9: launch_v<spec_feat(9)>(L, grid, instr, s); break;
        case 10: launch_v<spec_feat(10)>(L, grid, instr, s); break;
        case 11: launch_v<spec_feat(11)>(L, grid, instr, s); break;
        case 12: launch_v<spec_feat(12)>(L, grid, instr, s); break;
        case 13: launch_v<spec_feat(13)>(L, grid, instr, s); break;
        case 14: launch_v<spec_feat(14)>(L, grid, instr, s); break;
        case 15: launch_v<spec_feat(15)>(L, grid, instr, s); break;
#endif
        default:
#if PATH_FEAT == 0
            if (L.all_diffuse) { launch_v<MTSG_FEAT_DIFF>(L, grid, instr, s); break; }
#endif
            launch_v<PATH_FEAT>(L, grid, instr, s);
            break;
    }
    return hipGetLastError();
}

int PF_NAME(mtsg_path_occupancy_f, PATH_FEAT)(const MtsgLaunch &L, int bits, int *bpc) {
    switch (bits) {
        case 1: return occupancy_v<spec_feat(1)>(L, bpc);
        case 2: return occupancy_v<spec_feat(2)>(L, bpc);
        case 3: return occupancy_v<spec_feat(3)>(L, bpc);
        case 4: return occupancy_v<spec_feat(4)>(L, bpc);
        case 5: return occupancy_v<spec_feat(5)>(L, bpc);
        case 6: return occupancy_v<spec_feat(6)>(L, bpc);
        case 7: return occupancy_v<spec_feat(7)>(L, bpc);
#if PATH_FEAT & 1
        case 9: return occupancy_v<spec_feat(9)>(L, bpc);
        case 10: return occupancy_v<spec_feat(10)>(L, bpc);
        case 11: return occupancy_v<spec_feat(11)>(L, bpc);
        case 12: return occupancy_v<spec_feat(12)>(L, bpc);
        case 13: return occupancy_v<spec_feat(13)>(L, bpc);
        case 14: return occupancy_v<spec_feat(14)>(L, bpc);
        case 15: return occupancy_v<spec_feat(15)>(L, bpc);
#endif
        default:
#if PATH_FEAT == 0
            if (L.all_diffuse) return occupancy_v<MTSG_FEAT_DIFF>(L, bpc);
#endif
            return occupancy_v<PATH_FEAT>(L, bpc);
    }
}
