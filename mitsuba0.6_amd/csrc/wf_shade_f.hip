// wf_shade_f.hip -- the wavefront engine's shade kernels (wf_impl.h) for one
// scene feature set WF_FEAT (MTSG_FEAT_ENV | EXT | ANA bits), built once per
// set by the Makefile (-DWF_FEAT=n -> wf_shade_f<n>.o)
#include "wf_impl.h"

#define MTSG_WF_PICK_NAME2(N) mtsg_wf_pick_##N
#define MTSG_WF_PICK_NAME(N) MTSG_WF_PICK_NAME2(N)
WfShadeFn MTSG_WF_PICK_NAME(WF_FEAT)(int wk, bool instr, bool ggx) { return wf_shade_pick_f<WF_FEAT>(wk, instr, ggx); }
