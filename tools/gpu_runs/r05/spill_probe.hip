// Compile-only probe (tools/gpu_runs/r05/spills.sh): the four benchmark megakernels
// (C2 DIFF+LDS, C3 set 49, C4 set 80, C5 set 115), for register/spill counts
// without building every variant.
#include "../../mitsuba0.6_amd/csrc/dmega.h"
size_t mtsg_path_lds_bytes(const MtsgLaunch &L) { return 0; }
template __global__ void path_kernel<false, true, 8, 4>(MtsgLaunch);
template __global__ void path_kernel<false, false, 49 | 256, 4>(MtsgLaunch);
template __global__ void path_kernel<false, false, 80 | 256, 4>(MtsgLaunch);
template __global__ void path_kernel<false, false, 115 | 256, 4>(MtsgLaunch);
template __global__ void path_kernel<false, false, 115 | 256 | 512, 4>(MtsgLaunch);
template __global__ void path_kernel<false, false, 49 | 256 | 512, 4>(MtsgLaunch);
