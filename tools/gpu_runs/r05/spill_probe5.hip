#include "../../mitsuba0.6_amd/csrc/dmega.h"
size_t mtsg_path_lds_bytes(const MtsgLaunch &L) { return 0; }
template __global__ void path_kernel<false, true, 8, 5>(MtsgLaunch);
template __global__ void path_kernel<false, false, 80 | 256, 5>(MtsgLaunch);
template __global__ void path_kernel<false, false, 49 | 256, 5>(MtsgLaunch);
