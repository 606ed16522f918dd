// probe_kernel.hip -- diagnostics: the path kernels' transcendentals, element-wise.
//
// mtsgpu_debug_libm runs the device's d_* routines (dmath.h: glibc_f32.h's
// restatement of glibc's float libm, double exp/log for math::fastexp/fastlog)
// over an input array, or over a range of float bit patterns, so that
// tests/test_gpu_libm.py can compare them with the host's libm.so.6 bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dmath.h"

namespace {

__global__ void libm_probe(int fn, const float *a, const float *b, float *out, size_t n, uint32_t first) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float x = a ? a[i] : glf_asfloat(first + (uint32_t)i);
        const float y = b ? b[i] : 0.0f;
        float r = 0.0f, s, c;
        switch (fn) {
        case 0: d_sincos(x, &s, &c); r = s; break;
        case 1: d_sincos(x, &s, &c); r = c; break;
        case 2: r = d_expf(x); break;
        case 3: r = d_acos(x); break;
        case 4: r = d_atan(x); break;
        case 5: r = d_tan(x); break;
        case 6: r = d_atan2(x, y); break;
        case 7: r = d_powf(x, y); break;
        case 8: r = d_fastexp(x); break;
        default: r = d_fastlog(x); break;
        }
        out[i] = r;
    }
}

}  // namespace

hipError_t mtsg_launch_libm_probe(int fn, const float *a, const float *b, float *out, size_t n, uint32_t first,
                                  hipStream_t s) {
    const size_t blocks = (n + 255) / 256;
    const unsigned grid = (unsigned)(blocks < 65536 ? blocks : 65536);
    hipLaunchKernelGGL(libm_probe, dim3(grid), dim3(256), 0, s, fn, a, b, out, n, first);
    return hipGetLastError();
}
