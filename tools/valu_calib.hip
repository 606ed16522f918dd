// valu_calib.hip -- calibration of the VALU roofline bench.py reports.
//
// A pure-VALU kernel: every lane runs 8 independent v_fma_f32 chains (no memory
// traffic inside the loop, no dependency stalls at >= 2 waves), launched at
// 1, 2, 4 and 8 waves per SIMD (grid = CUs x waves blocks of 4 waves, one per
// SIMD).  Per launch it prints the wave-instruction rate against the SIMD-cycles
// available (1024 SIMDs x the clock): the cycles one SIMD spends per wave64 VALU
// instruction at saturation.  MI355X_MICROARCH.md gives 2 (SIMD-32, two passes);
// one wave alone issues one every 4 cycles.  Under rocprofv3 with the SQ counters
// (tools/prof_valu_calib.sh) the same launches give SQ_INSTS_VALU and
// SQ_ACTIVE_INST_VALU against GRBM_GUI_ACTIVE, which is how bench.py's valu
// roofline is read off the path kernel's own SQ pass.
//
// usage: valu_calib [iterations]   (prints one JSON line per waves/SIMD setting)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr int CHAINS = 8;

// W only names the instantiation (one kernel name per occupancy in the profile)
template <int W>
__global__ __launch_bounds__(256) void valu_calib(float *out, int iters, float x, float y) {
    float a[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) a[c] = (float)(threadIdx.x + c);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) a[c] = __builtin_fmaf(a[c], x, y);
        }
    }
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += a[c];
    if (s == 12345.678f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;   // keeps the chains live
}

// the packed forms (two f32 lanes per lane and instruction): v_pk_fma_f32 (OP 0)
// and v_pk_mul_f32 + v_pk_add_f32 pairs (OP 1, what -ffp-contract=off code
// would pack); 4 independent pairs of chains = 8 f32 chains per lane as above
typedef float f2 __attribute__((ext_vector_type(2)));
template <int W, int OP>
__global__ __launch_bounds__(256) void valu_calib_pk(float *out, int iters, float x, float y) {
    f2 a[CHAINS / 2];
#pragma unroll
    for (int c = 0; c < CHAINS / 2; ++c) a[c] = f2{(float)(threadIdx.x + 2 * c), (float)(threadIdx.x + 2 * c + 1)};
    const f2 xv = {x, x}, yv = {y, y};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int c = 0; c < CHAINS / 2; ++c) {
                if (OP == 0) a[c] = __builtin_elementwise_fma(a[c], xv, yv);
                else a[c] = a[c] * xv + yv;
            }
        }
    }
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < CHAINS / 2; ++c) s += a[c].x + a[c].y;
    if (s == 12345.678f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int W, int OP>
static void run_pk(int cus, int iters, float *out) {
    const int grid = cus * W;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((valu_calib_pk<W, OP>), dim3(grid), dim3(256), 0, 0, out, iters / 8, 0.999f, 0.001f);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((valu_calib_pk<W, OP>), dim3(grid), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    // wave instructions: OP 0 one v_pk_fma per pair and step, OP 1 a v_pk_mul and a v_pk_add
    const double waveInsts = (double)grid * 4 * iters * 4 * (CHAINS / 2) * (OP == 0 ? 1 : 2);
    const double simds = (double)cus * 4;
    std::printf("{\"kernel\": \"valu_calib_pk<%d, %d>\", \"op\": \"%s\", \"waves_per_simd\": %d, \"grid\": %d, "
                "\"iters\": %d, \"kernel_ms\": %.4f, \"wave_valu_insts\": %.0f, \"wave_insts_per_simd_per_ns\": %.5f, "
                "\"f32_lane_ops_per_simd_per_ns\": %.3f}\n",
                W, OP, OP == 0 ? "v_pk_fma_f32" : "v_pk_mul_f32+v_pk_add_f32", W, grid, iters, ms, waveInsts,
                waveInsts / simds / (ms * 1e6), 2 * 64 * waveInsts / simds / (ms * 1e6));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

template <int W>
static void run(int cus, int iters, float *out) {
    const int grid = cus * W;   // 4 waves per block -> W waves per SIMD when all are resident
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(valu_calib<W>, dim3(grid), dim3(256), 0, 0, out, iters / 8, 0.999f, 0.001f);   // warm-up
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(valu_calib<W>, dim3(grid), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double waveInsts = (double)grid * 4 * iters * 4 * CHAINS;   // v_fma_f32 per wave
    const double simds = (double)cus * 4;
    // nominal 2.4 GHz: the rocprofv3 pass measures the clock (GRBM_GUI_ACTIVE / 8 / kernel time)
    const double cyclesPerInst = simds * 2.4e9 * (ms / 1e3) / waveInsts;
    std::printf("{\"kernel\": \"valu_calib<%d>\", \"waves_per_simd\": %d, \"grid\": %d, \"iters\": %d, "
                "\"kernel_ms\": %.4f, \"wave_valu_insts\": %.0f, \"wave_insts_per_simd_per_ns\": %.5f, "
                "\"simd_cycles_per_wave_inst_at_2p4GHz\": %.4f}\n",
                W, W, grid, iters, ms, waveInsts, waveInsts / simds / (ms * 1e6), cyclesPerInst);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 200000;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    float *out = nullptr;
    CHECK(hipMalloc(&out, (size_t)p.multiProcessorCount * 8 * 256 * sizeof(float)));
    run<1>(p.multiProcessorCount, iters, out);
    run<2>(p.multiProcessorCount, iters, out);
    run<4>(p.multiProcessorCount, iters, out);
    run<8>(p.multiProcessorCount, iters, out);
    run_pk<4, 0>(p.multiProcessorCount, iters, out);
    run_pk<8, 0>(p.multiProcessorCount, iters, out);
    run_pk<4, 1>(p.multiProcessorCount, iters, out);
    run_pk<8, 1>(p.multiProcessorCount, iters, out);
    CHECK(hipFree(out));
    return 0;
}
