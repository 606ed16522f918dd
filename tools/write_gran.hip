// write_gran.hip -- HBM write granularity of scattered 16 B stores (VERDICT r05 item 7:
// C2 writes 34.6 B per sample for a 16 B own-pixel splat record).  Four store
// patterns of the same 16 B records, each profiled with rocprofv3 --pmc WRITE_SIZE
// (tools/gpu_runs/r06/call7.sh): bytes the memory system writes per byte stored.
//   dense    -- lane g stores record g: every 128 B line written whole by one wave
//   stride2  -- record 2g: every other 16 B of each line
//   stride8  -- record 8g: one 16 B record per 128 B line
//   splat    -- the path kernel's pattern: record (j * P + pix) with each lane at its own
//               sample index j (lanes of a wave drift apart as their paths end at
//               different bounces), pix = the lane's pixel
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void store16(float4 *out, size_t n, unsigned P) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const float4 v = make_float4((float)g, 1.0f, 2.0f, 3.0f);
    if (MODE == 0) out[g] = v;
    if (MODE == 1) out[2 * g] = v;
    if (MODE == 2) out[8 * g] = v;
    if (MODE == 3) {
        const unsigned lane = threadIdx.x & 63, wave = (unsigned)(g >> 6);
        const unsigned j = (lane * 2654435761u >> 27) + (wave & 7);   // per-lane sample index, spread 0..38
        out[(size_t)j * P + (wave % (P / 64)) * 64 + lane] = v;
    }
}

int main() {
    const size_t n = (size_t)1 << 26;   // 64 Mi records of 16 B = 1 GiB stored per launch
    const unsigned P = 921600;          // pixels of a 1280x720 frame
    float4 *out;
    if (hipMalloc(&out, 8 * n * sizeof(float4))) return 2;
    const dim3 grid((unsigned)(n / 256)), block(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(store16<0>, grid, block, 0, 0, out, n, P);
        hipLaunchKernelGGL(store16<1>, grid, block, 0, 0, out, n, P);
        hipLaunchKernelGGL(store16<2>, grid, block, 0, 0, out, n, P);
        hipLaunchKernelGGL(store16<3>, grid, block, 0, 0, out, n, P);
    }
    if (hipDeviceSynchronize()) return 2;
    std::printf("{\"records\": %zu, \"bytes_stored_per_launch\": %zu}\n", n, n * 16);
    return hipFree(out) ? 2 : 0;
}
