// film_kernel.hip -- hdrfilm develop on the device.
//
// HDRFilm::develop (src/films/hdrfilm.cpp:481-495) converts the film's
// SpectrumAlphaWeight storage to the output pixel/component format with
// Bitmap::convert -> FormatConverterImpl (src/libcore/fmtconv.cpp:955-1030):
//   invWeight = weight != 0 ? 1/weight : weight
//   rgb   : (spec * invWeight)                      (toLinearRGB = identity in RGB mode)
//   lum   : spec.getLuminance() * invWeight         (spectrum.h:725)
//   xyz   : (spec * invWeight * multiplier).toXYZ() (spectrum.cpp:229-234)
//   alpha : alpha * invWeight
// then convertScalar<Dest> (fmtconv.cpp:1137-1160): value * multiplier, cast
// to half (round to nearest even), float, or uint32 (round + clamp).
// The film storage is the crop ImageBlock without border; Film::put of the
// rendered block (border b) clips the border away (imageblock.h put()), so the
// develop reads the interior [b, b+H) x [b, b+W) of the rendered film.
//
// One thread per output pixel, grid-stride; 20 B read + C * (2|4) B written
// per pixel -- an HBM-bound streaming kernel.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/mtsgpu.h"

namespace {

constexpr int DEV_BLOCK = 256;

__device__ __forceinline__ float smax_(float a, float b) { return (a < b) ? b : a; }   // std::max
__device__ __forceinline__ float smin_(float a, float b) { return (b < a) ? b : a; }   // std::min

template <int COMP> struct CompT;
template <> struct CompT<MTSGPU_COMP_FLOAT16> { typedef uint16_t T; };
template <> struct CompT<MTSGPU_COMP_FLOAT32> { typedef float T; };
template <> struct CompT<MTSGPU_COMP_UINT32> { typedef uint32_t T; };

template <int COMP>
__device__ __forceinline__ typename CompT<COMP>::T conv(float v, float mult) {
    v = v * mult;
    if constexpr (COMP == MTSGPU_COMP_FLOAT16) {
        return __half_as_ushort(__float2half_rn(v));
    } else if constexpr (COMP == MTSGPU_COMP_FLOAT32) {
        return v;
    } else {
        // min(max_u32, max(0, v * max_u32 + 0.5f)) in float, then the x86-64
        // float -> uint32 cast (cvttss2si to 64 bits, low word)
        const float m = 4294967295.0f;
        float r = smin_(m, smax_(0.0f, v * m + 0.5f));
        return (uint32_t)(uint64_t)(int64_t)r;
    }
}

template <int PIX, int COMP>
__global__ __launch_bounds__(DEV_BLOCK) void develop_kernel(const float *__restrict__ film, uint32_t full_w,
                                                            uint32_t border, uint32_t w, uint32_t h, float mult,
                                                            typename CompT<COMP>::T *__restrict__ out) {
    constexpr int C = (PIX == MTSGPU_PIX_LUMINANCE) ? 1 : (PIX == MTSGPU_PIX_LUMINANCE_ALPHA) ? 2
                    : (PIX == MTSGPU_PIX_RGB || PIX == MTSGPU_PIX_XYZ) ? 3 : 4;
    const size_t n = (size_t)w * h;
    for (size_t i = (size_t)blockIdx.x * DEV_BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * DEV_BLOCK) {
        const uint32_t y = (uint32_t)(i / w), x = (uint32_t)(i - (size_t)y * w);
        const float *px = film + ((size_t)(y + border) * full_w + (x + border)) * 5;
        const float s0 = px[0], s1 = px[1], s2 = px[2], alpha = px[3], weight = px[4];
        const float inv = (weight != 0.0f) ? 1.0f / weight : weight;
        typename CompT<COMP>::T *o = out + i * C;
        if constexpr (PIX == MTSGPU_PIX_LUMINANCE || PIX == MTSGPU_PIX_LUMINANCE_ALPHA) {
            const float lum = s0 * 0.212671f + s1 * 0.715160f + s2 * 0.072169f;
            o[0] = conv<COMP>(lum * inv, mult);
            if constexpr (PIX == MTSGPU_PIX_LUMINANCE_ALPHA) o[1] = conv<COMP>(alpha * inv, 1.0f);
        } else if constexpr (PIX == MTSGPU_PIX_RGB || PIX == MTSGPU_PIX_RGBA) {
            o[0] = conv<COMP>(s0 * inv, mult);
            o[1] = conv<COMP>(s1 * inv, mult);
            o[2] = conv<COMP>(s2 * inv, mult);
            if constexpr (PIX == MTSGPU_PIX_RGBA) o[3] = conv<COMP>(alpha * inv, 1.0f);
        } else {
            const float r = s0 * inv * mult, g = s1 * inv * mult, b = s2 * inv * mult;
            o[0] = conv<COMP>(r * 0.412453f + g * 0.357580f + b * 0.180423f, 1.0f);
            o[1] = conv<COMP>(r * 0.212671f + g * 0.715160f + b * 0.072169f, 1.0f);
            o[2] = conv<COMP>(r * 0.019334f + g * 0.119193f + b * 0.950227f, 1.0f);
            if constexpr (PIX == MTSGPU_PIX_XYZA) o[3] = conv<COMP>(alpha * inv, 1.0f);
        }
    }
}

template <int PIX, int COMP>
hipError_t launch_t(const float *film, uint32_t full_w, uint32_t border, uint32_t w, uint32_t h, float mult, void *out,
                    int grid, hipStream_t s) {
    develop_kernel<PIX, COMP><<<grid, DEV_BLOCK, 0, s>>>(film, full_w, border, w, h, mult,
                                                        (typename CompT<COMP>::T *)out);
    return hipGetLastError();
}

template <int PIX>
hipError_t launch_p(int comp, const float *film, uint32_t full_w, uint32_t border, uint32_t w, uint32_t h, float mult,
                    void *out, int grid, hipStream_t s) {
    switch (comp) {
        case MTSGPU_COMP_FLOAT16: return launch_t<PIX, MTSGPU_COMP_FLOAT16>(film, full_w, border, w, h, mult, out, grid, s);
        case MTSGPU_COMP_FLOAT32: return launch_t<PIX, MTSGPU_COMP_FLOAT32>(film, full_w, border, w, h, mult, out, grid, s);
        case MTSGPU_COMP_UINT32: return launch_t<PIX, MTSGPU_COMP_UINT32>(film, full_w, border, w, h, mult, out, grid, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace

int mtsg_develop_channels(int pixel_format) {
    switch (pixel_format) {
        case MTSGPU_PIX_LUMINANCE: return 1;
        case MTSGPU_PIX_LUMINANCE_ALPHA: return 2;
        case MTSGPU_PIX_RGB: case MTSGPU_PIX_XYZ: return 3;
        case MTSGPU_PIX_RGBA: case MTSGPU_PIX_XYZA: return 4;
    }
    return 0;
}

hipError_t mtsg_launch_develop(const mtsgpu_develop_params &P, const float *film, void *out, int num_cus,
                               hipStream_t s) {
    const uint32_t b = P.border, w = P.film_width - 2 * b, h = P.film_height - 2 * b;
    const size_t n = (size_t)w * h;
    // enough waves to cover HBM latency: up to 16 blocks per CU, never more than the pixels need
    const size_t want = (n + DEV_BLOCK - 1) / DEV_BLOCK, cap = (size_t)std::max(num_cus, 1) * 16;
    const int grid = (int)std::max<size_t>(1, std::min(want, cap));
    const int c = P.component_format;
    switch (P.pixel_format) {
        case MTSGPU_PIX_LUMINANCE: return launch_p<MTSGPU_PIX_LUMINANCE>(c, film, P.film_width, b, w, h, P.multiplier, out, grid, s);
        case MTSGPU_PIX_LUMINANCE_ALPHA: return launch_p<MTSGPU_PIX_LUMINANCE_ALPHA>(c, film, P.film_width, b, w, h, P.multiplier, out, grid, s);
        case MTSGPU_PIX_RGB: return launch_p<MTSGPU_PIX_RGB>(c, film, P.film_width, b, w, h, P.multiplier, out, grid, s);
        case MTSGPU_PIX_RGBA: return launch_p<MTSGPU_PIX_RGBA>(c, film, P.film_width, b, w, h, P.multiplier, out, grid, s);
        case MTSGPU_PIX_XYZ: return launch_p<MTSGPU_PIX_XYZ>(c, film, P.film_width, b, w, h, P.multiplier, out, grid, s);
        case MTSGPU_PIX_XYZA: return launch_p<MTSGPU_PIX_XYZA>(c, film, P.film_width, b, w, h, P.multiplier, out, grid, s);
    }
    return hipErrorInvalidValue;
}

// Film merge of a device group (mtsgpu_group_render): dst += src over the
// (W+2b)(H+2b)x5 ImageBlock, the Film::put sum of the per-device blocks
// (renderproc.cpp:142-149).  Streaming float4 pass, HBM-bound: 3 x 4 B per float.
__global__ __launch_bounds__(256) void film_accumulate(float4 *__restrict__ dst, const float4 *__restrict__ src,
                                                        size_t n4, float *__restrict__ dtail,
                                                        const float *__restrict__ stail, uint32_t ntail) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 a = dst[i];
        const float4 b = src[i];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        dst[i] = a;
    }
    if (blockIdx.x == 0 && threadIdx.x < ntail) dtail[threadIdx.x] += stail[threadIdx.x];
}

hipError_t mtsg_launch_film_accumulate(float *dst, const float *src, size_t n, int num_cus, hipStream_t s) {
    const size_t n4 = n / 4;
    const uint32_t tail = (uint32_t)(n - 4 * n4);
    const size_t want = (n4 + 255) / 256, cap = (size_t)std::max(num_cus, 1) * 8;
    const int grid = (int)std::max<size_t>(1, std::min(want, cap));
    hipLaunchKernelGGL(film_accumulate, dim3(grid), dim3(256), 0, s, (float4 *)dst, (const float4 *)src, n4,
                       dst + 4 * n4, src + 4 * n4, tail);
    return hipGetLastError();
}
