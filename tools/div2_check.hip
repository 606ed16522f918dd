// div2_check.hip -- dmath.h's packed division div2 against the compiler's IEEE f32
// division `/` on the device (gfx950), bit for bit (NaNs as a class): random bit
// patterns over the whole float range, random normal pairs, and the special values
// (zeros, denormals, infinities, NaNs, extreme exponents) crossed with each other.
// usage: div2_check [random pairs]   (prints one JSON line; exit 1 on a mismatch)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../mitsuba0.6_amd/csrc/dmath.h"

__global__ void div2_kernel(const float *a, const float2 *b, uint2 *mism, unsigned long long *nbad, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const f2v q = div2(a[i], f2v{b[i].x, b[i].y});
    const float r0 = a[i] / b[i].x, r1 = a[i] / b[i].y;
    const bool ok0 = (__float_as_uint(q.x) == __float_as_uint(r0)) || (q.x != q.x && r0 != r0);
    const bool ok1 = (__float_as_uint(q.y) == __float_as_uint(r1)) || (q.y != q.y && r1 != r1);
    if (!ok0 || !ok1) {
        const unsigned long long k = atomicAdd(nbad, 1ull);
        if (k < 16) mism[k] = make_uint2((uint32_t)i, ok0 ? 1u : 0u);
    }
}

static uint64_t s_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    s_state ^= s_state << 13; s_state ^= s_state >> 7; s_state ^= s_state << 17;
    return (uint32_t)(s_state >> 16);
}
static float bits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

int main(int argc, char **argv) {
    const size_t nr = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1u << 26);
    std::vector<float> a;
    std::vector<float2> b;
    const uint32_t sp[] = {0x00000000u, 0x80000000u, 0x00000001u, 0x80000001u, 0x007fffffu, 0x00800000u, 0x3f800000u,
                           0xbf800000u, 0x7f7fffffu, 0xff7fffffu, 0x7f800000u, 0xff800000u, 0x7fc00000u, 0x0b800000u,
                           0x33800000u, 0x4b800000u, 0x5f800000u, 0x1f800000u, 0x3f7fffffu, 0x3f800001u};
    const size_t ns = sizeof sp / sizeof sp[0];
    for (size_t i = 0; i < ns; ++i)
        for (size_t j = 0; j < ns; ++j)
            for (size_t k = 0; k < ns; ++k) { a.push_back(bits(sp[i])); b.push_back(make_float2(bits(sp[j]), bits(sp[k]))); }
    for (size_t i = 0; i < nr; ++i) {
        if (i & 1) {   // any bit pattern
            a.push_back(bits(rnd()));
            b.push_back(make_float2(bits(rnd()), bits(rnd())));
        } else {       // exponents within +-40 of 1: the quotients of real scenes
            auto nrm = [] { return bits((rnd() & 0x807fffffu) | ((uint32_t)(127 - 40 + rnd() % 81) << 23)); };
            a.push_back(nrm());
            b.push_back(make_float2(nrm(), nrm()));
        }
    }
    const size_t n = a.size();
    float *da; float2 *db; uint2 *dm; unsigned long long *dn;
    if (hipMalloc(&da, n * 4) || hipMalloc(&db, n * 8) || hipMalloc(&dm, 16 * 8) || hipMalloc(&dn, 8)) return 2;
    if (hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice) || hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice) ||
        hipMemset(dn, 0, 8))
        return 2;
    hipLaunchKernelGGL(div2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, da, db, dm, dn, n);
    unsigned long long nbad = 0;
    uint2 m[16];
    if (hipMemcpy(&nbad, dn, 8, hipMemcpyDeviceToHost) || hipMemcpy(m, dm, sizeof m, hipMemcpyDeviceToHost)) return 2;
    std::printf("{\"pairs\": %zu, \"quotients\": %zu, \"mismatches\": %llu", n, 2 * n, nbad);
    for (unsigned k = 0; k < nbad && k < 4; ++k) {
        const size_t i = m[k].x;
        std::printf(", \"m%u\": \"%a / (%a, %a)\"", k, a[i], b[i].x, b[i].y);
    }
    std::printf("}\n");
    return nbad ? 1 : 0;
}
