// Check of nhd::fdiv (nh_device.h: rcp_rn + one FMA correction, Markstein) against the correctly rounded
// division a / b on the GPU: every one of the 2^23 significands of b (both signs, exponents spread over
// the fast range [2^-40, 2^40]) against 256 a each (random significands and exponents over the range,
// exact zeros of both signs, a = b, a = -b, a near the range limits). Also runs the slow-path inputs
// (outside the range, NaN, inf, denormals) through fdiv to check the fallback. Prints the counts.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "nh_device.h"

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__global__ void check(uint32_t chunk, unsigned long long *tested, unsigned long long *bad, uint32_t *first_a,
                      uint32_t *first_b) {
    const uint32_t m = chunk * 65536u + blockIdx.x * 256u + threadIdx.x;  // significand of b, 0 .. 2^23-1
    if (m >= (1u << 23)) return;
    unsigned long long n = 0, nb = 0;
    for (uint32_t j = 0; j < 256; ++j) {
        const uint32_t h = mix(m * 2654435761u + j * 40503u + 17u), h2 = mix(h + 0x9e3779b9u);
        const uint32_t eb = 127 - 40 + (h % 81), ea = 127 - 40 + (h2 % 81);  // exponents within 2^-40 .. 2^40
        const uint32_t sb = (j & 1) << 31, sa = ((j >> 1) & 1) << 31;
        const float b = __uint_as_float(sb | (eb << 23) | m);
        float a = __uint_as_float(sa | (ea << 23) | (mix(h2) & 0x7fffffu));
        if (j % 64 == 3) a = __uint_as_float(sa);             // +-0
        if (j % 64 == 5) a = b;                               // exact 1
        if (j % 64 == 7) a = -b;                              // exact -1
        if (j % 64 == 9) a = __uint_as_float(sa | ((127 + 40) << 23) | (h2 & 0x7fffffu));  // top of range
        if (j % 64 == 11) a = __uint_as_float(sa | ((127 - 40) << 23));                     // bottom of range
        const float ref = a / b, got = nhd::fdiv(a, b);
        ++n;
        if (__float_as_uint(ref) != __float_as_uint(got) && !(ref != ref && got != got)) {
            ++nb;
            first_a[0] = __float_as_uint(a);
            first_b[0] = __float_as_uint(b);
        }
    }
    // the fallback: inputs outside the fast range
    const float specials[8] = {0x1p-60f, 0x1p60f, 1e-40f, __uint_as_float(0x7f800000u), __uint_as_float(0x7fc00000u),
                               0x1p-130f, -0x1p100f, 3.0f};
    for (int i = 0; i < 8; ++i)
        for (int k = 0; k < 8; ++k) {
            const float a = specials[i] * (1.0f + (float)(m & 255) / 256.f), b = specials[k];
            const float ref = a / b, got = nhd::fdiv(a, b);
            ++n;
            if (__float_as_uint(ref) != __float_as_uint(got) && !(ref != ref && got != got)) ++nb;
        }
    atomicAdd(tested, n);
    if (nb) atomicAdd(bad, nb);
}

int main() {
    unsigned long long *tested = nullptr, *bad = nullptr;
    uint32_t *fa = nullptr, *fb = nullptr;
    if (hipMalloc(&tested, 8) != hipSuccess || hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&fa, 4) != hipSuccess ||
        hipMalloc(&fb, 4) != hipSuccess)
        return 2;
    if (hipMemset(tested, 0, 8) != hipSuccess || hipMemset(bad, 0, 8) != hipSuccess) return 2;
    for (uint32_t c = 0; c < 128; ++c) hipLaunchKernelGGL(check, dim3(256), dim3(256), 0, 0, c, tested, bad, fa, fb);
    unsigned long long t = 0, b = 0;
    uint32_t a0 = 0, b0 = 0;
    if (hipMemcpy(&t, tested, 8, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(&b, bad, 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&a0, fa, 4, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(&b0, fb, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    std::printf("pairs %llu mismatches %llu (last a 0x%08x b 0x%08x)\n", t, b, a0, b0);
    return b == 0 ? 0 : 1;
}
