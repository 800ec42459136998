// Exhaustive check of nhd::rcp_rn (nh_traverse.h) against the correctly rounded division 1.0f / x
// for all 2^32 float bit patterns, on the GPU (tests/test_gpu_parity.py runs it). Prints the number
// of mismatches overall and inside the range the kernels use rcp_rn for (|x| in [2^-125, 2^126),
// exponent field 2..252); NaN results compare equal to NaN results.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "nh_traverse.h"

__global__ void check(uint32_t hi, unsigned long long *bad, unsigned long long *bad_in_range, uint32_t *first) {
    const uint32_t bits = (hi << 24) | (blockIdx.x * 256u + threadIdx.x);
    const float x = __uint_as_float(bits);
    const float ref = 1.0f / x;  // correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt)
    const float got = nhd::rcp_rn(x);
    const bool same = __float_as_uint(ref) == __float_as_uint(got) || (ref != ref && got != got);
    if (!same) {
        atomicAdd(bad, 1ull);
        const uint32_t ex = (bits >> 23) & 0xffu;
        if (ex >= 2 && ex <= 252) {
            atomicAdd(bad_in_range, 1ull);
            atomicMin(first, bits);
        }
    }
}

int main() {
    unsigned long long *bad = nullptr, *bad_in = nullptr;
    uint32_t *first = nullptr;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&bad_in, 8) != hipSuccess || hipMalloc(&first, 4) != hipSuccess)
        return 2;
    if (hipMemset(bad, 0, 8) != hipSuccess || hipMemset(bad_in, 0, 8) != hipSuccess ||
        hipMemset(first, 0xff, 4) != hipSuccess)
        return 2;
    for (uint32_t hi = 0; hi < 256; ++hi) hipLaunchKernelGGL(check, dim3(65536), dim3(256), 0, 0, hi, bad, bad_in, first);
    unsigned long long h = 0, hin = 0;
    uint32_t f = 0;
    if (hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&hin, bad_in, 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    std::printf("inputs 4294967296 mismatches %llu in_range_mismatches %llu first_in_range 0x%08x\n", h, hin, f);
    return hin == 0 ? 0 : 1;
}
