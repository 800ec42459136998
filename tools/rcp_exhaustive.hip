#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
// candidate: hardware reciprocal estimate + one FMA Newton step
__device__ __forceinline__ float rcp_fast(float x) {
    float r = __builtin_amdgcn_rcpf(x);
    float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__global__ void check(uint32_t hi, unsigned long long *bad, unsigned long long *bad_inrange, uint32_t *first) {
    uint32_t bits = (hi << 24) | (blockIdx.x * 256u + threadIdx.x);
    float x = __uint_as_float(bits);
    float ref = 1.0f / x;  // correctly rounded (built with -fhip-fp32-correctly-rounded-divide-sqrt)
    float got = rcp_fast(x);
    bool same = __float_as_uint(ref) == __float_as_uint(got) || (ref != ref && got != got);
    if (!same) {
        atomicAdd(bad, 1ull);
        uint32_t ex = (bits >> 23) & 0xff;
        if (ex >= 1 + 1 && ex <= 253 - 1) { atomicAdd(bad_inrange, 1ull); atomicMin(first, bits); }
    }
}
int main() {
    unsigned long long *bad, *bad_in; uint32_t *first;
    hipMalloc(&bad, 8); hipMalloc(&bad_in, 8); hipMalloc(&first, 4);
    hipMemset(bad, 0, 8); hipMemset(bad_in, 0, 8); hipMemset(first, 0xff, 4);
    for (uint32_t hi = 0; hi < 256; ++hi) hipLaunchKernelGGL(check, dim3(65536), dim3(256), 0, 0, hi, bad, bad_in, first);
    unsigned long long h, hin; uint32_t f;
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost); hipMemcpy(&hin, bad_in, 8, hipMemcpyDeviceToHost); hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
    printf("mismatches over all 2^32 inputs: %llu; with exponent field in [2, 252]: %llu (first 0x%08x = %g)\n", h, hin, f, *(float*)&f);
    return 0;
}
