// VALU issue ceiling of gfx950, measured: how many wave64 VALU instructions a CU issues per
// cycle with 1, 2, 4 and 8 waves per SIMD, for the instruction kinds the path kernels are made of -- fp32 FMA,
// packed fp32 FMA (v_pk_fma_f32), fp64 FMA (the fp64-evaluated transcendentals), fp32 sqrt (a transcendental-unit
// op) and a select / compare / integer mix. Each lane runs kChains independent dependency chains, so a single wave
// is never waiting on its own results for long; what remains is the SIMD's issue rate.
//
// Output: one line per (kind, waves/SIMD): wave64 VALU instructions per CU-cycle at the device's peak clock (from
// hipDeviceProp_t::clockRate) and the kernel time. Run it under `rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
// SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- tools/bin/valu_issue` for the counter view (scripts/valu_issue.sh).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kChains = 8;
constexpr int kIters = 4096;

typedef float f2 __attribute__((ext_vector_type(2)));

enum Kind { FMA32 = 0, PKFMA32 = 1, FMA64 = 2, SQRT32 = 3, MIX = 4 };
static const char *kName[] = {"v_fma_f32", "v_pk_fma_f32", "v_fma_f64", "v_sqrt_f32", "cmp+cndmask+xor+add_u32 mix"};

template <int KIND>
__global__ __launch_bounds__(256) void chains(float *out, float seed) {
    const float x = seed + (float)threadIdx.x * 1e-7f;
    float acc = 0.f;
    if constexpr (KIND == FMA32) {
        float a[kChains];
#pragma unroll
        for (int c = 0; c < kChains; ++c) a[c] = x + (float)c;
        for (int i = 0; i < kIters; ++i) {
#pragma unroll
            for (int c = 0; c < kChains; ++c)  // asm: the compiler would pair the chains into v_pk_fma_f32
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(0.999f), "v"(1e-3f));
        }
#pragma unroll
        for (int c = 0; c < kChains; ++c) acc += a[c];
    } else if constexpr (KIND == PKFMA32) {
        f2 a[kChains];
#pragma unroll
        for (int c = 0; c < kChains; ++c) a[c] = f2{x + (float)c, x - (float)c};
        const f2 m{0.999f, 0.998f}, b{1e-3f, 2e-3f};
        for (int i = 0; i < kIters; ++i) {
#pragma unroll
            for (int c = 0; c < kChains; ++c) a[c] = __builtin_elementwise_fma(a[c], m, b);
        }
#pragma unroll
        for (int c = 0; c < kChains; ++c) acc += a[c].x + a[c].y;
    } else if constexpr (KIND == FMA64) {
        double a[kChains];
#pragma unroll
        for (int c = 0; c < kChains; ++c) a[c] = (double)x + c;
        for (int i = 0; i < kIters; ++i) {
#pragma unroll
            for (int c = 0; c < kChains; ++c) a[c] = __builtin_fma(a[c], 0.999, 1e-3);
        }
#pragma unroll
        for (int c = 0; c < kChains; ++c) acc += (float)a[c];
    } else if constexpr (KIND == SQRT32) {
        float a[kChains];
#pragma unroll
        for (int c = 0; c < kChains; ++c) a[c] = x + (float)c + 2.f;
        for (int i = 0; i < kIters; ++i) {
#pragma unroll
            for (int c = 0; c < kChains; ++c) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[c]));
        }
#pragma unroll
        for (int c = 0; c < kChains; ++c) acc += a[c];
    } else {  // integer add, compare, select: the bookkeeping of traversal and ranking code
        unsigned a[kChains];
#pragma unroll
        for (int c = 0; c < kChains; ++c) a[c] = __float_as_uint(x) + c;
        for (int i = 0; i < kIters; ++i) {
#pragma unroll
            for (int c = 0; c < kChains; ++c) a[c] = (a[c] > 12345u ? a[c] : a[c] ^ 7u) + 0x9e37u;
        }
#pragma unroll
        for (int c = 0; c < kChains; ++c) acc += (float)(a[c] & 255u);
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int KIND>
static float run(int waves_per_simd, int n_cu, float *out, hipEvent_t a, hipEvent_t b) {
    // 256-thread workgroups = one wave per SIMD each; n_cu x W of them put W waves on every SIMD
    const dim3 grid(n_cu * waves_per_simd);
    hipLaunchKernelGGL(chains<KIND>, grid, dim3(256), 0, 0, out, 1.0f);  // warm
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(chains<KIND>, grid, dim3(256), 0, 0, out, 1.0f + r);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 5.f;
}

template <int KIND>
static void sweep(int n_cu, double clock_hz, float *out, hipEvent_t a, hipEvent_t b) {
    for (int w : {1, 2, 4, 8}) {
        const float ms = run<KIND>(w, n_cu, out, a, b);
        // wave64 instructions of the chains: waves x iterations x chains (x 4 for the mix: cmp, cndmask, xor, add)
        const double waves = (double)n_cu * w * 4;
        const double insts = waves * kIters * kChains * (KIND == MIX ? 4 : 1);
        const double cu_cycles = (double)ms * 1e-3 * clock_hz * n_cu;
        std::printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"wave_insts\": %.0f, "
                    "\"insts_per_cu_cycle_at_peak_clock\": %.3f}\n",
                    kName[KIND], w, ms, insts, insts / cu_cycles);
    }
}

int main(int argc, char **argv) {
    hipDeviceProp_t p{};
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 2;
    const int n_cu = p.multiProcessorCount;
    const double clock_hz = (double)p.clockRate * 1e3;
    std::printf("{\"device\": \"%s\", \"cus\": %d, \"peak_clock_mhz\": %.0f}\n", p.gcnArchName, n_cu, clock_hz / 1e6);
    float *out = nullptr;
    if (hipMalloc(&out, (size_t)n_cu * 8 * 256 * sizeof(float)) != hipSuccess) return 2;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int only = argc > 1 ? std::atoi(argv[1]) : -1;
    if (only < 0 || only == FMA32) sweep<FMA32>(n_cu, clock_hz, out, a, b);
    if (only < 0 || only == PKFMA32) sweep<PKFMA32>(n_cu, clock_hz, out, a, b);
    if (only < 0 || only == FMA64) sweep<FMA64>(n_cu, clock_hz, out, a, b);
    if (only < 0 || only == SQRT32) sweep<SQRT32>(n_cu, clock_hz, out, a, b);
    if (only < 0 || only == MIX) sweep<MIX>(n_cu, clock_hz, out, a, b);
    (void)hipFree(out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
