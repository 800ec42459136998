// GPU SimpleDenoiser: Denoiser::denoise on the master ImageBlock (src/utils/render.cpp:368-369) with the
// reference's own denoiser plugin, SimpleDenoiser (src/denoiser/simple.cpp:29-76), and its variance
// estimate computeVarianceFromImage (src/utils/common.cpp:339-398).
//
// The reference overwrites pixels in place, row-major: pixel p = (i, j) reads the new values of the pixels
// before it and the old values of the rest (p itself included). With the serial loop order (one TBB thread)
// that is a deterministic Gauss-Seidel sweep, and this is what the kernels compute: the pass reads the old
// image `src`, writes `dst`, and a term q of p reads dst when q precedes p in row-major order.
//
// Schedule. p depends on new values up to (i-1, j+r) and (i, j-1), so pixel (i, j) can run at wavefront
// step s = j + (r+1) i once every step < s is done; the pixels of one step are independent. Rows are cut
// into bands of kBandRows; one workgroup walks its band's steps in order (a barrier between steps), a launch
// runs `chunk` consecutive steps of every band in flight, and a band trails the band above it by enough
// launches that every value it needs from that band was written by an earlier launch (kernel boundaries
// make those writes visible across XCDs). One step of one pixel: the window's terms in parallel
// (weights into LDS), then the reference's sequential sums -- one lane per (pixel, channel) adding the
// terms in the reference's (i_, j_) order -- so the float sums are bit-for-bit the serial loop's.
#include "nh_internal.h"

namespace {

constexpr float kNoriEps = 1e-4f;
constexpr int kDnThreads = 256;
constexpr int kBandRows = 4;                 // rows per band (pixels per step per workgroup)
constexpr int kTermChunk = 256;              // window terms per LDS pass (range 7: 225 terms)
constexpr int kLanesPerPixel = 5;            // R, G, B, W sums and the weight sum
constexpr int kSumLanes = kBandRows * kLanesPerPixel;
constexpr int kMaxChunk = 16;                // steps per launch the tiled kernel precomputes (range <= 15)
static_assert(kSumLanes <= 64, "the sequential sums run in wave 0");

// Color4f::divideByFilterWeight().getLuminance() (include/nori/color.h:113-118, common.cpp:265-268)
__device__ __forceinline__ float block_luminance(float4 c) {
    float r = 0.f, g = 0.f, b = 0.f;
    if (fabsf(c.w) > kNoriEps) { r = c.x / c.w; g = c.y / c.w; b = c.z / c.w; }
    return r * 0.212671f + g * 0.715160f + b * 0.072169f;
}

// computeVarianceFromImage's raw 3x3 variance per pixel (common.cpp:341-377) and its max / min (:381-382)
// as ordered bit patterns (every value is +0 or positive: a sum of squares starting at +0). The C++ rules
// make std::pow(float, 2) a double pow: term and running sum in double, stored back to float.
__global__ __launch_bounds__(256) void dn_variance_kernel(DenoiseLaunch P) {
    const int j = blockIdx.x * 16 + (threadIdx.x & 15), i = blockIdx.y * 16 + (threadIdx.x >> 4);
    const bool in = i < P.height && j < P.width;
    unsigned vb_max = 0u, vb_min = 0x7f800000u;
    if (in) {
        float lum[9];
        bool ok[9];
        float mean = 0.f, sum = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int l = 0; l < 3; ++l) {
                const int i_ = i - 1 + k, j_ = j - 1 + l;
                const bool v = i_ >= 0 && i_ <= P.height - 1 && j_ >= 0 && j_ <= P.width - 1;
                ok[3 * k + l] = v;
                lum[3 * k + l] = 0.f;
                if (v) {
                    lum[3 * k + l] = fabsf(block_luminance(P.src[(size_t)i_ * P.src_stride + j_]));
                    mean += lum[3 * k + l];
                    sum += 1.f;
                }
            }
        mean /= sum;
        const double inv = (double)(1.f / sum);
        float col = 0.f;
#pragma unroll
        for (int n = 0; n < 9; ++n)
            if (ok[n]) {
                const double d = (double)(lum[n] - mean);
                col = (float)((double)col + inv * (d * d));
            }
        P.var[(size_t)i * P.width + j] = col;
        vb_max = vb_min = __float_as_uint(col);
    }
    for (int o = 32; o > 0; o >>= 1) {
        vb_max = max(vb_max, (unsigned)__shfl_xor((int)vb_max, o, 64));
        vb_min = min(vb_min, (unsigned)__shfl_xor((int)vb_min, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&P.minmax[0], vb_max);
        atomicMin(&P.minmax[1], vb_min);
    }
}

struct DnPixel {
    int i, j, is, js, nj, n;  // pixel, window origin, window width, window terms (0: no pixel this step)
    float4 ip;                // p's value at the start of the pass
    float vn;                 // normalised variance of p (common.cpp:383-395)
};

// One launch: `chunk` steps of every band in flight (see the schedule above). Band w runs its k-th chunk,
// k = L - w * lag, covering global steps [row0 (r+1) + k chunk, ... + chunk) (row0 (r+1): the band's first).
// TILE: the chunk's whole window -- input pixels and the denoised ones written by earlier launches -- is
// copied to LDS once (dynamic shared memory, DenoiseLaunch::tile_* bounds) and the steps run from LDS; the
// pixels this launch denoises go to the LDS copy as well as to dst. Without TILE every term reads HBM/L2.
template <bool TILE>
__global__ __launch_bounds__(kDnThreads) void dn_band_kernel(DenoiseLaunch P, int L) {
    extern __shared__ float4 s_tile[];                   // TILE: src window, then dst window
    __shared__ float s_val[kSumLanes][kTermChunk + 1];  // +1: the summing lanes read distinct banks
    __shared__ DnPixel s_px[kMaxChunk][kBandRows];      // per step of the chunk, per band row
    const int w = P.band_first + blockIdx.x;
    const int k = L - w * P.lag;
    const int row0 = w * kBandRows, rows = min(kBandRows, P.height - row0);
    const int span = (P.range + 1) * (rows - 1) + P.width;  // steps with work in this band
    if (k < 0 || rows <= 0 || k * P.chunk >= span) return;
    const int r = P.range, lane = threadIdx.x;
    const int s0 = row0 * (r + 1) + k * P.chunk;  // global wavefront step of the chunk's first step
    const int nst = TILE ? P.chunk : 1;           // steps whose pixel setup is precomputed at once
    // window of the chunk: rows [ti0, ti1], columns [tj0, tj1] (clamped to the image)
    const int ti0 = max(row0 - r, 0), ti1 = min(row0 + rows - 1 + r, P.height - 1);
    const int tj0 = max(s0 - (r + 1) * (row0 + rows - 1) - r, 0), tj1 = min(s0 + P.chunk - 1 - (r + 1) * row0 + r, P.width - 1);
    const int tw = tj1 - tj0 + 1, tn = tw > 0 ? (ti1 - ti0 + 1) * tw : 0;
    float4 *t_src = s_tile, *t_dst = s_tile + (TILE ? tn : 0);
    if constexpr (TILE) {
        for (int e = lane; e < tn; e += kDnThreads) {
            const int di = e / tw, i_ = ti0 + di, j_ = tj0 + (e - di * tw);
            t_src[e] = P.src[(size_t)i_ * P.src_stride + j_];
            t_dst[e] = P.dst[(size_t)i_ * P.dst_stride + j_];
        }
    }
    const float mx = __uint_as_float(P.minmax[0]), mn = __uint_as_float(P.minmax[1]);
    const bool flat = mx - mn < kNoriEps;
    float acc = 0.f;  // wave 0, lane < kSumLanes: running sum of (pixel lane / 5, channel lane % 5)
    for (int st = 0; st < P.chunk; ++st) {
        const int s = s0 + st;  // global wavefront step
        const int slot = TILE ? st : 0;
        if (!TILE || st == 0) {  // pixel setup: every step of the chunk at once (TILE) or this step
            for (int e = lane; e < nst * kBandRows; e += kDnThreads) {
                const int q = e / kBandRows, a = e - q * kBandRows;
                DnPixel px{};
                const int i = row0 + a, j = s + q - (r + 1) * i;
                if (a < rows && j >= 0 && j < P.width) {
                    px.i = i;
                    px.j = j;
                    px.is = max(i - r, 0);
                    px.js = max(j - r, 0);
                    px.nj = min(j + r + 1, P.width) - px.js;
                    px.n = (min(i + r + 1, P.height) - px.is) * px.nj;
                    px.ip = P.src[(size_t)i * P.src_stride + j];
                    const float v = P.var[(size_t)i * P.width + j];
                    px.vn = flat ? 0.f : 1.f + (v - mn) / (mx - mn) * 0.254f;
                }
                s_px[q][a] = px;
            }
            __syncthreads();
        }
        int n_max = 0;
#pragma unroll
        for (int a = 0; a < kBandRows; ++a) n_max = max(n_max, s_px[slot][a].n);
        if (n_max == 0) {
            if (!TILE) __syncthreads();
            continue;
        }
        if (lane < kSumLanes) acc = 0.f;
        for (int t0 = 0; t0 < n_max; t0 += kTermChunk) {
            // window terms: weight g * f and the four weighted channels (simple.cpp:56-66, f_prime :140-149)
            for (int task = lane; task < kBandRows * kTermChunk; task += kDnThreads) {
                const int a = task / kTermChunk, t = t0 + (task - a * kTermChunk);
                const DnPixel &px = s_px[slot][a];
                if (t >= px.n) continue;
                const int di = t / px.nj;
                const int i_ = px.is + di, j_ = px.js + (t - di * px.nj);
                // q before p in row-major order: its new value (dst), else the pass's input (src). One integer
                // comparison and a select of the row address: the short-circuit form (i_ < i || (i_ == i &&
                // j_ < j)) with the buffer chosen inside the branches was miscompiled (dst base with src stride)
                const bool before = i_ * P.width + j_ < px.i * P.width + px.j;
                float4 iq;
                if constexpr (TILE) {
                    const float4 *tb = before ? t_dst : t_src;
                    iq = tb[(i_ - ti0) * tw + (j_ - tj0)];
                } else {
                    const float4 *row = before ? P.dst + (size_t)i_ * P.dst_stride : P.src + (size_t)i_ * P.src_stride;
                    iq = row[j_];
                }
                const int dsq = (px.i - i_) * (px.i - i_) + (px.j - j_) * (px.j - j_);
                const float g = P.g[dsq];
                // Eigen Vector4f::lpNorm<1>: (|x0| + |x2|) + (|x1| + |x3|)
                const float l1 = (fabsf(px.ip.x - iq.x) + fabsf(px.ip.z - iq.z)) +
                                 (fabsf(px.ip.y - iq.y) + fabsf(px.ip.w - iq.w));
                const float x = (l1 * px.vn) / P.sigma_vr;
                const float f = (float)exp(-0.5 * ((double)x * (double)x));
                const float wgt = g * f;
                const int c = t - t0;
                s_val[a * kLanesPerPixel + 0][c] = iq.x * wgt;
                s_val[a * kLanesPerPixel + 1][c] = iq.y * wgt;
                s_val[a * kLanesPerPixel + 2][c] = iq.z * wgt;
                s_val[a * kLanesPerPixel + 3][c] = iq.w * wgt;
                s_val[a * kLanesPerPixel + 4][c] = wgt;
            }
            __syncthreads();
            // the reference's running sums, term by term in window order
            if (lane < kSumLanes) {
                const int a = lane / kLanesPerPixel;
                const int m = min(s_px[slot][a].n - t0, kTermChunk);
                const float *v = s_val[lane];
                float x = acc;
                // 16-term batches, the next batch's LDS reads issued before this batch's dependent adds
                constexpr int kB = 16;
                float cur[kB], nxt[kB];
                int t = 0;
                if (m >= kB) {
#pragma unroll
                    for (int u = 0; u < kB; ++u) cur[u] = v[u];
                    for (; t + 2 * kB <= m; t += kB) {
#pragma unroll
                        for (int u = 0; u < kB; ++u) nxt[u] = v[t + kB + u];
#pragma unroll
                        for (int u = 0; u < kB; ++u) x += cur[u];
#pragma unroll
                        for (int u = 0; u < kB; ++u) cur[u] = nxt[u];
                    }
#pragma unroll
                    for (int u = 0; u < kB; ++u) x += cur[u];
                    t += kB;
                }
                for (; t < m; ++t) x += v[t];
                acc = x;
            }
            if (t0 + kTermChunk < n_max) __syncthreads();  // s_val is refilled by the next term chunk
        }
        // result[k] / sum_weights (simple.cpp:71-72)
        if (threadIdx.x < 64) {
            const int a = lane / kLanesPerPixel, ch = lane - a * kLanesPerPixel;
            const float wsum = __shfl(acc, a * kLanesPerPixel + 4, 64);
            if (lane < kSumLanes && ch < 4 && s_px[slot][a].n > 0) {
                const DnPixel &px = s_px[slot][a];
                const float o = acc / wsum;
                reinterpret_cast<float *>(&P.dst[(size_t)px.i * P.dst_stride + px.j])[ch] = o;
                if constexpr (TILE) reinterpret_cast<float *>(&t_dst[(px.i - ti0) * tw + (px.j - tj0)])[ch] = o;
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void dn_copy_kernel(const float4 *src, int src_stride, float4 *dst, int dst_stride,
                                                      int width, int height) {
    const int j = blockIdx.x * 16 + (threadIdx.x & 15), i = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (i < height && j < width) dst[(size_t)i * dst_stride + j] = src[(size_t)i * src_stride + j];
}

}  // namespace

namespace nh {

void launch_denoise_variance(const DenoiseLaunch &P, hipStream_t st) {
    dim3 grid((P.width + 15) / 16, (P.height + 15) / 16);
    hipLaunchKernelGGL(dn_variance_kernel, grid, dim3(256), 0, st, P);
}

int denoise_band_rows() { return kBandRows; }

int denoise_max_chunk() { return kMaxChunk; }

// static LDS of the tiled band kernel (s_val + s_px), added to the dynamic tile when sizing a launch
size_t denoise_tile_static_lds() {
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&dn_band_kernel<true>)) != hipSuccess) return 0;
    return a.sharedSizeBytes;
}

void launch_denoise_band(const DenoiseLaunch &P, int L, int n_bands, size_t tile_bytes, hipStream_t st) {
    if (tile_bytes) hipLaunchKernelGGL(dn_band_kernel<true>, dim3(n_bands), dim3(kDnThreads), tile_bytes, st, P, L);
    else hipLaunchKernelGGL(dn_band_kernel<false>, dim3(n_bands), dim3(kDnThreads), 0, st, P, L);
}

void launch_denoise_copy(const float4 *src, int src_stride, float4 *dst, int dst_stride, int width, int height,
                         hipStream_t st) {
    dim3 grid((width + 15) / 16, (height + 15) / 16);
    hipLaunchKernelGGL(dn_copy_kernel, grid, dim3(256), 0, st, src, src_stride, dst, dst_stride, width, height);
}

}  // namespace nh
