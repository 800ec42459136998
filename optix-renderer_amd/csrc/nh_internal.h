// Internal structures shared between the C-ABI layer (nh_api.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nh_device.h"
#include "nh_traverse.h"

struct RayBatch {
    const float *ox, *oy, *oz, *dx, *dy, *dz, *mint, *maxt;
};
struct HitBatch {
    uint8_t *hit;
    float *t, *u, *v;
    int *k;
};
// floats per sample record: (r, g, b), padded to 4 with NH_REC_STRIDE=4 (16-B aligned records, an A/B build)
#ifndef NH_REC_STRIDE
#define NH_REC_STRIDE 3
#endif
constexpr int kRecFloats = NH_REC_STRIDE;

struct PathLaunch {
    int n_paths;            // n_rounds * n_list
    int n_list;             // pixels rendered by this context
    int s0;                 // first sample round of the chunk
    uint64_t seed;
    const int *pixel_list;  // y*W+x per list entry (ordered block by block)
    float *rec;             // (r, g, b) per (round, list entry); the splat recomputes the pixel jitter (sample_jitter)
    unsigned long long *counters;
};
// Row pitch (float4) of one (round, block) ImageBlock of (32+2b)^2 pixels in the splat's staging buffer: rows start
// on 128-B lines, so the merge's 16-pixel row segments (master columns 16a..16a+15 = block columns 0..15 / 16..31)
// read whole lines instead of straddling three (the unpadded 36-float4 rows start 64 B off a line every other row)
__host__ __device__ __forceinline__ int stage_pitch(int cols) { return (cols + 7) & ~7; }
// Offset (float4) of block-array pixel (xt, yt) in one (round, block) ImageBlock of the staging buffer (stride
// cols * stage_pitch(cols)). band = 1 (the 36x36 arrays of the tabulated splat): the 32x32 core row-major, then the
// right band (columns 32..35, 36 rows of 4), then the bottom band (rows 32..35, 32 columns), so the merge's reads --
// a wave's 4 rows x 16 master columns of one block's core, or of a neighbour's band -- are whole 128-B lines
__host__ __device__ __forceinline__ int stage_off(int cols, int band, int xt, int yt) {
    if (!band) return yt * stage_pitch(cols) + xt;
    if (xt >= 32) return 1024 + yt * 4 + (xt - 32);
    if (yt >= 32) return 1024 + 144 + (yt - 32) * 32 + xt;
    return yt * 32 + xt;
}

struct SplatLaunch {
    float *fb;              // master RGBW (W+2b)x(H+2b)
    int width, height, border, reach, nbx, n_rounds, n_list;
    const int *pixel_map;   // image pixel -> list entry or -1
    const int *block_rank;  // BlockGenerator spiral rank per block id
    const float *rec;       // (r, g, b) per (round, list entry)
    const float2 *jit;      // the stored jitter per record (A/B knob), else null: recomputed
    uint64_t seed;          // the chunk's seed and first sample round: the jitter of round k's sample at pixel p is
    int s0;                 // sample_jitter(seed, p, s0 + k), the camera sample's first two draws
    float radius, lookup;
    float table[33];
    // block-local ImageBlocks (one per (round, rendered block)), (32+2b)^2 RGBW each
    const int *blocks;      // rendered block ids, slot order
    const int *block_slot;  // block id -> slot or -1
    int n_blocks;
    float4 *staging;
    int staged;             // 1: staged pair (splat into staging, then merge); 0: the fused tile splat (no staging).
                            // Fixed when the chunk's staging was sized, so a knob change mid-pipeline cannot
                            // mismatch the two
    int direct;             // rounds the tab splat added to fb for pixels one block covers (the merge starts them there)
    int persist;            // tab splat: a grid of this many workgroups walks the items (0: one workgroup per item)
    int band;               // staging offsets: stage_off(.., band, ..) (1: the tabulated splat's core + band layout)
    const int *color_slots; // slots of the blocks with (bx + by) even, then odd: the pair splat's two launches
    int n_color0;           // how many are even
    int debug;              // timing experiments only (NH_SPLAT_DEBUG, images wrong): bits skip the fused splat's
                            // phase 1 (1), phase 2 (2), record fetch (4), master-border strips (8)
};

// SimpleDenoiser pass (nh_denoise.hip): interior pixel (i, j) of an image at ptr[i * stride + j]
struct DenoiseLaunch {
    const float4 *src;      // the image at the start of the pass
    int src_stride;
    float4 *dst;            // the denoised image (pixels before p in row-major order already final)
    int dst_stride;
    int width, height, range;
    float sigma_vr;
    const float *g;         // g_sigma by squared pixel distance, 2 range^2 + 1 entries (host expf)
    float *var;             // raw variance per pixel (width * height)
    unsigned *minmax;       // [0] max, [1] min of var (float bits)
    int band_first;         // band of workgroup 0 of this launch
    int lag;                // launches between a band's chunk k and the next band's chunk k
    int chunk;              // wavefront steps per band per launch
};

// In-kernel work counters (collect_stats): kStatShards copies of [0-3] queries, nodes, boxes, prims,
// [4] invalid samples, [8-11] the any-hit share, [16-19] / [20-23] the closest / any-hit work of
// the tail kernel, one copy per XCD (workgroup b adds to copy b % 8) so the per-wave atomics of
// concurrent workgroups do not serialise on one address.
constexpr int kStatShards = 8, kStatStride = 48, kStatAny = 8, kStatTail = 16, kStatTailAny = 20;
// wf_tail_rr calibration clocks: 4 phase cycle sums, path-bounces, longest chain (max over shards)
constexpr int kStatTailClk = 24;
constexpr int kStatTailCoopClk = 32;  // [32-35] the same phases for bounces carried by lane groups, [36] their count
// wf_bounce_rr calibration clocks: [40-45] cycle sums of its phases (load, body, shadow, closest, head, store),
// [46] the path-bounces it ran
constexpr int kStatBounceClk = 40;
__device__ __forceinline__ unsigned long long *stat_shard(unsigned long long *c) {
    return c + (blockIdx.x & (kStatShards - 1)) * kStatStride;
}

namespace nh {
void launch_trace(const nhd::DScene *S, const nhd::Traversal &tv, const RayBatch &rb, const HitBatch &hb, int n,
                  bool any, bool ordered, bool stats, int depth, unsigned long long *ctr, hipStream_t st);
void launch_trace_wide(const nhd::DScene *S, const nhd::Traversal &tv, const RayBatch &rb, const HitBatch &hb, int n,
                       bool any, bool ordered, bool stats, int2 *spill, int spill_depth, unsigned long long *ctr,
                       hipStream_t st, int wide = 4);
// pm: a path_mis scene without normal maps (the kernel instantiation with only li_path_mis and no normal maps)
void launch_path(const nhd::DScene *S, const nhd::Traversal &tv, const PathLaunch &L, bool ordered, bool stats,
                 int depth, bool pm, hipStream_t st);
void launch_splat(const SplatLaunch &P, hipStream_t st);
// false: launch_splat adds the records straight into the master (no per-(round, block) staging buffer)
bool splat_uses_staging(int border, int reach);
void launch_count_invalid(const float *rec, size_t n, unsigned long long *out, hipStream_t st);
void launch_denoise_variance(const DenoiseLaunch &P, hipStream_t st);
int denoise_band_rows();
int denoise_max_chunk();
int tree_top_nodes();  // wide nodes the persistent traversal stages in LDS (nh_wavefront.hip)
size_t denoise_tile_static_lds();
// tile_bytes > 0: the LDS-tiled kernel with that much dynamic shared memory (both windows of a chunk)
void launch_denoise_band(const DenoiseLaunch &P, int L, int n_bands, size_t tile_bytes, hipStream_t st);
void launch_denoise_copy(const float4 *src, int src_stride, float4 *dst, int dst_stride, int width, int height,
                         hipStream_t st);
}  // namespace nh

// Queue appends go to one counter per XCD (blocks are dealt round-robin over the 8 XCDs), so no
// address takes device-scope atomics from more than one XCD.
constexpr int kQueueShards = 8, kCountStride = 32;

// Wavefront path state (nh_wavefront.hip): one side of the double-buffered, dense SoA state.
// Slot s of a buffer holds one live path; pid is its sample-record index (round * n_list + entry).
struct WfBuf {
    float4 *ray_o;           // (origin, pdf of the BSDF sample that made the ray); mint = Epsilon
    float4 *ray_d;           // (direction, flags << kPidBits | pid); maxt = +inf, -inf for d = 0
    float4 *hit;             // (t, u, v, prim index bits or -1) from the extend kernel
    uint64_t *rng;           // pcg32 state (inc is derived from the sample index)
    float4 *li;              // (Li, w_mats)
    float4 *thr;             // (throughput, w_ems if the queued shadow ray is occluded)
    float4 *pend;            // queued NEE: (w_ems * t * Li_ems, w_ems if unoccluded)
    uint8_t *occl;           // any-hit result of the path's shadow ray
};
struct WfState {
    WfBuf buf[2];
    float4 *sh_o, *sh_d;     // shadow queue: (origin, mint), (direction, maxt)
    int *sh_slot;            // slot of the shadow ray's path in the buffer shade wrote
    unsigned *counts;        // per-shard append counters, one 128-B line each:
                             // [s * kCountStride] paths, [(kQueueShards + s) * kCountStride] shadow rays
};
// Queue counts live on the device: the shade kernel of bounce i appends into count slot
// (i+1)&1, the kernels of bounce i+1 read it (8 shard counts -> dense prefix) -- the host never
// sizes a grid from them, it only reads them back (one bounce behind) to know when to stop.
// A count slot holds 4 groups of kQueueShards counters, each on its own 128-B line:
//   group 0 path appends, 1 shadow-ray appends, 2 / 3 persistent extend / any-hit fetch cursors.
constexpr int kCountGroup = kQueueShards * kCountStride;
constexpr int kCountSlot = 4 * kCountGroup;

struct WfLaunch {
    WfState st;
    int n_paths, n_list, s0;
    uint64_t seed;
    const int *pixel_list;
    float *rec;             // (r, g, b) per (round, list entry)
    float2 *jit;            // NH_SPLAT_JITTER=stored only: the jitter per record, written at the first vertex
    int in_q;               // buffer (and count slot) read by this bounce
    int first;              // bounce 0: paths come from the camera, not from a buffer
    int cam_rays;           // bounce 0 of a thin-lens scene on the persistent kernels: the camera rays were written raw
                            // into buf[in_q].ray_o / ray_d by wf_camera_rays (the persistent refill builds pinhole
                            // rays only)
    unsigned *cnt_in;       // count slot of this bounce's input queues
    unsigned *cnt_out;      // count slot the shade kernel appends into
    int seg_cap;            // entries per shard segment of every queue / buffer
    // small scenes: float4 / int2 counts of the BVH arrays staged into LDS by the traversal
    // kernels (0 = traverse from HBM)
    int small_nodes, small_leaves, small_prims;
    int small_frames;  // 1: the fused kernels also stage the flat triangles' shading frames (Traversal::frames)
    // persistent traversal: per-lane stack spill area (kPersistentBlocks * 128 lanes x spill_depth
    // 32-bit words; the 4-wide traversal spills (ref, distance) pairs)
    uint32_t *trav_spill;
    int spill_depth;
    unsigned long long *counters;
};
// persistent traversal grid: 16 workgroups of 128 lanes per CU (the 8 waves/SIMD its registers allow)
constexpr int kPersistentBlocks = 256 * 16;
constexpr size_t kSmallSceneBytes = 16384;
constexpr int kSmallFramesMaxPrims = 256;  // frames staged (48 B per record) only for scenes this small
namespace nh {
void launch_wf_trace(const nhd::DScene *S, const nhd::Traversal &tv, const WfLaunch &L, bool ordered, bool stats,
                     bool shadow, bool persistent, int wide, int bound, int depth, hipStream_t st);
// sort: entries shaded in the order of their hit's BSDF type within each workgroup (material-sorted shading)
// closest-hit + any-hit queries of a bounce in one persistent launch (4-wide tree); bound = both queues' sum
void launch_wf_trace2(const nhd::DScene *S, const nhd::Traversal &tv, const WfLaunch &L, bool ordered, bool stats,
                      int wide, int bound, hipStream_t st);
// bounce 0 of a thin-lens scene on the persistent kernels: every camera ray (camera_ray with its lens sample) into
// buf[in_q].ray_o / ray_d, (origin, mint) / (direction, maxt), for the persistent refill to read (WfLaunch::cam_rays)
void launch_wf_camera_rays(const nhd::DScene *S, const WfLaunch &L, int bound, hipStream_t st);
void launch_wf_shade(const nhd::DScene *S, const nhd::Traversal &tv, const WfLaunch &L, bool sort, bool nmap, int bound,
                     hipStream_t st);
// fused shade + any-hit + closest-hit bounce for LDS-staged BVHs; sort = material-sorted output queue
void launch_wf_bounce(const nhd::DScene *S, const nhd::Traversal &tv, const WfLaunch &L, bool ordered, bool stats,
                      bool sort, int bound, hipStream_t st);
// RR-ahead variants of the fused bounce / tail (nh_wavefront.hip): the stored state is a path after its
// vertex's Russian roulette
// lean: the FULL = false body (no mirror / dielectric BSDF, no texture); nmap: the scene has shape normal maps (else the
// full body is the NMAP = false instantiation)
void launch_wf_bounce_rr(const nhd::DScene *S, const nhd::Traversal &tv, const WfLaunch &L, bool ordered, bool stats, bool sort,
                         bool lean, bool nmap, int bound, hipStream_t st);
void launch_wf_tail_rr(const nhd::DScene *S, const nhd::Traversal &tv, const WfLaunch &L, bool ordered, bool stats, int bound,
                       bool specular, bool lean, bool nmap, hipStream_t st);
void launch_wf_tail(const nhd::DScene *S, const nhd::Traversal &tv, const WfLaunch &L, bool ordered, bool stats,
                    int wide, int bound, int depth, hipStream_t st);
// copies the live RR-ahead paths of L's input queue (at most bound) densely into dst, count into dst_counts[0]
void launch_wf_pack_rr(const WfLaunch &L, const WfBuf &dst, unsigned *dst_counts, int bound, hipStream_t st);
// n_copy count words src -> host_dst (pinned, device-visible), then n_zero words of zero cleared (wf_counts_kernel)
void launch_wf_counts(const unsigned *src, unsigned *host_dst, int n_copy, unsigned *zero, int n_zero, hipStream_t st);
}  // namespace nh
