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
struct PathLaunch {
    int n_paths;            // n_rounds * n_list
    int n_list;             // pixels rendered by this context
    int s0;                 // first sample round of the chunk
    uint64_t seed;
    const int *pixel_list;  // y*W+x per list entry (ordered block by block)
    float4 *rec_rgbx;       // (r, g, b, jitter.x) per (round, list entry)
    float *rec_jy;          // jitter.y
    unsigned long long *counters;
};
struct SplatLaunch {
    float *fb;              // master RGBW (W+2b)x(H+2b)
    int width, height, border, reach, nbx, n_rounds, n_list;
    const int *pixel_map;   // image pixel -> list entry or -1
    const int *block_rank;  // BlockGenerator spiral rank per block id
    const float4 *rec_rgbx;
    const float *rec_jy;
    float radius, lookup;
    float table[33];
    // block-local ImageBlocks (one per (round, rendered block)), (32+2b)^2 RGBW each
    const int *blocks;      // rendered block ids, slot order
    const int *block_slot;  // block id -> slot or -1
    int n_blocks;
    float4 *staging;
};

namespace nh {
void launch_trace(const nhd::DScene *S, const nhd::Traversal &tv, const RayBatch &rb, const HitBatch &hb, int n,
                  bool any, bool ordered, bool stats, int depth, unsigned long long *ctr, hipStream_t st);
void launch_path(const nhd::DScene *S, const nhd::Traversal &tv, const PathLaunch &L, bool ordered, bool stats,
                 int depth, hipStream_t st);
void launch_splat(const SplatLaunch &P, hipStream_t st);
void launch_count_invalid(const float4 *rec, size_t n, unsigned long long *out, hipStream_t st);
}  // namespace nh

// Wavefront path state (nh_wavefront.hip): structure of arrays indexed by path id
// p = round * n_list + list entry, the same index as the sample records.
struct WfState {
    float4 *ray_o, *ray_d;   // (origin, mint), (direction, maxt) of the ray to trace next
    float4 *hit;             // (t, u, v, prim index bits or -1) from the extend kernel
    uint64_t *rng;           // pcg32 state (inc is derived from the sample index)
    float4 *li;              // (Li, w_mats)
    float4 *thr;             // (throughput, w_ems)
    float4 *pend_ems;        // pending NEE: (Li_ems, pdfems)
    float4 *pend_col;        // pending BSDF sample: (bsdf_col, pdfems_mats)
    float2 *pend_mis;        // (pdfmat, unused)
    float4 *sh_o, *sh_d;     // shadow ray (origin, mint), (direction, maxt)
    int *flags;              // measure | F_FIRST | F_NEE | path_mats counter
    uint8_t *occl;           // any-hit result of the shadow ray
    int *q_ext[2];           // extend queues (ping-pong)
    int *q_sh;               // shadow queue
    unsigned *counts;        // [0] next extend count, [1] shadow count
};
struct WfLaunch {
    WfState st;
    int n_paths, n_list, s0;
    uint64_t seed;
    const int *pixel_list;
    float4 *rec_rgbx;
    float *rec_jy;
    int n_ext, n_sh, in_q;
    unsigned long long *counters;
};
namespace nh {
void launch_wf_generate(const nhd::DScene *S, const WfLaunch &L, hipStream_t st);
void launch_wf_trace(const nhd::DScene *S, const nhd::Traversal &tv, const WfLaunch &L, bool ordered, bool stats,
                     bool shadow, int depth, hipStream_t st);
void launch_wf_shade(const nhd::DScene *S, const nhd::Traversal &tv, const WfLaunch &L, hipStream_t st);
}  // namespace nh
