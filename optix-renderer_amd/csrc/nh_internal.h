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
