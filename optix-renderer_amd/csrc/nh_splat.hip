// gfx950 kernels of the ImageBlock stage of the path_mis hot path (src/utils/block.cpp:93-134,
// src/utils/render.cpp:421-458): the sample records of a chunk of rounds -> the master ImageBlock.
//
//   nh_tile_splat_kernel   (2-pixel border, the default) splat + merge fused: per 32x32 master tile, every
//                          round's block values in BlockGenerator spiral order, straight into the master
//   nh_block_splat_*       ImageBlock::put(pos, value) into each (round, block)'s own ImageBlock, samples in
//                          getSampleIndices order (x outer, y inner), staged in HBM
//   nh_merge_kernel        ImageBlock::put(block) into the master: per master pixel, rounds in order, blocks in
//                          spiral order -- the serial reference's summation order, bit for bit
#include <cstdio>
#include <cstdlib>

#include "nh_internal.h"
#include "nh_shade.h"

using namespace nhd;

namespace {

// ImageBlock::put(pos, value) into the per-block ImageBlock of one (round, block)
// (src/utils/render.cpp:421-458 + src/utils/block.cpp:93-123). One workgroup per
// (block, round): phase 1 computes every sample's filter footprint once into LDS; phase 2
// gives each block-array pixel the ordered sum of its contributions, in the reference's
// getSampleIndices order (x outer, y inner), starting from the cleared block (0).
constexpr int kSplatMaxCols = 40;  // 32 + 2*border, border <= 4
constexpr int kStripRows = 6;      // block-array rows one thread sums in the strip variant

// sample record r: (r, g, b)
__device__ __forceinline__ F3 load_rec(const float *rec, size_t r) {
    return f3(rec[kRecFloats * r], rec[kRecFloats * r + 1], rec[kRecFloats * r + 2]);
}

// phase 1 of the block splat: every sample's footprint (block-array box), filter position and value into LDS
// (sample (lx, ly) at lx*33 + ly: x-major, the odd stride keeps neighbouring lx on distinct banks)
struct SplatLds {
    float val[3][32 * 33];
    float pos[2][32 * 33];
    int box[32 * 33];  // x0 | x1<<8 | y0<<16 | y1<<24 (block-array coords), x1 < x0: empty
    float tab[33];
};
__device__ __forceinline__ void splat_stage(const SplatLaunch &P, SplatLds &L, int ox, int oy, int sxb, int syb, int k,
                                            int cols) {
    const float r = P.radius;
    if (threadIdx.x < 33) L.tab[threadIdx.x] = P.table[threadIdx.x];
    const size_t rbase = (size_t)k * P.n_list;
    for (int i = threadIdx.x; i < 1024; i += 256) {
        // thread i loads pixel (lx, ly) = (i % 32, i / 32): neighbouring lanes read neighbouring pixels of a
        // block row, i.e. consecutive list entries (the pixel list is row-major inside a block), so each
        // wave's record loads are 16-B-per-lane contiguous runs; the LDS layout is x-major
        const int lx = i & 31, ly = i >> 5;
        int box = 0xff;  // x0 = 255 > x1 = 0: empty
        float vx = 0.f, vy = 0.f, vz = 0.f, px = 0.f, py = 0.f;
        if (lx < sxb && ly < syb) {
            const int li = P.pixel_map[(oy + ly) * P.width + (ox + lx)];
            if (li >= 0) {
                const F3 rec = load_rec(P.rec, rbase + li);
                if (is_valid(rec)) {  // invalid samples drop with their weight
                    float jx, jy;
                    sample_jitter_h(splitmix64(P.seed ^ (uint64_t)((oy + ly) * P.width + (ox + lx))),
                                    (uint64_t)(P.s0 + k), jx, jy);
                    const float spx = (float)(ox + lx) + jx, spy = (float)(oy + ly) + jy;
                    px = spx - 0.5f - (float)(ox - P.border);
                    py = spy - 0.5f - (float)(oy - P.border);
                    int x0 = max((int)ceilf(px - r), 0), y0 = max((int)ceilf(py - r), 0);
                    int x1 = min((int)floorf(px + r), cols - 1), y1 = min((int)floorf(py + r), cols - 1);
                    box = x0 | (x1 << 8) | (y0 << 16) | (y1 << 24);
                    vx = rec.x; vy = rec.y; vz = rec.z;
                }
            }
        }
        const int j = lx * 33 + ly;
        L.val[0][j] = vx; L.val[1][j] = vy; L.val[2][j] = vz;
        L.pos[0][j] = px; L.pos[1][j] = py;
        L.box[j] = box;
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void nh_block_splat_kernel(SplatLaunch P) {
    __shared__ SplatLds L;
    const int slot = blockIdx.x, k = blockIdx.y;
    const int bid = P.blocks[slot];
    const int by = bid / P.nbx, bx = bid - by * P.nbx;
    const int ox = bx * 32, oy = by * 32;
    const int sxb = min(32, P.width - ox), syb = min(32, P.height - oy);
    const int cols = 32 + 2 * P.border;
    splat_stage(P, L, ox, oy, sxb, syb, k, cols);
    const int pitch = stage_pitch(cols);
    float4 *out = P.staging + ((size_t)k * P.n_blocks + slot) * (size_t)(cols * pitch);
    const int R = P.reach, bd = P.border;
    for (int q = threadIdx.x; q < cols * cols; q += 256) {
        const int yt = q / cols, xt = q - yt * cols;
        float ar = 0.f, ag = 0.f, ab = 0.f, aw = 0.f;
        const int lx0 = max(xt - bd - R, 0), lx1 = min(xt - bd + R, sxb - 1);
        const int ly0 = max(yt - bd - R, 0), ly1 = min(yt - bd + R, syb - 1);
        for (int lx = lx0; lx <= lx1; ++lx)
            for (int ly = ly0; ly <= ly1; ++ly) {
                const int i = lx * 33 + ly;
                const int box = L.box[i];
                const int x0 = box & 0xff, x1 = (box >> 8) & 0xff, y0 = (box >> 16) & 0xff, y1 = (box >> 24) & 0xff;
                if (xt < x0 || xt > x1 || yt < y0 || yt > y1) continue;
                const float wx = L.tab[(int)(fabsf((float)xt - L.pos[0][i]) * P.lookup)];
                const float wy = L.tab[(int)(fabsf((float)yt - L.pos[1][i]) * P.lookup)];
                ar += L.val[0][i] * wx * wy;
                ag += L.val[1][i] * wx * wy;
                ab += L.val[2][i] * wx * wy;
                aw += 1.0f * wx * wy;
            }
        out[yt * pitch + xt] = make_float4(ar, ag, ab, aw);
    }
}

// The same block splat with each thread summing a strip of kStripRows block-array pixels of one column: a
// candidate sample's record, x test and column weight are read / computed once for the strip, and its products
// (v * wx) once as packed-FP32 pairs; each pixel of the strip then takes its row test, row weight and
// ((v * wx) * wy) products. Every pixel still sums its samples' contributions in getSampleIndices order (the
// strip walks samples x-major), so the floats are those of nh_block_splat_kernel.
typedef float sf2 __attribute__((ext_vector_type(2)));
// a * (b.x, b.x) and a * (b.y, b.y) as one v_pk_mul_f32 with the half of b picked by op_sel (the compiler otherwise
// copies a scalar operand into the low register of a pair first)
__device__ __forceinline__ sf2 pk_mul_lo(sf2 a, sf2 b) {
    sf2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ sf2 pk_mul_hi(sf2 a, sf2 b) {
    sf2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__global__ __launch_bounds__(256) void nh_block_splat_strip_kernel(SplatLaunch P) {
    __shared__ SplatLds L;
    const int slot = blockIdx.x, k = blockIdx.y;
    const int bid = P.blocks[slot];
    const int by = bid / P.nbx, bx = bid - by * P.nbx;
    const int ox = bx * 32, oy = by * 32;
    const int sxb = min(32, P.width - ox), syb = min(32, P.height - oy);
    const int cols = 32 + 2 * P.border;
    splat_stage(P, L, ox, oy, sxb, syb, k, cols);
    const int pitch = stage_pitch(cols);
    float4 *out = P.staging + ((size_t)k * P.n_blocks + slot) * (size_t)(cols * pitch);
    const int R = P.reach, bd = P.border;
    const int n_strips = (cols + kStripRows - 1) / kStripRows;
    for (int t = threadIdx.x; t < cols * n_strips; t += 256) {
        const int xt = t % cols, yt0 = (t / cols) * kStripRows;
        sf2 rg[kStripRows], bw[kStripRows];
#pragma unroll
        for (int j = 0; j < kStripRows; ++j) {
            rg[j] = sf2{0.f, 0.f};
            bw[j] = sf2{0.f, 0.f};
        }
        const int lx0 = max(xt - bd - R, 0), lx1 = min(xt - bd + R, sxb - 1);
        const int ly0 = max(yt0 - bd - R, 0), ly1 = min(yt0 + kStripRows - 1 - bd + R, syb - 1);
        const float fxt = (float)xt;
        for (int lx = lx0; lx <= lx1; ++lx)
            for (int ly = ly0; ly <= ly1; ++ly) {
                const int i = lx * 33 + ly;
                const int box = L.box[i];
                const int x0 = box & 0xff, x1 = (box >> 8) & 0xff;
                if (xt < x0 || xt > x1) continue;
                const int y0 = (box >> 16) & 0xff, y1 = (box >> 24) & 0xff;
                const float wx = L.tab[(int)(fabsf(fxt - L.pos[0][i]) * P.lookup)];
                const float py = L.pos[1][i];
                const sf2 vrg = sf2{L.val[0][i], L.val[1][i]} * wx, vbw = sf2{L.val[2][i], 1.0f} * wx;
#pragma unroll
                for (int j = 0; j < kStripRows; ++j) {
                    const int yt = yt0 + j;
                    if (yt < y0 || yt > y1) continue;
                    const float wy = L.tab[(int)(fabsf((float)yt - py) * P.lookup)];
                    rg[j] += vrg * wy;
                    bw[j] += vbw * wy;
                }
            }
#pragma unroll
        for (int j = 0; j < kStripRows; ++j)
            if (yt0 + j < cols) out[(yt0 + j) * pitch + xt] = make_float4(rg[j].x, rg[j].y, bw[j].x, bw[j].y);
    }
}

// Rendered blocks whose merged region ((sx+2b) x (sy+2b) at offset (ox, oy) in master coordinates)
// covers master pixel (mx, my), in BlockGenerator spiral order: the order ImageBlock::put(ImageBlock&)
// adds them (src/utils/block.cpp:125-134). Returns their number (<= 4) and slots.
__device__ __forceinline__ int covering_blocks(const SplatLaunch &P, int mx, int my, int *slot) {
    const int cols = 32 + 2 * P.border;
    int blk[4], nb = 0;
    const int bx_lo = max((mx - cols + 1 + 31) >> 5, 0), bx_hi = min(mx >> 5, P.nbx - 1);
    const int nby = (P.height + 31) >> 5;
    const int by_lo = max((my - cols + 1 + 31) >> 5, 0), by_hi = min(my >> 5, nby - 1);
    for (int by = by_lo; by <= by_hi; ++by)
        for (int bx = bx_lo; bx <= bx_hi; ++bx) {
            const int bid = by * P.nbx + bx;
            const int sl = P.block_slot[bid];
            if (sl < 0) continue;
            const int ox = bx * 32, oy = by * 32;
            const int sxb = min(32, P.width - ox), syb = min(32, P.height - oy);
            if (mx - ox >= sxb + 2 * P.border || my - oy >= syb + 2 * P.border) continue;
            blk[nb] = bid;
            slot[nb] = sl;
            ++nb;
        }
    for (int a = 1; a < nb; ++a)
        for (int b = a; b > 0 && P.block_rank[blk[b]] < P.block_rank[blk[b - 1]]; --b) {
            int t = blk[b]; blk[b] = blk[b - 1]; blk[b - 1] = t;
            t = slot[b]; slot[b] = slot[b - 1]; slot[b - 1] = t;
        }
    return nb;
}

// Block splat for the 2-pixel border (filter radius in (1.5, 2.5): Nori's default Gaussian, Mitchell-Netravali),
// where a sample at block pixel (lx, ly) can only reach block-array columns lx..lx+4 and rows ly..ly+4.
// Phase 1 tabulates each sample's filter weights for those five columns and rows -- wx[d] = the reference's
// m_weightsX entry for column lx+2+d, 0 outside its box -- so phase 2 does no box test and no table lookup.
// Phase 2 gives each thread a 6-pixel column strip; for every candidate sample (x-major, as getSampleIndices
// orders them) the rows the sample reaches are compile-time offsets, each taking ((v * wx) * wy) as packed
// pairs. A sample outside the block, absent or invalid has all weights 0: it adds (+-)0 to sums that start
// at +0 and can never be -0, and finite (v * wx) * 0 is 0, so every sum is the one the reference forms.
// Each workgroup walks kTabRounds rounds of one block; the next round's records are loaded during the
// current round's phase 2.
constexpr int kTabRounds = 8;  // 8: the lead workgroups take half the rounds (fewest staged bytes, fastest)
constexpr int kTabRow = 33;                 // plane row: lx 0..31 + a zero column (lx outside 0..31)
constexpr int kTabPlane = 40 * kTabRow;     // rows ly = -4..35 (ly + 4): 4 zero rows either side
// planes (kTabPlane floats each): 0-1 the (r, g) pairs, 2-3 the (b, 1) pairs -- float2 planes, so phase 2 loads
// each packed operand whole instead of assembling it from two planes -- then 5 column and 5 row weights
constexpr int kTabRG = 0, kTabBW = 2, kTabWX = 4, kTabWY = 9, kTabPlanes = 14;
// DIRECT: one workgroup walks all the chunk's rounds of its block, and block-array pixels whose master pixel no
// other rendered block covers (the block's 28x28 interior, and the master border of edge blocks) add each round's
// value straight into the master in round order -- the merge's sum for a pixel with one covering block -- so only
// the pixels shared with neighbouring blocks go through the staging buffer and nh_merge_kernel.
// DIRECT (tab_body): rounds [k0, k1) of the pixels this block alone covers go straight into the master, accumulated
// in registers; the kernel runs it for all rounds (nh_block_splat_tab_kernel<true>) or, by default, for the first
// workgroup of each block (rounds 0 .. ROUNDS-1: they come first in the merge's order, which starts those pixels at
// round P.direct). A separate inlined body per mode keeps the staged-only workgroups at their own register count.
// (A read-modify-write of the framebuffer per round instead of the registers was built and spills past 256 VGPRs.)
// JIT: the jitter read from P.jit (NH_SPLAT_JITTER=stored) instead of recomputed -- a template parameter: a runtime
// choice between the two costs the recomputing kernel 6 % (profiles/round4_session9_10_splat_ab.txt)
// T: workgroup threads. 256: 6-row strips, 4 phase-1 samples per thread; 512: 3-row strips, 2 samples per thread --
// the same LDS per workgroup, half the registers per thread, so twice the waves per CU fit (NH_SPLAT_T512)
// PAIR (with DIRECT, all rounds): the pair splat (launch_splat, NH_SPLAT_PAIR). The blocks run in two launches, those
// with (bx + by) even first. A master pixel two side-by-side blocks cover (the 4-pixel seams) is staged by the even
// block only; the odd block's workgroup reads that value back per round and adds both blocks' values to the master in
// spiral order itself, like a pixel only it covers. Pixels of the 4x4 corner squares with three or four covering blocks
// (or two diagonal ones) are staged by every covering block and finished by nh_corner_merge_kernel. The per-pixel
// summation order is the merge's: rounds in order, blocks in spiral order within a round.
template <bool DIRECT, bool JIT = false, int T = 256, bool PAIR = false>
__device__ __forceinline__ void tab_body(const SplatLaunch &P, float *W, float *tab, int slot, int k0, int k1) {
    constexpr int SR = T == 512 ? 3 : kStripRows, NS = 36 / SR, NQ = 1024 / T;
    static_assert(SR * NS == 36 && NQ * T == 1024, "strip tiling");
    const int bid = P.blocks[slot];
    const int by = bid / P.nbx, bx = bid - by * P.nbx;
    const int ox = bx * 32, oy = by * 32;
    const int sxb = min(32, P.width - ox), syb = min(32, P.height - oy);
    const float r = P.radius;
    if (threadIdx.x < 33) tab[threadIdx.x] = P.table[threadIdx.x];
    // the zero rows and column are never written again
    float2 *const W2 = reinterpret_cast<float2 *>(W);  // the pair planes, indexed like one float plane
    for (int i = threadIdx.x; i < (kTabPlanes - kTabWX) * 40; i += T) {
        const int p = kTabWX + i / 40, row = i % 40;
        W[p * kTabPlane + row * kTabRow + 32] = 0.f;
    }
    for (int i = threadIdx.x; i < (kTabPlanes - kTabWX) * 8 * 32; i += T) {
        const int p = kTabWX + (i >> 8), q = i & 255, row = q >> 5;
        W[p * kTabPlane + (row < 4 ? row : row + 32) * kTabRow + (q & 31)] = 0.f;
    }
    for (int i = threadIdx.x; i < 2 * 40; i += T) {  // pair planes: the zero column, then the zero rows
        const int p = i / 40, row = i % 40;
        W2[p * kTabPlane + row * kTabRow + 32] = make_float2(0.f, 0.f);
    }
    for (int i = threadIdx.x; i < 2 * 8 * 32; i += T) {
        const int p = i >> 8, q = i & 255, row = q >> 5;
        W2[p * kTabPlane + (row < 4 ? row : row + 32) * kTabRow + (q & 31)] = make_float2(0.f, 0.f);
    }
    // phase-1 samples of this thread: (lx, ly) = (s & 31, s >> 5), s = threadIdx.x + T q (block rows are
    // consecutive list entries: neighbouring lanes load neighbouring records)
    int li[NQ];
    F3 rec[NQ];
    uint64_t hs[NQ];  // splitmix64(seed ^ pixel) of each sample's path stream: its jitter is recomputed per round
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int s = threadIdx.x + T * q, lx = s & 31, ly = s >> 5;
        li[q] = (lx < sxb && ly < syb) ? P.pixel_map[(oy + ly) * P.width + (ox + lx)] : -1;
        hs[q] = splitmix64(P.seed ^ (uint64_t)((oy + ly) * P.width + (ox + lx)));
    }
    float sjx[NQ], sjy[NQ];  // the round's jitter, formed with the record fetch (during the previous round's sums)
    auto fetch = [&](int k) {
        const size_t rbase = (size_t)k * P.n_list;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (li[q] >= 0) rec[q] = load_rec(P.rec, rbase + li[q]);
            if (JIT) {  // NH_SPLAT_JITTER=stored (A/B)
                if (li[q] >= 0) {
                    const float2 jj = P.jit[rbase + li[q]];
                    sjx[q] = jj.x;
                    sjy[q] = jj.y;
                }
            } else {
                sample_jitter_h(hs[q], (uint64_t)(P.s0 + k), sjx[q], sjy[q]);
            }
        }
    };
    fetch(k0);
    // phase-2 strip of this thread: block-array column xt, rows yt0..yt0+5
    const int seg = threadIdx.x / 36, xt = threadIdx.x - seg * 36, yt0 = seg * SR;
    const int mcols = P.width + 4, mrows = P.height + 4;
    bool own[SR];
    float4 m[SR];
    float4 *const fb4 = reinterpret_cast<float4 *>(P.fb);
    // Pixels only this block covers (covering_blocks(..) == 1, the merge's test): inside the master and this
    // block's array, and not in the 4-pixel band a rendered neighbour's array also covers -- left / up neighbours
    // (full blocks) cover array columns / rows 0..3, right / down ones 32..35, diagonal ones the corner squares
    unsigned nbr = 0;  // rendered neighbours: bit (dy + 1) * 3 + (dx + 1)
    if (DIRECT) {
        const int nby = (P.height + 31) >> 5;
        for (int d = 0; d < 9; ++d) {
            const int bx2 = bx + d % 3 - 1, by2 = by + d / 3 - 1;
            if (d != 4 && bx2 >= 0 && bx2 < P.nbx && by2 >= 0 && by2 < nby && P.block_slot[by2 * P.nbx + bx2] >= 0)
                nbr |= 1u << d;
        }
    }
    const int cx = xt < 4 ? 0 : xt >= 32 ? 2 : 1;  // the column's band: left / none / right
    // PAIR: the seam pixels this (odd) block finishes: the partner's staged value of round 0 at pof[j] (-1: none), and
    // whether the partner comes first in spiral order (bit j of pfirst)
    int pof[SR];
    unsigned pfirst = 0;
    const size_t per_round = (size_t)P.n_blocks * (size_t)(36 * stage_pitch(36));
#pragma unroll
    for (int j = 0; j < SR; ++j) {
        own[j] = false;
        pof[j] = -1;
        m[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (PAIR && threadIdx.x < 36 * NS) {
            const int yt = yt0 + j, mx = ox + xt, my = oy + yt;
            if (mx < mcols && my < mrows && xt < sxb + 4 && yt < syb + 4) {
                int sl[4];
                const int nb = covering_blocks(P, mx, my, sl);
                if (nb == 1) {
                    own[j] = true;
                } else if (nb == 2) {
                    const int ps = sl[0] == slot ? sl[1] : sl[0], pb = P.blocks[ps];
                    const int pby = pb / P.nbx, pbx = pb - pby * P.nbx;
                    if (((bx + by) & 1) == 1 && ((pbx + pby) & 1) == 0) {  // a seam, and this block is its odd one
                        own[j] = true;
                        pof[j] = ps * (36 * stage_pitch(36)) + stage_off(36, 1, mx - pbx * 32, my - pby * 32);
                        if (sl[0] == ps) pfirst |= 1u << j;
                    }
                }
                if (own[j]) m[j] = fb4[(size_t)my * mcols + mx];
            }
        } else if (DIRECT && threadIdx.x < 36 * NS) {
            const int yt = yt0 + j, mx = ox + xt, my = oy + yt;  // block-array position -> master pixel
            const int cy = yt < 4 ? 0 : yt >= 32 ? 2 : 1;
            // neighbours whose array holds this pixel: the column band's, the row band's and their corner
            unsigned hold = 0;
            if (cx != 1) hold |= 1u << (4 + cx - 1);
            if (cy != 1) hold |= 1u << ((cy - 1 + 1) * 3 + 1);
            if (cx != 1 && cy != 1) hold |= 1u << (cy * 3 + cx);
            own[j] = mx < mcols && my < mrows && xt < sxb + 4 && yt < syb + 4 && !(nbr & hold);
            if (DIRECT && own[j]) m[j] = fb4[(size_t)my * mcols + mx];
        }
    }
#pragma unroll 1
    for (int k = k0; k < k1; ++k) {
        __syncthreads();  // the previous round's phase 2 is done with W (and tab / zero rows are in place)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int s = threadIdx.x + T * q, lx = s & 31, ly = s >> 5;
            float v[3] = {0.f, 0.f, 0.f}, wx[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, wy[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
            if (li[q] >= 0 && is_valid(rec[q])) {  // invalid samples drop with their weight
                const float spx = (float)(ox + lx) + sjx[q], spy = (float)(oy + ly) + sjy[q];
                const float px = spx - 0.5f - (float)(ox - 2), py = spy - 0.5f - (float)(oy - 2);
                const int x0 = max((int)ceilf(px - r), 0), y0 = max((int)ceilf(py - r), 0);
                const int x1 = min((int)floorf(px + r), 35), y1 = min((int)floorf(py + r), 35);
#pragma unroll
                for (int d = 0; d < 5; ++d) {
                    const int xc = lx + d, yc = ly + d;  // block-array column / row lx+2+(d-2)
                    if (xc >= x0 && xc <= x1) wx[d] = tab[(int)(fabsf((float)xc - px) * P.lookup)];
                    if (yc >= y0 && yc <= y1) wy[d] = tab[(int)(fabsf((float)yc - py) * P.lookup)];
                }
                v[0] = rec[q].x; v[1] = rec[q].y; v[2] = rec[q].z;
            }
            const int j = (ly + 4) * kTabRow + lx;
            W2[j] = make_float2(v[0], v[1]);
            W2[kTabPlane + j] = make_float2(v[2], 1.0f);
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                W[(kTabWX + d) * kTabPlane + j] = wx[d];
                W[(kTabWY + d) * kTabPlane + j] = wy[d];
            }
        }
        __syncthreads();
        if (k + 1 < k1) fetch(k + 1);  // in flight during phase 2
        float4 pv[SR];  // PAIR: the partner blocks' staged values of round k, in flight during phase 2
        if (PAIR)
#pragma unroll
            for (int j = 0; j < SR; ++j)
                if (pof[j] >= 0) pv[j] = P.staging[(size_t)k * per_round + pof[j]];
        if (threadIdx.x < 36 * NS) {
            sf2 rg[SR], bw[SR];
#pragma unroll
            for (int j = 0; j < SR; ++j) {
                rg[j] = sf2{0.f, 0.f};
                bw[j] = sf2{0.f, 0.f};
            }
            // (DIRECT keeps this loop rolled: unrolled, the hoisted loads and the master values spill)
#pragma unroll DIRECT ? 1 : 5
            for (int e = 0; e < 5; ++e) {  // sample column lx = xt - 4 + e: the pixel is its column offset 4 - e
                const int lx = xt - 4 + e;
                const float *base = W + yt0 * kTabRow + ((unsigned)lx < 32u ? lx : 32);
                const float2 *base2 = W2 + yt0 * kTabRow + ((unsigned)lx < 32u ? lx : 32);
#pragma unroll
                for (int i0 = 0; i0 < SR + 4; i0 += 2) {  // sample rows i0, i0 + 1 (ly = yt0 - 4 + i)
                    // each row weight of the two rows as one register pair (rows i0 and i0+1 of its plane): the
                    // products take it with the half selected in the instruction (pk_mul_lo / pk_mul_hi)
                    sf2 wyp[5];
#pragma unroll
                    for (int dy = 0; dy < 5; ++dy) {
                        const float *w = base + i0 * kTabRow + (kTabWY + dy) * kTabPlane;
                        wyp[dy] = sf2{w[0], i0 + 1 < SR + 4 ? w[kTabRow] : w[0]};  // (odd SR + 4: no row past)
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int i = i0 + h;
                        if (i >= SR + 4) continue;  // sample row ly = yt0 - 4 + i (plane row yt0 + i)
                        const float *w = base + i * kTabRow;
                        const float wx = w[(kTabWX + 4 - e) * kTabPlane];
                        const float2 prg = base2[i * kTabRow], pbw = base2[kTabPlane + i * kTabRow];
                        const sf2 vrg = sf2{prg.x, prg.y} * wx;
                        const sf2 vbw = sf2{pbw.x, pbw.y} * wx;
#pragma unroll
                        for (int dy = 0; dy < 5; ++dy) {  // row offset dy of the sample: strip row i - 4 + dy
                            const int j = i - 4 + dy;
                            if (j < 0 || j >= SR) continue;
                            rg[j] += h ? pk_mul_hi(vrg, wyp[dy]) : pk_mul_lo(vrg, wyp[dy]);
                            bw[j] += h ? pk_mul_hi(vbw, wyp[dy]) : pk_mul_lo(vbw, wyp[dy]);
                        }
                    }
                }
            }
            float4 *out = P.staging + ((size_t)k * P.n_blocks + slot) * (size_t)(36 * stage_pitch(36));
#pragma unroll
            for (int j = 0; j < SR; ++j) {
                if (PAIR && pof[j] >= 0 && ((pfirst >> j) & 1u)) {  // the partner's value first (spiral order)
                    m[j].x += pv[j].x;
                    m[j].y += pv[j].y;
                    m[j].z += pv[j].z;
                    m[j].w += pv[j].w;
                }
                if (DIRECT && own[j]) {  // round k of a pixel only this block covers: the master, in round order
                    m[j].x += rg[j].x;
                    m[j].y += rg[j].y;
                    m[j].z += bw[j].x;
                    m[j].w += bw[j].y;
                    if (PAIR && pof[j] >= 0 && !((pfirst >> j) & 1u)) {  // the partner's value second
                        m[j].x += pv[j].x;
                        m[j].y += pv[j].y;
                        m[j].z += pv[j].z;
                        m[j].w += pv[j].w;
                    }
                } else {
                    out[stage_off(36, 1, xt, yt0 + j)] = make_float4(rg[j].x, rg[j].y, bw[j].x, bw[j].y);
                }
            }
        }
    }
    if (DIRECT)
#pragma unroll
        for (int j = 0; j < SR; ++j)
            if (own[j]) fb4[(size_t)(oy + yt0 + j) * mcols + ox + xt] = m[j];
}

// PAIR: the pair splat's launch of the even blocks (1: their pixels classified as in the one-launch splat -- only they
// cover it, or staged) or of the odd blocks (2)
template <bool DIRECT, int ROUNDS = kTabRounds, bool JIT = false, bool PERSIST = false, int T = 256, int PAIR = 0>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(T / 128))) void nh_block_splat_tab_kernel(SplatLaunch P) {
    __shared__ float W[kTabPlanes * kTabPlane];
    __shared__ float tab[33];
    if (PAIR == 1) {
        tab_body<true, false, T, false>(P, W, tab, P.color_slots[blockIdx.x], 0, P.n_rounds);
        return;
    }
    if (PAIR == 2) {
        tab_body<true, false, T, true>(P, W, tab, P.color_slots[P.n_color0 + blockIdx.x], 0, P.n_rounds);
        return;
    }
    if (DIRECT) {
        tab_body<true, JIT, T>(P, W, tab, blockIdx.x, 0, P.n_rounds);
        return;
    }
    if (!PERSIST) {
        const int k0 = blockIdx.y * ROUNDS, k1 = min(k0 + ROUNDS, P.n_rounds);
        if (P.direct > 0 && blockIdx.y == 0) tab_body<true, JIT, T>(P, W, tab, blockIdx.x, k0, k1);
        else tab_body<false, JIT, T>(P, W, tab, blockIdx.x, k0, k1);
        return;
    }
    // PERSIST: a grid of P.persist workgroups walks the (block, round group) items, so the splat holds the LDS of
    // fewer CUs while the other pool's bounce kernels run beside it (A/B knob NH_SPLAT_WGS)
    const int groups = (P.n_rounds + ROUNDS - 1) / ROUNDS, n_items = P.n_blocks * groups;
#pragma unroll 1
    for (int v = blockIdx.x; v < n_items; v += gridDim.x) {
        const int slot = v % P.n_blocks, grp = v / P.n_blocks;
        __syncthreads();  // the previous item's sums are done with W before it is set up again
        const int k0 = grp * ROUNDS, k1 = min(k0 + ROUNDS, P.n_rounds);
        if (P.direct > 0 && grp == 0) tab_body<true, JIT, T>(P, W, tab, slot, k0, k1);
        else tab_body<false, JIT, T>(P, W, tab, slot, k0, k1);
    }
}

// Fused splat + merge for the 2-pixel border: one workgroup per 32x32 tile of MASTER pixels walks the chunk's
// rounds in order and adds every round's block values straight into the master pixels it owns, so no block
// ImageBlock is ever stored (the staged pair wrote and re-read 36x36 block arrays per (round, block)).
//
// Why the sums are the reference's. Master pixel (mx, my) receives, per round, ImageBlock::put(block) of every
// rendered block whose (32+4)^2 array covers it, in BlockGenerator spiral order (block.cpp:125-134); the value
// a block holds there is the sum, from +0 in getSampleIndices order (x outer, y inner), of
// (Color4f(v) * wx) * wy over the block's samples whose footprint covers the pixel (block.cpp:93-123). With a
// 2-pixel border and reach the footprint of the sample at image pixel (sx, sy) is exactly master columns
// sx..sx+4 and rows sy..sy+4 (never clipped by its block array), so master pixel (mx, my) sees the samples of
// the 5x5 window sx in [mx-4, mx], sy in [my-4, my]: those of its own block and, near a block edge, of the
// left / upper / upper-left neighbours. A tile owns master columns [32bx, 32bx+32) (the last tile: up to the
// master edge) and rows alike, so its windows reach samples [32bx-4, 32bx+32) x [32by-4, 32by+32): the 36x36
// sample region staged per round -- the quadrants cx < 4 / cy < 4 belong to the neighbour blocks. Per round
// the tile forms, for each of the (up to) four blocks in spiral order, that block's partial sum over the
// window (samples of other blocks masked to weight 0: (v * 0) * wy = +0 added to a sum that can never be -0
// changes nothing) and adds it to the master value held in registers; a block that does not cover the pixel
// contributes exactly +0. The weights are those of nh_block_splat_tab_kernel (each sample's five column and
// row weights, computed in its own block's coordinates), the products ((v * wx) * wy) the same floats.
//
// Work split: 512 threads, each owning a strip of 2 master rows of one column (its 2 float4 master values live
// in registers across the rounds). Strips whose windows hold only their own block's samples (columns 4..31,
// rows 4..31 of the tile: 392 of 512) run one unmasked pass in waves 0-5; the 120 strips at the tile's left and
// top edges run masked passes, one per neighbour block present, in waves 6-7; master pixels past the 32x32
// tile (the master border of the last block column / row) take a second, masked strip per thread, updated in
// place in the framebuffer.
constexpr int kTileThreads = 512;
constexpr int kRgn = 36, kRgnPx = kRgn * kRgn;   // sample region of a tile, row-major (cy * 36 + cx)
constexpr int kTV = 0, kTWX = 3, kTWY = 8, kTPlanes = 13;

// One block's partial sums for a 2-row strip (column c, rows r0, r0+1 of the tile; region window columns
// c..c+4, rows r0..r0+5). MASK: only the samples of region quadrant (xs, ys) count (xs = 0: cx < 4, the left
// block; ys = 0: cy < 4, the upper block) and samples outside the region (master border strips) are skipped.
template <bool MASK>
__device__ __forceinline__ void tile_strip_pass(const float *__restrict__ W, int c, int r0, int xs, int ys, sf2 rg[2],
                                                sf2 bw[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        rg[j] = sf2{0.f, 0.f};
        bw[j] = sf2{0.f, 0.f};
    }
    // the column loop stays rolled: unrolled, the scheduler hoists all 30 samples' loads and spills
#pragma unroll 1
    for (int e = 0; e < 5; ++e) {  // sample column cx = c + e, x-major as getSampleIndices; its weight index 4 - e
        const int cx = c + e;
        const bool xin = !MASK || ((cx < 4) == (xs == 0) && cx < kRgn);
        const int base = r0 * kRgn + cx;
        const float *Wx = W + (kTWX + 4 - e) * kRgnPx;
#pragma unroll
        for (int i = 0; i < 6; ++i) {  // sample row cy = r0 + i
            const int cy = r0 + i;
            const bool in = !MASK || (xin && (cy < 4) == (ys == 0) && cy < kRgn);
            const int a = MASK ? (in ? base + i * kRgn : 0) : base + i * kRgn;
            float wx = Wx[a];
            if (MASK) wx = in ? wx : 0.f;
            const sf2 vrg = sf2{W[(kTV + 0) * kRgnPx + a], W[(kTV + 1) * kRgnPx + a]} * wx;
            const sf2 vbw = sf2{W[(kTV + 2) * kRgnPx + a], 1.0f} * wx;
#pragma unroll
            for (int j = 0; j < 2; ++j) {  // strip row r0 + j: the sample's row weight index j + 4 - i
                const int dy = j + 4 - i;
                if (dy < 0 || dy > 4) continue;
                const float wy = W[(kTWY + dy) * kRgnPx + a];
                rg[j] += vrg * wy;
                bw[j] += vbw * wy;
            }
        }
    }
}

// One sweep of a 2-row strip's window (column c < 32, rows r0, r0+1): the running sums R (r, g) / B (b, w) take
// the contributions of sample rows i in [I0, I1), in getSampleIndices order (columns e outer). MASKY: per lane
// only the rows of one block -- upper (r0 + i < 4) when UPPER, own otherwise; a masked row adds (v*wx)*0 = +0
// to sums that start at +0 and are never -0, which changes nothing. XS: at column e == xsplit (per lane: the
// window's first own-block column) the sums so far are the left block's: they go to stash and restart from +0.
template <bool MASKY, bool UPPER, int I0, int I1, bool XS>
__device__ __forceinline__ void tile_sweep(const float *__restrict__ W, int c, int r0, int xsplit, float4 *stash,
                                           sf2 R[2], sf2 B[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) R[j] = B[j] = sf2{0.f, 0.f};
#pragma unroll 1
    for (int e = 0; e < 5; ++e) {  // sample column cx = c + e; its weight index 4 - e
        if (XS && e == xsplit) {   // few lanes (divergent)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                stash[j * 64] = make_float4(R[j].x, R[j].y, B[j].x, B[j].y);
                R[j] = B[j] = sf2{0.f, 0.f};
            }
        }
        const int a0 = r0 * kRgn + c + e;
        const float *Wx = W + (kTWX + 4 - e) * kRgnPx;
#pragma unroll
        for (int i = I0; i < I1; ++i) {  // sample row cy = r0 + i
            const int a = a0 + i * kRgn;
            const float wx = Wx[a];
            const sf2 vrg = sf2{W[(kTV + 0) * kRgnPx + a], W[(kTV + 1) * kRgnPx + a]} * wx;
            const sf2 vbw = sf2{W[(kTV + 2) * kRgnPx + a], 1.0f} * wx;
            const bool keep = !MASKY || ((r0 + i < 4) == UPPER);
#pragma unroll
            for (int j = 0; j < 2; ++j) {  // strip row r0 + j: the sample's row weight index j + 4 - i
                const int dy = j + 4 - i;
                if (dy < 0 || dy > 4) continue;
                float wy = W[(kTWY + dy) * kRgnPx + a];
                if (MASKY) wy = keep ? wy : 0.f;
                R[j] += vrg * wy;
                B[j] += vbw * wy;
            }
        }
    }
}

__global__ __launch_bounds__(kTileThreads) __attribute__((amdgpu_waves_per_eu(4))) void nh_tile_splat_kernel(SplatLaunch P) {
    __shared__ float W[kTPlanes * kRgnPx];
    __shared__ float tab[33];
    __shared__ float4 stash[2 * 6 * 64];  // waves 0 / 7: partials of the UL, U, L blocks [wave][quadrant][row][lane]
    const int tile = blockIdx.x;
    const int by = tile / P.nbx, bx = tile - by * P.nbx;
    const int nby = (P.height + 31) >> 5;
    // the blocks whose samples reach this tile, by region quadrant q = xs + 2 ys: 0 upper-left, 1 upper, 2 left,
    // 3 own; -1 = outside the image or not rendered by this context (its samples are absent: pixel_map -1)
    // (scalars, no arrays: a runtime-indexed array would live in scratch)
    unsigned present = 0;  // bit q: quadrant q's block is rendered
    int rk0, rk1, rk2, rk3;
    {
        auto rank_of = [&](int q) {
            const int qx = bx - 1 + (q & 1), qy = by - 1 + (q >> 1);
            if (qx < 0 || qy < 0 || P.block_slot[qy * P.nbx + qx] < 0) return 0x7fffffff;
            present |= 1u << q;
            return P.block_rank[qy * P.nbx + qx];
        };
        rk0 = rank_of(0); rk1 = rank_of(1); rk2 = rank_of(2); rk3 = rank_of(3);
    }
    if (!present) return;  // whole workgroup: no rendered block reaches the tile
    // position of each quadrant in spiral order (ties cannot occur between present blocks: ranks are distinct)
    auto pos_of = [&](int rk, int q) {
        return (rk0 < rk || (rk0 == rk && 0 < q)) + (rk1 < rk || (rk1 == rk && 1 < q)) +
               (rk2 < rk || (rk2 == rk && 2 < q)) + (rk3 < rk || (rk3 == rk && 3 < q));
    };
    const unsigned ordp = (0u << (2 * pos_of(rk0, 0))) | (1u << (2 * pos_of(rk1, 1))) | (2u << (2 * pos_of(rk2, 2))) |
                          (3u << (2 * pos_of(rk3, 3)));  // 2 bits per position: the quadrant added t-th
    const int mcols = P.width + 4, mrows = P.height + 4;
    const int ncols = bx == P.nbx - 1 ? mcols - 32 * bx : 32, nrows = by == nby - 1 ? mrows - 32 * by : 32;
    const float r = P.radius;
    if (threadIdx.x < 33) tab[threadIdx.x] = P.table[threadIdx.x];

    // phase-1 samples of this thread: region slot t = threadIdx.x + 512 q (x fastest: neighbouring lanes load
    // neighbouring pixels of one block row, consecutive list entries)
    int li[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int t = threadIdx.x + kTileThreads * q;
        const int sx = 32 * bx - 4 + t % kRgn, sy = 32 * by - 4 + t / kRgn;
        li[q] = (t < kRgnPx && sx >= 0 && sy >= 0 && sx < P.width && sy < P.height) ? P.pixel_map[sy * P.width + sx] : -1;
    }
    F3 rec[3];
    auto fetch = [&](int k) {  // every slot assigned (absent: zeros), so no earlier value stays live
        const size_t rbase = (size_t)k * P.n_list;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            rec[q] = f3(0.f, 0.f, 0.f);
            if (li[q] >= 0) rec[q] = load_rec(P.rec, rbase + li[q]);
        }
    };

    // phase-2 strips: u = 0 the tile's 32x32 pixels, u = 1 the master border beyond them (last block column / row)
    const int wave = threadIdx.x >> 6;
    int sc[2], sr[2];
    {
        const int l = threadIdx.x;
        int c, s;
        // waves 0-6: columns 4..31 (own block in x), 28 per strip row; wave 7: columns 0..3 (x-split)
        if (l < 448) { c = 4 + l % 28; s = l / 28; }
        else { c = (l - 448) & 3; s = (l - 448) >> 2; }
        sc[0] = c;
        sr[0] = 2 * s;
        const int nstr = (nrows + 1) >> 1, xc = max(ncols - 32, 0), n_right = xc * nstr;
        const int n_bottom = 32 * max(nstr - 16, 0);
        sc[1] = -1;
        sr[1] = 0;
        if (l < n_right) { sc[1] = 32 + l % xc; sr[1] = 2 * (l / xc); }
        else if (l < n_right + n_bottom) { sc[1] = (l - n_right) & 31; sr[1] = 2 * (16 + ((l - n_right) >> 5)); }
    }
    const bool ring = __any(sc[1] >= 0);  // any master-border strip in this wave
    // master values of the tile strip in registers across the rounds; a border strip (few, edge tiles only) is
    // updated in place in the framebuffer each round (same thread, program order)
    float4 m[2];
    float4 *const fb4 = reinterpret_cast<float4 *>(P.fb);
    auto fb_at = [&](int c, int row) -> float4 * { return fb4 + (size_t)(32 * by + row) * mcols + 32 * bx + c; };
#pragma unroll
    for (int j = 0; j < 2; ++j)
        m[j] = (sc[0] < ncols && sr[0] + j < nrows) ? *fb_at(sc[0], sr[0] + j) : make_float4(0.f, 0.f, 0.f, 0.f);

    fetch(0);
    for (int k = 0; k < P.n_rounds; ++k) {
        __syncthreads();  // the previous round's phase 2 is done with W (and tab is in place)
        auto stage = [&](const int q) {
            if (P.debug & 1) return;
            const int t = threadIdx.x + kTileThreads * q;
            const int cx = t % kRgn, cy = t / kRgn;
            const int sx = 32 * bx - 4 + cx, sy = 32 * by - 4 + cy;
            const int lx = sx & 31, ly = sy & 31, ox = sx - lx, oy = sy - ly;  // the sample's own block
            float v[3] = {0.f, 0.f, 0.f}, wx[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, wy[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
            if (li[q] >= 0 && is_valid(rec[q])) {  // invalid samples drop with their weight
                float jx, jy;
                sample_jitter_h(splitmix64(P.seed ^ (uint64_t)(sy * P.width + sx)), (uint64_t)(P.s0 + k), jx, jy);
                const float spx = (float)(ox + lx) + jx, spy = (float)(oy + ly) + jy;
                const float px = spx - 0.5f - (float)(ox - 2), py = spy - 0.5f - (float)(oy - 2);
                const int x0 = max((int)ceilf(px - r), 0), y0 = max((int)ceilf(py - r), 0);
                const int x1 = min((int)floorf(px + r), 35), y1 = min((int)floorf(py + r), 35);
#pragma unroll
                for (int d = 0; d < 5; ++d) {
                    const int xc = lx + d, yc = ly + d;  // block-array column / row = master column sx + d / row sy + d
                    if (xc >= x0 && xc <= x1) wx[d] = tab[(int)(fabsf((float)xc - px) * P.lookup)];
                    if (yc >= y0 && yc <= y1) wy[d] = tab[(int)(fabsf((float)yc - py) * P.lookup)];
                }
                v[0] = rec[q].x; v[1] = rec[q].y; v[2] = rec[q].z;
            }
            const int j = cy * kRgn + cx;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) W[(kTV + ch) * kRgnPx + j] = v[ch];
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                W[(kTWX + d) * kRgnPx + j] = wx[d];
                W[(kTWY + d) * kRgnPx + j] = wy[d];
            }
        };
        stage(0);
        stage(1);
        if (threadIdx.x + 2 * kTileThreads < kRgnPx) stage(2);
        __syncthreads();
        // next round's records in flight during phase 2 (waves with master-border strips fetch them after their
        // extra passes: the records' registers and the border passes' would not fit together)
        if (!ring && k + 1 < P.n_rounds && !(P.debug & 4)) fetch(k + 1);
        if (!(P.debug & 2)) {
            // Each block's partial sums, then master += each present block's partial in spiral order. Waves 1-6:
            // one unmasked sweep (own block only). Wave 0 (top rows) and wave 7 (left columns): a sweep of the upper
            // block's rows, then one of the own block's rows; wave 7's sweeps hand their left-block parts (UL, L) to
            // the stash at the column where the window enters the own block. Partials other than the own block's
            // wait in the LDS stash (registers).
            const int xsplit = (sc[0] < 4 && (present & 5u)) ? 4 - sc[0] : -1;  // left-block columns: e < 4 - c
            float4 *st = stash + (wave == 7 ? 6 * 64 : 0) + (threadIdx.x & 63);  // [quadrant UL, U, L][row][lane]
            sf2 R[2], B[2];
            if (wave == 7 || wave == 0) {
                if (wave == 7) tile_sweep<true, true, 0, 4, true>(W, sc[0], sr[0], xsplit, st, R, B);
                else tile_sweep<true, true, 0, 4, false>(W, sc[0], sr[0], -1, st, R, B);
#pragma unroll
                for (int j = 0; j < 2; ++j) st[(2 + j) * 64] = make_float4(R[j].x, R[j].y, B[j].x, B[j].y);
                if (wave == 7) tile_sweep<true, false, 0, 6, true>(W, sc[0], sr[0], xsplit, st + 4 * 64, R, B);
                else tile_sweep<true, false, 0, 6, false>(W, sc[0], sr[0], -1, st, R, B);
            } else {
                tile_sweep<false, false, 0, 6, false>(W, sc[0], sr[0], -1, st, R, B);
            }
#pragma unroll 1
            for (int t = 0; t < 4; ++t) {
                const int q = (int)(ordp >> (2 * t)) & 3;
                if (!((present >> q) & 1u)) continue;  // absent: its partial is +0
                if (q != 3 && wave != 7 && (q != 1 || wave != 0)) continue;  // no strip of this wave reaches it
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    float4 pv;
                    if (q == 3) pv = make_float4(R[j].x, R[j].y, B[j].x, B[j].y);
                    else if (q == 1) pv = st[(2 + j) * 64];
                    else pv = xsplit > 0 ? st[((q == 0 ? 0 : 4) + j) * 64] : make_float4(0.f, 0.f, 0.f, 0.f);
                    m[j].x += pv.x;
                    m[j].y += pv.y;
                    m[j].z += pv.z;
                    m[j].w += pv.w;
                }
            }
        }
        if (ring && !(P.debug & 8)) {  // master border strips of the last block column / row, in place in the framebuffer
#pragma unroll 1
            for (int t = 0; t < 4; ++t) {
                const int q = (int)(ordp >> (2 * t)) & 3;
                if (!((present >> q) & 1u)) continue;
                const int xs = q & 1, ys = q >> 1;
                if ((xs == 0 && !__any(sc[1] >= 0 && sc[1] < 4)) || (ys == 0 && !__any(sc[1] >= 0 && sr[1] < 4))) continue;
                if (sc[1] < 0) continue;
                sf2 rg[2], bw[2];
                tile_strip_pass<true>(W, sc[1], sr[1], xs, ys, rg, bw);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (sc[1] >= ncols || sr[1] + j >= nrows) continue;
                    float4 *mp = fb_at(sc[1], sr[1] + j);
                    float4 mv = *mp;
                    mv.x += rg[j].x;
                    mv.y += rg[j].y;
                    mv.z += bw[j].x;
                    mv.w += bw[j].y;
                    *mp = mv;
                }
            }
            if (k + 1 < P.n_rounds) fetch(k + 1);
        }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
        if (sc[0] < ncols && sr[0] + j < nrows) *fb_at(sc[0], sr[0] + j) = m[j];
}

// ImageBlock::put(ImageBlock&) into the master (src/utils/block.cpp:125-134): per master
// pixel, per round, the overlapping rendered blocks in BlockGenerator spiral order.
__global__ __launch_bounds__(256) void nh_merge_kernel(SplatLaunch P) {
    const int mcols = P.width + 2 * P.border, mrows = P.height + 2 * P.border;
    const int mx = blockIdx.x * 16 + (threadIdx.x & 15), my = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (mx >= mcols || my >= mrows) return;
    const int cols = 32 + 2 * P.border, pitch = stage_pitch(cols);
    int slot[4];
    const int nb = covering_blocks(P, mx, my, slot);
    // P.direct: rounds the tab splat already added to the pixels one block covers (all of them, or its first
    // workgroup's)
    if (nb == 0 || (nb == 1 && P.direct >= P.n_rounds)) return;
    int off[4];
    for (int q = 0; q < nb; ++q) {
        const int bid = P.blocks[slot[q]];
        const int by = bid / P.nbx, bx = bid - by * P.nbx;
        off[q] = stage_off(cols, P.band, mx - bx * 32, my - by * 32);
    }
    float4 *mp = reinterpret_cast<float4 *>(P.fb) + (size_t)my * mcols + mx;
    float4 m = *mp;
    const size_t blk = (size_t)cols * pitch, per_round = (size_t)P.n_blocks * blk;
    int k = nb == 1 ? P.direct : 0;
    if (nb == 1) {  // one covering block (most pixels): eight rounds' loads in flight, added in round order
        const float4 *src = P.staging + (size_t)slot[0] * blk + off[0];
        for (; k + 8 <= P.n_rounds; k += 8) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = src[(size_t)(k + j) * per_round];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                m.x += v[j].x;
                m.y += v[j].y;
                m.z += v[j].z;
                m.w += v[j].w;
            }
        }
    }
    // pixels of the 4-pixel bands (2-4 covering blocks): four rounds' loads of every block in flight, then added in
    // the same order as the loop below (rounds in order, blocks in spiral order within a round)
#ifndef NH_AB_MERGE_SERIAL
    for (; nb > 1 && k + 4 <= P.n_rounds; k += 4) {
        float4 v[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q < nb) v[j][q] = P.staging[(size_t)(k + j) * per_round + (size_t)slot[q] * blk + off[q]];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q < nb) {
                    m.x += v[j][q].x;
                    m.y += v[j][q].y;
                    m.z += v[j][q].z;
                    m.w += v[j][q].w;
                }
    }
#endif
    for (; k < P.n_rounds; ++k) {
        const float4 *base = P.staging + (size_t)k * per_round;
        for (int q = 0; q < nb; ++q) {
            const float4 v = base[(size_t)slot[q] * blk + off[q]];
            m.x += v.x;
            m.y += v.y;
            m.z += v.z;
            m.w += v.w;
        }
    }
    *mp = m;
}

// The pair splat's last step: master pixels of the interior 4x4 corner squares whose covering blocks are not one
// side-by-side pair (three or four blocks, or two diagonal ones: every one of them staged its value), summed like
// nh_merge_kernel's band pixels -- rounds in order, blocks in spiral order within a round. 4 corners per 64-thread
// workgroup (a few hundred workgroups spread over the CUs), one pixel per thread, eight rounds' loads in flight.
__global__ __launch_bounds__(64) void nh_corner_merge_kernel(SplatLaunch P) {
    const int nby = (P.height + 31) >> 5, ncx = P.nbx - 1;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 4);
    if (c >= ncx * (nby - 1)) return;
    const int cy = c / ncx + 1, cx = c - (cy - 1) * ncx + 1;
    const int mx = 32 * cx + (threadIdx.x & 3), my = 32 * cy + ((threadIdx.x >> 2) & 3);
    int slot[4];
    const int nb = covering_blocks(P, mx, my, slot);
    if (nb < 2) return;
    int off[4], par = 0;
    for (int q = 0; q < nb; ++q) {
        const int bid = P.blocks[slot[q]];
        const int by = bid / P.nbx, bx = bid - by * P.nbx;
        off[q] = slot[q] * (36 * stage_pitch(36)) + stage_off(36, 1, mx - bx * 32, my - by * 32);
        par += (bx + by) & 1;
    }
    if (nb == 2 && par == 1) return;  // a side-by-side pair: the odd block's workgroup finished it
    const int mcols = P.width + 4;
    float4 *mp = reinterpret_cast<float4 *>(P.fb) + (size_t)my * mcols + mx;
    float4 m = *mp;
    const size_t per_round = (size_t)P.n_blocks * (size_t)(36 * stage_pitch(36));
    int k = 0;
    for (; k + 8 <= P.n_rounds; k += 8) {
        float4 v[8][4];
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q < nb) v[j][q] = P.staging[(size_t)(k + j) * per_round + off[q]];
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q < nb) {
                    m.x += v[j][q].x;
                    m.y += v[j][q].y;
                    m.z += v[j][q].z;
                    m.w += v[j][q].w;
                }
    }
    for (; k < P.n_rounds; ++k)
        for (int q = 0; q < nb; ++q) {
            const float4 v = P.staging[(size_t)k * per_round + off[q]];
            m.x += v.x;
            m.y += v.y;
            m.z += v.z;
            m.w += v.w;
        }
    *mp = m;
}

// invalid-sample count (ImageBlock::put drops, block.cpp:94-99)
__global__ __launch_bounds__(256) void nh_count_invalid_kernel(const float *rec, size_t n, unsigned long long *out) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long c = 0;
    if (i < n) c = is_valid(load_rec(rec, i)) ? 0 : 1;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(stat_shard(out) + 4, c);
}

}  // namespace

namespace nh {

// A/B knobs, read per launch (one per chunk) so a process can switch them: NH_SPLAT_FUSED=1 -> the fused tile
// splat (below); NH_SPLAT_TAB=0 -> the staged pair's column-strip splat, NH_SPLAT_STRIP=0 -> one pixel per thread
static bool splat_knob(const char *name) {
    const char *e = std::getenv(name);
    return !e || e[0] != '0';
}

// The fused tile splat is bit-identical but slower than the staged pair (0.485 vs 0.275 + 0.100 ms per C2 chunk,
// rocprofv3, one pool): its 16 rounds per tile are a serial chain of record fetches (0.245 ms with both phases
// skipped) and the left / top edge strips lengthen each round. Opt-in: NH_SPLAT_FUSED=1.
bool splat_uses_staging(int border, int reach) {
    const char *e = std::getenv("NH_SPLAT_FUSED");
    return !(e && e[0] == '1' && border == 2 && reach == 2);
}

void launch_splat(const SplatLaunch &P, hipStream_t st) {
    const bool tabulated = splat_knob("NH_SPLAT_TAB"), strip = splat_knob("NH_SPLAT_STRIP");
    if (!P.staged) {  // splat + merge in one pass, no block staging
        const int n_tiles = P.nbx * ((P.height + 31) / 32);
        SplatLaunch Q = P;
        if (const char *e = std::getenv("NH_SPLAT_DEBUG")) Q.debug = std::atoi(e);
        static bool told = false;
        if (!told && std::getenv("NH_SPLAT_OCC")) {
            told = true;
            int a = 0, b = 0;
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, nh_tile_splat_kernel, kTileThreads, 0);
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, nh_block_splat_tab_kernel<false>, 256, 0);
            std::fprintf(stderr, "[nh] workgroups per CU: tile splat %d, tab splat %d\n", a, b);
        }
        hipLaunchKernelGGL(nh_tile_splat_kernel, dim3(n_tiles), dim3(kTileThreads), 0, st, Q);
        return;
    }
    SplatLaunch Q = P;
    Q.direct = 0;
    Q.band = tabulated && P.border == 2 && P.reach == 2 ? 1 : 0;  // the layout the tab kernel writes
    if (tabulated && P.border == 2 && P.reach == 2) {
        // one workgroup per block takes all the chunk's rounds of the pixels only that block covers (default since
        // round 5: with 512-thread workgroups it beats the lead split on C1 / C2 / C4, and stages only the 4-pixel
        // bands: 0.54 vs 0.77 GB per C2 chunk); NH_SPLAT_DIRECT=0 restores the per-round-group workgroups
        const bool all_direct = splat_knob("NH_SPLAT_DIRECT");
        const char *rv = std::getenv("NH_SPLAT_ROUNDS");  // rounds per workgroup: 1, 2, 4 or 8 (default)
        int tr = rv ? std::atoi(rv) : kTabRounds;
        if (tr != 1 && tr != 2 && tr != 4 && tr != 8) tr = kTabRounds;  // 0 / garbage: the default (no 0 divisor)
        if (P.jit) tr = 8;  // stored jitter (A/B): the default grouping only
        const char *ld = std::getenv("NH_SPLAT_LEAD");  // the first workgroup's rounds straight into the master
        const bool lead = !(ld && ld[0] == '0');
        Q.direct = all_direct ? P.n_rounds : lead ? std::min(tr, P.n_rounds) : 0;
        dim3 g(P.n_blocks, (P.n_rounds + tr - 1) / tr);
        const char *pw = std::getenv("NH_SPLAT_WGS");  // persistent splat grid (A/B): workgroups, 0 = one per item
        Q.persist = pw ? std::max(0, std::atoi(pw)) : 0;
        if (all_direct || tr != 8 || P.jit) Q.persist = 0;  // the persistent grid: default grouping only
        if (Q.persist) g = dim3(std::min<unsigned>((unsigned)Q.persist, g.x * g.y), 1);
        const bool t512 = splat_knob("NH_SPLAT_T512");  // 512-thread workgroups, 3-row strips (0: 256, 6-row)
        if (t512 && all_direct && !P.jit && splat_knob("NH_SPLAT_PAIR")) {
            // the pair splat: the even blocks, then the odd ones (which finish the seams), then the corner squares
            if (P.n_color0 > 0)
                hipLaunchKernelGGL((nh_block_splat_tab_kernel<true, 8, false, false, 512, 1>), dim3(P.n_color0), dim3(512), 0, st, Q);
            if (P.n_blocks > P.n_color0)
                hipLaunchKernelGGL((nh_block_splat_tab_kernel<true, 8, false, false, 512, 2>), dim3(P.n_blocks - P.n_color0),
                                   dim3(512), 0, st, Q);
            const int n_corners = (P.nbx - 1) * ((P.height + 31) / 32 - 1);
            if (n_corners > 0) hipLaunchKernelGGL(nh_corner_merge_kernel, dim3((n_corners + 3) / 4), dim3(64), 0, st, Q);
            return;
        }
        if (P.jit) {
            if (all_direct) hipLaunchKernelGGL((nh_block_splat_tab_kernel<true, 8, true>), dim3(P.n_blocks, 1), dim3(256), 0, st, Q);
            else hipLaunchKernelGGL((nh_block_splat_tab_kernel<false, 8, true>), g, dim3(256), 0, st, Q);
        }
        else if (t512 && all_direct)
            hipLaunchKernelGGL((nh_block_splat_tab_kernel<true, 8, false, false, 512>), dim3(P.n_blocks, 1), dim3(512), 0, st, Q);
        else if (t512 && tr == 8 && !Q.persist)
            hipLaunchKernelGGL((nh_block_splat_tab_kernel<false, 8, false, false, 512>), g, dim3(512), 0, st, Q);
        else if (all_direct) hipLaunchKernelGGL((nh_block_splat_tab_kernel<true>), dim3(P.n_blocks, 1), dim3(256), 0, st, Q);
        else if (tr == 1) hipLaunchKernelGGL((nh_block_splat_tab_kernel<false, 1>), g, dim3(256), 0, st, Q);
        else if (tr == 2) hipLaunchKernelGGL((nh_block_splat_tab_kernel<false, 2>), g, dim3(256), 0, st, Q);
        else if (tr == 4) hipLaunchKernelGGL((nh_block_splat_tab_kernel<false, 4>), g, dim3(256), 0, st, Q);
        else if (Q.persist) hipLaunchKernelGGL((nh_block_splat_tab_kernel<false, 8, false, true>), g, dim3(256), 0, st, Q);
        else hipLaunchKernelGGL((nh_block_splat_tab_kernel<false, 8>), g, dim3(256), 0, st, Q);
    }
    else if (strip) hipLaunchKernelGGL(nh_block_splat_strip_kernel, dim3(P.n_blocks, P.n_rounds), dim3(256), 0, st, P);
    else hipLaunchKernelGGL(nh_block_splat_kernel, dim3(P.n_blocks, P.n_rounds), dim3(256), 0, st, P);
    const int mcols = P.width + 2 * P.border, mrows = P.height + 2 * P.border;
    dim3 grid((mcols + 15) / 16, (mrows + 15) / 16);
    hipLaunchKernelGGL(nh_merge_kernel, grid, dim3(256), 0, st, Q);
}

void launch_count_invalid(const float *rec, size_t n, unsigned long long *out, hipStream_t st) {
    if (n == 0) return;
    dim3 grid((unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(nh_count_invalid_kernel, grid, dim3(256), 0, st, rec, n, out);
}

}  // namespace nh
