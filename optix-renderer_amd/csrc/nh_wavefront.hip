// Wavefront path_mis / path_mats for gfx950: the same per-path semantics as the megakernel
// (nh_kernels.hip li_path_mis, i.e. src/integrators/path_mis.cpp:16-150), split into
// kernels over SoA path state in HBM so each stage runs at its own occupancy:
//
//   (bounce 0)   renderBlock's per-pixel prologue (render.cpp:441-447: seeding, jitter, camera
//                ray) is evaluated in place by the first extend and shade kernels
//   wf_extend    closest-hit traversal of every live path's ray (the BSDF-sampled ray is the
//                MIS probe and the next bounce at once, path_mis.cpp:117/:146) -- the
//                BVH-traversal kernel whose roofline bench.py reports
//   wf_shadow    any-hit traversal of the shadow rays queued by the previous shade (:89)
//   wf_shade     finishes the previous bounce (an unoccluded shadow ray adds the light term that
//                bounce computed and sets w_ems; probe hit -> w_mats; discrete override,
//                :103-146), then shades the new hit (emitter term, Russian roulette, NEE sample,
//                BSDF sample, this bounce's MIS-weighted light term and t *= bsdf weight)
//
// Path state is double-buffered and kept DENSE: wf_shade reads live path i of buffer A and
// writes each surviving path's whole state to the next free slot of buffer B (ranks from wave
// ballots + LDS atomics, one device-scope atomic per workgroup and queue). Every kernel then
// streams its arrays coalesced, with no index indirection. Shadow rays are written densely to
// their own queue together with the slot of their path in B; wf_shadow stores the any-hit result
// into B's occlusion byte for that slot.
//
// Queues and buffers are split into kQueueShards segments of seg_cap entries: workgroup b
// appends to segment b % 8 (its XCD, as workgroups are dealt round-robin over the XCDs), so no
// counter takes device-scope atomics from two XCDs (one shared counter serialised the kernel).
//
// Each path's random numbers come from its own pcg32 stream in the reference's draw order,
// so the wavefront and megakernel renders are identical.
#include "nh_internal.h"
#include "nh_shade.h"

#include <algorithm>
#include <cstdlib>

using namespace nhd;

namespace {

// Path flags. Stored (6 bits, packed with the path id into ray_d.w):
//   F_DISCRETE  the BSDF sample of the last bounce was discrete (path_mis.cpp:136-140)
//   F_NEE       the last bounce queued a shadow ray; its contribution waits in pend
//   F_ZERO_COL  the last BSDF sample's weight was zero (isZero, path_mis.cpp:115): no MIS probe
//   F_ZNAN      (w_ems * t) * 0 of an occluded light sample would not be 0 (non-finite t)
//   bits 4-5    path_mats bounce counter
// F_FIRST (bounce 0, paths straight from the camera) lives in registers only.
enum : int { F_DISCRETE = 1, F_NEE = 2, F_ZERO_COL = 4, F_ZNAN = 8, F_FIRST = 64 };
constexpr int kPidBits = 26;  // path id bits of ray_d.w (nh_api.hip caps a chunk at 2^26 paths)

// rank of this lane among the wave's lanes with pred set, offset by the wave's reservation in
// *counter (an LDS counter here)
__device__ __forceinline__ int wave_append(unsigned *counter, bool pred) {
    const unsigned long long mask = __ballot(pred);
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)mask) - 1;
    unsigned base = 0;
    if (mask != 0ull && lane == leader) base = atomicAdd(counter, (unsigned)__popcll(mask));
    base = __shfl(base, leader < 0 ? 0 : leader, 64);
    return (int)base + __popcll(mask & ((1ull << lane) - 1ull));
}

__device__ __forceinline__ F3 xyz(float4 v) { return f3(v.x, v.y, v.z); }

__device__ __forceinline__ int queue_slot(const int *pre, int seg_cap, int q) {
    int slot = q;
#pragma unroll
    for (int s = 1; s < kQueueShards; ++s)
        if (q >= pre[s]) slot = s * seg_cap + (q - pre[s]);
    return slot;
}

// dense prefix over the 8 shard counts of one count group
struct QView {
    int n;
    int pre[kQueueShards + 1];
};
__device__ __forceinline__ QView queue_view(const unsigned *group) {
    QView v;
    v.pre[0] = 0;
#pragma unroll
    for (int s = 0; s < kQueueShards; ++s) v.pre[s + 1] = v.pre[s] + (int)group[s * kCountStride];
    v.n = v.pre[kQueueShards];
    return v;
}

__device__ __forceinline__ void flush_trav_stats(unsigned long long *dst, unsigned long long queries,
                                                 const TravStats &st) {
    unsigned long long v[4] = {queries, st.nodes, st.boxes, st.prims};
    for (int j = 0; j < 4; ++j) {
        unsigned long long x = v[j];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(&dst[j], x);
    }
}

// the state one shade step produces for a surviving path
struct PState {
    float4 ro, rd;   // next ray (origin, mint), (direction, maxt)
    float4 li, thr;  // (Li, w_mats), (throughput, w_ems if the shadow ray is occluded)
    float4 pe;       // queued NEE: (w_ems * t * Li_ems, w_ems if the shadow ray is unoccluded)
    float pdfmat;    // pdf of the BSDF sample (MIS weight of an emitter the probe may hit)
    uint64_t rng;
    int flags, pid;
};

// HBM layout of a path (WfBuf): mint of a bounce ray is always Epsilon and maxt +inf, or -inf for
// the zero direction Diffuse::sample leaves behind, so those two words carry pdfmat and
// (flags << kPidBits | pid) instead.
__device__ __forceinline__ void store_state(const WfBuf &B, int s, const PState &o) {
    B.ray_o[s] = make_float4(o.ro.x, o.ro.y, o.ro.z, o.pdfmat);
    B.ray_d[s] = make_float4(o.rd.x, o.rd.y, o.rd.z, __int_as_float((int)(((unsigned)o.flags << kPidBits) | (unsigned)o.pid)));
    B.li[s] = o.li;
    B.thr[s] = o.thr;
    if (o.flags & F_NEE) B.pend[s] = o.pe;
    B.rng[s] = o.rng;
}

// the traced ray of a stored path state
__device__ __forceinline__ void unpack_ray(float4 &ro, float4 &rd) {
    ro.w = kEps;
    rd.w = (rd.x == 0 && rd.y == 0 && rd.z == 0) ? -INFINITY : INFINITY;
}

}  // namespace

// renderBlock's per-pixel prologue for path p = round * n_list + entry (render.cpp:441-447): seeding,
// pixel jitter, the unused aperture sample, PerspectiveCamera::sampleRay (perspective.cpp:97-141).
// Bounce 0 evaluates it in place -- in the extend kernel for the ray, again in the shade kernel
// for its state -- instead of a generate kernel writing ~100 B per path that both read back.
template <bool DOF = true>
__device__ __forceinline__ void camera_sample(const DScene &S, const WfLaunch &L, int p, Rng &rng, float4 &ro,
                                              float4 &rd, float &jx, float &jy) {
    const int k = p / L.n_list, i = p - k * L.n_list;
    const int pix = L.pixel_list[i];
    const int py = pix / S.width, px = pix - py * S.width;
    rng = path_rng(L.seed, (uint64_t)pix, (uint64_t)(L.s0 + k));
    jx = rng.next1d();
    jy = rng.next1d();
    rng.next1d();  // apertureSample (render.cpp:443): unused (the lens sample comes from the camera's own sampler)
    rng.next1d();
    F3 o, d;
    float mint, maxt;
    camera_ray<DOF>(S, (float)px + jx, (float)py + jy, o, d, mint, maxt, L.s0 + k, pix);
    ro = make_float4(o.x, o.y, o.z, mint);
    rd = make_float4(d.x, d.y, d.z, maxt);
}

// the ray of queue entry q / slot s of this bounce (DOF: camera rays may be thin-lens ones, camera_ray)
template <bool DOF = true>
__device__ __forceinline__ void load_ray(const DScene &S, const WfLaunch &L, const WfBuf &B, int q, int s, float4 &ro,
                                         float4 &rd) {
    if (L.first) {  // dense queue: slot = path id
        Rng rng;
        float jx, jy;
        camera_sample<DOF>(S, L, q, rng, ro, rd, jx, jy);
    } else {
        ro = B.ray_o[s];
        rd = B.ray_d[s];
        unpack_ray(ro, rd);
    }
}


// float4 offset of the pair table in the dynamic LDS of a small scene (after nodes, primitives, leaves)
__host__ __device__ __forceinline__ int small_pairs_offset_f4(const WfLaunch &L) {
    return L.small_nodes + L.small_prims + (L.small_leaves + 1) / 2;
}

// Stage a small BVH (nodes, leaf table, primitives) into dynamic LDS and return a traversal view
// of the copy. Instantiated only for SMALL kernels, so every traversal pointer derives from the
// __shared__ array: the compiler emits ds_read, not flat loads. Called by the whole workgroup.
// PAIRS: also the pair-interleaved copy of the primitive records (Traversal::ppairs, kPairF4 float4 per
// record, after the leaf table; record n_prims = zeros).
template <bool PAIRS = false>
__device__ __forceinline__ Traversal stage_small_scene(const Traversal &tv, const WfLaunch &L, float4 *lds) {
    float4 *nodes = lds, *prims = lds + L.small_nodes;
    int2 *leaves = reinterpret_cast<int2 *>(prims + L.small_prims);
    for (int i = threadIdx.x; i < L.small_nodes; i += blockDim.x) nodes[i] = tv.nodes[i];
    for (int i = threadIdx.x; i < L.small_prims; i += blockDim.x) prims[i] = tv.prims[i];
    for (int i = threadIdx.x; i < L.small_leaves; i += blockDim.x) leaves[i] = tv.leaves[i];
    Traversal t;
    t.nodes = nodes;
    t.prims = prims;
    t.leaves = leaves;
    t.ppairs = nullptr;
    t.frames = nullptr;
    t.wnodes = tv.wnodes;
    t.n_top = 0;
    if constexpr (PAIRS) {
        float4 *pairs = lds + small_pairs_offset_f4(L);
        const int n = L.small_prims / 3;
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            const float4 a = tv.prims[3 * k], b = tv.prims[3 * k + 1], c = tv.prims[3 * k + 2];
            const bool nx = k + 1 < n;
            const float4 a1 = nx ? tv.prims[3 * k + 3] : z, b1 = nx ? tv.prims[3 * k + 4] : z,
                         c1 = nx ? tv.prims[3 * k + 5] : z;
            float4 *q = pairs + (size_t)kPairF4 * k;
            // Moller-Trumbore's edges (mesh.cpp:105-106), subtracted once here instead of in every test
            q[0] = make_float4(a.x, a1.x, a.y, a1.y);
            q[1] = make_float4(a.z, a1.z, a.w, a1.w);
            q[2] = make_float4(b.x - a.x, b1.x - a1.x, b.y - a.y, b1.y - a1.y);
            q[3] = make_float4(b.z - a.z, b1.z - a1.z, c.x - a.x, c1.x - a1.x);
            q[4] = make_float4(c.y - a.y, c1.y - a1.y, c.z - a.z, c1.z - a1.z);
            q[5] = make_float4(c.w, c1.w, 0.f, 0.f);
        }
        t.ppairs = pairs;
        if (L.small_frames) {  // flat triangles' shading frames (hit_info), from the records just read
            float4 *fr = pairs + (size_t)kPairF4 * n;
            for (int k = threadIdx.x; k < n; k += blockDim.x) {
                const float4 a = tv.prims[3 * k], b = tv.prims[3 * k + 1], c = tv.prims[3 * k + 2];
                Frame f{};
                if (prim_is_tri(c)) {
                    const F3 p0 = f3(a.x, a.y, a.z);
                    f = frame_from_n(normalized(cross(sub(f3(b.x, b.y, b.z), p0), sub(f3(c.x, c.y, c.z), p0))));
                }
                fr[3 * k] = make_float4(f.s.x, f.s.y, f.s.z, 0.f);
                fr[3 * k + 1] = make_float4(f.t.x, f.t.y, f.t.z, 0.f);
                fr[3 * k + 2] = make_float4(f.n.x, f.n.y, f.n.z, 0.f);
            }
            t.frames = fr;
        }
    }
    __syncthreads();
    return t;
}

// float4 count of the dynamic LDS of the fused kernels: BVH + pair records + the flat triangles' frames
__host__ __device__ __forceinline__ int rr_lds_f4(const WfLaunch &L) {
    return small_pairs_offset_f4(L) + kPairF4 * (L.small_prims / 3) + (L.small_frames ? 3 * (L.small_prims / 3) : 0);
}

template <bool SMALL>
__device__ __forceinline__ Traversal traversal_view(const Traversal &tv, const WfLaunch &L, float4 *lds) {
    if constexpr (SMALL) return stage_small_scene(tv, L, lds);
    else return tv;
}

// Grid-stride over the live queue (its length is read from the device count slot).
template <int DEPTH, bool ORDERED, bool STATS, bool SMALL>
__global__ __launch_bounds__(128) void wf_extend(const DScene *__restrict__ Sp, Traversal tv_g, WfLaunch L) {
    __shared__ uint32_t stk[DEPTH * 128];
    extern __shared__ float4 lds_scene[];
    const DScene &S = *Sp;
    const Traversal tv = traversal_view<SMALL>(tv_g, L, lds_scene);
    const QView qv = queue_view(L.cnt_in);
    const WfBuf &B = L.st.buf[L.in_q];
    TravStats st{0, 0, 0};
    unsigned long long queries = 0;
    for (int q = blockIdx.x * 128 + threadIdx.x; q < qv.n; q += gridDim.x * 128) {
        const int s = queue_slot(qv.pre, L.seg_cap, q);
        float4 ro, rd;
        load_ray(S, L, B, q, s, ro, rd);
        Hit h;
        // a zero BSDF direction (maxt = -inf) misses every primitive: not traversed, as in the megakernel
        const bool live = rd.w >= ro.w;
        queries += live ? 1 : 0;
        const bool found = live && trace<DEPTH, ORDERED, false, STATS>(tv, S, xyz(ro), xyz(rd), ro.w, rd.w, h,
                                                                       stk + threadIdx.x, 128, st);
        B.hit[s] = make_float4(h.t, h.u, h.v, __int_as_float(found ? h.k : -1));
    }
    if (STATS) flush_trav_stats(stat_shard(L.counters), queries, st);
}

template <int DEPTH, bool ORDERED, bool STATS, bool SMALL>
__global__ __launch_bounds__(128) void wf_shadow(const DScene *__restrict__ Sp, Traversal tv_g, WfLaunch L) {
    __shared__ uint32_t stk[DEPTH * 128];
    extern __shared__ float4 lds_scene[];
    const DScene &S = *Sp;
    const Traversal tv = traversal_view<SMALL>(tv_g, L, lds_scene);
    const QView qv = queue_view(L.cnt_in + kCountGroup);
    TravStats st{0, 0, 0};
    unsigned long long queries = 0;
    for (int q = blockIdx.x * 128 + threadIdx.x; q < qv.n; q += gridDim.x * 128) {
        const int s = queue_slot(qv.pre, L.seg_cap, q);
        const float4 so = L.st.sh_o[s], sd = L.st.sh_d[s];
        Hit h;
        ++queries;
        const bool occ = trace<DEPTH, ORDERED, true, STATS>(tv, S, xyz(so), xyz(sd), so.w, sd.w, h,
                                                            stk + threadIdx.x, 128, st);
        L.st.buf[L.in_q].occl[L.st.sh_slot[s]] = occ ? 1 : 0;
    }
    if (STATS) flush_trav_stats(stat_shard(L.counters) + 8, queries, st);
}

// Persistent traversal: a fixed grid of waves pulls rays in batches of kFetchBatch from eight
// fetch segments (segment f = [f*n/8, (f+1)*n/8) of the dense queue index; a wave starts on the
// segment of its XCD, blockIdx % 8, and moves on when it runs dry), and refills every lane whose
// traversal finished before the next Tracer step. A wave thus stays busy until the pool is empty
// instead of waiting for its slowest ray (the 64-lane divergence that made one wave execute
// ~10x the instructions of an average ray on the 1M-triangle scene).
#ifndef NH_FETCH_BATCH
#define NH_FETCH_BATCH 128
#endif
constexpr int kFetchBatch = NH_FETCH_BATCH;
constexpr int kTraceBlocksMax = 1 << 20;
#ifndef NH_RING_ENTRIES
#define NH_RING_ENTRIES 16
#endif
constexpr int kRingEntries = NH_RING_ENTRIES;
#ifndef NH_TOP_NODES
#define NH_TOP_NODES 16
#endif
constexpr int kTopNodes = NH_TOP_NODES;  // wide nodes per LDS copy of the top of the tree (kTopNodes * 128 B)
//
// WIDE: 0 the binary tree (Tracer), 4 / 8 the 4- / 8-wide collapse of the tree (Tracer4 / Tracer8), LDS window of 8
// (ref, distance) pairs per lane.
template <int WIDE>
struct PtStack {
    using type = RingStack2<kRingEntries / 2>;
    static __device__ __forceinline__ type make(uint32_t *lds, const WfLaunch &L) {
        type s;
        s.lds_ref = reinterpret_cast<int *>(lds) + threadIdx.x;
        s.lds_near = reinterpret_cast<float *>(lds + kRingEntries / 2 * 128) + threadIdx.x;
        s.stride = 128;
        // kPersistentBlocks * 128 lanes x spill_depth / 2 entries (every WIDE grid is capped at kPersistentBlocks)
        s.glob = reinterpret_cast<int2 *>(L.trav_spill);
        s.lanes = (unsigned)kPersistentBlocks * 128u;
        s.g = blockIdx.x * 128u + threadIdx.x;
        return s;
    }
};
template <>
struct PtStack<0> {
    using type = RingStack<kRingEntries>;
    static __device__ __forceinline__ type make(uint32_t *lds, const WfLaunch &L) {
        type s;
        s.lds = lds + threadIdx.x;
        s.stride = 128;
        s.glob = L.trav_spill + ((size_t)blockIdx.x * 128 + threadIdx.x) * (size_t)L.spill_depth;
        return s;
    }
};
template <int WIDE, bool ORDERED, bool ANY, bool STATS, class Stk, bool RT = false>
struct PtTracer { using type = Tracer<ORDERED, ANY, STATS, Stk>; };
template <bool ORDERED, bool ANY, bool STATS, class Stk, bool RT>
struct PtTracer<4, ORDERED, ANY, STATS, Stk, RT> { using type = Tracer4<ORDERED, ANY, STATS, Stk, RT>; };
template <bool ORDERED, bool ANY, bool STATS, class Stk, bool RT>
struct PtTracer<8, ORDERED, ANY, STATS, Stk, RT> { using type = Tracer8<ORDERED, ANY, STATS, Stk, RT>; };
// float4 per wide node, and the wide nodes of the LDS copy of the top of the tree (the same bytes for both widths)
template <int WIDE>
constexpr int wide_f4() { return WIDE == 8 ? kWide8F4 : kWideF4; }

// one traversal run to completion by this lane (tail kernel): binary tree with the whole stack in
// LDS (stk: DEPTH x 128 words), or the 4-wide tree with the persistent kernels' LDS window + spill
template <int WIDE, int DEPTH, bool ORDERED, bool ANY, bool STATS>
__device__ __forceinline__ bool trace_lane(const Traversal &tv, const DScene &S, const WfLaunch &L, F3 o, F3 d,
                                           float mint, float maxt, Hit &h, uint32_t *stk, TravStats &st) {
    if constexpr (WIDE > 0) {
        using Stk = typename PtStack<WIDE>::type;
        Stk s = PtStack<WIDE>::make(stk, L);
        typename PtTracer<WIDE, ORDERED, ANY, STATS, Stk>::type tr;
        tr.begin(S, tv, o, d, mint, maxt, st);
#pragma unroll 1
        while (!tr.done) tr.step(tv, s, st);
        h = tr.best;
        return tr.found;
    } else {
        return trace<DEPTH, ORDERED, ANY, STATS>(tv, S, o, d, mint, maxt, h, stk + threadIdx.x, 128, st);
    }
}

#ifndef NH_REFILL_MIN
#define NH_REFILL_MIN 32
#endif
#ifndef NH_PT_WAVES
#define NH_PT_WAVES 5
#endif
// waves per SIMD of the any-hit instantiations (A/B: -DNH_PT_WAVES_ANY=6)
#ifndef NH_PT_WAVES_ANY
#define NH_PT_WAVES_ANY NH_PT_WAVES
#endif
template <int DEPTH, bool ORDERED, bool ANY, bool STATS, int WIDE>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(ANY ? NH_PT_WAVES_ANY : NH_PT_WAVES))) void wf_trace_pt(const DScene *__restrict__ Sp, Traversal tv, WfLaunch L) {
    __shared__ uint32_t stk[kRingEntries * 128];
    __shared__ float4 s_top[WIDE ? kTopNodes * kWideF4 : 1];  // the top of the wide tree (nodes 0 .. n_top-1)
    const DScene &S = *Sp;
    const int n_top = WIDE ? min(tv.n_top, kTopNodes * kWideF4 / wide_f4<WIDE>()) : 0;
    if constexpr (WIDE > 0) {
        for (int i = threadIdx.x; i < n_top * wide_f4<WIDE>(); i += 128) s_top[i] = tv.wnodes[i];
        __syncthreads();
    }
    const QView qv = queue_view(L.cnt_in + (ANY ? kCountGroup : 0));
    const int n = qv.n;
    const int *pre = qv.pre;
    unsigned *fetch = L.cnt_in + (ANY ? 3 : 2) * kCountGroup;
    const WfBuf &B = L.st.buf[L.in_q];
    const int lane = threadIdx.x & 63;
    using Stk = typename PtStack<WIDE>::type;
    Stk my_stk = PtStack<WIDE>::make(stk, L);
    int seg = blockIdx.x & (kQueueShards - 1), tried = 0;
    int batch_next = 0, batch_end = 0;  // wave-uniform
    int slot = -1;                      // this lane's ray (queue slot), -1 = idle
    typename PtTracer<WIDE, ORDERED, ANY, STATS, Stk>::type tr;
    TravStats st{0, 0, 0};
    unsigned long long queries = 0;
    for (;;) {
        const bool idle = slot < 0;
        const unsigned long long im = __ballot(idle);
        // refill once enough lanes are idle (each refill costs the ray fetch, 1/d and the root box
        // test), or when the whole wave is idle
        if (im && (__popcll(im) >= NH_REFILL_MIN || im == ~0ull)) {
            while (batch_next >= batch_end && tried < kQueueShards) {  // wave-uniform refill
                const int lo = (int)((long long)seg * n / kQueueShards);
                const int hi = (int)((long long)(seg + 1) * n / kQueueShards);
                unsigned base = 0;
                if (lane == 0) base = atomicAdd(&fetch[seg * kCountStride], (unsigned)kFetchBatch);
                base = __shfl(base, 0, 64);
                if ((long long)lo + base < hi) {
                    batch_next = lo + (int)base;
                    batch_end = min(batch_next + kFetchBatch, hi);
                } else {
                    seg = (seg + 1) & (kQueueShards - 1);
                    ++tried;
                }
            }
            const int rank = __popcll(im & ((1ull << lane) - 1ull));
            if (idle && batch_next + rank < batch_end) {
                const int q = batch_next + rank;
                slot = queue_slot(pre, L.seg_cap, q);
                float4 ro, rd;
                if (ANY) {
                    ro = L.st.sh_o[slot];
                    rd = L.st.sh_d[slot];
                } else if (L.first && L.cam_rays) {  // thin-lens camera rays, precomputed (wf_camera_rays)
                    ro = B.ray_o[slot];
                    rd = B.ray_d[slot];
                } else {
                    load_ray<false>(S, L, B, q, slot, ro, rd);  // (pinhole camera rays only)
                }
                // a zero BSDF direction (maxt = -inf) misses every primitive without a traversal
                if (STATS && (ANY || rd.w >= ro.w)) ++queries;
                tr.begin(S, tv, xyz(ro), xyz(rd), ro.w, rd.w, st);
            }
            batch_next = min(batch_next + __popcll(im), batch_end);
        }
        if (!__any(slot >= 0)) break;
        if (slot >= 0) {
            if constexpr (WIDE > 0) {
                if (!tr.done) tr.step(tv, my_stk, st, s_top, n_top);
            } else {
                if (!tr.done) tr.step(tv, my_stk, st);
            }
            if (tr.done) {
                if (ANY) {
                    B.occl[L.st.sh_slot[slot]] = tr.found ? 1 : 0;
                } else {
                    B.hit[slot] = make_float4(tr.best.t, tr.best.u, tr.best.v, __int_as_float(tr.found ? tr.best.k : -1));
                }
                slot = -1;
            }
        }
    }
    if (STATS) flush_trav_stats(stat_shard(L.counters) + (ANY ? 8 : 0), queries, st);
}

// Both traversal queries of a bounce in one persistent launch (deep BVHs, 4-wide tree): the closest hit of every
// live path's ray (wf_extend's queue) and the any hit of every queued light sample (wf_shadow's), each answered
// exactly as wf_trace_pt answers it -- same Tracer4 visits, tests and order per ray; only which lane runs which
// ray changes. A wave takes batches from the closest-hit segments first (the longer queries) and then from the
// any-hit segments, so the launch has one tail (its slowest rays) where two launches had two, and an XCD whose
// closest-hit work is done moves on to shadow rays while others finish.
template <bool ORDERED, bool STATS, int WIDE = 4>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(NH_PT_WAVES))) void wf_trace_pt2(const DScene *__restrict__ Sp, Traversal tv, WfLaunch L) {
    __shared__ uint32_t stk[kRingEntries * 128];
    __shared__ float4 s_top[kTopNodes * kWideF4];  // the top of the wide tree (nodes 0 .. n_top-1)
    const DScene &S = *Sp;
    const int n_top = min(tv.n_top, kTopNodes * kWideF4 / wide_f4<WIDE>());
    for (int i = threadIdx.x; i < n_top * wide_f4<WIDE>(); i += 128) s_top[i] = tv.wnodes[i];
    __syncthreads();
    const QView qe = queue_view(L.cnt_in), qs = queue_view(L.cnt_in + kCountGroup);
    unsigned *fetch_e = L.cnt_in + 2 * kCountGroup, *fetch_s = L.cnt_in + 3 * kCountGroup;
    const WfBuf &B = L.st.buf[L.in_q];
    const int lane = threadIdx.x & 63;
    using Stk = typename PtStack<WIDE>::type;
    Stk my_stk = PtStack<WIDE>::make(stk, L);
    // segments 0-7: closest-hit queue, 8-15: any-hit queue; a wave starts on its XCD's segment of each
    int seg = blockIdx.x & (kQueueShards - 1), tried = 0;
    int batch_next = 0, batch_end = 0;  // wave-uniform
    bool batch_any = false;             // wave-uniform: the queue of the current batch
    int slot = -1;                      // this lane's ray (queue slot), -1 = idle
    typename PtTracer<WIDE, ORDERED, false, STATS, Stk, true>::type tr;
    TravStats st_e{0, 0, 0}, st_s{0, 0, 0};
    unsigned long long q_e = 0, q_s = 0;
    for (;;) {
        const bool idle = slot < 0;
        const unsigned long long im = __ballot(idle);
        if (im && (__popcll(im) >= NH_REFILL_MIN || im == ~0ull)) {
            while (batch_next >= batch_end && tried < 2 * kQueueShards) {  // wave-uniform refill
                const bool any = tried >= kQueueShards;
                const int n = any ? qs.n : qe.n;
                const int lo = (int)((long long)seg * n / kQueueShards);
                const int hi = (int)((long long)(seg + 1) * n / kQueueShards);
                unsigned base = 0;
                if (lane == 0) base = atomicAdd(&(any ? fetch_s : fetch_e)[seg * kCountStride], (unsigned)kFetchBatch);
                base = __shfl(base, 0, 64);
                if ((long long)lo + base < hi) {
                    batch_next = lo + (int)base;
                    batch_end = min(batch_next + kFetchBatch, hi);
                    batch_any = any;
                } else {
                    seg = (seg + 1) & (kQueueShards - 1);
                    ++tried;
                }
            }
            const int rank = __popcll(im & ((1ull << lane) - 1ull));
            if (idle && batch_next + rank < batch_end) {
                const int q = batch_next + rank;
                float4 ro, rd;
                if (batch_any) {
                    slot = queue_slot(qs.pre, L.seg_cap, q);
                    ro = L.st.sh_o[slot];
                    rd = L.st.sh_d[slot];
                    if (STATS) ++q_s;
                } else {
                    slot = queue_slot(qe.pre, L.seg_cap, q);
                    if (L.first && L.cam_rays) {  // thin-lens camera rays, precomputed (wf_camera_rays)
                        ro = B.ray_o[slot];
                        rd = B.ray_d[slot];
                    } else {
                        load_ray<false>(S, L, B, q, slot, ro, rd);  // (pinhole camera rays only)
                    }
                    // a zero BSDF direction (maxt = -inf) misses every primitive without a traversal
                    if (STATS && rd.w >= ro.w) ++q_e;
                }
                tr.any_q = batch_any;
                tr.begin(S, tv, xyz(ro), xyz(rd), ro.w, rd.w, batch_any ? st_s : st_e);
            }
            batch_next = min(batch_next + __popcll(im), batch_end);
        }
        if (!__any(slot >= 0)) break;
        if (slot >= 0) {
            if (!tr.done) {
                if (STATS) {
                    if (tr.any_q) tr.step(tv, my_stk, st_s, s_top, n_top);
                    else tr.step(tv, my_stk, st_e, s_top, n_top);
                } else {
                    tr.step(tv, my_stk, st_e, s_top, n_top);
                }
            }
            if (tr.done) {
                if (tr.any_q) B.occl[L.st.sh_slot[slot]] = tr.found ? 1 : 0;
                else B.hit[slot] = make_float4(tr.best.t, tr.best.u, tr.best.v, __int_as_float(tr.found ? tr.best.k : -1));
                slot = -1;
            }
        }
    }
    if (STATS) {
        flush_trav_stats(stat_shard(L.counters), q_e, st_e);
        flush_trav_stats(stat_shard(L.counters) + 8, q_s, st_s);
    }
}

// Where shade_path reads a path's state from: slot s of a path buffer (MemState), or the registers
// of the previous shade step of the same thread (RegState, the tail kernel: no store -> load round
// trip through memory per bounce on its latency-bound chains). Both hand shade_path the same values.
struct MemState {
    const WfBuf &B;
    int s;
    __device__ __forceinline__ void load(float4 &ro, float4 &rd, float4 &li, float4 &thr, uint64_t &rng) const {
        ro = B.ray_o[s];
        rd = B.ray_d[s];
        li = B.li[s];
        thr = B.thr[s];
        rng = B.rng[s];
    }
    __device__ __forceinline__ bool occluded() const { return B.occl[s] != 0; }
    __device__ __forceinline__ float4 pending() const { return B.pend[s]; }
};
struct RegState {
    const PState &o;
    bool occl;
    __device__ __forceinline__ void load(float4 &ro, float4 &rd, float4 &li, float4 &thr, uint64_t &rng) const {
        ro = make_float4(o.ro.x, o.ro.y, o.ro.z, o.pdfmat);
        rd = make_float4(o.rd.x, o.rd.y, o.rd.z,
                         __int_as_float((int)(((unsigned)o.flags << kPidBits) | (unsigned)o.pid)));
        li = o.li;
        thr = o.thr;
        rng = o.rng;
    }
    __device__ __forceinline__ bool occluded() const { return occl; }
    __device__ __forceinline__ float4 pending() const { return o.pe; }
};

// A path between two kernels or shade steps: its vertex's incoming ray (org, d), Li, throughput t, the MIS
// weights, its random-number stream, flags and path id.
struct PathV {
    F3 org, d, li, t;
    float w_mats, w_ems;
    Rng rng;
    int flags, pid;
};

// The head of a shade step (path_mis.cpp:26-71 / path_mats.cpp:22-56): with the hit of the path's ray,
// finish the previous bounce's MIS probe weight (w_mats, :117-140), take the escaped ray's environment term
// or the hit's emitter term, then Russian roulette. Returns whether the path survives; its = the hit's
// Intersection. The previous bounce's pending light sample (F_NEE) must be resolved already. NMAP: hit_info's normal
// maps (false only in the lean bounce kernel, for scenes without textures).
template <bool NMAP = true>
__device__ __forceinline__ bool shade_head(const DScene &S, const Traversal &tv, PathV &v, const Hit &h, bool found,
                                           float pdfmat, Its &its) {
    bool have_its = false;
    if (S.integrator == 1) {  // ---------------- path_mats (path_mats.cpp:16-78)
        if (!found) {  // path_mats.cpp:26-35
            if (S.envmap >= 0) v.li = add(v.li, mulc(v.t, env_eval(S, v.d)));
            return false;
        }
        hit_info<NMAP>(S, tv, h, v.org, v.d, its);
        const DShape shape = S.shapes[its.shape];
        if (shape.emitter >= 0) {
            const F3 wi = normalized(sub(its.p, v.org));
            v.li = add(v.li, mulc(v.t, emitter_eval(S.emitters[shape.emitter], v.org, its.sh.n, wi)));
        }
        int counter = (v.flags >> 4) & 3;
        const float succ = e_min(max_coeff(v.t), 0.99f);
        if (counter < 3) counter++;
        else if (v.rng.next1d() > succ) return false;
        else v.t = divs(v.t, succ);
        v.flags = (v.flags & ~0x30) | (counter << 4);
        return true;
    }
    // ---------------- path_mis
    const float n_lights = (float)S.n_emitters;
    if (!(v.flags & F_FIRST)) {  // finish the previous bounce (path_mis.cpp:115-140)
        // the MIS probe hit an emitter (:117-133): w_mats from the pdfs of both strategies
        if (!(v.flags & F_ZERO_COL) && found) {
            hit_info<NMAP>(S, tv, h, v.org, v.d, its);
            have_its = true;
            const int hem = S.shapes[its.shape].emitter;
            if (hem >= 0) {
                const F3 wim = normalized(sub(its.p, v.org));
                const float pdfmat_ems = emitter_pdf(S, S.emitters[hem], v.org, its.p, its.sh.n, wim) / n_lights;
                if ((pdfmat + pdfmat_ems) > kEps) v.w_mats = pdfmat / (pdfmat + pdfmat_ems);
            }
        }
        if (v.flags & F_DISCRETE) v.w_mats = 1.f;  // :136-140
    }
    if (!found) {  // path_mis.cpp:32-44: escaped rays see the environment map, no MIS weight
        if (S.envmap >= 0) v.li = add(v.li, mulc(v.t, env_eval(S, v.d)));
        return false;
    }
    if (!have_its) hit_info<NMAP>(S, tv, h, v.org, v.d, its);
    const DShape shape = S.shapes[its.shape];
    if (shape.emitter >= 0) {  // path_mis.cpp:51-56, ref = ray origin
        const F3 wi = normalized(sub(its.p, v.org));
        v.li = add(v.li, mulc(scl(v.w_mats, v.t), emitter_eval(S.emitters[shape.emitter], v.org, its.sh.n, wi)));
    }
    float succ = e_min(max_coeff(v.t), 0.99f);  // RR from depth 0 (path_mis.cpp:58-71)
    succ = e_max(succ, kEps);
    if (v.rng.next1d() > succ) return false;
    v.t = divs(v.t, succ);
    return true;
}

// The body of a shade step for a path that survived its head (path_mis.cpp:73-146 / path_mats.cpp:58-76):
// NEE sample (path_mis), BSDF sample, this bounce's MIS-weighted light term and t *= bsdf weight. Writes the
// path's next state to o; nee = a light sample whose shadow ray (so, sd) decides o.pe (F_NEE).
// FULL = false (scenes with no mirror / dielectric BSDF and no albedo texture): the light-sample skip and the texture
// lookup compiled out (rr_step also drops the isolated-sphere test) -- their branches cost C2's bounce kernel ~1 %
// though they never fire there (profiles/round4_session14_16_c2_ab.txt)
template <bool FULL = true>
__device__ __forceinline__ void shade_body(const DScene &S, const Traversal &tv, PathV &v, const Its &its, PState &o,
                                           bool &nee, float4 &so, float4 &sd) {
    const DShape shape = S.shapes[its.shape];
    const DBsdf bsdf = S.bsdfs[shape.bsdf];
    const F3 alb = FULL ? bsdf_albedo(S, bsdf, its.u, its.v) : f3(bsdf.ar, bsdf.ag, bsdf.ab);
    nee = false;
    if (S.integrator == 1) {  // path_mats: BSDF sample only
        const float bx = v.rng.next1d(), by = v.rng.next1d();
        F3 wo;
        int measure;
        const F3 col = bsdf_sample(bsdf, to_local(its.sh, neg(v.d)), bx, by, wo, measure, alb);
        const F3 nd = to_world(its.sh, wo);
        v.t = mulc(v.t, col);  // path_mats.cpp: the throughput update of this bounce
        o.pdfmat = 0.f;
        o.ro = make_float4(its.p.x, its.p.y, its.p.z, kEps);
        o.rd = make_float4(nd.x, nd.y, nd.z, (nd.x == 0 && nd.y == 0 && nd.z == 0) ? -INFINITY : INFINITY);
        o.flags = v.flags & 0x30;
    } else {
        const float n_lights = (float)S.n_emitters;
        // the draws in the reference's order: emitter pick, light sample, BSDF sample
        const float e0 = v.rng.next1d(), ex = v.rng.next1d(), ey = v.rng.next1d();
        const F3 wi_l = to_local(its.sh, neg(v.d));
        // whether the BSDF sample will be discrete, known before it is drawn (bsdf_sample: a dielectric always, a
        // mirror unless wi.z <= 0), so the light sample below runs in the reference's order
        const bool discrete = bsdf.type == BSDF_DIELECTRIC || (bsdf.type == BSDF_MIRROR && !(wi_l.z <= 0));
        // The light sample (path_mis.cpp:80-106). After a discrete BSDF sample its weight is zeroed (:136-140) and
        // f = 0 (discrete BSDFs evaluate to 0), so it adds (0 * t) * (Le/pdf * cos * 0 * n) = +-0 and leaves every
        // other state as it was -- unless a factor is non-finite. S.nee_finite (upload: area / envmap lights only,
        // finite radiance, every light's box apart from every discrete-BSDF shape's, so the sampled point is never
        // the shading point) rules out a non-finite light sample, and t is checked here: then it is not computed.
#ifndef NH_AB_NO_NEE_SKIP  // cost attribution builds only: every light sample computed
        const bool skip_nee = FULL && discrete && S.nee_finite && isfinite(v.t.x) && isfinite(v.t.y) && isfinite(v.t.z);
#else
        const bool skip_nee = false;
#endif
        F3 li_ems = f3(0, 0, 0);
        float pdfems = 0.f, pdfems_mats = 0.f;
        if (!skip_nee) {
            const int ei = emitter_pick(S, e0);
            const DEmitter em = S.emitters[ei];
            ESample es;
            const F3 ems_col = emitter_sample(S, em, its.p, ex, ey, es);
            nee = !is_zero(ems_col);
            if (nee) {
                const F3 we = to_local(its.sh, es.wi);
                const F3 f = bsdf_eval(bsdf, wi_l, we, M_SOLID_ANGLE, alb);
                const float cs = we.z;
                li_ems = f3(ems_col.x * cs * f.x * n_lights, ems_col.y * cs * f.y * n_lights,
                            ems_col.z * cs * f.z * n_lights);
                pdfems_mats = bsdf_pdf(bsdf, wi_l, we, M_SOLID_ANGLE);
                pdfems = emitter_pdf(S, em, its.p, es.p, es.n, es.wi) / n_lights;
                so = make_float4(es.so.x, es.so.y, es.so.z, es.smint);
                sd = make_float4(es.sd.x, es.sd.y, es.sd.z, es.smaxt);
            }
        }
        const float bx = v.rng.next1d(), by = v.rng.next1d();
        F3 wo;
        int measure;
        const F3 bsdf_col = bsdf_sample(bsdf, wi_l, bx, by, wo, measure, alb);
        const float pdfmat = bsdf_pdf(bsdf, wi_l, wo, measure);
        const F3 nd = to_world(its.sh, wo);
        // w_ems of this bounce (:103-106): the occluded shadow ray leaves both pdfs 0 (w_ems keeps its
        // value), the unoccluded one sets it from them; a discrete sample zeroes it either way (:136-140)
        float w_occ = v.w_ems, w_un = v.w_ems;
        if (nee && (pdfems_mats + pdfems) > kEps) w_un = pdfems / (pdfems_mats + pdfems);
        if (discrete) w_occ = w_un = 0.f;
        int fl = (discrete ? F_DISCRETE : 0) | (is_zero(bsdf_col) ? F_ZERO_COL : 0);
        if (nee && discrete) {
            // the discrete sample zeroes both weights: a finite term (0 * t) * li_ems adds exactly zero
            // occluded or not (Li never holds -0), so no shadow ray is queued (as the megakernel)
            const F3 c = mulc(scl(w_un, v.t), li_ems), z = mulc(scl(w_occ, v.t), f3(0, 0, 0));
            if (c.x == 0.f && c.y == 0.f && c.z == 0.f && z.x == 0.f && z.y == 0.f && z.z == 0.f) {
                nee = false;
                li_ems = f3(0, 0, 0);  // the unoccluded term is +-0: Li is unchanged either way
            }
        }
        if (nee) {
            // Li += w_ems * t * Li_ems (:142) once the shadow ray is known to be unoccluded
            const F3 c = mulc(scl(w_un, v.t), li_ems);
            o.pe = make_float4(c.x, c.y, c.z, w_un);
            const F3 z = mulc(scl(w_occ, v.t), f3(0, 0, 0));
            fl |= F_NEE | ((z.x != 0.f || z.y != 0.f || z.z != 0.f) ? F_ZNAN : 0);
        } else {
            v.li = add(v.li, mulc(scl(w_occ, v.t), li_ems));  // li_ems = 0: the same term, added now
        }
        v.w_ems = w_occ;
        v.t = mulc(v.t, bsdf_col);  // :145
        o.pdfmat = pdfmat;
        o.ro = make_float4(its.p.x, its.p.y, its.p.z, kEps);
        o.rd = make_float4(nd.x, nd.y, nd.z, (nd.x == 0 && nd.y == 0 && nd.z == 0) ? -INFINITY : INFINITY);
        o.flags = fl;
    }
    o.li = make_float4(v.li.x, v.li.y, v.li.z, v.w_mats);
    o.thr = make_float4(v.t.x, v.t.y, v.t.z, v.w_ems);
    o.rng = v.rng.state;
    o.pid = v.pid;
}

// the path (state before its head) that a shade step's output o describes, its ray ending at the next hit
__device__ __forceinline__ PathV path_of(const WfLaunch &L, const PState &o) {
    PathV v;
    v.org = xyz(o.ro);
    v.d = xyz(o.rd);
    v.li = xyz(o.li);
    v.w_mats = o.li.w;
    v.t = xyz(o.thr);
    v.w_ems = o.thr.w;
    v.rng.state = o.rng;
    v.rng.inc = ((uint64_t)(L.s0 + o.pid / L.n_list) << 1u) | 1u;
    v.flags = o.flags;
    v.pid = o.pid;
    return v;
}

__device__ __forceinline__ void write_radiance(const WfLaunch &L, const PathV &v) {
    float *r = L.rec + kRecFloats * (size_t)v.pid;
    r[0] = v.li.x;
    r[1] = v.li.y;
    r[2] = v.li.z;
}

// One shade step of the path whose state src holds (slot s of the input queue), hv = the hit of its
// ray: head + body. Returns whether the path continues (its next state in o); sets nee when it sampled a
// light (shadow ray in so/sd). A terminated path writes its radiance to its sample record.
template <class Src, bool NMAP = true>
__device__ __forceinline__ bool shade_path(const DScene &S, const Traversal &tv, const WfLaunch &L, const Src &src,
                                           int s, const float4 hv, PState &o, bool &nee, float4 &so, float4 &sd) {
    float4 ro, rd, li4, th4;
    PathV v;
    if (L.first) {  // bounce 0: the state wf_generate used to write (dense queue: slot = path id)
        float jx, jy;
        camera_sample(S, L, s, v.rng, ro, rd, jx, jy);
        li4 = make_float4(0.f, 0.f, 0.f, 1.f);   // Li, w_mats
        th4 = make_float4(1.f, 1.f, 1.f, 0.f);  // throughput, w_ems
        v.flags = F_FIRST;
        v.pid = s;
        if (L.jit) L.jit[s] = make_float2(jx, jy);
    } else {
        src.load(ro, rd, li4, th4, v.rng.state);
        const int bits = __float_as_int(rd.w);
        v.flags = (int)((unsigned)bits >> kPidBits);
        v.pid = bits & ((1 << kPidBits) - 1);
        v.rng.inc = ((uint64_t)(L.s0 + v.pid / L.n_list) << 1u) | 1u;
    }
    v.org = xyz(ro);
    v.d = xyz(rd);
    v.li = xyz(li4);
    v.t = xyz(th4);
    v.w_mats = li4.w;
    v.w_ems = th4.w;
    Hit h;
    h.t = hv.x;
    h.u = hv.y;
    h.v = hv.z;
    h.k = __float_as_int(hv.w);
    const bool found = h.k >= 0;
    // the previous bounce's light sample counts unless occluded: its MIS-weighted term was computed by
    // that bounce, Li += w_ems * t * Li_ems (:142), and w_ems is the unoccluded weight (:103-106)
    if (S.integrator != 1 && !(v.flags & F_FIRST) && (v.flags & F_NEE)) {
        if (!src.occluded()) {
            const float4 pe = src.pending();
            v.li = add(v.li, xyz(pe));
            v.w_ems = pe.w;
        } else if (v.flags & F_ZNAN) {
            v.li = add(v.li, f3(NAN, NAN, NAN));  // (w_ems * t) * 0 with a non-finite product
        }
    }
    Its its;
    if (!shade_head<NMAP>(S, tv, v, h, found, ro.w, its)) {
        write_radiance(L, v);
        return false;
    }
    shade_body(S, tv, v, its, o, nee, so, sd);
    return true;
}

// One queue entry per thread; survivors are ranked within the workgroup (wave ballots + LDS
// atomics), the workgroup reserves its ranges of the next buffer and the shadow queue with one
// device-scope atomic each, then every thread stores its state at its final slot.
//
// SORT (material-sorted shading, scenes mixing BSDF types on deep BVHs): the workgroup first reads its
// 256 entries' hits, ranks them by the BSDF type of the hit primitive (kPrimMatShift bits of its record;
// misses last) and thread t then shades the t-th entry of that order, so each wave runs mostly one BSDF's
// code (microfacet's Beckmann sampling and evaluation, or diffuse) instead of interleaving them lane by lane.
// Only which thread shades which entry changes; every path's operations are the same.
#ifndef NH_SHADE_WAVES
#define NH_SHADE_WAVES 4
#endif
// NMAP: hit_info's normal maps (false for scenes without them, as the full RR-ahead bodies)
template <bool SORT, bool NMAP = true>
__global__ __launch_bounds__(256, NH_SHADE_WAVES) void wf_shade(const DScene *__restrict__ Sp, Traversal tv, WfLaunch L) {
    __shared__ unsigned s_n[2], s_base[2];
    __shared__ unsigned s_cls[SORT ? 6 : 1];
    __shared__ short s_perm[SORT ? 256 : 1];
    const DScene &S = *Sp;
    const QView qv = queue_view(L.cnt_in);
    // one 256-entry chunk per workgroup: the grid covers the host's upper bound of qv.n
    const int base = blockIdx.x * 256;
    if (base >= qv.n) return;  // whole workgroup
    // gridDim.x is a multiple of kQueueShards, so shard s receives the chunks c = s (mod 8):
    // at most seg_cap entries (nh_api.hip sizes seg_cap so)
    const int shard = blockIdx.x & (kQueueShards - 1);
    if (threadIdx.x < 2) s_n[threadIdx.x] = 0u;
    const WfBuf &B = L.st.buf[L.in_q];
    int q = base + (int)threadIdx.x;
    if constexpr (SORT) {
        if (threadIdx.x < 6) s_cls[threadIdx.x] = 0u;
        __syncthreads();
        int cls = 5;  // past the queue's end: last
        if (q < qv.n) {
            const int k = __float_as_int(B.hit[queue_slot(qv.pre, L.seg_cap, q)].w);
            cls = k >= 0 ? prim_material(tv.prims[3 * k + 2]) : 4;
        }
        int rank = 0;
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            const int r = wave_append(&s_cls[c], cls == c);
            if (cls == c) rank = r;
        }
        __syncthreads();
        unsigned off = 0;
        for (int c = 0; c < cls; ++c) off += s_cls[c];
        s_perm[off + rank] = (short)threadIdx.x;
        __syncthreads();
        q = base + (int)s_perm[threadIdx.x];
    } else {
        __syncthreads();
    }
    bool cont = false, nee = false;
    PState o;
    float4 so, sd;
    if (q < qv.n) {
        const int s = queue_slot(qv.pre, L.seg_cap, q);
        cont = shade_path<MemState, NMAP>(S, tv, L, MemState{B, s}, s, B.hit[s], o, nee, so, sd);
    }
    const int le = wave_append(&s_n[0], cont);
    const int ls = wave_append(&s_n[1], cont && nee);
    __syncthreads();
    if (threadIdx.x == 0) {
        s_base[0] = s_n[0] ? atomicAdd(&L.cnt_out[shard * kCountStride], s_n[0]) : 0u;
        s_base[1] = s_n[1] ? atomicAdd(&L.cnt_out[kCountGroup + shard * kCountStride], s_n[1]) : 0u;
    }
    __syncthreads();
    if (cont) {
        const int slot = shard * L.seg_cap + (int)s_base[0] + le;
        store_state(L.st.buf[1 - L.in_q], slot, o);
        if (nee) {
            const int ss = shard * L.seg_cap + (int)s_base[1] + ls;
            L.st.sh_o[ss] = so;
            L.st.sh_d[ss] = sd;
            L.st.sh_slot[ss] = slot;
        }
    }
}

// Fused bounce for BVHs staged in LDS (the Cornell-box configurations, < 16 KB of nodes and
// primitives): traversal there is ALU work on an LDS copy, so extend / any-hit / shade as three
// kernels only add queue round trips through HBM and two launches per bounce. One thread per live
// path runs the bounce end to end -- shade (shade_path), the any-hit query of the light sample it
// queued, the closest hit of the next ray -- and stores the path state with that hit. The same
// operations on the same values as the split kernels: the unoccluded light term is added to Li
// where the next shade would have added it (before that bounce's emitter term), so the image is
// bit-identical.
//
// Material-sorted queue: survivors are ranked within the workgroup by the BSDF type of their next
// hit (kPrimMatShift bits of the primitive record; misses last), so the next bounce's waves shade
// runs of one material instead of interleaving the diffuse, mirror, dielectric and microfacet
// code paths lane by lane (SURVEY.md north star: material-sorted shade queues).
constexpr int kMatClasses = 5;  // 4 BSDF types + rays that leave the scene
#ifndef NH_TAIL_WAVES
#define NH_TAIL_WAVES 1
#endif
#ifndef NH_BOUNCE_WAVES
#define NH_BOUNCE_WAVES 4
#endif
template <bool ORDERED, bool STATS, bool SORT>
__global__ __launch_bounds__(256, NH_BOUNCE_WAVES) void wf_bounce(const DScene *__restrict__ Sp, Traversal tv_g,
                                                                  WfLaunch L) {
    __shared__ uint32_t stk[16 * 256];
    __shared__ unsigned s_n[kMatClasses], s_off[kMatClasses], s_base;
    extern __shared__ float4 lds_scene[];
    const DScene &S = *Sp;
    const QView qv = queue_view(L.cnt_in);
    const int base = blockIdx.x * 256;
    if (base >= qv.n) return;  // whole workgroup
    if (threadIdx.x < kMatClasses) s_n[threadIdx.x] = 0u;  // visible after the staging barrier
    const Traversal tv = stage_small_scene<true>(tv_g, L, lds_scene);
    // gridDim.x is a multiple of kQueueShards: shard s receives the chunks c = s (mod 8), at most
    // seg_cap entries (as wf_shade)
    const int shard = blockIdx.x & (kQueueShards - 1);
    const int q = base + (int)threadIdx.x;
    const WfBuf &B = L.st.buf[L.in_q];
    uint32_t *my_stk = stk + threadIdx.x;
    TravStats st_e{0, 0, 0}, st_s{0, 0, 0};
    unsigned long long q_e = 0, q_s = 0;
    bool cont = false;
    PState o;
    float4 hit_out = make_float4(0.f, 0.f, 0.f, 0.f);
    int cls = kMatClasses - 1;
    if (q < qv.n) {
        const int s = queue_slot(qv.pre, L.seg_cap, q);
        float4 hv;
        if (L.first) {  // the camera ray's closest hit (wf_extend at bounce 0)
            float4 ro, rd;
            load_ray(S, L, B, q, s, ro, rd);
            Hit h;
            const bool live = rd.w >= ro.w;
            q_e += live ? 1 : 0;
            const bool found = live && trace<16, ORDERED, false, STATS, true>(tv, S, xyz(ro), xyz(rd), ro.w, rd.w, h,
                                                                        my_stk, 256, st_e);
            hv = make_float4(h.t, h.u, h.v, __int_as_float(found ? h.k : -1));
        } else {
            hv = B.hit[s];
        }
        bool nee = false;
        float4 so, sd;
        cont = shade_path(S, tv, L, MemState{B, s}, s, hv, o, nee, so, sd);
        if (cont) {
            if (nee) {  // the light sample's any-hit query (wf_shadow), its outcome applied as shade_path would
                Hit hs;
                ++q_s;
                if (!trace<16, ORDERED, true, STATS, true>(tv, S, xyz(so), xyz(sd), so.w, sd.w, hs, my_stk, 256, st_s)) {
                    o.li.x = o.li.x + o.pe.x;
                    o.li.y = o.li.y + o.pe.y;
                    o.li.z = o.li.z + o.pe.z;
                    o.thr.w = o.pe.w;
                } else if (o.flags & F_ZNAN) {
                    o.li.x = o.li.x + NAN;
                    o.li.y = o.li.y + NAN;
                    o.li.z = o.li.z + NAN;
                }
                o.flags &= ~(F_NEE | F_ZNAN);
            }
            Hit h;  // the next ray's closest hit (wf_extend)
            const bool live = o.rd.w >= o.ro.w;
            q_e += live ? 1 : 0;
#ifdef NH_EXPERIMENT_TRACE_TWICE  // cost attribution only: the closest-hit query runs twice (same answer)
            {
                Hit h2;
                if (live && trace<16, ORDERED, false, STATS, true>(tv, S, xyz(o.ro), xyz(o.rd), o.ro.w, o.rd.w, h2, my_stk, 256, st_e))
                    o.rng ^= (uint64_t)(h2.k == -7);
            }
#endif
            const bool found = live && trace_next<16, ORDERED, STATS, true>(tv, S, __float_as_int(hv.w), xyz(o.ro),
                                                                      xyz(o.rd), o.ro.w, o.rd.w, h, my_stk, 256, st_e);
            hit_out = make_float4(h.t, h.u, h.v, __int_as_float(found ? h.k : -1));
            if (found) cls = prim_material(tv.prims[3 * h.k + 2]);
        }
    }
    // rank survivors: by material class (sorted queue) or in lane order
    int rank = 0;
    if (SORT) {
#pragma unroll
        for (int c = 0; c < kMatClasses; ++c) {
            const int r = wave_append(&s_n[c], cont && cls == c);
            if (cls == c) rank = r;
        }
    } else {
        cls = 0;
        rank = wave_append(&s_n[0], cont);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned tot = 0;
        for (int c = 0; c < kMatClasses; ++c) {
            s_off[c] = tot;
            tot += s_n[c];
        }
        s_base = tot ? atomicAdd(&L.cnt_out[shard * kCountStride], tot) : 0u;
    }
    __syncthreads();
    if (cont) {
        const WfBuf &Bo = L.st.buf[1 - L.in_q];
        const int slot = shard * L.seg_cap + (int)(s_base + s_off[cls]) + rank;
        store_state(Bo, slot, o);
        Bo.hit[slot] = hit_out;
    }
    if (STATS) {
        flush_trav_stats(stat_shard(L.counters), q_e, st_e);
        flush_trav_stats(stat_shard(L.counters) + kStatAny, q_s, st_s);
    }
}

// ---------------------------------------------------------------------------------------------------------
// Russian roulette ahead (LDS-staged BVHs, default). A wf_bounce launch loses about a third of its lanes at the
// roulette of path_mis.cpp:58-71 (C2: 29.4M -> 19.4M paths at the first bounce), and those lanes then idle
// through the light sample's any-hit and the next closest-hit traversals, most of the launch's work
// (measured: VALUUtilization 48 %, profiles/round3_c2_pmc_valu_summary.txt). Here a launch ends with the head
// of the NEXT vertex instead -- its probe MIS weight, emitter term and roulette draw (shade_head: every
// operand is known once the next ray's closest hit is) -- and stores only the paths that survive it, so the
// next launch's lanes all carry live paths through body, shadow ray and traversal. The same float operations
// and random draws in the same order per path; only where the kernel boundary falls moves.
//
// Stored state of a live path (WfBuf, as store_state): its vertex's incoming ray (org, d), Li / w_mats,
// throughput / w_ems after the roulette division, the stream after the roulette draw, path_mats' counter,
// and the ray's hit; the next launch recomputes the Intersection from the hit (hit_info is a pure function).
__device__ __forceinline__ void store_post_head(const WfBuf &B, int s, const PathV &v, const Hit &h) {
    B.ray_o[s] = make_float4(v.org.x, v.org.y, v.org.z, 0.f);
    B.ray_d[s] = make_float4(v.d.x, v.d.y, v.d.z, __int_as_float((int)(((unsigned)(v.flags & 0x30) << kPidBits) | (unsigned)v.pid)));
    B.li[s] = make_float4(v.li.x, v.li.y, v.li.z, v.w_mats);
    B.thr[s] = make_float4(v.t.x, v.t.y, v.t.z, v.w_ems);
    B.rng[s] = v.rng.state;
    B.hit[s] = make_float4(h.t, h.u, h.v, __int_as_float(h.k));
}

template <bool NMAP = true>
__device__ __forceinline__ void load_post_head(const DScene &S, const Traversal &tv, const WfLaunch &L, const WfBuf &B,
                                               int s, PathV &v, Hit &h, Its &its) {
    const float4 ro = B.ray_o[s], rd = B.ray_d[s], li4 = B.li[s], th4 = B.thr[s], hv = B.hit[s];
    v.rng.state = B.rng[s];
    const int bits = __float_as_int(rd.w);
    v.flags = (int)((unsigned)bits >> kPidBits);
    v.pid = bits & ((1 << kPidBits) - 1);
    v.rng.inc = ((uint64_t)(L.s0 + v.pid / L.n_list) << 1u) | 1u;
    v.org = xyz(ro);
    v.d = xyz(rd);
    v.li = xyz(li4);
    v.w_mats = li4.w;
    v.t = xyz(th4);
    v.w_ems = th4.w;
    h.t = hv.x;
    h.u = hv.y;
    h.v = hv.z;
    h.k = __float_as_int(hv.w);
    hit_info<NMAP>(S, tv, h, v.org, v.d, its);
}

// the camera path of queue entry s at bounce 0, up to its first vertex's head
template <bool ORDERED, bool STATS, bool NMAP = true>
__device__ __forceinline__ bool first_vertex(const DScene &S, const Traversal &tv, const WfLaunch &L, int s, PathV &v,
                                             Hit &h, Its &its, uint32_t *stk, int stride, TravStats &st_e,
                                             unsigned long long &q_e) {
    float4 ro, rd;
    float jx, jy;
    camera_sample(S, L, s, v.rng, ro, rd, jx, jy);
    if (L.jit) L.jit[s] = make_float2(jx, jy);
    v.org = xyz(ro);
    v.d = xyz(rd);
    v.li = f3(0.f, 0.f, 0.f);
    v.t = f3(1.f, 1.f, 1.f);
    v.w_mats = 1.f;
    v.w_ems = 0.f;
    v.flags = F_FIRST;
    v.pid = s;
    const bool live = rd.w >= ro.w;
    q_e += live ? 1 : 0;
    const bool found = live && trace<16, ORDERED, false, STATS, true>(tv, S, v.org, v.d, ro.w, rd.w, h, stk, stride, st_e);
    if (!shade_head<NMAP>(S, tv, v, h, found, 0.f, its)) {
        write_radiance(L, v);
        return false;
    }
    return true;
}

// Cycle counters of the tail kernel's phases (calibration launches only, CLK): shade body, the light sample's
// any-hit query, the next closest hit, the next vertex's head -- summed over lanes -- and the path-bounces run.
struct TailClocks {
    unsigned long long c[4] = {0, 0, 0, 0};
    unsigned long long bounces = 0, max_bounces = 0;
    unsigned long long cc[4] = {0, 0, 0, 0}, coop_bounces = 0;  // the same, for bounces carried by lane groups
};

// body of the current vertex, its light sample's any-hit query, the next ray's closest hit, and the next
// vertex's head; false once the path has ended (its radiance written). G > 1: the path is carried by a G-lane
// group (every lane the same state and arithmetic; leaf primitives tested cooperatively; one lane writes and counts).
// NMAP: hit_info's normal maps (FULL kernels of scenes without normal maps compile them out: the inlined normal-map
// branches and their tex_eval calls cost C1 / C4 2.5 % when present, profiles/round6_ab_nmap.txt)
template <bool ORDERED, bool STATS, bool CLK = false, int G = 1, bool FULL = true, bool NMAP = FULL>
__device__ __forceinline__ bool rr_step(const DScene &S, const Traversal &tv, const WfLaunch &L, PathV &v, Its &its,
                                        Hit &h, uint32_t *stk, int stride, TravStats &st_e, TravStats &st_s,
                                        unsigned long long &q_e, unsigned long long &q_s, TailClocks *clk = nullptr) {
    const bool lead = G == 1 || (threadIdx.x & (G - 1)) == 0;
    PState o;
    bool nee = false;
    float4 so, sd;
    unsigned long long t0 = 0, t1 = 0;
    unsigned long long *cs = CLK ? (G > 1 ? clk->cc : clk->c) : nullptr;
    if constexpr (CLK) t0 = clock64();
    shade_body<FULL>(S, tv, v, its, o, nee, so, sd);
    if constexpr (CLK) {
        t1 = clock64();
        if (lead) cs[0] += t1 - t0;
        t0 = t1;
    }
    if (nee) {  // the light sample's any-hit query, its outcome applied as the next shade_path would
        Hit hs;
        if (lead) ++q_s;
        if (!trace<16, ORDERED, true, STATS, true, G>(tv, S, xyz(so), xyz(sd), so.w, sd.w, hs, stk, stride, st_s)) {
            o.li.x = o.li.x + o.pe.x;
            o.li.y = o.li.y + o.pe.y;
            o.li.z = o.li.z + o.pe.z;
            o.thr.w = o.pe.w;
        } else if (o.flags & F_ZNAN) {
            o.li.x = o.li.x + NAN;
            o.li.y = o.li.y + NAN;
            o.li.z = o.li.z + NAN;
        }
        o.flags &= ~(F_NEE | F_ZNAN);
    }
    if constexpr (CLK) {
        t1 = clock64();
        if (lead) cs[1] += t1 - t0;
        t0 = t1;
    }
    const bool live = o.rd.w >= o.ro.w;
    if (lead) q_e += live ? 1 : 0;
    const bool found = live && trace_next<16, ORDERED, STATS, true, G, FULL>(tv, S, h.k, xyz(o.ro), xyz(o.rd), o.ro.w,
                                                                      o.rd.w, h, stk, stride, st_e);
    if constexpr (CLK) {
        t1 = clock64();
        if (lead) cs[2] += t1 - t0;
        t0 = t1;
    }
    v = path_of(L, o);
    const bool alive = shade_head<NMAP>(S, tv, v, h, found, o.pdfmat, its);
    if constexpr (CLK) {
        if (lead) cs[3] += clock64() - t0;
        if (lead) ++(G > 1 ? clk->coop_bounces : clk->bounces);
    }
    if (!alive) {
        if (lead) write_radiance(L, v);
        return false;
    }
    return true;
}

// threads per wf_bounce_rr workgroup (A/B builds: -DNH_BOUNCE_TB=128)
#ifndef NH_BOUNCE_TB
#define NH_BOUNCE_TB 256
#endif

// one queue entry of a RR-ahead bounce: load its path (or, at bounce 0, its camera ray and first hit) and run
// rr_step; true when the path lives on (v, h: its state to store)
template <bool ORDERED, bool STATS, bool FULL, bool NMAP = FULL>
__device__ __forceinline__ bool bounce_path(const DScene &S, const Traversal &tv, const WfLaunch &L, const QView &qv,
                                            int q, uint32_t *my_stk, PathV &v, Hit &h, TravStats &st_e,
                                            TravStats &st_s, unsigned long long &q_e, unsigned long long &q_s,
                                            TailClocks &clk, unsigned long long &c_load) {
    const int s = queue_slot(qv.pre, L.seg_cap, q);
    Its its;
    bool alive = true;
    unsigned long long t_ph = 0;
    if constexpr (STATS) t_ph = clock64();
    if (L.first) alive = first_vertex<ORDERED, STATS, NMAP>(S, tv, L, s, v, h, its, my_stk, NH_BOUNCE_TB, st_e, q_e);
    else load_post_head<NMAP>(S, tv, L, L.st.buf[L.in_q], s, v, h, its);
    if constexpr (STATS) c_load += clock64() - t_ph;
    return alive && rr_step<ORDERED, STATS, STATS, 1, FULL, NMAP>(S, tv, L, v, its, h, my_stk, NH_BOUNCE_TB, st_e, st_s, q_e,
                                                            q_s, &clk);
}

template <bool ORDERED, bool STATS, bool SORT, bool FULL = true, bool NMAP = FULL>
__global__ __launch_bounds__(NH_BOUNCE_TB, NH_BOUNCE_WAVES) void wf_bounce_rr(const DScene *__restrict__ Sp, Traversal tv_g,
                                                                     WfLaunch L) {
    __shared__ uint32_t stk[16 * NH_BOUNCE_TB];
    __shared__ unsigned s_n[kMatClasses], s_off[kMatClasses], s_base;
    extern __shared__ float4 lds_scene[];
    const QView qv = queue_view(L.cnt_in);
    const int base = blockIdx.x * NH_BOUNCE_TB;
    if (base >= qv.n) return;  // whole workgroup
    if (threadIdx.x < kMatClasses) s_n[threadIdx.x] = 0u;  // visible after the staging barrier
    const DScene &S = *Sp;
    const Traversal tv = stage_small_scene<true>(tv_g, L, lds_scene);
    const int shard = blockIdx.x & (kQueueShards - 1);
    const int q = base + (int)threadIdx.x;
    uint32_t *my_stk = stk + threadIdx.x;
    TravStats st_e{0, 0, 0}, st_s{0, 0, 0};
    unsigned long long q_e = 0, q_s = 0;
    bool cont = false;
    PathV v;
    Hit h;
    int cls = kMatClasses - 1;
    // STATS (calibration launch): clock64 per phase -- load (path state + its hit's Intersection, or the camera
    // ray and its closest hit at bounce 0), then rr_step's body / shadow / closest / head, then rank + store
    TailClocks clk;
    unsigned long long c_load = 0, c_store = 0, t_ph = 0;
    if (q < qv.n) {
        cont = bounce_path<ORDERED, STATS, FULL, NMAP>(S, tv, L, qv, q, my_stk, v, h, st_e, st_s, q_e, q_s, clk, c_load);
        if (cont) cls = prim_material(tv.prims[3 * h.k + 2]);  // a live path's ray has hit something
        if constexpr (STATS) t_ph = clock64();
    }
    int rank = 0;  // survivors ranked by the material class of their hit (sorted queue) or in lane order
    if (SORT) {
#pragma unroll
        for (int c = 0; c < kMatClasses; ++c) {
            const int r = wave_append(&s_n[c], cont && cls == c);
            if (cls == c) rank = r;
        }
    } else {
        cls = 0;
        rank = wave_append(&s_n[0], cont);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned tot = 0;
        for (int c = 0; c < kMatClasses; ++c) {
            s_off[c] = tot;
            tot += s_n[c];
        }
        s_base = tot ? atomicAdd(&L.cnt_out[shard * kCountStride], tot) : 0u;
    }
    __syncthreads();
    if (cont) store_post_head(L.st.buf[1 - L.in_q], shard * L.seg_cap + (int)(s_base + s_off[cls]) + rank, v, h);
    if (STATS) {
        if (q < qv.n) c_store = clock64() - t_ph;
        flush_trav_stats(stat_shard(L.counters), q_e, st_e);
        flush_trav_stats(stat_shard(L.counters) + kStatAny, q_s, st_s);
        unsigned long long *dst = stat_shard(L.counters) + kStatBounceClk;
        for (int j = 0; j < 7; ++j) {
            unsigned long long x = j == 0 ? c_load : j < 5 ? clk.c[j - 1] : j == 5 ? c_store : clk.bounces;
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
            if ((threadIdx.x & 63) == 0) atomicAdd(&dst[j], x);
        }
    }
}

// the chunk's last paths (RR-ahead state) finished in place, one thread per path, as wf_tail
// TB: threads per workgroup. A tail workgroup keeps its LDS (stacks + scene copy) until its longest path ends
// (~1000 specular bounces), so 64-thread workgroups pin a quarter of what 256-thread ones do.
// W: waves per SIMD the registers must allow. W = 1 (240-255 VGPRs) holds half a SIMD's register file per tail
// wave for the tail's whole length, which halves the occupancy of the next chunks' bounce kernels (128 VGPRs)
// beside it; W = 4 (the bounce kernel's budget) leaves them their 4 waves.
// Cooperative finish (NH_TAIL_COOP, default 16): once a tail wave carries few enough paths, each remaining path is
// handed through LDS to a group of lanes that carries it from then on (rr_step<.., G>): the chain of specular
// bounces that sets the tail's length then tests each leaf's primitives in one parallel step instead of one after
// the other. Only which lanes run which operation changes; every path's operations and draws are the same.
constexpr int kTailCoopWords = 48;  // 32-bit words of one handed-over path (PathV, Hit, Its, bounce count)
// FULL = false: the lean body of wf_bounce_rr<.., FULL = false> (scenes with no mirror / dielectric BSDF and no texture)
template <bool ORDERED, bool STATS, int TB, int W, bool FULL = true, bool NMAP = FULL>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(W))) void wf_tail_rr(
    const DScene *__restrict__ Sp, Traversal tv_g, WfLaunch L, int coop) {
    __shared__ uint32_t stk[16 * TB];
    __shared__ uint32_t xfer[TB == 64 ? 4 * kTailCoopWords : 1];
    extern __shared__ float4 lds_scene[];
    const DScene &S = *Sp;
    const Traversal tv = stage_small_scene<true>(tv_g, L, lds_scene);
    const QView qv = queue_view(L.cnt_in);
    const WfBuf &B = L.st.buf[L.in_q];
    TravStats st_e{0, 0, 0}, st_s{0, 0, 0};
    unsigned long long q_e = 0, q_s = 0;
    TailClocks clk;
    // one path per lane (the host sizes the grid to the live count, at most kTailCap)
    const int q = blockIdx.x * TB + threadIdx.x;
    bool alive = q < qv.n;
    PathV v;
    Hit h;
    Its its;
    unsigned long long nb = 0;  // bounces of this lane's path
    if (alive) load_post_head<NMAP>(S, tv, L, B, queue_slot(qv.pre, L.seg_cap, q), v, h, its);
    const bool can_coop = TB == 64 && coop == 16;
    for (;;) {
        const unsigned long long m = __ballot(alive);
        if (m == 0ull || (can_coop && __popcll(m) <= 4)) break;
        if (alive) {
            alive = rr_step<ORDERED, STATS, STATS, 1, FULL, NMAP>(S, tv, L, v, its, h, stk + threadIdx.x, TB, st_e, st_s,
                                                            q_e, q_s, &clk);
            ++nb;
        }
    }
    if (STATS && !can_coop) clk.max_bounces = max(clk.max_bounces, nb);
    if constexpr (TB == 64) {
        const unsigned long long m = __ballot(alive);
        if (can_coop && m) {
            // hand the (at most 4) remaining paths to 16-lane groups: path of rank r -> lanes 16r .. 16r+15
            const int lane = threadIdx.x & 63;
            if (alive) {
                uint32_t *w = xfer + __popcll(m & ((1ull << lane) - 1ull)) * kTailCoopWords;
                static_assert(sizeof(PathV) + sizeof(Hit) + sizeof(Its) + 8 <= kTailCoopWords * 4, "xfer slot");
                __builtin_memcpy(w, &v, sizeof(PathV));
                __builtin_memcpy(w + sizeof(PathV) / 4, &h, sizeof(Hit));
                __builtin_memcpy(w + (sizeof(PathV) + sizeof(Hit)) / 4, &its, sizeof(Its));
                __builtin_memcpy(w + (sizeof(PathV) + sizeof(Hit) + sizeof(Its)) / 4, &nb, 8);
            }
            __syncthreads();  // TB == 64: the workgroup is this one wave
            const int g = lane >> 4;
            bool carry = g < __popcll(m);
            if (carry) {
                const uint32_t *w = xfer + g * kTailCoopWords;
                __builtin_memcpy(&v, w, sizeof(PathV));
                __builtin_memcpy(&h, w + sizeof(PathV) / 4, sizeof(Hit));
                __builtin_memcpy(&its, w + (sizeof(PathV) + sizeof(Hit)) / 4, sizeof(Its));
                __builtin_memcpy(&nb, w + (sizeof(PathV) + sizeof(Hit) + sizeof(Its)) / 4, 8);
            }
            while (__ballot(carry)) {
                if (carry) {
                    carry = rr_step<ORDERED, STATS, STATS, 16, FULL, NMAP>(S, tv, L, v, its, h, stk + threadIdx.x, TB, st_e,
                                                                    st_s, q_e, q_s, &clk);
                    ++nb;
                }
            }
            if (STATS && (lane & 15) == 0 && g < __popcll(m)) clk.max_bounces = max(clk.max_bounces, nb);
        } else if (STATS && can_coop) {
            clk.max_bounces = max(clk.max_bounces, nb);
        }
    }
    if (STATS) {  // the tail's own counter slots (kStatTail*), so stage rates stay per kernel
        flush_trav_stats(stat_shard(L.counters) + kStatTail, q_e, st_e);
        flush_trav_stats(stat_shard(L.counters) + kStatTailAny, q_s, st_s);
        unsigned long long *dst = stat_shard(L.counters) + kStatTailClk;
        for (int j = 0; j < 5; ++j) {
            unsigned long long x = j < 4 ? clk.c[j] : clk.bounces;
            unsigned long long y = j < 4 ? clk.cc[j] : clk.coop_bounces;
            for (int off = 32; off > 0; off >>= 1) {
                x += __shfl_xor(x, off, 64);
                y += __shfl_xor(y, off, 64);
            }
            if ((threadIdx.x & 63) == 0) {
                atomicAdd(&dst[j], x);
                atomicAdd(&dst[kStatTailCoopClk - kStatTailClk + j], y);
            }
        }
        unsigned long long mx = clk.max_bounces;
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, (unsigned long long)__shfl_xor(mx, off, 64));
        if ((threadIdx.x & 63) == 0) atomicMax(&dst[5], mx);
    }
}

// Asynchronous tail hand-off: the chunk's live paths (RR-ahead state, 88 B each) are copied into a small buffer
// of their own, densely from slot 0 (all in count shard 0; the other shards and groups are zeroed by the host),
// so the pool's path state is free for the next chunk while this chunk's tail kernel runs on another stream.
#if !defined(NH_WF_PART) || NH_WF_PART == 1  // non-template kernels: defined in one part only
// After a bounce's appending kernel: its output counts (n_copy words) to the pool's pinned host ring, and the
// count slot its input came from (dead now, the next bounce's output) zeroed -- one kernel in place of the
// runtime's two blit kernels (a device-to-host copy and a memset) per bounce. The host reads the ring once the
// event recorded after this kernel has completed: system-scope stores, then a system fence.
__global__ __launch_bounds__(256) void wf_counts_kernel(const unsigned *src, unsigned *host_dst, int n_copy,
                                                        unsigned *zero, int n_zero) {
    for (int i = threadIdx.x; i < n_copy; i += 256)
        __hip_atomic_store(&host_dst[i], src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int i = threadIdx.x; i < n_zero; i += 256) zero[i] = 0u;
    __threadfence_system();
}
#endif
#if !defined(NH_WF_PART) || NH_WF_PART == 1  // a non-template kernel: defined in one part only
// bounce 0's camera rays of a thin-lens scene, for the persistent traversal kernels, whose refill code builds pinhole
// rays only (camera_ray<false>: the lens arithmetic spilled it): the same camera_sample as every other kernel, stored
// raw -- (origin, mint), (direction, maxt) -- in the input buffer's ray words, which bounce 0 does not use otherwise
__global__ __launch_bounds__(256) void wf_camera_rays(const DScene *__restrict__ Sp, WfLaunch L) {
    const DScene &S = *Sp;
    const QView qv = queue_view(L.cnt_in);
    const WfBuf &B = L.st.buf[L.in_q];
    for (int q = blockIdx.x * 256 + threadIdx.x; q < qv.n; q += gridDim.x * 256) {
        const int s = queue_slot(qv.pre, L.seg_cap, q);
        float4 ro, rd;
        load_ray<true>(S, L, B, q, s, ro, rd);  // L.first: the camera ray of path q
        B.ray_o[s] = ro;
        B.ray_d[s] = rd;
    }
}

__global__ __launch_bounds__(256) void wf_pack_rr(WfLaunch L, WfBuf dst, unsigned *dst_counts) {
    const QView qv = queue_view(L.cnt_in);
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q == 0) dst_counts[0] = (unsigned)qv.n;
    if (q >= qv.n) return;
    const WfBuf &B = L.st.buf[L.in_q];
    const int s = queue_slot(qv.pre, L.seg_cap, q);
    dst.ray_o[q] = B.ray_o[s];
    dst.ray_d[q] = B.ray_d[s];
    dst.li[q] = B.li[s];
    dst.thr[q] = B.thr[s];
    dst.rng[q] = B.rng[s];
    dst.hit[q] = B.hit[s];
}
#endif

// Tail of a chunk: once few paths are alive, per-bounce launches cost more than the work they
// carry (three kernels + count traffic for a few thousand paths). wf_tail takes the live queue
// of a bounce whose extend / any-hit traversals are done and finishes every path in place, one
// thread per path: shade, then its next closest-hit and shadow traversals, until it terminates --
// the same operations in the same order as further wavefront bounces.
template <int DEPTH, bool ORDERED, bool STATS, bool SMALL, int WIDE>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(NH_TAIL_WAVES))) void wf_tail(const DScene *__restrict__ Sp, Traversal tv_g, WfLaunch L) {
    __shared__ uint32_t stk[DEPTH * 128];
    extern __shared__ float4 lds_scene[];
    const DScene &S = *Sp;
    const Traversal tv = traversal_view<SMALL>(tv_g, L, lds_scene);
    const QView qv = queue_view(L.cnt_in);
    const WfBuf &B = L.st.buf[L.in_q];
    TravStats st_e{0, 0, 0}, st_s{0, 0, 0};
    unsigned long long q_e = 0, q_s = 0;
    for (int q = blockIdx.x * 128 + threadIdx.x; q < qv.n; q += gridDim.x * 128) {
        const int s = queue_slot(qv.pre, L.seg_cap, q);
        // the first step reads the path from the buffer; later steps take the previous step's state,
        // hit and occlusion straight from registers (nothing else reads them: the chunk ends here)
        PState o;
        bool nee = false, occ = false;
        float4 so, sd;
        const float4 hv0 = B.hit[s];
        if (!shade_path(S, tv, L, MemState{B, s}, s, hv0, o, nee, so, sd)) continue;
        int kp = __float_as_int(hv0.w);  // the primitive the next ray leaves (trace_next)
        for (;;) {
            Hit h;
            const bool live = o.rd.w >= o.ro.w;
            q_e += live ? 1 : 0;
            const bool found =
                live && ((S.iso_spheres && S.root_kind != 0 && iso_sphere_hit<STATS>(tv, kp, xyz(o.ro), xyz(o.rd), o.ro.w, o.rd.w, h, st_e)) ||
                         trace_lane<WIDE, DEPTH, ORDERED, false, STATS>(tv, S, L, xyz(o.ro), xyz(o.rd), o.ro.w, o.rd.w, h,
                                                                        stk, st_e));
            kp = found ? h.k : -1;
            const float4 hv = make_float4(h.t, h.u, h.v, __int_as_float(found ? h.k : -1));
            occ = false;
            if (nee) {
                ++q_s;
                Hit hs;
                occ = trace_lane<WIDE, DEPTH, ORDERED, true, STATS>(tv, S, L, xyz(so), xyz(sd), so.w, sd.w, hs, stk, st_s);
            }
            const PState prev = o;
            nee = false;
            if (!shade_path(S, tv, L, RegState{prev, occ}, s, hv, o, nee, so, sd)) break;
        }
    }
    if (STATS) {  // the tail's own counter slots (kStatTail*), so stage rates stay per kernel
        flush_trav_stats(stat_shard(L.counters) + kStatTail, q_e, st_e);
        flush_trav_stats(stat_shard(L.counters) + kStatTailAny, q_s, st_s);
    }
}

// The launchers are split into parts so the build can compile this file as several translation units in parallel
// (Makefile: -DNH_WF_PART=k; each part instantiates only its own kernels). Without NH_WF_PART: every part.
#ifdef NH_WF_PART
#define NH_WF_HAS_PART(k) (NH_WF_PART == (k))
#else
#define NH_WF_HAS_PART(k) 1
#endif

namespace nh {

#if NH_WF_HAS_PART(0)
int tree_top_nodes() { return kTopNodes; }
#endif

// Persistent grids hold exactly the workgroups that are resident at once (occupancy of this
// instantiation x CUs, at most kPersistentBlocks -- the spill area's size): a workgroup that
// waits for a free slot would find the pool drained by the time it starts, or leave a tail.
template <auto KERN>
static void launch_persistent(int want, hipStream_t st, const DScene *S, const Traversal &tv, const WfLaunch &L) {
    static const int resident = [] {
        int per_cu = 0, dev = 0, n_cu = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, KERN, 128, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        if (hipGetDevice(&dev) == hipSuccess)
            (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
        return std::min(kPersistentBlocks, per_cu * std::max(n_cu, 1));
    }();
    hipLaunchKernelGGL(KERN, dim3(std::min(want, resident)), dim3(128), 0, st, S, tv, L);
}

#if NH_WF_HAS_PART(0) || NH_WF_HAS_PART(3)
template <int DEPTH>
static void launch_wf_trace_d(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats,
                              bool shadow, bool persistent, int wide, int bound, hipStream_t st) {
    // the queue length is only known on the device: size the grid from the host's upper bound
    // (the kernels stride over whatever the device count says)
    const int want = std::max(1, (bound + 127) / 128);
    const dim3 grid(std::min(want, persistent ? kPersistentBlocks : kTraceBlocksMax));
    if (persistent) {
#define NH_PT(A, O, T)                                                                               \
    do {                                                                                             \
        if (wide == 8) { if constexpr (O) launch_persistent<wf_trace_pt<DEPTH, O, A, T, 8>>(want, st, S, tv, L); } \
        else if (wide) launch_persistent<wf_trace_pt<DEPTH, O, A, T, 4>>(want, st, S, tv, L);              \
        else launch_persistent<wf_trace_pt<DEPTH, O, A, T, 0>>(want, st, S, tv, L);                  \
    } while (0)
        if (shadow) {
            if (ordered) { if (stats) NH_PT(true, true, true); else NH_PT(true, true, false); }
            else { if (stats) NH_PT(true, false, true); else NH_PT(true, false, false); }
        } else {
            if (ordered) { if (stats) NH_PT(false, true, true); else NH_PT(false, true, false); }
            else { if (stats) NH_PT(false, false, true); else NH_PT(false, false, false); }
        }
#undef NH_PT
        return;
    }
    const bool small = DEPTH == 16 && L.small_nodes + L.small_prims > 0;
    const size_t lds = small ? 16 * (size_t)(L.small_nodes + L.small_prims) + 8 * (size_t)L.small_leaves : 0;
#define NH_WF2(K, O, T, SM) hipLaunchKernelGGL((K<DEPTH, O, T, SM>), grid, dim3(128), lds, st, S, tv, L)
#define NH_WF(K, O, T) { if constexpr (DEPTH == 16) { if (small) NH_WF2(K, O, T, true); else NH_WF2(K, O, T, false); } \
                         else NH_WF2(K, O, T, false); }
    if (shadow) {
        if (ordered) { if (stats) NH_WF(wf_shadow, true, true) else NH_WF(wf_shadow, true, false) }
        else { if (stats) NH_WF(wf_shadow, false, true) else NH_WF(wf_shadow, false, false) }
    } else {
        if (ordered) { if (stats) NH_WF(wf_extend, true, true) else NH_WF(wf_extend, true, false) }
        else { if (stats) NH_WF(wf_extend, false, true) else NH_WF(wf_extend, false, false) }
    }
#undef NH_WF2
#undef NH_WF
}

#endif

void launch_wf_trace_deep(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats,
                          bool shadow, bool persistent, int wide, int bound, int depth, hipStream_t st);
#if NH_WF_HAS_PART(0)
void launch_wf_trace(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats, bool shadow,
                     bool persistent, int wide, int bound, int depth, hipStream_t st) {
    if (depth <= 16) launch_wf_trace_d<16>(S, tv, L, ordered, stats, shadow, persistent, wide, bound, st);
    else if (depth <= 32) launch_wf_trace_d<32>(S, tv, L, ordered, stats, shadow, persistent, wide, bound, st);
    else launch_wf_trace_deep(S, tv, L, ordered, stats, shadow, persistent, wide, bound, depth, st);
}
#endif
#if NH_WF_HAS_PART(3)
void launch_wf_trace_deep(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats,
                          bool shadow, bool persistent, int wide, int bound, int depth, hipStream_t st) {
    if (depth <= 64) launch_wf_trace_d<64>(S, tv, L, ordered, stats, shadow, persistent, wide, bound, st);
    else launch_wf_trace_d<128>(S, tv, L, ordered, stats, shadow, persistent, wide, bound, st);
}
#endif

#if NH_WF_HAS_PART(1)
template <int DEPTH>
static void launch_wf_tail_d(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats,
                             int wide, int bound, hipStream_t st) {
    // grid-stride; the wide variant's lanes own spill areas of the persistent grid's size
    const dim3 grid(std::min(std::max(1, (bound + 127) / 128), wide ? kPersistentBlocks : kTraceBlocksMax));
    const bool small = DEPTH == 16 && L.small_nodes + L.small_prims > 0;
    const size_t lds = small ? 16 * (size_t)(L.small_nodes + L.small_prims) + 8 * (size_t)L.small_leaves : 0;
#define NH_TL2(O, T, SM, W) hipLaunchKernelGGL((wf_tail<DEPTH, O, T, SM, W>), grid, dim3(128), lds, st, S, tv, L)
#define NH_TLW(O, T) { if (wide == 8) { if constexpr (O) NH_TL2(O, T, false, 8); } \
                       else if (wide) NH_TL2(O, T, false, 4); else NH_TL2(O, T, false, 0); }
#define NH_TL(O, T) { if constexpr (DEPTH == 16) { if (small) NH_TL2(O, T, true, 0); else NH_TLW(O, T) } \
                      else NH_TLW(O, T) }
    if (ordered) { if (stats) NH_TL(true, true) else NH_TL(true, false) }
    else { if (stats) NH_TL(false, true) else NH_TL(false, false) }
#undef NH_TL2
#undef NH_TLW
#undef NH_TL
}

void launch_wf_trace2(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats, int wide,
                      int bound, hipStream_t st) {
    // the wide trees are walked near-first only (nh_api.hip uses them for ordered traversals)
    (void)ordered;
    const int want = std::max(1, (bound + 127) / 128);
    if (wide == 8) {
        if (stats) launch_persistent<wf_trace_pt2<true, true, 8>>(want, st, S, tv, L);
        else launch_persistent<wf_trace_pt2<true, false, 8>>(want, st, S, tv, L);
        return;
    }
    if (stats) launch_persistent<wf_trace_pt2<true, true>>(want, st, S, tv, L);
    else launch_persistent<wf_trace_pt2<true, false>>(want, st, S, tv, L);
}

void launch_wf_tail(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats, int wide,
                    int bound, int depth, hipStream_t st) {
    if (depth <= 16) launch_wf_tail_d<16>(S, tv, L, ordered, stats, wide, bound, st);
    else if (depth <= 32) launch_wf_tail_d<32>(S, tv, L, ordered, stats, wide, bound, st);
    else if (depth <= 64) launch_wf_tail_d<64>(S, tv, L, ordered, stats, wide, bound, st);
    else launch_wf_tail_d<128>(S, tv, L, ordered, stats, wide, bound, st);
}


void launch_wf_bounce(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats, bool sort,
                      int bound, hipStream_t st) {
    int blocks = std::max(1, (bound + 255) / 256);
    blocks = (blocks + kQueueShards - 1) / kQueueShards * kQueueShards;
    const size_t lds = 16 * (size_t)rr_lds_f4(L);
#define NH_FB(O, T, SO) hipLaunchKernelGGL((wf_bounce<O, T, SO>), dim3(blocks), dim3(256), lds, st, S, tv, L)
    if (ordered) {
        if (stats) { if (sort) NH_FB(true, true, true); else NH_FB(true, true, false); }
        else { if (sort) NH_FB(true, false, true); else NH_FB(true, false, false); }
    } else {
        if (stats) { if (sort) NH_FB(false, true, true); else NH_FB(false, true, false); }
        else { if (sort) NH_FB(false, false, true); else NH_FB(false, false, false); }
    }
#undef NH_FB
}

#endif

#if NH_WF_HAS_PART(2)
void launch_wf_bounce_rr(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats, bool sort,
                         bool lean, bool nmap, int bound, hipStream_t st) {
    int blocks = std::max(1, (bound + NH_BOUNCE_TB - 1) / NH_BOUNCE_TB);
    blocks = (blocks + kQueueShards - 1) / kQueueShards * kQueueShards;
    const size_t lds = 16 * (size_t)rr_lds_f4(L);
#define NH_FB(O, T, SO) hipLaunchKernelGGL((wf_bounce_rr<O, T, SO>), dim3(blocks), dim3(NH_BOUNCE_TB), lds, st, S, tv, L)
#define NH_FBN(T, SO) hipLaunchKernelGGL((wf_bounce_rr<true, T, SO, false>), dim3(blocks), dim3(NH_BOUNCE_TB), lds, st, S, tv, L)
#define NH_FBF(T, SO) hipLaunchKernelGGL((wf_bounce_rr<true, T, SO, true, false>), dim3(blocks), dim3(NH_BOUNCE_TB), lds, st, S, tv, L)
    if (ordered && lean) {  // no discrete BSDF, no texture: wf_bounce_rr<.., FULL = false>
        if (stats) { if (sort) NH_FBN(true, true); else NH_FBN(true, false); }
        else { if (sort) NH_FBN(false, true); else NH_FBN(false, false); }
    } else if (ordered && !nmap) {  // the full body without normal maps: wf_bounce_rr<.., FULL = true, NMAP = false>
        if (stats) { if (sort) NH_FBF(true, true); else NH_FBF(true, false); }
        else { if (sort) NH_FBF(false, true); else NH_FBF(false, false); }
    } else if (ordered) {
        if (stats) { if (sort) NH_FB(true, true, true); else NH_FB(true, true, false); }
        else { if (sort) NH_FB(true, false, true); else NH_FB(true, false, false); }
    } else {
        if (stats) { if (sort) NH_FB(false, true, true); else NH_FB(false, true, false); }
        else { if (sort) NH_FB(false, false, true); else NH_FB(false, false, false); }
    }
#undef NH_FB
#undef NH_FBN
#undef NH_FBF
}

void launch_wf_tail_rr(const DScene *S, const Traversal &tv, const WfLaunch &L, bool ordered, bool stats, int bound,
                       bool specular, bool lean, bool nmap, hipStream_t st) {
    const char *e = std::getenv("NH_TAIL_WG");  // threads per tail workgroup: 64 (default) or 256
    const int tb = e && std::atoi(e) == 256 ? 256 : 64;
    // register budget, NH_TAIL_RR_WAVES=1|2|4: by default 1 wave/SIMD for scenes with mirror / dielectric BSDFs (their
    // long chains: shorter tails on C1 and C4, profiles/round4_session4_ab.txt) and 2 otherwise: spill-free (the
    // 4-wave budget spilled 448 B per lane inside the bounce loop), the tail 4-6 % shorter, the C2 step level with 4
    // waves (profiles/round6_ab_tail_waves.txt). lean (NH_TAIL_LEAN=0 off): the FULL = false body
    const char *w = std::getenv("NH_TAIL_RR_WAVES");
    const int waves = w ? (std::atoi(w) == 1 ? 1 : std::atoi(w) == 2 ? 2 : 4) : specular ? 1 : 2;
    const char *ln = std::getenv("NH_TAIL_LEAN");
    if (ln && ln[0] == '0') lean = false;
    const char *cp = std::getenv("NH_TAIL_COOP");  // lanes per path once <= 4 remain in a wave: 16 (default) or 1
    const int coop = cp && std::atoi(cp) == 1 ? 1 : 16;
    // one path per lane: the grid covers the bound (tail bounds are <= kTailCap paths)
    const dim3 grid(std::max(1, (bound + tb - 1) / tb));
    const size_t lds = 16 * (size_t)rr_lds_f4(L);
#define NH_TR(O, T)                                                                                         \
    do {                                                                                                    \
        if (tb == 256) hipLaunchKernelGGL((wf_tail_rr<O, T, 256, 1>), grid, dim3(256), lds, st, S, tv, L, coop); \
        else if (waves == 1 && !nmap && O)                                                                  \
            hipLaunchKernelGGL((wf_tail_rr<O, T, 64, 1, true, false>), grid, dim3(64), lds, st, S, tv, L, coop); \
        else if (waves == 1) hipLaunchKernelGGL((wf_tail_rr<O, T, 64, 1>), grid, dim3(64), lds, st, S, tv, L, coop); \
        else if (lean && waves == 2)                                                                        \
            hipLaunchKernelGGL((wf_tail_rr<O, T, 64, 2, false>), grid, dim3(64), lds, st, S, tv, L, coop);  \
        else if (waves == 2) hipLaunchKernelGGL((wf_tail_rr<O, T, 64, 2>), grid, dim3(64), lds, st, S, tv, L, coop); \
        else if (lean) hipLaunchKernelGGL((wf_tail_rr<O, T, 64, 4, false>), grid, dim3(64), lds, st, S, tv, L, coop); \
        else hipLaunchKernelGGL((wf_tail_rr<O, T, 64, 4>), grid, dim3(64), lds, st, S, tv, L, coop);           \
    } while (0)
    if (ordered) { if (stats) NH_TR(true, true); else NH_TR(true, false); }
    else { if (stats) NH_TR(false, true); else NH_TR(false, false); }
#undef NH_TR
}

#endif

#if NH_WF_HAS_PART(1)
void launch_wf_camera_rays(const DScene *S, const WfLaunch &L, int bound, hipStream_t st) {
    const int blocks = std::min(std::max(1, (bound + 255) / 256), kTraceBlocksMax);
    hipLaunchKernelGGL(wf_camera_rays, dim3(blocks), dim3(256), 0, st, S, L);
}
#endif

#if NH_WF_HAS_PART(1)
void launch_wf_counts(const unsigned *src, unsigned *host_dst, int n_copy, unsigned *zero, int n_zero, hipStream_t st) {
    hipLaunchKernelGGL(wf_counts_kernel, dim3(1), dim3(256), 0, st, src, host_dst, n_copy, zero, n_zero);
}

void launch_wf_pack_rr(const WfLaunch &L, const WfBuf &dst, unsigned *dst_counts, int bound, hipStream_t st) {
    hipLaunchKernelGGL(wf_pack_rr, dim3(std::max(1, (bound + 255) / 256)), dim3(256), 0, st, L, dst, dst_counts);
}

void launch_wf_shade(const DScene *S, const Traversal &tv, const WfLaunch &L, bool sort, bool nmap, int bound,
                     hipStream_t st) {
    // one 256-entry chunk per workgroup up to the bound; a multiple of kQueueShards (see wf_shade)
    int blocks = std::max(1, (bound + 255) / 256);
    blocks = (blocks + kQueueShards - 1) / kQueueShards * kQueueShards;
    if (sort && nmap) hipLaunchKernelGGL((wf_shade<true>), dim3(blocks), dim3(256), 0, st, S, tv, L);
    else if (sort) hipLaunchKernelGGL((wf_shade<true, false>), dim3(blocks), dim3(256), 0, st, S, tv, L);
    else if (nmap) hipLaunchKernelGGL((wf_shade<false>), dim3(blocks), dim3(256), 0, st, S, tv, L);
    else hipLaunchKernelGGL((wf_shade<false, false>), dim3(blocks), dim3(256), 0, st, S, tv, L);
}

#endif

}  // namespace nh
