// C-ABI device side of the MI355X path_mis hot path (declared in include/nori_hip.h).
//
// One nh_ctx per GPU owns every device allocation: scene records, the GPU BVH, the
// (W+2b)x(H+2b) RGBW master framebuffer and the per-chunk sample records. Rendering
// a sample range launches, per chunk of sample rounds, the path megakernel (one
// thread per (pixel, round)) and the ImageBlock splat gather on one HIP stream.
// This replaces the reference's OptiX state (include/nori/optix/OptixState*.cpp) and the
// CPU render loop (src/utils/render.cpp:232-459) behind the same plugin boundary.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <memory>
#include <thread>
#include <functional>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "nh_internal.h"
#include "nori_hip.h"

using nhd::DBsdf;
using nhd::DEmitter;
using nhd::DShape;

// ---- wavefront pipeline state (used by nh_render, see the pipeline section below) ----
constexpr int kRing = 4;   // bounce-count copies in flight per pool
// path pools in flight: while one drains its last bounces (long specular chains are a latency chain of
// hundreds of bounces) the next ones fill the GPU; NH_POOLS=1..kPools overrides the default (2 measured
// best: C4 2134-2147 Msamples/s vs 1913-1938 at 3 pools and 2078-2092 at 4; C2 / bumpy-1M unchanged)
constexpr int kPools = 4;
// tail slots: a chunk whose last live paths were handed off (RR-ahead pipeline, several pools) finishes its tail
// kernel and splat on one of these (own stream, small packed path buffer), while its pool takes the next chunk
constexpr int kTails = 3;
constexpr int kTailCap = 65536;  // paths a tail slot holds (the fused bounce's tail threshold is at most this)
#ifndef NH_DEFAULT_POOLS
#define NH_DEFAULT_POOLS 2
#endif
constexpr int kMaxStack = 128;  // deepest per-lane LDS stack of the binary-tree kernels (DEPTH template)

// one chunk of sample rounds of one nh_render call
struct WfJob {
    uint64_t seq;  // submission order = splat order
    int s0, rounds;
    uint64_t seed;
    bool ordered, stats;
    bool staged;   // splat layout, decided once when the chunk's buffers are sized (NH_SPLAT_FUSED read then only):
                   // per-(round, block) staging + merge, or the fused tile splat with no staging
    bool jit;      // NH_SPLAT_JITTER=stored (A/B): the first vertex stores each sample's jitter for the splat
};

// A path pool: the device state one chunk needs (double-buffered path state, shadow queue, sample
// records, block ImageBlocks, traversal spill area) plus its own stream, events and pinned
// count ring, and the host-side state machine of the chunk it is running.
struct WfPool {
    hipStream_t stream = nullptr;
    WfState wf{};
    std::vector<void *> bufs;
    size_t cap = 0;  // paths
    float *rec = nullptr;  // (r, g, b) per sample
    size_t rec_cap = 0;
    float2 *jit = nullptr;  // stored jitter (NH_SPLAT_JITTER=stored only)
    size_t jit_cap = 0;
    float4 *staging = nullptr;
    size_t staging_cap = 0;
    uint32_t *spill = nullptr;
    int spill_words = 0;
    unsigned *h_counts = nullptr;  // pinned: kRing bounce-count copies + one initial count slot
    hipEvent_t copy_ev[kRing] = {};
    std::vector<hipEvent_t> events;  // 4 per bounce (timing)
    hipEvent_t ev_begin = nullptr, ev_path = nullptr, ev_splat0 = nullptr, ev_splat = nullptr;
    hipEvent_t ev_handoff = nullptr;  // the packed tail paths are written (a tail slot's stream waits for it)
    enum State { IDLE, ENQUEUE, COUNTS, SPLAT, FINISH } state = IDLE;
    WfJob job{};
    WfLaunch L{};
    bool persistent = false, wide = false, trace2 = false, tail = false, draining = false;
    bool fused = false, sorted = false;  // one wf_bounce kernel per bounce (LDS-staged BVH); material-sorted queue
    bool rr = false;                     // fused kernels with the next vertex's Russian roulette ahead (wf_bounce_rr)
    bool shade_sorted = false;           // wf_shade entries in BSDF-type order (deep BVHs, mixed materials)
    int64_t tail_at = 0, drain_at = 0;
    int it = 0;
    std::vector<uint64_t> in_e, in_s;  // live paths / shadow rays entering each bounce
};

// RCCL communicators of one set of contexts (nh_reduce_framebuffers), created once and reused while the
// same contexts (by creation id, in the same order) reduce again; destroyed with the last holder.
struct CommSet {
    std::vector<uint64_t> ids;  // nh_ctx::id of the members, in rank order
    std::vector<int> devices;
    std::vector<ncclComm_t> comms;
    ~CommSet() {
        int cur = 0;
        const bool have = hipGetDevice(&cur) == hipSuccess;
        for (size_t i = 0; i < comms.size(); ++i) {
            (void)hipSetDevice(devices[i]);
            (void)ncclCommDestroy(comms[i]);
        }
        if (have) (void)hipSetDevice(cur);  // leave the caller's thread on its own device
    }
};

// restores the calling thread's current device when an entry point that walks several devices returns
struct DeviceGuard {
    int dev = 0;
    bool ok = false;
    DeviceGuard() { ok = hipGetDevice(&dev) == hipSuccess; }
    ~DeviceGuard() {
        if (ok) (void)hipSetDevice(dev);
    }
};

struct nh_ctx {
    uint64_t id = 0;  // unique per context (process lifetime): identifies comm-set members
    std::shared_ptr<CommSet> comms;
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // host copies needed to build primitive records
    std::vector<nh_shape> shapes;
    std::vector<float> V;
    std::vector<uint32_t> F;
    int width = 0, height = 0, border = 0, n_emitters = 0, integrator = 0;
    nh_filter filter{};
    nhd::DScene S{};
    nhd::DScene *d_scene = nullptr;  // device copy of S read by the kernels
    nhd::Traversal tv{};
    std::vector<void *> scene_bufs, bvh_bufs;
    bool has_scene = false, has_bvh = false;
    int depth = 0;
    int depth_wide = 0;  // stack bound of the wide traversal
    int wide_w = 4;      // children per wide node of tv.wnodes: 4, or 8 (NH_WIDE8=1)
    int n_node_f4 = 0, n_leaves = 0, n_prim_f4 = 0;  // GPU BVH sizes (float4 / int2 entries)
    std::vector<uint32_t> bvh_indices, shape_offset;
    std::vector<int> shape_bsdf_type;  // BSDF type of each shape (material key of the sorted queues)
    int n_bsdf_types = 0;              // distinct BSDF types in the scene
    bool specular = false;             // a mirror or dielectric BSDF: long discrete chains, long chunk tails
    bool textured = false;             // a BSDF with an albedo texture
    bool normal_mapped = false;        // a shape with a normal map (the full bounce / tail bodies' NMAP instantiation)
    float *fb = nullptr;
    size_t fb_floats = 0;
    float *rec = nullptr;  // (r, g, b) per sample
    size_t rec_cap = 0;  // entries
    int *pixel_list = nullptr, *pixel_map = nullptr, *block_rank = nullptr;
    int *block_ids = nullptr, *block_slot = nullptr;
    int *color_slots = nullptr;  // slots of the (bx + by) even blocks, then the odd ones (the pair splat's two launches)
    int n_blocks = 0, n_color0 = 0;
    float4 *staging = nullptr;
    size_t staging_cap = 0;  // float4 entries
    int n_list = 0, nbx = 0, nby = 0;
    std::vector<int32_t> list_key;
    bool have_list = false;
    unsigned long long *counters = nullptr;  // [0-3] queries, nodes, boxes, prims; [4] invalid; [8-11] wavefront shadow share
    nh_render_stats stats{};
    // wavefront pipeline (see "Wavefront pipeline" below): path pools, each on its own stream, and
    // the queue of chunks not yet started
    WfPool pools[kPools + kTails];  // [0, kPools): path pools; then the tail slots
    std::deque<WfJob> jobs;
    uint64_t job_seq = 0, splat_seq = 0;  // chunks are splatted into fb in submission order
    hipEvent_t fb_ev = nullptr;           // the last enqueued write of fb (clear or splat)
    bool fb_ev_set = false;
    uint64_t stats_comm_inits = 0;  // communicator cliques this context created as reduce root
};

extern "C" {
static void pool_free(WfPool &p);
static int pipeline_drain(nh_ctx *c);
}

namespace {

bool fail(nh_ctx *c, const std::string &m) {
    if (c) c->err = m;
    return false;
}

#define HIP_TRY(ctx, expr)                                                                               \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) {                                                                          \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                              \
            return NH_ERR_DEVICE;                                                                        \
        }                                                                                                \
    } while (0)

template <typename T>
int upload(nh_ctx *c, std::vector<void *> &owner, const T *src, size_t n, const T **dst) {
    void *p = nullptr;
    // a multiple of 16 B: the LDS staging of small scenes copies whole float4s of every record array
    size_t bytes = (std::max<size_t>(n * sizeof(T), 16) + 15) / 16 * 16;
    HIP_TRY(c, hipMalloc(&p, bytes));
    owner.push_back(p);
    if (n) HIP_TRY(c, hipMemcpyAsync(p, src, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
    *dst = reinterpret_cast<const T *>(p);
    return NH_OK;
}

void free_all(std::vector<void *> &v) {
    for (void *p : v) (void)hipFree(p);
    v.clear();
}

// BlockGenerator spiral order (src/utils/block.cpp:151-199) -> rank per block id
std::vector<int> spiral_rank(int w, int h, int bs, int &nbx, int &nby) {
    nbx = (int)std::ceil(w / (float)bs);
    nby = (int)std::ceil(h / (float)bs);
    std::vector<int> rank((size_t)nbx * nby, 0);
    int left = nbx * nby, dir = 0, bx = nbx / 2, by = nby / 2, steps_left = 1, num_steps = 1, r = 0;
    while (left > 0) {
        rank[(size_t)by * nbx + bx] = r++;
        if (--left == 0) break;
        do {
            switch (dir) {
                case 0: ++bx; break;
                case 1: ++by; break;
                case 2: --bx; break;
                case 3: --by; break;
            }
            if (--steps_left == 0) {
                dir = (dir + 1) % 4;
                if (dir == 0 || dir == 2) ++num_steps;
                steps_left = num_steps;
            }
        } while (bx < 0 || by < 0 || bx >= nbx || by >= nby);
    }
    return rank;
}

// DScene::emit_faces: each emitting face's vertices and the normal Mesh::sampleSurface computes for it
// (normalized(cross(p1 - p0, p2 - p0)), mesh.cpp:64-69), by the device functions the light sample would run
__global__ void emit_face_kernel(const float *V, const uint4 *tri, int n, float4 *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 t = tri[i];
    const nhd::F3 p0 = nhd::ldv(V, t.x), p1 = nhd::ldv(V, t.y), p2 = nhd::ldv(V, t.z);
    const nhd::F3 nn = nhd::normalized(nhd::cross(nhd::sub(p1, p0), nhd::sub(p2, p0)));
    out[3 * i] = make_float4(p0.x, p0.y, p0.z, nn.x);
    out[3 * i + 1] = make_float4(p1.x, p1.y, p1.z, nn.y);
    out[3 * i + 2] = make_float4(p2.x, p2.y, p2.z, nn.z);
}

// The position of each pixel's camera ray within one sample round of the reference's serial render order: blocks
// in BlockGenerator order (edge blocks clipped, block.cpp:174-176), then Independent::getSampleIndices' x-major
// pixel order (independent.cpp:85-99: x outer, y inner)
std::vector<uint32_t> serial_ray_index(int w, int h, int bs) {
    int nbx = 0, nby = 0;
    const std::vector<int> rank = spiral_rank(w, h, bs, nbx, nby);
    std::vector<int> by_rank(rank.size());
    for (size_t b = 0; b < rank.size(); ++b) by_rank[(size_t)rank[b]] = (int)b;
    std::vector<uint32_t> idx((size_t)w * h);
    uint32_t k = 0;
    for (int b : by_rank) {
        const int ox = (b % nbx) * bs, oy = (b / nbx) * bs;
        const int sx = std::min(bs, w - ox), sy = std::min(bs, h - oy);
        for (int x = 0; x < sx; ++x)
            for (int y = 0; y < sy; ++y) idx[(size_t)(oy + y) * w + (ox + x)] = k++;
    }
    return idx;
}

// pcg32::advance (pcg32.h:131-150) as an affine map of the state: advance(x, delta) = a * x + c (mod 2^64)
struct PcgAffine {
    uint64_t a = 1u, c = 0u;
};
PcgAffine pcg_affine(uint64_t inc, uint64_t delta) {
    uint64_t cur_mult = 0x5851f42d4c957f2dULL, cur_plus = inc;
    PcgAffine r;
    while (delta > 0) {
        if (delta & 1) {
            r.a *= cur_mult;
            r.c = r.c * cur_mult + cur_plus;
        }
        cur_plus = (cur_mult + 1) * cur_plus;
        cur_mult *= cur_mult;
        delta /= 2;
    }
    return r;
}
// g after f: x -> g.a * (f.a * x + f.c) + g.c
PcgAffine pcg_then(const PcgAffine &f, const PcgAffine &g) {
    PcgAffine r;
    r.a = g.a * f.a;
    r.c = g.a * f.c + g.c;
    return r;
}

// Lens-stream tables (nh_shade.h lens_uniform): camera ray k = round * W * H + pos[pixel] starts at draw 2k of the
// default-state stream, i.e. state(2k) = A_pos * (A_lo * S_hi + C_lo) + C_pos with round = 256 h + l,
// S_hi[h] = state(2 * 256 h * W * H), (A_lo, C_lo)[l] = advance by 2 l W H, (A_pos, C_pos) = advance by 2 pos:
// two 64-bit multiply-adds per ray instead of pcg_advance's O(log k) loop, and the same state (the maps commute)
constexpr uint64_t kLensDefaultState = 0x853c49e6748fea9bULL, kLensDefaultStream = 0xda3e39cb94b95bdbULL;
struct LensTables {
    std::vector<ulonglong2> pix, lo;
    std::vector<uint64_t> hi;
};
LensTables lens_tables(int w, int h) {
    LensTables t;
    const std::vector<uint32_t> pos = serial_ray_index(w, h, 32);
    const uint64_t wh = (uint64_t)w * (uint64_t)h;
    // per pixel, in serial order: advance by 2 pos
    std::vector<PcgAffine> by_pos(wh);
    const PcgAffine two = pcg_affine(kLensDefaultStream, 2);
    PcgAffine cur;
    for (uint64_t k = 0; k < wh; ++k) {
        by_pos[k] = cur;
        cur = pcg_then(cur, two);
    }
    t.pix.resize(wh);
    for (uint64_t i = 0; i < wh; ++i) t.pix[i] = make_ulonglong2(by_pos[pos[i]].a, by_pos[pos[i]].c);
    const PcgAffine round1 = pcg_affine(kLensDefaultStream, 2 * wh);
    cur = PcgAffine();
    t.lo.resize(nhd::kLensLo);
    for (int l = 0; l < nhd::kLensLo; ++l) {
        t.lo[l] = make_ulonglong2(cur.a, cur.c);
        cur = pcg_then(cur, round1);
    }
    const PcgAffine round_hi = pcg_affine(kLensDefaultStream, 2 * wh * (uint64_t)nhd::kLensLo);
    uint64_t st = kLensDefaultState;
    t.hi.resize(nhd::kLensHi);
    for (int hh = 0; hh < nhd::kLensHi; ++hh) {
        t.hi[hh] = st;
        st = round_hi.a * st + round_hi.c;
    }
    return t;
}

}  // namespace

extern "C" {

const char *nh_last_error(const nh_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int nh_get_device_count(int *n) {
    if (!n) return NH_ERR_INVALID;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return NH_OK;
}

int nh_create(int device, nh_ctx **out) {
    if (!out) return NH_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return NH_ERR_DEVICE;
    auto *c = new nh_ctx();
    static std::atomic<uint64_t> next_id{1};
    c->id = next_id++;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->counters, kStatShards * kStatStride * sizeof(unsigned long long)) != hipSuccess ||
        hipEventCreateWithFlags(&c->fb_ev, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return NH_ERR_DEVICE;
    }
    (void)hipMemset(c->counters, 0, kStatShards * kStatStride * sizeof(unsigned long long));
    *out = c;
    return NH_OK;
}

void nh_destroy(nh_ctx *c) {
    if (!c) return;
    DeviceGuard guard;
    (void)hipSetDevice(c->device);
    (void)pipeline_drain(c);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_all(c->scene_bufs);
    free_all(c->bvh_bufs);
    (void)hipFree(c->fb);
    (void)hipFree(c->rec);
    (void)hipFree(c->pixel_list);
    (void)hipFree(c->pixel_map);
    (void)hipFree(c->block_rank);
    (void)hipFree(c->block_ids);
    (void)hipFree(c->block_slot);
    (void)hipFree(c->color_slots);
    (void)hipFree(c->staging);
    (void)hipFree(c->counters);
    (void)hipFree(c->d_scene);
    for (WfPool &p : c->pools) pool_free(p);
    c->comms.reset();  // the communicators go with the last context of their set
    if (c->fb_ev) (void)hipEventDestroy(c->fb_ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

// Can a light sample ever be non-finite, or land on a discrete-BSDF (mirror / dielectric) shading point? No, when:
// every emitter is an area light or the envmap, with finite radiance (and a finite constant env colour); every
// shape's box is finite and well inside float range (no overflow in the sample's squared distance); and the box of
// every area light's shape, widened by a relative margin for rounding, is disjoint from the widened box of every
// shape with a discrete BSDF (so the sampled point p and the shading point ref always differ: a zero distance is the
// only way the area light's pdf becomes 0/0, emitter_pdf). Then the wavefront shade may skip the light sample of a
// discrete BSDF sample, which is zeroed by the reference anyway (path_mis.cpp:136-140).
// A non-constant envmap also needs a finite, positive luminance normalization.
static bool nee_finite(const nh_scene_desc *d) {
    auto fin = [](float x) { return std::fabs(x) < 1e15f; };
    for (uint32_t i = 0; i < d->n_emitters; ++i) {
        const nh_emitter &e = d->emitters[i];
        if (e.type == NH_EMITTER_POINT) return false;
        for (int k = 0; k < 3; ++k)
            if (!std::isfinite(e.radiance[k])) return false;
    }
    if (d->envmap >= 0 && d->env.constant && d->env.rgba)
        for (int k = 0; k < 3; ++k)
            if (!std::isfinite(d->env.rgba[k])) return false;
    // a PNG envmap's luminance table must be a proper distribution: an all-black image leaves its normalization
    // 1/0, and the reference's light sample is then NaN, which ImageBlock drops with the whole sample
    if (d->envmap >= 0 && !d->env.constant && !(std::isfinite(d->env.normalization) && d->env.normalization > 0.f))
        return false;
    struct Box { float lo[3], hi[3]; };
    auto widened = [&](const nh_shape &s, Box &b) {
        float ext = 0.f;
        for (int k = 0; k < 3; ++k) {
            if (!fin(s.bbox_min[k]) || !fin(s.bbox_max[k])) return false;
            ext = std::max(ext, std::max(std::fabs(s.bbox_min[k]), std::fabs(s.bbox_max[k])));
        }
        const float m = 1e-3f * ext + 1e-6f;
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = s.bbox_min[k] - m;
            b.hi[k] = s.bbox_max[k] + m;
        }
        return true;
    };
    for (uint32_t i = 0; i < d->n_shapes; ++i) {
        const nh_shape &si = d->shapes[i];
        Box bi;
        if (!widened(si, bi)) return false;
        if (si.emitter < 0) continue;
        for (uint32_t j = 0; j < d->n_shapes; ++j) {
            const nh_shape &sj = d->shapes[j];
            const int t = d->bsdfs[sj.bsdf].type;
            if (t != NH_BSDF_MIRROR && t != NH_BSDF_DIELECTRIC) continue;
            Box bj;
            if (!widened(sj, bj)) return false;
            bool apart = false;
            for (int k = 0; k < 3; ++k) apart = apart || bi.hi[k] < bj.lo[k] || bj.hi[k] < bi.lo[k];
            if (!apart) return false;
        }
    }
    return true;
}

int nh_upload_scene(nh_ctx *c, const nh_scene_desc *d) {
    if (!c || !d) return NH_ERR_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc_ = pipeline_drain(c)) return rc_;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (d->camera.width <= 0 || d->camera.height <= 0) return fail(c, "invalid camera resolution"), NH_ERR_INVALID;
    if (d->envmap >= 0) {
        const nh_envmap &e = d->env;
        if ((uint32_t)d->envmap >= d->n_emitters || d->emitters[d->envmap].type != NH_EMITTER_ENVMAP)
            return fail(c, "envmap index does not name an envmap emitter"), NH_ERR_INVALID;
        if (e.width <= 0 || e.height <= 0 || !e.rgba || !e.cdf) return fail(c, "invalid envmap texture"), NH_ERR_INVALID;
    }
    free_all(c->scene_bufs);
    free_all(c->bvh_bufs);
    c->has_scene = c->has_bvh = false;
    c->have_list = false;

    std::vector<DShape> ds(d->n_shapes);
    for (uint32_t i = 0; i < d->n_shapes; ++i) {
        const nh_shape &s = d->shapes[i];
        if (s.bsdf < 0 || (uint32_t)s.bsdf >= d->n_bsdfs) return fail(c, "shape without a valid BSDF"), NH_ERR_INVALID;
        DShape &o = ds[i];
        std::memset(&o, 0, sizeof(o));
        o.type = s.type;
        o.bsdf = s.bsdf;
        o.emitter = s.emitter;
        o.v_off = (int)s.v_offset;
        o.f_off = (int)s.f_offset;
        o.n_faces = (int)s.n_faces;
        o.has_n = s.has_normals;
        o.has_uv = s.has_uvs;
        o.cx = s.center[0]; o.cy = s.center[1]; o.cz = s.center[2];
        o.radius = s.radius;
        o.pdf_off = (int)s.pdf_offset;
        o.pdf_norm = s.pdf_normalization;
        if (s.normal_map > d->n_textures || (s.normal_map && !d->textures))
            return fail(c, "shape normal map index out of range"), NH_ERR_INVALID;
        // bit 0: uv read (textured albedo or normal map); bits 1+: 1 + the normal map's texture index
        o.tex_uv = ((int)s.normal_map << 1) |
                   ((d->bsdfs[s.bsdf].type == NH_BSDF_DIFFUSE && d->bsdfs[s.bsdf].albedo_texture != 0) || s.normal_map
                        ? 1 : 0);
        o.ef_off = -1;
    }
    // emitting meshes without vertex normals: one emit_faces record per face (vertex index triples here)
    std::vector<uint4> ef_tri;
    if (!(std::getenv("NH_EMIT_FACES") && std::getenv("NH_EMIT_FACES")[0] == '0'))
        for (uint32_t i = 0; i < d->n_shapes; ++i) {
            const nh_shape &s = d->shapes[i];
            if (s.type != NH_SHAPE_MESH || s.emitter < 0 || s.has_normals) continue;
            if ((uint64_t)s.f_offset + s.n_faces > d->n_faces) return fail(c, "shape faces out of range"), NH_ERR_INVALID;
            ds[i].ef_off = (int)ef_tri.size();
            for (uint32_t f = 0; f < s.n_faces; ++f) {
                const uint32_t *fi = &d->F[3 * ((size_t)s.f_offset + f)];
                const uint32_t i0 = s.v_offset + fi[0], i1 = s.v_offset + fi[1], i2 = s.v_offset + fi[2];
                if (i0 >= d->n_vertices || i1 >= d->n_vertices || i2 >= d->n_vertices)
                    return fail(c, "face vertex index out of range"), NH_ERR_INVALID;
                ef_tri.push_back(make_uint4(i0, i1, i2, 0u));
            }
        }
    std::vector<DBsdf> db(d->n_bsdfs);
    for (uint32_t i = 0; i < d->n_bsdfs; ++i) {
        const nh_bsdf &b = d->bsdfs[i];
        DBsdf &o = db[i];
        std::memset(&o, 0, sizeof(o));
        o.type = b.type;
        o.ar = b.albedo[0]; o.ag = b.albedo[1]; o.ab = b.albedo[2];
        o.alpha = b.alpha; o.int_ior = b.int_ior; o.ext_ior = b.ext_ior; o.ks = b.ks;
        o.kr = b.kd[0]; o.kg = b.kd[1]; o.kb = b.kd[2];
        if (b.albedo_texture > d->n_textures || (b.albedo_texture && !d->textures))
            return fail(c, "BSDF albedo texture index out of range"), NH_ERR_INVALID;
        o.tex = b.type == NH_BSDF_DIFFUSE ? (int)b.albedo_texture : 0;
    }
    std::vector<nhd::DTex> dt(d->n_textures);
    for (uint32_t i = 0; i < d->n_textures; ++i) {
        const nh_texture &t = d->textures[i];
        nhd::DTex &o = dt[i];
        std::memset(&o, 0, sizeof(o));
        if (t.type < NH_TEXTURE_CONSTANT || t.type > NH_TEXTURE_PNG) return fail(c, "unknown texture type"), NH_ERR_INVALID;
        if (t.type == NH_TEXTURE_PNG &&
            (t.width <= 0 || t.height <= 0 || !d->texels ||
             t.texel_offset + (uint64_t)t.width * (uint64_t)t.height > d->n_texels))
            return fail(c, "png texture outside the scene's texels"), NH_ERR_INVALID;
        o.type = t.type;
        o.w = t.width; o.h = t.height; o.spherical = t.spherical;
        o.v1r = t.value1[0]; o.v1g = t.value1[1]; o.v1b = t.value1[2];
        o.v2r = t.value2[0]; o.v2g = t.value2[1]; o.v2b = t.value2[2];
        o.dx = t.delta[0]; o.dy = t.delta[1]; o.sx = t.scale[0]; o.sy = t.scale[1];
        o.su = t.scale_u; o.sv = t.scale_v; o.ou = t.offset_u; o.ov = t.offset_v;
        o.off = (long long)t.texel_offset;
        std::memcpy(o.rot, t.rotation, sizeof(o.rot));
        o.linear = t.type == NH_TEXTURE_PNG && t.linear;
        o.intensity = t.intensity;
    }
    std::vector<DEmitter> de(d->n_emitters);
    for (uint32_t i = 0; i < d->n_emitters; ++i) {
        const nh_emitter &e = d->emitters[i];
        if (e.type == NH_EMITTER_ENVMAP && (int32_t)i != d->envmap)
            return fail(c, "only one environment map per scene is supported"), NH_ERR_UNSUPPORTED;
        DEmitter &o = de[i];
        std::memset(&o, 0, sizeof(o));
        o.type = e.type;
        o.shape = e.shape;
        o.lr = e.radiance[0]; o.lg = e.radiance[1]; o.lb = e.radiance[2];
        o.px = e.position[0]; o.py = e.position[1]; o.pz = e.position[2];
    }
    nhd::DScene &S = c->S;
    std::memset(&S, 0, sizeof(S));
    int rc;
    const size_t nv = d->n_vertices;
    if ((rc = upload(c, c->scene_bufs, ds.data(), ds.size(), &S.shapes))) return rc;
    if ((rc = upload(c, c->scene_bufs, db.data(), db.size(), &S.bsdfs))) return rc;
    if ((rc = upload(c, c->scene_bufs, de.data(), de.size(), &S.emitters))) return rc;
    if ((rc = upload(c, c->scene_bufs, d->emitter_cdf, (size_t)d->n_emitters + 1, &S.emitter_cdf))) return rc;
    if ((rc = upload(c, c->scene_bufs, d->V, 3 * nv, &S.V))) return rc;
    if ((rc = upload(c, c->scene_bufs, d->N, 3 * nv, &S.N))) return rc;
    if ((rc = upload(c, c->scene_bufs, d->UV, 2 * nv, &S.UV))) return rc;
    if ((rc = upload(c, c->scene_bufs, d->T, 3 * nv, &S.T))) return rc;
    if ((rc = upload(c, c->scene_bufs, d->BT, 3 * nv, &S.BT))) return rc;
    if ((rc = upload(c, c->scene_bufs, d->F, 3 * (size_t)d->n_faces, &S.F))) return rc;
    S.emit_faces = nullptr;
    if (!ef_tri.empty()) {
        const uint4 *tri = nullptr;
        if ((rc = upload(c, c->scene_bufs, ef_tri.data(), ef_tri.size(), &tri))) return rc;
        float4 *faces = nullptr;
        HIP_TRY(c, hipMalloc(&faces, 3 * ef_tri.size() * sizeof(float4)));
        c->scene_bufs.push_back(faces);
        const int n = (int)ef_tri.size();
        hipLaunchKernelGGL(emit_face_kernel, dim3((n + 255) / 256), dim3(256), 0, c->stream, S.V, tri, n, faces);
        HIP_TRY(c, hipGetLastError());
        S.emit_faces = faces;
    }
    if ((rc = upload(c, c->scene_bufs, d->area_cdf, (size_t)d->n_area_cdf, &S.area_cdf))) return rc;
    if (!dt.empty() && (rc = upload(c, c->scene_bufs, dt.data(), dt.size(), &S.texs))) return rc;
    if (d->n_texels) {
        const float *tx = nullptr;
        if ((rc = upload(c, c->scene_bufs, d->texels, 4 * (size_t)d->n_texels, &tx))) return rc;
        S.texels = reinterpret_cast<const float4 *>(tx);
    }
    S.envmap = d->envmap;
    if (d->envmap >= 0) {
        const nh_envmap &e = d->env;
        const size_t texels = (size_t)e.width * (size_t)e.height;
        const float *rgba = nullptr;
        if ((rc = upload(c, c->scene_bufs, e.rgba, 4 * texels, &rgba))) return rc;
        S.env_rgba = reinterpret_cast<const float4 *>(rgba);
        if ((rc = upload(c, c->scene_bufs, e.cdf, texels + 1, &S.env_cdf))) return rc;
        // guide table of the CDF search (nh_device.h dpdf_sample_guided): guide[j] = the first index i in [0, n]
        // with !(cdf[i] < j / 2^bits) (n + 1 if none), the same float comparison as the device's search; about 4
        // texels per bracket (NH_ENV_GUIDE=0: the plain search)
        S.env_guide = nullptr;
        S.env_guide_bits = 0;
        // (only for a non-decreasing CDF without NaN, where the first entry not below x is monotone in x)
        bool monotone = true;
        for (size_t i = 0; i <= texels && monotone; ++i)
            monotone = !std::isnan(e.cdf[i]) && (i == 0 || !(e.cdf[i] < e.cdf[i - 1]));
        if (monotone && texels >= 64 && !(std::getenv("NH_ENV_GUIDE") && std::getenv("NH_ENV_GUIDE")[0] == '0')) {
            int bits = 0;
            while (bits < 20 && ((size_t)1 << (bits + 2)) < texels) ++bits;
            const size_t M = (size_t)1 << bits;
            std::vector<int> guide(M + 1);
            size_t i = 0;
            for (size_t j = 0; j <= M; ++j) {
                const float t = (float)((double)j / (double)M);  // exact: j / 2^bits
                while (i <= texels && e.cdf[i] < t) ++i;
                guide[j] = (int)i;
            }
            const int *g = nullptr;
            if ((rc = upload(c, c->scene_bufs, guide.data(), guide.size(), &g))) return rc;
            HIP_TRY(c, hipStreamSynchronize(c->stream));  // (guide is a local)
            S.env_guide = g;
            S.env_guide_bits = bits;
        }
        S.env_w = e.width;
        S.env_h = e.height;
        S.env_spherical = e.spherical;
        std::memcpy(S.env_rot, e.rotation, sizeof(S.env_rot));
        S.env_constant = e.constant;
        S.env_norm = e.normalization;
        S.env_su = e.scale_u;
        S.env_sv = e.scale_v;
        S.env_ou = e.offset_u;
        S.env_ov = e.offset_v;
        S.env_r = e.radiance[0];
        S.env_g = e.radiance[1];
        S.env_b = e.radiance[2];
    }
    S.n_emitters = (int)d->n_emitters;
    S.nee_finite = nee_finite(d) ? 1 : 0;
    if (d->integrator < NH_INTEGRATOR_PATH_MIS || d->integrator > NH_INTEGRATOR_NORMALS)
        return fail(c, "unknown integrator"), NH_ERR_INVALID;
    S.integrator = d->integrator;
    for (int i = 0; i < 3; ++i) S.ndir[i] = d->normals_direction[i];
    std::memcpy(S.s2c, d->camera.sample_to_camera, sizeof(S.s2c));
    std::memcpy(S.c2w, d->camera.camera_to_world, sizeof(S.c2w));
    {  // camera_ray's origin for a (0, 0, 0) local origin (nh_shade.h): the same operations in the same order
        float ow[4];
        const float z = 0.0f;
        for (int i = 0; i < 4; ++i) {
            float acc = S.c2w[4 * i] * z;
            acc = acc + S.c2w[4 * i + 1] * z;
            acc = acc + S.c2w[4 * i + 2] * z;
            acc = acc + S.c2w[4 * i + 3] * 1.0f;
            ow[i] = acc;
        }
        for (int i = 0; i < 3; ++i) S.cam_o[i] = ow[i] / ow[3];
    }
    S.inv_w = d->camera.inv_output_size[0];
    S.inv_h = d->camera.inv_output_size[1];
    S.near_clip = d->camera.near_clip;
    S.far_clip = d->camera.far_clip;
    S.width = d->camera.width;
    S.height = d->camera.height;
    // depth of field (perspective.cpp:114: lensRadius > Epsilon): each pixel's camera-ray position within a sample
    // round of the serial render order, which places its lens sample in the camera's static pcg32 stream
    // (nh_shade.h lens_uniform)
    S.dof = d->camera.lens_radius > 1e-4f ? 1 : 0;
    S.lens_radius = d->camera.lens_radius;
    S.focal_distance = d->camera.focal_distance;
    S.lens_rtl = d->camera.lens_draw_order == NH_LENS_DRAWS_RTL ? 1 : 0;
    S.lens_pix = S.lens_lo = nullptr;
    S.lens_hi = nullptr;
    if (S.dof) {
        const LensTables lt = lens_tables(S.width, S.height);
        if ((rc = upload(c, c->scene_bufs, lt.pix.data(), lt.pix.size(), &S.lens_pix))) return rc;
        if ((rc = upload(c, c->scene_bufs, lt.lo.data(), lt.lo.size(), &S.lens_lo))) return rc;
        if ((rc = upload(c, c->scene_bufs, lt.hi.data(), lt.hi.size(), &S.lens_hi))) return rc;
        HIP_TRY(c, hipStreamSynchronize(c->stream));  // (the tables are locals)
    }
    S.filter_radius = d->filter.radius;
    S.lookup = d->filter.lookup_factor;
    S.border = d->filter.border;
    std::memcpy(S.table, d->filter.table, sizeof(S.table));

    c->shapes.assign(d->shapes, d->shapes + d->n_shapes);
    c->shape_bsdf_type.clear();
    unsigned types = 0;
    for (uint32_t i = 0; i < d->n_shapes; ++i) {
        const int t = d->bsdfs[d->shapes[i].bsdf].type & 3;
        c->shape_bsdf_type.push_back(t);
        types |= 1u << t;
    }
    c->n_bsdf_types = __builtin_popcount(types);
    c->specular = (types & ((1u << NH_BSDF_MIRROR) | (1u << NH_BSDF_DIELECTRIC))) != 0;
    // any BSDF with an albedo texture or shape with a normal map (wf_bounce_rr's lean instantiation has no lookup)
    c->textured = false;
    for (uint32_t i = 0; i < d->n_bsdfs; ++i) c->textured = c->textured || d->bsdfs[i].albedo_texture != 0;
    c->normal_mapped = false;
    for (uint32_t i = 0; i < d->n_shapes; ++i) c->normal_mapped = c->normal_mapped || d->shapes[i].normal_map != 0;
    c->textured = c->textured || c->normal_mapped;
    c->V.assign(d->V, d->V + 3 * nv);
    c->F.assign(d->F, d->F + 3 * (size_t)d->n_faces);
    c->width = d->camera.width;
    c->height = d->camera.height;
    c->border = d->filter.border;
    c->filter = d->filter;
    c->n_emitters = (int)d->n_emitters;
    c->integrator = S.integrator;

    // master ImageBlock
    (void)hipFree(c->fb);
    c->fb = nullptr;
    c->fb_floats = 4 * (size_t)(c->width + 2 * c->border) * (size_t)(c->height + 2 * c->border);
    HIP_TRY(c, hipMalloc(&c->fb, c->fb_floats * sizeof(float)));
    HIP_TRY(c, hipMemsetAsync(c->fb, 0, c->fb_floats * sizeof(float), c->stream));
    // block spiral ranks
    auto rank = spiral_rank(c->width, c->height, 32, c->nbx, c->nby);
    (void)hipFree(c->block_rank);
    HIP_TRY(c, hipMalloc(&c->block_rank, rank.size() * sizeof(int)));
    HIP_TRY(c, hipMemcpyAsync(c->block_rank, rank.data(), rank.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->has_scene = true;
    return NH_OK;
}

// Isolated spheres (nhd::kPrimIsolated, nh_traverse.h trace_next): a dielectric sphere's record whose box grown by 2m
// lies apart from every other primitive's box gets the bit (only a dielectric sends its rays inside: for the others
// the sphere test would almost always be a wasted one), and m in its record 1 .x (only read by the sphere shortcut). m is
// 1e-4 of the scene's largest extent -- far above the float rounding of any hit point, far below the gaps of
// real scenes (the Cornell box's spheres clear its floor by 6e-3). Boxes are compared in double, closed: a box
// that touches or holds a NaN is not apart. NH_ISO_SPHERE=0 leaves every sphere unmarked (every ray walks the
// tree). Spheres x primitives box tests, skipped (no marks) past 2e8. Returns the number marked.
// Primitives whose box meets the query box [qlo, qhi] (double): a walk of the uploaded binary tree (child boxes in
// the parent, float) with the query grown by `slack` at the node tests, so a node box that rounds inward of its
// primitives' double boxes cannot hide one; the primitive boxes themselves decide (was a linear scan of
// every primitive per dielectric sphere).
static void prims_near_box(const std::vector<float4> &nodes, const std::vector<int2> &leaves, int root_kind,
                           const double qlo[3], const double qhi[3], double slack, std::vector<uint32_t> &out) {
    out.clear();
    auto leaf = [&](int l) {
        const int2 lf = leaves[(size_t)l];
        for (int k = 0; k < lf.y; ++k) out.push_back((uint32_t)(lf.x + k));
    };
    if (root_kind == 2) leaf(0);
    if (root_kind != 1) return;
    auto meets = [&](const float lo[3], const float hi[3]) {
        for (int a = 0; a < 3; ++a)
            if ((double)hi[a] < qlo[a] - slack || (double)lo[a] > qhi[a] + slack) return false;
        return true;
    };
    std::vector<int> st{0};
    while (!st.empty()) {
        const int g = st.back();
        st.pop_back();
        const float4 *n = &nodes[4 * (size_t)g];
        const float llo[3] = {n[0].x, n[0].y, n[0].z}, lhi[3] = {n[0].w, n[1].x, n[1].y};
        const float rlo[3] = {n[1].z, n[1].w, n[2].x}, rhi[3] = {n[2].y, n[2].z, n[2].w};
        int4 r4;
        std::memcpy(&r4, &n[3], sizeof(int4));
        const int ref[2] = {r4.x, r4.y};
        const bool hit[2] = {meets(llo, lhi), meets(rlo, rhi)};
        for (int ch = 0; ch < 2; ++ch)
            if (hit[ch]) {
                if (ref[ch] >= 0) st.push_back(ref[ch]);
                else leaf(~ref[ch]);
            }
    }
}

// Marks dielectric spheres whose box, grown by 2m (m = 1e-4 of the scene extent), is apart from every other
// primitive's box (the isolated-sphere closest hit of nh_traverse.h `trace_next`); m goes into the record.
static int mark_isolated_spheres(std::vector<float4> &prims, const std::vector<float4> &nodes,
                                 const std::vector<int2> &leaves, int root_kind) {
    const char *e = std::getenv("NH_ISO_SPHERE");
    if (e && e[0] == '0') return 0;
    const size_t n = prims.size() / 3;
    std::vector<size_t> sph;
    for (size_t k = 0; k < n; ++k) {
        int bits;
        std::memcpy(&bits, &prims[3 * k + 2].w, 4);
        if ((bits & nhd::kPrimSphere) && ((bits >> nhd::kPrimMatShift) & 3) == nhd::BSDF_DIELECTRIC) sph.push_back(k);
    }
    if (sph.empty()) return 0;
    auto prim_box = [&](size_t k, double lo[3], double hi[3]) {
        const float4 *p = &prims[3 * k];
        int bits;
        std::memcpy(&bits, &p[2].w, 4);
        for (int a = 0; a < 3; ++a) {
            const double v0 = a == 0 ? p[0].x : a == 1 ? p[0].y : p[0].z;
            if (bits & nhd::kPrimSphere) {
                lo[a] = v0 - (double)p[0].w;
                hi[a] = v0 + (double)p[0].w;
            } else {
                const double v1 = a == 0 ? p[1].x : a == 1 ? p[1].y : p[1].z;
                const double v2 = a == 0 ? p[2].x : a == 1 ? p[2].y : p[2].z;
                lo[a] = std::min(v0, std::min(v1, v2));
                hi[a] = std::max(v0, std::max(v1, v2));
            }
        }
    };
    // the scene extent from the root box (the union of every primitive's float box)
    double ext = 0.0, mag = 0.0;
    if (root_kind == 0) return 0;
    {
        double slo[3] = {INFINITY, INFINITY, INFINITY}, shi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t k = 0; k < n; ++k) {
            double lo[3], hi[3];
            prim_box(k, lo, hi);
            for (int a = 0; a < 3; ++a) {
                slo[a] = std::min(slo[a], lo[a]);
                shi[a] = std::max(shi[a], hi[a]);
            }
        }
        ext = std::max(shi[0] - slo[0], std::max(shi[1] - slo[1], shi[2] - slo[2]));
        for (int a = 0; a < 3; ++a) mag = std::max(mag, std::max(std::fabs(slo[a]), std::fabs(shi[a])));
    }
    if (!(ext > 0.0) || !std::isfinite(ext)) return 0;
    const float m = (float)(1e-4 * ext);
    // far above the float rounding (2^-24 relative) of any node box coordinate in the scene
    const double slack = 1e-6 * (ext + mag);
    int marked = 0;
    std::vector<uint32_t> near;
    for (size_t s : sph) {
        const float4 a = prims[3 * s];
        if (!(a.w > 0.f) || !std::isfinite(a.w) || !std::isfinite(a.x) || !std::isfinite(a.y) || !std::isfinite(a.z))
            continue;
        const double g = (double)a.w + 2.0 * (double)m;
        const double glo[3] = {(double)a.x - g, (double)a.y - g, (double)a.z - g};
        const double ghi[3] = {(double)a.x + g, (double)a.y + g, (double)a.z + g};
        prims_near_box(nodes, leaves, root_kind, glo, ghi, slack, near);
        bool apart = true;
        for (uint32_t k : near) {
            if (k == s) continue;
            double lo[3], hi[3];
            prim_box(k, lo, hi);
            bool sep = false;
            for (int ax = 0; ax < 3; ++ax) sep = sep || hi[ax] < glo[ax] || lo[ax] > ghi[ax];
            if (!sep) {
                apart = false;
                break;
            }
        }
        if (!apart) continue;
        int bits;
        std::memcpy(&bits, &prims[3 * s + 2].w, 4);
        bits |= nhd::kPrimIsolated;
        std::memcpy(&prims[3 * s + 2].w, &bits, 4);
        prims[3 * s + 1].x = m;
        ++marked;
    }
    return marked;
}

// W-wide collapse (W = 4 or 8) of the GPU binary tree (nh_traverse.h Tracer4 / Tracer8): every wide node takes
// the two children of a binary node and, while it has fewer than W, replaces its largest-area inner child by that
// child's two children in place (left-first DFS order of the slots is kept). Wide nodes are numbered depth first,
// the first child next to its parent. Boxes are the binary tree's own. An 8-wide node is two 4-wide lines
// (children 0-3, 4-7), each in the 4-wide layout.
static std::vector<float4> collapse_wide(const std::vector<float4> &nodes, const std::vector<int2> &leaves,
                                         int &depth_out, int W = 4) {
    struct Child {
        float mn[3], mx[3];
        int ref;  // binary: >= 0 inner node, < 0 leaf ~index
    };
    auto child = [&](int g, int side) {
        const float *f = reinterpret_cast<const float *>(&nodes[4 * (size_t)g]);
        Child ch;
        const int o = side ? 6 : 0;
        for (int i = 0; i < 3; ++i) { ch.mn[i] = f[o + i]; ch.mx[i] = f[o + 3 + i]; }
        int refs[2];
        std::memcpy(refs, &nodes[4 * (size_t)g + 3], 8);
        ch.ref = refs[side];
        return ch;
    };
    auto area = [](const Child &c) {
        const float x = c.mx[0] - c.mn[0], y = c.mx[1] - c.mn[1], z = c.mx[2] - c.mn[2];
        return x * y + y * z + z * x;
    };
    std::vector<float4> wide;
    depth_out = 0;
    if (nodes.empty()) return wide;
    const int lines = W / 4, nf4 = lines * nhd::kWideF4;
    std::function<int(int, int)> make = [&](int g, int depth) -> int {
        depth_out = std::max(depth_out, depth);
        const int idx = (int)(wide.size() / nf4);
        wide.resize(wide.size() + nf4);
        std::vector<Child> ch{child(g, 0), child(g, 1)};
        while ((int)ch.size() < W) {
            int best = -1;
            float best_a = -1.f;
            for (int i = 0; i < (int)ch.size(); ++i)
                if (ch[i].ref >= 0 && area(ch[i]) > best_a) { best = i; best_a = area(ch[i]); }
            if (best < 0) break;
            const int gi = ch[best].ref;
            ch[best] = child(gi, 1);
            ch.insert(ch.begin() + best, child(gi, 0));
        }
        int refs[8];
        float box[6][8];
        for (int j = 0; j < 8; ++j) {
            refs[j] = nhd::kWideEmpty;
            for (int a = 0; a < 3; ++a) { box[a][j] = 0.f; box[3 + a][j] = 0.f; }
        }
        for (int j = 0; j < (int)ch.size(); ++j) {
            for (int a = 0; a < 3; ++a) { box[a][j] = ch[j].mn[a]; box[3 + a][j] = ch[j].mx[a]; }
            if (ch[j].ref >= 0) {
                refs[j] = make(ch[j].ref, depth + 1);
            } else {
                const int2 lf = leaves[(size_t)~ch[j].ref];
                refs[j] = lf.y > 0 ? ~lf.x : nhd::kWideEmpty;  // an empty leaf holds nothing to hit
            }
        }
        for (int h = 0; h < lines; ++h) {
            float4 *n = &wide[(size_t)idx * nf4 + (size_t)h * nhd::kWideF4];
            for (int a = 0; a < 6; ++a)
                n[a] = make_float4(box[a][4 * h], box[a][4 * h + 1], box[a][4 * h + 2], box[a][4 * h + 3]);
            std::memcpy(&n[6], refs + 4 * h, 16);
            n[7] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        return idx;
    };
    make(0, 1);
    return wide;
}

// Number the K wide nodes most rays visit first, so the persistent traversal can keep them in LDS: the
// connected top of the tree grown from the root by the largest child-box surface area (a ray's chance
// of entering a box grows with its area). The other nodes keep their depth-first order. Renumbering
// moves no box and changes no visit order: every answer is unchanged. Returns the top's size.
static int number_top_first(std::vector<float4> &wide, const float root_min[3], const float root_max[3], int K,
                            int W = 4) {
    const int lines = W / 4, nf4 = lines * nhd::kWideF4;
    const int n = (int)(wide.size() / nf4);
    if (n == 0 || K <= 0) return 0;
    auto area = [](const float *mn, const float *mx) {
        const float x = mx[0] - mn[0], y = mx[1] - mn[1], z = mx[2] - mn[2];
        return x * y + y * z + z * x;
    };
    std::vector<int> order;  // new index -> old index, for the top
    std::vector<char> in_top(n, 0);
    std::vector<std::pair<float, int>> heap{{area(root_min, root_max), 0}};
    while (!heap.empty() && (int)order.size() < K) {
        std::pop_heap(heap.begin(), heap.end());
        const int g = heap.back().second;
        heap.pop_back();
        order.push_back(g);
        in_top[g] = 1;
        for (int h = 0; h < lines; ++h) {
            const float *f = reinterpret_cast<const float *>(&wide[(size_t)g * nf4 + (size_t)h * nhd::kWideF4]);
            int refs[4];
            std::memcpy(refs, f + 24, 16);
            for (int j = 0; j < 4; ++j) {
                if (refs[j] < 0) continue;  // a leaf or an empty slot
                const float mn[3] = {f[j], f[4 + j], f[8 + j]}, mx[3] = {f[12 + j], f[16 + j], f[20 + j]};
                heap.push_back({area(mn, mx), refs[j]});
                std::push_heap(heap.begin(), heap.end());
            }
        }
    }
    std::vector<int> perm(n);  // old -> new
    for (int i = 0; i < (int)order.size(); ++i) perm[order[i]] = i;
    int next = (int)order.size();
    for (int g = 0; g < n; ++g)
        if (!in_top[g]) perm[g] = next++;
    std::vector<float4> out(wide.size());
    for (int g = 0; g < n; ++g) {
        float4 *dst = &out[(size_t)perm[g] * nf4];
        std::memcpy(dst, &wide[(size_t)g * nf4], nf4 * sizeof(float4));
        for (int h = 0; h < lines; ++h) {
            int refs[4];
            std::memcpy(refs, &dst[h * nhd::kWideF4 + 6], 16);
            for (int j = 0; j < 4; ++j)
                if (refs[j] >= 0) refs[j] = perm[refs[j]];
            std::memcpy(&dst[h * nhd::kWideF4 + 6], refs, 16);
        }
    }
    wide.swap(out);
    return (int)order.size();
}

int nh_upload_bvh(nh_ctx *c, const nh_bvh_desc *b) {
    if (!c || !b) return NH_ERR_INVALID;
    if (!c->has_scene) return fail(c, "nh_upload_bvh: upload the scene first"), NH_ERR_STATE;
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc_ = pipeline_drain(c)) return rc_;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    free_all(c->bvh_bufs);
    c->has_bvh = false;
    // primitive id -> (shape, local)
    std::vector<uint32_t> off(1, 0u);
    for (auto &s : c->shapes) off.push_back(off.back() + (s.type == NH_SHAPE_MESH ? s.n_faces : 1u));
    if (b->n_indices != off.back()) return fail(c, "BVH primitive count does not match the scene"), NH_ERR_INVALID;
    if (b->n_indices > 0 && b->n_nodes == 0) return fail(c, "empty BVH for a non-empty scene"), NH_ERR_INVALID;

    std::vector<float4> nodes;
    std::vector<int2> leaves;
    uint32_t tree_depth = 0;
    nhd::DScene &S = c->S;
    if (b->n_nodes == 0) {
        S.root_kind = 0;
    } else {
        const nh_bvh_node *N = b->nodes;
        for (int i = 0; i < 3; ++i) { S.root_min[i] = N[0].bbox_min[i]; S.root_max[i] = N[0].bbox_max[i]; }
        if (N[0].word0 & 1u) {
            S.root_kind = 2;
            leaves.push_back(make_int2((int)N[0].word1, (int)(N[0].word0 >> 1)));
        } else {
            S.root_kind = 1;
            // DFS (left first) over inner nodes assigning GPU ids in visit order
            // (the tree's depth is measured here, not taken from nh_bvh_desc::max_depth: it sizes the
            // traversal stacks)
            std::vector<int> gid(b->n_nodes, -1);
            std::vector<uint32_t> order;
            std::vector<std::pair<uint32_t, uint32_t>> st{{0u, 0u}};  // (node, level)
            while (!st.empty()) {
                const uint32_t i = st.back().first, lvl = st.back().second;
                st.pop_back();
                tree_depth = std::max(tree_depth, lvl);
                if (N[i].word0 & 1u) continue;
                if (gid[i] >= 0) return fail(c, "corrupt BVH: node reached twice"), NH_ERR_INVALID;
                gid[i] = (int)order.size();
                order.push_back(i);
                if (N[i].word1 >= b->n_nodes || i + 1 >= b->n_nodes)
                    return fail(c, "corrupt BVH child index"), NH_ERR_INVALID;
                st.push_back({N[i].word1, lvl + 1});
                st.push_back({i + 1, lvl + 1});
            }
            nodes.resize(4 * order.size());
            auto child_ref = [&](uint32_t ch) -> int {
                if (N[ch].word0 & 1u) {
                    leaves.push_back(make_int2((int)N[ch].word1, (int)(N[ch].word0 >> 1)));
                    return ~(int)(leaves.size() - 1);
                }
                return gid[ch];
            };
            for (size_t g = 0; g < order.size(); ++g) {
                uint32_t i = order[g];
                const nh_bvh_node &L = N[i + 1], &R = N[N[i].word1];
                int lr = child_ref(i + 1), rr = child_ref(N[i].word1);
                nodes[4 * g] = make_float4(L.bbox_min[0], L.bbox_min[1], L.bbox_min[2], L.bbox_max[0]);
                nodes[4 * g + 1] = make_float4(L.bbox_max[1], L.bbox_max[2], R.bbox_min[0], R.bbox_min[1]);
                nodes[4 * g + 2] = make_float4(R.bbox_min[2], R.bbox_max[0], R.bbox_max[1], R.bbox_max[2]);
                int4 r4 = make_int4(lr, rr, 0, 0);
                std::memcpy(&nodes[4 * g + 3], &r4, sizeof(int4));
            }
        }
    }
    // primitives in leaf order
    std::vector<float4> prims(3 * (size_t)b->n_indices);
    for (uint32_t k = 0; k < b->n_indices; ++k) {
        uint32_t g = b->indices[k];
        if (g >= off.back()) return fail(c, "BVH index out of range"), NH_ERR_INVALID;
        uint32_t s = (uint32_t)(std::upper_bound(off.begin(), off.end(), g) - off.begin()) - 1;
        uint32_t local = g - off[s];
        const nh_shape &sh = c->shapes[s];
        float4 *p = &prims[3 * (size_t)k];
        int si = (int)s, one = 1, zero = 0;
        float fs, f1, f0;
        std::memcpy(&fs, &si, 4);
        std::memcpy(&f1, &one, 4);
        std::memcpy(&f0, &zero, 4);
        const int mat = c->shape_bsdf_type[s] << nhd::kPrimMatShift;
        if (sh.type == NH_SHAPE_SPHERE) {
            const int flags = 1 | mat;
            std::memcpy(&f1, &flags, 4);
            p[0] = make_float4(sh.center[0], sh.center[1], sh.center[2], sh.radius);
            p[1] = make_float4(0, 0, 0, fs);
            p[2] = make_float4(0, 0, 0, f1);
        } else {
            std::memcpy(&f0, &mat, 4);
            const uint32_t *f = &c->F[3 * ((size_t)sh.f_offset + local)];
            const float *p0 = &c->V[3 * ((size_t)sh.v_offset + f[0])], *p1 = &c->V[3 * ((size_t)sh.v_offset + f[1])],
                        *p2 = &c->V[3 * ((size_t)sh.v_offset + f[2])];
            int li = (int)local;
            float fl;
            std::memcpy(&fl, &li, 4);
            p[0] = make_float4(p0[0], p0[1], p0[2], fl);
            p[1] = make_float4(p1[0], p1[1], p1[2], fs);
            p[2] = make_float4(p2[0], p2[1], p2[2], f0);
        }
    }
    S.iso_spheres = mark_isolated_spheres(prims, nodes, leaves, S.root_kind);
    // leaf-end bits: the 4-wide traversal walks a leaf's records until this bit
    for (const int2 &lf : leaves)
        if (lf.y > 0) {
            float4 &w = prims[3 * ((size_t)lf.x + lf.y - 1) + 2];
            int bits;
            std::memcpy(&bits, &w.w, 4);
            bits |= nhd::kPrimLeafEnd;
            std::memcpy(&w.w, &bits, 4);
        }
    // The binary-tree kernels keep a per-lane stack of at most kMaxStack entries (the deferred
    // children of one root-to-leaf path; the reference keeps 64, bvh.cpp:403)
    if (tree_depth + 2 > (uint32_t)kMaxStack)
        return fail(c, "BVH deeper than " + std::to_string(kMaxStack - 2) + " levels is not supported"), NH_ERR_UNSUPPORTED;
    // the wide tree of the persistent kernels: 4-wide, or 8-wide with NH_WIDE8=1 (A/B)
    c->wide_w = std::getenv("NH_WIDE8") && std::getenv("NH_WIDE8")[0] == '1' ? 8 : 4;
    int depth4 = 0;
    std::vector<float4> wide = collapse_wide(nodes, leaves, depth4, c->wide_w);
    // the top of the tree the persistent kernels stage in LDS (NH_TREE_TOP: its size, 0 = none): the same bytes for
    // both widths
    int top_k = nh::tree_top_nodes() * 4 / c->wide_w;
    if (const char *e = std::getenv("NH_TREE_TOP")) top_k = std::min(std::max(0, std::atoi(e)), top_k);
    c->tv.n_top = S.root_kind == 1 ? number_top_first(wide, S.root_min, S.root_max, top_k, c->wide_w) : 0;
    int rc;
    c->n_node_f4 = (int)nodes.size();
    c->n_leaves = (int)leaves.size();
    c->n_prim_f4 = (int)prims.size();
    // one zero record past the end: the 4-wide traversal loads record k+1 together with record k
    // (and tests it only when k does not end its leaf)
    prims.resize(prims.size() + 3, make_float4(0.f, 0.f, 0.f, 0.f));
    if ((rc = upload(c, c->bvh_bufs, nodes.data(), nodes.size(), &c->tv.nodes))) return rc;
    if ((rc = upload(c, c->bvh_bufs, leaves.data(), leaves.size(), &c->tv.leaves))) return rc;
    if ((rc = upload(c, c->bvh_bufs, prims.data(), prims.size(), &c->tv.prims))) return rc;
    c->tv.wnodes = nullptr;
    if (!wide.empty() && (rc = upload(c, c->bvh_bufs, wide.data(), wide.size(), &c->tv.wnodes))) return rc;
    // deferred entries: at most W - 1 per wide level (+1 slack)
    c->depth_wide = (c->wide_w - 1) * depth4 + 1;
    S.nodes = c->tv.nodes;
    S.prims = c->tv.prims;
    c->bvh_indices.assign(b->indices, b->indices + b->n_indices);
    c->shape_offset = off;
    c->depth = (int)tree_depth + 2;
    if (!c->d_scene) HIP_TRY(c, hipMalloc(&c->d_scene, sizeof(nhd::DScene)));
    HIP_TRY(c, hipMemcpyAsync(c->d_scene, &c->S, sizeof(nhd::DScene), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->has_bvh = true;
    return NH_OK;
}

int nh_trace_rays(nh_ctx *c, const nh_ray_soa *r, int32_t n, int32_t any_hit, int32_t traversal, nh_hit_soa *out) {
    if (!c || !r || !out || n < 0) return NH_ERR_INVALID;
    if (!c->has_bvh) return fail(c, "nh_trace_rays: no BVH uploaded"), NH_ERR_STATE;
    if (n == 0) return NH_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc_ = pipeline_drain(c)) return rc_;
    std::vector<void *> tmp;
    const float *in[8];
    const float *src[8] = {r->ox, r->oy, r->oz, r->dx, r->dy, r->dz, r->mint, r->maxt};
    int rc;
    for (int i = 0; i < 8; ++i)
        if ((rc = upload(c, tmp, src[i], (size_t)n, &in[i]))) { free_all(tmp); return rc; }
    RayBatch rb{in[0], in[1], in[2], in[3], in[4], in[5], in[6], in[7]};
    HitBatch hb{};
    void *p;
    size_t nn = (size_t)n;
    HIP_TRY(c, hipMalloc(&p, nn)); tmp.push_back(p); hb.hit = (uint8_t *)p;
    HIP_TRY(c, hipMalloc(&p, nn * 4)); tmp.push_back(p); hb.t = (float *)p;
    HIP_TRY(c, hipMalloc(&p, nn * 4)); tmp.push_back(p); hb.u = (float *)p;
    HIP_TRY(c, hipMalloc(&p, nn * 4)); tmp.push_back(p); hb.v = (float *)p;
    HIP_TRY(c, hipMalloc(&p, nn * 4)); tmp.push_back(p); hb.k = (int *)p;
    if (traversal == NH_TRAVERSAL_WIDE && c->tv.wnodes) {
        HIP_TRY(c, hipMalloc(&p, nn * (size_t)c->depth_wide * sizeof(int2)));
        tmp.push_back(p);
        nh::launch_trace_wide(c->d_scene, c->tv, rb, hb, n, any_hit != 0, true, false, (int2 *)p, c->depth_wide,
                              c->counters, c->stream, c->wide_w);
    } else {
        nh::launch_trace(c->d_scene, c->tv, rb, hb, n, any_hit != 0, traversal != NH_TRAVERSAL_REFERENCE, false,
                         c->depth, c->counters, c->stream);
    }
    HIP_TRY(c, hipGetLastError());
    std::vector<int> k(nn);
    HIP_TRY(c, hipMemcpyAsync(out->hit, hb.hit, nn, hipMemcpyDeviceToHost, c->stream));
    if (!any_hit) {
        if (out->t) HIP_TRY(c, hipMemcpyAsync(out->t, hb.t, nn * 4, hipMemcpyDeviceToHost, c->stream));
        if (out->u) HIP_TRY(c, hipMemcpyAsync(out->u, hb.u, nn * 4, hipMemcpyDeviceToHost, c->stream));
        if (out->v) HIP_TRY(c, hipMemcpyAsync(out->v, hb.v, nn * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipMemcpyAsync(k.data(), hb.k, nn * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    free_all(tmp);
    if (!any_hit)
        for (size_t i = 0; i < nn; ++i) {
            uint32_t prim = 0xffffffffu, shape = 0xffffffffu;
            if (k[i] >= 0) {
                prim = c->bvh_indices[(size_t)k[i]];
                shape = (uint32_t)(std::upper_bound(c->shape_offset.begin(), c->shape_offset.end(), prim) -
                                   c->shape_offset.begin()) - 1;
            }
            if (out->prim) out->prim[i] = prim;
            if (out->shape) out->shape[i] = shape;
        }
    return NH_OK;
}


// ============================================================================================
// Wavefront pipeline
//
// nh_render splits its sample rounds into chunks (jobs) and runs each chunk on a path pool:
// camera paths -> {extend, any-hit, shade} per bounce until no path is alive (the tail kernel
// finishes the last few in place) -> ImageBlock splat of the chunk's sample records into the
// master framebuffer. Queue lengths stay on the device (nh_internal.h count slots); the host
// enqueues bounce i+1 before it reads bounce i's counts (2 KB into pinned memory), so the GPU never
// idles on a host round trip, and exactly one empty bounce is enqueued at the end.
//
// The last bounces of a chunk carry few paths whose traversals are long latency chains: a lone
// pool leaves most of the GPU idle there. kPools pools on their own streams overlap that drain
// with the next chunk's full bounces (of the same call or of the next nh_render call: a wavefront
// nh_render returns once every chunk it submitted has started and every running pool is draining;
// anything that reads results -- nh_synchronize, nh_get_framebuffer, nh_get_stats, ... -- first
// runs the pipeline to completion). Splats are enqueued in submission order, each waiting for the
// previous write of the framebuffer, so the master ImageBlock receives chunks in the serial
// reference's order and the image is bit-identical to a one-pool run.
// ============================================================================================

constexpr size_t kWfBytesPerPath = 2 * (16 * 6 + 8 + 1) + 36;  // two buffers + shadow queue

static int pool_alloc(nh_ctx *c, WfPool &p, size_t n, size_t rec_n, size_t staging_f4, bool jit = false) {
    if (!p.stream) {  // the stream is created last: a pool with a stream has all of these
        if (!p.h_counts && hipHostMalloc(reinterpret_cast<void **>(&p.h_counts),
                                         (kRing * 2 * kCountGroup + kCountSlot) * sizeof(unsigned)) != hipSuccess) {
            p.h_counts = nullptr;
            return fail(c, "hipHostMalloc failed"), NH_ERR_DEVICE;
        }
        for (hipEvent_t &e : p.copy_ev)
            if (!e) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (hipEvent_t *e : {&p.ev_begin, &p.ev_path, &p.ev_splat0, &p.ev_splat})
            if (!*e) HIP_TRY(c, hipEventCreate(e));
        if (!p.ev_handoff) HIP_TRY(c, hipEventCreateWithFlags(&p.ev_handoff, hipEventDisableTiming));
        HIP_TRY(c, hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking));
    }
    if (p.cap < n) {
        free_all(p.bufs);
        p.wf = WfState{};
        p.cap = 0;
        auto alloc = [&](auto *&ptr, size_t count) -> bool {
            void *q = nullptr;
            if (hipMalloc(&q, count * sizeof(*ptr)) != hipSuccess) return false;
            p.bufs.push_back(q);
            ptr = static_cast<std::remove_reference_t<decltype(ptr)>>(q);
            return true;
        };
        WfState &W = p.wf;
        const size_t nq = n + (size_t)(kQueueShards + 2) * 256;  // shard segments round up to whole shade blocks
        bool ok = true;
        for (WfBuf &B : W.buf)
            ok = ok && alloc(B.ray_o, nq) && alloc(B.ray_d, nq) && alloc(B.hit, nq) && alloc(B.rng, nq) &&
                 alloc(B.li, nq) && alloc(B.thr, nq) && alloc(B.pend, nq) && alloc(B.occl, nq);
        ok = ok && alloc(W.sh_o, nq) && alloc(W.sh_d, nq) && alloc(W.sh_slot, nq) && alloc(W.counts, 2 * kCountSlot);
        if (!ok) {
            free_all(p.bufs);
            p.wf = WfState{};
            return fail(c, "hipMalloc failed for wavefront path state"), NH_ERR_DEVICE;
        }
        p.cap = n;
    }
    // the chunk's sample records: owned by whichever pool or tail slot holds the chunk (they move with it)
    if (p.rec_cap < rec_n) {
        (void)hipFree(p.rec);
        p.rec = nullptr;
        p.rec_cap = 0;
        HIP_TRY(c, hipMalloc(&p.rec, rec_n * kRecFloats * sizeof(float)));
        p.rec_cap = rec_n;
    }
    if (jit && p.jit_cap < rec_n) {
        (void)hipFree(p.jit);
        p.jit = nullptr;
        p.jit_cap = 0;
        HIP_TRY(c, hipMalloc(&p.jit, rec_n * sizeof(float2)));
        p.jit_cap = rec_n;
    }
    if (p.staging_cap < staging_f4) {
        (void)hipFree(p.staging);
        p.staging = nullptr;
        p.staging_cap = 0;
        HIP_TRY(c, hipMalloc(&p.staging, staging_f4 * sizeof(float4)));
        p.staging_cap = staging_f4;
    }
    return NH_OK;
}

static void pool_free(WfPool &p) {
    free_all(p.bufs);
    (void)hipFree(p.rec);
    (void)hipFree(p.jit);
    (void)hipFree(p.staging);
    (void)hipFree(p.spill);
    if (p.h_counts) (void)hipHostFree(p.h_counts);
    for (hipEvent_t e : p.events) (void)hipEventDestroy(e);
    for (hipEvent_t e : p.copy_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {p.ev_begin, p.ev_path, p.ev_splat0, p.ev_splat, p.ev_handoff})
        if (e) (void)hipEventDestroy(e);
    if (p.stream) (void)hipStreamDestroy(p.stream);
    p = WfPool{};
}

static SplatLaunch make_splat(const nh_ctx *c, const float *rec, uint64_t seed, int s0, float4 *staging, int rounds,
                              bool staged) {
    SplatLaunch P{};
    P.staged = staged ? 1 : 0;
    P.fb = c->fb;
    P.width = c->width;
    P.height = c->height;
    P.border = c->border;
    P.reach = (int)std::floor(c->filter.radius + 0.5f);
    P.nbx = c->nbx;
    P.n_rounds = rounds;
    P.n_list = c->n_list;
    P.pixel_map = c->pixel_map;
    P.block_rank = c->block_rank;
    P.rec = rec;
    P.seed = seed;
    P.s0 = s0;
    P.radius = c->filter.radius;
    P.lookup = c->filter.lookup_factor;
    std::memcpy(P.table, c->filter.table, sizeof(P.table));
    P.blocks = c->block_ids;
    P.block_slot = c->block_slot;
    P.n_blocks = c->n_blocks;
    P.color_slots = c->color_slots;
    P.n_color0 = c->n_color0;
    P.staging = staging;
    return P;
}

// the splat layout of a chunk starting now: staged pair, or the fused tile splat (NH_SPLAT_FUSED=1)
static bool splat_staged(const nh_ctx *c) {
    return nh::splat_uses_staging(c->border, (int)std::floor(c->filter.radius + 0.5f));
}
// float4 entries of one (round, block) ImageBlock in the splat's staging buffer (0: the fused splat stages nothing)
static size_t block_px(const nh_ctx *c, bool staged) {
    if (!staged) return 0;
    return (size_t)(32 + 2 * c->border) * (size_t)stage_pitch(32 + 2 * c->border);
}

// path pools driven by pipeline_run (NH_POOLS: 1 = no overlap, for A/B and tests). Scenes with mirror or
// dielectric BSDFs get a third pool: their chunks end in tails of discrete chains that survive Russian roulette
// with probability 0.99 per bounce (path_mis.cpp:58-70), 5-6 ms whatever the chunk size, longer than a C1
// chunk's bounce phase; with three pools two tails overlap the next chunk (C1 2744 -> 3321 Msamples/s; C2,
// perf-1M and C5 unchanged). Each pool's stream needs its own hardware queue (GPU_MAX_HW_QUEUES >= 5; with HIP's
// default of 4, two pool streams share one and a tail blocks the other pool's bounces).
static int active_pools(const nh_ctx *c) {
    const char *np = std::getenv("NH_POOLS");
    const int def = c->specular ? NH_DEFAULT_POOLS + 1 : NH_DEFAULT_POOLS;
    return std::max(1, std::min(kPools, np ? std::atoi(np) : def));
}

// asynchronous tails: NH_TAIL_ASYNC=1 (default off until measured faster than in-place tails)
static bool tail_async_enabled() {
    const char *e = std::getenv("NH_TAIL_ASYNC");
    return e && e[0] == '1';
}

// start job j on idle pool p: buffers, traversal choice, initial queue (all n_paths camera paths)
static int pool_start(nh_ctx *c, WfPool &p, const WfJob &job) {
    WfJob j = job;
    j.staged = splat_staged(c);  // the staging below is sized for this layout; the chunk's splat uses the same
    const char *jv = std::getenv("NH_SPLAT_JITTER");
    j.jit = jv && std::strcmp(jv, "stored") == 0;
    const int n_paths = j.rounds * c->n_list;
    int rc = pool_alloc(c, p, (size_t)n_paths, (size_t)n_paths, (size_t)j.rounds * c->n_blocks * block_px(c, j.staged), j.jit);
    if (rc) return rc;
    // the other pools in use get the same capacity now (idle ones only: nothing of theirs is in
    // flight), so the first render call, not a later one, pays for their allocation
    for (int i = 0; i < active_pools(c); ++i) {
        WfPool &o = c->pools[i];
        if (&o == &p || o.state != WfPool::IDLE) continue;
        if ((rc = pool_alloc(c, o, (size_t)n_paths, (size_t)n_paths, (size_t)j.rounds * c->n_blocks * block_px(c, j.staged), j.jit)))
            return rc;
    }
    // so do the idle tail slots' record and staging buffers: chunks hand theirs over at a tail hand-off and take the
    // slot's, and a pool that had to grow them later would free and allocate inside the pipeline (hipFree waits
    // for the whole device: a 6-9 ms stall behind the running tails)
    if (active_pools(c) > 1 && tail_async_enabled())
        for (int i = kPools; i < kPools + kTails; ++i) {
            WfPool &o = c->pools[i];
            if (o.state != WfPool::IDLE) continue;
            if ((rc = pool_alloc(c, o, (size_t)kTailCap, (size_t)n_paths, (size_t)j.rounds * c->n_blocks * block_px(c, j.staged), j.jit)))
                return rc;
        }
    p.job = j;
    WfLaunch &L = p.L;
    L = WfLaunch{};
    L.st = p.wf;
    L.n_paths = n_paths;
    L.n_list = c->n_list;
    L.s0 = j.s0;
    L.seed = j.seed;
    L.pixel_list = c->pixel_list;
    L.rec = p.rec;
    L.jit = j.jit ? p.jit : nullptr;
    L.counters = c->counters;
    // scenes whose BVH fits in a few KB (the Cornell box: < 1 KB) are traversed from an LDS copy
    const size_t scene_bytes = 16 * (size_t)(c->n_node_f4 + c->n_prim_f4) + 8 * (size_t)c->n_leaves;
    bool small = scene_bytes <= kSmallSceneBytes;
    if (const char *e = std::getenv("NH_LDS_SCENE")) small = small && e[0] != '0';
    if (small) {
        L.small_nodes = c->n_node_f4;
        L.small_leaves = c->n_leaves;
        L.small_prims = c->n_prim_f4;
        // the flat triangles' shading frames staged beside the records (hit_info reads them instead of a
        // normalize + frame construction per hit) while they add little LDS
        L.small_frames = c->n_prim_f4 / 3 <= kSmallFramesMaxPrims;
        if (const char *e = std::getenv("NH_LDS_FRAMES")) L.small_frames = L.small_frames && e[0] != '0';
    }
    const int per_chunk = 256;  // wf_shade's chunk
    const int max_chunks = (n_paths + per_chunk - 1) / per_chunk;
    L.seg_cap = (max_chunks + kQueueShards - 1) / kQueueShards * per_chunk;
    // persistent traversal pays off on deep BVHs (long, divergent traversals); cbox-like scenes
    // traverse faster with one ray per lane
    p.persistent = c->depth > 20;
    if (const char *e = std::getenv("NH_PERSISTENT")) p.persistent = e[0] == '1';
    // the persistent kernels generate pinhole camera rays only (camera_ray<false>: the lens arithmetic spilled their
    // refill code): for a thin-lens scene wf_camera_rays writes bounce 0's rays first (WfLaunch::cam_rays)
    // the persistent kernels walk the 4-wide collapse of the tree (half the dependent node fetches)
    // unless the reference's own visit order was asked for
    p.wide = p.persistent && j.ordered && c->tv.wnodes != nullptr;
    if (const char *e = std::getenv("NH_WIDE")) p.wide = p.wide && e[0] != '0';
    // both queries of a bounce in one persistent launch (one tail per bounce instead of two) while the tree fits in
    // the 256 MB MALL (perf-1M +10 %, C3 +7 %); past it the two queries' node sets compete for the cache in one
    // grid (C5, 0.8 GB: 22.3 GB of HBM traffic per fused launch vs 6.9 + 12.3 GB split, 15 % slower), so the
    // closest-hit and any-hit launches stay separate. NH_TRACE2=0|1 overrides.
    p.trace2 = p.wide && scene_bytes <= (size_t)256 << 20;
    if (const char *e = std::getenv("NH_TRACE2")) p.trace2 = p.wide && e[0] != '0';
    c->stats.trace_fused = p.trace2 ? 1 : 0;
    // spill words per lane: binary entries are one word, wide entries two (8-B aligned)
    const int spill_words = p.wide ? 2 * c->depth_wide : (c->depth + 1) / 2 * 2;
    if (p.persistent && p.spill_words < spill_words) {
        HIP_TRY(c, hipStreamSynchronize(p.stream));
        (void)hipFree(p.spill);
        p.spill = nullptr;
        p.spill_words = 0;
        HIP_TRY(c, hipMalloc(&p.spill, (size_t)kPersistentBlocks * 128 * spill_words * sizeof(uint32_t)));
        p.spill_words = spill_words;
    }
    // BVHs staged in LDS: one fused bounce kernel instead of extend + any-hit + shade, its output queue
    // sorted by the next hit's BSDF type when the scene mixes BSDF types
    p.fused = small && !p.persistent && c->depth <= 16;
    if (const char *e = std::getenv("NH_FUSED")) p.fused = p.fused && e[0] != '0';
    p.sorted = p.fused && c->n_bsdf_types > 1;
    p.rr = p.fused;
    if (const char *e = std::getenv("NH_RR_AHEAD")) p.rr = p.fused && e[0] != '0';
    // material-sorted shading on deep BVHs is measured slower (C3 1640 -> 1590, C5 1542 -> 1526 Msamples/s:
    // the extra hit read and barriers cost more than the divergence saved): off unless NH_SORT_SHADE=1
    p.shade_sorted = false;
    if (const char *e = std::getenv("NH_SORT_SHADE")) p.shade_sorted = !p.fused && e[0] == '1';
    if (const char *e = std::getenv("NH_SORT")) p.sorted = p.fused && e[0] == '1';
    c->stats.fused_bounce = p.fused ? 1 : 0;
    c->stats.node_bytes = p.wide ? 16 * nhd::kWideF4 * (c->wide_w / 4) : 64;
    c->stats.lds_scene = small && !p.persistent && c->depth <= 16 ? 1 : 0;  // the SMALL instantiations (DEPTH 16)
    L.trav_spill = p.spill;
    L.spill_depth = p.spill_words;
    // measured on 16.7M-path chunks: C2 3025 / 3030 / 2692 Msamples/s at 64k / 262k / 1M,
    // bumpy-1M 708 / 744 / 739 / 603 at 64k / 262k / 1M / 3M; 67M-path C4 chunks 2102 / 2206 / 2226 / 2209
    // at 1M / 262k / 131k / 64k
    // at 67M / 16.7M paths with the fused bounce (round 2): C4 3134 / 3229 / 3254 Msamples/s at
    // 262k / 64k / 32k, C2 3680 / 3717 at 262k / 64k, bumpy-1M (persistent traversal) 1404 / 1378 at
    // 262k / 64k -- an LDS-staged bounce stays efficient down to fewer paths than a deep-tree one
    // round 5, with the scratch-free traversal: 64k / 32k / 16k / 8k -- C2 5567 / 5591 / 5577 / 5585, C1 4409 / 4408 /
    // 4459, C4 4891 / 4906 / 4929 Msamples/s (profiles/round5_ab_tail_threshold.txt)
    p.tail_at = p.fused ? std::min<int64_t>(std::max<int64_t>(n_paths / 1024, 8192), 16384)
                        : std::min<int64_t>(std::max<int64_t>(n_paths / 64, 8192), 262144);
    if (const char *e = std::getenv("NH_TAIL")) p.tail_at = std::atoll(e);
    // below this many live paths the pool counts as draining: the next chunk may start beside it
    p.drain_at = std::max<int64_t>(n_paths / 8, p.tail_at);
    HIP_TRY(c, hipEventRecord(p.ev_begin, p.stream));
    // bounce 0 reads the dense camera queue: shard 0 holds all n_paths
    unsigned *h_init = p.h_counts + kRing * 2 * kCountGroup;
    std::memset(h_init, 0, kCountSlot * sizeof(unsigned));
    h_init[0] = (unsigned)n_paths;
    HIP_TRY(c, hipMemcpyAsync(p.wf.counts, h_init, kCountSlot * sizeof(unsigned), hipMemcpyHostToDevice, p.stream));
    p.in_e.assign(1, (uint64_t)n_paths);
    p.in_s.assign(1, 0);
    p.it = 0;
    p.tail = false;
    p.draining = false;
    p.state = WfPool::ENQUEUE;
    return NH_OK;
}

// The chunk (everything but the pool's stream and path state) moves between a pool and a tail slot: its job and
// launch parameters, timing events, pinned count ring, bounce counts, sample records and staging.
static void chunk_swap(WfPool &a, WfPool &b) {
    std::swap(a.h_counts, b.h_counts);
    std::swap(a.copy_ev, b.copy_ev);
    std::swap(a.events, b.events);
    std::swap(a.ev_begin, b.ev_begin);
    std::swap(a.ev_path, b.ev_path);
    std::swap(a.ev_splat0, b.ev_splat0);
    std::swap(a.ev_splat, b.ev_splat);
    std::swap(a.job, b.job);
    std::swap(a.L, b.L);
    std::swap(a.persistent, b.persistent);
    std::swap(a.wide, b.wide);
    std::swap(a.trace2, b.trace2);
    std::swap(a.tail, b.tail);
    std::swap(a.draining, b.draining);
    std::swap(a.fused, b.fused);
    std::swap(a.sorted, b.sorted);
    std::swap(a.rr, b.rr);
    std::swap(a.shade_sorted, b.shade_sorted);
    std::swap(a.tail_at, b.tail_at);
    std::swap(a.drain_at, b.drain_at);
    std::swap(a.it, b.it);
    std::swap(a.in_e, b.in_e);
    std::swap(a.in_s, b.in_s);
    std::swap(a.rec, b.rec);
    std::swap(a.rec_cap, b.rec_cap);
    std::swap(a.jit, b.jit);
    std::swap(a.jit_cap, b.jit_cap);
    std::swap(a.staging, b.staging);
    std::swap(a.staging_cap, b.staging_cap);
}

// an idle tail slot for pool p's chunk, or null: the tail then runs in place on the pool's stream. Off with one
// pool (the serialized roofline pass: kernels alone on the GPU) and unless NH_TAIL_ASYNC=1.
static WfPool *free_tail_slot(nh_ctx *c, const WfPool &p, int bound) {
    if (!p.rr || bound > kTailCap || active_pools(c) < 2) return nullptr;
    if (!tail_async_enabled()) return nullptr;
    for (int i = kPools; i < kPools + kTails; ++i)
        if (c->pools[i].state == WfPool::IDLE) return &c->pools[i];
    return nullptr;
}

// Hand the chunk's tail to tail slot T: pack the (at most bound) live paths into T's buffer on the pool's stream,
// move the chunk to T, and run its tail kernel on T's stream once the pack is done. The pool is idle at once:
// stream order keeps its next chunk's kernels behind the pack. The tail's paths, draws and arithmetic are the
// in-place tail's; the chunk's splat still waits for its turn (submission order), so the image is unchanged.
static int pool_handoff(nh_ctx *c, WfPool &p, WfPool &T, int bound, hipEvent_t *ev) {
    int rc = pool_alloc(c, T, (size_t)kTailCap, 0, 0);
    if (rc) return rc;
    HIP_TRY(c, hipMemsetAsync(T.wf.counts, 0, kCountSlot * sizeof(unsigned), p.stream));
    nh::launch_wf_pack_rr(p.L, T.wf.buf[0], T.wf.counts, bound, p.stream);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(p.ev_handoff, p.stream));
    chunk_swap(p, T);
    WfLaunch &L = T.L;  // the packed queue: buffer 0 of T, all paths in count shard 0
    L.st = T.wf;
    L.in_q = 0;
    L.cnt_in = T.wf.counts;  // (seg_cap stays the pool's: with one shard it does not address the packed queue, and
                             // it still bounds the pool's own counts the finish reads back)
    HIP_TRY(c, hipStreamWaitEvent(T.stream, p.ev_handoff, 0));
    HIP_TRY(c, hipEventRecord(ev[1], T.stream));
    HIP_TRY(c, hipEventRecord(ev[2], T.stream));
    nh::launch_wf_tail_rr(c->d_scene, c->tv, L, T.job.ordered, T.job.stats, bound, c->specular,
                          !c->specular && !c->textured, c->normal_mapped, T.stream);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(ev[3], T.stream));
    T.tail = true;
    T.draining = true;
    T.state = WfPool::SPLAT;
    p.state = WfPool::IDLE;
    c->stats.tails_async++;
    return NH_OK;
}

// NH_COUNT_KERNEL=0: the runtime's device-to-host copy and memset per bounce instead of wf_counts_kernel (A/B)
static bool count_kernel() {
    static const bool on = [] {
        const char *e = std::getenv("NH_COUNT_KERNEL");
        return !(e && e[0] == '0');
    }();
    return on;
}

// after bounce `it`'s appending kernel: its output counts (slot `out`) to the pinned ring, its input slot `in_slot`
// (the next bounce's output) cleared, then the event the host polls before reading the ring
static int count_service(nh_ctx *c, WfPool &p, unsigned *out, unsigned *in_slot, int it) {
    unsigned *h = p.h_counts + (size_t)(it % kRing) * 2 * kCountGroup;
    if (count_kernel()) {
        nh::launch_wf_counts(out, h, 2 * kCountGroup, in_slot, kCountSlot, p.stream);
        HIP_TRY(c, hipGetLastError());
    } else {
        HIP_TRY(c, hipMemcpyAsync(h, out, 2 * kCountGroup * sizeof(unsigned), hipMemcpyDeviceToHost, p.stream));
    }
    HIP_TRY(c, hipEventRecord(p.copy_ev[it % kRing], p.stream));
    return NH_OK;
}

// enqueue bounce p.it (extend, any-hit, then shade or, once few paths are left, the tail kernel)
static int pool_enqueue(nh_ctx *c, WfPool &p) {
    WfLaunch &L = p.L;
    const int it = p.it, in = it & 1;
    unsigned *slot[2] = {p.wf.counts, p.wf.counts + kCountSlot};
    L.in_q = in;
    L.first = it == 0;
    L.cam_rays = it == 0 && p.persistent && c->S.dof ? 1 : 0;
    L.cnt_in = slot[in];
    L.cnt_out = slot[in ^ 1];
    while ((size_t)(it + 1) * 4 > p.events.size()) {
        hipEvent_t e;
        HIP_TRY(c, hipEventCreate(&e));
        p.events.push_back(e);
    }
    hipEvent_t *ev = &p.events[(size_t)it * 4];
    // upper bound of this bounce's live paths: the input of the previous bounce (known: the host
    // has read the counts up to bounce it-2)
    const int bound = (int)p.in_e[it == 0 ? 0 : it - 1];
    const bool ordered = p.job.ordered, stats = p.job.stats;
    // this bounce's output slot must start at zero: bounce 0's is cleared here, every later one by the count
    // kernel of the bounce before it (count_service)
    if (it == 0 || !count_kernel()) HIP_TRY(c, hipMemsetAsync(slot[in ^ 1], 0, kCountSlot * sizeof(unsigned), p.stream));
    HIP_TRY(c, hipEventRecord(ev[0], p.stream));
    if (p.fused) {  // one kernel per bounce: its input already carries the hits (and no pending light samples)
        if (it > 0 && (int64_t)bound <= p.tail_at)
            if (WfPool *T = free_tail_slot(c, p, bound)) return pool_handoff(c, p, *T, bound, ev);
        HIP_TRY(c, hipEventRecord(ev[1], p.stream));
        HIP_TRY(c, hipEventRecord(ev[2], p.stream));
        if (it > 0 && (int64_t)bound <= p.tail_at) {
            if (p.rr)
                nh::launch_wf_tail_rr(c->d_scene, c->tv, L, ordered, stats, bound, c->specular, !c->specular && !c->textured,
                                      c->normal_mapped, p.stream);
            else nh::launch_wf_tail(c->d_scene, c->tv, L, ordered, stats, false, bound, c->depth, p.stream);
            HIP_TRY(c, hipGetLastError());
            HIP_TRY(c, hipEventRecord(ev[3], p.stream));
            p.tail = true;
            p.draining = true;
            p.state = WfPool::SPLAT;
            return NH_OK;
        }
        if (p.rr) nh::launch_wf_bounce_rr(c->d_scene, c->tv, L, ordered, stats, p.sorted, !c->specular && !c->textured,
                                          c->normal_mapped, bound, p.stream);
        else nh::launch_wf_bounce(c->d_scene, c->tv, L, ordered, stats, p.sorted, bound, p.stream);
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, hipEventRecord(ev[3], p.stream));
        if (int rc_ = count_service(c, p, slot[in ^ 1], slot[in], it)) return rc_;
        if (it == 0) p.it = 1;
        else p.state = WfPool::COUNTS;
        return NH_OK;
    }
    if (it == 0 && L.cam_rays) {
        nh::launch_wf_camera_rays(c->d_scene, L, bound, p.stream);
        HIP_TRY(c, hipGetLastError());
    }
    if (p.trace2) {  // both queries in one launch: its time counts as the extend stage's, the shadow stage's is 0
        nh::launch_wf_trace2(c->d_scene, c->tv, L, ordered, stats, c->wide_w, it == 0 ? bound : 2 * bound, p.stream);
        HIP_TRY(c, hipEventRecord(ev[1], p.stream));
        HIP_TRY(c, hipEventRecord(ev[2], p.stream));
    } else {
        nh::launch_wf_trace(c->d_scene, c->tv, L, ordered, stats, false, p.persistent, p.wide ? c->wide_w : 0, bound,
                            c->depth, p.stream);
        HIP_TRY(c, hipEventRecord(ev[1], p.stream));
        // bounce 0 has no shadow rays (the launch still runs: the kernels read the count on the device)
        nh::launch_wf_trace(c->d_scene, c->tv, L, ordered, stats, true, p.persistent, p.wide ? c->wide_w : 0,
                            it == 0 ? 0 : bound, c->depth, p.stream);
        HIP_TRY(c, hipEventRecord(ev[2], p.stream));
    }
    if (it > 0 && (int64_t)bound <= p.tail_at) {
        nh::launch_wf_tail(c->d_scene, c->tv, L, ordered, stats, p.wide ? c->wide_w : 0, bound, c->depth, p.stream);
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, hipEventRecord(ev[3], p.stream));
        p.tail = true;
        p.draining = true;
        p.state = WfPool::SPLAT;
        return NH_OK;
    }
    nh::launch_wf_shade(c->d_scene, c->tv, L, p.shade_sorted, c->normal_mapped, bound, p.stream);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(ev[3], p.stream));
    if (int rc_ = count_service(c, p, slot[in ^ 1], slot[in], it)) return rc_;
    if (it == 0) {
        p.it = 1;  // bounce 1 is sized by bounce 0's input: enqueue it before reading any count
    } else {
        p.state = WfPool::COUNTS;
    }
    return NH_OK;
}

// counts appended by bounce b (live paths, shadow rays entering bounce b+1)
static int pool_counts(nh_ctx *c, WfPool &p, int b, uint64_t &ne, uint64_t &ns) {
    const unsigned *hp = p.h_counts + (size_t)(b % kRing) * 2 * kCountGroup;
    ne = ns = 0;
    for (int s = 0; s < kQueueShards; ++s) {
        const unsigned ce = hp[s * kCountStride], cs = hp[kCountGroup + s * kCountStride];
        if (ce > (unsigned)p.L.seg_cap || cs > ce) return fail(c, "wavefront queue counts out of range"), NH_ERR_DEVICE;
        ne += ce;
        ns += cs;
    }
    if (ne > (uint64_t)p.L.n_paths) return fail(c, "wavefront queue counts out of range"), NH_ERR_DEVICE;
    return NH_OK;
}

// bounce it-1's counts have arrived: bounce it was enqueued empty (done) or enqueue bounce it+1
static int pool_read(nh_ctx *c, WfPool &p) {
    uint64_t ne, ns;
    int rc = pool_counts(c, p, p.it - 1, ne, ns);
    if (rc) return rc;
    p.in_e.push_back(ne);
    p.in_s.push_back(ns);
    if ((int64_t)ne < p.drain_at) p.draining = true;
    if (ne == 0) {
        p.state = WfPool::SPLAT;
        return NH_OK;
    }
    if (++p.it > 100000) return fail(c, "wavefront did not terminate"), NH_ERR_DEVICE;
    p.state = WfPool::ENQUEUE;
    return NH_OK;
}

// the chunk's paths are enqueued to completion: splat its records into the master ImageBlock
// after the previous write of the framebuffer (called in submission order)
static int pool_splat(nh_ctx *c, WfPool &p) {
    HIP_TRY(c, hipEventRecord(p.ev_path, p.stream));
    if (p.job.stats) nh::launch_count_invalid(p.rec, (size_t)p.L.n_paths, c->counters, p.stream);
    if (c->fb_ev_set) HIP_TRY(c, hipStreamWaitEvent(p.stream, c->fb_ev, 0));
    HIP_TRY(c, hipEventRecord(p.ev_splat0, p.stream));
    SplatLaunch sp = make_splat(c, p.rec, p.L.seed, p.L.s0, p.staging, p.job.rounds, p.job.staged);
    sp.jit = p.L.jit;
    nh::launch_splat(sp, p.stream);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(p.ev_splat, p.stream));
    HIP_TRY(c, hipEventRecord(c->fb_ev, p.stream));
    c->fb_ev_set = true;
    c->splat_seq++;
    p.draining = true;
    p.state = WfPool::FINISH;
    return NH_OK;
}

// the chunk has finished on the device: kernel times and byte accounting into the stats
static int pool_finish(nh_ctx *c, WfPool &p) {
    if (p.tail) {  // the last regular bounce's output counts, for the byte accounting below
        uint64_t ne, ns;
        int rc = pool_counts(c, p, p.it - 1, ne, ns);
        if (rc) return rc;
        p.in_e.push_back(ne);
        p.in_s.push_back(ns);
    }
    static const bool trace_counts = std::getenv("NH_TRACE_COUNTS") != nullptr;  // diagnostics: per-bounce profile
    if (trace_counts) {
        float t_all = 0.f;
        (void)hipEventElapsedTime(&t_all, p.ev_begin, p.ev_path);
        std::fprintf(stderr, "[nh] chunk seq %llu: %d paths, %d bounces%s, %.3f ms, live/bounce(ms):",
                     (unsigned long long)p.job.seq, p.L.n_paths, p.it + 1, p.tail ? " (last = tail kernel)" : "", t_all);
        for (int b = 0; b <= p.it && b < (int)p.in_e.size(); ++b) {
            float d = 0.f, e = 0.f, sh = 0.f;
            (void)hipEventElapsedTime(&d, p.events[(size_t)b * 4], p.events[(size_t)b * 4 + 3]);
            (void)hipEventElapsedTime(&e, p.events[(size_t)b * 4], p.events[(size_t)b * 4 + 1]);
            (void)hipEventElapsedTime(&sh, p.events[(size_t)b * 4 + 1], p.events[(size_t)b * 4 + 2]);
            std::fprintf(stderr, " %llu(%.3f e%.3f s%.3f)", (unsigned long long)p.in_e[b], d, e, sh);
        }
        std::fprintf(stderr, "\n");
    }
    for (int b = 0; b <= p.it; ++b) {
        hipEvent_t *ev = &p.events[(size_t)b * 4];
        float a = 0.f, sh = 0.f, d = 0.f;
        (void)hipEventElapsedTime(&a, ev[0], ev[1]);
        (void)hipEventElapsedTime(&sh, ev[1], ev[2]);
        (void)hipEventElapsedTime(&d, ev[2], ev[3]);
        c->stats.kernel_ms_extend += a;
        c->stats.kernel_ms_shadow += sh;
        c->stats.launches_extend++;
        c->stats.launches_shadow++;
        if (p.tail && b == p.it) {
            c->stats.kernel_ms_tail += d;
            c->stats.launches_tail++;
        } else {
            c->stats.kernel_ms_shade += d;
            c->stats.launches_shade++;
        }
    }
    float tp = 0.f, ts = 0.f;
    (void)hipEventElapsedTime(&tp, p.ev_begin, p.ev_path);
    (void)hipEventElapsedTime(&ts, p.ev_splat0, p.ev_splat);
    c->stats.kernel_ms_path += tp;
    c->stats.kernel_ms_splat += ts;
    c->stats.launches_splat++;
    c->stats.samples += (uint64_t)p.L.n_paths;
    // bytes by construction (nh_wavefront.hip), per bounce shaded by wf_shade (the tail kernel's work
    // is not part of this account); extend moves 48 B per ray (16 at bounce 0: no ray load).
    for (size_t b = 0; b + 1 < p.in_e.size(); ++b) {
        const uint64_t shaded = p.in_e[b], nsh = p.in_s[b], ne = p.in_e[b + 1], ns = p.in_s[b + 1];
        // bounce 0: hit in, sample record out. Later: path state (ray_o, ray_d, li, thr 16 B each,
        // rng 8 B) + hit in, the occlusion byte of a queued light sample (its 16-B pending term is
        // read only when unoccluded, not counted); out: survivors' state, the pending term + shadow
        // ray of each queued light sample, the radiance of each finished path
        c->stats.paths_shaded += shaded;
        if (p.fused) {  // wf_bounce: state + hit in (none at bounce 0), survivors' state + hit out, records
            const uint64_t loads = b == 0 ? 0 : shaded * (72 + 16);
            c->stats.shade_state_bytes += loads + (b == 0 ? shaded * 20 : 0) + ne * (72 + 16) + (shaded - ne) * 12;
            continue;
        }
        const uint64_t loads = b == 0 ? shaded * (16 + 20) : shaded * (72 + 16) + nsh * 1;
        c->stats.shade_state_bytes += loads + ne * 72 + ns * (16 + 36) + (shaded - ne) * 12;
        c->stats.extend_queue_bytes += shaded * (b == 0 ? 16 : 48);
        c->stats.shadow_queue_bytes += nsh * 37;  // ray in, path slot, occlusion byte out
    }
    p.state = WfPool::IDLE;
    return NH_OK;
}

// 1 = the event completed, 0 = pending; an error (a fault in the work before the event) goes to err
static int event_done(hipEvent_t e, hipError_t &err) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return 1;
    if (q != hipErrorNotReady) err = q;
    return 0;
}

// Device errors of this context's work so far (HIP errors are sticky per thread): checked at the end of
// nh_render / nh_synchronize, so a fault in a render's kernels is reported by the call that submitted or
// completed them, not by the next unrelated call (a denoise, a framebuffer read).
// Judged from this context's own streams only: the thread's last-error slot may hold another context's (or the
// host application's) error, which must not fail this call nor be cleared by it. Launch errors of this context's
// kernels are caught right after each launch (HIP_TRY(hipGetLastError())); a fault while they run shows in
// the status of their stream.
static int check_device(nh_ctx *c, const char *where) {
    hipError_t e = hipSuccess;
    {
        for (WfPool &p : c->pools) {
            if (!p.stream) continue;
            const hipError_t q = hipStreamQuery(p.stream);
            if (q != hipSuccess && q != hipErrorNotReady) { e = q; break; }
        }
    }
    if (e == hipSuccess && c->stream) {
        const hipError_t q = hipStreamQuery(c->stream);
        if (q != hipSuccess && q != hipErrorNotReady) e = q;
    }
    if (e != hipSuccess) {
        c->err = std::string(where) + ": device error in the rendering kernels: " + hipGetErrorString(e);
        return NH_ERR_DEVICE;
    }
    return NH_OK;
}

static void pipeline_reset(nh_ctx *c) {
    for (WfPool &p : c->pools)
        if (p.stream) (void)hipStreamSynchronize(p.stream);
    for (WfPool &p : c->pools) p.state = WfPool::IDLE;
    c->jobs.clear();
    c->splat_seq = c->job_seq;
}

// Drive the pools. all = run until every chunk has finished; otherwise return once every
// submitted chunk has started and every busy pool is draining.
static int pipeline_run(nh_ctx *c, bool all) {
    const int n_pools = active_pools(c);
    c->stats.pools_active = (uint64_t)n_pools;
    for (;;) {
        bool progress = false;
        hipError_t ev_err = hipSuccess;
        for (WfPool &p : c->pools) {
            int rc = NH_OK;
            // a chunk starts on an idle pool once every running chunk is draining (staggered pools)
            bool others_draining = true;
            for (const WfPool &o : c->pools) others_draining = others_draining && (o.state == WfPool::IDLE || o.draining);
            if (p.state == WfPool::IDLE && !c->jobs.empty() && &p - c->pools < n_pools && others_draining) {
                rc = pool_start(c, p, c->jobs.front());
                c->jobs.pop_front();
                progress = true;
            }
            if (!rc && p.state == WfPool::ENQUEUE) {
                rc = pool_enqueue(c, p);
                progress = true;
            }
            if (!rc && p.state == WfPool::COUNTS && event_done(p.copy_ev[(p.it - 1) % kRing], ev_err)) {
                rc = pool_read(c, p);
                progress = true;
            }
            if (!rc && p.state == WfPool::SPLAT && p.job.seq == c->splat_seq) {
                rc = pool_splat(c, p);
                progress = true;
            }
            if (!rc && p.state == WfPool::FINISH && event_done(p.ev_splat, ev_err)) {
                rc = pool_finish(c, p);
                progress = true;
            }
            if (!rc && ev_err != hipSuccess) {
                c->err = std::string("wavefront pipeline: ") + hipGetErrorString(ev_err);
                rc = NH_ERR_DEVICE;
            }
            if (rc) {
                pipeline_reset(c);
                return rc;
            }
        }
        if (c->jobs.empty()) {
            bool idle = true, draining = true;
            for (const WfPool &p : c->pools) {
                idle = idle && p.state == WfPool::IDLE;
                draining = draining && (p.state == WfPool::IDLE || p.draining);
            }
            if (idle || (!all && draining)) return NH_OK;
        }
        if (!progress) std::this_thread::yield();  // waiting on the device
    }
}

static int pipeline_drain(nh_ctx *c) {
    int rc = pipeline_run(c, true);
    if (rc) return rc;
    for (WfPool &p : c->pools)
        if (p.stream) HIP_TRY(c, hipStreamSynchronize(p.stream));
    return NH_OK;
}

static int ensure_pixel_list(nh_ctx *c, const nh_render_req *q) {
    std::vector<int32_t> key;
    if (q->n_blocks > 0 && q->blocks) key.assign(q->blocks, q->blocks + q->n_blocks);
    if (c->have_list && key == c->list_key) return NH_OK;
    if (int rc = pipeline_drain(c)) return rc;  // chunks in flight read the current list
    std::vector<int32_t> blocks = key;
    if (blocks.empty())
        for (int i = 0; i < c->nbx * c->nby; ++i) blocks.push_back(i);
    std::vector<int> list, map((size_t)c->width * c->height, -1);
    for (int32_t bid : blocks) {
        if (bid < 0 || bid >= c->nbx * c->nby) return fail(c, "block id out of range"), NH_ERR_INVALID;
        int bx = bid % c->nbx, by = bid / c->nbx;
        for (int y = by * 32; y < std::min(c->height, by * 32 + 32); ++y)
            for (int x = bx * 32; x < std::min(c->width, bx * 32 + 32); ++x) {
                int pix = y * c->width + x;
                if (map[pix] >= 0) return fail(c, "duplicate block id"), NH_ERR_INVALID;
                map[pix] = (int)list.size();
                list.push_back(pix);
            }
    }
    std::vector<int> slot_map((size_t)c->nbx * c->nby, -1);
    for (size_t i = 0; i < blocks.size(); ++i) slot_map[blocks[i]] = (int)i;
    (void)hipFree(c->pixel_list);
    (void)hipFree(c->pixel_map);
    (void)hipFree(c->block_ids);
    (void)hipFree(c->block_slot);
    (void)hipFree(c->color_slots);
    c->pixel_list = c->pixel_map = c->block_ids = c->block_slot = c->color_slots = nullptr;
    std::vector<int> color_slots;
    for (int col = 0; col < 2; ++col)
        for (size_t i = 0; i < blocks.size(); ++i)
            if (((blocks[i] % c->nbx + blocks[i] / c->nbx) & 1) == col) color_slots.push_back((int)i);
    c->n_color0 = 0;
    for (int32_t bid : blocks) c->n_color0 += ((bid % c->nbx + bid / c->nbx) & 1) == 0;
    HIP_TRY(c, hipMalloc(&c->color_slots, std::max<size_t>(color_slots.size(), 1) * sizeof(int)));
    if (!color_slots.empty())
        HIP_TRY(c, hipMemcpyAsync(c->color_slots, color_slots.data(), color_slots.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMalloc(&c->block_ids, std::max<size_t>(blocks.size(), 1) * sizeof(int)));
    HIP_TRY(c, hipMalloc(&c->block_slot, slot_map.size() * sizeof(int)));
    if (!blocks.empty())
        HIP_TRY(c, hipMemcpyAsync(c->block_ids, blocks.data(), blocks.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->block_slot, slot_map.data(), slot_map.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    c->n_blocks = (int)blocks.size();
    HIP_TRY(c, hipMalloc(&c->pixel_list, std::max<size_t>(list.size(), 1) * sizeof(int)));
    HIP_TRY(c, hipMalloc(&c->pixel_map, map.size() * sizeof(int)));
    if (!list.empty())
        HIP_TRY(c, hipMemcpyAsync(c->pixel_list, list.data(), list.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->pixel_map, map.data(), map.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->n_list = (int)list.size();
    c->list_key = key;
    c->have_list = true;
    return NH_OK;
}

int nh_render(nh_ctx *c, const nh_render_req *q) {
    if (!c || !q) return NH_ERR_INVALID;
    if (!c->has_scene || !c->has_bvh) return fail(c, "nh_render: scene and BVH must be uploaded"), NH_ERR_STATE;
    if (q->sample_end < q->sample_begin || q->sample_begin < 0) return fail(c, "invalid sample range"), NH_ERR_INVALID;
    if (c->S.dof && q->sample_end > nhd::kLensLo * nhd::kLensHi)  // the lens tables' range (nh_shade.h lens_uniform)
        return fail(c, "depth of field: sample rounds beyond 2^24"), NH_ERR_UNSUPPORTED;
    // path_mis throws it (path_mis.cpp:76-79); direct_mis would pick from an empty emitter list
    if ((c->integrator == NH_INTEGRATOR_PATH_MIS || c->integrator == NH_INTEGRATOR_DIRECT_MIS) && c->n_emitters == 0)
        return fail(c, "No Emitter in scene!"), NH_ERR_INVALID;
    if (q->mode != NH_MODE_MEGAKERNEL && q->mode != NH_MODE_WAVEFRONT) return fail(c, "unknown render mode"), NH_ERR_INVALID;
    // the single-bounce direct integrators always run as the megakernel: one closest hit, the light
    // sample(s) and at most one BSDF ray per path leave no bounce loop for path queues to balance
    const bool wavefront = q->mode == NH_MODE_WAVEFRONT && c->integrator <= NH_INTEGRATOR_PATH_MATS;
    if (q->traversal < NH_TRAVERSAL_REFERENCE || q->traversal > NH_TRAVERSAL_WIDE)
        return fail(c, "unknown traversal"), NH_ERR_INVALID;
    if (c->border > 4) return fail(c, "reconstruction filters wider than border 4 are not supported"), NH_ERR_UNSUPPORTED;
    HIP_TRY(c, hipSetDevice(c->device));
    // only asynchronous wavefront renders overlap earlier chunks still in flight
    int rc = NH_OK;
    if (!wavefront || q->collect_stats || q->clear) rc = pipeline_drain(c);
    if (rc) return rc;
    rc = ensure_pixel_list(c, q);
    if (rc) return rc;
    c->stats.node_bytes = 64;  // binary tree unless a wavefront pool picks the 4-wide one
    c->stats.trace_fused = 0;
    c->stats.lds_scene = 0;
    c->stats.fused_bounce = 0;
    if (q->clear) {
        HIP_TRY(c, hipMemsetAsync(c->fb, 0, c->fb_floats * sizeof(float), c->stream));
        HIP_TRY(c, hipEventRecord(c->fb_ev, c->stream));  // pools' splats wait for it
        c->fb_ev_set = true;
    }
    const int rounds = q->sample_end - q->sample_begin;
    if (rounds == 0 || c->n_list == 0) return NH_OK;
    if (q->collect_stats)
        HIP_TRY(c, hipMemsetAsync(c->counters, 0, kStatShards * kStatStride * sizeof(unsigned long long), c->stream));
    const size_t per_round = (size_t)c->n_list;
    const char *jv = std::getenv("NH_SPLAT_JITTER");  // stored jitter (A/B): 8 more bytes per sample record
    const size_t rec_bytes = kRecFloats * 4 + (wavefront && jv && std::strcmp(jv, "stored") == 0 ? 8 : 0);
    const size_t per_round_bytes = per_round * rec_bytes + (size_t)c->n_blocks * block_px(c, splat_staged(c)) * 16 +
                                   (wavefront ? per_round * kWfBytesPerPath : 0);
    // device memory per chunk: sample records + block ImageBlocks (+ path state, per pool). Every
    // wavefront chunk ends in a tail whose length is set by its longest path (C4: ~5-7 ms of
    // dielectric / mirror chains, whatever the chunk's size), so chunks are as large as the 26-bit
    // path ids allow: one chunk per C4 step (67M paths, ~18 GB per pool) instead of 7 + 7 + 2 rounds
    // under an 8 GiB budget (C4 2590 -> 3140 Msamples/s); 288 GB of HBM holds two such pools.
    size_t budget = wavefront ? (size_t)24 << 30 : (size_t)1 << 30;
    if (const char *e = std::getenv(wavefront ? "NH_WF_BUDGET_MB" : "NH_RECORD_BUDGET_MB"))
        budget = (size_t)std::max(1L, std::atol(e)) << 20;
    if (wavefront) {
        // every active pool is sized for the chunk: cap the budget at this device's free memory (plus what
        // the pools already hold) shared by the pools, with headroom, so several contexts on one GPU get
        // smaller chunks instead of a failed allocation
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            size_t held = 0;
            for (const WfPool &p : c->pools)
                held += p.cap * kWfBytesPerPath + p.rec_cap * kRecFloats * 4 + p.jit_cap * 8 + p.staging_cap * sizeof(float4);
            // asynchronous tails: each tail slot also holds a whole chunk's sample records and staging (and
            // kTailCap paths of state), so it counts as one more chunk-sized share
            const int shares = active_pools(c) + (active_pools(c) > 1 && tail_async_enabled() ? kTails : 0);
            const size_t avail = (size_t)((double)(free_b + held) * 0.85) / (size_t)shares;
            budget = std::min(budget, std::max(avail, per_round_bytes));
        }
    }
    int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)rounds, budget / per_round_bytes));
    while ((size_t)chunk * per_round > (size_t)0x7fffffff) chunk = std::max(1, chunk / 2);
    if (wavefront) {  // path ids of a chunk are packed into 26 bits of the path state (nh_wavefront.hip)
        if (per_round > ((size_t)1 << 26))
            return fail(c, "wavefront mode renders at most 2^26 pixels per context"), NH_ERR_UNSUPPORTED;
        chunk = std::min(chunk, (int)(((size_t)1 << 26) / per_round));
    }

    if (wavefront) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));  // pixel list / clear / counters are in place
        for (int s = q->sample_begin; s < q->sample_end; s += chunk)
            c->jobs.push_back(WfJob{c->job_seq++, s, std::min(chunk, q->sample_end - s), q->seed,
                                    q->traversal != NH_TRAVERSAL_REFERENCE, q->collect_stats != 0});
        rc = q->collect_stats ? pipeline_drain(c) : pipeline_run(c, false);
        if (rc) return rc;
        if (int e = check_device(c, "nh_render")) return e;
    } else {
        if (c->rec_cap < (size_t)chunk * per_round) {
            (void)hipFree(c->rec);
            c->rec = nullptr;
            c->rec_cap = 0;
            const size_t cap = (size_t)chunk * per_round;
            HIP_TRY(c, hipMalloc(&c->rec, cap * kRecFloats * sizeof(float)));
            c->rec_cap = cap;
        }
        const bool staged = splat_staged(c);
        if (c->staging_cap < (size_t)chunk * c->n_blocks * block_px(c, staged)) {
            (void)hipFree(c->staging);
            c->staging = nullptr;
            c->staging_cap = 0;
            const size_t cap = (size_t)chunk * c->n_blocks * block_px(c, staged);
            HIP_TRY(c, hipMalloc(&c->staging, cap * sizeof(float4)));
            c->staging_cap = cap;
        }
        struct Ev {
            hipEvent_t a, b, d;
        };
        std::vector<Ev> evs;
        for (int s = q->sample_begin; s < q->sample_end; s += chunk) {
            const int k = std::min(chunk, q->sample_end - s);
            PathLaunch L{};
            L.n_paths = k * c->n_list;
            L.n_list = c->n_list;
            L.s0 = s;
            L.seed = q->seed;
            L.pixel_list = c->pixel_list;
            L.rec = c->rec;
            L.counters = c->counters;
            Ev ev;
            HIP_TRY(c, hipEventCreate(&ev.a));
            HIP_TRY(c, hipEventCreate(&ev.b));
            HIP_TRY(c, hipEventCreate(&ev.d));
            HIP_TRY(c, hipEventRecord(ev.a, c->stream));
            nh::launch_path(c->d_scene, c->tv, L, q->traversal != NH_TRAVERSAL_REFERENCE, q->collect_stats != 0,
                            c->depth, c->integrator == NH_INTEGRATOR_PATH_MIS && !c->normal_mapped, c->stream);
            HIP_TRY(c, hipGetLastError());
            HIP_TRY(c, hipEventRecord(ev.b, c->stream));
            if (q->collect_stats) nh::launch_count_invalid(c->rec, (size_t)L.n_paths, c->counters, c->stream);
            nh::launch_splat(make_splat(c, c->rec, q->seed, s, c->staging, k, staged), c->stream);
            HIP_TRY(c, hipGetLastError());
            HIP_TRY(c, hipEventRecord(ev.d, c->stream));
            evs.push_back(ev);
        }
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        for (auto &ev : evs) {
            float a = 0, b = 0;
            (void)hipEventElapsedTime(&a, ev.a, ev.b);
            (void)hipEventElapsedTime(&b, ev.b, ev.d);
            c->stats.kernel_ms_path += a;
            c->stats.kernel_ms_splat += b;
            c->stats.launches_path++;
            c->stats.launches_splat++;
            (void)hipEventDestroy(ev.a);
            (void)hipEventDestroy(ev.b);
            (void)hipEventDestroy(ev.d);
        }
        c->stats.samples += (uint64_t)rounds * (uint64_t)c->n_list;
    }
    if (q->collect_stats) {
        unsigned long long hs[kStatShards * kStatStride], h[kStatStride] = {};
        HIP_TRY(c, hipMemcpy(hs, c->counters, sizeof(hs), hipMemcpyDeviceToHost));
        for (int sh = 0; sh < kStatShards; ++sh)
            for (int j = 0; j < kStatStride; ++j) h[j] += hs[sh * kStatStride + j];
        h[kStatTailClk + 5] = 0;  // the longest tail chain: a max over the shards, not a sum
        for (int sh = 0; sh < kStatShards; ++sh)
            h[kStatTailClk + 5] = std::max(h[kStatTailClk + 5], hs[sh * kStatStride + kStatTailClk + 5]);
        c->stats.tail_cycles_body += h[kStatTailClk];
        c->stats.tail_cycles_shadow += h[kStatTailClk + 1];
        c->stats.tail_cycles_closest += h[kStatTailClk + 2];
        c->stats.tail_cycles_head += h[kStatTailClk + 3];
        c->stats.tail_bounces += h[kStatTailClk + 4];
        c->stats.tail_max_bounces = std::max<uint64_t>(c->stats.tail_max_bounces, h[kStatTailClk + 5]);
        c->stats.tail_coop_cycles_body += h[kStatTailCoopClk];
        c->stats.tail_coop_cycles_shadow += h[kStatTailCoopClk + 1];
        c->stats.tail_coop_cycles_closest += h[kStatTailCoopClk + 2];
        c->stats.tail_coop_cycles_head += h[kStatTailCoopClk + 3];
        c->stats.tail_coop_bounces += h[kStatTailCoopClk + 4];
        c->stats.bounce_cycles_load += h[kStatBounceClk];
        c->stats.bounce_cycles_body += h[kStatBounceClk + 1];
        c->stats.bounce_cycles_shadow += h[kStatBounceClk + 2];
        c->stats.bounce_cycles_closest += h[kStatBounceClk + 3];
        c->stats.bounce_cycles_head += h[kStatBounceClk + 4];
        c->stats.bounce_cycles_store += h[kStatBounceClk + 5];
        c->stats.bounce_bounces += h[kStatBounceClk + 6];
        const unsigned long long *cl = h, *an = h + kStatAny, *tc = h + kStatTail, *ta = h + kStatTailAny;
        c->stats.ray_queries += cl[0] + an[0] + tc[0] + ta[0];
        c->stats.nodes_visited += cl[1] + an[1] + tc[1] + ta[1];
        c->stats.boxes_tested += cl[2] + an[2] + tc[2] + ta[2];
        c->stats.prims_tested += cl[3] + an[3] + tc[3] + ta[3];
        c->stats.invalid_samples += h[4];
        c->stats.shadow_queries += an[0] + ta[0];
        c->stats.shadow_nodes_visited += an[1] + ta[1];
        c->stats.shadow_boxes_tested += an[2] + ta[2];
        c->stats.shadow_prims_tested += an[3] + ta[3];
        c->stats.tail_queries += tc[0] + ta[0];
        c->stats.tail_nodes_visited += tc[1] + ta[1];
        c->stats.tail_boxes_tested += tc[2] + ta[2];
        c->stats.tail_prims_tested += tc[3] + ta[3];
        c->stats.tail_shadow_queries += ta[0];
        c->stats.tail_shadow_nodes_visited += ta[1];
        c->stats.tail_shadow_boxes_tested += ta[2];
        c->stats.tail_shadow_prims_tested += ta[3];
    }
    return NH_OK;
}

int nh_synchronize(nh_ctx *c) {
    if (!c) return NH_ERR_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    int rc = pipeline_drain(c);
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return check_device(c, "nh_synchronize");
}

int nh_get_framebuffer(nh_ctx *c, float *rgbw, size_t n) {
    if (!c || !rgbw) return NH_ERR_INVALID;
    if (!c->has_scene) return fail(c, "no scene"), NH_ERR_STATE;
    if (n < c->fb_floats) return fail(c, "framebuffer destination too small"), NH_ERR_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    int rc = pipeline_drain(c);
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(rgbw, c->fb, c->fb_floats * sizeof(float), hipMemcpyDeviceToHost));
    return NH_OK;
}

int nh_framebuffer_device_ptr(nh_ctx *c, void **dptr, size_t *n) {
    if (!c || !dptr || !n) return NH_ERR_INVALID;
    if (!c->has_scene) return fail(c, "no scene"), NH_ERR_STATE;
    // The pipeline advances only inside library calls (the host reads queue counts to enqueue the
    // next bounce): run every submitted chunk to completion first, so a caller that hands the
    // pointer to its own stream or collective (RCCL reduce) reads the finished image.
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc = pipeline_drain(c)) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    *dptr = c->fb;
    *n = c->fb_floats;
    return NH_OK;
}

int nh_get_stats(nh_ctx *c, nh_render_stats *out) {
    if (!c || !out) return NH_ERR_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    int rc = pipeline_drain(c);  // kernel times of chunks still in flight
    if (rc) return rc;
    *out = c->stats;
    out->comm_inits = c->stats_comm_inits;
    return NH_OK;
}

int nh_reset_stats(nh_ctx *c) {
    if (!c) return NH_ERR_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    int rc = pipeline_drain(c);
    if (rc) return rc;
    std::memset(&c->stats, 0, sizeof(c->stats));
    return NH_OK;
}

// SimpleDenoiser on a device ImageBlock (nh_denoise.hip): `amount` passes, each the raw variance + its
// max / min, then the banded wavefront schedule of the in-place row-major sweep. Scratch is per call.
static int run_denoise(nh_ctx *c, float *fb, int W, int H, int bs, const nh_denoiser *p) {
    if (!p || p->type != NH_DENOISER_SIMPLE) return fail(c, "denoise: type must be NH_DENOISER_SIMPLE"), NH_ERR_INVALID;
    // SimpleDenoiser's constructor clamps (simple.cpp:15-24): anything outside is not a reference configuration
    if (!(p->sigma_d >= 1e-4f && p->sigma_d <= 10.f) || !(p->sigma_vr >= 1e-4f && p->sigma_vr <= 10.f) ||
        p->range < 0 || p->range > 50 || p->amount < 1 || p->amount > 10)
        return fail(c, "denoise: parameters outside SimpleDenoiser's clamps"), NH_ERR_INVALID;
    if (W <= 0 || H <= 0 || bs < 0) return fail(c, "denoise: empty image"), NH_ERR_INVALID;
    const int r = p->range, cols = W + 2 * bs;
    // g_sigma (simple.cpp:136-139) depends only on the squared pixel distance: the reference's float expf per
    // distance, tabulated
    std::vector<float> g((size_t)2 * r * r + 1);
    for (size_t d = 0; d < g.size(); ++d) g[d] = std::exp((float)-(int)d / 2.f / p->sigma_d / p->sigma_d);
    std::vector<void *> tmp;
    struct Free {
        std::vector<void *> &v;
        ~Free() { free_all(v); }
    } guard{tmp};
    float4 *B = nullptr;
    float *var = nullptr, *dg = nullptr;
    unsigned *minmax = nullptr;
    HIP_TRY(c, hipMalloc(&B, (size_t)W * H * sizeof(float4)));
    tmp.push_back(B);
    HIP_TRY(c, hipMalloc(&var, (size_t)W * H * sizeof(float)));
    tmp.push_back(var);
    HIP_TRY(c, hipMalloc(&dg, g.size() * sizeof(float)));
    tmp.push_back(dg);
    HIP_TRY(c, hipMalloc(&minmax, 2 * sizeof(unsigned)));
    tmp.push_back(minmax);
    HIP_TRY(c, hipMemcpyAsync(dg, g.data(), g.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    float4 *F = reinterpret_cast<float4 *>(fb) + (size_t)bs * cols + bs;
    // schedule: bands of BH rows start (r+1) BH wavefront steps apart; a launch runs `chunk` steps of each
    // band in flight; band w's chunk k runs in launch w lag + k, lag = ceil((skew - 1) / chunk) + 1, so the
    // band above has finished every step this chunk reads before the launch starts
    const int BH = nh::denoise_band_rows();
    const int n_bands = (H + BH - 1) / BH, skew = BH * (r + 1);
    const int chunk = std::max(1, skew / 4);
    const int lag = (skew - 1 + chunk - 1) / chunk + 1;
    const int k_max = ((r + 1) * (BH - 1) + W + chunk - 1) / chunk;
    const int n_launch = (n_bands - 1) * lag + k_max;
    // LDS tile of a chunk's window (input + denoised pixels): rows BH + 2r, columns chunk + (r+1)(BH-1) + 2r
    const size_t tile_rows = (size_t)std::min(H, BH + 2 * r);
    const size_t tile_cols = (size_t)std::min(W, chunk + (r + 1) * (BH - 1) + 2 * r);
    size_t tile_bytes = 2 * tile_rows * tile_cols * sizeof(float4);
    // the tile plus the kernel's static LDS must fit one workgroup's LDS (and the 64 KiB of dynamic LDS a
    // launch may request without raising the function's attribute)
    int lds_per_block = 0;
    HIP_TRY(c, hipDeviceGetAttribute(&lds_per_block, hipDeviceAttributeMaxSharedMemoryPerBlock, c->device));
    const size_t static_lds = nh::denoise_tile_static_lds();
    if (tile_bytes > 64 * 1024 || tile_bytes + static_lds > (size_t)lds_per_block || chunk > nh::denoise_max_chunk() ||
        std::getenv("NH_DENOISE_NO_TILE"))
        tile_bytes = 0;
    hipEvent_t e0, e1;
    HIP_TRY(c, hipEventCreate(&e0));
    HIP_TRY(c, hipEventCreate(&e1));
    HIP_TRY(c, hipEventRecord(e0, c->stream));
    uint64_t launches = 0;
    for (int pass = 0; pass < p->amount; ++pass) {
        DenoiseLaunch P{};
        const bool even = (pass & 1) == 0;
        P.src = even ? F : B;
        P.src_stride = even ? cols : W;
        P.dst = even ? B : F;
        P.dst_stride = even ? W : cols;
        P.width = W;
        P.height = H;
        P.range = r;
        P.sigma_vr = p->sigma_vr;
        P.g = dg;
        P.var = var;
        P.minmax = minmax;
        P.lag = lag;
        P.chunk = chunk;
        HIP_TRY(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(minmax), 0, 1, c->stream));
        HIP_TRY(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(minmax + 1), 0x7f800000, 1, c->stream));
        nh::launch_denoise_variance(P, c->stream);
        launches += 1;
        for (int L = 0; L < n_launch; ++L) {
            const int w_lo = std::max(0, (L - k_max + 1 + lag - 1) / lag), w_hi = std::min(n_bands - 1, L / lag);
            if (w_hi < w_lo) continue;
            P.band_first = w_lo;
            nh::launch_denoise_band(P, L, w_hi - w_lo + 1, tile_bytes, c->stream);
            ++launches;
        }
    }
    if (p->amount & 1) {  // the last pass wrote the scratch image
        nh::launch_denoise_copy(B, W, F, cols, W, H, c->stream);
        ++launches;
    }
    HIP_TRY(c, hipEventRecord(e1, c->stream));
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    c->stats.kernel_ms_denoise += ms;
    c->stats.launches_denoise += launches;
    return NH_OK;
}

int nh_denoise(nh_ctx *c, const nh_denoiser *params) {
    if (!c || !params) return NH_ERR_INVALID;
    if (!c->has_scene) return fail(c, "no scene"), NH_ERR_STATE;
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc = pipeline_drain(c)) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return run_denoise(c, c->fb, c->width, c->height, c->border, params);
}

int nh_denoise_image(nh_ctx *c, float *rgbw, int32_t width, int32_t height, int32_t border,
                     const nh_denoiser *params) {
    if (!c || !rgbw || !params || width <= 0 || height <= 0 || border < 0) return NH_ERR_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc = pipeline_drain(c)) return rc;
    const size_t n = 4 * (size_t)(width + 2 * border) * (size_t)(height + 2 * border);
    float *d = nullptr;
    HIP_TRY(c, hipMalloc(&d, n * sizeof(float)));
    std::vector<void *> own{d};
    struct Free {
        std::vector<void *> &v;
        ~Free() { free_all(v); }
    } guard{own};
    HIP_TRY(c, hipMemcpyAsync(d, rgbw, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if (int rc = run_denoise(c, d, width, height, border, params)) return rc;
    HIP_TRY(c, hipMemcpy(rgbw, d, n * sizeof(float), hipMemcpyDeviceToHost));
    return NH_OK;
}

int nh_reduce_framebuffers(nh_ctx **ctxs, int32_t n, int32_t root) {
    if (!ctxs || n <= 0 || root < 0 || root >= n) return NH_ERR_INVALID;
    DeviceGuard guard;
    for (int i = 0; i < n; ++i)
        if (!ctxs[i] || !ctxs[i]->has_scene || ctxs[i]->fb_floats != ctxs[0]->fb_floats) return NH_ERR_INVALID;
    for (int i = 0; i < n; ++i) {
        (void)hipSetDevice(ctxs[i]->device);
        if (pipeline_drain(ctxs[i])) return NH_ERR_DEVICE;
    }
    // one communicator clique per set of contexts, reused across calls (ncclCommInitAll costs far more
    // than the reduce of a framebuffer); any change of members or order builds a new one
    std::vector<uint64_t> ids(n);
    for (int i = 0; i < n; ++i) ids[i] = ctxs[i]->id;
    std::shared_ptr<CommSet> cs = ctxs[0]->comms;
    if (!cs || cs->ids != ids) {
        for (int i = 0; i < n; ++i) ctxs[i]->comms.reset();
        cs = std::make_shared<CommSet>();
        cs->ids = ids;
        cs->devices.resize(n);
        cs->comms.resize(n);
        for (int i = 0; i < n; ++i) cs->devices[i] = ctxs[i]->device;
        if (ncclCommInitAll(cs->comms.data(), n, cs->devices.data()) != ncclSuccess) {
            cs->comms.clear();
            ctxs[root]->err = "ncclCommInitAll failed";
            return NH_ERR_DEVICE;
        }
        for (int i = 0; i < n; ++i) ctxs[i]->comms = cs;
        ctxs[root]->stats_comm_inits++;
    }
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; i < n && r == ncclSuccess; ++i) {
        (void)hipSetDevice(ctxs[i]->device);
        r = ncclReduce(ctxs[i]->fb, ctxs[i]->fb, ctxs[i]->fb_floats, ncclFloat, ncclSum, root, cs->comms[i],
                       ctxs[i]->stream);
    }
    const ncclResult_t g = ncclGroupEnd();
    if (r == ncclSuccess) r = g;
    for (int i = 0; i < n; ++i) {
        (void)hipSetDevice(ctxs[i]->device);
        (void)hipStreamSynchronize(ctxs[i]->stream);
    }
    if (r != ncclSuccess) {
        ctxs[root]->err = std::string("ncclReduce failed: ") + ncclGetErrorString(r);
        for (int i = 0; i < n; ++i) ctxs[i]->comms.reset();
        return NH_ERR_DEVICE;
    }
    return NH_OK;
}

}  // extern "C"
