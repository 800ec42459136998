// gfx950 kernels of the path_mis hot path.
//
//   nh_trace_kernel   BVH::rayIntersect over an SoA ray batch (parity entry point)
//   nh_path_kernel    megakernel: one thread per (pixel, sample) camera path --
//                     renderBlock's per-pixel body + PathMISIntegrator::Li / PathMatsIntegrator::Li
//                     (src/utils/render.cpp:436-458, src/integrators/path_mis.cpp:16-150,
//                     path_mats.cpp:16-78), writing (radiance, jitter) sample records
//   (the ImageBlock stage -- splat and merge of the sample records -- is in nh_splat.hip)
#include <cstdlib>
#include <type_traits>

#include "nh_internal.h"

#ifndef NH_DEFAULT_PATH_WAVES
#define NH_DEFAULT_PATH_WAVES 4
#endif
#include "nh_traverse.h"
#include "nh_shade.h"

using namespace nhd;

namespace {

// PathMISIntegrator::Li (src/integrators/path_mis.cpp:16-150). Lanes of a wave stay in
// lockstep: shade, then one shadow traversal (any hit, :89) for the lanes that sample a
// light, then one closest-hit traversal of the BSDF-sampled ray for every lane -- that ray
// is both the MIS probe (:117-119) and the next bounce (:146 -> :34) and is traced once.
// Everything that does not depend on a traversal result is evaluated before it (pure
// functions, same operands, same random-number draw order: traversals draw nothing), which
// keeps the state that is live across traversals small.
template <int DEPTH, bool ORDERED, bool STATS, bool NMAP = true>
__device__ F3 li_path_mis(const DScene &S, const Traversal &tv, Rng &rng, F3 o, F3 d, float mint, float maxt,
                          uint32_t *stk, int stride, TravStats &st, uint32_t &queries) {
    F3 li = f3(0, 0, 0), t = f3(1, 1, 1);
    float w_mats = 1.f, w_ems = 0.f;
    const float n_lights = (float)S.n_emitters;
    Hit h;
    if (STATS) queries++;
    bool found = trace<DEPTH, ORDERED, false, STATS>(tv, S, o, d, mint, maxt, h, stk, stride, st);
    for (;;) {
        if (!found) {  // path_mis.cpp:32-44: escaped rays see the environment map, no MIS weight
            if (S.envmap >= 0) li = add(li, mulc(t, env_eval(S, d)));
            break;
        }
        Its its;
        hit_info<NMAP>(S, tv, h, o, d, its);
        const DShape shape = S.shapes[its.shape];
        const DBsdf bsdf = S.bsdfs[shape.bsdf];
        const F3 alb = bsdf_albedo(S, bsdf, its.u, its.v);
        if (shape.emitter >= 0) {  // path_mis.cpp:51-56
            const DEmitter em = S.emitters[shape.emitter];
            const F3 wi = normalized(sub(its.p, o));
            li = add(li, mulc(scl(w_mats, t), emitter_eval(em, o, its.sh.n, wi)));
        }
        float succ = e_min(max_coeff(t), 0.99f);  // RR from depth 0 (path_mis.cpp:58-71)
        succ = e_max(succ, kEps);
        if (rng.next1d() > succ) break;
        t = divs(t, succ);

        // emitter sampling (path_mis.cpp:75-102)
        const int ei = emitter_pick(S, rng.next1d());
        const DEmitter em = S.emitters[ei];
        const float ex = rng.next1d(), ey = rng.next1d();
        ESample es;
        const F3 ems_col = emitter_sample(S, em, its.p, ex, ey, es);
        const F3 wi_l = to_local(its.sh, neg(d));
        const bool nee = !is_zero(ems_col);
        F3 li_ems = f3(0, 0, 0);
        float pdfems = 0.f, pdfems_mats = 0.f;
        if (nee) {
            const F3 we = to_local(its.sh, es.wi);
            const F3 f = bsdf_eval(bsdf, wi_l, we, M_SOLID_ANGLE, alb);
            const float cs = we.z;
            li_ems = f3(ems_col.x * cs * f.x * n_lights, ems_col.y * cs * f.y * n_lights,
                        ems_col.z * cs * f.z * n_lights);
            pdfems_mats = bsdf_pdf(bsdf, wi_l, we, M_SOLID_ANGLE);
            pdfems = emitter_pdf(S, em, its.p, es.p, es.n, es.wi) / n_lights;
        }
        // BSDF sampling (path_mis.cpp:109-113)
        const float bx = rng.next1d(), by = rng.next1d();
        F3 wo;
        int measure;
        const F3 bsdf_col = bsdf_sample(bsdf, wi_l, bx, by, wo, measure, alb);
        const float pdfmat = bsdf_pdf(bsdf, wi_l, wo, measure);  // used only if the probe hits an emitter
        const F3 nd = to_world(its.sh, wo);
        const F3 no = its.p;

        // A discrete BSDF sample zeroes w_ems (path_mis.cpp:136-140): the light term (0 * t) * li_ems then
        // adds exactly zero whether or not the shadow ray is occluded, as long as it is finite (Li never
        // holds -0, so +-0 leaves it unchanged) -- that query is not traced (same draws, same result;
        // the wavefront shade makes the same decision)
        bool trace_shadow = nee;
        if (nee && measure == M_DISCRETE) {
            const F3 c = mulc(scl(0.f, t), li_ems), z = mulc(scl(0.f, t), f3(0, 0, 0));
            if (c.x == 0.f && c.y == 0.f && c.z == 0.f && z.x == 0.f && z.y == 0.f && z.z == 0.f) trace_shadow = false;
        }
        if (trace_shadow) {  // shadow ray (path_mis.cpp:89): occluded -> no contribution, pdfs stay 0
            Hit hs;
            if (STATS) queries++;
            if (trace<DEPTH, ORDERED, true, STATS>(tv, S, es.so, es.sd, es.smint, es.smaxt, hs, stk, stride, st)) {
                li_ems = f3(0, 0, 0);
                pdfems = 0.f;
                pdfems_mats = 0.f;
            }
        }
        if ((pdfems_mats + pdfems) > kEps) w_ems = pdfems / (pdfems_mats + pdfems);

        // probe ray == next bounce (path_mis.cpp:115-146); a zero direction misses every
        // primitive (det == 0 / NaN roots), so its traversal is skipped
        if (nd.x == 0 && nd.y == 0 && nd.z == 0) {
            found = false;
        } else {
            if (STATS) queries++;
            found = trace_next<DEPTH, ORDERED, STATS>(tv, S, h.k, no, nd, kEps, INFINITY, h, stk, stride, st);
        }
        if (!is_zero(bsdf_col) && found) {
            const int hs_shape = __float_as_int(tv.prims[3 * h.k + 1].w);
            const int hem = S.shapes[hs_shape].emitter;
            if (hem >= 0) {
                Its its_s;
                hit_info<NMAP>(S, tv, h, no, nd, its_s);
                const DEmitter em2 = S.emitters[hem];
                const F3 wim = normalized(sub(its_s.p, no));
                const float pdfmat_ems = emitter_pdf(S, em2, no, its_s.p, its_s.sh.n, wim) / n_lights;
                if ((pdfmat + pdfmat_ems) > kEps) w_mats = pdfmat / (pdfmat + pdfmat_ems);
            }
        }
        if (measure == M_DISCRETE) {
            w_ems = 0.f;
            w_mats = 1.f;
        }
        li = add(li, mulc(scl(w_ems, t), li_ems));
        t = mulc(t, bsdf_col);
        o = no;
        d = nd;
    }
    return li;
}

// PathMatsIntegrator::Li (src/integrators/path_mats.cpp:16-78)
template <int DEPTH, bool ORDERED, bool STATS>
__device__ F3 li_path_mats(const DScene &S, const Traversal &tv, Rng &rng, F3 o, F3 d, float mint, float maxt,
                           uint32_t *stk, int stride, TravStats &st, uint32_t &queries) {
    F3 li = f3(0, 0, 0), t = f3(1, 1, 1);
    int counter = 0;
    Hit h;
    h.k = -1;  // the camera ray leaves no surface
    for (;;) {
        bool found;
        if (d.x == 0 && d.y == 0 && d.z == 0) {
            found = false;
        } else {
            if (STATS) queries++;
            found = trace_next<DEPTH, ORDERED, STATS>(tv, S, h.k, o, d, mint, maxt, h, stk, stride, st);
        }
        if (!found) {  // path_mats.cpp:26-35
            if (S.envmap >= 0) li = add(li, mulc(t, env_eval(S, d)));
            break;
        }
        Its its;
        hit_info(S, tv, h, o, d, its);
        const DShape shape = S.shapes[its.shape];
        const DBsdf bsdf = S.bsdfs[shape.bsdf];
        const F3 alb = bsdf_albedo(S, bsdf, its.u, its.v);
        if (shape.emitter >= 0) {
            F3 wi = normalized(sub(its.p, o));
            li = add(li, mulc(t, emitter_eval(S.emitters[shape.emitter], o, its.sh.n, wi)));
        }
        float succ = e_min(max_coeff(t), 0.99f);
        if (counter < 3) counter++;
        else if (rng.next1d() > succ) break;
        else t = divs(t, succ);
        const float bx = rng.next1d(), by = rng.next1d();
        F3 wo;
        int measure;
        F3 col = bsdf_sample(bsdf, to_local(its.sh, neg(d)), bx, by, wo, measure, alb);
        t = mulc(t, col);
        d = to_world(its.sh, wo);
        o = its.p;
        mint = kEps;
        maxt = INFINITY;
    }
    return li;
}

__device__ __forceinline__ void flush_stats(const TravStats &st, uint32_t queries, unsigned long long *counters) {
    // one atomic per wave: reduce over the 64 lanes first
    unsigned long long v[4] = {queries, st.nodes, st.boxes, st.prims};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        unsigned long long x = v[i];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(&counters[i], x);
    }
}

}  // namespace

template <int BLOCK, int DEPTH, bool ORDERED, bool ANY, bool STATS>
__global__ __launch_bounds__(BLOCK) void nh_trace_kernel(const DScene *__restrict__ Sp, Traversal tv, RayBatch rb,
                                                         HitBatch hb, int n, unsigned long long *counters) {
    __shared__ uint32_t stk[DEPTH * BLOCK];
    const DScene &S = *Sp;
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    TravStats st{0, 0, 0};
    if (i < n) {
        F3 o = f3(rb.ox[i], rb.oy[i], rb.oz[i]), d = f3(rb.dx[i], rb.dy[i], rb.dz[i]);
        Hit h;
        bool hit = trace<DEPTH, ORDERED, ANY, STATS>(tv, S, o, d, rb.mint[i], rb.maxt[i], h, stk + threadIdx.x, BLOCK, st);
        hb.hit[i] = hit ? 1 : 0;
        if (!ANY) {
            hb.t[i] = hit ? h.t : INFINITY;
            hb.u[i] = hit ? h.u : 0.f;
            hb.v[i] = hit ? h.v : 0.f;
            hb.k[i] = hit ? h.k : -1;
        }
    }
    if (STATS) flush_stats(st, i < n ? 1u : 0u, stat_shard(counters));
}

// The same entry point over the 4-wide (or 8-wide, W = 8) collapse (nh_traverse.h Tracer4 / Tracer8), run to
// completion per lane: LDS window of 16 (ref, distance) entries, deeper entries in the lane's `spill` area.
template <bool ORDERED, bool ANY, bool STATS, int W = 4>
__global__ __launch_bounds__(64) void nh_trace_wide_kernel(const DScene *__restrict__ Sp, Traversal tv, RayBatch rb,
                                                           HitBatch hb, int n, int2 *spill, int spill_depth,
                                                           unsigned long long *counters) {
    __shared__ int s_ref[16 * 64];
    __shared__ float s_near[16 * 64];
    const DScene &S = *Sp;
    const int i = blockIdx.x * 64 + threadIdx.x;
    TravStats st{0, 0, 0};
    if (i < n) {
        RingStack2<16> stk{s_ref + threadIdx.x, s_near + threadIdx.x, 64, spill, (unsigned)n, (unsigned)i};
        typename std::conditional<W == 8, Tracer8<ORDERED, ANY, STATS, RingStack2<16>>,
                                  Tracer4<ORDERED, ANY, STATS, RingStack2<16>>>::type tr;
        tr.begin(S, tv, f3(rb.ox[i], rb.oy[i], rb.oz[i]), f3(rb.dx[i], rb.dy[i], rb.dz[i]), rb.mint[i], rb.maxt[i], st);
        while (!tr.done) tr.step(tv, stk, st);
        hb.hit[i] = tr.found ? 1 : 0;
        if (!ANY) {
            hb.t[i] = tr.found ? tr.best.t : INFINITY;
            hb.u[i] = tr.found ? tr.best.u : 0.f;
            hb.v[i] = tr.found ? tr.best.v : 0.f;
            hb.k[i] = tr.found ? tr.best.k : -1;
        }
    }
    if (STATS) flush_stats(st, i < n ? 1u : 0u, stat_shard(counters));
}


// ---- single-bounce direct integrators (one closest hit from the camera) --------------------
// Miss: the environment map, if any (direct_*.cpp:17-26). Hit on an emitter: its radiance toward
// the camera, unweighted (:33-39).
#define NH_DIRECT_PROLOGUE                                                                       \
    Hit h;                                                                                       \
    if (STATS) queries++;                                                                        \
    if (!trace<DEPTH, ORDERED, false, STATS>(tv, S, o, d, mint, maxt, h, stk, stride, st))      \
        return S.envmap >= 0 ? env_eval(S, d) : f3(0, 0, 0);                                     \
    Its its;                                                                                     \
    hit_info(S, tv, h, o, d, its);                                                               \
    const DShape shape = S.shapes[its.shape];                                                    \
    const DBsdf bsdf = S.bsdfs[shape.bsdf];                                                      \
    const F3 alb = bsdf_albedo(S, bsdf, its.u, its.v);                                           \
    F3 result = f3(0, 0, 0);                                                                     \
    if (shape.emitter >= 0)                                                                      \
        result = add(result, emitter_eval(S.emitters[shape.emitter], o, its.sh.n, normalized(sub(its.p, o))));

// DirectEMSIntegrator::Li (src/integrators/direct_ems.cpp:14-70): one light sample per emitter, in
// scene order, each with its own 2D sample; unoccluded ones add li * |cos| * f.
template <int DEPTH, bool ORDERED, bool STATS>
__device__ F3 li_direct_ems(const DScene &S, const Traversal &tv, Rng &rng, F3 o, F3 d, float mint, float maxt,
                            uint32_t *stk, int stride, TravStats &st, uint32_t &queries) {
    NH_DIRECT_PROLOGUE
    const F3 wo = to_local(its.sh, neg(d));
    for (int l = 0; l < S.n_emitters; ++l) {
        const float ex = rng.next1d(), ey = rng.next1d();
        ESample es;
        const F3 li = emitter_sample(S, S.emitters[l], its.p, ex, ey, es);
        if (is_zero(li)) continue;
        Hit hs;
        if (STATS) queries++;
        if (trace<DEPTH, ORDERED, true, STATS>(tv, S, es.so, es.sd, es.smint, es.smaxt, hs, stk, stride, st)) continue;
        const F3 we = to_local(its.sh, es.wi);
        const F3 f = bsdf_eval(bsdf, wo, we, M_SOLID_ANGLE, alb);
        result = add(result, mulc(scl(fabsf(we.z), li), f));
    }
    return result;
}

// DirectMATSIntegrator::Li (src/integrators/direct_mats.cpp:16-83): one BSDF sample (the record's
// measure preset to ESolidAngle); its ray adds the environment on a miss or the emitter it hits.
template <int DEPTH, bool ORDERED, bool STATS>
__device__ F3 li_direct_mats(const DScene &S, const Traversal &tv, Rng &rng, F3 o, F3 d, float mint, float maxt,
                             uint32_t *stk, int stride, TravStats &st, uint32_t &queries) {
    NH_DIRECT_PROLOGUE
    const float bx = rng.next1d(), by = rng.next1d();
    F3 wo;
    int measure;
    const F3 col = bsdf_sample(bsdf, to_local(its.sh, neg(d)), bx, by, wo, measure, alb);
    if (is_zero(col)) return result;
    const F3 nd = to_world(its.sh, wo);
    Hit h2;
    if (STATS) queries++;
    if (!trace<DEPTH, ORDERED, false, STATS>(tv, S, its.p, nd, kEps, INFINITY, h2, stk, stride, st)) {
        if (S.envmap >= 0) result = add(result, mulc(env_eval(S, nd), col));
        return result;
    }
    Its its2;
    hit_info(S, tv, h2, its.p, nd, its2);
    const int hem = S.shapes[its2.shape].emitter;
    if (hem >= 0)
        result = add(result, mulc(emitter_eval(S.emitters[hem], its.p, its2.sh.n, normalized(sub(its2.p, its.p))), col));
    return result;
}

// DirectMISIntegrator::Li (src/integrators/direct_mis.cpp:15-143): one emitter picked at random and
// one BSDF sample, balance-heuristic weights; result + w_ems * result_ems + w_mat * result_mats.
// Occluded light samples and BSDF rays that miss emitters still fill result_ems / result_mats with
// the environment (:84-92, :127-135) under a weight of 0.
template <int DEPTH, bool ORDERED, bool STATS>
__device__ F3 li_direct_mis(const DScene &S, const Traversal &tv, Rng &rng, F3 o, F3 d, float mint, float maxt,
                            uint32_t *stk, int stride, TravStats &st, uint32_t &queries) {
    NH_DIRECT_PROLOGUE
    const float n_lights = (float)S.n_emitters;
    F3 result_ems = f3(0, 0, 0), result_mats = f3(0, 0, 0);
    float w_ems = 0.f, w_mat = 0.f;
    const int ei = emitter_pick(S, rng.next1d());
    const DEmitter em = S.emitters[ei];
    const float ex = rng.next1d(), ey = rng.next1d();
    ESample es;
    const F3 li = emitter_sample(S, em, its.p, ex, ey, es);
    const F3 wi_l = to_local(its.sh, neg(d));
    if (!is_zero(li)) {
        Hit hs;
        if (STATS) queries++;
        if (!trace<DEPTH, ORDERED, true, STATS>(tv, S, es.so, es.sd, es.smint, es.smaxt, hs, stk, stride, st)) {
            const F3 we = to_local(its.sh, es.wi);
            const F3 f = bsdf_eval(bsdf, wi_l, we, M_SOLID_ANGLE, alb);
            const float cs = we.z;
            const float pdf_ems = emitter_pdf(S, em, its.p, es.p, es.n, es.wi) / n_lights;
            const float pdf_mat = bsdf_pdf(bsdf, wi_l, we, M_SOLID_ANGLE);
            result_ems = f3(li.x * cs * f.x * n_lights, li.y * cs * f.y * n_lights, li.z * cs * f.z * n_lights);
            if (pdf_ems + pdf_mat > kEps) w_ems = pdf_ems / (pdf_ems + pdf_mat);
        } else if (S.envmap >= 0) {
            result_ems = mulc(li, env_eval(S, es.sd));
        }
    }
    const float bx = rng.next1d(), by = rng.next1d();
    F3 wo;
    int measure;
    const F3 col = bsdf_sample(bsdf, wi_l, bx, by, wo, measure, alb);
    if (measure == M_UNKNOWN) measure = M_SOLID_ANGLE;  // bqr_mat.measure = ESolidAngle before sample (:102)
    if (!is_zero(col)) {
        const F3 nd = to_world(its.sh, wo);
        Hit h2;
        if (STATS) queries++;
        const bool hit2 = trace<DEPTH, ORDERED, false, STATS>(tv, S, its.p, nd, kEps, INFINITY, h2, stk, stride, st);
        int hem = -1;
        Its its2;
        if (hit2) {
            hit_info(S, tv, h2, its.p, nd, its2);
            hem = S.shapes[its2.shape].emitter;
        }
        if (hem >= 0) {
            const DEmitter e2 = S.emitters[hem];
            const F3 wim = normalized(sub(its2.p, its.p));
            result_mats = mulc(col, emitter_eval(e2, its.p, its2.sh.n, wim));
            const float pdf_mat = bsdf_pdf(bsdf, wi_l, wo, measure);
            const float pdf_e = emitter_pdf(S, e2, its.p, its2.p, its2.sh.n, wim) / n_lights;
            if (pdf_mat + pdf_e > kEps) w_mat = pdf_mat / (pdf_mat + pdf_e);
        } else if (S.envmap >= 0) {
            result_mats = mulc(col, env_eval(S, nd));
        }
    }
    return add(add(result, scl(w_ems, result_ems)), scl(w_mat, result_mats));
}
#undef NH_DIRECT_PROLOGUE

// DirectIntegrator::Li (src/integrators/direct.cpp:17-63, the point-light integrator of scenes/pa1):
// every emitter sampled once in scene order (its own 2D sample), its shadow ray always traced;
// unoccluded samples add li * |wi . n| / |wi| * f(wi = toward the light, wo = toward the ray
// origin). No emitter-hit term.
template <int DEPTH, bool ORDERED, bool STATS>
__device__ F3 li_direct_simple(const DScene &S, const Traversal &tv, Rng &rng, F3 o, F3 d, float mint, float maxt,
                               uint32_t *stk, int stride, TravStats &st, uint32_t &queries) {
    Hit h;
    if (STATS) queries++;
    if (!trace<DEPTH, ORDERED, false, STATS>(tv, S, o, d, mint, maxt, h, stk, stride, st))
        return S.envmap >= 0 ? env_eval(S, d) : f3(0, 0, 0);
    Its its;
    hit_info(S, tv, h, o, d, its);
    const DBsdf bsdf = S.bsdfs[S.shapes[its.shape].bsdf];
    const F3 alb = bsdf_albedo(S, bsdf, its.u, its.v);
    const F3 wo = to_local(its.sh, normalized(sub(o, its.p)));
    F3 result = f3(0, 0, 0);
    for (int l = 0; l < S.n_emitters; ++l) {
        const float ex = rng.next1d(), ey = rng.next1d();
        ESample es;
        const F3 li = emitter_sample(S, S.emitters[l], its.p, ex, ey, es);
        const F3 wi = to_local(its.sh, es.wi);
        Hit hs;
        if (STATS) queries++;
        if (trace<DEPTH, ORDERED, true, STATS>(tv, S, es.so, es.sd, es.smint, es.smaxt, hs, stk, stride, st)) continue;
        const F3 f = bsdf_eval(bsdf, wi, wo, M_SOLID_ANGLE, alb);
        const float cs = fabsf(dot(es.wi, its.sh.n)) / f_sqrt(dot(es.wi, es.wi));
        result = add(result, mulc(scl(cs, li), f));
    }
    return result;
}

// NormalIntegrator::Li (src/integrators/normals.cpp:15-33): the shading frame of the first hit, as
// |shFrame.toWorld(direction)| (Frame::toWorld = s x + t y + n z); a miss sees the envmap (EnvMap::eval, wi = ray.d)
template <int DEPTH, bool ORDERED, bool STATS>
__device__ F3 li_normals(const DScene &S, const Traversal &tv, F3 o, F3 d, float mint, float maxt, uint32_t *stk,
                         int stride, TravStats &st, uint32_t &queries) {
    Hit h;
    if (STATS) queries++;
    if (!trace<DEPTH, ORDERED, false, STATS>(tv, S, o, d, mint, maxt, h, stk, stride, st))
        return S.envmap >= 0 ? env_eval(S, d) : f3(0, 0, 0);
    Its its;
    hit_info(S, tv, h, o, d, its);
    const F3 n = to_world(its.sh, f3(S.ndir[0], S.ndir[1], S.ndir[2]));
    return f3(fabsf(n.x), fabsf(n.y), fabsf(n.z));
}

// PM: a path_mis scene without normal maps -- only li_path_mis, normal maps compiled out. The kernel with every
// integrator (and hit_info's normal-map calls) holds registers and code that cost the path_mis megakernel 6 %
// (profiles/round6_ab_nmap.txt).
template <int BLOCK, int DEPTH, bool ORDERED, bool STATS, int MINW, bool PM = false>
__global__ __launch_bounds__(BLOCK, MINW) void nh_path_kernel(const DScene *__restrict__ Sp, Traversal tv, PathLaunch L) {
    __shared__ uint32_t stk[DEPTH * BLOCK];
    const DScene &S = *Sp;
    const int gid = blockIdx.x * BLOCK + threadIdx.x;
    TravStats st{0, 0, 0};
    uint32_t queries = 0;
    if (gid < L.n_paths) {
        const int k = gid / L.n_list, i = gid - k * L.n_list;
        const int pix = L.pixel_list[i];
        const int py = pix / S.width, px = pix - py * S.width;
        const int sample = L.s0 + k;
        Rng rng = path_rng(L.seed, (uint64_t)pix, (uint64_t)sample);
        // renderBlock (render.cpp:441-447): pixel jitter, unused aperture sample
        const float jx = rng.next1d(), jy = rng.next1d();
        rng.next1d();
        rng.next1d();
        const float spx = (float)px + jx, spy = (float)py + jy;
        F3 o, d;
        float mint, maxt;
        camera_ray(S, spx, spy, o, d, mint, maxt, sample, pix);
        F3 li;
        if (PM) li = li_path_mis<DEPTH, ORDERED, STATS, false>(S, tv, rng, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries);
        else switch (S.integrator) {
            case 1: li = li_path_mats<DEPTH, ORDERED, STATS>(S, tv, rng, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries); break;
            case 2: li = li_direct_ems<DEPTH, ORDERED, STATS>(S, tv, rng, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries); break;
            case 3: li = li_direct_mats<DEPTH, ORDERED, STATS>(S, tv, rng, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries); break;
            case 4: li = li_direct_mis<DEPTH, ORDERED, STATS>(S, tv, rng, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries); break;
            case 5: li = li_direct_simple<DEPTH, ORDERED, STATS>(S, tv, rng, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries); break;
            case 6: li = li_normals<DEPTH, ORDERED, STATS>(S, tv, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries); break;
            default: li = li_path_mis<DEPTH, ORDERED, STATS>(S, tv, rng, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries); break;
        }
        const size_t r = (size_t)k * L.n_list + i;
        L.rec[kRecFloats * r] = li.x;
        L.rec[kRecFloats * r + 1] = li.y;
        L.rec[kRecFloats * r + 2] = li.z;
    }
    if (STATS) flush_stats(st, queries, stat_shard(L.counters));
}

// ---------------------------------------------------------------------------
// host-side launchers (called from nh_api.hip)
// ---------------------------------------------------------------------------
namespace nh {

template <int BLOCK, int DEPTH>
static void launch_trace_d(const DScene *S, const Traversal &tv, const RayBatch &rb, const HitBatch &hb, int n,
                           bool any, bool ordered, bool stats, unsigned long long *ctr, hipStream_t st) {
    dim3 grid((n + BLOCK - 1) / BLOCK);
#define NH_TK(O, A, T) hipLaunchKernelGGL((nh_trace_kernel<BLOCK, DEPTH, O, A, T>), grid, dim3(BLOCK), 0, st, S, tv, rb, hb, n, ctr)
    if (ordered) {
        if (any) { if (stats) NH_TK(true, true, true); else NH_TK(true, true, false); }
        else { if (stats) NH_TK(true, false, true); else NH_TK(true, false, false); }
    } else {
        if (any) { if (stats) NH_TK(false, true, true); else NH_TK(false, true, false); }
        else { if (stats) NH_TK(false, false, true); else NH_TK(false, false, false); }
    }
#undef NH_TK
}

void launch_trace(const DScene *S, const Traversal &tv, const RayBatch &rb, const HitBatch &hb, int n, bool any,
                  bool ordered, bool stats, int depth, unsigned long long *ctr, hipStream_t st) {
    if (n <= 0) return;
    if (depth <= 16) launch_trace_d<128, 16>(S, tv, rb, hb, n, any, ordered, stats, ctr, st);
    else if (depth <= 32) launch_trace_d<128, 32>(S, tv, rb, hb, n, any, ordered, stats, ctr, st);
    else if (depth <= 64) launch_trace_d<64, 64>(S, tv, rb, hb, n, any, ordered, stats, ctr, st);
    else launch_trace_d<64, 128>(S, tv, rb, hb, n, any, ordered, stats, ctr, st);
}

void launch_trace_wide(const DScene *S, const Traversal &tv, const RayBatch &rb, const HitBatch &hb, int n, bool any,
                       bool ordered, bool stats, int2 *spill, int spill_depth, unsigned long long *ctr,
                       hipStream_t st, int wide) {
    if (n <= 0) return;
    dim3 grid((n + 63) / 64);
#define NH_TW(O, A, T)                                                                                              \
    do {                                                                                                           \
        if (wide == 8) hipLaunchKernelGGL((nh_trace_wide_kernel<O, A, T, 8>), grid, dim3(64), 0, st, S, tv, rb, hb, n, \
                                          spill, spill_depth, ctr);                                                \
        else hipLaunchKernelGGL((nh_trace_wide_kernel<O, A, T>), grid, dim3(64), 0, st, S, tv, rb, hb, n, spill,      \
                                spill_depth, ctr);                                                                 \
    } while (0)
    if (ordered) {
        if (any) { if (stats) NH_TW(true, true, true); else NH_TW(true, true, false); }
        else { if (stats) NH_TW(true, false, true); else NH_TW(true, false, false); }
    } else {
        if (any) { if (stats) NH_TW(false, true, true); else NH_TW(false, true, false); }
        else { if (stats) NH_TW(false, false, true); else NH_TW(false, false, false); }
    }
#undef NH_TW
}

template <int BLOCK, int DEPTH, int MINW>
static void launch_path_w(const DScene *S, const Traversal &tv, const PathLaunch &L, bool ordered, bool stats,
                          bool pm, hipStream_t st) {
    dim3 grid((L.n_paths + BLOCK - 1) / BLOCK);
#define NH_PK(O, T) hipLaunchKernelGGL((nh_path_kernel<BLOCK, DEPTH, O, T, MINW>), grid, dim3(BLOCK), 0, st, S, tv, L)
#define NH_PKP(T) hipLaunchKernelGGL((nh_path_kernel<BLOCK, DEPTH, true, T, MINW, true>), grid, dim3(BLOCK), 0, st, S, tv, L)
    if (ordered && pm) { if (stats) NH_PKP(true); else NH_PKP(false); }
    else if (ordered) { if (stats) NH_PK(true, true); else NH_PK(true, false); }
    else { if (stats) NH_PK(false, true); else NH_PK(false, false); }
#undef NH_PK
#undef NH_PKP
}

// occupancy target of the megakernel (waves per SIMD the register allocator must allow)
static int path_min_waves() {
    static int w = [] {
        const char *e = std::getenv("NH_PATH_WAVES");
        int v = e ? std::atoi(e) : NH_DEFAULT_PATH_WAVES;
        return (v >= 1 && v <= 4) ? v : NH_DEFAULT_PATH_WAVES;
    }();
    return w;
}

template <int BLOCK, int DEPTH>
static void launch_path_d(const DScene *S, const Traversal &tv, const PathLaunch &L, bool ordered, bool stats, bool pm,
                          hipStream_t st) {
    // 4 waves/SIMD measured best (13.7 / 13.8 / 9.8 / 8.3 ms per 16M C2 samples at 1 / 2 / 3 / 4);
    // the 2-wave build stays selectable (NH_PATH_WAVES=2) for register-heavy experiments
    // deep stacks (DEPTH > 32) are LDS-limited below 4 waves anyway: build them for 2
    if constexpr (DEPTH > 32) {
        launch_path_w<BLOCK, DEPTH, 2>(S, tv, L, ordered, stats, pm, st);
    } else {
        if (path_min_waves() == 2) launch_path_w<BLOCK, DEPTH, 2>(S, tv, L, ordered, stats, pm, st);
        else launch_path_w<BLOCK, DEPTH, 4>(S, tv, L, ordered, stats, pm, st);
    }
}

void launch_path(const DScene *S, const Traversal &tv, const PathLaunch &L, bool ordered, bool stats, int depth,
                 bool pm, hipStream_t st) {
    if (L.n_paths <= 0) return;
    if (depth <= 16) launch_path_d<128, 16>(S, tv, L, ordered, stats, pm, st);
    else if (depth <= 32) launch_path_d<128, 32>(S, tv, L, ordered, stats, pm, st);
    else if (depth <= 64) launch_path_d<64, 64>(S, tv, L, ordered, stats, pm, st);
    else launch_path_d<64, 128>(S, tv, L, ordered, stats, pm, st);
}

}  // namespace nh
