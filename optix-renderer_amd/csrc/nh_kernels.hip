// gfx950 kernels of the path_mis hot path.
//
//   nh_trace_kernel   BVH::rayIntersect over an SoA ray batch (parity entry point)
//   nh_path_kernel    megakernel: one thread per (pixel, sample) camera path --
//                     renderBlock's per-pixel body + PathMISIntegrator::Li / PathMatsIntegrator::Li
//                     (src/utils/render.cpp:436-458, src/integrators/path_mis.cpp:16-150,
//                     path_mats.cpp:16-78), writing (radiance, jitter) sample records
//   nh_splat_kernel   ImageBlock::put(pos, value) into per-block blocks + ImageBlock::put(block)
//                     into the master (src/utils/block.cpp:93-134) as a gather per master
//                     pixel that reproduces the reference's summation order: per round, blocks
//                     in BlockGenerator spiral order, within a block samples in
//                     getSampleIndices order (x outer, y inner)
#include "nh_internal.h"
#include "nh_traverse.h"

using namespace nhd;

namespace {

struct Its {  // Intersection (include/nori/shape.h:41-79); geoFrame only where needed
    F3 p;
    float u, v;
    Frame sh;
    int shape;
};

// Mesh::setHitInformation (mesh.cpp:141-196) / Sphere::setHitInformation (sphere.cpp:96-124)
__device__ __forceinline__ void hit_info(const DScene &S, const Traversal &tv, const Hit &h, F3 o, F3 d, Its &its) {
    const float4 a = tv.prims[3 * h.k], b = tv.prims[3 * h.k + 1];
    const int shape = __float_as_int(b.w);
    const DShape sh = S.shapes[shape];
    its.shape = shape;
    if (sh.type == SHAPE_SPHERE) {
        its.p = add(o, scl(h.t, d));
        F3 n = normalized(sub(its.p, f3(sh.cx, sh.cy, sh.cz)));
        F3 mn = neg(n);
        float theta = f_acos(mn.z), phi = f_atan2(mn.y, mn.x);
        if (phi < 0) phi += 2 * kPi;
        its.u = phi / (2.f * kPi);
        its.v = theta / kPi;
        F3 t = normalized(cross(f3(0, 0, 1), n));
        its.sh.s = t;
        its.sh.t = cross(n, t);
        its.sh.n = n;
        return;
    }
    const int local = __float_as_int(a.w);
    const uint32_t *f = S.F + 3 * (size_t)(sh.f_off + local);
    const uint32_t i0 = sh.v_off + f[0], i1 = sh.v_off + f[1], i2 = sh.v_off + f[2];
    const float bx = 1 - (h.u + h.v), by = h.u, bz = h.v;
    const F3 p0 = ldv(S.V, i0), p1 = ldv(S.V, i1), p2 = ldv(S.V, i2);
    its.p = add(add(scl(bx, p0), scl(by, p1)), scl(bz, p2));
    its.u = h.u;
    its.v = h.v;
    if (sh.has_uv) {
        its.u = bx * S.UV[2 * i0] + by * S.UV[2 * i1] + bz * S.UV[2 * i2];
        its.v = bx * S.UV[2 * i0 + 1] + by * S.UV[2 * i1 + 1] + bz * S.UV[2 * i2 + 1];
    }
    if (sh.has_n) {
        F3 nrm = normalized(add(add(scl(bx, ldv(S.N, i0)), scl(by, ldv(S.N, i1))), scl(bz, ldv(S.N, i2))));
        if (sh.has_uv) {
            its.sh.s = normalized(add(add(scl(bx, ldv(S.T, i0)), scl(by, ldv(S.T, i1))), scl(bz, ldv(S.T, i2))));
            its.sh.t = normalized(add(add(scl(bx, ldv(S.BT, i0)), scl(by, ldv(S.BT, i1))), scl(bz, ldv(S.BT, i2))));
            its.sh.n = nrm;
        } else {
            its.sh = frame_from_n(nrm);
        }
    } else {
        its.sh = frame_from_n(normalized(cross(sub(p1, p0), sub(p2, p0))));
    }
}

// AreaEmitter / PointLight (src/emitters/arealight.cpp:58-125, pointlight.cpp:47-78)
__device__ __forceinline__ float emitter_pdf(const DScene &S, const DEmitter &e, F3 ref, F3 p, F3 n, F3 wi) {
    if (e.type == EMITTER_POINT) return 1.f;
    if (dot(n, neg(wi)) < 0.f) return 0.f;
    const DShape sh = S.shapes[e.shape];
    // Sphere::pdfSurface: std::pow(1.f / r, 2) (double, exact square) * (0.25f / M_PI)
    float prob = sh.type == SHAPE_MESH
                     ? sh.pdf_norm
                     : (float)((double)(1.f / sh.radius) * (double)(1.f / sh.radius) * (double)(0.25f / kPi));
    return prob * dot(sub(p, ref), sub(p, ref)) / fabsf(dot(n, neg(wi)));
}
__device__ __forceinline__ F3 emitter_eval(const DEmitter &e, F3 ref, F3 n, F3 wi) {
    if (e.type == EMITTER_POINT) {
        F3 dd = sub(ref, f3(e.px, e.py, e.pz));
        float q = dot(dd, dd);
        return f3(e.lr / q, e.lg / q, e.lb / q);
    }
    if (dot(n, neg(wi)) < 0.f) return f3(0, 0, 0);
    return f3(e.lr, e.lg, e.lb);
}

struct ESample {
    F3 wi, p, n;
    F3 so, sd;  // shadow ray, from the light towards ref
    float smint, smaxt;
};

__device__ __forceinline__ F3 emitter_sample(const DScene &S, const DEmitter &e, F3 ref, float sx, float sy,
                                             ESample &es) {
    if (e.type == EMITTER_POINT) {
        F3 pos = f3(e.px, e.py, e.pz);
        F3 rp = sub(ref, pos);
        es.so = pos;
        es.sd = normalized(rp);
        es.smint = kEps;
        es.smaxt = f_sqrt(dot(rp, rp)) - kEps;
        es.wi = normalized(sub(pos, ref));
        es.p = f3(0, 0, 0);
        es.n = f3(0, 0, 0);
        return emitter_eval(e, ref, es.n, es.wi);
    }
    const DShape sh = S.shapes[e.shape];
    F3 p, n;
    if (sh.type == SHAPE_MESH) {  // Mesh::sampleSurface (mesh.cpp:50-71)
        const float *cdf = S.area_cdf + sh.pdf_off;
        int idt = dpdf_sample(cdf, sh.n_faces, sx);
        sx = (sx - cdf[idt]) / (cdf[idt + 1] - cdf[idt]);
        float su1 = f_sqrt(sx);  // squareToUniformTriangle (warp.cpp:162-166)
        float bu = 1.f - su1, bv = sy * su1, bw = 1.f - bu - bv;
        const uint32_t *f = S.F + 3 * (size_t)(sh.f_off + idt);
        const uint32_t i0 = sh.v_off + f[0], i1 = sh.v_off + f[1], i2 = sh.v_off + f[2];
        const F3 p0 = ldv(S.V, i0), p1 = ldv(S.V, i1), p2 = ldv(S.V, i2);
        p = add(add(scl(bu, p0), scl(bv, p1)), scl(bw, p2));
        if (sh.has_n)
            n = normalized(add(add(scl(bu, ldv(S.N, i0)), scl(bv, ldv(S.N, i1))), scl(bw, ldv(S.N, i2))));
        else
            n = normalized(cross(sub(p1, p0), sub(p2, p0)));
    } else {  // Sphere::sampleSurface (sphere.cpp:126-131)
        F3 q = uniform_sphere(sx, sy);
        p = add(f3(sh.cx, sh.cy, sh.cz), scl(sh.radius, q));
        n = q;
    }
    es.p = p;
    es.n = n;
    F3 pr = sub(p, ref);
    es.wi = normalized(pr);
    es.so = p;
    es.sd = neg(es.wi);
    es.smint = kEps;
    es.smaxt = f_sqrt(dot(pr, pr)) - kEps;
    float probs = emitter_pdf(S, e, ref, p, n, es.wi);
    if (fabsf(probs) < kEps) return f3(0, 0, 0);
    F3 ev = emitter_eval(e, ref, n, es.wi);
    return f3(ev.x / probs, ev.y / probs, ev.z / probs);
}

// PerspectiveCamera::sampleRay without depth of field (perspective.cpp:97-141)
__device__ __forceinline__ void camera_ray(const DScene &S, float px, float py, F3 &o, F3 &d, float &mint,
                                           float &maxt) {
    const float in0 = px * S.inv_w, in1 = py * S.inv_h;
    float r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float acc = S.s2c[4 * i] * in0;
        acc = acc + S.s2c[4 * i + 1] * in1;
        acc = acc + S.s2c[4 * i + 2] * 0.0f;
        acc = acc + S.s2c[4 * i + 3] * 1.0f;
        r[i] = acc;
    }
    F3 dl = normalized(f3(r[0] / r[3], r[1] / r[3], r[2] / r[3]));
    float ow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float acc = S.c2w[4 * i] * 0.0f;
        acc = acc + S.c2w[4 * i + 1] * 0.0f;
        acc = acc + S.c2w[4 * i + 2] * 0.0f;
        acc = acc + S.c2w[4 * i + 3] * 1.0f;
        ow[i] = acc;
    }
    o = f3(ow[0] / ow[3], ow[1] / ow[3], ow[2] / ow[3]);
    const float *w = S.c2w;
    d = f3(w[0] * dl.x + (w[1] * dl.y + w[2] * dl.z), w[4] * dl.x + (w[5] * dl.y + w[6] * dl.z),
           w[8] * dl.x + (w[9] * dl.y + w[10] * dl.z));
    const float inv_z = 1.0f / dl.z;
    mint = S.near_clip * inv_z;
    maxt = S.far_clip * inv_z;
}

template <int DEPTH, bool ORDERED, bool STATS>
__device__ __forceinline__ bool closest(const Traversal &tv, const DScene &S, F3 o, F3 d, float mint, float maxt,
                                        Hit &h, uint2 *stk, int stride, TravStats &st) {
    return trace<DEPTH, ORDERED, false, STATS>(tv, S, o, d, mint, maxt, h, stk, stride, st);
}

// PathMISIntegrator::Li (src/integrators/path_mis.cpp:16-150). The BSDF-sampled ray is
// both the MIS probe (:117-119) and the next bounce (:146 -> :34): it is traced once.
template <int DEPTH, bool ORDERED, bool STATS>
__device__ F3 li_path_mis(const DScene &S, const Traversal &tv, Rng &rng, F3 o, F3 d, float mint, float maxt,
                          uint2 *stk, int stride, TravStats &st, uint32_t &queries) {
    F3 li = f3(0, 0, 0), t = f3(1, 1, 1);
    float w_mats = 1.f, w_ems = 0.f;
    const float n_lights = (float)S.n_emitters;
    Hit h;
    if (STATS) queries++;
    bool found = closest<DEPTH, ORDERED, STATS>(tv, S, o, d, mint, maxt, h, stk, stride, st);
    Its its;
    if (found) hit_info(S, tv, h, o, d, its);
    while (true) {
        if (!found) break;  // no environment map: nothing is added on a miss (path_mis.cpp:34-44)
        const DShape shape = S.shapes[its.shape];
        const DBsdf bsdf = S.bsdfs[shape.bsdf];
        if (shape.emitter >= 0) {
            const DEmitter em = S.emitters[shape.emitter];
            F3 wi = normalized(sub(its.p, o));
            F3 e = emitter_eval(em, o, its.sh.n, wi);
            li = add(li, mulc(scl(w_mats, t), e));
        }
        float succ = e_min(max_coeff(t), 0.99f);
        succ = e_max(succ, kEps);
        if (rng.next1d() > succ) break;
        t = divs(t, succ);

        // ---- emitter sampling (path_mis.cpp:75-106)
        const int ei = dpdf_sample(S.emitter_cdf, S.n_emitters, rng.next1d());
        const DEmitter em = S.emitters[ei];
        const float ex = rng.next1d(), ey = rng.next1d();
        ESample es;
        F3 ems_col = emitter_sample(S, em, its.p, ex, ey, es);
        F3 we = to_local(its.sh, es.wi);
        const F3 wi_l = to_local(its.sh, neg(d));
        F3 li_ems = f3(0, 0, 0);
        float pdfems = 0.f, pdfems_mats = 0.f;
        if (!is_zero(ems_col)) {
            Hit hs;
            if (STATS) queries++;
            if (!trace<DEPTH, ORDERED, true, STATS>(tv, S, es.so, es.sd, es.smint, es.smaxt, hs, stk, stride, st)) {
                F3 f = bsdf_eval(bsdf, wi_l, we, M_SOLID_ANGLE);
                float cs = we.z;
                li_ems = f3(ems_col.x * cs * f.x * n_lights, ems_col.y * cs * f.y * n_lights,
                            ems_col.z * cs * f.z * n_lights);
                pdfems_mats = bsdf_pdf(bsdf, wi_l, we, M_SOLID_ANGLE);
                pdfems = emitter_pdf(S, em, its.p, es.p, es.n, es.wi) / n_lights;
            }
        }
        if ((pdfems_mats + pdfems) > kEps) w_ems = pdfems / (pdfems_mats + pdfems);

        // ---- BSDF sampling + probe (path_mis.cpp:108-146)
        const float bx = rng.next1d(), by = rng.next1d();
        F3 wo;
        int measure;
        F3 bsdf_col = bsdf_sample(bsdf, wi_l, bx, by, wo, measure);
        const F3 nd = to_world(its.sh, wo);
        const F3 no = its.p;
        Its its_s;
        if (nd.x == 0 && nd.y == 0 && nd.z == 0) {
            found = false;  // zero direction: every primitive test rejects (det == 0 / NaN roots)
        } else {
            if (STATS) queries++;
            found = closest<DEPTH, ORDERED, STATS>(tv, S, no, nd, kEps, INFINITY, h, stk, stride, st);
            if (found) hit_info(S, tv, h, no, nd, its_s);
        }
        if (!is_zero(bsdf_col) && found) {
            const DShape hs = S.shapes[its_s.shape];
            if (hs.emitter >= 0) {
                const DEmitter em2 = S.emitters[hs.emitter];
                F3 wim = normalized(sub(its_s.p, its.p));
                float pdfmat = bsdf_pdf(bsdf, wi_l, wo, measure);
                float pdfmat_ems = emitter_pdf(S, em2, its.p, its_s.p, its_s.sh.n, wim) / n_lights;
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
        its = its_s;
    }
    return li;
}

// PathMatsIntegrator::Li (src/integrators/path_mats.cpp:16-78)
template <int DEPTH, bool ORDERED, bool STATS>
__device__ F3 li_path_mats(const DScene &S, const Traversal &tv, Rng &rng, F3 o, F3 d, float mint, float maxt,
                           uint2 *stk, int stride, TravStats &st, uint32_t &queries) {
    F3 li = f3(0, 0, 0), t = f3(1, 1, 1);
    int counter = 0;
    Hit h;
    for (;;) {
        bool found;
        if (d.x == 0 && d.y == 0 && d.z == 0) {
            found = false;
        } else {
            if (STATS) queries++;
            found = closest<DEPTH, ORDERED, STATS>(tv, S, o, d, mint, maxt, h, stk, stride, st);
        }
        if (!found) break;
        Its its;
        hit_info(S, tv, h, o, d, its);
        const DShape shape = S.shapes[its.shape];
        const DBsdf bsdf = S.bsdfs[shape.bsdf];
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
        F3 col = bsdf_sample(bsdf, to_local(its.sh, neg(d)), bx, by, wo, measure);
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
__global__ __launch_bounds__(BLOCK) void nh_trace_kernel(DScene S, Traversal tv, RayBatch rb, HitBatch hb, int n,
                                                         unsigned long long *counters) {
    __shared__ uint2 stk[DEPTH * BLOCK];
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
    if (STATS) flush_stats(st, i < n ? 1u : 0u, counters);
}

template <int BLOCK, int DEPTH, bool ORDERED, bool STATS>
__global__ __launch_bounds__(BLOCK) void nh_path_kernel(DScene S, Traversal tv, PathLaunch L) {
    __shared__ uint2 stk[DEPTH * BLOCK];
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
        camera_ray(S, spx, spy, o, d, mint, maxt);
        F3 li = S.integrator == 1
                    ? li_path_mats<DEPTH, ORDERED, STATS>(S, tv, rng, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries)
                    : li_path_mis<DEPTH, ORDERED, STATS>(S, tv, rng, o, d, mint, maxt, stk + threadIdx.x, BLOCK, st, queries);
        const size_t r = (size_t)k * L.n_list + i;
        L.rec_rgbx[r] = make_float4(li.x, li.y, li.z, jx);
        L.rec_jy[r] = jy;
    }
    if (STATS) flush_stats(st, queries, L.counters);
}

// One thread per master-block pixel; loops over the chunk's rounds.
__global__ __launch_bounds__(256) void nh_splat_kernel(SplatLaunch P) {
    const int mcols = P.width + 2 * P.border, mrows = P.height + 2 * P.border;
    const int mx = blockIdx.x * 16 + (threadIdx.x & 15), my = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (mx >= mcols || my >= mrows) return;
    const int qx = mx - P.border, qy = my - P.border;
    const int R = P.reach;
    const int xa = max(qx - R, 0), xb = min(qx + R, P.width - 1);
    const int ya = max(qy - R, 0), yb = min(qy + R, P.height - 1);
    if (xa > xb || ya > yb) return;
    // candidate blocks (at most 2x2), sorted by spiral rank
    int blk[4], nb = 0;
    for (int by = ya >> 5; by <= (yb >> 5); ++by)
        for (int bx = xa >> 5; bx <= (xb >> 5); ++bx) blk[nb++] = by * P.nbx + bx;
    for (int a = 1; a < nb; ++a)
        for (int b = a; b > 0 && P.block_rank[blk[b]] < P.block_rank[blk[b - 1]]; --b) {
            int tmp = blk[b]; blk[b] = blk[b - 1]; blk[b - 1] = tmp;
        }
    float4 *mp = reinterpret_cast<float4 *>(P.fb) + (size_t)my * mcols + mx;
    float4 m = *mp;
    const int cols = 32 + 2 * P.border;
    const float r = P.radius;
    for (int k = 0; k < P.n_rounds; ++k) {
        const size_t rbase = (size_t)k * P.n_list;
        for (int q = 0; q < nb; ++q) {
            const int bid = blk[q], by = bid / P.nbx, bx = bid - by * P.nbx;
            const int ox = bx * 32, oy = by * 32;
            const int sxb = min(32, P.width - ox), syb = min(32, P.height - oy);
            const int xt = mx - ox, yt = my - oy;  // block-array coordinates of this master pixel
            if (xt < 0 || yt < 0 || xt >= sxb + 2 * P.border || yt >= syb + 2 * P.border) continue;
            float ar = 0.f, ag = 0.f, ab = 0.f, aw = 0.f;
            bool any = false;
            const int x0 = max(xa, ox), x1 = min(xb, ox + 31), y0 = max(ya, oy), y1 = min(yb, oy + 31);
            for (int px = x0; px <= x1; ++px)
                for (int py = y0; py <= y1; ++py) {
                    const int li = P.pixel_map[py * P.width + px];
                    if (li < 0) continue;
                    const float4 rec = P.rec_rgbx[rbase + li];
                    const F3 v = f3(rec.x, rec.y, rec.z);
                    if (!is_valid(v)) continue;  // dropped with its filter weight
                    const float jy = P.rec_jy[rbase + li];
                    const float spx = (float)px + rec.w, spy = (float)py + jy;
                    const float posx = spx - 0.5f - (float)(ox - P.border);
                    const float posy = spy - 0.5f - (float)(oy - P.border);
                    int bx0 = (int)ceilf(posx - r), by0 = (int)ceilf(posy - r);
                    int bx1 = (int)floorf(posx + r), by1 = (int)floorf(posy + r);
                    bx0 = max(bx0, 0); by0 = max(by0, 0);
                    bx1 = min(bx1, cols - 1); by1 = min(by1, cols - 1);
                    if (xt < bx0 || xt > bx1 || yt < by0 || yt > by1) continue;
                    const float wx = P.table[(int)(fabsf((float)xt - posx) * P.lookup)];
                    const float wy = P.table[(int)(fabsf((float)yt - posy) * P.lookup)];
                    ar += v.x * wx * wy;
                    ag += v.y * wx * wy;
                    ab += v.z * wx * wy;
                    aw += 1.0f * wx * wy;
                    any = true;
                }
            if (any) {
                m.x += ar;
                m.y += ag;
                m.z += ab;
                m.w += aw;
            }
        }
    }
    *mp = m;
}

// invalid-sample count (ImageBlock::put drops, block.cpp:94-99)
__global__ __launch_bounds__(256) void nh_count_invalid_kernel(const float4 *rec, size_t n, unsigned long long *out) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long c = 0;
    if (i < n) {
        float4 v = rec[i];
        c = is_valid(f3(v.x, v.y, v.z)) ? 0 : 1;
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// ---------------------------------------------------------------------------
// host-side launchers (called from nh_api.hip)
// ---------------------------------------------------------------------------
namespace nh {

template <int BLOCK, int DEPTH>
static void launch_trace_d(const DScene &S, const Traversal &tv, const RayBatch &rb, const HitBatch &hb, int n,
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

void launch_trace(const DScene &S, const Traversal &tv, const RayBatch &rb, const HitBatch &hb, int n, bool any,
                  bool ordered, bool stats, int depth, unsigned long long *ctr, hipStream_t st) {
    if (n <= 0) return;
    if (depth <= 16) launch_trace_d<128, 16>(S, tv, rb, hb, n, any, ordered, stats, ctr, st);
    else if (depth <= 32) launch_trace_d<128, 32>(S, tv, rb, hb, n, any, ordered, stats, ctr, st);
    else if (depth <= 64) launch_trace_d<64, 64>(S, tv, rb, hb, n, any, ordered, stats, ctr, st);
    else launch_trace_d<64, 128>(S, tv, rb, hb, n, any, ordered, stats, ctr, st);
}

template <int BLOCK, int DEPTH>
static void launch_path_d(const DScene &S, const Traversal &tv, const PathLaunch &L, bool ordered, bool stats,
                          hipStream_t st) {
    dim3 grid((L.n_paths + BLOCK - 1) / BLOCK);
#define NH_PK(O, T) hipLaunchKernelGGL((nh_path_kernel<BLOCK, DEPTH, O, T>), grid, dim3(BLOCK), 0, st, S, tv, L)
    if (ordered) { if (stats) NH_PK(true, true); else NH_PK(true, false); }
    else { if (stats) NH_PK(false, true); else NH_PK(false, false); }
#undef NH_PK
}

void launch_path(const DScene &S, const Traversal &tv, const PathLaunch &L, bool ordered, bool stats, int depth,
                 hipStream_t st) {
    if (L.n_paths <= 0) return;
    if (depth <= 16) launch_path_d<128, 16>(S, tv, L, ordered, stats, st);
    else if (depth <= 32) launch_path_d<128, 32>(S, tv, L, ordered, stats, st);
    else if (depth <= 64) launch_path_d<64, 64>(S, tv, L, ordered, stats, st);
    else launch_path_d<64, 128>(S, tv, L, ordered, stats, st);
}

void launch_splat(const SplatLaunch &P, hipStream_t st) {
    const int mcols = P.width + 2 * P.border, mrows = P.height + 2 * P.border;
    dim3 grid((mcols + 15) / 16, (mrows + 15) / 16);
    hipLaunchKernelGGL(nh_splat_kernel, grid, dim3(256), 0, st, P);
}

void launch_count_invalid(const float4 *rec, size_t n, unsigned long long *out, hipStream_t st) {
    if (n == 0) return;
    dim3 grid((unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(nh_count_invalid_kernel, grid, dim3(256), 0, st, rec, n, out);
}

}  // namespace nh
